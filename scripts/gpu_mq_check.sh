# Query-set parity tests, then configs[3] with the set in one launch per segment vs one query at a time.
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_queries.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/mq_tests.log 2>&1; rc=$?; tail -15 gpurun_out/mq_tests.log; [ $rc -ne 0 ] && exit $rc
for cfg in "SWBANK_MQ=1" "SWBANK_MQ=0"; do
  env $cfg timeout -k 10 300 python bench.py --workload reads150x1k > gpurun_out/bench_mq.json 2>gpurun_out/bench_mq.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/bench_mq.json'));print('$cfg', d['value'], d['kernel'], d['roofline']['achieved'], d['parity_sample'])"
done
