# configs[3] query-set variants A/B on one box (tuning aid).
cd $GRAFT_REPO_ROOT
for rep in 1 2; do
for cfg in "SWBANK_MQ_PAIR=1" "SWBANK_MQ_PAIR=0"; do
  env $cfg timeout -k 10 300 python bench.py --workload reads150x1k --cpu-seconds 0 --steps 10 > gpurun_out/bench_mq.json 2>gpurun_out/bench_mq.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/bench_mq.json'));print('$cfg', d['value'], d['kernel'], d['roofline']['achieved'])"
done
done
export TMPDIR=/tmp; cd /tmp
SWBANK_MQ_PAIR=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_mq -o trace -- python3 $GRAFT_REPO_ROOT/bench.py --workload reads150x1k --profile-only --steps 3 --warmup 1 > /dev/null 2>&1 || exit 1
head -5 $GRAFT_REPO_ROOT/gpurun_out/prof_mq/trace_kernel_stats.csv | cut -c1-200
