# Feeder parity tests, then host-API timings: uniform and ragged.
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_feeder.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "feeder or ragged or partial" > gpurun_out/feeder_tests.log 2>&1; rc=$?; tail -3 gpurun_out/feeder_tests.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
for cfg in "SWBANK_UNIFORM=1" "SWBANK_UNIFORM=0"; do
  env $cfg timeout -k 10 120 python scripts/host_api_bench.py --iters 8 > gpurun_out/hab.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/hab.json'));print('uniform $cfg', d['host_api_ms'], d['host_api_all_ms'], d['feeder_gather_ms_per_call'], d['host_api_gcups'], d.get('records_api_ms'))"
done
done
timeout -k 10 120 python scripts/host_api_bench.py --iters 8 --no-records --ragged --n-frac 0.001 > gpurun_out/hab.json 2>/dev/null || exit 1
python -c "import json;d=json.load(open('gpurun_out/hab.json'));print('ragged', d['host_api_ms'], d['host_api_all_ms'], d['feeder_gather_ms_per_call'], d['host_api_gcups'])"
