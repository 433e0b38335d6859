# Host-API timing vs hardware queue count (tuning aid: do the feeder's 4 streams share queues?).
cd $GRAFT_REPO_ROOT
for rep in 1 2; do
for cfg in "GPU_MAX_HW_QUEUES=4" "GPU_MAX_HW_QUEUES=8"; do
  env $cfg timeout -k 10 120 python scripts/host_api_bench.py --iters 8 --no-records > gpurun_out/hab.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/hab.json'));print('$cfg', d['host_api_ms'], d['host_api_all_ms'], d['feeder_gather_ms_per_call'])"
done
done
