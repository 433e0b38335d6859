# Host-buffer API A/B on one box (tuning aid): env settings alternated, best of 6 calls each.
cd $GRAFT_REPO_ROOT
for rep in 1 2; do
for cfg in "SWBANK_CHUNK_OCC=2" "SWBANK_CHUNK_OCC=3" "SWBANK_CHUNK_OCC=0" "SWBANK_OVERLAP=0" "SWBANK_CHUNK_MB=32" "SWBANK_CHUNK_MB=8" "SWBANK_CHUNK_FIRST_KB=2048"; do
  env $cfg timeout -k 10 120 python scripts/host_api_bench.py --iters 6 --no-records > gpurun_out/hab.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/hab.json'));print('$cfg', d['host_api_ms'], d['host_api_all_ms'], d['feeder_gather_ms_per_call'], d['launches_per_call'], d['host_api_gcups'])"
done
done
SWBANK_TRACE_FILE=gpurun_out/trace_ragged.txt timeout -k 10 120 python scripts/host_api_bench.py --iters 2 --no-records --ragged --n-frac 0.001 > gpurun_out/hab.json 2>/dev/null || exit 1
