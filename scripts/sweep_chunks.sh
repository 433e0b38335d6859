for cfg in "" "SWBANK_CHUNK_FIRST_KB=2048" "SWBANK_CHUNK_FIRST_KB=8192" "SWBANK_CHUNK_MB=24 SWBANK_CHUNK_FIRST_KB=4096" "SWBANK_CHUNK_MB=12 SWBANK_CHUNK_FIRST_KB=3072" "SWBANK_CHUNK_MB=32 SWBANK_CHUNK_FIRST_KB=4096"; do
  env $cfg timeout -k 10 120 python scripts/host_api_bench.py --iters 5 --no-records > gpurun_out/sw.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/sw.json'));print('$cfg', d['host_api_ms'], d['host_api_all_ms'], d['launches_per_call'])"
done
