#!/bin/bash
# ragged host path: streamed (one kernel per call) vs the chunked feeder, min and median of 10
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for r in 1 2 3; do
  for s in 1 0; do
    SWBANK_STREAM_RAGGED=$s timeout -k 10 120 python -u scripts/host_api_bench.py --iters 10 --ragged --no-records \
      > gpurun_out/rs.log 2>&1 || { echo "ragged $s failed"; tail -3 gpurun_out/rs.log; exit 1; }
    python - $s <<'PY'
import json, sys, statistics
d = json.loads(open("gpurun_out/rs.log").read().strip().splitlines()[-1])
a = d["host_api_all_ms"]
print("STREAM_RAGGED", sys.argv[1], "min", min(a), "median", statistics.median(a), "gather", d["feeder_gather_ms_per_call"], d["kernel"])
PY
  done
done
timeout -k 10 200 python -u scripts/stream_trace.py --ragged > gpurun_out/rtrace.log 2>&1 && grep -v amdgpu.ids gpurun_out/rtrace.log | cut -c1-1500
