#!/bin/bash
# chunked host paths with and without the tapered last chunk (SWBANK_CHUNK_TAIL)
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
one() {  # label extra-env...
  local lab=$1; shift
  env "$@" timeout -k 10 120 python -u scripts/host_api_bench.py --iters 10 $ARGS > gpurun_out/ct.log 2>&1 \
    || { echo "$lab failed"; tail -3 gpurun_out/ct.log; exit 1; }
  python - "$lab" <<'PY'
import json, sys, statistics
d = json.loads(open("gpurun_out/ct.log").read().strip().splitlines()[-1])
a = d["host_api_all_ms"]
print(sys.argv[1], "min", min(a), "median", statistics.median(a), "records", d.get("records_api_ms"))
PY
}
for r in 1 2; do
  ARGS="--ragged --no-records" one "ragged tail=0" SWBANK_CHUNK_TAIL=0
  ARGS="--ragged --no-records" one "ragged tail=1" SWBANK_CHUNK_TAIL=1
  ARGS="" one "uniform-chunked tail=0" SWBANK_STREAM=0 SWBANK_CHUNK_TAIL=0
  ARGS="" one "uniform-chunked tail=1" SWBANK_STREAM=0 SWBANK_CHUNK_TAIL=1
done
