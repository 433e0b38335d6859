#!/bin/bash
# host path vs feeder thread count (CPU-quota headroom), min and median of 10 calls:
# streamed uniform, chunked uniform (SWBANK_STREAM=0), ragged
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
one() {  # label threads extra-args...
  local lab=$1 t=$2; shift 2
  env SWBANK_HOST_THREADS=$t $ENVX timeout -k 10 120 python -u scripts/host_api_bench.py --iters 10 --no-records "$@" \
    > gpurun_out/ht.log 2>&1 || { echo "$lab $t failed"; tail -3 gpurun_out/ht.log; exit 1; }
  python - "$lab" $t <<'PY'
import json, sys, statistics
d = json.loads(open("gpurun_out/ht.log").read().strip().splitlines()[-1])
a = d["host_api_all_ms"]
print(sys.argv[1], "threads", sys.argv[2], "min", min(a), "median", statistics.median(a), "gather", d["feeder_gather_ms_per_call"])
PY
}
for r in 1 2; do
  for t in 16 12; do ENVX= one streamed $t; done
  for t in 16 12; do ENVX=SWBANK_STREAM=0 one chunked $t; done
  for t in 16 12; do ENVX= one ragged $t --ragged; done
done
