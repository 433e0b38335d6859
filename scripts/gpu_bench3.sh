#!/bin/bash
# Full GPU tests, then the headline / ragged / data500 benches (each step time-limited; a
# fault, abort or timeout ends the script).  usage: scripts/gpu_bench3.sh TAG
set -u
TAG=${1:-r02}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT"
fatal() { case "$1" in 0|1) return 1;; esac; return 0; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread > "$OUT/pytest_gpu_$TAG.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest_gpu_$TAG.log"; if fatal $rc; then exit $rc; fi
for w in ${WORKLOADS:-q100xdata500 ragged data500}; do
  timeout -k 10 600 python bench.py --workload $w ${BENCH_ARGS:-} > "$OUT/bench_${TAG}_$w.json" 2> "$OUT/bench_${TAG}_$w.err"
  rc=$?; echo "bench $w rc=$rc"; cut -c1-400 "$OUT/bench_${TAG}_$w.json"; if [ $rc -ne 0 ]; then tail -5 "$OUT/bench_${TAG}_$w.err"; exit $rc; fi
done
