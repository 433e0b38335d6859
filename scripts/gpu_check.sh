#!/bin/bash
# One GPU-box session: parity tests, bench, rocprofv3 kernel trace.  Each GPU step has its own
# time limit; a fault/abort/timeout ends the script (no retries).  Test FAILURES (exit 1) do
# not stop the bench, so one call yields both.
# usage: scripts/gpu_check.sh [tag]
set -u
TAG=${1:-r01}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT"
fatal() { case "$1" in 124|134|137|139) return 0;; esac; [ "$1" -gt 128 ] && return 0; return 1; }

echo "[gpu_check] pytest -m gpu" | tee "$OUT/steps.log"
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > "$OUT/pytest_gpu_$TAG.log" 2>&1
rc=$?; echo "pytest rc=$rc" | tee -a "$OUT/steps.log"; tail -5 "$OUT/pytest_gpu_$TAG.log"
if fatal $rc; then echo "fatal after pytest"; exit $rc; fi

echo "[gpu_check] smoke" | tee -a "$OUT/steps.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1
rc=$?; echo "smoke rc=$rc" | tee -a "$OUT/steps.log"; tail -2 "$OUT/smoke_$TAG.log"
if fatal $rc; then exit $rc; fi

echo "[gpu_check] bench" | tee -a "$OUT/steps.log"
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err"
rc=$?; echo "bench rc=$rc" | tee -a "$OUT/steps.log"; cat "$OUT/bench_$TAG.json"; tail -5 "$OUT/bench_$TAG.err"
if [ $rc -ne 0 ]; then exit $rc; fi

echo "[gpu_check] rocprofv3 kernel trace" | tee -a "$OUT/steps.log"
export TMPDIR=/tmp
( cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$OUT/prof_$TAG" -o trace -- python3 "$ROOT/bench.py" --profile-only ${BENCH_ARGS:-} \
    > "$OUT/prof_$TAG.log" 2>&1 )
rc=$?; echo "rocprof rc=$rc" | tee -a "$OUT/steps.log"; tail -3 "$OUT/prof_$TAG.log"
find "$OUT/prof_$TAG" -name "*stats*" | head
exit $rc
