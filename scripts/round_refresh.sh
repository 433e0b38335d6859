#!/bin/bash
# Round-end evidence on one GPU box: parity tests, smoke, the three bench workloads, rocprofv3
# kernel trace of the headline bench and its PMC passes (scripts/gpu_profile.sh).  Each GPU
# step has its own time limit; a fault/abort/timeout ends the script.
# usage: scripts/round_refresh.sh TAG      (outputs under gpurun_out/)
set -u
TAG=${1:-r01}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT"
fatal() { case "$1" in 0|1) return 1;; esac; return 0; }
step() { echo "[refresh] $1 rc=$2"; }
# PHASES: which parts run (default all; a gpurun call is capped at 20 minutes, so a refresh
# can be split: PHASES="tests bench" then PHASES="prof")
PHASES=${PHASES:-"tests bench prof"}
if [[ " $PHASES " == *" tests "* ]]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/pytest_gpu_$TAG.log" 2>&1
rc=$?; step pytest $rc; tail -2 "$OUT/pytest_gpu_$TAG.log"; if fatal $rc; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1
rc=$?; step smoke $rc; tail -1 "$OUT/smoke_$TAG.log"; if [ $rc -ne 0 ]; then exit $rc; fi
fi
if [[ " $PHASES " == *" bench "* ]]; then
for w in q100xdata500 reads150x1k protein512x1k ragged data500; do
  extra=""; [ $w = reads150x1k ] && extra="--full-parity"  # every pair re-checked (~30 s)
  timeout -k 10 600 python bench.py --workload $w $extra > "$OUT/bench_${TAG}_$w.json" 2> "$OUT/bench_${TAG}_$w.err"
  rc=$?; step "bench $w" $rc; cut -c1-200 "$OUT/bench_${TAG}_$w.json"; if [ $rc -ne 0 ]; then exit $rc; fi
done
# configs[4]'s whole 100k-target batch on one GPU (8-wave blocks, 4 waves per SIMD)
timeout -k 10 600 python bench.py --workload protein512x1k --ptargets 100000 > "$OUT/bench_${TAG}_protein100k.json" 2> "$OUT/bench_${TAG}_protein100k.err"
rc=$?; step "bench protein100k" $rc; cut -c1-200 "$OUT/bench_${TAG}_protein100k.json"; if [ $rc -ne 0 ]; then exit $rc; fi
fi
[[ " $PHASES " == *" prof "* ]] || exit 0
bash scripts/gpu_profile.sh "$TAG"
rc=$?; step profile $rc; if [ $rc -ne 0 ]; then exit $rc; fi
bash scripts/gpu_profile.sh "${TAG}_protein" --workload protein512x1k
rc=$?; step profile_protein $rc; if [ $rc -ne 0 ]; then exit $rc; fi
bash scripts/gpu_profile.sh "${TAG}_reads" --workload reads150x1k
rc=$?; step profile_reads $rc; if [ $rc -ne 0 ]; then exit $rc; fi
bash scripts/gpu_profile.sh "${TAG}_ragged" --workload ragged
rc=$?; step profile_ragged $rc; if [ $rc -ne 0 ]; then exit $rc; fi
bash scripts/gpu_profile.sh "${TAG}_protein100k" --workload protein512x1k --ptargets 100000
rc=$?; step profile_protein100k $rc
exit $rc
