#!/bin/bash
# Alternating bench lines of environment settings: ENVS="A=1|A=0" W=workload [ROUNDS=2]
# [TESTS="pytest targets" run first] [BENCH_ARGS=...].  Outputs gpurun_out/ab_<TAG>_*.json.
set -u
TAG=${TAG:-ab}; ROUNDS=${ROUNDS:-2}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; cd "$ROOT"
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -x -q -p no:cacheprovider --timeout 300 \
    --timeout-method thread > "$OUT/pytest_$TAG.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest_$TAG.log"; [ $rc -eq 0 ] || exit $rc
fi
IFS='|' read -ra E <<< "$ENVS"
for r in $(seq 1 $ROUNDS); do
  for i in "${!E[@]}"; do
    ev=""; [ "${E[$i]}" != "-" ] && ev="${E[$i]}"
    env $ev timeout -k 10 300 python bench.py --workload $W --cpu-seconds 0 ${BENCH_ARGS:-} \
      > "$OUT/ab_${TAG}_${i}_$r.json" 2> "$OUT/ab_${TAG}_${i}_$r.err"
    rc=$?; [ $rc -eq 0 ] || { echo "bench ${E[$i]} rc=$rc"; tail -3 "$OUT/ab_${TAG}_${i}_$r.err"; exit $rc; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['kernel_ms']['score'], d['roofline']['frac'], d['parity_sample']['mismatches'], (d.get('pcie_inclusive') or {}).get('ms'), d['kernel'][-50:])" "$OUT/ab_${TAG}_${i}_$r.json" "${E[$i]}"
  done
done
