#!/bin/bash
# Round 5: balanced two-pairs ranges -- parity tests, then configs[4] bench lines: balanced,
# SWBANK_WAVE_BAL=0 (segmented tail) and 12,288 targets (no remainder) for reference.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 900 python -u -m pytest tests/test_gpu_wave_balanced.py tests/test_gpu_faults.py \
  tests/test_gpu_wave_half.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > "$OUT/pytest_r5c.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 "$OUT/pytest_r5c.log"; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for cfg in "bal:" "tail:SWBANK_WAVE_BAL=0" "n12288:"; do
    name=${cfg%%:*}; envs=${cfg#*:}; extra=""
    [ "$name" = n12288 ] && extra="--ptargets 12288"
    env $envs timeout -k 10 300 python bench.py --workload protein512x1k --cpu-seconds 0 $extra \
      > "$OUT/bench_r5c_${name}_$i.json" 2> "$OUT/bench_r5c_${name}_$i.err"
    rc=$?; [ $rc -eq 0 ] || { echo "bench $name rc=$rc"; tail -3 "$OUT/bench_r5c_${name}_$i.err"; exit $rc; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['kernel_ms']['score'], d['roofline']['frac'], d['kernel'][-40:], d['parity_sample'])" "$OUT/bench_r5c_${name}_$i.json" $name
  done
done
