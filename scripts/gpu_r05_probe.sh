#!/bin/bash
# Round 5 probes, one box: (1) host-buffer figures by both methods (gpu_host_same_box.sh);
# (2) large protein batches: tile vs two-pairs wave kernel (the host's kernel choice model);
# (3) headline FETCH/WRITE with and without balanced ranges (HBM accounting).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; cd "$ROOT"
bash scripts/gpu_host_same_box.sh || exit $?
for pt in 50000 100000; do
  TAG=kc$pt ENVS="SWBANK_KERNEL=tile|SWBANK_KERNEL=wave|-" W=protein512x1k ROUNDS=1 \
    BENCH_ARGS="--ptargets $pt" bash scripts/gpu_env_ab.sh || exit $?
done
export TMPDIR=/tmp
for bal in 1 0; do
  for c in FETCH_SIZE WRITE_SIZE; do
    ( cd /tmp && SWBANK_BAL=$bal timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c --output-format csv \
      -d "$OUT/pmc_bal$bal/$c" -o pmc -- python3 "$ROOT/bench.py" --profile-only --steps 3 --warmup 1 \
      > "$OUT/pmc_bal${bal}_$c.log" 2>&1 )
    rc=$?; echo "pmc bal=$bal $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
