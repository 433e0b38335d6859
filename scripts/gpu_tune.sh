#!/bin/bash
# Variant sweep + PMC counter passes on the GPU box (each step time-limited, stop on fault).
set -u
TAG=${1:-tune}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 600 python scripts/tune.py ${TUNE_ARGS:-} > "$OUT/tune_$TAG.jsonl" 2> "$OUT/tune_$TAG.err"
rc=$?; echo "tune rc=$rc"; cat "$OUT/tune_$TAG.jsonl"; tail -3 "$OUT/tune_$TAG.err"
[ $rc -ne 0 ] && exit $rc
export TMPDIR=/tmp
cd /tmp
rocprofv3 -L > "$OUT/counters_avail.txt" 2>&1 || true
for pass in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
            "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VALU" \
            "FETCH_SIZE" "WRITE_SIZE" ; do
  name=$(echo $pass | cut -d' ' -f1)
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $pass --output-format csv -d "$OUT/pmc_$TAG/$name" -o pmc \
     -- python3 "$ROOT/bench.py" --profile-only --steps 3 --warmup 1 > "$OUT/pmc_${TAG}_$name.log" 2>&1
  rc=$?; echo "pmc $name rc=$rc"; tail -2 "$OUT/pmc_${TAG}_$name.log"
  case $rc in 0) ;; 124|134|137|139) exit $rc;; *) ;; esac
done
exit 0
