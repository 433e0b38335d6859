#!/bin/bash
# rocprofv3 evidence for the bench kernel, on the GPU box: kernel trace + stats, then PMC
# counters in separate --kernel-trace-only passes (TCC slots: FETCH_SIZE and WRITE_SIZE apart).
# Each step time-limited; a fault/abort/timeout ends the script.
# usage: scripts/gpu_profile.sh TAG [bench args...]   (outputs under gpurun_out/prof_TAG*)
set -u
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"; export TMPDIR=/tmp; cd /tmp
fatal() { case "$1" in 0) return 1;; 124|134|137|139) return 0;; esac; [ "$1" -gt 128 ]; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o trace \
  -- python3 "$ROOT/bench.py" --profile-only "$@" > "$OUT/prof_$TAG.log" 2>&1
rc=$?; echo "trace rc=$rc"; tail -1 "$OUT/prof_$TAG.log"
if [ $rc -ne 0 ]; then exit $rc; fi
for pass in "FETCH_SIZE" "WRITE_SIZE" \
            "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
            "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY" \
            "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS" ; do
  name=$(echo $pass | cut -d' ' -f1)
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $pass --output-format csv \
    -d "$OUT/pmc_$TAG/$name" -o pmc -- python3 "$ROOT/bench.py" --profile-only --steps 3 --warmup 1 "$@" \
    > "$OUT/pmc_${TAG}_$name.log" 2>&1
  rc=$?; echo "pmc $name rc=$rc"
  if fatal $rc; then exit $rc; fi
done
exit 0
