#!/bin/bash
# PMC passes (separate --pmc runs, kernel-trace only) over scripts/tune.py for one case.
# usage: scripts/gpu_pmc.sh TAG "<tune.py args>"
set -u
TAG=$1; ARGS=$2
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"; export TMPDIR=/tmp; cd /tmp
for pass in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
            "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY" \
            "SQ_WAIT_INST_LDS SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM" ; do
  name=$(echo $pass | cut -d' ' -f1)
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $pass --output-format csv -d "$OUT/pmc_$TAG/$name" -o pmc \
     -- python3 "$ROOT/scripts/tune.py" $ARGS > "$OUT/pmc_${TAG}_$name.log" 2>&1
  rc=$?; echo "pmc $TAG $name rc=$rc"
  case $rc in 0) ;; 124|134|137|139) exit $rc;; *) tail -3 "$OUT/pmc_${TAG}_$name.log";; esac
done
exit 0
