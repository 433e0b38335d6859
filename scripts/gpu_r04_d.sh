#!/bin/bash
# Round 4, fourth pass: rotating wave priorities in the tile kernel (SWK_PRIO_ROT) against the
# build without them, on the headline, ragged, data500 and reads; the rotation period; the
# stamps of the rotated build.  Each step time-limited.
set -u
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_balanced.py -x -q -p no:cacheprovider \
  --timeout 300 --timeout-method thread > gpurun_out/pytest_r04d.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_r04d.log; [ $rc -ne 0 ] && exit $rc
LIBS="main|noprio|prio14|prio19" W=q100xdata500 bash scripts/gpu_lib_ab.sh || exit $?
LIBS="main|noprio" W=ragged bash scripts/gpu_lib_ab.sh || exit $?
LIBS="main|noprio" W=reads150x1k bash scripts/gpu_lib_ab.sh || exit $?
SL=$PWD/smith-waterman-fpga-module_amd/lib/libswbank_stamps.so
SWBANK_LIB=$SL timeout -k 10 300 python scripts/stamps.py --bal 1 --dump gpurun_out/stamps_prio.npy > gpurun_out/stamps_prio.json || exit $?
SWBANK_LIB=$SL timeout -k 10 300 python scripts/stamps.py --ragged --dump gpurun_out/stamps_prio_ragged.npy > gpurun_out/stamps_prio_ragged.json || exit $?
echo stamps done
