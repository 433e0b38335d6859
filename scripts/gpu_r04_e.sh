#!/bin/bash
# Round 4, fifth pass: the rotation period of the wave priorities (SWK_PRIO_SHIFT, main = 19)
# on the headline, ragged and protein, against no rotation; stamps of the main build.
set -u
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
LIBS="main|p18|p20|p21|p22|noprio" W=q100xdata500 bash scripts/gpu_lib_ab.sh || exit $?
LIBS="main|p21|noprio" W=ragged bash scripts/gpu_lib_ab.sh || exit $?
LIBS="main|p21|noprio" W=protein512x1k bash scripts/gpu_lib_ab.sh || exit $?
SL=$PWD/smith-waterman-fpga-module_amd/lib/libswbank_stamps.so
SWBANK_LIB=$SL timeout -k 10 300 python scripts/stamps.py --bal 1 --dump gpurun_out/stamps_p19.npy > gpurun_out/stamps_p19.json || exit $?
echo stamps done
