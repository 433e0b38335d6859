#!/bin/bash
# Round 4: progress-based priorities (SWK_PRIO_ROT=2 build) against the time rotation (main).
set -u
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
LIBS="main|pprog" W=q100xdata500 bash scripts/gpu_lib_ab.sh || exit $?
LIBS="main|pprog" W=ragged bash scripts/gpu_lib_ab.sh || exit $?
LIBS="main|pprog" W=data500 bash scripts/gpu_lib_ab.sh || exit $?
