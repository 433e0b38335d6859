#!/bin/bash
# Round 4: priority rotation counted in phases (SWK_PRIO_PHASE builds) against the clock-based one.
set -u
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
for r in 1 2; do
LIBS="main|ph3|ph4|ph5" W=q100xdata500 bash scripts/gpu_lib_ab.sh || exit $?
done
LIBS="main|ph3|ph4|ph5" W=ragged bash scripts/gpu_lib_ab.sh || exit $?
