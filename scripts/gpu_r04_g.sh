#!/bin/bash
# Round 4: priorities in the two-pairs protein kernel (split-tail waves on top, main waves
# rotating over 3 levels; SWK_PRIO_WAVE builds) against the kept build.
set -u
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
LIBS="main|pw16|pw18|pw20" W=protein512x1k bash scripts/gpu_lib_ab.sh || exit $?
