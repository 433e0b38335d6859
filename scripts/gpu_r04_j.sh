#!/bin/bash
# Round 4: stage priorities in the 16-wave query-set workgroups (SWK_PRIO_STAGE builds).
set -u
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
LIBS="main|sup|sdown" W=reads150x1k bash scripts/gpu_lib_ab.sh || exit $?
