#!/bin/bash
# Round 4: rotation period around the kept 2^18 on the headline, ragged and query-set shapes.
set -u
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
LIBS="main|p17|p19|p20" W=q100xdata500 bash scripts/gpu_lib_ab.sh || exit $?
LIBS="main|p17|p19|p20" W=reads150x1k bash scripts/gpu_lib_ab.sh || exit $?
LIBS="main|p17|p19" W=ragged bash scripts/gpu_lib_ab.sh || exit $?
