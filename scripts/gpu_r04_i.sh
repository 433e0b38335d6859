#!/bin/bash
# Round 4: faster priority rotation over the last part of each workgroup's phases (SWK_PRIO_END
# builds eXfY: 2^X times faster over the last 1/2^Y) against the kept rotation.
set -u
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
LIBS="main|e2f3|e3f3|e2f2|e3f4" W=q100xdata500 bash scripts/gpu_lib_ab.sh || exit $?
LIBS="main|e2f3|e3f3|e2f2|e3f4" W=ragged bash scripts/gpu_lib_ab.sh || exit $?
