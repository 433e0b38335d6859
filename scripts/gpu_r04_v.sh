#!/bin/bash
# Round 4: faster end-of-range rotation variants (SWK_PRIO_END / _FRAC) against the kept e3f4.
set -u
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
for r in 1 2; do
LIBS="main|e4f4|e5f4|e4f3" W=q100xdata500 bash scripts/gpu_lib_ab.sh || exit $?
done
LIBS="main|e4f4|e5f4|e4f3" W=ragged bash scripts/gpu_lib_ab.sh || exit $?
