#!/bin/bash
# Round 4: the GPU suite on the sorted-metadata build, its A/B on the ragged batch, then the
# rotation period around the kept 2^18 on the headline, ragged and query-set shapes.
set -u
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread > gpurun_out/pytest_r04o.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_r04o.log; [ $rc -ne 0 ] && exit $rc
ENVS="SWBANK_DSORT_META=0|SWBANK_DSORT_META=1" W=ragged bash scripts/gpu_env_ab.sh || exit $?
LIBS="main|p17|p19|p20" W=q100xdata500 bash scripts/gpu_lib_ab.sh || exit $?
LIBS="main|p17|p19" W=ragged bash scripts/gpu_lib_ab.sh || exit $?
LIBS="main|p17|p19|p20" W=reads150x1k bash scripts/gpu_lib_ab.sh || exit $?
