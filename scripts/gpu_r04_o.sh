#!/bin/bash
# Round 4: the device sort writing offsets / lengths in its order (SWBANK_DSORT_META): the GPU
# suite, then A/B on the ragged device batch.
set -u
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread > gpurun_out/pytest_r04o.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_r04o.log; [ $rc -ne 0 ] && exit $rc
ENVS="SWBANK_DSORT_META=0|SWBANK_DSORT_META=1" W=ragged bash scripts/gpu_env_ab.sh || exit $?
ENVS="SWBANK_DSORT_META=0|SWBANK_DSORT_META=1" W=ragged bash scripts/gpu_env_ab.sh || exit $?
