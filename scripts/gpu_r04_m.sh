#!/bin/bash
# Round 4: balanced-range parity after the device-side uniform plan; headline and ragged lines.
set -u
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_balanced.py tests/test_gpu_abi2.py -x -q \
  -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_r04m.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_r04m.log; [ $rc -ne 0 ] && exit $rc
ENVS="-" W=q100xdata500 bash scripts/gpu_env_ab.sh || exit $?
