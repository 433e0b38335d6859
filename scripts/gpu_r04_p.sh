#!/bin/bash
# Round 4: the segmented protein tail (SWBANK_WAVE_SPLIT_P=8) with its waves at the top issue
# priority (main) and without (tailnp), against the default P = 4 split tail.
set -u
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest "tests/test_gpu_wave_half.py::test_half_segmented_tail_policy" -x -q \
  -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_r04p.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_r04p.log; [ $rc -ne 0 ] && exit $rc
ENVS="-|SWBANK_WAVE_SPLIT_P=8" W=protein512x1k bash scripts/gpu_env_ab.sh || exit $?
SWBANK_WAVE_SPLIT_P=8 LIBS="main|tailnp" W=protein512x1k bash scripts/gpu_lib_ab.sh || exit $?
