#!/bin/bash
# Round 4: the bench-flow GPU tests after the segmented-tail default.
set -u
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench.py tests/test_gpu_wave_half.py -x -q \
  -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_r04s.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_r04s.log; exit $rc
