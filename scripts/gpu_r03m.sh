#!/bin/bash
set -u
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_wave_half.py tests/test_gpu_split.py tests/test_gpu_fuzz.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_m.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_m.log; [ $rc -ne 0 ] && exit $rc
AB_LIBS="libswbank_h0.so libswbank.so" W=protein512x1k ROUNDS=3 PMC=0 bash scripts/gpu_ab_pmc.sh
