set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_wave_balanced.py tests/test_gpu_wave_half.py tests/test_gpu_fuzz.py tests/test_gpu_faults.py -m gpu > gpurun_out/r6g_tests.log 2>&1 && \
LIBS="main|noabs" PT="12500 16384 100000" ROUNDS=2 timeout -k 10 500 bash scripts/gpu_lib_ab2.sh > gpurun_out/r6g_ab.txt 2>&1
