set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_c_abi.py tests/test_gpu_bench.py tests/test_gpu_wave_balanced.py tests/test_gpu_faults.py tests/test_gpu_abi2.py -m gpu > gpurun_out/r6a_tests.log 2>&1 && \
timeout -k 10 200 python bench.py > gpurun_out/r6a_bench.json 2> gpurun_out/r6a_bench.err
