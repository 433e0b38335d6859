set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_feeder.py tests/test_gpu_stream.py tests/test_gpu_abi2.py tests/test_gpu_faults.py tests/test_c_abi.py tests/test_gpu_parity.py -m gpu > gpurun_out/r6f_tests.log 2>&1
