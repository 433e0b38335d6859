set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_abi2.py tests/test_gpu_balanced.py tests/test_gpu_feeder.py -m gpu > gpurun_out/r6e_tests.log 2>&1
