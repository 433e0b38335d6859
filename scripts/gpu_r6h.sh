set -o pipefail
cd $GRAFT_REPO_ROOT
SWBANK_WBAL_SOAK_BASE=100 SWBANK_WBAL_SOAK_SEEDS=60 SWBANK_DEAL_SOAK_BASE=100 SWBANK_DEAL_SOAK_SEEDS=60 SWBANK_FUZZ_BASE=50000 SWBANK_FUZZ_SEEDS=600 \
timeout -k 10 1000 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_wave_balanced.py tests/test_gpu_abi2.py tests/test_gpu_fuzz.py -m gpu -k "soak or fuzz" > gpurun_out/r6h_soak.log 2>&1
