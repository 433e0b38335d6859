#!/bin/bash
# round-3 scratch: the full GPU suite on the working-tree library, then protein A/B vs base
set -u
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_k.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_k.log; [ $rc -ne 0 ] && exit $rc
AB_LIBS="libswbank_base.so libswbank.so libswbank_vp.so" W=protein512x1k ROUNDS=3 PMC=0 bash scripts/gpu_ab_pmc.sh
ENVS="-|SWBANK_WAVE_HALF=0" W=protein512x1k bash scripts/gpu_env_ab.sh
