#!/bin/bash
# Round 4, third pass: balanced ranges with the plan read once and the head flag deferred
# (parity, then A/B on the headline and the ragged batch), the stamps attribution with per-XCC
# clocks, the protein default (P = 4 split tail).  Each step time-limited.
set -u
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_balanced.py \
  "tests/test_gpu_wave_half.py::test_half_segmented_tail_policy" -x -q -p no:cacheprovider \
  --timeout 300 --timeout-method thread > gpurun_out/pytest_r04c.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_r04c.log; [ $rc -ne 0 ] && exit $rc
ENVS="SWBANK_BAL=0|SWBANK_BAL=1" W=q100xdata500 bash scripts/gpu_env_ab.sh || exit $?
ENVS="SWBANK_BAL_RAGGED=0|SWBANK_BAL_RAGGED=1" W=ragged bash scripts/gpu_env_ab.sh || exit $?
ENVS="-" W=protein512x1k bash scripts/gpu_env_ab.sh || exit $?
SL=$PWD/smith-waterman-fpga-module_amd/lib/libswbank_stamps.so
for bal in 0 1; do
  SWBANK_LIB=$SL timeout -k 10 300 python scripts/stamps.py --bal $bal --dump gpurun_out/stamps_bal$bal.npy > gpurun_out/stamps_bal$bal.json || exit $?
  cat gpurun_out/stamps_bal$bal.json
done
for extra in "--ragged" "--ragged --bal-ragged" "--ragged --presorted"; do
  tag=$(echo $extra | tr -d ' -')
  SWBANK_LIB=$SL timeout -k 10 300 python scripts/stamps.py $extra --dump gpurun_out/stamps_$tag.npy > gpurun_out/stamps_$tag.json || exit $?
  cat gpurun_out/stamps_$tag.json
done
