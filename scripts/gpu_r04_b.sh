#!/bin/bash
# Round 4, second pass: parity of the segmented protein tail and 256-row query-set segments,
# then A/Bs (protein tail P = 4 vs 8; query sets 512 vs 256 rows), then the stamps build's
# wave-time attribution of the headline (balanced ranges on and off).  Each step time-limited.
set -u
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_wave_half.py tests/test_gpu_balanced.py \
  "tests/test_gpu_queries.py::test_query_set_pair_tables" -x -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread > gpurun_out/pytest_r04b.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_r04b.log; [ $rc -ne 0 ] && exit $rc
ENVS="SWBANK_WAVE_SPLIT_P=4|-" W=protein512x1k bash scripts/gpu_env_ab.sh || exit $?
ENVS="SWBANK_MQ_PAIR_ROWS=512|SWBANK_MQ_PAIR_ROWS=256" W=reads150x1k bash scripts/gpu_env_ab.sh || exit $?
for bal in 0 1; do
  SWBANK_LIB=$PWD/smith-waterman-fpga-module_amd/lib/libswbank_stamps.so timeout -k 10 300 \
    python scripts/stamps.py --bal $bal > gpurun_out/stamps_bal$bal.json || exit $?
  cat gpurun_out/stamps_bal$bal.json
done
