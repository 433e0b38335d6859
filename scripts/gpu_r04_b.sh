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
# a build whose tiles stop at their last column holding a code (SWK_TRIM=1) against the kept one
LIBS="main|trim" W=ragged bash scripts/gpu_lib_ab.sh || exit $?
LIBS="main|trim" W=data500 bash scripts/gpu_lib_ab.sh || exit $?
LIBS="main|trim" W=q100xdata500 bash scripts/gpu_lib_ab.sh || exit $?
ENVS="SWBANK_BAL_RAGGED=0|SWBANK_BAL_RAGGED=1" W=ragged bash scripts/gpu_env_ab.sh || exit $?
ENVS="SWBANK_WAVE_SPLIT_P=4|-" W=protein512x1k bash scripts/gpu_env_ab.sh || exit $?
ENVS="SWBANK_MQ_PAIR_ROWS=512|SWBANK_MQ_PAIR_ROWS=256" W=reads150x1k bash scripts/gpu_env_ab.sh || exit $?
for bal in 0 1; do
  SWBANK_LIB=$PWD/smith-waterman-fpga-module_amd/lib/libswbank_stamps.so timeout -k 10 300 \
    python scripts/stamps.py --bal $bal > gpurun_out/stamps_bal$bal.json || exit $?
  cat gpurun_out/stamps_bal$bal.json
done
# rank 0's N = 8 ingest (7 ranks x 4 B x 1,021,952 targets = 28.6 MB per step) as concurrent
# device-to-device copies beside the headline kernel, against none
for i in 1 2; do
for mb in 0 28.6; do
  timeout -k 10 300 python bench.py --cpu-seconds 0 --emulate-ingest $mb > gpurun_out/ingest.json 2> gpurun_out/ingest.err || { tail -5 gpurun_out/ingest.err; exit 3; }
  python -c "import json; d=json.load(open('gpurun_out/ingest.json')); print('ingest', '$mb', d['value'], d['ms_per_step'], d['kernel_ms'])"
done; done
# the ragged device batch: wave-time attribution, with the permutation and presorted
for extra in "--ragged" "--ragged --presorted" "--ragged --bal-ragged"; do
  SWBANK_LIB=$PWD/smith-waterman-fpga-module_amd/lib/libswbank_stamps.so timeout -k 10 300 \
    python scripts/stamps.py $extra > gpurun_out/stamps_r.json || exit $?
  cat gpurun_out/stamps_r.json
done
