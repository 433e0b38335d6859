#!/bin/bash
# Round 4, sixth pass: the whole GPU suite on the rotating-priority build, then ragged balanced
# ranges re-measured under it, and the host-buffer ragged path.  Each step time-limited.
set -u
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread > gpurun_out/pytest_r04f.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_r04f.log; [ $rc -ne 0 ] && exit $rc
ENVS="SWBANK_BAL_RAGGED=0|SWBANK_BAL_RAGGED=1" W=ragged bash scripts/gpu_env_ab.sh || exit $?
LIBS="main|noprio" W=data500 bash scripts/gpu_lib_ab.sh || exit $?
timeout -k 10 400 python scripts/host_ab.py --shape ragged --rounds 6 --calls 3 > gpurun_out/host_ab_ragged_f.json || exit $?
python -c "import json; d=json.load(open('gpurun_out/host_ab_ragged_f.json')); print({k: (v['median_ms'], v['iqr_ms'], v['best_ms'], v['median_gcups'], v['median_frac_of_device']) for k, v in d['configs'].items()}, d['device_api_ms'])"
