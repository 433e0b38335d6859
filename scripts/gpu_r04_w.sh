#!/bin/bash
# Round 4: the host-buffer A/B harness on the final library (ragged 10 rounds, uniform 4).
set -u
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
timeout -k 10 400 python scripts/host_ab.py --shape ragged --rounds 10 --calls 3 > gpurun_out/host_ab_ragged_final.json || exit $?
python -c "import json; d=json.load(open('gpurun_out/host_ab_ragged_final.json')); print({k: (v['median_ms'], v['iqr_ms'], v['best_ms'], v['median_gcups'], v['median_frac_of_device']) for k, v in d['configs'].items()}, d['device_api_ms'])"
timeout -k 10 400 python scripts/host_ab.py --shape uniform --rounds 4 --calls 3 > gpurun_out/host_ab_uniform_final.json || exit $?
python -c "import json; d=json.load(open('gpurun_out/host_ab_uniform_final.json')); print({k: (v['median_ms'], v['iqr_ms'], v['best_ms'], v['median_gcups'], v['median_frac_of_device']) for k, v in d['configs'].items()}, d['device_api_ms'])"
