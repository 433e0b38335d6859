#!/bin/bash
# Round 4: a headline A/B of SWBANK_BAL, the VALU issue-rate
# microbenchmark (profiles/r04/valu_rate.jsonl), the in-process host A/B harness on the ragged
# and uniform host batches.  Each step time-limited; a failure ends the script.
set -u
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
ENVS="SWBANK_BAL=0|SWBANK_BAL=1" W=q100xdata500 bash scripts/gpu_env_ab.sh || exit $?
timeout -k 10 300 ./scripts/ubench/valu_rate > gpurun_out/valu_rate.jsonl || exit $?
tail -16 gpurun_out/valu_rate.jsonl
timeout -k 10 400 python scripts/host_ab.py --shape ragged --rounds 10 --calls 3 ${HOSTAB_ARGS:-} > gpurun_out/host_ab_ragged.json || exit $?
python -c "import json; d=json.load(open('gpurun_out/host_ab_ragged.json')); print({k: (v['median_ms'], v['iqr_ms'], v['best_ms'], v['median_frac_of_device']) for k, v in d['configs'].items()}, d['device_api_ms'])"
timeout -k 10 400 python scripts/host_ab.py --shape uniform --rounds 4 --calls 3 > gpurun_out/host_ab_uniform.json || exit $?
python -c "import json; d=json.load(open('gpurun_out/host_ab_uniform.json')); print({k: (v['median_ms'], v['iqr_ms'], v['best_ms'], v['median_frac_of_device']) for k, v in d['configs'].items()}, d['device_api_ms'])"
