#!/bin/bash
# Round 4: balanced ranges on / off under the priority rotation (headline, data500, ragged).
set -u
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
for r in 1 2; do
ENVS="SWBANK_BAL=0|SWBANK_BAL=1" W=q100xdata500 bash scripts/gpu_env_ab.sh || exit $?
done
ENVS="SWBANK_BAL=0|SWBANK_BAL=1" W=ragged bash scripts/gpu_env_ab.sh || exit $?
