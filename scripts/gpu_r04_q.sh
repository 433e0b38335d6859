#!/bin/bash
# Round 4: P = 4 split tail against the segmented tail at top priority, 3 alternating rounds.
set -u
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
for r in 1 2 3; do
ENVS="-|SWBANK_WAVE_SPLIT_P=8" W=protein512x1k bash scripts/gpu_env_ab.sh || exit $?
done
