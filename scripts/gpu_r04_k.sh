#!/bin/bash
# Round 4: query sets with 256-row (8-wave, 2 workgroups per CU, rotating priorities) segments
# against 512-row ones; the rotation against none on the 8-wave form.
set -u
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
ENVS="SWBANK_MQ_PAIR_ROWS=512|SWBANK_MQ_PAIR_ROWS=256" W=reads150x1k bash scripts/gpu_env_ab.sh || exit $?
SWBANK_MQ_PAIR_ROWS=256 LIBS="main|noprio" W=reads150x1k bash scripts/gpu_lib_ab.sh || exit $?
