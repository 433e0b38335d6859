#!/bin/bash
# Round 4: query-set segment rows 128 / 256 (default) / 512 under rotating priorities; the
# query-set parity tests on the new default.
set -u
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_queries.py -x -q -p no:cacheprovider \
  --timeout 300 --timeout-method thread > gpurun_out/pytest_r04l.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_r04l.log; [ $rc -ne 0 ] && exit $rc
ENVS="SWBANK_MQ_PAIR_ROWS=128|-|SWBANK_MQ_PAIR_ROWS=512" W=reads150x1k bash scripts/gpu_env_ab.sh || exit $?
