#!/bin/bash
# round-3 scratch: query-set 512-row pair tables (tests + A/B vs 128 rows + PMC), protein variant matrix
set -u
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_queries.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_q.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_q.log; [ $rc -ne 0 ] && exit $rc
ENVS="-|SWBANK_MQ_PAIR_ROWS=128|SWBANK_MQ_PAIR=0" W=reads150x1k bash scripts/gpu_env_ab.sh || exit $?
bash scripts/gpu_profile.sh reads512 --workload reads150x1k || exit $?
AB_LIBS="libswbank_base.so libswbank_v0.so libswbank_vu.so libswbank_vc.so libswbank_vg.so libswbank_vh.so" W=protein512x1k ROUNDS=2 PMC=0 bash scripts/gpu_ab_pmc.sh
