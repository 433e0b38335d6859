#!/bin/bash
# Round 4: the protein main waves rotating over priority levels 0-2 (the segmented tail on 3),
# SWK_PRIO_MAIN builds, against the kept build; the wave-half parity tests first.
set -u
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_wave_half.py -x -q \
  -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_r04r.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_r04r.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
LIBS="main|pm18|pm20" W=protein512x1k bash scripts/gpu_lib_ab.sh || exit $?
done
