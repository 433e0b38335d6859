#!/bin/bash
# The -m gpu suite twice in a row (an intermittent failure shows in either), then the benches.
set -u
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 \
  --timeout-method thread > gpurun_out/pytest_suite$i.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_suite$i.log; [ $rc -gt 1 ] && exit $rc
done
bash scripts/gpu_check.sh b "bench"
