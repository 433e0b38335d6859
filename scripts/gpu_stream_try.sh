#!/bin/bash
# streamed host batches: parity tests, then the host-API A/B (chunked vs streamed)
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_stream.py > gpurun_out/stream_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/stream_tests.log
[ $rc -eq 0 ] || exit $rc
for s in 0 1 0 1; do
  SWBANK_STREAM=$s timeout -k 10 120 python -u scripts/host_api_bench.py --iters 5 --no-records \
    > gpurun_out/stream_ab_$s.log 2>&1 || { echo "bench $s failed"; tail -5 gpurun_out/stream_ab_$s.log; exit 1; }
  echo "STREAM=$s"; tail -3 gpurun_out/stream_ab_$s.log
done
SWBANK_STREAM=1 timeout -k 10 120 python -u scripts/host_api_bench.py --iters 5 --no-records --n-frac 0.001 \
  > gpurun_out/stream_ab_n.log 2>&1 && { echo "STREAM=1 nfrac"; tail -3 gpurun_out/stream_ab_n.log; }
timeout -k 10 200 python -u scripts/stream_trace.py > gpurun_out/stream_trace.log 2>&1 && grep -v amdgpu.ids gpurun_out/stream_trace.log | cut -c1-900
