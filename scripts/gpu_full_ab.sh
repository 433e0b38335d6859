#!/bin/bash
# Full GPU suite on the working-tree library; on a failure, the same suite (minus the streamed
# tests) on the HEAD library (ablib/) for comparison.  Then the host-API and default benches.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/gpu_all.log 2>&1
rc=$?; echo "cur rc=$rc"; tail -4 gpurun_out/gpu_all.log
if [ $rc -ne 0 ]; then
  [ $rc -eq 1 ] || exit $rc
  if [ -f ablib/libswbank_head.so ]; then
    SWBANK_LIB=$PWD/ablib/libswbank_head.so timeout -k 10 600 python -u -m pytest tests -m gpu -q \
      --timeout 120 --timeout-method thread --deselect tests/test_gpu_stream.py \
      --ignore tests/test_gpu_stream.py > gpurun_out/gpu_all_head.log 2>&1
    echo "head rc=$?"; tail -4 gpurun_out/gpu_all_head.log
  fi
  exit 1
fi
timeout -k 10 300 python -u scripts/host_api_bench.py --iters 5 --no-records > gpurun_out/hab.log 2>&1 \
  && tail -1 gpurun_out/hab.log | cut -c1-400
timeout -k 10 300 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
rc=$?; cut -c1-300 gpurun_out/bench_default.json
python -c "import json;d=json.load(open('gpurun_out/bench_default.json'));print(d.get('pcie_inclusive'))"
exit $rc
