#!/bin/bash
# One GPU box pass: the -m gpu suite, then the headline / protein / query-set benches (JSON lines
# under gpurun_out/).  Each GPU step has its own time limit and a failure ends the script.
#   scripts/gpu_check.sh TAG [pytest -k expr]
set -u
TAG=${1:-chk}; K=${2:-}
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
if [ -n "$K" ]; then KA=(-k "$K"); else KA=(); fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 \
  --timeout-method thread "${KA[@]}" > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -ne 0 ] && exit $rc
for w in q100xdata500 protein512x1k reads150x1k; do
  timeout -k 10 300 python bench.py --workload $w --cpu-seconds 0 > gpurun_out/bench_${TAG}_$w.json \
    2> gpurun_out/bench_${TAG}_$w.err || { tail -5 gpurun_out/bench_${TAG}_$w.err; exit 3; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['kernel'], d['kernel_ms'], d['roofline']['frac'], d.get('parity_sample'))" gpurun_out/bench_${TAG}_$w.json $w
done
