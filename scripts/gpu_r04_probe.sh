#!/bin/bash
# Round-4 probes: headline batch sizes around the persistent grid's quantisation (998 vs 1,024
# workgroups) and the protein tail (12,288 vs 12,500 targets).  Each step time-limited.
set -u
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
run() {  # tag, args...
  local tag=$1; shift
  timeout -k 10 300 python bench.py --cpu-seconds 0 "$@" > gpurun_out/probe_$tag.json 2> gpurun_out/probe_$tag.err \
    || { tail -5 gpurun_out/probe_$tag.err; exit 3; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['kernel'], d['kernel_ms']['score'], d['roofline']['frac'], d.get('parity_sample'))" gpurun_out/probe_$tag.json $tag
}
for i in 1 2; do
  run q1021952 --targets 1021952
  run q1048576 --targets 1048576
  run q1044480 --targets 1044480
  run p12500 --workload protein512x1k --ptargets 12500
  run p12288 --workload protein512x1k --ptargets 12288
done
