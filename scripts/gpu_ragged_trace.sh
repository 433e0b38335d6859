#!/bin/bash
# Host-buffer ragged batch (bench.py's ragged shape): kernel + copy trace and the feeder's host
# phase marks (SWBANK_TRACE_FILE) of the last calls.   usage: scripts/gpu_ragged_trace.sh [TAG]
set -u
TAG=${1:-rt}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$ROOT/gpurun_out/ragged_trace_$TAG; mkdir -p $O; export TMPDIR=/tmp
rm -f $O/phases.txt
cd /tmp && SWBANK_TRACE_FILE=$O/phases.txt timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace \
  --output-format csv -d $O/prof -o trace -- python3 $ROOT/scripts/host_api_bench.py --iters 6 \
  --bench-ragged > $O/hab.json 2> $O/hab.err || { tail -5 $O/hab.err; exit 1; }
cat $O/hab.json
python3 $ROOT/scripts/host_timeline.py $O/prof 6 > $O/timeline.txt; tail -60 $O/timeline.txt
awk 'BEGIN{RS="--\n"} {last=$0} END{print last}' $O/phases.txt
