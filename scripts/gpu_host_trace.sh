#!/bin/bash
# Kernel + memory-copy trace of the host-buffer API (tuning aid): the headline batch, or with
# ARGS="--bench-ragged" bench.py's ragged batch; plus the feeder's own phase trace
# (SWBANK_TRACE_FILE: host-side marks per call).  Outputs gpurun_out/host_trace/.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/host_trace; mkdir -p $O
cd /tmp && SWBANK_TRACE_FILE=$O/phases.txt timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/prof -o trace -- python3 $GRAFT_REPO_ROOT/scripts/host_api_bench.py --iters 4 --no-records ${ARGS:-} > $O/hab.json 2>$O/hab.err || exit 1
cat $O/hab.json
python3 $GRAFT_REPO_ROOT/scripts/host_timeline.py $O/prof 6 > $O/timeline.txt; cat $O/timeline.txt
