# Kernel + memory-copy trace of the host-buffer API on the headline batch (tuning aid).
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/host_trace; mkdir -p $O
cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/prof -o trace -- python3 $GRAFT_REPO_ROOT/scripts/host_api_bench.py --iters 4 --no-records > $O/hab.json 2>$O/hab.err || exit 1
cat $O/hab.json
python3 $GRAFT_REPO_ROOT/scripts/host_timeline.py $O/prof 6 > $O/timeline.txt; cat $O/timeline.txt
