cd $GRAFT_REPO_ROOT
SWBANK_TRACE_FILE=gpurun_out/trace_ragged2.txt timeout -k 10 120 python scripts/host_api_bench.py --iters 2 --no-records --ragged --n-frac 0.001 > gpurun_out/hab_r.json 2>/dev/null || exit 1
SWBANK_TRACE_FILE=gpurun_out/trace_uniform2.txt timeout -k 10 120 python scripts/host_api_bench.py --iters 2 --no-records > gpurun_out/hab_u.json 2>/dev/null || exit 1
cat gpurun_out/hab_r.json gpurun_out/hab_u.json
