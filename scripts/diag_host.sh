set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/diag1; mkdir -p $O
timeout -k 10 120 python scripts/host_api_bench.py --iters 6 --no-records > $O/hab1.json 2>$O/hab1.err || exit 1
cat $O/hab1.json
SWBANK_TRACE_FILE=$O/trace.txt timeout -k 10 120 python scripts/host_api_bench.py --iters 3 --no-records > $O/hab2.json 2>&1 || exit 1
cat $O/hab2.json
timeout -k 10 200 python bench.py --cpu-seconds 0 > $O/bench.json 2>$O/bench.err || exit 1
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'], d['pcie_inclusive'])"
