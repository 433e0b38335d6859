# bench.py's host-API (PCIe-inclusive) figure under process-environment variants (tuning aid).
cd $GRAFT_REPO_ROOT
for cfg in "X=1" "OMP_WAIT_POLICY=PASSIVE" "SWBANK_HOST_THREADS=16 OMP_NUM_THREADS=1" "X=2"; do
  env $cfg timeout -k 10 200 python bench.py --cpu-seconds 0 --steps 10 > gpurun_out/bp.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/bp.json'));print('$cfg', d['value'], d['pcie_inclusive'])"
done
timeout -k 10 120 python scripts/host_api_bench.py --iters 6 --no-records > gpurun_out/hab.json 2>/dev/null || exit 1
python -c "import json;d=json.load(open('gpurun_out/hab.json'));print('hab', d['host_api_ms'], d['host_api_all_ms'])"
