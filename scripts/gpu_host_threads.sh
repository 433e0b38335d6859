# Host feeder thread count vs call-time outliers (tuning aid).
cd $GRAFT_REPO_ROOT
cat /sys/fs/cgroup/cpu.max 2>/dev/null; nproc; echo "OMP=$OMP_NUM_THREADS"; cat /sys/fs/cgroup/cpu.stat 2>/dev/null | head -6
for rep in 1 2; do
for t in 16 14 12 8; do
  SWBANK_HOST_THREADS=$t timeout -k 10 120 python scripts/host_api_bench.py --iters 10 --no-records > gpurun_out/hab.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/hab.json'));print('threads $t', d['host_api_ms'], d['host_api_all_ms'], d['feeder_gather_ms_per_call'])"
done
done
cat /sys/fs/cgroup/cpu.stat 2>/dev/null | head -6
