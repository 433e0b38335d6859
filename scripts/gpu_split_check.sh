# Split-tail parity tests, then the protein wave-kernel sweep with P = 2 and P = 4 (tuning aid).
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_split.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/split_tests.log 2>&1; rc=$?; tail -30 gpurun_out/split_tests.log; [ $rc -ne 0 ] && exit $rc
for p in 2 4; do
  SWBANK_WAVE_SPLIT_P=$p timeout -k 10 200 python scripts/wave_sweep.py --ns 12288,12500,13312,12800 --wpb 4 --iters 10 2>&1 | grep qlen || exit 1
done
