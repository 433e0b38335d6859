cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_gpu_fuzz.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/fuzz_split.log 2>&1; rc=$?; tail -3 gpurun_out/fuzz_split.log; exit $rc
