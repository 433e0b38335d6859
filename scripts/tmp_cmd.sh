set -u
AB_LIBS="libswbank_base.so libswbank_noahead.so libswbank.so" W=protein512x1k ROUNDS=2 bash scripts/gpu_ab_pmc.sh || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "rccl_gather or bench_workloads or stream_same or memory_cap or device_range" > gpurun_out/pytest_f.log 2>&1; tail -3 gpurun_out/pytest_f.log
