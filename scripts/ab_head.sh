# A/B of the headline kernel: lib/libswbank_orig.so vs the current build (scratch tuning)
set -u
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pt.log 2>&1; rc=$?; tail -2 gpurun_out/pt.log; [ $rc -gt 1 ] && exit $rc
L=$PWD/smith-waterman-fpga-module_amd/lib
for i in 1 2 3; do
for lib in libswbank_orig.so libswbank.so; do
SWBANK_LIB=$L/$lib timeout -k 10 300 python bench.py --cpu-seconds 0 ${BENCH_ARGS:-} > gpurun_out/ab.json || exit 3
python -c "import json; d=json.load(open('gpurun_out/ab.json')); print('$lib', d['value'], d['roofline']['kernel_gcups'], d['kernel'])"
done; done
