# A/B of two builds of libswbank on the headline bench (scratch tuning):
#   AB_LIBS="libswbank.so libswbank_exp.so" bash scripts/ab_lib.sh
set -u
cd $GRAFT_REPO_ROOT
L=$PWD/smith-waterman-fpga-module_amd/lib
for i in 1 2 3; do
for lib in ${AB_LIBS}; do
SWBANK_LIB=$L/$lib timeout -k 10 300 python bench.py --cpu-seconds 0 ${BENCH_ARGS:-} > gpurun_out/ab.json || exit 3
python -c "import json; d=json.load(open('gpurun_out/ab.json')); print('$lib', d['value'], d['roofline']['kernel_gcups'], d['kernel'], d.get('parity_sample'))"
done; done
