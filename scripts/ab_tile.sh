# A/B of tile-kernel builds on protein shapes: lib/libswbank_orig.so vs current (scratch tuning)
set -u
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pt.log 2>&1; rc=$?; tail -2 gpurun_out/pt.log; [ $rc -gt 1 ] && exit $rc
L=$PWD/smith-waterman-fpga-module_amd/lib
for i in 1 2; do
for lib in libswbank_orig.so libswbank.so; do
echo $lib
SWBANK_LIB=$L/$lib timeout -k 10 300 python scripts/wave_sweep.py --kernel tile --qlen 128 --L 300 --ns 131072 --wpb 4 || exit 3
SWBANK_LIB=$L/$lib timeout -k 10 300 python scripts/wave_sweep.py --kernel tile --qlen 256 --L 300 --ns 65536 --wpb 4 || exit 3
done; done
