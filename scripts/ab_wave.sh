# A/B of wave-kernel builds on the configs[4] protein workload (scratch tuning script)
set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/ab_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/ab_pytest.log; [ $rc -gt 1 ] && exit $rc
run() { # tag env...
  tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --workload protein512x1k --cpu-seconds 0 > gpurun_out/ab_$tag.json 2>gpurun_out/ab_err.log || exit 3
  echo "$tag $(python -c "import json;d=json.load(open('gpurun_out/ab_$tag.json'));print(d['value'], d['parity_sample'])")"
}
L=$PWD/smith-waterman-fpga-module_amd/lib
for i in 1 2; do
run orig SWBANK_LIB=$L/libswbank_orig.so
run new SWBANK_WAVE_BLOCK=4
done
timeout -k 10 400 python scripts/wave_sweep.py --wpb 4 --ns 12288,12500,24576 
