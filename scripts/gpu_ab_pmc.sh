#!/bin/bash
# A/B of libswbank builds on one workload: alternating bench rounds, then the rocprofv3 kernel
# trace + PMC passes of each build (scripts/gpu_profile.sh).  Outputs under gpurun_out/.
#   AB_LIBS="libswbank_base.so libswbank.so" W=protein512x1k [ROUNDS=3] [PMC=1] bash scripts/gpu_ab_pmc.sh
set -u
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
R=$PWD; L=$R/smith-waterman-fpga-module_amd/lib
mkdir -p gpurun_out
for i in $(seq 1 ${ROUNDS:-3}); do
for lib in ${AB_LIBS}; do
SWBANK_LIB=$L/$lib timeout -k 10 300 python bench.py --cpu-seconds 0 --workload ${W:-protein512x1k} > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 3; }
python -c "import json; d=json.load(open('gpurun_out/ab.json')); print('$lib', d['value'], d['kernel_ms'], d.get('parity_sample'))"
done; done
[ "${PMC:-1}" = 1 ] || exit 0
for lib in ${AB_LIBS}; do
  t=${lib%.so}; t=${t#libswbank}; t=ab${t:-_head}
  SWBANK_LIB=$L/$lib bash scripts/gpu_profile.sh $t --workload ${W:-protein512x1k} || exit $?
done
