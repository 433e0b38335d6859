#!/bin/bash
# Library A/B on one workload (alternating, 2 rounds), each library built by
# scripts/build_variant.sh NAME (main = lib/libswbank.so):
#   LIBS="main|notrim" W=ragged bash scripts/gpu_lib_ab.sh
set -u
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
L=$PWD/smith-waterman-fpga-module_amd/lib
IFS='|' read -ra V <<< "$LIBS"
for i in 1 2; do
for v in "${V[@]}"; do
  so=$L/libswbank.so; [ "$v" != "main" ] && so=$L/libswbank_$v.so
  SWBANK_LIB=$so timeout -k 10 300 python bench.py --cpu-seconds 0 --workload ${W:-ragged} > gpurun_out/libab.json 2> gpurun_out/libab.err || { tail -5 gpurun_out/libab.err; exit 3; }
  python -c "import json; d=json.load(open('gpurun_out/libab.json')); print('$v', '${W:-ragged}', d['value'], d['kernel'], d['kernel_ms'], d.get('parity_sample'))"
done; done
