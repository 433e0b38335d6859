#!/bin/bash
# Library A/B (alternating rounds) on the protein workload at given target counts, each library
# built by scripts/build_variant.sh NAME (main = lib/libswbank.so):
#   LIBS="main|w8a0" PT="12500 16384" ROUNDS=2 bash scripts/gpu_lib_ab2.sh
set -u
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
L=$PWD/smith-waterman-fpga-module_amd/lib
IFS='|' read -ra V <<< "$LIBS"
for i in $(seq ${ROUNDS:-2}); do
for pt in ${PT:-12500}; do
for v in "${V[@]}"; do
  so=$L/libswbank.so; [ "$v" != "main" ] && so=$L/libswbank_$v.so
  SWBANK_LIB=$so timeout -k 10 300 python bench.py --cpu-seconds 0 --workload ${W:-protein512x1k} --ptargets $pt ${EXTRA:-} > gpurun_out/libab.json 2> gpurun_out/libab.err || { tail -5 gpurun_out/libab.err; exit 3; }
  python -c "import json; d=json.load(open('gpurun_out/libab.json')); print('$v', $pt, d['value'], d['roofline']['frac'], d['kernel'], d['kernel_ms'], d.get('parity_sample',{}).get('mismatches'))"
done; done; done
