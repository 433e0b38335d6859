#!/bin/bash
# Host-buffer API A/B of library variants (scripts/build_variant.sh NAME; main = lib/libswbank.so),
# alternating ROUNDS rounds:  LIBS="main|v1" ARGS="--qlen 100" bash scripts/gpu_host_lib_ab.sh
set -u
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
L=$PWD/smith-waterman-fpga-module_amd/lib
IFS='|' read -ra V <<< "$LIBS"
for i in $(seq ${ROUNDS:-3}); do
for v in "${V[@]}"; do
  so=$L/libswbank.so; [ "$v" != "main" ] && so=$L/libswbank_$v.so
  SWBANK_LIB=$so timeout -k 10 300 python scripts/host_api_bench.py --iters ${ITERS:-15} --no-records ${ARGS:-} \
    > gpurun_out/hostlab.json 2> gpurun_out/hostlab.err || { tail -5 gpurun_out/hostlab.err; exit 3; }
  python -c "import json; d=json.load(open('gpurun_out/hostlab.json')); a=sorted(d['host_api_all_ms']); print('$v', d['host_api_ms'], 'median', a[len(a)//2], a[:3], d['kernel'][:60])"
done; done
