#!/bin/bash
# Bench lines over libswbank builds x bench argument sets, alternating, one JSON summary line
# each (value, score-kernel ms, parity).  Outputs under gpurun_out/.
#   LIBS="libswbank.so libswbank_x.so" ARGS="--workload protein512x1k --ptargets 12288|..." \
#     [ROUNDS=2] bash scripts/gpu_sweep.sh
set -u
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
L=$PWD/smith-waterman-fpga-module_amd/lib
mkdir -p gpurun_out
IFS='|' read -ra SETS <<< "$ARGS"
for i in $(seq 1 ${ROUNDS:-2}); do
for a in "${SETS[@]}"; do
for lib in ${LIBS}; do
SWBANK_LIB=$L/$lib timeout -k 10 300 python bench.py --cpu-seconds 0 $a > gpurun_out/sw.json 2> gpurun_out/sw.err || { tail -5 gpurun_out/sw.err; exit 3; }
python -c "import json; d=json.load(open('gpurun_out/sw.json')); print('$lib', '$a', d['value'], d['kernel_ms'], d.get('parity_sample'), d['kernel'])"
done; done; done
