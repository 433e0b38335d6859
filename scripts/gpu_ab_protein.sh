#!/bin/bash
# A/B of two libswbank builds on one workload (alternating, 3 rounds), after a parity pass of
# the second build:   AB_LIBS="libswbank.so libswbank_pf.so" W=protein512x1k bash scripts/gpu_ab_protein.sh
set -u
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
L=$PWD/smith-waterman-fpga-module_amd/lib
mkdir -p gpurun_out
set -- $AB_LIBS
SWBANK_LIB=$L/$2 timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider \
  --timeout 120 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1 || { tail -5 gpurun_out/pytest_ab.log; exit 3; }
tail -1 gpurun_out/pytest_ab.log
for i in 1 2 3; do
for lib in ${AB_LIBS}; do
SWBANK_LIB=$L/$lib timeout -k 10 300 python bench.py --cpu-seconds 0 --workload ${W:-protein512x1k} > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 3; }
python -c "import json; d=json.load(open('gpurun_out/ab.json')); print('$lib', d['value'], d['kernel_ms'], d.get('parity_sample'))"
done; done
