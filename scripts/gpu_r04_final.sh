#!/bin/bash
# Round 4 final pass: round_refresh (GPU suite, smoke, every bench line, rocprofv3 kernel stats
# + PMC for four workloads), then the stamps of the final build (per-workgroup durations).
set -u
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
bash scripts/round_refresh.sh r04d || exit $?
SL=$PWD/smith-waterman-fpga-module_amd/lib/libswbank_stamps.so
SWBANK_LIB=$SL timeout -k 10 300 python scripts/stamps.py --bal 1 --dump gpurun_out/stamps_final.npy > gpurun_out/stamps_final.json || exit $?
echo stamps done
