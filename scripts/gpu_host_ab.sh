#!/bin/bash
# Env-knob A/B of the host-buffer API (scripts/host_api_bench.py, best and all of ITERS calls),
# alternating ROUNDS rounds:   ENVS="X=0|X=1" ARGS="--bench-ragged" bash scripts/gpu_host_ab.sh
set -u
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
IFS='|' read -ra E <<< "$ENVS"
for i in $(seq 1 ${ROUNDS:-3}); do
for e in "${E[@]}"; do
  ev=""; [ "$e" != "-" ] && ev="$e"
  env $ev timeout -k 10 300 python scripts/host_api_bench.py --iters ${ITERS:-8} --no-records ${ARGS:-} \
    > gpurun_out/hostab.json 2> gpurun_out/hostab.err || { tail -5 gpurun_out/hostab.err; exit 3; }
  python -c "import json; d=json.load(open('gpurun_out/hostab.json')); print('$e', d['host_api_ms'], d['host_api_gcups'], sorted(d['host_api_all_ms'])[:4], d['kernel'][:60])"
done; done
