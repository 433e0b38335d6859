#!/bin/bash
# Env-knob A/B on one workload (alternating, 2 rounds):
#   ENVS="X=1|X=2" W=protein512x1k bash scripts/gpu_env_ab.sh      ("-" = no extra env)
set -u
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
IFS='|' read -ra E <<< "$ENVS"
for i in 1 2; do
for e in "${E[@]}"; do
  ev=""; [ "$e" != "-" ] && ev="$e"
  env $ev timeout -k 10 300 python bench.py --cpu-seconds 0 --workload ${W:-protein512x1k} > gpurun_out/envab.json 2> gpurun_out/envab.err || { tail -5 gpurun_out/envab.err; exit 3; }
  python -c "import json; d=json.load(open('gpurun_out/envab.json')); print('$e', d['value'], d['kernel'], d['kernel_ms'], d.get('parity_sample'))"
done; done
