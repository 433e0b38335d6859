#!/bin/bash
# headline: persistent grid evened out (every workgroup the same tile count) vs every slot
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
run() {
  env "$@" timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --cpu-seconds 0 \
    > gpurun_out/ge.json 2> gpurun_out/ge.err || { tail -3 gpurun_out/ge.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/ge.json')); print(sys.argv[1], d['value'], d['ms_per_step'], d['parity'] if 'parity' in d else '')" "$*"
}
for i in 1 2; do run SWBANK_GRID_EVEN=1; run SWBANK_GRID_EVEN=0; done
