#!/bin/bash
# configs[4]: the wave kernel's split-tail policy (P = 2 / 4 for the tail, no split, every
# pair split) against the default
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
run() {
  env "$@" timeout -k 10 200 python -u bench.py --workload protein512x1k --steps 20 --warmup 3 \
    --cpu-seconds 0 > gpurun_out/psplit.json 2> gpurun_out/psplit.err || { tail -3 gpurun_out/psplit.err; exit 1; }
  python - "$*" <<'PY'
import json, sys
d = json.load(open("gpurun_out/psplit.json"))
print(sys.argv[1] or "default", d["value"], d["ms_per_step"], d.get("parity", ""))
PY
}
for i in 1 2; do
run X=0
run SWBANK_WAVE_SPLIT_P=2
run SWBANK_WAVE_SPLIT=0
done
