#!/bin/bash
# configs[4]: the wave kernel's split form for every pair (P = 2 / 4) against the default
# policy (split tail only)
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
run() {
  env "$@" timeout -k 10 200 python -u bench.py --workload protein512x1k --steps 20 --warmup 3 \
    --cpu-seconds 0 > gpurun_out/psplit.json 2> gpurun_out/psplit.err || { tail -3 gpurun_out/psplit.err; exit 1; }
  python - "$*" <<'PY'
import json, sys
d = json.load(open("gpurun_out/psplit.json"))
print(sys.argv[1] or "default", d["value"], d["ms_per_step"], d.get("config", {}).get("kernel", ""), d.get("parity", ""))
PY
}
run X=0
run SWBANK_WAVE_SPLIT=1000000 SWBANK_WAVE_SPLIT_P=2
run SWBANK_WAVE_SPLIT=1000000 SWBANK_WAVE_SPLIT_P=4
run X=0
