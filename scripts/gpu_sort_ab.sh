#!/bin/bash
# Device-sort kernel A/B: rocprofv3 kernel stats of the ragged bench per library variant
# (scripts/build_variant.sh NAME; main = lib/libswbank.so), alternating ROUNDS rounds:
#   LIBS="main|si4" ROUNDS=2 bash scripts/gpu_sort_ab.sh
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp; cd /tmp
L=$ROOT/smith-waterman-fpga-module_amd/lib
IFS='|' read -ra V <<< "$LIBS"
for i in $(seq ${ROUNDS:-2}); do
for v in "${V[@]}"; do
  so=$L/libswbank.so; [ "$v" != "main" ] && so=$L/libswbank_$v.so
  d=$OUT/sortab_${v}_$i; rm -rf $d
  SWBANK_LIB=$so timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o t \
    -- python3 $ROOT/bench.py --profile-only --workload ${W:-ragged} --steps 20 > $d.log 2>&1 \
    || { echo "$v rc=$?"; tail -3 $d.log; exit 3; }
  python3 - "$d" "$v" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
r = {x["Name"].split("(")[0].split("<")[0].split("::")[-1]: float(x["AverageNs"]) / 1e3
     for x in csv.DictReader(open(f))}
print(sys.argv[2], {k: round(v, 2) for k, v in r.items() if "sort" in k or "score" in k})
PY
done; done
