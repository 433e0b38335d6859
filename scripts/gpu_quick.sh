#!/bin/bash
# Quick GPU iteration: the given pytest targets, then bench lines for WORKLOADS, then a
# rocprofv3 kernel trace of the first workload (each step time-limited; stops at the first
# fault / abort / timeout).   usage: scripts/gpu_quick.sh TAG "pytest targets"
set -u
TAG=$1; TESTS=${2:-}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; cd "$ROOT"
fatal() { case "$1" in 0|1) return 1;; esac; return 0; }
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -q -p no:cacheprovider --timeout 300 \
    --timeout-method thread > "$OUT/pytest_$TAG.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest_$TAG.log"; if fatal $rc; then exit $rc; fi
fi
for w in ${WORKLOADS:-q100xdata500}; do
  timeout -k 10 600 python bench.py --workload $w --cpu-seconds 0 ${BENCH_ARGS:-} > "$OUT/bench_${TAG}_$w.json" 2> "$OUT/bench_${TAG}_$w.err"
  rc=$?; if [ $rc -ne 0 ]; then echo "bench $w rc=$rc"; tail -5 "$OUT/bench_${TAG}_$w.err"; exit $rc; fi
  python - "$OUT/bench_${TAG}_$w.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
r = d["roofline"]
print(d["config"]["workload"][:60], "|", d["value"], "GCUPS", d["kernel"], d["kernel_ms"],
      "frac", r["frac"], "issue", r["issue_frac"], "pcie", d.get("pcie_inclusive", {}).get("ms"),
      d.get("parity_sample"))
PY
done
if [ -n "${PROF:-}" ]; then
  export TMPDIR=/tmp
  for w in $PROF; do
    ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$OUT/prof_${TAG}_$w" -o trace -- python3 "$ROOT/bench.py" --profile-only --workload $w ${BENCH_ARGS:-} \
      > "$OUT/prof_${TAG}_$w.log" 2>&1 )
    rc=$?; echo "rocprof $w rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
    python - "$OUT/prof_${TAG}_$w" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:8]:
    print(f"  {r['Name'][:90]:90s} calls={r['Calls']:>4} avg_us={float(r['AverageNs'])/1e3:9.2f}")
PY
  done
fi
