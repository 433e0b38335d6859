#!/bin/bash
# One box, back to back: the host-buffer API measured by scripts/host_ab.py (12 rounds x 4
# calls, median / IQR) and by bench.py's pcie_inclusive field (15 calls after 2 warm ones), for
# the ragged and the uniform batch -- the two figures must agree.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; cd "$ROOT"
for shape in ragged uniform; do
  timeout -k 10 300 python scripts/host_ab.py --shape $shape > "$OUT/host_same_$shape.json" 2> "$OUT/host_same_$shape.err"
  rc=$?; [ $rc -eq 0 ] || { echo "host_ab $shape rc=$rc"; tail -3 "$OUT/host_same_$shape.err"; exit $rc; }
  tail -2 "$OUT/host_same_$shape.json"
  w=ragged; [ $shape = uniform ] && w=q100xdata500
  timeout -k 10 300 python bench.py --workload $w --cpu-seconds 0 > "$OUT/host_same_bench_$shape.json" 2> "$OUT/host_same_bench_$shape.err"
  rc=$?; [ $rc -eq 0 ] || { echo "bench $w rc=$rc"; tail -3 "$OUT/host_same_bench_$shape.err"; exit $rc; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print('bench', sys.argv[2], d['pcie_inclusive'])" "$OUT/host_same_bench_$shape.json" $shape
done
