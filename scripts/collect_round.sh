# After scripts/round_refresh.sh TAG ran on the GPU box (its gpurun_out/ merged back here):
# copy the bench lines, the GPU test log, the rocprofv3 kernel stats and the PMC summaries into
# profiles/TAG/ and print the figures DESIGN.md quotes.
# usage: bash scripts/collect_round.sh TAG
set -eu
TAG=${1:-r01}
cd "$(dirname "$0")/.."
O=gpurun_out
# the workload names are bench.py's Workload.name (its pmc_traffic() matches on them)
python scripts/collect_profiles.py "$TAG" $O/prof_$TAG $O/pmc_$TAG query100x1021952x128 > /dev/null
python scripts/collect_profiles.py "$TAG" $O/prof_${TAG}_protein $O/pmc_${TAG}_protein \
  protein512x12500x1k score_wave protein > /dev/null
if [ -d $O/prof_${TAG}_reads ]; then
  python scripts/collect_profiles.py "$TAG" $O/prof_${TAG}_reads $O/pmc_${TAG}_reads \
    reads150x131072x1k16 score_kernel reads > /dev/null
  python scripts/pmc_decompose.py profiles/$TAG/pmc_summary_reads150x131072x1k16.json \
    $((125 * 16 * 131072 * 150)) profiles/$TAG/pmc_decomposition_reads.json | grep -E "valu_instr|valu_busy"
fi
python scripts/pmc_decompose.py profiles/$TAG/pmc_summary.json $((128 * 1021952 * 128)) \
  profiles/$TAG/pmc_decomposition.json | grep -E "valu_instr|valu_busy|kernel_ms"
python scripts/pmc_decompose.py profiles/$TAG/pmc_summary_protein512x12500x1k.json \
  $((512 * 12500 * 1000)) profiles/$TAG/pmc_decomposition_protein.json | grep -E "valu_instr|valu_busy"
cp $O/bench_${TAG}_q100xdata500.json profiles/$TAG/bench.json
cp $O/bench_${TAG}_reads150x1k.json profiles/$TAG/bench_reads150x1k.json
cp $O/bench_${TAG}_protein512x1k.json profiles/$TAG/bench_protein512x1k.json
for w in ragged data500; do
  if [ -f $O/bench_${TAG}_$w.json ]; then cp $O/bench_${TAG}_$w.json profiles/$TAG/bench_$w.json; fi
done
cp $O/smoke_$TAG.log profiles/$TAG/smoke.log
cp $O/pytest_gpu_$TAG.log profiles/$TAG/pytest_gpu.log
tail -1 profiles/$TAG/pytest_gpu.log
python -c "
import csv, sys
for f in sys.argv[1:]:
    r = next(csv.DictReader(open(f)))
    print(f, r['Name'][:60], r['Calls'], round(float(r['AverageNs']) / 1e6, 4), 'ms avg')
" profiles/$TAG/kernel_stats*.csv
python - "$TAG" <<'EOF'
import json, sys
t = sys.argv[1]
for f in ("bench.json", "bench_reads150x1k.json", "bench_protein512x1k.json"):
    d = json.load(open(f"profiles/{t}/{f}"))
    r = d["roofline"]
    print(f, d["value"], r["achieved"], r["frac"], r["issue_frac"],
          (d.get("pcie_inclusive") or {}).get("value"), d.get("parity_sample"),
          (d.get("cpu_baseline") or {}).get("value"))
EOF
