#!/usr/bin/env python3
"""Summarise rocprofv3 PMC csv passes for the score kernel: per-dispatch means and the
wave-time decomposition (ACTIVE / WAIT_INST / WAIT quad-cycles, guide §rocprofv3 PMC slots).
usage: python scripts/pmc_summary.py gpurun_out/pmc_TAG [kernel-substring]"""
import collections
import csv
import glob
import json
import sys

root = sys.argv[1]
kname = sys.argv[2] if len(sys.argv) > 2 else "score_dna"
agg = collections.defaultdict(list)
for f in glob.glob(f"{root}/*/pmc_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if kname in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
m = {k: sum(v) / len(v) for k, v in agg.items()}
out = {k: float(f"{v:.4g}") for k, v in sorted(m.items())}
if "SQ_WAVE_CYCLES" in m and "SQ_WAIT_ANY" in m:
    wc = m["SQ_WAVE_CYCLES"]
    out["frac_wait_any"] = round(m["SQ_WAIT_ANY"] / wc, 3)
    out["frac_wait_inst"] = round(m.get("SQ_WAIT_INST_ANY", 0) / wc, 3)
    out["frac_active"] = round(m.get("SQ_ACTIVE_INST_ANY", 0) / wc, 3)
if "GRBM_GUI_ACTIVE" in m and "SQ_INSTS_VALU" in m:
    cyc = m["GRBM_GUI_ACTIVE"] / 8  # summed over 8 XCDs
    out["valu_util"] = round(m["SQ_INSTS_VALU"] * 2 / (1024 * cyc), 3)  # 2 cyc/wave64 on SIMD32
    out["avg_waves_per_simd"] = round(m["SQ_WAVE_CYCLES"] * 4 / (1024 * cyc), 2)
print(json.dumps(out))
