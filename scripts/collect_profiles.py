#!/usr/bin/env python3
"""Copy the rocprofv3 summaries worth keeping from gpurun_out/ into profiles/<round>/ and
write profiles/pmc_summary.json (HBM bytes per score launch, read by bench.py).

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE come from separate
--pmc passes (TCC slot budget), are in KiB, and FETCH_SIZE reads half the bytes of a wide
coalesced stream on gfx950, so it is doubled (our 8-byte-per-lane code loads are not a
calibrated width: the doubled figure is an estimate, within ~10% of the algorithmic bytes).
usage: python scripts/collect_profiles.py ROUND PROF_DIR PMC_DIR WORKLOAD [KERNEL [SUFFIX]]
  WORKLOAD: bench.py's workload name (its JSON line's traffic lookup), e.g. query100x1021952x128,
            query100xragged1021952, reads150x131072x1k16, protein512x12500x1k
  KERNEL: substring of the kernel name the counters are averaged over (default score_kernel)
  SUFFIX: file suffix for a second workload (kernel_stats_SUFFIX.csv, pmc_SUFFIX_*.csv,
          pmc_summary_WORKLOAD.json); without it the files are the headline's
"""
import csv
import glob
import json
import os
import shutil
import sys

rnd, prof, pmc, workload = sys.argv[1:5]
kname = sys.argv[5] if len(sys.argv) > 5 else "score_kernel"
suffix = sys.argv[6] if len(sys.argv) > 6 else ""
tag = f"_{suffix}" if suffix else ""
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
dst = os.path.join(REPO, "profiles", rnd)
os.makedirs(dst, exist_ok=True)
for f in glob.glob(os.path.join(prof, "*kernel_stats.csv")):
    shutil.copy(f, os.path.join(dst, f"kernel_stats{tag}.csv"))


def mean_counter(name):
    vals = []
    for f in glob.glob(os.path.join(pmc, "*", "pmc_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if kname in r["Kernel_Name"] and r["Counter_Name"] == name:
                vals.append(float(r["Counter_Value"]))
    return sum(vals) / len(vals) if vals else None


summary = {"workload": workload}
for c in ("FETCH_SIZE", "WRITE_SIZE", "SQ_INSTS_VALU", "SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY",
          "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "GRBM_GUI_ACTIVE", "SQ_INSTS_LDS",
          "SQ_INSTS_SALU", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "SQ_WAIT_INST_LDS"):
    v = mean_counter(c)
    if v is not None:
        summary[c] = v
if "FETCH_SIZE" in summary and "WRITE_SIZE" in summary:
    summary["hbm_bytes_per_launch"] = int((2 * summary["FETCH_SIZE"] + summary["WRITE_SIZE"]) * 1024)
    summary["hbm_bytes_note"] = "(2*FETCH_SIZE + WRITE_SIZE) KiB; FETCH doubled per gfx950 calibration"
for f in glob.glob(os.path.join(pmc, "*", "pmc_counter_collection.csv")):
    sub = os.path.basename(os.path.dirname(f))
    shutil.copy(f, os.path.join(dst, f"pmc{tag}_{sub}.csv"))
summary["kernel"] = kname
out = "pmc_summary.json" if not suffix else f"pmc_summary_{workload}.json"
json.dump(summary, open(os.path.join(dst, out), "w"), indent=1)
json.dump(summary, open(os.path.join(REPO, "profiles", out), "w"), indent=1)
print(json.dumps(summary))
