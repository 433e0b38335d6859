#!/usr/bin/env python3
"""Decompose a committed PMC summary (scripts/collect_profiles.py) into per-cell figures:
VALU instructions per 128 cells (one wave-instruction advances one query row for a lane's two
packed targets), VALU busy fraction, per-wave wait fractions.
GRBM_GUI_ACTIVE is summed over the 8 XCDs; a packed VALU wave-instruction occupies a SIMD
for 4 cycles (scripts/ubench/valu_rate.hip); 1024 SIMDs.
usage: python scripts/pmc_decompose.py SUMMARY.json CELLS_PER_LAUNCH [OUT.json]"""
import json
import sys

s = json.load(open(sys.argv[1]))
cells = float(sys.argv[2])
gr_per_xcd = s["GRBM_GUI_ACTIVE"] / 8
out = dict(s)
out.update({
    "cells_per_launch": cells,
    "valu_instr_per_128_cells": round(s["SQ_INSTS_VALU"] / (cells / 128), 3),
    "valu_busy": round(s["SQ_INSTS_VALU"] * 4 / 1024 / gr_per_xcd, 3),
    "grbm_cycles_per_xcd": gr_per_xcd,
    "kernel_ms_at_2.4GHz": round(gr_per_xcd / 2.4e6, 4),
    "frac_wait_any": round(s["SQ_WAIT_ANY"] / s["SQ_WAVE_CYCLES"], 3),
    "frac_wait_inst": round(s["SQ_WAIT_INST_ANY"] / s["SQ_WAVE_CYCLES"], 3),
    "frac_active": round(s["SQ_ACTIVE_INST_ANY"] / s["SQ_WAVE_CYCLES"], 3),
})
text = json.dumps(out, indent=1)
if len(sys.argv) > 3:
    open(sys.argv[3], "w").write(text + "\n")
print(text)
