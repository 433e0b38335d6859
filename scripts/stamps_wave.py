#!/usr/bin/env python3
"""Where the protein two-pairs kernel's time goes (a fixed ≈ 50 µs per launch):
runs configs[4]'s batch once through the measurement build (scripts/build_variant.sh stamps
"-DSWK_STAMPS=1", selected with SWBANK_LIB) that records per wave, with s_memtime, its entry,
exit, the end of its block's profile copy, the ticks it spent waiting for a hand-off, and its
HW_ID / XCC.

s_memtime is one counter per XCD (not aligned across XCDs), so everything is taken per XCD.
Prints one JSON object:
  ramp      mean entry after the XCD's first entry, as a share of the XCD's span
  copy      mean (profile copy end - entry) share
  wait      mean hand-off wait share
  exit      mean (XCD's last exit - the wave's exit) share: the end-of-kernel drain
  simd_occupancy  share of each SIMD's span with 3 / 2 / 1 / 0 of its waves resident
  exit_rank  per SIMD, the waves' exits ordered by entry (age): mean gap to the SIMD's last exit
usage: SWBANK_LIB=.../libswbank_stamps.so python scripts/stamps_wave.py [--targets 12500]"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "smith-waterman-fpga-module_amd"))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--targets", type=int, default=12500)
    ap.add_argument("--L", type=int, default=1000)
    ap.add_argument("--dump", default="")
    args = ap.parse_args()
    import torch
    import swbank as S
    from bench import make_codes
    from oracle.oracle import BLOSUM62

    n, L = args.targets, args.L
    dev = torch.device("cuda", 0)
    res = make_codes(3000, n, L, 20).reshape(-1)
    q = make_codes(99, 1, 512, 20)[0]
    d_res = torch.from_numpy(res).to(dev)
    d_offs = torch.arange(n, dtype=torch.int64, device=dev) * L
    d_lens = torch.full((n,), L, dtype=torch.int32, device=dev)
    d_sc = torch.zeros(n, dtype=torch.int32, device=dev)
    stamps = torch.zeros(4096 * 4 * 8, dtype=torch.int64, device=dev)
    lib = S.lib()
    lib.swk_set_stamps.argtypes = [ctypes.c_void_p]
    with S.ScoreBank(device=0, alphabet=S.ALPHABET_PROTEIN, gap_model=S.GAP_GOTOH) as bank:
        bank.set_matrix(BLOSUM62, -11, -1)
        bank.load_query(q)
        call = lambda: bank.score_batch_device(d_res.data_ptr(), d_offs.data_ptr(),
                                               d_lens.data_ptr(), n, L, d_sc.data_ptr(),
                                               min_len=L)
        call()
        torch.cuda.synchronize()
        lib.swk_set_stamps(stamps.data_ptr())
        call()
        torch.cuda.synchronize()
        lib.swk_set_stamps(None)
        kern = bank.last_kernel()
    st = stamps.cpu().numpy().reshape(-1, 8).astype(np.int64)
    st = st[st[:, 1] > 0]
    if args.dump:
        np.save(args.dump, st)
    t0, t1, tc, tw, hw, xcc = st[:, 0], st[:, 1], st[:, 2], st[:, 3], st[:, 4], st[:, 5]
    out = {"kernel": kern, "targets": n, "waves": int(len(st))}
    sh = {"ramp": 0.0, "copy": 0.0, "wait": 0.0, "exit": 0.0}
    occ = np.zeros(4)
    gaps = {}
    spans = []
    for x in np.unique(xcc):
        m = xcc == x
        a, b = t0[m].min(), t1[m].max()
        span = float(b - a)
        spans.append(span)
        sh["ramp"] += float((t0[m] - a).sum()) / span
        sh["copy"] += float((tc[m] - t0[m]).sum()) / span
        sh["wait"] += float(tw[m].sum()) / span
        sh["exit"] += float((b - t1[m]).sum()) / span
        # per SIMD of this XCD (HW_ID: simd 5:4, cu 11:8, sh 12, se 15:13)
        hx = hw[m]
        key = ((hx >> 13) & 7) * 1000 + ((hx >> 12) & 1) * 100 + ((hx >> 8) & 15) * 10 + ((hx >> 4) & 3)
        e0, e1 = t0[m], t1[m]
        for k in np.unique(key):
            w = key == k
            s0, s1 = e0[w], e1[w]
            lo, hi = s0.min(), s1.max()
            grid = np.linspace(lo, hi, 200)
            alive = ((grid[:, None] >= s0[None, :]) & (grid[:, None] < s1[None, :])).sum(1)
            for c in range(4):
                occ[c] += float((np.minimum(alive, 3) == c).mean())
            order = np.argsort(s0)
            for r, i in enumerate(order):
                gaps.setdefault(r, []).append(float(hi - s1[i]) / span)
    W = len(st)
    out["share"] = {k: round(v / W, 4) for k, v in sh.items()}
    nsimd = occ.sum()
    out["simd_occupancy"] = {f"{c}_waves": round(float(occ[c] / nsimd), 4) for c in (3, 2, 1, 0)}
    out["exit_rank"] = {f"age_{r}": round(float(np.mean(g)), 4) for r, g in sorted(gaps.items())}
    out["span_ticks"] = {"min": min(spans), "max": max(spans)}
    out["visits"] = {"min": int(st[:, 6].min()), "max": int(st[:, 6].max())}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
