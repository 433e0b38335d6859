#!/usr/bin/env python3
"""Where the headline tile kernel's wave time goes: runs the headline
batch once through a measurement build of the library (scripts/build_variant.sh stamps
"-DSWK_STAMPS=1"; selected with SWBANK_LIB) that records per wave, with s_memtime, its entry
and exit, the cycles of its active phases (column work), of its fill/drain phases (phases
without a chunk of its own, spent at the barrier) and of the per-phase barrier wait.

Prints one JSON object: the kernel span, and summed over all waves, the shares of
  ramp     entry after the first wave's entry (dispatch skew)
  active   phases with a chunk of the wave's own (compute + its waits inside the phase)
  barrier  waiting at the per-phase barrier after an active phase
  filldrain phases of the pipeline fill / drain (no chunk of its own, barrier included)
  exit     from the wave's exit to the last wave's exit (the end-of-kernel quantisation)
which sum to 100 % of (waves x span); plus the per-SIMD spread of active cycles.
usage: SWBANK_LIB=.../libswbank_stamps.so python scripts/stamps.py [--targets N] [--bal 0|1]"""
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
    ap.add_argument("--targets", type=int, default=499 * 2048)
    ap.add_argument("--L", type=int, default=128)
    ap.add_argument("--bal", default="1")
    ap.add_argument("--ragged", action="store_true",
                    help="bench.py's ragged batch (64-150 bp, 0.1 %% N; the device sort)")
    ap.add_argument("--presorted", action="store_true",
                    help="with --ragged: the batch physically reordered longest first, so the "
                         "kernel reads it without the permutation (its gathered loads)")
    ap.add_argument("--bal-ragged", action="store_true",
                    help="with --ragged: balanced chunk ranges over the sorted tiles")
    ap.add_argument("--dump", default="", help="save the raw per-wave records (.npy)")
    args = ap.parse_args()
    os.environ["SWBANK_BAL"] = args.bal
    os.environ["SWBANK_BAL_RAGGED"] = "1" if args.bal_ragged else "0"
    if args.presorted:  # caller's order = longest first: no device sort, no permutation
        os.environ["SWBANK_DSORT"] = "0"
    import torch
    import swbank as S
    from bench import PEN, load_query, make_codes

    L, n = args.L, args.targets
    q = load_query()
    dev = torch.device("cuda", 0)
    lens = np.full(n, L, np.uint32)
    if args.ragged:
        from bench import ragged_batch
        res, offs, lens = ragged_batch(1000, n)
        if args.presorted:  # longest first, stable (the device sort's order)
            order = np.argsort(-lens.astype(np.int64), kind="stable")
            seqs = [res[int(offs[k]):int(offs[k] + lens[k])] for k in order]
            lens = lens[order]
            offs = np.zeros(n, np.uint64)
            offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
            res = np.concatenate(seqs)
        L = int(lens.max())
        d_offs = torch.from_numpy(offs.view(np.int64)).to(dev)
        d_lens = torch.from_numpy(lens.view(np.int32)).to(dev)
        min_len = int(lens.min())
    else:
        res = make_codes(1000, n, L).reshape(-1)
        d_offs = (torch.arange(n, dtype=torch.int64, device=dev) * L)
        d_lens = torch.full((n,), L, dtype=torch.int32, device=dev)
        min_len = L
    d_res = torch.from_numpy(res).to(dev)
    d_sc = torch.zeros(n, dtype=torch.int32, device=dev)
    stamps = torch.zeros(4096 * 16 * 16, dtype=torch.int64, device=dev)
    lib = S.lib()
    lib.swk_set_stamps.argtypes = [ctypes.c_void_p]
    with S.ScoreBank(device=0) as bank:
        bank.set_penalties(*PEN)
        bank.load_query(q)
        call = lambda: bank.score_batch_device(d_res.data_ptr(), d_offs.data_ptr(),
                                               d_lens.data_ptr(), n, L, d_sc.data_ptr(),
                                               min_len=min_len)
        call()
        torch.cuda.synchronize()
        lib.swk_set_stamps(stamps.data_ptr())
        call()
        torch.cuda.synchronize()
        lib.swk_set_stamps(None)
        kern = bank.last_kernel()
    st = stamps.cpu().numpy().reshape(-1, 16).astype(np.int64)
    st = st[st[:, 1] > 0]
    if args.dump:
        np.save(args.dump, st)
    t0, t1, act, idle, bar, hw, xcc, bload = (st[:, 0], st[:, 1], st[:, 2], st[:, 3], st[:, 4],
                                              st[:, 5], st[:, 7], st[:, 8])
    # s_memtime counts each XCD's own clock (the XCDs' counters are not aligned): spans, ramps
    # and exits are taken per XCC, then summed
    waves = len(st)
    tot = ramp = exit_ = 0.0
    spans = {}
    for x in np.unique(xcc):
        m = xcc == x
        sp = float(t1[m].max() - t0[m].min())
        spans[int(x)] = sp
        tot += sp * m.sum()
        ramp += float((t0[m] - t0[m].min()).sum())
        exit_ += float((t1[m].max() - t1[m]).sum())
    inner = (t1 - t0) - act - idle - bar  # loop set-up and the epilogue
    out = {"kernel": kern, "targets": n, "waves": waves,
           "span_ticks_per_xcc": {"min": min(spans.values()), "max": max(spans.values())},
           "chunks_per_wave": {"min": int(st[:, 6].min()), "max": int(st[:, 6].max())},
           "share": {"ramp": round(ramp / tot, 4), "active": round(act.sum() / tot, 4),
                     "barrier": round(bar.sum() / tot, 4),
                     "filldrain": round(idle.sum() / tot, 4),
                     "setup": round(inner.sum() / tot, 4),
                     "exit": round(exit_ / tot, 4)},
           "tail_state_load": round(bload.sum() / tot, 5)}
    # per SIMD: active ticks of its waves (HW_ID: simd 5:4, cu 11:8, sh 12, se 15:13) and XCC
    key = (xcc * 10000 + ((hw >> 13) & 7) * 1000 + ((hw >> 12) & 1) * 100 + ((hw >> 8) & 15) * 10
           + ((hw >> 4) & 3))
    per = {}
    for k, a, x in zip(key.tolist(), act.tolist(), xcc.tolist()):
        per[k] = per.get(k, 0) + a / spans[int(x)]
    v = np.array(list(per.values()), dtype=np.float64)
    out["simds_seen"] = len(per)
    out["simd_active_spread"] = {"min": round(v.min(), 4), "median": round(float(np.median(v)), 4),
                                 "max": round(v.max(), 4)}
    # the work a tile does beyond its targets' cells: lanes past their target's end (a tile runs
    # to its longest lane) and the last chunk's padding columns (8-column chunks); tiles in the
    # longest-first order the device sort visits
    srt = np.sort(lens.astype(np.int64))[::-1]
    nt = (n + 127) // 128
    tmax = srt[::128][:nt]
    cells = float(srt.sum())
    lane_cols = float(np.minimum(tmax, 10**9).sum()) * 128
    chunk_cols = float((np.maximum(1, (tmax + 7) // 8) * 8).sum()) * 128
    out["tile_work"] = {"idle_lanes": round((lane_cols - cells) / chunk_cols, 4),
                        "chunk_padding": round((chunk_cols - lane_cols) / chunk_cols, 4)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
