#!/usr/bin/env python3
"""Sweep compiled score-kernel variants (SWBANK_R / SWBANK_RB / SWBANK_F16) on the bench workload
in ONE process (interleaved rounds, cdna_hip_programming.md §5.4 rule 24) and check that every
variant returns identical scores (and a sample against the oracle).

usage: python scripts/tune.py [--reps 1024] [--rounds 3] [--variants 32,8,4 16,8,4 ...]
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "smith-waterman-fpga-module_amd"))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=1024)
    ap.add_argument("--len", type=int, default=128)
    ap.add_argument("--qlen", type=int, default=0, help="0 = query100.fa (128 bp)")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--variants", nargs="*",
                    default=["32,4", "32,4,u16", "16,4", "32,8", "64,4"],
                    help="R,RB[,u16] tile-kernel variants (u16: SWBANK_F16=0) or wave")
    args = ap.parse_args()
    import torch

    import swbank as S
    from oracle import oracle as O

    if args.qlen:
        q = O.random_codes(77, args.qlen, 4)
    else:
        q = O.encode_dna(O.read_fasta(O.golden_fasta("query100.fa"))[0][1])
    n, L = 499 * args.reps, args.len
    tg = O.random_codes(1000, n * L, 4)
    dev = torch.device("cuda", 0)
    d_res = torch.from_numpy(tg).to(dev)
    d_offs = torch.arange(n, dtype=torch.int64, device=dev) * L
    d_lens = torch.full((n,), L, dtype=torch.int32, device=dev)
    d_sc = torch.zeros(n, dtype=torch.int32, device=dev)
    bank = S.ScoreBank(device=0)
    bank.set_penalties(5, -4, -12, -4)
    stream = torch.cuda.current_stream().cuda_stream
    cells = n * L * len(q)

    ref = None
    results = {v: [] for v in args.variants}
    for rnd in range(args.rounds):
        for v in args.variants:
            if v == "wave":
                os.environ["SWBANK_KERNEL"] = "wave"
            else:
                R, RB, *mode = v.split(",")
                os.environ["SWBANK_R"], os.environ["SWBANK_RB"] = R, RB
                os.environ["SWBANK_F16"] = "0" if mode == ["u16"] else "1"
                os.environ["SWBANK_KERNEL"] = "tile"
            bank.load_query(q)  # re-prepare with the new variant
            bank.set_timing(False)
            bank.score_batch_device(d_res.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(), n, L,
                                    d_sc.data_ptr(), stream)
            torch.cuda.synchronize()
            sc = d_sc.cpu().numpy().copy()
            if ref is None:
                idx = np.arange(0, n, max(1, n // 3000))
                offs = (idx * L).astype(np.uint64)
                want = O.score_batch(q, tg, offs, np.full(len(idx), L, np.uint32),
                                     O.dna_matrix(), -12, -4)
                assert (sc[idx] == want).all(), "variant disagrees with the oracle"
                ref = sc
            assert (sc == ref).all(), f"variant {v} differs from the first variant"
            bank.timing()
            bank.set_timing(True)
            for _ in range(args.iters):
                bank.score_batch_device(d_res.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(),
                                        n, L, d_sc.data_ptr(), stream)
            launches, _, ms = bank.timing()
            results[v].append(cells * launches / (ms / 1e3) / 1e9)
    for v, g in results.items():
        print(json.dumps({"variant": v, "gcups_median": round(float(np.median(g)), 1),
                          "gcups_all": [round(x, 1) for x in g]}))


if __name__ == "__main__":
    main()
