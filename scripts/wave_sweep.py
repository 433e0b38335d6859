#!/usr/bin/env python3
"""Wave-kernel GCUPS vs batch size and split-tail segment count (tuning aid: occupancy / tail
effects; SWBANK_WAVE_SPLIT_P: 0 = the policy's choice, 2 or 4 forced).
usage: python scripts/wave_sweep.py [--qlen 512] [--L 1000] [--ns 8192,12500,...] [--split 0,2,4]"""
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
    ap.add_argument("--qlen", type=int, default=512)
    ap.add_argument("--L", type=int, default=1000)
    ap.add_argument("--ns", default="6144,8192,10240,12288,12500,14336,16384,24576,25000")
    ap.add_argument("--split", default="0,2,4")
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--kernel", default="wave")
    args = ap.parse_args()
    import torch

    import swbank as S
    from oracle import oracle as O

    dev = torch.device("cuda", 0)
    os.environ["SWBANK_KERNEL"] = args.kernel
    q = O.random_codes(5, args.qlen, 20)
    bank = S.ScoreBank(device=0, alphabet=S.ALPHABET_PROTEIN, gap_model=S.GAP_GOTOH)
    bank.set_matrix(O.BLOSUM62, -11, -1)
    bank.load_query(q)
    ts = torch.cuda.Stream()  # a real stream handle (torch's default stream is handle 0)
    torch.cuda.set_stream(ts)
    stream = ts.cuda_stream
    for n in [int(x) for x in args.ns.split(",")]:
        L = args.L
        tg = O.random_codes(9, n * L, 20)
        d_res = torch.from_numpy(tg).to(dev)
        d_offs = torch.arange(n, dtype=torch.int64, device=dev) * L
        d_lens = torch.full((n,), L, dtype=torch.int32, device=dev)
        d_sc = torch.zeros(n, dtype=torch.int32, device=dev)
        out = {"qlen": args.qlen, "L": L, "n": n}
        for w in args.split.split(","):
            os.environ["SWBANK_WAVE_SPLIT_P"] = w
            call = lambda: bank.score_batch_device(d_res.data_ptr(), d_offs.data_ptr(),
                                                   d_lens.data_ptr(), n, L, d_sc.data_ptr(),
                                                   stream)
            call()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                call()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / args.iters
            out[f"P{w}"] = round(args.qlen * L * n / ms / 1e6, 1)
        out["kernel"] = bank.last_kernel()
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
