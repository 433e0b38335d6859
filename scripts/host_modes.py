#!/usr/bin/env python3
"""Host-API timing per bank: several banks one after another in ONE process, each scoring the
bench's ragged (or uniform) host batch a few times -- does a process's fast/slow mode follow
the bank (streams, buffers) or the process?   usage: host_modes.py [--banks 5] [--uniform]"""
import argparse
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "smith-waterman-fpga-module_amd"))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--banks", type=int, default=5)
    ap.add_argument("--iters", type=int, default=6)
    ap.add_argument("--uniform", action="store_true")
    args = ap.parse_args()
    import swbank as S
    from oracle import oracle as O
    from bench import ragged_batch
    n = 1021952
    if args.uniform:
        lens = np.full(n, 128, np.uint32)
        offs = np.arange(n, dtype=np.uint64) * 128
        res = O.random_codes(2, n * 128, 4)
    else:
        res, offs, lens = ragged_batch(1000, n)
    q = O.random_codes(1, 128, 4)
    out = np.empty(n, np.int32)
    for k in range(args.banks):
        with S.ScoreBank(device=0) as bank:
            bank.set_penalties(5, -4, -12, -4)
            bank.load_query(q)
            bank.score_batch(res, offs, lens, out=out)
            ts = []
            for _ in range(args.iters):
                t0 = time.perf_counter()
                bank.score_batch(res, offs, lens, out=out)
                ts.append((time.perf_counter() - t0) * 1e3)
            print(f"{os.environ.get('TAG', '')} bank {k}: best {min(ts):.2f} ms, all {[round(t, 2) for t in ts]}", flush=True)


if __name__ == "__main__":
    main()
