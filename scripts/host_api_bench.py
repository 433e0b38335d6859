#!/usr/bin/env python3
"""Host-buffer API throughput (sw_score_batch / sw_score_records: host arrays in, scores out,
PCIe and host-side gather included) on the headline shape, next to the resident-in-HBM
device API.  usage: python scripts/host_api_bench.py [--n 1021952] [--L 128] [--iters 3]"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "smith-waterman-fpga-module_amd"))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1021952)
    ap.add_argument("--L", type=int, default=128)
    ap.add_argument("--qlen", type=int, default=128)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--ragged", action="store_true", help="lengths uniform in [L/2, L]")
    ap.add_argument("--no-records", action="store_true")
    ap.add_argument("--n-frac", type=float, default=0.0,
                    help="fraction of residues set to N (the feeder then sends 4-bit chunks)")
    ap.add_argument("--bench-ragged", action="store_true",
                    help="bench.py's ragged shape: lengths uniform in [64, 150], 0.1%% N")
    args = ap.parse_args()
    import swbank as S
    from oracle import oracle as O

    n, L = args.n, args.L
    q = O.random_codes(1, args.qlen, 4)
    rng = np.random.default_rng(7)
    lens = (rng.integers(L // 2, L + 1, n) if args.ragged else np.full(n, L)).astype(np.uint32)
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    res = O.random_codes(2, int(lens.sum()), 4)
    if args.n_frac > 0:
        res[rng.random(res.size) < args.n_frac] = 4
    if args.bench_ragged:
        from bench import ragged_batch
        res, offs, lens = ragged_batch(1000, n)
        args.ragged = True
    cells = float(args.qlen) * float(lens.sum())
    out = {"n": n, "L": L, "qlen": args.qlen, "ragged": args.ragged, "n_frac": args.n_frac}
    with S.ScoreBank(device=0) as bank:
        bank.set_penalties(5, -4, -12, -4)
        bank.load_query(q)
        ref = bank.score_batch(res, offs, lens)  # warm-up (allocations, pinned staging)
        ts = []
        bank.timing()
        bank.set_timing(True)
        buf = np.empty(n, np.int32)
        bank.score_batch(res, offs, lens, out=buf)  # touch the output pages once
        for _ in range(args.iters):
            t0 = time.perf_counter()
            got = bank.score_batch(res, offs, lens, out=buf)
            ts.append(time.perf_counter() - t0)
        bank.set_timing(False)
        launches, pack_ms, score_ms = bank.timing()
        assert np.array_equal(got, ref)
        out["host_api_ms"] = round(min(ts) * 1e3, 2)
        out["host_api_all_ms"] = [round(t * 1e3, 2) for t in ts]
        out["feeder_gather_ms_per_call"] = round(pack_ms / args.iters, 3)
        out["score_kernel_ms_per_call"] = round(score_ms / args.iters, 3)
        out["launches_per_call"] = launches / args.iters
        out["host_api_gcups"] = round(cells / min(ts) / 1e9, 1)
        out["kernel"] = bank.last_kernel()
        if not args.no_records and not args.ragged and not args.n_frac and L <= S.RECORD_MAX_BASES:
            recs = S.make_records(res.reshape(n, L))
            bank.score_records(recs)
            ts = []
            for _ in range(args.iters):
                t0 = time.perf_counter()
                r2 = bank.score_records(recs)
                ts.append(time.perf_counter() - t0)
            assert np.array_equal(r2, ref)
            out["records_api_ms"] = round(min(ts) * 1e3, 2)
            out["records_api_gcups"] = round(cells / min(ts) / 1e9, 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
