#!/usr/bin/env python3
"""In-process A/B of host-buffer API configurations (sw_score_batch: host arrays in, scores
out, gather + PCIe + kernel inside the clock), interleaved A B A B ... in ONE process so that
the box state (the "fast" / "slow" host-memory levels LEDGER §2.2 records) hits every config
alike.  Each config has its own bank, created and called under its environment (knobs read at
bank creation and knobs read per call both apply).  Reports per config the median, the IQR
(p25-p75) and the best of all calls, and the device-API rate of the same resident batch.

A knob is worth keeping only when its median moves by more than the IQRs (LEDGER §2.2 rule).

usage: python scripts/host_ab.py [--shape ragged|uniform] [--rounds 12] [--calls 4]
                                  [--config NAME:ENV=V,ENV=V ...]
  no --config: the kept feeder alone ("default"), i.e. the measurement of the shipped path.
"""
import argparse
import contextlib
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "smith-waterman-fpga-module_amd"))
sys.path.insert(0, REPO)


@contextlib.contextmanager
def env(kv):
    old = {k: os.environ.get(k) for k in kv}
    os.environ.update(kv)
    try:
        yield
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def parse_config(s):
    name, _, rest = s.partition(":")
    kv = dict(x.split("=", 1) for x in rest.split(",") if x)
    return name, kv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", choices=["ragged", "uniform"], default="ragged")
    ap.add_argument("--n", type=int, default=1021952)
    ap.add_argument("--rounds", type=int, default=12)
    ap.add_argument("--calls", type=int, default=4, help="calls per config per round")
    ap.add_argument("--config", action="append", default=[])
    args = ap.parse_args()
    import torch
    import swbank as S
    from bench import load_query, make_codes, ragged_batch, PEN

    q = load_query()
    n = args.n
    if args.shape == "ragged":  # bench.py --workload ragged: 64-150 bp, 0.1 % N
        res, offs, lens = ragged_batch(1000, n)
    else:
        res = make_codes(1000, n, 128).reshape(-1)
        offs = np.arange(n, dtype=np.uint64) * 128
        lens = np.full(n, 128, np.uint32)
    cells = float(len(q)) * float(lens.sum(dtype=np.uint64))
    configs = [parse_config(c) for c in args.config] or [("default", {})]
    banks = {}
    for name, kv in configs:
        with env(kv):
            b = S.ScoreBank(device=0)
            b.set_penalties(*PEN)
            b.load_query(q)
            b.score_batch(res, offs, lens)  # sizes the pinned slots, starts the threads
        banks[name] = b
    ref = None
    out_buf = np.empty(n, np.int32)
    times = {name: [] for name, _ in configs}
    for r in range(args.rounds):
        order = configs if r % 2 == 0 else configs[::-1]
        for name, kv in order:
            with env(kv):
                for _ in range(args.calls):
                    t0 = time.perf_counter()
                    got = banks[name].score_batch(res, offs, lens, out=out_buf)
                    times[name].append(time.perf_counter() - t0)
                if ref is None:
                    ref = got.copy()
                elif not np.array_equal(got, ref):
                    raise SystemExit(f"config {name}: scores differ")
    # the same batch resident in HBM (the device API's rate, the ceiling of the host path)
    dev = torch.device("cuda", 0)
    d_res = torch.from_numpy(res).to(dev)
    d_offs = torch.from_numpy(offs.view(np.int64)).to(dev)
    d_lens = torch.from_numpy(lens.view(np.int32)).to(dev)
    d_sc = torch.empty(n, dtype=torch.int32, device=dev)
    b0 = banks[configs[0][0]]
    st = torch.cuda.Stream()
    dts = []
    for _ in range(6):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        b0.score_batch_device(d_res.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(), n,
                              int(lens.max()), d_sc.data_ptr(), st.cuda_stream,
                              min_len=int(lens.min()))
        st.synchronize()
        dts.append(time.perf_counter() - t0)
    dev_ms = float(np.median(dts[1:])) * 1e3
    assert np.array_equal(d_sc.cpu().numpy(), ref)
    rep = {"shape": args.shape, "n": n, "cells": cells, "rounds": args.rounds,
           "calls_per_round": args.calls, "device_api_ms": round(dev_ms, 3),
           "device_api_gcups": round(cells / dev_ms / 1e6, 1), "configs": {}}
    for name, kv in configs:
        t = np.array(times[name]) * 1e3
        p25, med, p75 = np.percentile(t, [25, 50, 75])
        rep["configs"][name] = {
            "env": kv, "calls": len(t), "median_ms": round(med, 3),
            "iqr_ms": [round(p25, 3), round(p75, 3)], "best_ms": round(t.min(), 3),
            "median_gcups": round(cells / med / 1e6, 1),
            "median_frac_of_device": round(dev_ms / med, 3),
            "all_ms": [round(x, 3) for x in t]}
        b = banks[name]
        rep["configs"][name]["counters"] = b.counters()
        rep["configs"][name]["kernel"] = b.last_kernel()
    for b in banks.values():
        b.close()
    print(json.dumps(rep))


if __name__ == "__main__":
    main()
