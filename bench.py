#!/usr/bin/env python3
"""bench.py — GCUPS of the MI355X Smith-Waterman score bank (BASELINE.json metric).

Workload (BASELINE.json configs[2], the 1-GPU GCUPS config; north_star "100 bp x 500 bp
batches"): the reference query ``data/query100.fa`` (128 bp, committed as a fixture) scored
against a data500-shaped batch — ``--reps`` copies of 499 synthetic, seeded, uniform ACGT
128-bp targets per GPU (``data/generate.py:6-23`` shape; splitmix64, seed 1000+rank).
Penalties 5/-4/-12/-4 (data/smith-waterman.py:6-10), merged gap model (the ScoreBank PE).

A step = one pass of the hot path over the batch: feeder (pack) kernel + score kernel on
inputs already resident in HBM, plus — at N>1 — the RCCL gather of the int32 score vector
to rank 0 (the only collective; pairs are sharded, scaling is weak).

Launch: ``python bench.py [--gpus N --steps K --warmup W]``; for N>1 under
``torch.distributed.run`` (one process per GPU, RCCL).  Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "smith-waterman-fpga-module_amd"))
sys.path.insert(0, REPO)

# MI355X constants (/opt/skills/guides/MI355X_MICROARCH.md, chip-level parameters)
CUS, SIMD_PER_CU, LANES_PER_SIMD_CLK, CLK_GHZ = 256, 4, 32, 2.4
VALU_PEAK_TOPS_U16 = CUS * SIMD_PER_CU * LANES_PER_SIMD_CLK * 2 * CLK_GHZ / 1e3  # 157.3
HBM_PEAK_GBS = 8000.0
OPS_PER_CELL = 10  # 1 select, 6 max, 3 add per cell of the §8.0 recurrence
PEN = (5, -4, -12, -4)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--reps", type=int, default=2048,
                    help="copies of the 499-target data500 batch per GPU")
    ap.add_argument("--target-len", type=int, default=128)
    ap.add_argument("--cpu-seconds", type=float, default=8.0,
                    help="wall budget of the CPU-baseline sample (0 disables)")
    ap.add_argument("--profile-only", action="store_true",
                    help="run warmup+steps and exit without the CPU leg (for rocprofv3)")
    return ap.parse_args()


def load_query():
    from oracle.oracle import encode_dna, golden_fasta, read_fasta  # fixture reader only
    return encode_dna(read_fasta(golden_fasta("query100.fa"))[0][1])


def make_targets(seed: int, n: int, L: int) -> np.ndarray:
    """n x L uniform ACGT codes from a splitmix64 stream (same generator as the tests)."""
    from oracle.oracle import random_codes
    return random_codes(seed, n * L, 4).reshape(n, L)


def pmc_traffic(workload: str):
    """HBM bytes per score launch from the committed rocprofv3 PMC summary, if it matches."""
    path = os.path.join(REPO, "profiles", "pmc_summary.json")
    try:
        d = json.load(open(path))
        if d.get("workload") == workload:
            return d.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        pass
    return None


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    import swbank as S

    q = load_query()
    n = 499 * args.reps
    L = args.target_len
    tg = make_targets(1000 + rank, n, L)
    d_res = torch.from_numpy(tg.reshape(-1)).to(dev)
    d_offs = torch.arange(n, dtype=torch.int64, device=dev) * L
    d_lens = torch.full((n,), L, dtype=torch.int32, device=dev)
    d_sc = torch.zeros(n, dtype=torch.int32, device=dev)
    gather = [torch.empty_like(d_sc) for _ in range(world)] if (world > 1 and rank == 0) else None

    bank = S.ScoreBank(device=dev.index)
    bank.set_penalties(*PEN)
    bank.load_query(q)
    stream = torch.cuda.current_stream()

    def step():
        bank.score_batch_device(d_res.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(), n, L,
                                d_sc.data_ptr(), stream.cuda_stream)
        if world > 1:
            dist.gather(d_sc, gather_list=gather, dst=0)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    bank.timing()  # drop warmup events
    bank.set_timing(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    bank.set_timing(False)
    launches, pack_ms, score_ms = bank.timing()
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    cells_rank = n * L * len(q)
    value = world * cells_rank * args.steps / elapsed / 1e9
    if args.profile_only:
        if rank == 0:
            print(json.dumps({"profile_only": True, "gcups": value}), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return

    score_s = score_ms / max(launches, 1) / 1e3
    pack_s = pack_ms / max(launches, 1) / 1e3
    workload = f"query100x{n}x{L}"
    achieved_tops = OPS_PER_CELL * cells_rank / score_s / 1e12
    alg_bytes = n * (L + 4) + len(q)  # 1 B per residue read once + 4 B per score written
    traffic = pmc_traffic(workload)

    out = {
        "metric": "GCUPS",
        "value": round(value, 2),
        "unit": "GCUPS",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u16",
        "data": "synthetic",
        "config": {
            "workload": f"query100.fa (128 bp) x data500-shaped batch: {args.reps} x 499 "
                        f"synthetic {L}-bp ACGT targets per GPU (BASELINE configs[2])",
            "query_len": int(len(q)),
            "targets_per_gpu": n,
            "target_len": L,
            "penalties": list(PEN),
            "gap_model": "merged (ScoreBank PE)",
            "parallelism": f"dp{world}: pairs sharded, RCCL gather of scores to rank 0",
        },
        "kernel_ms": {"pack": round(pack_s * 1e3, 4), "score": round(score_s * 1e3, 4)},
        "roofline": {
            "bound": "valu",
            "achieved": round(achieved_tops, 2),
            "peak": round(VALU_PEAK_TOPS_U16, 1),
            "unit": "Tops/s (u16 int ops, 10 per cell)",
            "frac": round(achieved_tops / VALU_PEAK_TOPS_U16, 4),
            "traffic": traffic,
        },
        "roofline_hbm": {
            "bound": "hbm",
            "achieved": round(alg_bytes / score_s / 1e9, 2),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(alg_bytes / score_s / 1e9 / HBM_PEAK_GBS, 6),
            "traffic": traffic,
        },
        "cpu_baseline": None,
    }

    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        out["cpu_baseline"], out["parity_sample"] = cpu_baseline(q, tg, d_sc, L, args.cpu_seconds)

    if rank == 0:
        print(json.dumps(out), flush=True)
    bank.close()
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline(q, tg, d_sc, L, budget_s):
    """The oracle's C restatement (OpenMP over targets) on this box's host cores, on a bounded
    prefix of the same batch; its scores double as a parity sample of the GPU result."""
    from oracle import oracle as O
    cores = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    sub = O.dna_matrix(PEN[0], PEN[1])
    gpu = d_sc.cpu().numpy()

    def run(m):
        offs = (np.arange(m, dtype=np.uint64) * L)
        lens = np.full(m, L, dtype=np.uint32)
        t0 = time.perf_counter()
        cpu = O.score_batch(q, tg[:m].reshape(-1), offs, lens, sub, PEN[2], PEN[3], O.GAP_MERGED,
                            cores)
        return cpu, time.perf_counter() - t0

    _, dt0 = run(499 * 4)  # calibration (also warms the threads)
    m = int(min(len(tg), max(499, 499 * 4 * budget_s / max(dt0, 1e-3))))
    cpu, dt = run(m)
    mism = int((cpu != gpu[:m]).sum())
    base = {"value": round(m * L * len(q) / dt / 1e9, 3), "unit": "GCUPS", "cores": cores,
            "kind": "port",
            "sample": f"first {m} targets of the rank-0 batch ({m * L * len(q):.3g} cells), "
                      f"{dt:.2f} s wall, oracle/sw_oracle.c -O3 OpenMP"}
    return base, {"targets": m, "mismatches": mism}


if __name__ == "__main__":
    main()
