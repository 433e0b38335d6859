#!/usr/bin/env python3
"""bench.py — GCUPS of the MI355X Smith-Waterman score bank (BASELINE.json metric).

Default workload (BASELINE.json configs[2], the 1-GPU GCUPS config; north_star "100 bp x
500 bp batches"): the reference query ``data/query100.fa`` (128 bp, committed as a fixture)
scored against a data500-shaped batch — ``--reps`` copies of 499 synthetic, seeded, uniform
ACGT 128-bp targets per GPU (``data/generate.py:6-23`` shape; splitmix64, seed 1000+rank).
Penalties 5/-4/-12/-4 (data/smith-waterman.py:6-10), merged gap model (the ScoreBank PE).

Other workloads (``--workload``), same JSON line:
  reads150x1k    configs[3]: per GPU ``--reads`` synthetic 150-bp reads x a fixed slice of
                 ``--slice`` 1-kbp targets (every read x every target of the slice); each
                 1-kbp target is the bank query (2 segments of 512 rows), the reads the batch.
  protein512x1k  configs[4]: a 512-aa query x ``--ptargets`` 1-kaa targets per GPU,
                 BLOSUM62, gap -11/-1, Gotoh (ssearch36 semantics), uniform 20-letter residues.

A step = one pass of the hot path over the batch (score kernel launches) on inputs already
resident in HBM, plus — at N>1 — the RCCL gather of the int32 score vector to rank 0 (the
only collective; pairs are sharded, scaling is weak).

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
CUS, SIMD_PER_CU, CLK_GHZ = 256, 4, 2.4
HBM_PEAK_GBS = 8000.0
# VALU roofline.  Algorithmic work = 10 ops per cell for the merged-gap
# recurrence, 11 for Gotoh (1 select, 6 max, 3 add).  Peak = packed 16-bit VALU rate: packed
# ops (v_pk_*_f16/u16) and v_perm_b32 issue one wave64 instruction per 4 cycles per SIMD
# (scripts/ubench/valu_rate.hip on MI355X: 0.244-0.27 wave-instr/SIMD/cycle at 2.4 GHz; f32
# ops reach 0.44) = 16 lanes x 2 halves per clock per SIMD -> 78.6 T ops/s.  max3 and perm fuse
# several algorithmic ops into one instruction, so frac > 1 is possible.
# Issue bound: one instruction advances one query row for a lane's 2 targets (128 cells per
# wave-instruction); instructions per row of the column body (csrc/swbank_kernels.hip):
# f16 merged 6.5 (5.5 with the letter-pair table: no v_perm per row), f16 Gotoh 8.5, u16
# merged 9, u16 Gotoh 11 (the column body both kernels share; the tile kernel adds 0.1-0.7 per
# row of loop overhead, the wave kernel ~7 per step of K rows plus the 63-step lane skew).
OPS_PER_CELL = {"merged": 10, "gotoh": 11}
VALU_PEAK_TOPS_16 = CUS * SIMD_PER_CU * 16 * 2 * CLK_GHZ / 1e3  # 78.6
VALU_ISSUE_PER_SIMD_CLK = 0.25
VALU_INSTR_PER_ROW = {"f16": 6.5, "f16-pair": 5.5, "f16-gotoh": 8.5, "u16": 9.0,
                      "u16-gotoh": 11.0}


def valu_peak_gcups(mode: str) -> float:
    per_row = VALU_INSTR_PER_ROW[mode]
    return CUS * SIMD_PER_CU * CLK_GHZ * VALU_ISSUE_PER_SIMD_CLK * 128 / per_row
PEN = (5, -4, -12, -4)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="q100xdata500",
                    choices=["q100xdata500", "reads150x1k", "protein512x1k"])
    ap.add_argument("--reps", type=int, default=2048,
                    help="q100xdata500: copies of the 499-target data500 batch per GPU")
    ap.add_argument("--target-len", type=int, default=128)
    ap.add_argument("--reads", type=int, default=131072, help="reads150x1k: reads per GPU")
    ap.add_argument("--slice", type=int, default=16, help="reads150x1k: 1-kbp targets")
    ap.add_argument("--ptargets", type=int, default=12500, help="protein512x1k: per GPU")
    ap.add_argument("--records", action="store_true",
                    help="q100xdata500: feed the targets as 64-byte CAPI sequence_t records "
                         "(2-bit codes, aligner_Header.h) instead of one code byte per base")
    ap.add_argument("--cpu-seconds", type=float, default=8.0,
                    help="wall budget of the CPU-baseline sample (0 disables)")
    ap.add_argument("--profile-only", action="store_true",
                    help="run warmup+steps and exit without the CPU leg (for rocprofv3)")
    return ap.parse_args()


def load_query():
    from oracle.oracle import encode_dna, golden_fasta, read_fasta  # fixture reader only
    return encode_dna(read_fasta(golden_fasta("query100.fa"))[0][1])


def make_codes(seed: int, n: int, L: int, alpha: int = 4) -> np.ndarray:
    """n x L uniform codes from a splitmix64 stream (same generator as the tests)."""
    from oracle.oracle import random_codes
    return random_codes(seed, n * L, alpha).reshape(n, L)


def pmc_traffic(workload: str):
    """HBM bytes per score launch from the committed rocprofv3 PMC summaries, if one matches
    (profiles/pmc_summary.json: the headline; profiles/pmc_summary_<workload>.json: others)."""
    for name in ("pmc_summary.json", f"pmc_summary_{workload}.json"):
        try:
            d = json.load(open(os.path.join(REPO, "profiles", name)))
            if d.get("workload") == workload:
                return d.get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            pass
    return None


class Workload:
    """One rank's share: a list of (bank, query) jobs over one resident batch."""

    def __init__(self, args, rank, dev, S, torch):
        self.args = args
        w = args.workload
        if w == "q100xdata500":
            q = load_query()
            n, L = 499 * args.reps, args.target_len
            self.batch = make_codes(1000 + rank, n, L)
            self.queries = [q]
            self.bank = S.ScoreBank(device=dev.index)
            self.bank.set_penalties(*PEN)
            self.model = "merged"
            self.name = f"query100x{n}x{L}"
            self.desc = (f"query100.fa (128 bp) x data500-shaped batch: {args.reps} x 499 "
                         f"synthetic {L}-bp ACGT targets per GPU (BASELINE configs[2])")
            self.params = {"penalties": list(PEN), "gap_model": "merged (ScoreBank PE)"}
        elif w == "reads150x1k":
            n, L = args.reads, 150
            self.batch = make_codes(2000 + rank, n, L)
            self.queries = list(make_codes(77, args.slice, 1000))  # the fixed 1-kbp slice
            self.bank = S.ScoreBank(device=dev.index)
            self.bank.set_penalties(*PEN)
            self.model = "merged"
            self.name = f"reads150x{n}x1k{args.slice}"
            self.desc = (f"{n} synthetic 150-bp reads per GPU x a slice of {args.slice} "
                         f"synthetic 1-kbp targets (BASELINE configs[3]); target = bank query "
                         f"(2 x 512-row segments), reads = batch")
            self.params = {"penalties": list(PEN), "gap_model": "merged (ScoreBank PE)"}
        else:
            n, L = args.ptargets, 1000
            self.batch = make_codes(3000 + rank, n, L, 20)
            self.queries = [make_codes(99, 1, 512, 20)[0]]
            self.bank = S.ScoreBank(device=dev.index, alphabet=S.ALPHABET_PROTEIN,
                                    gap_model=S.GAP_GOTOH)
            from oracle.oracle import BLOSUM62
            self.bank.set_matrix(BLOSUM62, -11, -1)
            self.model = "gotoh"
            self.name = f"protein512x{n}x1k"
            self.desc = (f"512-aa query x {n} synthetic 1-kaa targets per GPU, BLOSUM62, "
                         f"gap -11/-1, Gotoh (BASELINE configs[4])")
            self.params = {"matrix": "BLOSUM62", "gap_open": -11, "gap_extend": -1,
                           "gap_model": "gotoh (ssearch36)"}
        self.n, self.L = n, L
        self.d_res = torch.from_numpy(self.batch.reshape(-1)).to(dev)
        self.d_offs = torch.arange(n, dtype=torch.int64, device=dev) * L
        self.d_lens = torch.full((n,), L, dtype=torch.int32, device=dev)
        self.d_sc = torch.zeros((len(self.queries), n), dtype=torch.int32, device=dev)
        self.d_rec = None
        if getattr(args, "records", False):
            if w != "q100xdata500" or L > S.RECORD_MAX_BASES:
                raise SystemExit("--records: q100xdata500 with targets <= 232 bp only")
            self.d_rec = torch.from_numpy(S.make_records(self.batch).reshape(-1)).to(dev)
            self.desc += "; targets as CAPI 2-bit sequence_t records"
        if len(self.queries) == 1:
            self.bank.load_query(self.queries[0])
        self.cells = sum(len(q) for q in self.queries) * n * L

    def run(self, stream, d_sc=None):
        d_sc = self.d_sc if d_sc is None else d_sc
        for k, q in enumerate(self.queries):
            if len(self.queries) > 1:
                self.bank.load_query(q)  # ld_sequence: a new query for the same batch
            if self.d_rec is not None:
                self.bank.score_records_device(self.d_rec.data_ptr(), self.n,
                                               d_sc[k].data_ptr(), stream)
                continue
            self.bank.score_batch_device(self.d_res.data_ptr(), self.d_offs.data_ptr(),
                                         self.d_lens.data_ptr(), self.n, self.L,
                                         d_sc[k].data_ptr(), stream)


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal knobs (not used by the driver): SWBENCH_BACKEND=gloo with SWBENCH_SHARE_GPU=1
    # runs several ranks on one GPU to exercise the multi-rank flow
    backend = os.environ.get("SWBENCH_BACKEND", "nccl")
    if os.environ.get("SWBENCH_SHARE_GPU") == "1":
        local = 0
    if world > 1:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    import swbank as S

    wl = Workload(args, rank, dev, S, torch)
    gdev = dev if backend == "nccl" else torch.device("cpu")
    gather = ([torch.empty_like(wl.d_sc, device=gdev) for _ in range(world)]
              if (world > 1 and rank == 0) else None)
    stream = torch.cuda.current_stream()
    # Two score buffers: step i scores into bufs[i % 2] while the RCCL gather of step i-1
    # (async, on RCCL's stream) still reads the other one; a buffer is rewritten only after
    # the gather that read it has completed (work.wait() orders the compute stream after it).
    bufs = [wl.d_sc, torch.empty_like(wl.d_sc)]
    pending = [None, None]
    nstep = [0]

    def step():
        b = nstep[0] % 2
        if pending[b] is not None:
            pending[b].wait()
            pending[b] = None
        wl.run(stream.cuda_stream, bufs[b])
        if world > 1 and backend == "nccl":
            pending[b] = dist.gather(bufs[b], gather_list=gather, dst=0, async_op=True)
        elif world > 1:
            dist.gather(bufs[b].cpu(), gather_list=gather, dst=0)
        nstep[0] += 1

    def drain():
        for b in (0, 1):
            if pending[b] is not None:
                pending[b].wait()
                pending[b] = None

    for _ in range(args.warmup):
        step()
    drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    wl.bank.timing()  # drop warmup events
    wl.bank.set_timing(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    wl.bank.set_timing(False)
    launches, pack_ms, score_ms = wl.bank.timing()
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=gdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    cells_rank = wl.cells
    value = world * cells_rank * args.steps / elapsed / 1e9
    if args.profile_only:
        if rank == 0:
            print(json.dumps({"profile_only": True, "gcups": value}), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return

    # score-kernel time per step (one "launch" = one sw_score_batch_device call, which may
    # run several segment kernels for long queries)
    calls_per_step = len(wl.queries)
    score_s = score_ms / max(launches, 1) / 1e3 * calls_per_step
    pack_s = pack_ms / max(launches, 1) / 1e3 * calls_per_step
    kernel = wl.bank.last_kernel()
    arith = "f16" if " f16" in kernel else "u16"
    mode = arith if wl.model == "merged" else f"{arith}-gotoh"
    if mode == "f16" and " pair " in kernel:
        mode = "f16-pair"
    kernel_gcups = cells_rank / score_s / 1e9
    # issue bound of the column body (both kernels); the wave kernel's per-step overhead and
    # lane skew come on top
    peak_gcups = valu_peak_gcups(mode)
    ops = OPS_PER_CELL[wl.model]
    achieved_tops = ops * kernel_gcups / 1e3
    # algorithmic bytes: 1 B per residue read once per query + 4 B per score written
    per_target = S.RECORD_BYTES if wl.d_rec is not None else wl.L
    alg_bytes = len(wl.queries) * wl.n * (per_target + 4) + sum(len(q) for q in wl.queries)
    traffic = pmc_traffic(wl.name)

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
        "dtype": arith,
        "data": "synthetic",
        "config": {
            "workload": wl.desc,
            "query_len": [int(len(q)) for q in wl.queries][:1][0],
            "queries": len(wl.queries),
            "targets_per_gpu": wl.n,
            "target_len": wl.L,
            **wl.params,
            "parallelism": f"dp{world}: pairs sharded, RCCL gather of scores to rank 0",
        },
        "kernel": kernel,
        "kernel_ms": {"pack": round(pack_s * 1e3, 4), "score": round(score_s * 1e3, 4)},
        "roofline": {
            "bound": "valu",
            "achieved": round(achieved_tops, 2),
            "peak": round(VALU_PEAK_TOPS_16, 1),
            "unit": (f"T ops/s ({ops} algorithmic int ops per cell, SURVEY 8.2; peak = packed "
                     f"16-bit VALU, 1024 SIMDs x 32 ops/clk x {CLK_GHZ} GHz, measured issue rate)"),
            "frac": round(achieved_tops / VALU_PEAK_TOPS_16, 4),
            "traffic": traffic,
            "kernel_gcups": round(kernel_gcups, 1),
            "issue_bound_gcups": round(peak_gcups, 1) if peak_gcups else None,
            "issue_frac": round(kernel_gcups / peak_gcups, 4) if peak_gcups else None,
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

    if rank == 0 and world == 1 and wl.d_rec is None and len(wl.queries) == 1:
        out["pcie_inclusive"] = host_api_rate(wl, bufs[(nstep[0] - 1) % 2])
    if rank == 0 and world == 1 and args.cpu_seconds > 0 and args.workload == "q100xdata500":
        out["cpu_baseline"], out["parity_sample"] = cpu_baseline(
            wl.queries[0], wl.batch, bufs[(nstep[0] - 1) % 2][0], wl.L, args.cpu_seconds)
    elif rank == 0:
        out["parity_sample"] = parity_sample(wl, bufs[(nstep[0] - 1) % 2])

    if rank == 0:
        print(json.dumps(out), flush=True)
    wl.bank.close()
    if world > 1:
        dist.destroy_process_group()


def host_api_rate(wl, d_sc, iters=5):
    """The same batch through the host-buffer API (sw_score_batch: host arrays in, scores out;
    gather, PCIe both ways and the kernel inside the clock) -- reported next to `value`, which
    is the HBM-resident rate.  Also checks its scores against the device-API run."""
    n, L = wl.n, wl.L
    res = wl.batch.reshape(-1)
    offs = np.arange(n, dtype=np.uint64) * L
    lens = np.full(n, L, dtype=np.uint32)
    got = wl.bank.score_batch(res, offs, lens)  # first call sizes the pinned staging slots
    best = float("inf")
    for _ in range(iters):
        t0 = time.perf_counter()
        wl.bank.score_batch(res, offs, lens)
        best = min(best, time.perf_counter() - t0)
    same = bool(np.array_equal(got, d_sc[0].cpu().numpy()))
    return {"value": round(len(wl.queries[0]) * n * L / best / 1e9, 1), "unit": "GCUPS",
            "ms": round(best * 1e3, 3), "matches_device_api": same,
            "api": "sw_score_batch: host buffers, gather + PCIe + kernel + scores back, best of "
                   f"{iters}"}


def parity_sample(wl, d_sc, m=256):
    """Every query's scores for the first m targets of this rank's batch, re-computed by the
    oracle (test infrastructure) and compared: the bench's own bit-exactness evidence."""
    from oracle import oracle as O
    gpu = d_sc.cpu().numpy()
    m = min(m, wl.n)
    offs = (np.arange(m, dtype=np.uint64) * wl.L)
    lens = np.full(m, wl.L, dtype=np.uint32)
    if wl.model == "gotoh":
        sub, go, ge, model = O.BLOSUM62, -11, -1, O.GAP_GOTOH
    else:
        sub, go, ge, model = O.dna_matrix(PEN[0], PEN[1]), PEN[2], PEN[3], O.GAP_MERGED
    mism = 0
    for k, q in enumerate(wl.queries):
        cpu = O.score_batch(q, wl.batch[:m].reshape(-1), offs, lens, sub, go, ge, model)
        mism += int((cpu != gpu[k][:m]).sum())
    return {"targets": m * len(wl.queries), "mismatches": mism}


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
    # SURVEY §8.2 also asks for a single-core figure and the pure-Python restatement on
    # configs[0] (query1 x data1, 20 pairs)
    m1 = 499
    offs1 = (np.arange(m1, dtype=np.uint64) * L)
    t0 = time.perf_counter()
    O.score_batch(q, tg[:m1].reshape(-1), offs1, np.full(m1, L, np.uint32), sub, PEN[2], PEN[3],
                  O.GAP_MERGED, 1)
    dt1 = time.perf_counter() - t0
    q1 = O.encode_dna(O.read_fasta(O.golden_fasta("query1.fa"))[0][1])
    lib1 = [O.encode_dna(sq) for _, sq in O.read_fasta(O.golden_fasta("data1.fa"))]
    t0 = time.perf_counter()
    for t in lib1:
        O.py_score_merged(q1, t, sub, PEN[2], PEN[3])
    dtp = time.perf_counter() - t0
    cells1 = len(q1) * sum(len(t) for t in lib1)
    base = {"value": round(m * L * len(q) / dt / 1e9, 3), "unit": "GCUPS", "cores": cores,
            "kind": "port",
            "sample": f"first {m} targets of the rank-0 batch ({m * L * len(q):.3g} cells), "
                      f"{dt:.2f} s wall, oracle/sw_oracle.c -O3 OpenMP",
            "single_core_gcups": round(m1 * L * len(q) / dt1 / 1e9, 4),
            "python_configs0_mcups": round(cells1 / dtp / 1e6, 3)}
    return base, {"targets": m, "mismatches": mism}


if __name__ == "__main__":
    main()
