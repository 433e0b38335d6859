#!/usr/bin/env python3
"""bench.py — GCUPS of the MI355X Smith-Waterman score bank (BASELINE.json metric).

Default workload (BASELINE.json configs[2], the 1-GPU GCUPS config; north_star "100 bp x
500 bp batches"): the reference query ``data/query100.fa`` (128 bp, committed as a fixture)
scored against a SYNTHETIC data500-shaped batch — ``--reps`` x 499 seeded, uniform ACGT
128-bp targets per GPU (the shape of ``data/data500.fa`` and of ``data/generate.py:6-23``;
splitmix64, seed 1000+rank).  Penalties 5/-4/-12/-4 (data/smith-waterman.py:6-10), merged gap
model (the ScoreBank PE).

Other workloads (``--workload``), same JSON line:
  data500        the literal reference batch ``data/data500.fa`` (committed fixture), replicated
                 ``--reps`` times per GPU (cross-check of the synthetic default).
  ragged         query100.fa x ``--reps`` x 499 synthetic targets per GPU with lengths uniform in
                 [64, 150] and 0.1 % N (real reads are not uniform): the device API sorts them
                 longest first on the device.
  reads150x1k    configs[3]: per GPU ``--reads`` synthetic 150-bp reads x a fixed slice of
                 ``--slice`` 1-kbp targets (every read x every target of the slice); each
                 1-kbp target is the bank query (a query set in 128-row segments), the reads
                 the batch.
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
# The path is bound by VALU issue, not HBM or MFMA.
# Ceiling (roofline.peak): a SIMD issues one wave64 VALU instruction per 4 cycles (packed
# 16-bit ops, v_perm_b32 and 32-bit integer ops alike: scripts/ubench/valu_rate.hip measured
# 0.221-0.231 for packed f16 and 0.245-0.248 for 32-bit ops at 4 waves/SIMD, 0.374 for f32:
# profiles/r04/valu_rate.jsonl), and one packed 16-bit instruction advances one query row
# for 64 lanes x 2 targets = 128 cells.  The fewest such instructions per row the recurrence
# needs on gfx950 (DESIGN §6 derivation: every add is its own instruction because no
# instruction fuses an add into a max; v_pk_maximum3_f16 takes 3 inputs; the add's clamp is
# max(0, .) for free; substitution words come from an LDS letter-pair table, off the VALU):
#   merged (the ScoreBank PE): M = clamp(Hd + s), H = max3(M, Tu, Tl), MO = M - o,
#     G = max3(MO, Tu, Tl), T = G - e, best = max3(best, H, H') per 2 rows -> 5.5
#   Gotoh: D = clamp(Hd + s), H = max3(D, E, F), HN = H - o - e, E' = max3(0, HN, E - e) (2),
#     F' = max3(0, HN, F - e) (2), best 0.5 -> 7.5
# peak GCUPS = 1024 SIMDs x 2.4 GHz x 0.25 x 128 / that count; kernel-independent, so frac <= 1.
# The kernel's own instruction stream (issue_bound_gcups / issue_frac) and the SURVEY's
# 10-ops-per-cell unit (ops_basis, frac > 1 because max3 / clamp fuse ops) are side fields.
OPS_PER_CELL = {"merged": 10, "gotoh": 11}
VALU_PEAK_TOPS_16 = CUS * SIMD_PER_CU * 16 * 2 * CLK_GHZ / 1e3  # 78.6
VALU_ISSUE_PER_SIMD_CLK = 0.25
MIN_INSTR_PER_ROW = {"merged": 5.5, "gotoh": 7.5}
# the kernels' own column bodies (csrc/swbank_ktile.hip, swbank_kwave.hip): f16 merged 6.5 (5.5 with the
# letter-pair table), f16 Gotoh 8.5, u16 merged 9, u16 Gotoh 11; the tile kernel adds 0.1-0.7
# per row of loop overhead, the wave kernel ~7 per step of K rows plus the 63-step lane skew
VALU_INSTR_PER_ROW = {"f16": 6.5, "f16-pair": 5.5, "f16-gotoh": 8.5, "u16": 9.0,
                      "u16-gotoh": 11.0}


def gcups_at(instr_per_row: float) -> float:
    return CUS * SIMD_PER_CU * CLK_GHZ * VALU_ISSUE_PER_SIMD_CLK * 128 / instr_per_row


def valu_peak_gcups(mode: str) -> float:
    return gcups_at(VALU_INSTR_PER_ROW[mode])
PEN = (5, -4, -12, -4)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); without a launcher (no WORLD_SIZE) and N > 1, "
                         "bench.py starts torch.distributed.run with N ranks itself; under a "
                         "launcher N must equal WORLD_SIZE (default: WORLD_SIZE, else 1)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="q100xdata500",
                    choices=["q100xdata500", "data500", "ragged", "reads150x1k", "protein512x1k"])
    ap.add_argument("--reps", type=int, default=2048,
                    help="q100xdata500 / data500 / ragged: copies of the 499-target data500 "
                         "batch per GPU")
    ap.add_argument("--target-len", type=int, default=128)
    ap.add_argument("--targets", type=int, default=0,
                    help="q100xdata500: targets per GPU (default --reps x 499)")
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
    ap.add_argument("--full-parity", action="store_true",
                    help="re-check EVERY score of rank 0's batch against the oracle (by default "
                         "batches past 2e10 cells check a sample); reads150x1k: 3.1e11 cells, "
                         "about 30 s on 16 host cores")
    ap.add_argument("--emulate-ingest", type=float, default=0.0, metavar="MB",
                    help="(rehearsal, N=1) each step also copies MB of device memory on a second "
                         "stream beside the kernel: rank 0's share of the score gather at N>1 "
                         "(N-1 ranks x 4 B per target); reported as a separate field")
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


def ragged_batch(seed: int, n: int, lo: int = 64, hi: int = 150, p_n: float = 0.001):
    """n synthetic DNA reads with lengths uniform in [lo, hi] and ~p_n N codes (seeded, the
    same splitmix64 stream as make_codes): (codes, offsets u64, lens u32)."""
    from oracle.oracle import random_codes, splitmix64_bytes
    lens = (lo + (splitmix64_bytes(seed + 7, 2 * n).view(np.uint16).astype(np.uint32)
                  % (hi - lo + 1))).astype(np.uint32)
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    total = int(lens.sum())
    res = random_codes(seed, total, 4)
    if p_n > 0:
        u = splitmix64_bytes(seed + 11, 2 * total).view(np.uint16)
        res[u < int(p_n * 65536)] = 4
    return res, offs, lens


class Workload:
    """One rank's share: a list of (bank, query) jobs over one resident batch
    (res / offs / lens: the batch's codes, offsets and lengths on the host)."""

    def __init__(self, args, rank, dev, S, torch):
        self.args = args
        self.rank = rank
        w = self.kind = args.workload
        self.model = "merged"
        self.params = {"penalties": list(PEN), "gap_model": "merged (ScoreBank PE)"}
        self.sub = None
        if w in ("q100xdata500", "data500", "ragged"):
            self.queries = [load_query()]
            self.bank = S.ScoreBank(device=dev.index)
            self.bank.set_penalties(*PEN)
        if w == "q100xdata500":
            n, L = args.targets or 499 * args.reps, args.target_len
            self.set_uniform(make_codes(1000 + rank, n, L))
            self.name = f"query100x{n}x{L}"
            self.desc = (f"query100.fa (128 bp) x synthetic data500-shaped batch: {n} "
                         f"(= {n / 499:g} x 499) seeded uniform-ACGT {L}-bp targets per GPU (the "
                         f"shape of data/data500.fa; BASELINE configs[2])")
        elif w == "data500":
            from oracle.oracle import encode_dna, golden_fasta, read_fasta
            lib = [encode_dna(sq) for _, sq in read_fasta(golden_fasta("data500.fa"))]
            if len({len(t) for t in lib}) != 1:
                raise SystemExit("data500.fa: expected equal-length targets")
            self.set_uniform(np.tile(np.stack(lib), (args.reps, 1)))
            self.name = f"query100xdata500x{args.reps}"
            self.desc = (f"query100.fa (128 bp) x the literal data/data500.fa (499 x "
                         f"{len(lib[0])} bp) replicated {args.reps}x per GPU (BASELINE configs[2])")
        elif w == "ragged":
            n = 499 * args.reps
            self.res, self.offs, self.lens = ragged_batch(1000 + rank, n)
            self.n, self.L = n, int(self.lens.max())
            self.name = f"query100xragged{n}"
            self.desc = (f"query100.fa (128 bp) x {n} synthetic reads per GPU, lengths uniform in "
                         f"[64, 150], 0.1% N (device API: on-device longest-first sort)")
        elif w == "reads150x1k":
            n, L = args.reads, 150
            self.set_uniform(make_codes(2000 + rank, n, L))
            self.queries = list(make_codes(77, args.slice, 1000))  # the fixed 1-kbp slice
            self.bank = S.ScoreBank(device=dev.index)
            self.bank.set_penalties(*PEN)
            self.name = f"reads150x{n}x1k{args.slice}"
            self.desc = (f"{n} synthetic 150-bp reads per GPU x a slice of {args.slice} "
                         f"synthetic 1-kbp targets (BASELINE configs[3]); target = bank query "
                         f"(a query set in 128-row segments), reads = batch")
        elif w == "protein512x1k":
            n, L = args.ptargets, 1000
            self.set_uniform(make_codes(3000 + rank, n, L, 20))
            self.queries = [make_codes(99, 1, 512, 20)[0]]
            self.bank = S.ScoreBank(device=dev.index, alphabet=S.ALPHABET_PROTEIN,
                                    gap_model=S.GAP_GOTOH)
            from oracle.oracle import BLOSUM62
            self.sub = BLOSUM62
            self.bank.set_matrix(BLOSUM62, -11, -1)
            self.model = "gotoh"
            self.name = f"protein512x{n}x1k"
            self.desc = (f"512-aa query x {n} synthetic 1-kaa targets per GPU, BLOSUM62, "
                         f"gap -11/-1, Gotoh (BASELINE configs[4])")
            self.params = {"matrix": "BLOSUM62", "gap_open": -11, "gap_extend": -1,
                           "gap_model": "gotoh (ssearch36)"}
        n = self.n
        self.Lmin = int(self.lens.min())
        self.d_res = torch.from_numpy(self.res).to(dev)
        self.d_offs = torch.from_numpy(self.offs.view(np.int64)).to(dev)
        self.d_lens = torch.from_numpy(self.lens.view(np.int32)).to(dev)
        self.d_sc = torch.zeros((len(self.queries), n), dtype=torch.int32, device=dev)
        self.d_rec = None
        if getattr(args, "records", False):
            if w != "q100xdata500" or self.L > S.RECORD_MAX_BASES:
                raise SystemExit("--records: q100xdata500 with targets <= 232 bp only")
            self.d_rec = torch.from_numpy(
                S.make_records(self.res.reshape(n, self.L)).reshape(-1)).to(dev)
            self.desc += "; targets as CAPI 2-bit sequence_t records"
        if len(self.queries) == 1:
            self.bank.load_query(self.queries[0])
        else:  # a query set: one call scores the batch against every query (nq x n scores)
            self.bank.load_queries(self.queries)
        self.cells = sum(len(q) for q in self.queries) * int(self.lens.sum(dtype=np.uint64))

    def set_uniform(self, batch: np.ndarray):
        n, L = batch.shape
        self.res = np.ascontiguousarray(batch).reshape(-1)
        self.offs = np.arange(n, dtype=np.uint64) * L
        self.lens = np.full(n, L, dtype=np.uint32)
        self.n, self.L = n, L

    def regen_rows(self, rank: int, rows: np.ndarray):
        """Targets `rows` of rank `rank`'s batch, regenerated from its seed (rank 0 checks the
        slices it gathered from the other ranks; the code streams are counter-based, so a row
        needs no prefix): (res, offs, lens)."""
        from oracle.oracle import random_codes
        w, L = self.kind, self.L
        seed_alpha = {"q100xdata500": (1000, 4), "reads150x1k": (2000, 4),
                      "protein512x1k": (3000, 20)}
        if w in seed_alpha:
            seed, alpha = seed_alpha[w]
            b = np.stack([random_codes(seed + rank, L, alpha, start=int(k) * L) for k in rows])
        elif w == "data500":
            b = self.res.reshape(self.n, L)[rows]
        else:
            res, offs, lens = ragged_batch(1000 + rank, self.n)
            seqs = [res[int(offs[k]):int(offs[k] + lens[k])] for k in rows]
            ln = np.array([len(t) for t in seqs], np.uint32)
            of = np.zeros(len(seqs), np.uint64)
            of[1:] = np.cumsum(ln[:-1], dtype=np.uint64)
            return np.concatenate(seqs), of, ln
        m = len(rows)
        return (np.ascontiguousarray(b).reshape(-1), np.arange(m, dtype=np.uint64) * L,
                np.full(m, L, np.uint32))

    def run(self, stream, d_sc=None):
        d_sc = self.d_sc if d_sc is None else d_sc
        if len(self.queries) > 1:
            self.bank.score_batch_device(self.d_res.data_ptr(), self.d_offs.data_ptr(),
                                         self.d_lens.data_ptr(), self.n, self.L,
                                         d_sc.data_ptr(), stream, min_len=self.Lmin)
            return
        for k, q in enumerate(self.queries):
            if self.d_rec is not None:
                self.bank.score_records_device(self.d_rec.data_ptr(), self.n,
                                               d_sc[k].data_ptr(), stream)
                continue
            # the caller's length range (sw_score_batch_device_range): a fixed-length batch
            # needs no visiting order, a ragged one is sorted longest first on the device
            self.bank.score_batch_device(self.d_res.data_ptr(), self.d_offs.data_ptr(),
                                         self.d_lens.data_ptr(), self.n, self.L,
                                         d_sc[k].data_ptr(), stream, min_len=self.Lmin)


def resolve_world(args) -> int | None:
    """The rank count `--gpus` asks for, checked against the launcher's WORLD_SIZE BEFORE any
    GPU call.  Returns the world size to run with, or None when this process has started the
    N ranks itself (it then only waits for them).  A mismatch exits non-zero: a line printed
    with the wrong n_gpus would be worse than none."""
    env = os.environ.get("WORLD_SIZE")
    if env is not None:
        world = int(env)
        if args.gpus is not None and args.gpus != world:
            sys.stderr.write(f"bench.py: --gpus {args.gpus} but the launcher started "
                             f"WORLD_SIZE={world} ranks\n")
            raise SystemExit(2)
        return world
    if args.gpus is None or args.gpus == 1:
        return 1
    if args.gpus < 1:
        raise SystemExit(f"bench.py: --gpus {args.gpus}")
    # No launcher: start the N ranks as a CHILD launcher (never exec from this process) and
    # exit with its return code.  Nothing here has touched the GPU yet.
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1",
           "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    import subprocess
    rc = subprocess.call(cmd, env=dict(os.environ, MASTER_ADDR="127.0.0.1"))
    raise SystemExit(rc)


def rank_device(torch, dev) -> dict:
    """This rank's GPU as the driver can check it: PCI address and UUID."""
    p = torch.cuda.get_device_properties(dev)
    return {"pci": f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}",
            "uuid": str(getattr(p, "uuid", "")), "index": dev.index,
            "name": p.name}


def main():
    args = parse()
    world = resolve_world(args)
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal knobs (not used by the driver): SWBENCH_BACKEND=gloo with SWBENCH_SHARE_GPU=1
    # runs several ranks on one GPU to exercise the multi-rank flow (tests/test_gpu_bench.py)
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
    # What the collective actually saw: its world size and every rank's GPU, gathered to rank 0
    devices = [rank_device(torch, dev)]
    dist_info = {"world_size": 1, "backend": None}
    if world > 1:
        devices = [None] * world
        dist.all_gather_object(devices, rank_device(torch, dev))
        dist_info = {"world_size": dist.get_world_size(), "backend": dist.get_backend()}
        if dist_info["world_size"] != world:
            raise SystemExit(f"bench.py: process group has {dist_info['world_size']} ranks, "
                             f"expected {world}")
    dist_info["devices"] = devices
    dist_info["distinct_gpus"] = len({d["pci"] + d["uuid"] for d in devices})

    import swbank as S

    wl = Workload(args, rank, dev, S, torch)
    probe_host = {}
    if os.environ.get("SWBENCH_PROBE_HOST") == "1":  # (tuning aid) host-API medians by phase
        def _hmed(tag):
            o = np.empty(wl.n, np.int32)
            wl.bank.score_batch(wl.res, wl.offs, wl.lens, out=o)
            ts = []
            for _ in range(9):
                t0 = time.perf_counter()
                wl.bank.score_batch(wl.res, wl.offs, wl.lens, out=o)
                ts.append(time.perf_counter() - t0)
            probe_host[tag] = round(float(np.median(ts)) * 1e3, 3)
        _hmed("after_workload")
    gdev = dev if backend == "nccl" else torch.device("cpu")
    # The scoring stream, made torch's current one: on ROCm the default current stream's handle
    # is 0, which the library reads as "the bank's own (non-blocking) stream", so a score copy
    # or collective enqueued by torch on the default stream would not wait for the kernel (the
    # gathered scores of a 2-rank run were then stale now and then: tests/test_gpu_bench.py)
    stream = torch.cuda.Stream(device=dev)
    stream.wait_stream(torch.cuda.current_stream())  # (the workload's uploads and fills)
    torch.cuda.set_stream(stream)
    assert stream.cuda_stream != 0
    # Two score buffers: step i scores into one while the async gather of step i-1 (RCCL's
    # stream) still reads the other (swbank.dist.StepGather; gloo gathers a host copy).  The
    # CPU tests run this same class under gloo (tests/test_dist.py).
    from swbank.dist import StepGather
    sg = StepGather(wl.d_sc, dst=0, stage_cpu=backend != "nccl")

    # (rehearsal) rank 0's ingest of the other ranks' score vectors at N>1, as concurrent
    # device-to-device copies on another stream: the collective's traffic and its copy kernels
    # share rank 0's CUs with the score kernel, and `value` divides by the max over ranks
    ingest = None
    if args.emulate_ingest > 0:
        nb = int(args.emulate_ingest * 2**20) // 4 * 4
        ingest = (torch.cuda.Stream(), torch.empty(nb // 4, dtype=torch.int32, device=dev),
                  torch.empty(nb // 4, dtype=torch.int32, device=dev))

    def step():
        if ingest is not None:
            s2, src, dst = ingest
            s2.wait_stream(stream)
            with torch.cuda.stream(s2):
                dst.copy_(src, non_blocking=True)
        wl.run(stream.cuda_stream, sg.buffer())
        if ingest is not None:
            stream.wait_stream(ingest[0])  # the next step starts after this step's ingest
        sg.submit()

    def drain():
        sg.drain()

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
    # the bank's per-call HIP-event time, summed over the timed steps (one call per step, which
    # runs several launches for long queries / query sets)
    score_s = score_ms / args.steps / 1e3
    wl.bank_kernel_ms = score_s * 1e3  # (the host-buffer path's bound, host_api_rate)
    pack_s = pack_ms / args.steps / 1e3
    kernel = wl.bank.last_kernel()
    arith = "f16" if " f16" in kernel else "u16"
    mode = arith if wl.model == "merged" else f"{arith}-gotoh"
    if mode == "f16" and " pair " in kernel:
        mode = "f16-pair"
    kernel_gcups = cells_rank / score_s / 1e9
    peak = gcups_at(MIN_INSTR_PER_ROW[wl.model])          # kernel-independent ceiling
    own = valu_peak_gcups(mode)                           # this kernel's column body
    ops = OPS_PER_CELL[wl.model]
    achieved_tops = ops * kernel_gcups / 1e3
    # algorithmic bytes: 1 B per residue read once per query + 4 B per score written
    per_target = S.RECORD_BYTES * wl.n if wl.d_rec is not None else int(wl.lens.sum())
    alg_bytes = len(wl.queries) * (per_target + 4 * wl.n) + sum(len(q) for q in wl.queries)
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
        "data": "synthetic" if wl.kind != "data500" else "reference fixture data/data500.fa",
        "config": {
            "workload": wl.desc,
            "query_len": [int(len(q)) for q in wl.queries][:1][0],
            "queries": len(wl.queries),
            "targets_per_gpu": wl.n,
            "target_len": wl.L if wl.kind != "ragged" else "64-150",
            **wl.params,
            "parallelism": f"dp{world}: pairs sharded, RCCL gather of scores to rank 0",
        },
        "kernel": kernel,
        "dist": dist_info,
        **({"emulated_ingest_mb": args.emulate_ingest} if args.emulate_ingest > 0 else {}),
        "kernel_ms": {"pack": round(pack_s * 1e3, 4), "score": round(score_s * 1e3, 4)},
        "roofline": {
            "bound": "valu",
            "achieved": round(kernel_gcups, 1),
            "peak": round(peak, 1),
            "unit": (f"GCUPS (peak = VALU issue ceiling: 1024 SIMDs x {CLK_GHZ} GHz x 1 wave64 "
                     f"instr / 4 clk x 128 cells / {MIN_INSTR_PER_ROW[wl.model]} instr per row, "
                     f"the fewest packed-16 instructions the {wl.model} recurrence needs on "
                     f"gfx950, DESIGN §6)"),
            "frac": round(kernel_gcups / peak, 4),
            "traffic": traffic,
            "issue_bound_gcups": round(own, 1),
            "issue_frac": round(kernel_gcups / own, 4),
            "ops_basis": {"achieved_tops": round(achieved_tops, 2),
                          "peak_tops": round(VALU_PEAK_TOPS_16, 1),
                          "frac": round(achieved_tops / VALU_PEAK_TOPS_16, 4),
                          "unit": f"T int ops/s at {ops} algorithmic ops per cell (SURVEY 8.2); "
                                  "max3 / clamp fuse ops, so > 1 is possible"},
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

    last = sg.last()
    gather = sg.gathered
    if probe_host:
        _hmed("before_host_api_rate")
        out["probe_host"] = probe_host
    if rank == 0 and world == 1 and wl.d_rec is None and len(wl.queries) == 1:
        out["pcie_inclusive"] = host_api_rate(wl, last)
    if rank == 0 and world == 1 and args.cpu_seconds > 0 and wl.kind == "q100xdata500":
        out["cpu_baseline"], out["parity_sample"] = cpu_baseline(
            wl.queries[0], wl.res.reshape(wl.n, wl.L), last[0], wl.L, args.cpu_seconds)
    elif rank == 0:
        out["parity_sample"] = parity_sample(wl, [g for g in gather] if gather else [last],
                                             full_cells=float("inf") if args.full_parity
                                             else 2e10)

    if rank == 0:
        print(json.dumps(out), flush=True)
    wl.bank.close()
    if world > 1:
        dist.destroy_process_group()


def host_api_rate(wl, d_sc, iters=15):
    """The same batch through the host-buffer API (sw_score_batch: host arrays in, scores out;
    gather, PCIe both ways and the kernel inside the clock) -- reported next to `value`, which
    is the HBM-resident rate.  Two warm calls (the first sizes the pinned slots), then `iters`
    timed calls: the median and the interquartile range of the call times (the method of
    scripts/host_ab.py; calls switch between fast and slow host-memory levels, DESIGN §3.4, so a
    best-of-N figure overstates the rate).  Also checks its scores against the device-API run."""
    got = wl.bank.score_batch(wl.res, wl.offs, wl.lens)
    out = np.empty_like(got)  # the caller's output buffer, pages already touched
    warm = []
    for _ in range(int(os.environ.get("SWBENCH_HOST_WARM", "1"))):
        t0 = time.perf_counter()
        wl.bank.score_batch(wl.res, wl.offs, wl.lens, out=out)
        warm.append(round((time.perf_counter() - t0) * 1e3, 3))
    h2d0 = wl.bank.counters()["h2d_bytes"]
    ts = []
    for _ in range(iters):
        t0 = time.perf_counter()
        wl.bank.score_batch(wl.res, wl.offs, wl.lens, out=out)
        ts.append(time.perf_counter() - t0)
    q1, med, q3 = np.percentile(ts, [25, 50, 75])
    same = bool(np.array_equal(got, d_sc[0].cpu().numpy()) and np.array_equal(out, got))
    # The path's own ceiling: its host->device bytes per call (the library's count) at this
    # box's pinned H2D rate (one timed copy of that many bytes), or the kernel, whichever is
    # longer; frac = that bound / the median call.
    nb = (wl.bank.counters()["h2d_bytes"] - h2d0) // iters
    rate = h2d_rate(max(nb, 1 << 20))
    kernel_ms = wl.bank_kernel_ms
    bound_ms = max(kernel_ms, nb / rate / 1e6)
    return {"value": round(wl.cells / med / 1e9, 1), "unit": "GCUPS",
            "ms": round(med * 1e3, 3), "ms_iqr": [round(q1 * 1e3, 3), round(q3 * 1e3, 3)],
            "ms_best": round(min(ts) * 1e3, 3), "calls": iters, "matches_device_api": same,
            "ms_warm": warm, "ms_calls": [round(t * 1e3, 3) for t in ts],
            "bytes_h2d": int(nb), "h2d_gbs": round(rate, 1),
            "bound_ms": round(bound_ms, 3),
            "frac": round(bound_ms / (med * 1e3), 3),
            "frac_of_device_rate": round(kernel_ms / (med * 1e3), 3),
            "api": "sw_score_batch: host buffers, gather + PCIe + kernel + scores back; median "
                   f"of {iters} calls after 2 warm calls (value = cells / median); bound_ms = "
                   "max(score kernel, bytes_h2d / h2d_gbs), frac = bound_ms / median"}


def h2d_rate(nbytes: int) -> float:
    """This box's pinned host -> device copy rate (GB/s) for one copy of nbytes: best of 3,
    HIP events on the copy's stream."""
    import torch
    src = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    dst = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    s = torch.cuda.Stream()
    best = float("inf")
    for _ in range(4):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(s):
            a.record(s)
            dst.copy_(src, non_blocking=True)
            b.record(s)
        b.synchronize()
        best = min(best, a.elapsed_time(b))
    return nbytes / (best / 1e3) / 1e9


def parity_sample(wl, per_rank, m=4096, full_cells=2e10):
    """Every query's scores re-computed by the oracle (test infrastructure, the multi-threaded
    C restatement) and compared: the bench's own bit-exactness evidence.  A rank's whole batch
    when it is at most `full_cells` cells (configs[2] / data500 / ragged: every one of the
    ~1.02 M targets, ~1.5 s; configs[4]: all 12,500 protein targets), else the
    first and the last m/4 targets and m/2 seeded random ones between (the last ones are where
    the wave kernel's split tail runs).  Rank 0's own scores, and at N>1 the slices it gathered
    from the others, regenerated from their seeds."""
    from oracle import oracle as O
    if wl.model == "gotoh":
        sub, go, ge, model = wl.sub, -11, -1, O.GAP_GOTOH
    else:
        sub, go, ge, model = O.dna_matrix(PEN[0], PEN[1]), PEN[2], PEN[3], O.GAP_MERGED
    if wl.cells <= full_cells:
        rows = np.arange(wl.n)
    else:
        pick = np.random.default_rng(12345).integers(0, wl.n, m // 2)
        rows = np.unique(np.concatenate([np.arange(min(m // 4, wl.n)),
                                         np.arange(max(0, wl.n - m // 4), wl.n), pick]))
    mism, checked, by_rank = 0, 0, []
    for r, sc in enumerate(per_rank):
        gpu = sc.cpu().numpy()
        if r == wl.rank:  # this rank's own batch is on the host already
            res, offs, lens = wl.res, np.ascontiguousarray(wl.offs[rows]), \
                np.ascontiguousarray(wl.lens[rows])
        else:
            res, offs, lens = wl.regen_rows(r, rows)
        m0 = mism
        for k, q in enumerate(wl.queries):
            cpu = O.score_batch(q, res, offs, lens, sub, go, ge, model)
            mism += int((cpu != gpu[k][rows]).sum())
            checked += len(rows)
        by_rank.append(mism - m0)
    out = {"targets": checked, "ranks": len(per_rank), "mismatches": mism,
            "of_targets": len(per_rank) * len(wl.queries) * wl.n,
            "full": bool(len(rows) == wl.n)}
    if len(per_rank) > 1:
        out["mismatches_by_rank"] = by_rank
    return out


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
