"""World-size-2 gloo tests of the multi-GPU path's host logic (sharding + score gather).

On the GPU box each rank's ``bank`` is a ScoreBank on its own device and the process group is
RCCL; here the per-rank scorer is the oracle (a test double exposing ``score_batch``), so the
test exercises exactly the sharding and the gather collective that bench.py and
swbank.dist.score_sharded use."""
import os
import socket
import sys

import numpy as np
import pytest

import swbank.dist as D
from oracle import oracle as O


def test_shard_is_a_balanced_partition():
    rng = np.random.default_rng(0)
    lens = rng.integers(0, 1000, 1001)
    for world in (1, 2, 3, 8):
        parts = D.shard(lens, world)
        allidx = np.sort(np.concatenate(parts))
        assert (allidx == np.arange(len(lens))).all()
        cells = [int(lens[p].sum()) for p in parts]
        assert max(cells) - min(cells) <= int(lens.max())


class _OracleBank:
    """Test double with the ScoreBank.score_batch signature (CPU oracle)."""

    def __init__(self, q):
        self.q = q

    def score_batch(self, res, offs, lens):
        return O.score_batch(self.q, res, offs, lens, O.dna_matrix(), -12, -4)


def _worker(rank, world, port, ret):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(42)  # same batch on every rank
        q = rng.integers(0, 4, 100, dtype=np.uint8)
        seqs = [rng.integers(0, 4, int(rng.integers(0, 200)), dtype=np.uint8) for _ in range(257)]
        res, offs, lens = O.pack_residues(seqs)
        out = D.score_sharded(_OracleBank(q), res, offs, lens)
        if rank == 0:
            want = O.score_batch(q, res, offs, lens, O.dna_matrix(), -12, -4)
            ret.put(bool((out == want).all()))
        else:
            ret.put(out is None)
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2])
def test_gloo_sharded_scores_equal_single_process(world):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(results)


def _stepgather_worker(rank, world, port, ret):
    """bench.py's step loop under gloo: StepGather with async_op=True gathers, double-buffered,
    each step's scores produced by the oracle into sg.buffer() (the bank on the GPU box)."""
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(100 + rank)  # each rank its own batch (weak scaling)
        q = rng.integers(0, 4, 64, dtype=np.uint8)
        n = 300
        like = torch.zeros(n, dtype=torch.int32)
        sg = D.StepGather(like, dst=0, stage_cpu=True)
        bank = _OracleBank(q)
        last = None
        seen_bufs = set()
        for step in range(7):
            seqs = [rng.integers(0, 4, int(rng.integers(1, 120)), dtype=np.uint8) for _ in range(n)]
            res, offs, lens = O.pack_residues(seqs)
            buf = sg.buffer()
            seen_bufs.add(buf.data_ptr())
            buf.copy_(torch.from_numpy(bank.score_batch(res, offs, lens)))
            sg.submit()
            last = buf.clone()
        sg.drain()
        assert len(seen_bufs) == 2 and torch.equal(sg.last(), last)
        # every rank's last-step vector, gathered to rank 0
        allv = [torch.empty_like(last) for _ in range(world)] if rank == 0 else None
        dist.gather(last, gather_list=allv, dst=0)
        if rank == 0:
            # the last step's vectors (every step scores a different batch, so a list holding
            # step 5's vector for some rank would differ)
            ret.put(all(torch.equal(g, v) for g, v in zip(sg.gathered, allv))
                    and sg.lists[0] is not sg.lists[1])
        else:
            ret.put(sg.gathered is None)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_gloo_step_gather_async_double_buffered(world):
    """The bench's N>1 flow on CPU: async double-buffered gathers (StepGather) deliver every
    rank's scores of the last step to rank 0, with gloo as the backend."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_stepgather_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(results)
