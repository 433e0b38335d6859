"""GPU: balanced chunk ranges.  A uniform device batch through the pair-table
kernel gives every resident workgroup slot the same number of 8-column chunks; a tile cut by a
range boundary is scored in two visits by two workgroups, the column state (H and T of every
row, the diagonal above, the running best) handed over through global memory and a flag.

Checked: bit-exact against the same bank with SWBANK_BAL=0 (whole tiles per workgroup) on every
target, and against the oracle on every target of every cut tile (the cut positions follow from
the grid the call reports), over query lengths that give 1-4 waves, target lengths that give 1-16
chunks (a partial last chunk included), batch ends inside a tile, back-to-back calls (the flags'
generation), poisoned device buffers."""
import re

import numpy as np
import pytest

import swbank as S
from oracle import oracle as O

pytestmark = pytest.mark.gpu

REF = (5, -4, -12, -4)


def _cut_tiles(ntiles, K, grid):
    """Tiles whose chunks a range boundary splits (A_g = g * ntiles * K // grid)."""
    at = ntiles * K
    cuts = {(at * g // grid) // K for g in range(1, grid) if (at * g // grid) % K}
    return np.array(sorted(cuts), dtype=np.int64)


@pytest.mark.parametrize("qlen,L,n", [(128, 128, 340_000), (100, 100, 300_001), (40, 9, 600_000),
                                      (77, 64, 400_000), (128, 1, 300_000)])
def test_balanced_ranges_exact(qlen, L, n, poisoned_buffers, monkeypatch):
    torch = pytest.importorskip("torch")
    dev = torch.device("cuda", 0)
    q = O.random_codes(500 + qlen, qlen, 4)
    res = O.random_codes(600 + L, n * L, 4)
    # homologous targets past the first chunks, so a cut tile's best often lies after the cut
    rng = np.random.default_rng(L)
    for k in rng.choice(n, n // 50, replace=False):
        m = min(L, qlen)
        res[k * L:k * L + m] = q[:m]
    offs = np.arange(n, dtype=np.uint64) * L
    lens = np.full(n, L, np.uint32)
    d_res = torch.from_numpy(res).to(dev)
    d_offs = torch.from_numpy(offs.view(np.int64)).to(dev)
    d_lens = torch.from_numpy(lens.view(np.int32)).to(dev)

    def run(bal):
        monkeypatch.setenv("SWBANK_BAL", bal)
        st = torch.cuda.Stream()
        out = []
        with S.ScoreBank() as bank:
            bank.set_penalties(*REF)
            bank.load_query(q)
            for _ in range(2):  # back to back: the second call's flags carry a new generation
                sc = torch.full((n,), -7, dtype=torch.int32, device=dev)
                bank.score_batch_device(d_res.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(),
                                        n, L, sc.data_ptr(), st.cuda_stream, min_len=L)
                out.append(sc)
            st.synchronize()
            kern, ctr = bank.last_kernel(), bank.counters()
        return [x.cpu().numpy() for x in out], kern, ctr

    (a1, a2), kern, ctr = run("1")
    (b1, _), kern0, _ = run("0")
    assert "balanced" in kern and "balanced" not in kern0, (kern, kern0)
    assert ctr["balanced_calls"] == 2 and ctr["balanced_timeouts"] == 0, ctr
    assert np.array_equal(a1, b1) and np.array_equal(a2, b1)
    grid = int(re.search(r"grid=(\d+)", kern).group(1))
    ntiles = (n + 127) // 128
    cut = _cut_tiles(ntiles, (L + 7) // 8, grid)
    if L > 8:
        assert len(cut) >= grid // 4  # range boundaries fall inside tiles
    rows = np.concatenate([np.arange(t * 128, min(n, t * 128 + 128)) for t in cut]) \
        if len(cut) else np.arange(0)
    rows = np.unique(np.concatenate([rows, np.arange(min(n, 256)), np.arange(n - 256, n)]))
    want = O.score_batch(q, res, np.ascontiguousarray(offs[rows]), np.ascontiguousarray(lens[rows]),
                         O.dna_matrix(*REF[:2]), *REF[2:])
    assert np.array_equal(a1[rows], want)


def test_balanced_needs_uniform_lengths(monkeypatch):
    """A ragged batch (min_len < max_len) or a batch of fewer than two tiles per slot keeps whole
    tiles per workgroup."""
    torch = pytest.importorskip("torch")
    dev = torch.device("cuda", 0)
    n, L = 200_000, 128
    q = O.random_codes(1, 128, 4)
    res = O.random_codes(2, n * L, 4)
    d_res = torch.from_numpy(res).to(dev)
    d_offs = torch.from_numpy((np.arange(n, dtype=np.uint64) * L).view(np.int64)).to(dev)
    d_lens = torch.from_numpy(np.full(n, L, np.int32)).to(dev)
    sc = torch.empty(n, dtype=torch.int32, device=dev)
    with S.ScoreBank() as bank:
        bank.set_penalties(*REF)
        bank.load_query(q)
        bank.score_batch_device(d_res.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(), 1000, L,
                                sc.data_ptr(), min_len=L)
        assert "balanced" not in bank.last_kernel()  # 8 tiles
        bank.score_batch_device(d_res.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(), n, L,
                                sc.data_ptr(), min_len=L - 1)
        assert "balanced" not in bank.last_kernel()
        torch.cuda.synchronize()
        assert bank.counters()["balanced_calls"] == 0


@pytest.mark.parametrize("qlen,lo,hi,n", [(128, 64, 150, 1_000_003), (40, 30, 61, 1_500_000),
                                          (100, 1, 24, 2_000_000)])
def test_balanced_ranges_ragged(qlen, lo, hi, n, poisoned_buffers, monkeypatch):
    """A ragged device batch: the device sort visits it longest first and also computes where
    each workgroup's range starts (tiles of different chunk counts); bit-exact against whole
    tiles per workgroup on every target, and against the oracle on a sample."""
    torch = pytest.importorskip("torch")
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(qlen + hi)
    q = O.random_codes(700 + qlen, qlen, 4)
    lens = rng.integers(lo, hi + 1, n).astype(np.uint32)
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    res = O.random_codes(800 + hi, int(lens.sum(dtype=np.uint64)), 4)
    for k in rng.choice(n, n // 50, replace=False):  # homologous targets
        m = int(min(lens[k], qlen))
        res[int(offs[k]):int(offs[k]) + m] = q[:m]
    d_res = torch.from_numpy(res).to(dev)
    d_offs = torch.from_numpy(offs.view(np.int64)).to(dev)
    d_lens = torch.from_numpy(lens.view(np.int32)).to(dev)

    def run(bal):
        monkeypatch.setenv("SWBANK_BAL", bal)
        monkeypatch.setenv("SWBANK_BAL_RAGGED", bal)
        st = torch.cuda.Stream()
        out = []
        with S.ScoreBank() as bank:
            bank.set_penalties(*REF)
            bank.load_query(q)
            for _ in range(2):
                sc = torch.full((n,), -7, dtype=torch.int32, device=dev)
                bank.score_batch_device(d_res.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(),
                                        n, hi, sc.data_ptr(), st.cuda_stream, min_len=lo)
                out.append(sc)
            st.synchronize()
            kern, ctr = bank.last_kernel(), bank.counters()
        return [x.cpu().numpy() for x in out], kern, ctr

    (a1, a2), kern, ctr = run("1")
    (b1, _), kern0, _ = run("0")
    assert "balanced" in kern and "dsort" in kern and "balanced" not in kern0, (kern, kern0)
    assert ctr["balanced_calls"] == 2 and ctr["balanced_timeouts"] == 0, ctr
    assert np.array_equal(a1, b1) and np.array_equal(a2, b1)
    rows = np.unique(np.concatenate([rng.choice(n, 3000, replace=False), np.arange(200),
                                     np.arange(n - 200, n)]))
    want = O.score_batch(q, res, np.ascontiguousarray(offs[rows]), np.ascontiguousarray(lens[rows]),
                         O.dna_matrix(*REF[:2]), *REF[2:])
    assert np.array_equal(a1[rows], want)


@pytest.mark.parametrize("mode,tag", [("1", "gather"), ("2", "gather4")])
def test_ragged_sorted_copy(mode, tag, poisoned_buffers, monkeypatch):
    """SWBANK_RAGGED_GATHER (opt-in): the ragged batch copied in its sorted order
    (bytes, or 4-bit codes) and scored without the permutation, each score written through it;
    bit-exact against the default permuted reads on every target, N codes included."""
    torch = pytest.importorskip("torch")
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(17)
    n, lo, hi, qlen = 700_001, 64, 150, 128  # (balanced: tiles x 8 >= 2 x grid x 19 chunks)
    q = O.random_codes(71, qlen, 4)
    lens = rng.integers(lo, hi + 1, n).astype(np.uint32)
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    res = O.random_codes(72, int(lens.sum(dtype=np.uint64)), 4)
    res[rng.choice(res.size, res.size // 100, replace=False)] = 4  # N
    for k in rng.choice(n, n // 50, replace=False):
        m = int(min(lens[k], qlen))
        res[int(offs[k]):int(offs[k]) + m] = q[:m]
    d_res = torch.from_numpy(res).to(dev)
    d_offs = torch.from_numpy(offs.view(np.int64)).to(dev)
    d_lens = torch.from_numpy(lens.view(np.int32)).to(dev)

    monkeypatch.setenv("SWBANK_TRIM", "1")  # (the copy's scores go through the trimmed kernel)

    def run(gather):
        monkeypatch.setenv("SWBANK_RAGGED_GATHER", gather)
        with S.ScoreBank() as bank:
            bank.set_penalties(*REF)
            bank.load_query(q)
            sc = torch.full((n,), -7, dtype=torch.int32, device=dev)
            bank.score_batch_device(d_res.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(), n, hi,
                                    sc.data_ptr(), min_len=lo)
            torch.cuda.synchronize()
            return sc.cpu().numpy(), bank.last_kernel()

    got, kern = run(mode)
    want, kern0 = run("0")
    assert kern.endswith(tag) and "gather" not in kern0, (kern, kern0)
    assert np.array_equal(got, want)
    rows = np.unique(np.concatenate([rng.choice(n, 2000, replace=False), np.arange(100)]))
    ref = O.score_batch(q, res, np.ascontiguousarray(offs[rows]), np.ascontiguousarray(lens[rows]),
                        O.dna_matrix(*REF[:2]), *REF[2:])
    assert np.array_equal(got[rows], ref)


#  SWBANK_BAL_SOAK_SEEDS=n (default 3) / SWBANK_BAL_SOAK_BASE=b: seeds b .. b+n-1 (soak runs)
_SOAK_BASE = int(__import__("os").environ.get("SWBANK_BAL_SOAK_BASE", "0"))
_SOAK_SEEDS = int(__import__("os").environ.get("SWBANK_BAL_SOAK_SEEDS", "3"))


@pytest.mark.parametrize("seed", range(_SOAK_BASE, _SOAK_BASE + _SOAK_SEEDS))
def test_balanced_ragged_soak(seed, monkeypatch):
    """Seeded device batches for the balanced ranges, ragged over the device sort's plan (or, one
    in four, uniform over the host's): random length ranges (short to 2,047 codes), 4-wave query
    lengths, N rates and homologs, the
    batch sized just past the point where balanced ranges apply; bit-exact against whole tiles
    per workgroup (SWBANK_BAL=0) on every target and against the oracle on a sample."""
    torch = pytest.importorskip("torch")
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(40_000 + seed)
    lo = int(rng.integers(1, 200))
    hi = int(min(2047, lo + rng.integers(1, 3 * lo + 8)))
    if rng.random() < 0.25:  # a uniform batch: the host's plan instead of the sort's
        lo = hi = int(rng.integers(1, 400))
    kmin, kmax = max(1, (lo + 7) // 8), (hi + 7) // 8
    # balanced ranges need tiles x kmin >= 2 x grid x kmax (grid <= 1024 slots)
    n = int(2 * 1024 * kmax * 128 / kmin * float(rng.uniform(1.05, 1.5))) + int(rng.integers(0, 128))
    if n > 3_000_000:
        pytest.skip(f"lengths {lo}-{hi}: {n} targets")
    qlen = int(rng.choice([97, 100, 113, 128]))  # 4 waves: the 1,024-slot grid assumed above
    q = O.random_codes(seed + 17, qlen, 4)
    lens = rng.integers(lo, hi + 1, n).astype(np.uint32)
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    res = O.random_codes(seed + 23, int(lens.sum(dtype=np.uint64)), 4)
    if rng.random() < 0.5:
        res[rng.random(res.size) < float(rng.uniform(0.0, 0.02))] = 4  # N
    for k in rng.choice(n, n // 40, replace=False):
        m = int(min(lens[k], qlen))
        res[int(offs[k]):int(offs[k]) + m] = q[:m]
    d_res = torch.from_numpy(res).to(dev)
    d_offs = torch.from_numpy(offs.view(np.int64)).to(dev)
    d_lens = torch.from_numpy(lens.view(np.int32)).to(dev)

    def run(bal):
        monkeypatch.setenv("SWBANK_BAL", bal)
        with S.ScoreBank() as bank:
            bank.set_penalties(*REF)
            bank.load_query(q)
            sc = torch.full((n,), -7, dtype=torch.int32, device=dev)
            bank.score_batch_device(d_res.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(), n, hi,
                                    sc.data_ptr(), min_len=lo)
            torch.cuda.synchronize()
            return sc.cpu().numpy(), bank.last_kernel()

    got, kern = run("1")
    want, kern0 = run("0")
    assert "balanced" in kern and "balanced" not in kern0, (kern, kern0, lo, hi, n)
    assert np.array_equal(got, want), (kern, lo, hi, n, int((got != want).sum()))
    rows = np.unique(np.concatenate([rng.choice(n, 1500, replace=False), np.arange(64),
                                     np.arange(n - 64, n)]))
    ref = O.score_batch(q, res, np.ascontiguousarray(offs[rows]), np.ascontiguousarray(lens[rows]),
                        O.dna_matrix(*REF[:2]), *REF[2:])
    assert np.array_equal(got[rows], ref), kern
