"""GPU: balanced ranges of the two-pairs protein wave kernel.

Every resident wave slot scores the same number of 32-step blocks of the unit sequence (a unit =
two pairs = four targets); a unit cut by a range boundary is scored in two visits by two waves
(or, with fewer units than slots, in up to four: middle visits), the lane state (rows, running
best, diagonal, bottom row) handed over through global memory and a flag.  configs[4]'s 12,500
targets per GPU are 3,125 units on 3,072 wave slots of 4-wave blocks: without the balance the
last 53 units would set the kernel's length (or run as a segmented tail); from 16,384 targets
the launch takes 8-wave blocks (4,096 slots, 4 waves per SIMD).

Checked: bit-exact against SWBANK_WAVE_BAL=0 (the segmented-tail path) and against the oracle on
every target, over batch sizes just past one unit per slot to 1.5 units per slot, an odd target
count (a last unit with one target), both gap models, homologous targets whose scores pass the
optimistic f16 threshold inside cut units (re-scored in u16 by the finishing visit), back-to-back
calls (the flags' generation), poisoned device buffers, and a host-buffer call."""
import numpy as np
import pytest

import swbank as S
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _batch(rng, n, qlen, L):
    q = rng.integers(0, 20, qlen, dtype=np.uint8)
    res = rng.integers(0, 20, n * L, dtype=np.uint8)
    for k in rng.choice(n, max(4, n // 400), replace=False):  # near-copies: scores past 2048
        t = np.resize(q, L).copy()
        t[::9] = rng.integers(0, 20, len(t[::9]))
        res[k * L:(k + 1) * L] = t
    return q, res, np.arange(n, dtype=np.uint64) * L, np.full(n, L, np.uint32)


@pytest.mark.parametrize("n,model,w", [(12_500, S.GAP_GOTOH, 8), (12_290, S.GAP_GOTOH, 8),
                                       (18_001, S.GAP_MERGED, 8), (12_500, S.GAP_MERGED, 8),
                                       (8_000, S.GAP_GOTOH, 8), (5_001, S.GAP_MERGED, 8),
                                       (12_500, S.GAP_GOTOH, 4), (18_001, S.GAP_MERGED, 4),
                                       (12_500, S.GAP_GOTOH, 0), (18_001, S.GAP_GOTOH, 0)])
def test_wave_balanced_exact(n, model, w, monkeypatch, poisoned_buffers):
    """w = 8 (default): 8-wave blocks, 4 waves per SIMD, 4,096 wave slots: configs[4]'s 3,125
    units are fewer than the slots, so units are cut up to twice (8,000 / 5,001 targets: up to
    three and four times), middle visits waiting for their predecessor and handing on to their
    successor.  w = 4 (SWBANK_WAVE_W=4): 3,072 slots, each unit cut at most once.  w = 0: the
    library's choice -- 8-wave blocks from a unit per slot (18,001 targets), else 4."""
    torch = pytest.importorskip("torch")
    if w:
        monkeypatch.setenv("SWBANK_WAVE_W", str(w))
    else:
        monkeypatch.delenv("SWBANK_WAVE_W", raising=False)
        w = 8 if n >= 16_384 else 4
    rng = np.random.default_rng(n + model)
    qlen, L = 512, 1000
    q, res, offs, lens = _batch(rng, n, qlen, L)
    dev = torch.device("cuda", 0)
    d_res = torch.from_numpy(res).to(dev)
    d_offs = torch.from_numpy(offs.view(np.int64)).to(dev)
    d_lens = torch.from_numpy(lens.view(np.int32)).to(dev)

    def run(bal):
        monkeypatch.setenv("SWBANK_WAVE_BAL", bal)
        out = []
        with S.ScoreBank(alphabet=S.ALPHABET_PROTEIN, gap_model=model) as bank:
            bank.set_matrix(O.BLOSUM62, -11, -1)
            bank.load_query(q)
            for _ in range(2):  # back to back: the second call's flags carry a new generation
                sc = torch.full((n,), -7, dtype=torch.int32, device=dev)
                bank.score_batch_device(d_res.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(),
                                        n, L, sc.data_ptr(), min_len=L)
                out.append(sc)
            bank.sync()
            kern, ctr = bank.last_kernel(), bank.counters()
        return [x.cpu().numpy() for x in out], kern, ctr

    (a1, a2), kern, ctr = run("1")
    (b1, _), kern0, _ = run("0")
    assert "pairs/wave=2" in kern and "balanced" in kern and f"x{w}" in kern, kern
    assert "balanced" not in kern0, kern0
    assert ctr["tail_timeouts"] == 0 and ctr["balanced_timeouts"] == 0, ctr
    want = O.score_batch(q, res, offs, lens, O.BLOSUM62, -11, -1,
                         O.GAP_GOTOH if model == S.GAP_GOTOH else O.GAP_MERGED)
    assert want.max() > 2048  # the optimistic f16 re-score runs
    for got in (a1, a2, b1):
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, (kern, [(int(i), int(got[i]), int(want[i])) for i in bad[:8]])


def test_wave_balanced_needs_one_unit_per_slot(monkeypatch):
    """Fewer units than wave slots (or a whole number of units per slot) keeps one unit per
    wave (with the segmented tail where it applies)."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(5)
    q, res, offs, lens = _batch(rng, 4_000, 512, 300)
    dev = torch.device("cuda", 0)
    d = [torch.from_numpy(x).to(dev) for x in (res, offs.view(np.int64), lens.view(np.int32))]
    sc = torch.empty(4_000, dtype=torch.int32, device=dev)
    with S.ScoreBank(alphabet=S.ALPHABET_PROTEIN, gap_model=S.GAP_GOTOH) as bank:
        bank.set_matrix(O.BLOSUM62, -11, -1)
        bank.load_query(q)
        bank.score_batch_device(d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), 4_000, 300,
                                sc.data_ptr(), min_len=300)
        bank.sync()
        assert "balanced" not in bank.last_kernel()
    want = O.score_batch(q, res, offs, lens, O.BLOSUM62, -11, -1, O.GAP_GOTOH)
    assert np.array_equal(sc.cpu().numpy(), want)


def test_wave_balanced_host_call(monkeypatch):
    """The host-buffer API on configs[4]'s shape: equal-length chunks reach the balanced path
    when a chunk holds a unit per slot, and the scores are exact either way."""
    rng = np.random.default_rng(11)
    n, L = 12_500, 1000
    q, res, offs, lens = _batch(rng, n, 512, L)
    with S.ScoreBank(alphabet=S.ALPHABET_PROTEIN, gap_model=S.GAP_GOTOH) as bank:
        bank.set_matrix(O.BLOSUM62, -11, -1)
        bank.load_query(q)
        got = bank.score_batch(res, offs, lens)
    want = O.score_batch(q, res, offs, lens, O.BLOSUM62, -11, -1, O.GAP_GOTOH)
    assert np.array_equal(got, want)


def test_wave_balanced_stall_fails_loudly(monkeypatch):
    """A tail visit whose predecessor never publishes: SW_ERR_TIMEOUT at sw_bank_sync (device
    call), a re-run without hand-offs for a host call; exact again afterwards."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(12)
    n, L = 12_500, 1000
    q, res, offs, lens = _batch(rng, n, 512, L)
    want = O.score_batch(q, res, offs, lens, O.BLOSUM62, -11, -1, O.GAP_GOTOH)
    dev = torch.device("cuda", 0)
    d = [torch.from_numpy(x).to(dev) for x in (res, offs.view(np.int64), lens.view(np.int32))]
    sc = torch.full((n,), -7, dtype=torch.int32, device=dev)
    with S.ScoreBank(alphabet=S.ALPHABET_PROTEIN, gap_model=S.GAP_GOTOH) as bank:
        bank.set_matrix(O.BLOSUM62, -11, -1)
        bank.load_query(q)
        monkeypatch.setenv("SWBANK_STALL", "7")
        monkeypatch.setenv("SWBANK_POLL_LIMIT", "2000")
        bank.score_batch_device(d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), n, L,
                                sc.data_ptr(), min_len=L)
        assert "balanced" in bank.last_kernel()
        with pytest.raises(S.SwbankError) as ei:
            bank.sync()
        assert ei.value.status == S.ERR_TIMEOUT
        # the kind is counted and named (it used to count nothing, name nothing)
        assert "wave balanced ranges" in str(ei.value), str(ei.value)
        ctr = bank.counters()
        assert ctr["wave_balanced_timeouts"] == 1 and ctr["balanced_timeouts"] == 0, ctr
        monkeypatch.delenv("SWBANK_STALL")
        monkeypatch.delenv("SWBANK_POLL_LIMIT")
        bank.score_batch_device(d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), n, L,
                                sc.data_ptr(), min_len=L)
        bank.sync()
        assert np.array_equal(sc.cpu().numpy(), want)


#  SWBANK_WBAL_SOAK_SEEDS=n (default 3) / SWBANK_WBAL_SOAK_BASE=b: seeds b .. b+n-1
_WS_BASE = int(__import__("os").environ.get("SWBANK_WBAL_SOAK_BASE", "0"))
_WS_SEEDS = int(__import__("os").environ.get("SWBANK_WBAL_SOAK_SEEDS", "3"))


@pytest.mark.parametrize("seed", range(_WS_BASE, _WS_BASE + _WS_SEEDS))
def test_wave_balanced_soak(seed, monkeypatch):
    """Seeded protein batches for the balanced two-pairs kernel: random target length (equal in
    a batch), query length (500-512 rows), batch size from one unit per wave slot to three, gap
    model and penalties; bit-exact against the segmented-tail
    path (SWBANK_WAVE_BAL=0) on every target and against the oracle on a sample."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(70_000 + seed)
    # (shapes the kernel choice sends to the balanced two-pairs kernel: a query of nearly 512
    # rows against long targets -- else the tile kernel wins -- and, for merged gaps, o + e
    # above BLOSUM62's largest score, so the column-0 rule is off)
    L = int(rng.integers(850, 1300))
    qlen = int(rng.integers(500, 513))
    n = int(rng.integers(12_300, 37_000))
    model = S.GAP_GOTOH if rng.random() < 0.6 else S.GAP_MERGED
    go, ge = -int(rng.integers(10, 15)), -int(rng.integers(1, 4))
    q, res, offs, lens = _batch(rng, n, qlen, L)
    dev = torch.device("cuda", 0)
    d_res = torch.from_numpy(res).to(dev)
    d_offs = torch.from_numpy(offs.view(np.int64)).to(dev)
    d_lens = torch.from_numpy(lens.view(np.int32)).to(dev)

    def run(bal):
        monkeypatch.setenv("SWBANK_WAVE_BAL", bal)
        with S.ScoreBank(alphabet=S.ALPHABET_PROTEIN, gap_model=model) as bank:
            bank.set_matrix(O.BLOSUM62, go, ge)
            bank.load_query(q)
            sc = torch.full((n,), -7, dtype=torch.int32, device=dev)
            bank.score_batch_device(d_res.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(), n, L,
                                    sc.data_ptr(), min_len=L)
            bank.sync()
            return sc.cpu().numpy(), bank.last_kernel()

    got, kern = run("1")
    want, kern0 = run("0")
    assert "pairs/wave=2" in kern and "balanced" in kern and "balanced" not in kern0, (kern, kern0)
    assert np.array_equal(got, want), (kern, L, qlen, n, int((got != want).sum()))
    rows = np.unique(np.concatenate([rng.choice(n, 300, replace=False), np.arange(n - 40, n)]))
    ref = O.score_batch(q, res, np.ascontiguousarray(offs[rows]), np.ascontiguousarray(lens[rows]),
                        O.BLOSUM62, go, ge, O.GAP_GOTOH if model == S.GAP_GOTOH else O.GAP_MERGED)
    assert np.array_equal(got[rows], ref), kern
