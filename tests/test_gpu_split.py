"""GPU parity for the wave kernel's split tail: pairs past a whole number of waves per SIMD run
as two half-height row segments (one wave each, the upper segment's bottom row handed down
through a 256-column ring one 64-step phase apart).  SWBANK_WAVE_SPLIT=N forces the last N
pairs through it; every case is checked against the oracle."""
import numpy as np
import pytest

import swbank as S
from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, params=["f16-P2", "u16-P2", "f16-P4", "u16-P4"])
def arith(request, monkeypatch):
    """Both arithmetics, each with 2 and 4 row segments per split pair."""
    ar, p = request.param.split("-")
    monkeypatch.setenv("SWBANK_KERNEL", "wave")
    monkeypatch.setenv("SWBANK_F16", "0" if ar == "u16" else "1")
    monkeypatch.setenv("SWBANK_WAVE_SPLIT_P", p[1])
    return request.param


def _targets(rng, n, lo, hi, alpha, q=None, homologs=0):
    seqs = [rng.integers(0, alpha, int(rng.integers(lo, hi + 1)), dtype=np.uint8)
            for _ in range(n)]
    for k in range(homologs):  # near-copies of the query: scores far above 2048 (optimistic f16)
        j = int(rng.integers(0, n))
        t = q.copy()
        t[::11] = rng.integers(0, alpha, len(t[::11]))
        seqs[j] = t
    return seqs


def _check(bank, q, seqs, sub, go, ge, model, split, expect_split=True):
    got = bank.score_targets(seqs)
    res, offs, lens = O.pack_residues(seqs)
    want = O.score_batch(q, res, offs, lens, sub, go, ge, model)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, (bank.last_kernel(), [(int(i), int(lens[i]), int(got[i]),
                                                 int(want[i])) for i in bad[:8]])
    if expect_split:
        assert f"split={split}/" in bank.last_kernel(), bank.last_kernel()


@pytest.mark.parametrize("qlen", [257, 300, 511, 512, 600, 1024])
@pytest.mark.parametrize("split", [1, 2, 7, 64])
def test_split_protein_gotoh(qlen, split, monkeypatch):
    """BLOSUM62 Gotoh (configs[4]'s model), K = 8 (queries 257-512) and K = 16 (513-1024):
    split counts odd (a block with one real pair) and even, ragged targets incl. empty ones."""
    rng = np.random.default_rng(qlen * 100 + split)
    q = rng.integers(0, 20, qlen, dtype=np.uint8)
    seqs = _targets(rng, 150, 0, 700, 20, q, homologs=3)
    monkeypatch.setenv("SWBANK_WAVE_SPLIT", str(split))
    with S.ScoreBank(alphabet=S.ALPHABET_PROTEIN, gap_model=S.GAP_GOTOH) as bank:
        bank.set_matrix(O.BLOSUM62, -11, -1)
        bank.load_query(q)
        _check(bank, q, seqs, O.BLOSUM62, -11, -1, O.GAP_GOTOH, split)


@pytest.mark.parametrize("model", [S.GAP_MERGED, S.GAP_GOTOH])
@pytest.mark.parametrize("pen", [(5, -4, -12, -4), (2, -3, -1, -1)])
def test_split_dna_lut_all_pairs(model, pen, monkeypatch):
    """DNA LUT kernels, every pair split (the whole batch is tail); (2, -3, -1, -1) with the
    merged model has max(s) > o + e: the HDL column-0 rule in both segments."""
    rng = np.random.default_rng(7 + model)
    q = rng.integers(0, 5, 400, dtype=np.uint8)
    seqs = _targets(rng, 101, 1, 900, 5, q, homologs=2)
    monkeypatch.setenv("SWBANK_WAVE_SPLIT", "1000000")
    with S.ScoreBank(gap_model=model) as bank:
        bank.set_penalties(*pen)
        bank.load_query(q)
        _check(bank, q, seqs, O.dna_matrix(pen[0], pen[1]), pen[2], pen[3], model, 51)


def test_split_protein_merged_col0(monkeypatch):
    """Protein profile, merged gaps with the column-0 rule live (BLOSUM62, -2/-1)."""
    rng = np.random.default_rng(21)
    q = rng.integers(0, 20, 480, dtype=np.uint8)
    seqs = _targets(rng, 90, 1, 500, 20, q, homologs=2)
    monkeypatch.setenv("SWBANK_WAVE_SPLIT", "30")
    with S.ScoreBank(alphabet=S.ALPHABET_PROTEIN) as bank:
        bank.set_matrix(O.BLOSUM62, -2, -1)
        bank.load_query(q)
        _check(bank, q, seqs, O.BLOSUM62, -2, -1, O.GAP_MERGED, 30)


def test_split_records(monkeypatch):
    """The CAPI record path (2-bit codes read in-kernel) through split blocks."""
    rng = np.random.default_rng(5)
    q = rng.integers(0, 4, 300, dtype=np.uint8)
    codes = rng.integers(0, 4, (77, 200), dtype=np.uint8)
    recs = S.make_records(codes)
    monkeypatch.setenv("SWBANK_WAVE_SPLIT", "13")
    with S.ScoreBank() as bank:
        bank.set_penalties(5, -4, -12, -4)
        bank.load_query(q)
        got = bank.score_records(recs)
        assert "split=13/" in bank.last_kernel(), bank.last_kernel()
    seqs = list(codes)
    res, offs, lens = O.pack_residues(seqs)
    want = O.score_batch(q, res, offs, lens, O.dna_matrix(), -12, -4)
    assert np.array_equal(got, want)


def test_split_auto_policy(arith):
    """Without the override a batch of U x k + r pairs (r <= U / 2) splits its last r pairs,
    U = the pairs of one wave per SIMD: SIMDs, or 2 x SIMDs for the f16 profile kernel's two
    pairs per wave; the scores match the unsplit run (SWBANK_WAVE_SPLIT=0) and a sample of
    them the oracle."""
    import os

    import torch
    simds = 4 * torch.cuda.get_device_properties(0).multi_processor_count
    rng = np.random.default_rng(99)
    q = rng.integers(0, 20, 512, dtype=np.uint8)
    units = 2 * simds if arith.startswith("f16") else simds
    n = 2 * (units + 37)
    seqs = [rng.integers(0, 20, 120, dtype=np.uint8) for _ in range(n)]
    with S.ScoreBank(alphabet=S.ALPHABET_PROTEIN, gap_model=S.GAP_GOTOH) as bank:
        bank.set_matrix(O.BLOSUM62, -11, -1)
        bank.load_query(q)
        got = bank.score_targets(seqs)
        assert "split=37/" in bank.last_kernel(), bank.last_kernel()
        os.environ["SWBANK_WAVE_SPLIT"] = "0"
        try:
            ref = bank.score_targets(seqs)
            assert "split" not in bank.last_kernel()
        finally:
            del os.environ["SWBANK_WAVE_SPLIT"]
    assert np.array_equal(got, ref)
    tail = seqs[-80:]
    res, offs, lens = O.pack_residues(tail)
    want = O.score_batch(q, res, offs, lens, O.BLOSUM62, -11, -1, O.GAP_GOTOH)
    assert np.array_equal(got[-80:], want)
