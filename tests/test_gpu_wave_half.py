"""GPU parity for the wave kernel's two-pairs-per-wave form (swbank_kernels.hip wave_two_pairs:
f16 profile, queries of 257-512 rows, lanes 0-31 on one pair and 32-63 on the next, 16 rows per
lane).  Every case against the oracle and against one pair per wave (SWBANK_WAVE_HALF=0):
odd pair counts (a last wave with one real half), empty and ragged targets, the split tail
beside it, near-copies of the query (scores far past 2048: the in-kernel u16 re-score of a
flagged half), both gap models, and DNA profile matrices fed as 2-bit / 4-bit host chunks and
as CAPI records (the packed code loads)."""
import numpy as np
import pytest

import swbank as S
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _targets(rng, n, lo, hi, alpha, q=None, homologs=0):
    seqs = [rng.integers(0, alpha, int(rng.integers(lo, hi + 1)), dtype=np.uint8)
            for _ in range(n)]
    for k in range(homologs):
        j = int(rng.integers(0, n))
        t = q.copy()
        t[::11] = rng.integers(0, alpha, len(t[::11]))
        seqs[j] = t
    return seqs


def _both(monkeypatch, bank, score):
    """Scores with two pairs per wave (and its kernel name), then with one pair per wave."""
    monkeypatch.delenv("SWBANK_WAVE_HALF", raising=False)
    got = score()
    kern = bank.last_kernel()
    monkeypatch.setenv("SWBANK_WAVE_HALF", "0")
    one = score()
    assert "pairs/wave=2" not in bank.last_kernel()
    monkeypatch.delenv("SWBANK_WAVE_HALF")
    return got, one, kern


@pytest.mark.parametrize("model", [S.GAP_GOTOH, S.GAP_MERGED])
@pytest.mark.parametrize("qlen", [257, 400, 512])
@pytest.mark.parametrize("n", [1, 2, 3, 4, 17, 333])
def test_half_protein(monkeypatch, model, qlen, n):
    monkeypatch.setenv("SWBANK_KERNEL", "wave")
    rng = np.random.default_rng(qlen * 1000 + n + 7 * model)
    q = rng.integers(0, 20, qlen, dtype=np.uint8)
    seqs = _targets(rng, n, 0, 900, 20, q, homologs=min(2, n))
    with S.ScoreBank(alphabet=S.ALPHABET_PROTEIN, gap_model=model) as bank:
        bank.set_matrix(O.BLOSUM62, -11, -1)
        bank.load_query(q)
        got, one, kern = _both(monkeypatch, bank, lambda: bank.score_targets(seqs))
    assert "pairs/wave=2" in kern, kern
    res, offs, lens = O.pack_residues(seqs)
    want = O.score_batch(q, res, offs, lens, O.BLOSUM62, -11, -1,
                         O.GAP_GOTOH if model == S.GAP_GOTOH else O.GAP_MERGED)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, (kern, [(int(i), int(lens[i]), int(got[i]), int(want[i]))
                                  for i in bad[:8]])
    assert np.array_equal(one, want)


@pytest.mark.parametrize("split", [1, 2, 5, 64])
def test_half_with_split_tail(monkeypatch, split):
    """The split tail's blocks (one pair per 2 or 4 waves) ahead of the two-pairs blocks."""
    monkeypatch.setenv("SWBANK_KERNEL", "wave")
    monkeypatch.setenv("SWBANK_WAVE_SPLIT", str(split))
    rng = np.random.default_rng(split)
    q = rng.integers(0, 20, 512, dtype=np.uint8)
    seqs = _targets(rng, 301, 1, 1000, 20, q, homologs=3)
    with S.ScoreBank(alphabet=S.ALPHABET_PROTEIN, gap_model=S.GAP_GOTOH) as bank:
        bank.set_matrix(O.BLOSUM62, -11, -1)
        bank.load_query(q)
        got, one, kern = _both(monkeypatch, bank, lambda: bank.score_targets(seqs))
    assert "pairs/wave=2" in kern and f"split={split}/" in kern, kern
    res, offs, lens = O.pack_residues(seqs)
    want = O.score_batch(q, res, offs, lens, O.BLOSUM62, -11, -1, O.GAP_GOTOH)
    assert np.array_equal(got, want) and np.array_equal(one, want), kern


@pytest.mark.parametrize("layout", ["2bit", "nibble", "records"])
def test_half_dna_profile_packed(monkeypatch, layout):
    """A DNA matrix the row-LUT kernels cannot take (a non-uniform N column) runs in profile
    mode; host chunks arrive as 2-bit or 4-bit codes, records as 2-bit sequence_t data."""
    monkeypatch.setenv("SWBANK_KERNEL", "wave")
    monkeypatch.setenv("SWBANK_STREAM", "0")
    rng = np.random.default_rng(len(layout))
    m = O.dna_matrix(5, -4).astype(np.int8).copy()
    m[4, :4] = m[:4, 4] = np.array([-1, -2, -3, -1], np.int8)
    q = rng.integers(0, 4, 450, dtype=np.uint8)
    hi = 232 if layout == "records" else 700
    seqs = _targets(rng, 257, 1, hi, 4, q[:hi] if hi < 450 else q, homologs=2)
    if layout == "nibble":
        for t in seqs[::5]:
            t[rng.random(len(t)) < 0.05] = 4
    with S.ScoreBank(gap_model=S.GAP_GOTOH) as bank:
        bank.set_matrix(m, -6, -2)
        bank.load_query(q)
        if layout == "records":
            rec = S.make_records(seqs)
            got, one, kern = _both(monkeypatch, bank, lambda: bank.score_records(rec))
        else:
            got, one, kern = _both(monkeypatch, bank, lambda: bank.score_targets(seqs))
    assert "pairs/wave=2" in kern, kern
    res, offs, lens = O.pack_residues(seqs)
    want = O.score_batch(q, res, offs, lens, m, -6, -2, O.GAP_GOTOH)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, (kern, [(int(i), int(lens[i]), int(got[i]), int(want[i]))
                                  for i in bad[:8]])
    assert np.array_equal(one, want)
