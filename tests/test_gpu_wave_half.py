"""GPU parity for the wave kernel's two-pairs-per-wave form (swbank_kwave.hip wave_two_pairs:
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


@pytest.mark.parametrize("P", [4, 8])
@pytest.mark.parametrize("split", [1, 2, 5, 64])
def test_half_with_split_tail(monkeypatch, split, P):
    """The split tail beside the two-pairs blocks: P = 4, one pair per block of 4 segment waves
    ahead of them (barrier hand-off), or P = 8, 64-row segments one wave each after them (hand-off
    through global memory; the policy's choice for a tail of at most SIMDs / 8 pairs)."""
    monkeypatch.setenv("SWBANK_KERNEL", "wave")
    monkeypatch.setenv("SWBANK_WAVE_SPLIT", str(split))
    monkeypatch.setenv("SWBANK_WAVE_SPLIT_P", str(P))
    rng = np.random.default_rng(split)
    q = rng.integers(0, 20, 512, dtype=np.uint8)
    seqs = _targets(rng, 301, 1, 1000, 20, q, homologs=3)
    with S.ScoreBank(alphabet=S.ALPHABET_PROTEIN, gap_model=S.GAP_GOTOH) as bank:
        bank.set_matrix(O.BLOSUM62, -11, -1)
        bank.load_query(q)
        got, one, kern = _both(monkeypatch, bank, lambda: bank.score_targets(seqs))
    tag = f"tail={split}/8" if P == 8 else f"split={split}/4"
    assert "pairs/wave=2" in kern and tag in kern, kern
    res, offs, lens = O.pack_residues(seqs)
    want = O.score_batch(q, res, offs, lens, O.BLOSUM62, -11, -1, O.GAP_GOTOH)
    assert np.array_equal(got, want) and np.array_equal(one, want), kern


@pytest.mark.parametrize("tail", ["default", "split4"])
@pytest.mark.parametrize("model", [S.GAP_GOTOH, S.GAP_MERGED])
@pytest.mark.parametrize("n,qlen", [(12500, 512), (2300, 480), (4127, 300)])
def test_half_segmented_tail_policy(monkeypatch, poisoned_buffers, model, n, qlen, tail):
    """The policy's own tail (configs[4]'s shape: 6,250 pairs = 3 two-pair waves per SIMD + 106
    pairs, as 8 x 64-row segments on separate SIMDs by default, or as P = 4 row segments in one
    block with SWBANK_WAVE_SPLIT_P=4), ragged and empty targets among the tail pairs,
    near-copies of the query past 2048 in the tail (the last segment re-scores its pair in u16),
    both gap models, poisoned device buffers; device API (no host chunking)."""
    torch = pytest.importorskip("torch")
    monkeypatch.setenv("SWBANK_KERNEL", "wave")
    if tail == "split4":
        monkeypatch.setenv("SWBANK_WAVE_SPLIT_P", "4")
    rng = np.random.default_rng(n + qlen + model)
    q = rng.integers(0, 20, qlen, dtype=np.uint8)
    seqs = _targets(rng, n, 900, 1000, 20)
    for k in range(n - 220, n, 7):  # the tail's pairs: ragged, empty, homologous
        seqs[k] = rng.integers(0, 20, int(rng.integers(0, 1000)), dtype=np.uint8)
    seqs[n - 3] = np.zeros(0, np.uint8)
    for k in (n - 5, n - 40, n - 150):
        t = np.resize(q, 1000).copy()
        t[::13] = rng.integers(0, 20, len(t[::13]))
        seqs[k] = t
    res, offs, lens = O.pack_residues(seqs)
    dev = torch.device("cuda", 0)
    d_res = torch.from_numpy(res).to(dev)
    d_offs = torch.from_numpy(offs.view(np.int64)).to(dev)
    d_lens = torch.from_numpy(lens.view(np.int32)).to(dev)
    d_sc = torch.full((n,), -9, dtype=torch.int32, device=dev)
    with S.ScoreBank(alphabet=S.ALPHABET_PROTEIN, gap_model=model) as bank:
        bank.set_matrix(O.BLOSUM62, -11, -1)
        bank.load_query(q)
        bank.score_batch_device(d_res.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(), n,
                                int(lens.max()), d_sc.data_ptr())
        torch.cuda.synchronize()
        kern = bank.last_kernel()
    got = d_sc.cpu().numpy()
    assert "pairs/wave=2" in kern, kern
    if n == 12500:
        assert ("split=106/4" if tail == "split4" else "tail=106/8") in kern, kern
    want = O.score_batch(q, res, offs, lens, O.BLOSUM62, -11, -1,
                         O.GAP_GOTOH if model == S.GAP_GOTOH else O.GAP_MERGED)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, (kern, [(int(i), int(lens[i]), int(got[i]), int(want[i]))
                                  for i in bad[:8]])
    if qlen == 512:  # (a 300-row query's near-copies stay below 2048)
        assert want[n - 5] > 2048


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
