"""GPU parity for query sets (sw_load_queries): a device batch against every query of a set in
one launch per query segment (the tile kernel's several-queries variant: units = (query,
tile) pairs, per-query row LUTs, per-unit edge rows), or one query at a time where that
variant does not apply (profiles, the column-0 rule, optimistic f16).  Every score is checked
against the oracle, query by query, and the one-launch path against the one-at-a-time path
(SWBANK_MQ=0)."""
import numpy as np
import pytest

import swbank as S
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _device_batch(seqs):
    torch = pytest.importorskip("torch")
    dev = torch.device("cuda", 0)
    res, offs, lens = S.pack_targets(seqs)
    return (torch.from_numpy(res).to(dev), torch.from_numpy(offs.astype(np.int64)).to(dev),
            torch.from_numpy(lens.astype(np.int32)).to(dev), int(lens.max()) if len(lens) else 0)


def _score_set(bank, queries, seqs):
    torch = pytest.importorskip("torch")
    d_res, d_offs, d_lens, maxlen = _device_batch(seqs)
    n = len(seqs)
    d_sc = torch.full((len(queries), n), -1, dtype=torch.int32, device=d_res.device)
    s = torch.cuda.Stream()
    bank.score_batch_device(d_res.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(), n, maxlen,
                            d_sc.data_ptr(), s.cuda_stream)
    s.synchronize()
    return d_sc.cpu().numpy()


def _oracle_set(queries, seqs, sub, go, ge, model):
    res, offs, lens = O.pack_residues(seqs)
    return np.stack([O.score_batch(q, res, offs, lens, sub, go, ge, model) for q in queries])


def _targets(rng, n, lo, hi, A, queries=(), p_n=0.0):
    seqs = [rng.integers(0, A, int(rng.integers(lo, hi + 1)), dtype=np.uint8) for _ in range(n)]
    for k in range(0, n, 9):  # local homologs of some query
        q = queries[k % len(queries)] if queries else None
        if q is not None and len(q) > 10:
            a = int(rng.integers(0, len(q) - 5))
            t = q[a:a + int(rng.integers(5, hi + 1))].copy()
            t[::8] = rng.integers(0, A, len(t[::8]))
            seqs[k] = t
    if p_n:
        for t in seqs:
            t[rng.random(len(t)) < p_n] = 4
    return seqs


@pytest.mark.parametrize("arith", ["f16", "u16"])
@pytest.mark.parametrize("model", [S.GAP_MERGED, S.GAP_GOTOH])
@pytest.mark.parametrize("qlens", [(130, 1000, 1000, 513, 40), (17, 200, 129), (1100, 2100, 7)])
def test_query_set_one_launch(monkeypatch, arith, model, qlens):
    """Queries of different lengths (several segments for the longest; the shorter ones padded
    to its layout), a ragged batch with N codes and empty targets."""
    monkeypatch.setenv("SWBANK_F16", "0" if arith == "u16" else "1")
    monkeypatch.setenv("SWBANK_KERNEL", "tile")
    rng = np.random.default_rng(sum(qlens) + model)
    queries = [rng.integers(0, 4, L, dtype=np.uint8) for L in qlens]
    seqs = _targets(rng, 700, 0, 190, 4, queries, p_n=0.02)
    pen = (5, -4, -10, -1) if model == S.GAP_GOTOH else (5, -4, -12, -4)
    with S.ScoreBank(gap_model=model) as bank:
        bank.set_penalties(*pen)
        bank.load_queries(queries)
        assert bank.query_count() == len(queries)
        got = _score_set(bank, queries, seqs)
        kern = bank.last_kernel()
        assert f"queries={len(queries)}" in kern, kern
        monkeypatch.setenv("SWBANK_MQ", "0")
        loop = _score_set(bank, queries, seqs)
    assert np.array_equal(got, loop), kern
    want = _oracle_set(queries, seqs, O.dna_matrix(*pen[:2]), *pen[2:],
                       O.GAP_GOTOH if model == S.GAP_GOTOH else O.GAP_MERGED)
    bad = np.argwhere(got != want)
    assert bad.size == 0, (kern, [(int(i), int(k), int(got[i, k]), int(want[i, k]))
                                  for i, k in bad[:6]])


def test_query_set_edge_ranges(monkeypatch):
    """A tiny edge budget splits the batch into position ranges, each with its own per-unit
    edge rows (several segments, several queries)."""
    monkeypatch.setenv("SWBANK_EDGE_MB", "1")
    monkeypatch.setenv("SWBANK_KERNEL", "tile")
    rng = np.random.default_rng(77)
    queries = [rng.integers(0, 4, L, dtype=np.uint8) for L in (1000, 600, 800)]
    seqs = _targets(rng, 2000, 100, 150, 4, queries)
    with S.ScoreBank() as bank:
        bank.set_penalties(5, -4, -12, -4)
        bank.load_queries(queries)
        got = _score_set(bank, queries, seqs)
        assert "queries=3" in bank.last_kernel()
    assert np.array_equal(got, _oracle_set(queries, seqs, O.dna_matrix(), -12, -4, O.GAP_MERGED))


@pytest.mark.parametrize("case", ["protein", "col0", "optimistic", "wave"])
def test_query_set_one_at_a_time(monkeypatch, case):
    """Where the one-launch variant does not apply the queries run one after the other (the
    scores are the same).  "optimistic": a bound past f16's exact range runs the one-launch
    variant in exact u16 instead of one optimistic f16 pass per query."""
    rng = np.random.default_rng(len(case))
    if case == "wave":
        monkeypatch.setenv("SWBANK_KERNEL", "wave")
    if case == "protein":
        queries = [rng.integers(0, 20, L, dtype=np.uint8) for L in (300, 120)]
        seqs = _targets(rng, 300, 1, 200, 20, queries)
        sub, go, ge, model = O.BLOSUM62, -11, -1, O.GAP_GOTOH
        kw = dict(alphabet=S.ALPHABET_PROTEIN, gap_model=S.GAP_GOTOH)
    else:
        queries = [rng.integers(0, 4, L, dtype=np.uint8) for L in (500, 250, 90)]
        hi = 900 if case == "optimistic" else 200  # optimistic: a bound past 2048
        seqs = _targets(rng, 300, 1, hi, 4, queries)
        if case == "optimistic":
            seqs[3] = np.tile(queries[0], 2)
        pen = (3, -3, -1, -1) if case == "col0" else (5, -4, -12, -4)  # col0: max s > o + e
        sub, go, ge, model = O.dna_matrix(*pen[:2]), pen[2], pen[3], O.GAP_MERGED
        kw = {}
    with S.ScoreBank(**kw) as bank:
        if case == "protein":
            bank.set_matrix(O.BLOSUM62, -11, -1)
        else:
            bank.set_penalties(int(sub[0, 0]), int(sub[0, 1]), go, ge)
        bank.load_queries(queries)
        got = _score_set(bank, queries, seqs)
        kern = bank.last_kernel()
        if case == "optimistic":
            assert kern.startswith("tile u16") and f"queries={len(queries)}" in kern, kern
        else:
            assert f"x{len(queries)} queries" in kern, kern
    assert np.array_equal(got, _oracle_set(queries, seqs, sub, go, ge, model)), kern


def test_query_set_api_rules():
    """The host-buffer and record calls refuse while a set is loaded (SW_ERR_STATE); a best hit
    over a set is unsupported; sw_load_query goes back to one query."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(3)
    queries = [rng.integers(0, 4, 50, dtype=np.uint8) for _ in range(2)]
    seqs = [rng.integers(0, 4, 60, dtype=np.uint8) for _ in range(10)]
    with S.ScoreBank() as bank:
        bank.set_penalties(5, -4, -12, -4)
        bank.load_queries(queries, ids=[7, 8])
        with pytest.raises(S.SwbankError) as ei:
            bank.score_targets(seqs)
        assert ei.value.status == S.ERR_STATE
        d_res, d_offs, d_lens, maxlen = _device_batch(seqs)
        d_ids = torch.arange(10, dtype=torch.int64, device=d_res.device)
        d_sc = torch.zeros((2, 10), dtype=torch.int32, device=d_res.device)
        with pytest.raises(S.SwbankError) as ei:
            bank.score_batch_device(d_res.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(), 10,
                                    maxlen, d_sc.data_ptr(), 0, d_ids=d_ids.data_ptr())
        assert ei.value.status == S.ERR_UNSUPPORTED
        bank.load_query(queries[1])
        assert bank.query_count() == 1
        got = bank.score_targets(seqs)
    res, offs, lens = O.pack_residues(seqs)
    assert np.array_equal(got, O.score_batch(queries[1], res, offs, lens, O.dna_matrix(), -12, -4))


@pytest.mark.parametrize("rows", [512, 256, 128])
@pytest.mark.parametrize("nq", [2, 5, 16, 33])
def test_query_set_pair_tables(monkeypatch, nq, rows):
    """DNA merged f16 sets run on letter-pair tables, one query per workgroup (the grid a
    multiple of nq): 512-row segments (16 waves, 4-column chunks; the default) or 128-row ones
    (4 waves, 8-column chunks), equal to the row-LUT variant (SWBANK_MQ_PAIR=0) and the oracle,
    for set sizes that do and do not divide the resident slots, queries of 1-3 segments."""
    monkeypatch.setenv("SWBANK_KERNEL", "tile")
    monkeypatch.setenv("SWBANK_MQ_PAIR_ROWS", str(rows))
    rng = np.random.default_rng(nq)
    queries = [rng.integers(0, 4, int(rng.integers(60, 1100)), dtype=np.uint8) for _ in range(nq)]
    seqs = _targets(rng, 900, 0, 150, 4, queries, p_n=0.01)
    with S.ScoreBank() as bank:
        bank.set_penalties(5, -4, -12, -4)
        bank.load_queries(queries)
        got = _score_set(bank, queries, seqs)
        kern = bank.last_kernel()
        assert " pair " in kern and f"queries={nq}" in kern, kern
        assert f" W={min(rows, max(len(q) for q in queries) + 31) // 32} " in kern, kern
        monkeypatch.setenv("SWBANK_MQ_PAIR", "0")
        bank.load_queries(queries)  # the tables are rebuilt without pair tables
        lut = _score_set(bank, queries, seqs)
        assert " pair " not in bank.last_kernel()
    assert np.array_equal(got, lut), kern
    want = _oracle_set(queries, seqs, O.dna_matrix(), -12, -4, O.GAP_MERGED)
    bad = np.argwhere(got != want)
    assert bad.size == 0, (kern, [(int(i), int(k), int(got[i, k]), int(want[i, k]))
                                  for i, k in bad[:6]])


@pytest.mark.parametrize("qmax", [513, 520, 530, 1025])
def test_query_set_pair_short_last_segment(monkeypatch, poisoned_buffers, qmax):
    """A set whose longest query ends just past a 512-row segment: the last segment has 1-2
    waves.  Every segment must run with the same column chunk (4), so the last one reads exactly
    the edge columns the one before it wrote (with 8 it read up to 4 columns nobody wrote,
    bytes from earlier allocations, and short tiles scored their padding columns)."""
    monkeypatch.setenv("SWBANK_KERNEL", "tile")
    rng = np.random.default_rng(qmax)
    queries = [rng.integers(0, 4, L, dtype=np.uint8) for L in (qmax, 100, 300)]
    seqs = _targets(rng, 700, 0, 21, 4, queries, p_n=0.01)  # many tiles of 1-6 chunks
    with S.ScoreBank() as bank:
        bank.set_penalties(5, -4, -12, -4)
        bank.load_queries(queries)
        got = _score_set(bank, queries, seqs)
        kern = bank.last_kernel()
    assert " pair " in kern, kern
    want = _oracle_set(queries, seqs, O.dna_matrix(), -12, -4, O.GAP_MERGED)
    bad = np.argwhere(got != want)
    assert bad.size == 0, (kern, [(int(i), int(k), int(got[i, k]), int(want[i, k]))
                                  for i, k in bad[:6]])
