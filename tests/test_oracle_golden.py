"""Pin the oracle (CPU restatement) against every golden vector the reference holds.

Sources (tests/golden/, written by tests/golden/make_golden.py from /root/reference/data):
  * 730 ScoreBank HDL transcript scores  (data/*_out.txt; ScoreBank/ScoreBank_v1_tb.sv:271-285)
  * 598 ssearch36 scores                 (data/score.txt, data/score500.txt column 6)
  * the CAPI host's result for query1 vs db18 (build/main_test_output.txt: "result: 102")
  * swalign negative control             (data/sw_testing.txt; gap = go + (k-1)*ge)
  * charTo2bit bytes for query1          (build/main_test_output.txt)
"""
import itertools
import os

import numpy as np
import pytest

from oracle import oracle as O

REF_PARAMS = (O.REF_GAP_OPEN, O.REF_GAP_EXTEND)


def _fasta_cache():
    cache = {}

    def get(name):
        if name not in cache:
            cache[name] = dict(O.read_fasta(O.golden_fasta(name)))
        return cache[name]
    return get


FA = _fasta_cache()


def _query(name):
    recs = O.read_fasta(O.golden_fasta(name))
    return O.encode_dna(recs[0][1])


def test_golden_counts():
    rows = O.load_ref_scores()
    by_src = {}
    for r in rows:
        by_src[r[0]] = by_src.get(r[0], 0) + 1
    assert by_src == {"hdl": 730, "ssearch36": 598, "capi": 1}


@pytest.mark.parametrize("model", [O.GAP_MERGED, O.GAP_GOTOH])
def test_oracle_matches_every_golden_score(model):
    sub = O.dna_matrix()
    bad = []
    for src, lib, q, t, s in O.load_ref_scores():
        got = O.score_pair(_query(q), O.encode_dna(FA(lib)[t]), sub, *REF_PARAMS, model)
        if got != s:
            bad.append((src, lib, t, s, got))
    assert not bad, bad[:10]


def test_rtl_model_matches_every_golden_score():
    """Bit-level 12-bit biased model of the PE array reproduces the transcripts too."""
    sub = O.dna_matrix()
    for src, lib, q, t, s in O.load_ref_scores():
        assert O.score_pair_rtl(_query(q), O.encode_dna(FA(lib)[t]), sub, *REF_PARAMS, 12) == s


def test_batch_api_matches_pairwise():
    sub = O.dna_matrix()
    q = _query("query100.fa")
    recs = O.read_fasta(O.golden_fasta("data500.fa"))
    seqs = [O.encode_dna(s) for _, s in recs]
    res, offs, lens = O.pack_residues(seqs)
    out = O.score_batch(q, res, offs, lens, sub, *REF_PARAMS)
    want = {t: s for src, lib, qq, t, s in O.load_ref_scores() if lib == "data500.fa" and
            src == "hdl"}
    for (name, _), got in zip(recs, out):
        if name in want:
            assert got == want[name], name


def test_swalign_negative_control():
    """swalign charges go+(k-1)*ge; under the reference convention 4/16 must differ."""
    sub = O.dna_matrix()
    q = _query("query1.fa")
    ctrl = O.load_swalign_control()
    diff = sorted(t for t, s in ctrl.items()
                  if O.score_pair(q, O.encode_dna(FA("data1.fa")[t]), sub, *REF_PARAMS) != s)
    assert diff == ["db10", "db12", "db13", "db8"]
    # ...and Gotoh with open' = open - extend reproduces all 16 (it is the same model).
    for t, s in ctrl.items():
        assert O.score_pair(q, O.encode_dna(FA("data1.fa")[t]), sub, -12 + 4, -4,
                            O.GAP_GOTOH) == s


def test_c_matches_pure_python_random():
    rng = np.random.default_rng(7)
    for model, fn in ((O.GAP_MERGED, O.py_score_merged), (O.GAP_GOTOH, O.py_score_gotoh)):
        for params in ((5, -4, -12, -4), (5, -4, -10, -1), (2, -3, -5, -2), (20, -4, -2, -1)):
            sub = O.dna_matrix(params[0], params[1])
            for _ in range(40):
                q = rng.integers(0, 5, rng.integers(0, 40), dtype=np.uint8)
                t = rng.integers(0, 5, rng.integers(0, 40), dtype=np.uint8)
                assert O.score_pair(q, t, sub, params[2], params[3], model) == \
                    fn(list(q), list(t), sub, params[2], params[3])


def test_merged_equals_gotoh_when_2ge_le_min_sub():
    """the models agree when 2*ge <= min substitution, differ otherwise."""
    rng = np.random.default_rng(11)
    sub = O.dna_matrix(5, -4)
    seqs = [(rng.integers(0, 4, 60, dtype=np.uint8), rng.integers(0, 4, 60, dtype=np.uint8))
            for _ in range(200)]
    for q, t in seqs:
        assert O.score_pair(q, t, sub, -12, -4, O.GAP_MERGED) == \
            O.score_pair(q, t, sub, -12, -4, O.GAP_GOTOH)
    ndiff = sum(O.score_pair(q, t, sub, -10, -1, O.GAP_MERGED) !=
                O.score_pair(q, t, sub, -10, -1, O.GAP_GOTOH) for q, t in seqs)
    assert ndiff > 0
    # merged never scores below Gotoh (it only adds corner-turning gaps)
    for q, t in seqs[:50]:
        assert O.score_pair(q, t, sub, -10, -1, O.GAP_MERGED) >= \
            O.score_pair(q, t, sub, -10, -1, O.GAP_GOTOH)


def test_rtl_equals_exact_below_12bit_limit_and_wraps_above():
    rng = np.random.default_rng(3)
    sub = O.dna_matrix()
    for _ in range(100):
        q = rng.integers(0, 4, rng.integers(1, 129), dtype=np.uint8)
        t = rng.integers(0, 4, rng.integers(1, 129), dtype=np.uint8)
        assert O.score_pair_rtl(q, t, sub, -12, -4, 12) == O.score_pair(q, t, sub, -12, -4)
    # identical 500-bp sequences score 2500 exactly; the 12-bit RTL cannot represent it
    q = rng.integers(0, 4, 500, dtype=np.uint8)
    assert O.score_pair(q, q, sub, -12, -4) == 2500
    assert O.score_pair_rtl(q, q, sub, -12, -4, 12) != 2500
    assert O.score_pair_rtl(q, q, sub, -12, -4, 16) == 2500


def test_column0_rule_matters_only_when_match_pays_for_open():
    """The PE's first column ignores its neighbours in I (SW_ProcessingElement_v1.0.v:131-141).
    With match + open + extend > 0 that is visible; the oracle must follow the RTL model."""
    rng = np.random.default_rng(5)
    sub = O.dna_matrix(20, -4)
    seen_diff = False
    for _ in range(200):
        q = rng.integers(0, 4, rng.integers(1, 30), dtype=np.uint8)
        t = rng.integers(0, 4, rng.integers(1, 30), dtype=np.uint8)
        a = O.score_pair(q, t, sub, -2, -1)
        assert a == O.score_pair_rtl(q, t, sub, -2, -1, 16)
        assert a == O.py_score_merged(list(q), list(t), sub, -2, -1, col0_rule=True)
        seen_diff |= a != O.py_score_merged(list(q), list(t), sub, -2, -1, col0_rule=False)
    assert seen_diff
    # at the reference parameters the rule is invisible
    sub = O.dna_matrix()
    for _ in range(100):
        q = rng.integers(0, 4, rng.integers(1, 40), dtype=np.uint8)
        t = rng.integers(0, 4, rng.integers(1, 40), dtype=np.uint8)
        assert O.score_pair(q, t, sub, -12, -4) == \
            O.py_score_merged(list(q), list(t), sub, -12, -4, col0_rule=False)


def test_blosum62_is_symmetric_and_known():
    B = O.BLOSUM62
    assert B.shape == (24, 24) and (B == B.T).all()
    diag = dict(zip(O.PROT_LETTERS, np.diag(B)))
    assert diag == {"A": 4, "R": 5, "N": 6, "D": 6, "C": 9, "Q": 5, "E": 5, "G": 6, "H": 8,
                    "I": 4, "L": 4, "K": 5, "M": 5, "F": 6, "P": 7, "S": 4, "T": 5, "W": 11,
                    "Y": 7, "V": 4, "B": 4, "Z": 4, "X": -1, "*": 1}
    idx = {c: i for i, c in enumerate(O.PROT_LETTERS)}
    assert B[idx["W"], idx["C"]] == -2 and B[idx["E"], idx["Z"]] == 4 and B[idx["I"], idx["V"]] == 3


def test_charto2bit_fixture():
    """Our 2-bit packing model vs the bytes the CAPI host printed for query1."""
    want = open(os.path.join(O.GOLDEN, "charto2bit_query1.hex")).read().split()
    q = O.read_fasta(O.golden_fasta("query1.fa"))[0][1]
    codes = O.encode_dna(q)
    packed = np.zeros((len(codes) + 3) // 4, np.uint8)
    for i, c in enumerate(codes):
        packed[i // 4] |= (int(c) & 3) << (2 * (i % 4))
    assert [f"{b:02x}" for b in packed] == want


def test_splitmix_workload_is_deterministic():
    a = O.random_codes(1234, 1000, 4)
    b = O.random_codes(1234, 1000, 4)
    assert (a == b).all() and a.max() == 3 and a.min() == 0
    counts = np.bincount(a, minlength=4)
    assert counts.min() > 200


def test_random_codes_windows():
    """The seeded code stream is counter-based: any window equals the slice of the whole
    stream (bench.py regenerates the rows it re-checks, e.g. a batch's last targets)."""
    whole = O.random_codes(4242, 5000, 20)
    for start, n in [(0, 10), (1, 7), (8, 64), (13, 1000), (4990, 10)]:
        assert (O.random_codes(4242, n, 20, start=start) == whole[start:start + n]).all()
