"""GPU parity for long queries: past 512 rows the query runs as segments of SWBANK_SEG rows
whose bottom rows are handed on through HBM (LDS-DMA in, plain stores out)."""
import json
import os

import numpy as np
import pytest

import swbank as S
from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, params=["tile", "tile-u16", "wave", "wave-u16"])
def kernel_choice(request, monkeypatch):
    """Run every parity test through each score kernel: the tile kernel (waves = row blocks,
    lanes = targets) and the wave kernel (lanes = rows, DPP hand-off), each with its f16
    arithmetic where eligible ("tile", "wave": exact below the f16 bound, optimistic with a
    u16 re-score above it) and forced to u16 ("-u16").  Past 1024 rows the wave kernel runs
    the query as 1024-row segments."""
    kern = request.param.split("-")[0]
    monkeypatch.setenv("SWBANK_KERNEL", kern)
    monkeypatch.setenv("SWBANK_F16", "0" if request.param.endswith("-u16") else "1")
    return request.param


def _random_case(rng, qlen, ntargets, maxlen, p_n=0.02):
    q = rng.integers(0, 4, qlen, dtype=np.uint8)
    q[rng.random(qlen) < p_n] = 4
    seqs = []
    for _ in range(ntargets):
        t = rng.integers(0, 4, int(rng.integers(0, maxlen + 1)), dtype=np.uint8)
        t[rng.random(len(t)) < p_n] = 4
        seqs.append(t)
    return q, seqs


@pytest.mark.parametrize("model", [S.GAP_MERGED, S.GAP_GOTOH])
@pytest.mark.parametrize("qlen", [513, 700, 1000, 2048])
def test_long_query_dna_vs_oracle(model, qlen):
    rng = np.random.default_rng(qlen + model)
    q, seqs = _random_case(rng, qlen, 140, 400)
    for k in range(0, 140, 5):
        a = int(rng.integers(0, qlen - 300))
        seqs[k] = q[a:a + int(rng.integers(50, 300))].copy()
        seqs[k][::9] = rng.integers(0, 4, len(seqs[k][::9]))
    with S.ScoreBank(gap_model=model) as bank:
        bank.set_penalties(5, -4, -10, -1)
        bank.load_query(q)
        got = bank.score_targets(seqs)
    res, offs, lens = O.pack_residues(seqs)
    want = O.score_batch(q, res, offs, lens, O.dna_matrix(), -10, -1, model)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(int(i), int(lens[i]), int(got[i]), int(want[i])) for i in bad[:8]]


@pytest.mark.parametrize("seg", ["64", "128", "512"])
def test_long_query_segment_sizes_agree(seg, monkeypatch):
    rng = np.random.default_rng(3)
    q, seqs = _random_case(rng, 900, 200, 200)
    monkeypatch.setenv("SWBANK_SEG", seg)
    with S.ScoreBank() as bank:
        bank.set_penalties(5, -4, -12, -4)
        bank.load_query(q)
        got = bank.score_targets(seqs)
    res, offs, lens = O.pack_residues(seqs)
    assert (got == O.score_batch(q, res, offs, lens, O.dna_matrix(), -12, -4)).all()


def test_long_query_protein_col0_rule():
    """merged model, BLOSUM62 with -2/-1: max(s)=11 > o+e, so the HDL column-0 rule is live in
    every segment."""
    rng = np.random.default_rng(12)
    q = rng.integers(0, 20, 800, dtype=np.uint8)
    seqs = [rng.integers(0, 20, int(rng.integers(1, 300)), dtype=np.uint8) for _ in range(130)]
    with S.ScoreBank(alphabet=S.ALPHABET_PROTEIN) as bank:
        bank.set_matrix(O.BLOSUM62, -2, -1)
        bank.load_query(q)
        got = bank.score_targets(seqs)
    res, offs, lens = O.pack_residues(seqs)
    assert (got == O.score_batch(q, res, offs, lens, O.BLOSUM62, -2, -1)).all()


def test_generated_golden_swapped_orientation():
    """configs[3] orientation the bench uses: the 1-kbp target as the bank query, the 150-bp
    read as the batch.  Both gap models are symmetric under transposition at these parameters
    (no column-0 rule in play), so the fixture scores must come back unchanged."""
    cases = {c["name"]: c for c in
             json.load(open(os.path.join(O.GOLDEN, "generated.json")))["cases"]}
    for name, model in (("dna150x1000_merged", S.GAP_MERGED),
                        ("dna150x1000_gotoh_10_1", S.GAP_GOTOH)):
        c = cases[name]
        with S.ScoreBank(gap_model=model) as bank:
            bank.set_penalties(*c["match_mismatch"], c["gap_open"], c["gap_extend"])
            for t, want in zip(c["targets"][:12], c["scores"][:12]):
                bank.load_query(S.encode(t))
                assert bank.score_targets([S.encode(c["query"])]).tolist() == [want]


@pytest.mark.parametrize("alphabet", ["dna", "protein"])
@pytest.mark.parametrize("model", [S.GAP_MERGED, S.GAP_GOTOH])
def test_optimistic_f16_rescore(alphabet, model, kernel_choice):
    """Past the exact f16 bound the tile kernel scores every pair in f16 and re-scores, in
    u16, only the pairs whose f16 score exceeds 2048 - max(s) (the only ones a rounded value
    can have touched).  Half the targets here are near-copies scoring far above 2048, half
    are random; long queries run as several segments in both passes."""
    rng = np.random.default_rng(11 + model + (alphabet == "dna"))
    A = 4 if alphabet == "dna" else 20
    qlen = 1200 if alphabet == "dna" else 700
    q = rng.integers(0, A, qlen, dtype=np.uint8)
    seqs = []
    for k in range(260):
        if k % 2:
            seqs.append(rng.integers(0, A, int(rng.integers(0, 900)), dtype=np.uint8))
        else:
            a = int(rng.integers(0, qlen // 3))
            t = q[a:a + int(rng.integers(300, 900))].copy()
            t[::13] = rng.integers(0, A, len(t[::13]))
            seqs.append(t)
    with S.ScoreBank(alphabet=S.ALPHABET_DNA if alphabet == "dna" else S.ALPHABET_PROTEIN,
                     gap_model=model) as bank:
        if alphabet == "dna":
            bank.set_penalties(5, -4, -10, -1)
            sub, go, ge = O.dna_matrix(5, -4), -10, -1
        else:
            bank.set_matrix(O.BLOSUM62, -11, -1)
            sub, go, ge = O.BLOSUM62, -11, -1
        bank.load_query(q)
        got = bank.score_targets(seqs)
        kern = bank.last_kernel()
    res, offs, lens = O.pack_residues(seqs)
    want = O.score_batch(q, res, offs, lens, sub, go, ge, model)
    assert want.max() > 2048 and (want < 2000).sum() > 100
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, (kern, [(int(i), int(got[i]), int(want[i])) for i in bad[:8]])
    if kernel_choice == "tile":
        assert kern.startswith("tile f16+u16-rescore"), kern
    elif kernel_choice == "wave":  # past 1024 rows the wave kernel runs 1024-row segments
        assert kern.startswith("wave f16+u16-rescore"), kern
        assert kern.endswith(f"segs={(qlen + 1023) // 1024}"), kern


def test_segmented_batch_in_position_ranges(monkeypatch):
    """A small SWBANK_EDGE_MB splits a segmented batch into position ranges (each with its own
    HBM edge rows), in both the f16 pass and the optimistic u16 re-score."""
    monkeypatch.setenv("SWBANK_EDGE_MB", "1")
    rng = np.random.default_rng(5)
    q = rng.integers(0, 4, 1100, dtype=np.uint8)
    seqs = []
    for k in range(600):
        if k % 3 == 0:
            a = int(rng.integers(0, 400))
            seqs.append(q[a:a + int(rng.integers(400, 700))].copy())
        else:
            seqs.append(rng.integers(0, 4, int(rng.integers(0, 700)), dtype=np.uint8))
    with S.ScoreBank() as bank:
        bank.set_penalties(5, -4, -10, -1)
        bank.load_query(q)
        got = bank.score_targets(seqs)
    res, offs, lens = O.pack_residues(seqs)
    want = O.score_batch(q, res, offs, lens, O.dna_matrix(), -10, -1)
    assert want.max() > 2048
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(int(i), int(got[i]), int(want[i])) for i in bad[:8]]
