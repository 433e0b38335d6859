"""Seeded fuzz: random alphabets, matrices, gap penalties, gap models, query and target
lengths (incl. empty, 1, segment and f16-bound edges), homologous and random targets —
every case bit-exact against the oracle, through tile/wave x f16/u16 (the autouse fixture)."""
import os

import numpy as np
import pytest

import swbank as S
from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, params=["tile", "tile-u16", "wave", "wave-u16", "wave-split",
                                      "wave-split-u16"])
def kernel_choice(request, monkeypatch):
    """-split: every pair through the wave kernel's split tail (queries of 257-1024 rows; the
    segment count P = 2 or 4 drawn from the case seed in the test)"""
    monkeypatch.setenv("SWBANK_KERNEL", request.param.split("-")[0])
    monkeypatch.setenv("SWBANK_F16", "0" if request.param.endswith("-u16") else "1")
    if "-split" in request.param:
        monkeypatch.setenv("SWBANK_WAVE_SPLIT", "1000000")
    return request.param


def _case(seed):
    rng = np.random.default_rng(seed)
    dna = rng.random() < 0.6
    A = S.DNA_ALPHA if dna else S.PROTEIN_ALPHA
    letters = 4 if dna else 20
    if dna and rng.random() < 0.6:
        ma, mm = int(rng.integers(1, 13)), int(rng.integers(-10, 1))
        sub = O.dna_matrix(ma, mm)
        pen = ("pen", ma, mm)
    elif dna:
        m = rng.integers(-9, 12, (A, A)).astype(np.int8)
        m = np.triu(m) + np.triu(m, 1).T
        m[:, 4] = m[4, :] = int(rng.integers(-6, 1))
        sub, pen = m, ("matrix",)
    elif rng.random() < 0.5:
        sub, pen = O.BLOSUM62, ("matrix",)
    else:
        m = rng.integers(-8, 13, (A, A)).astype(np.int8)
        sub, pen = np.triu(m) + np.triu(m, 1).T, ("matrix",)
    go, ge = -int(rng.integers(1, 21)), -int(rng.integers(1, 6))
    model = S.GAP_GOTOH if rng.random() < 0.5 else S.GAP_MERGED
    qlen = int(rng.choice([1, 2, 15, 16, 17, 63, 100, 255, 256, 257, 400, 513, 700, 1100]))
    q = rng.integers(0, letters, qlen, dtype=np.uint8)
    n = int(rng.integers(1, 300))
    maxlen = int(rng.choice([1, 8, 9, 150, 600, 1200]))
    seqs = []
    for k in range(n):
        if k % 4 == 0 and qlen > 1:
            a = int(rng.integers(0, qlen))
            t = q[a:a + int(rng.integers(1, maxlen + 1))].copy()
            t[::7] = rng.integers(0, letters, len(t[::7]))
        else:
            t = rng.integers(0, letters, int(rng.integers(0, maxlen + 1)), dtype=np.uint8)
        if dna and len(t) and rng.random() < 0.2:
            t[rng.random(len(t)) < 0.05] = 4  # N
        seqs.append(t)
    return dna, A, sub, pen, go, ge, model, q, seqs


#  SWBANK_FUZZ_SEEDS=n (default 150) / SWBANK_FUZZ_BASE=b: seeds b .. b+n-1 (long soak runs)
_BASE = int(os.environ.get("SWBANK_FUZZ_BASE", "0"))
_SEEDS = int(os.environ.get("SWBANK_FUZZ_SEEDS", "150"))


@pytest.mark.parametrize("seed", range(_BASE, _BASE + _SEEDS))
def test_fuzz_vs_oracle(seed, kernel_choice, monkeypatch):
    if "-split" in kernel_choice:
        monkeypatch.setenv("SWBANK_WAVE_SPLIT_P", "2" if seed % 2 else "4")
    dna, A, sub, pen, go, ge, model, q, seqs = _case(seed)
    with S.ScoreBank(alphabet=S.ALPHABET_DNA if dna else S.ALPHABET_PROTEIN,
                     gap_model=model) as bank:
        if pen[0] == "pen":
            bank.set_penalties(pen[1], pen[2], go, ge)
        else:
            bank.set_matrix(sub, go, ge)
        bank.load_query(q)
        try:
            got = bank.score_targets(seqs)
        except S.SwbankError as e:  # only a 16-bit range refusal is acceptable
            assert e.status == S.ERR_RANGE, e
            return
        kern = bank.last_kernel()
    res, offs, lens = O.pack_residues(seqs)
    want = O.score_batch(q, res, offs, lens, sub.astype(np.int8), go, ge, model)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, (kern, [(int(i), int(lens[i]), int(got[i]), int(want[i]))
                                  for i in bad[:6]])
