#!/usr/bin/env python3
"""Generate golden vectors for shapes the reference's own fixtures do not cover, with the
oracle C restatement AFTER it has been pinned on every reference fixture
(tests/test_oracle_golden.py).  These pin the GPU path at the BASELINE configs[3]/[4] shapes
and at parameters where the merged (ScoreBank PE) and Gotoh (ssearch36) gap models differ.

    python tests/golden/make_generated.py      # writes tests/golden/generated.json

Sequences are stored as ASCII; the scores are the oracle's.  Protein entries are "parity
unpinned by the reference" (the reference has no protein mode); they pin our kernel to the
restated Gotoh/merged recurrence with BLOSUM62.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import oracle as O  # noqa: E402

DNA = "TCAG"  # code -> letter (ConvertToBase order T=0 C=1 A=2 G=3)


def dna_str(codes):
    return "".join(DNA[c] for c in codes)


def prot_str(codes):
    return "".join(O.PROT_LETTERS[c] for c in codes)


def mutate(rng, q, alpha, rate=0.1):
    """A homologous target: substitutions + short indels, so gapped alignments score high."""
    out = []
    for c in q:
        r = rng.random()
        if r < rate / 3:
            continue
        if r < 2 * rate / 3:
            out.append(int(rng.integers(0, alpha)))
        out.append(int(c) if r >= rate / 3 * 2 or r < rate / 3 else int(rng.integers(0, alpha)))
        if rng.random() < rate / 3:
            out.extend(int(x) for x in rng.integers(0, alpha, int(rng.integers(1, 4))))
    return np.array(out, dtype=np.uint8)


def case(name, alphabet, q, targets, sub, go, ge, model):
    res, offs, lens = O.pack_residues(targets)
    scores = O.score_batch(q, res, offs, lens, sub, go, ge, model)
    to_s = dna_str if alphabet == "dna" else prot_str
    return {"name": name, "alphabet": alphabet, "gap_model": "gotoh" if model else "merged",
            "gap_open": go, "gap_extend": ge,
            "match_mismatch": None if alphabet == "protein" else [int(sub[0, 0]), int(sub[0, 1])],
            "query": to_s(q), "targets": [to_s(t) for t in targets],
            "scores": [int(s) for s in scores]}


def main():
    rng = np.random.default_rng(20261015)
    cases = []
    # configs[3] shape: 150-bp reads vs 1-kbp targets (reads planted in a third of them)
    q = rng.integers(0, 4, 150, dtype=np.uint8)
    ts = []
    for k in range(48):
        t = rng.integers(0, 4, 1000, dtype=np.uint8)
        if k % 3 == 0:
            m = mutate(rng, q, 4)
            pos = int(rng.integers(0, 1000 - len(m)))
            t[pos:pos + len(m)] = m
        ts.append(t)
    cases.append(case("dna150x1000_merged", "dna", q, ts, O.dna_matrix(5, -4), -12, -4,
                      O.GAP_MERGED))
    cases.append(case("dna150x1000_gotoh_10_1", "dna", q, ts, O.dna_matrix(5, -4), -10, -1,
                      O.GAP_GOTOH))
    # merged != Gotoh parameters (2*ge > min substitution)
    q2 = rng.integers(0, 4, 100, dtype=np.uint8)
    ts2 = [mutate(rng, q2, 4, 0.25) for _ in range(64)]
    cases.append(case("dna100_merged_10_1", "dna", q2, ts2, O.dna_matrix(5, -4), -10, -1,
                      O.GAP_MERGED))
    cases.append(case("dna100_gotoh_10_1", "dna", q2, ts2, O.dna_matrix(5, -4), -10, -1,
                      O.GAP_GOTOH))
    # configs[4] shape: 512-aa protein query vs 1-kaa targets, BLOSUM62 -11/-1
    qp = rng.integers(0, 20, 512, dtype=np.uint8)
    tp = []
    for k in range(16):
        t = rng.integers(0, 20, 1000, dtype=np.uint8)
        if k % 2 == 0:
            m = mutate(rng, qp[100:400], 20, 0.3)
            t[200:200 + len(m)] = m
        tp.append(t)
    cases.append(case("prot512x1000_gotoh_11_1", "protein", qp, tp, O.BLOSUM62, -11, -1,
                      O.GAP_GOTOH))
    cases.append(case("prot512x1000_merged_11_1", "protein", qp, tp, O.BLOSUM62, -11, -1,
                      O.GAP_MERGED))
    out = os.path.join(HERE, "generated.json")
    json.dump({"generator": "tests/golden/make_generated.py (oracle/sw_oracle.c)",
               "cases": cases}, open(out, "w"))
    print(f"wrote {out}: " + ", ".join(f"{c['name']}({len(c['scores'])})" for c in cases))


if __name__ == "__main__":
    main()
