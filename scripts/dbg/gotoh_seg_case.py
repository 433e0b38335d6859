#!/usr/bin/env python3
"""Repro: tests/test_gpu_long.py::test_long_query_dna_vs_oracle[tile-700-1] under several
knobs (pair table on/off, segment size, f16/u16); prints the mismatches of each."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "smith-waterman-fpga-module_amd"))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import swbank as S  # noqa: E402
from oracle import oracle as O  # noqa: E402
from test_gpu_long import _random_case  # noqa: E402

import torch  # noqa: E402

# stale device memory, as a long test session leaves it: the banks below reuse these pages
junk = torch.full((1 << 28,), 0x3C003C00, dtype=torch.int32, device="cuda")
del junk
torch.cuda.empty_cache()
for qlen, model in ((700, 1), (700, 0), (600, 1), (1000, 1)):
    rng = np.random.default_rng(qlen + model)
    q, seqs = _random_case(rng, qlen, 140, 400)
    for k in range(0, 140, 5):
        a = int(rng.integers(0, qlen - 300))
        seqs[k] = q[a:a + int(rng.integers(50, 300))].copy()
        seqs[k][::9] = rng.integers(0, 4, len(seqs[k][::9]))
    res, offs, lens = O.pack_residues(seqs)
    want = O.score_batch(q, res, offs, lens, O.dna_matrix(), -10, -1, model)
    for env in ({}, {"SWBANK_PAIR": "0"}, {"SWBANK_SEG": "256"}, {"SWBANK_F16": "0"},
                {"SWBANK_DSORT": "0"}, {"SWBANK_SEG": "256", "SWBANK_PAIR": "0"}):
        os.environ["SWBANK_KERNEL"] = "tile"
        for k in ("SWBANK_PAIR", "SWBANK_SEG", "SWBANK_F16", "SWBANK_DSORT"):
            os.environ.pop(k, None)
        os.environ.update(env)
        with S.ScoreBank(gap_model=model) as bank:
            bank.set_penalties(5, -4, -10, -1)
            bank.load_query(q)
            got = bank.score_targets(seqs)
            kern = bank.last_kernel()
        bad = np.nonzero(got != want)[0]
        print(qlen, model, env, kern, len(bad),
              [(int(i), int(lens[i]), int(got[i]), int(want[i])) for i in bad[:6]], flush=True)
