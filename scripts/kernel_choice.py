#!/usr/bin/env python3
"""Measure tile vs wave kernel GCUPS over (query length, target length, gap model, alphabet)
to calibrate the host's kernel choice (csrc/swbank_launch.hip, launch()).  One process,
interleaved, device buffers resident; prints one JSON line per case.
usage: python scripts/kernel_choice.py [--cells 2e10]"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "smith-waterman-fpga-module_amd"))
sys.path.insert(0, REPO)

CASES = [  # (alphabet, model, qlen, L, ntargets)
    ("dna", "gotoh", 128, 128, 262144), ("dna", "gotoh", 256, 256, 131072),
    ("dna", "merged", 256, 256, 131072), ("dna", "merged", 512, 512, 65536),
    ("dna", "merged", 1000, 150, 65536), ("dna", "gotoh", 512, 512, 65536),
    ("protein", "gotoh", 128, 300, 131072), ("protein", "gotoh", 256, 300, 65536),
    ("protein", "merged", 512, 1000, 25000), ("protein", "gotoh", 1024, 1000, 12500),
    ("protein", "gotoh", 128, 150, 524288), ("protein", "merged", 128, 150, 524288),
    ("dna", "gotoh", 256, 150, 524288),
    ("dna", "merged", 4000, 1000, 2000), ("protein", "gotoh", 3000, 500, 5000),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--kernels", default="tile,tile-u16,wave,wave-u16,auto",
                    help="comma list; -lut: SWBANK_PAIR=0 (row LUT instead of the pair table)")
    ap.add_argument("--only", default="", help="alphabet:model filter, e.g. dna:gotoh")
    ap.add_argument("--repeat", type=int, default=1,
                    help="rounds over the kernel list (interleaved); the best rate is kept")
    args = ap.parse_args()
    import torch

    import swbank as S
    from oracle import oracle as O

    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream().cuda_stream
    for alpha, model, qlen, L, n in CASES:
        if args.only and args.only != f"{alpha}:{model}":
            continue
        A = 4 if alpha == "dna" else 20
        q = O.random_codes(5 + qlen, qlen, A)
        tg = O.random_codes(9 + L, n * L, A)
        d_res = torch.from_numpy(tg).to(dev)
        d_offs = torch.arange(n, dtype=torch.int64, device=dev) * L
        d_lens = torch.full((n,), L, dtype=torch.int32, device=dev)
        d_sc = torch.zeros(n, dtype=torch.int32, device=dev)
        bank = S.ScoreBank(device=0, alphabet=S.ALPHABET_DNA if alpha == "dna" else
                           S.ALPHABET_PROTEIN, gap_model=S.GAP_MERGED if model == "merged"
                           else S.GAP_GOTOH)
        if alpha == "dna":
            bank.set_penalties(5, -4, -10, -1)
        else:
            bank.set_matrix(O.BLOSUM62, -11, -1)
        bank.load_query(q)
        out = {"alphabet": alpha, "model": model, "qlen": qlen, "L": L, "n": n}
        ref = None
        for kern in args.kernels.split(",") * args.repeat:
            os.environ["SWBANK_KERNEL"] = kern.split("-")[0]
            os.environ["SWBANK_F16"] = "0" if kern.endswith("-u16") else "1"
            os.environ["SWBANK_PAIR"] = "0" if kern.endswith("-lut") else "1"
            bank.score_batch_device(d_res.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(), n, L,
                                    d_sc.data_ptr(), stream)
            torch.cuda.synchronize()
            sc = d_sc.cpu().numpy().copy()
            if ref is None:
                ref = sc
            assert (sc == ref).all(), (kern, "differs")
            bank.timing()
            bank.set_timing(True)
            for _ in range(args.iters):
                bank.score_batch_device(d_res.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(),
                                        n, L, d_sc.data_ptr(), stream)
            launches, _, ms = bank.timing()
            bank.set_timing(False)
            out[kern] = max(out.get(kern, 0.0), round(qlen * L * n * launches / (ms / 1e3) / 1e9, 1))
            out[kern + "_kernel"] = bank.last_kernel()
        os.environ.pop("SWBANK_KERNEL")
        os.environ.pop("SWBANK_F16")
        os.environ.pop("SWBANK_PAIR")
        bank.close()
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
