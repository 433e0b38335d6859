#!/usr/bin/env python3
"""Phase trace of one host-API call (SWBANK_TRACE_FILE) on the headline host shape, for the
streamed and the chunked feeder: gather / copy publication / kernel marks in microseconds."""
import os
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "smith-waterman-fpga-module_amd"))
sys.path.insert(0, REPO)


def main():
    import swbank as S
    from oracle import oracle as O
    n, L = 1021952, 128
    q = O.random_codes(1, 128, 4)
    if "--ragged" in sys.argv:  # lengths 64-128, 0.1 % N
        rng = np.random.default_rng(7)
        lens = rng.integers(L // 2, L + 1, n).astype(np.uint32)
        offs = np.zeros(n, np.uint64)
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
        res = O.random_codes(2, int(lens.sum()), 4)
        res[rng.random(res.size) < 0.001] = 4
    else:
        res = O.random_codes(2, n * L, 4)
        offs = np.arange(n, dtype=np.uint64) * L
        lens = np.full(n, L, np.uint32)
    for mode in ("1", "0", "1"):
        os.environ["SWBANK_STREAM"] = mode
        path = tempfile.mktemp()
        with S.ScoreBank() as bank:
            bank.set_penalties(5, -4, -12, -4)
            bank.load_query(q)
            for _ in range(4):
                bank.score_batch(res, offs, lens)
            os.environ["SWBANK_TRACE_FILE"] = path
            bank.score_batch(res, offs, lens)
            del os.environ["SWBANK_TRACE_FILE"]
            print(f"== SWBANK_STREAM={mode}: {bank.last_kernel()}")
        lines = [l.split() for l in open(path).read().split("--")[0].strip().splitlines()]
        print(" ".join(f"{w}@{float(t):.0f}" for w, t in lines))
        os.unlink(path)


if __name__ == "__main__":
    main()
