#!/usr/bin/env python3
"""Host-to-device copy rate from pinned memory: one stream vs the same bytes split over 2-4
streams (does a second copy engine raise the streamed feeder's PCIe ceiling?).
usage: python scripts/ubench/h2d_rate.py [MiB per chunk] [chunks]"""
import sys
import time

import torch

mb = int(sys.argv[1]) if len(sys.argv) > 1 else 8
nch = int(sys.argv[2]) if len(sys.argv) > 2 else 8
size = mb << 20
src = torch.empty(size * nch, dtype=torch.uint8).pin_memory()
src.fill_(1)
dst = torch.empty(size * nch, dtype=torch.uint8, device="cuda")
streams = [torch.cuda.Stream() for _ in range(4)]
for ns in (1, 2, 3, 4, 1, 2, 4):
    best = 1e9
    for rep in range(5):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        part = size // ns
        for c in range(nch):
            for k in range(ns):
                a = c * size + k * part
                b = c * size + (k + 1) * part if k + 1 < ns else (c + 1) * size
                with torch.cuda.stream(streams[k]):
                    dst[a:b].copy_(src[a:b], non_blocking=True)
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    print(f"streams={ns} chunk={mb} MiB x {nch}: {size * nch / best / 1e9:.1f} GB/s "
          f"({best * 1e3:.2f} ms)", flush=True)
