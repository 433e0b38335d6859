"""Probe 3: bisect bench.py's ragged host-API slowdown through its own set-up steps."""
import os, sys, time, json
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "smith-waterman-fpga-module_amd")]
import bench
args = bench.parse.__wrapped__() if hasattr(bench.parse, "__wrapped__") else None
import argparse
sys.argv = ["bench.py", "--workload", "ragged", "--cpu-seconds", "0"]
args = bench.parse()
import torch
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
import swbank as S
def med(wl, k=9):
    out = np.empty(wl.n, np.int32)
    wl.bank.score_batch(wl.res, wl.offs, wl.lens, out=out)
    wl.bank.score_batch(wl.res, wl.offs, wl.lens, out=out)
    ts = []
    for _ in range(k):
        t0 = time.perf_counter(); wl.bank.score_batch(wl.res, wl.offs, wl.lens, out=out); ts.append(time.perf_counter() - t0)
    return round(float(np.median(ts)) * 1e3, 3)
r = {}
wl = bench.Workload(args, 0, dev, S, torch)
r["after_workload"] = med(wl)
stream = torch.cuda.Stream(device=dev)
stream.wait_stream(torch.cuda.current_stream())
torch.cuda.set_stream(stream)
r["after_set_stream"] = med(wl)
from swbank.dist import StepGather
sg = StepGather(wl.d_sc, dst=0, stage_cpu=False)
r["after_stepgather"] = med(wl)
for _ in range(3):
    wl.run(stream.cuda_stream, sg.buffer()); sg.submit()
sg.drain(); torch.cuda.synchronize()
r["after_warmup"] = med(wl)
wl.bank.timing(); wl.bank.set_timing(True)
for _ in range(20):
    wl.run(stream.cuda_stream, sg.buffer()); sg.submit()
sg.drain(); torch.cuda.synchronize()
wl.bank.set_timing(False); wl.bank.timing()
r["after_steps"] = med(wl)
torch.cuda.set_stream(torch.cuda.default_stream())
r["default_stream_again"] = med(wl)
print(json.dumps(r), flush=True)
