"""Probe: why bench.py's host-API median (ragged) is slower than scripts/host_api_bench.py's on
the same box.  Times sw_score_batch on the bench's ragged batch in several process / bank
states (median of 9 calls each)."""
import os, sys, time, json
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "smith-waterman-fpga-module_amd")]
import swbank as S
from bench import ragged_batch, load_query
import torch

def med(bank, res, offs, lens, k=9):
    out = np.empty(len(lens), np.int32)
    bank.score_batch(res, offs, lens, out=out)
    bank.score_batch(res, offs, lens, out=out)
    ts = []
    for _ in range(k):
        t0 = time.perf_counter(); bank.score_batch(res, offs, lens, out=out); ts.append(time.perf_counter() - t0)
    return round(float(np.median(ts)) * 1e3, 3), round(min(ts) * 1e3, 3)

n = 499 * 2048
res, offs, lens = ragged_batch(1000, n)
q = load_query()
r = {}
b1 = S.ScoreBank(device=0); b1.set_penalties(5, -4, -12, -4); b1.load_query(q)
r["fresh_bank_no_torch_cuda"] = med(b1, res, offs, lens)
dev = torch.device("cuda", 0)
d = [torch.from_numpy(x).to(dev) for x in (res, offs.view(np.int64), lens.view(np.int32))]
sc = torch.empty(n, dtype=torch.int32, device=dev)
st = torch.cuda.Stream()
for _ in range(20):
    b1.score_batch_device(d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), n, 150, sc.data_ptr(), st.cuda_stream, min_len=64)
torch.cuda.synchronize()
r["same_bank_after_device_calls"] = med(b1, res, offs, lens)
b2 = S.ScoreBank(device=0); b2.set_penalties(5, -4, -12, -4); b2.load_query(q)
r["second_bank"] = med(b2, res, offs, lens)
r["first_bank_again"] = med(b1, res, offs, lens)
res2 = res.copy(); offs2 = offs.copy(); lens2 = lens.copy()
r["first_bank_copied_arrays"] = med(b1, res2, offs2, lens2)
b1.set_timing(True); b1.timing()
r["first_bank_timing_on"] = med(b1, res, offs, lens)
b1.set_timing(False)
print(json.dumps(r), flush=True)
