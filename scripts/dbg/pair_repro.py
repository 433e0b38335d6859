"""Debug: feeder vs device API vs oracle on the bad-code feeder case, pair on/off."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "smith-waterman-fpga-module_amd"))
import numpy as np
import torch
import swbank as S
from oracle import oracle as O

REF = (5, -4, -12, -4)
rng = np.random.default_rng(13)
n = 30000
lens = rng.integers(50, 151, n).astype(np.uint32)
offs = np.zeros(n, np.uint64); offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
res = rng.integers(0, 4, int(lens.sum()), dtype=np.uint8)
q = rng.integers(0, 4, 64, dtype=np.uint8)
sub = [res[int(offs[k]):int(offs[k]) + int(lens[k])] for k in range(n)]
want = O.score_batch(q, *S.pack_targets(sub), O.dna_matrix(*REF[:2]), *REF[2:])

def dev_scores(bank):
    dev = torch.device("cuda", 0)
    d_res = torch.from_numpy(res).to(dev)
    d_offs = torch.from_numpy(offs.astype(np.int64)).to(dev)
    d_lens = torch.from_numpy(lens.astype(np.int32)).to(dev)
    d_sc = torch.zeros(n, dtype=torch.int32, device=dev)
    bank.score_batch_device(d_res.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(), n,
                            int(lens.max()), d_sc.data_ptr(), 0)
    torch.cuda.synchronize()
    return d_sc.cpu().numpy()

# chunk boundaries of the feeder at SWBANK_CHUNK_MB=1
target = 1 << 20
bounds = []; c0 = 0; acc = 0
for k in range(n):
    acc += int(lens[k])
    if acc >= target or k + 1 == n:
        bounds.append((c0, k + 1)); c0 = k + 1; acc = 0
print("chunks", bounds, flush=True)
os.environ["SWBANK_KERNEL"] = "tile"
for pair in ("1", "0"):
    os.environ["SWBANK_PAIR"] = pair
    with S.ScoreBank() as bank:
        bank.set_penalties(*REF)
        bank.load_query(q)
        for (a, b) in bounds:
            idx = np.arange(a, b)
            for order in ("input", "sorted"):
                sel = idx if order == "input" else idx[np.argsort(-lens[a:b].astype(np.int64), kind="stable")]
                sub2 = [sub[k] for k in sel]
                r2, o2, l2 = S.pack_targets(sub2)
                dev = torch.device("cuda", 0)
                d_res = torch.from_numpy(r2).to(dev)
                d_offs = torch.from_numpy(o2.astype(np.int64)).to(dev)
                d_lens = torch.from_numpy(l2.astype(np.int32)).to(dev)
                d_sc = torch.zeros(len(sel), dtype=torch.int32, device=dev)
                bank.score_batch_device(d_res.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(), len(sel),
                                        int(l2.max()), d_sc.data_ptr(), 0)
                torch.cuda.synchronize()
                d = d_sc.cpu().numpy()
                bad = np.nonzero(d != want[sel])[0]
                print(f"pair={pair} chunk=({a},{b}) n={b-a} {order} [{bank.last_kernel()}] bad={len(bad)} pos={bad[:8].tolist()} tiles={sorted(set((bad//128).tolist()))[:5]} lanes={sorted(set((bad%128).tolist()))[:12]}", flush=True)
