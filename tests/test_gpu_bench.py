"""GPU: bench.py's own flows, end to end, as the driver runs them.

* N = 2 ranks under ``torch.distributed.run`` on the box's one GPU (SWBENCH_SHARE_GPU=1 puts both
  ranks on device 0; SWBENCH_BACKEND=gloo because RCCL refuses two ranks on one device): one
  JSON line with n_gpus 2, and rank 0's parity check covers the slice it GATHERED from rank 1
  (regenerated from rank 1's seed and re-scored by the oracle).
* the ragged and literal-data500 workloads at reduced size (parity sample 0 mismatches).
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _json_line(out):
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out[-2000:]
    return json.loads(lines[0])


@pytest.mark.parametrize("workload,steps,extra", [("q100xdata500", 3, {}), ("ragged", 3, {}),
                                                  ("q100xdata500", 1, {"SWBANK_F16": "0"})])
def test_bench_two_ranks_gathered_parity(workload, steps, extra):
    """Two ranks on the box's GPU (gloo): rank 0's gathered slices are bit-exact.  The u16 case
    with one timed step is the one whose slices were stale while bench.py scored on torch's
    default stream (handle 0 = the bank's own stream, so the gather's copy did not wait)."""
    env = dict(os.environ, SWBENCH_BACKEND="gloo", SWBENCH_SHARE_GPU="1",
               MASTER_ADDR="127.0.0.1", **extra)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", str(steps), "--warmup", "1",
           "--reps", "64", "--cpu-seconds", "0", "--workload", workload]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["scaling"] == "weak"
    assert d["dist"]["world_size"] == 2 and len(d["dist"]["devices"]) == 2
    ps = d["parity_sample"]
    assert ps["ranks"] == 2 and ps["mismatches"] == 0 and ps["targets"] >= 2 * 256, ps


def test_bench_gpus_flag_starts_the_ranks():
    """`python bench.py --gpus 2` with NO launcher (how the driver runs the N=1 leg): bench.py
    starts the two ranks itself, and the line proves it -- n_gpus 2, the process group's world
    size 2, both ranks' devices listed, rank 1's gathered slice bit-exact."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(SWBENCH_BACKEND="gloo", SWBENCH_SHARE_GPU="1")
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "2",
           "--warmup", "1", "--reps", "64", "--cpu-seconds", "0"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    assert d["n_gpus"] == 2, d
    assert d["dist"]["world_size"] == 2 and d["dist"]["backend"] == "gloo"
    assert len(d["dist"]["devices"]) == 2 and all(x["pci"] for x in d["dist"]["devices"])
    assert d["dist"]["distinct_gpus"] == 1  # both ranks share the box's one GPU here
    ps = d["parity_sample"]
    assert ps["ranks"] == 2 and ps["mismatches"] == 0, ps


@pytest.mark.parametrize("workload", ["ragged", "data500", "reads150x1k", "protein512x1k"])
def test_bench_workloads_one_gpu(workload):
    """Every bench workload the driver does not run itself, at reduced size: configs[3] (the
    query-set path, 4 x 1-kbp queries) and configs[4] (protein, the wave kernel with its segmented
    tail: 4,300 targets = 2,150 pairs, 102 past two pairs per SIMD)."""
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--steps", "2", "--warmup", "1",
           "--reps", "64", "--reads", "8192", "--slice", "4", "--ptargets", "4300",
           "--cpu-seconds", "0", "--workload", workload]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    assert d["n_gpus"] == 1 and d["parity_sample"]["mismatches"] == 0
    assert d["parity_sample"]["targets"] > 0
    if workload != "reads150x1k":  # (one query: the host API runs beside it)
        assert d["pcie_inclusive"]["matches_device_api"] is True
    assert 0 < d["roofline"]["frac"] <= 1.0
    if workload == "reads150x1k":
        assert "queries=4" in d["kernel"], d["kernel"]
    if workload == "protein512x1k":
        assert d["kernel"].startswith("wave") and "tail=102/8" in d["kernel"], d["kernel"]
