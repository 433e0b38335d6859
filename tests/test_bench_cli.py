"""CPU: bench.py's rank-count contract, checked before any GPU call.

`--gpus N` under a launcher must equal the launcher's WORLD_SIZE (a line printed with the wrong
n_gpus would void a scaling run); the check runs before torch touches a device, so it is
testable here.
"""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def _run(args, **env):
    e = dict(os.environ, **env)
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args,
                          capture_output=True, text=True, timeout=120, env=e, cwd=REPO)


def test_gpus_mismatch_with_launcher_exits_nonzero():
    r = _run(["--gpus", "1", "--steps", "1"], WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    assert r.returncode == 2, (r.returncode, r.stderr[-1000:])
    assert "WORLD_SIZE=2" in r.stderr
    r = _run(["--gpus", "8", "--steps", "1"], WORLD_SIZE="4", RANK="0", LOCAL_RANK="0")
    assert r.returncode == 2 and "--gpus 8" in r.stderr


def test_resolve_world_rules():
    import argparse
    import bench
    old = os.environ.pop("WORLD_SIZE", None)
    try:
        assert bench.resolve_world(argparse.Namespace(gpus=None)) == 1
        assert bench.resolve_world(argparse.Namespace(gpus=1)) == 1
        os.environ["WORLD_SIZE"] = "4"
        assert bench.resolve_world(argparse.Namespace(gpus=None)) == 4
        assert bench.resolve_world(argparse.Namespace(gpus=4)) == 4
    finally:
        os.environ.pop("WORLD_SIZE", None)
        if old is not None:
            os.environ["WORLD_SIZE"] = old
