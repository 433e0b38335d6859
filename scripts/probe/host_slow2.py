"""Probe 2: bench.py's ragged host-API measurement under variations of what runs before it."""
import os, sys, time, json, subprocess
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
def run(args, env=None):
    e = dict(os.environ, **(env or {}))
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--workload", "ragged", "--cpu-seconds", "0"] + args, capture_output=True, text=True, env=e, timeout=250)
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    p = d["pcie_inclusive"]
    return [p["ms"], p["ms_best"], p["ms_iqr"]]
out = {}
out["default"] = run([])
out["steps1"] = run(["--steps", "1", "--warmup", "0"])
out["omp1"] = run([], {"OMP_NUM_THREADS": "1"})
out["threads16"] = run([], {"SWBANK_HOST_THREADS": "16"})
out["default2"] = run([])
print(json.dumps(out))
