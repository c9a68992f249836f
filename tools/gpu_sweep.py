"""Bench configuration sweep on the GPU box (one process per config, sequential).

``python tools/gpu_sweep.py [--legacy] [extra bench args]``

``SWEEP="6:3,8:4,10:4"`` (procs:inflight pairs) overrides the default grid.
"""
import json
import os
import subprocess
import sys

CONFIGS = ([["--procs", str(p), "--inflight", str(i)] for p in (4, 6, 8) for i in (2, 3, 4)]
           + [["--procs", "6", "--inflight", "3", "--workers", "512"]])
if os.environ.get("SWEEP"):
    CONFIGS = [["--procs", p, "--inflight", i] for p, i in (c.split(":") for c in os.environ["SWEEP"].split(","))]
if len(sys.argv) > 1 and sys.argv[1] == "--legacy":
    CONFIGS = [["--transport", "inproc"], ["--inflight", "1"], ["--inflight", "2"], ["--inflight", "3"],
               ["--inflight", "4"], ["--inflight", "2", "--workers", "128"], ["--inflight", "2", "--workers", "512"],
               ["--inflight", "2", "--events", "2000"], ["--inflight", "2", "--kube-connections", "64"]]
    sys.argv.pop(1)
out = []
for extra in CONFIGS:
    steps = os.environ.get("SWEEP_STEPS", "6")
    cmd = [sys.executable, "bench.py", "--steps", steps, "--warmup", "1", "--no-real-oom"] + extra + sys.argv[1:]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    line = p.stdout.strip().splitlines()[-1] if p.stdout.strip() else ""
    try:
        d = json.loads(line)
        rec = {"args": extra, "value": d["value"], "p50_ms": d["p50_ms"], "p99_ms": d["p99_ms"], "errors": d["errors"],
               "cpu": d["config"].get("cpu_util_rank0")}
    except Exception:
        rec = {"args": extra, "error": p.stderr[-800:]}
    print(json.dumps(rec), flush=True)
    out.append(rec)
with open("gpurun_out/sweep.json", "w") as f:
    json.dump(out, f, indent=1)
