"""CPU cost per pod-failure event of the supervisor and cluster processes (wire mode).

Wall-clock throughput in a syscall-heavy sandbox says little; CPU-µs per event does.
"""
import asyncio
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nexus_supervisor_amd.bench import wire as W  # noqa: E402
from nexus_supervisor_amd.bench.runner import BenchConfig, run_rank  # noqa: E402


def cpu_of(pid):
    with open(f"/proc/{pid}/stat") as f:
        parts = f.read().rsplit(")", 1)[1].split()
    return (int(parts[11]) + int(parts[12])) / os.sysconf("SC_CLK_TCK")


marks = {}
orig = W.WireHarness.step


async def step(self, events):
    key = "0" if "t0" not in marks else "1"
    marks["t" + key] = time.monotonic()
    marks["c" + key] = time.process_time()
    marks["p" + key] = cpu_of(self.proc.pid)
    marks["q" + key] = cpu_of(self.cql.proc.pid)
    marks["n"] = marks.get("n", 0) + 1
    return await orig(self, events)

W.WireHarness.step = step
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 6
cfg = BenchConfig(steps=steps, warmup=1, transport="wire", workdir="/tmp", inflight=1)
r = asyncio.run(run_rank(cfg, lambda: None))
n_ev = (marks["n"] - 1 - 1) * cfg.events  # events between the first timed mark and the last mark
us = lambda a, b: 1e6 * (marks[b] - marks[a]) / n_ev
print(f"eps={r['events'] / r['elapsed']:.0f} supervisor={us('c0', 'c1'):.0f}us/ev cluster={us('p0', 'p1'):.0f}us/ev "
      f"cqlsrv={us('q0', 'q1'):.0f}us/ev")
