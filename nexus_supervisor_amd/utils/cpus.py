"""CPU share of this process: the affinity mask, capped by a cgroup-v2 CPU quota
(a Kubernetes CPU limit shows up as ``cpu.max``).  Sizes the process-per-core runtime
(``runtime.worker-processes: 0``) and the benchmark's shard-worker count."""
from __future__ import annotations

import os

CPU_MAX = "/sys/fs/cgroup/cpu.max"


def cpu_share(cpu_max_path: str = CPU_MAX) -> float:
    try:
        n = float(len(os.sched_getaffinity(0)))
    except (AttributeError, OSError):
        n = float(os.cpu_count() or 1)
    try:
        with open(cpu_max_path) as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            n = min(n, int(quota) / int(period))
    except (OSError, ValueError):
        pass
    return max(n, 1.0)


AUTO_WORKERS_CAP = 6


def auto_worker_processes(reserve: float = 1.0, cap: int = AUTO_WORKERS_CAP, share: float = 0.0) -> int:
    """Shard workers for the CPU share, keeping ``reserve`` CPUs for the coordinating
    parent (watch hub, lease, /metrics): at least 1 (= single-process supervisor), at most
    six — the efficiency knee measured on MI355X hosts in rounds 2-4 (``bench.py``
    ``auto_procs``, ``profiles/r4_sweep``): six saturated workers sustain 35-45k failures/s;
    past six the CPU per failure rises 20-40 % while the throughput stays within the
    run-to-run spread (more workers only lower burst latency; set
    ``runtime.worker-processes`` explicitly for that)."""
    n = share or cpu_share()
    return max(1, min(cap, int(n - reserve)))
