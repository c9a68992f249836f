"""CPU placement of the supervisor's processes on a GPU node.

An MI355X host is a two-socket machine (the pool's: 2 × EPYC 9575F, 64 cores and 128
hardware threads per NUMA node).  The replica is a group of processes that talk over
pipes and sockets all the time: the watch hub parent, its shard workers, and the store
and API connections.  Left to the scheduler, they spread over both sockets and share
physical cores with each other and with other tenants.  Each message that crosses the
socket boundary then moves its cache lines over the inter-socket link, and an SMT
sibling halves a core's throughput.

:func:`plan` picks one NUMA node (the GPU's, or node 0), and within it one hardware
thread per physical core (``numa-cores``) or every thread (``numa``).  It intersects
that with what the process may already use (a cgroup cpuset or the kubelet's static CPU
manager), and can leave out the cores other tenants keep busy right now (:func:`cpu_busy`).
:func:`apply` sets it on the calling process; children inherit it over fork and exec.  A
plan smaller than ``min_cpus`` is not applied: a tight pod cpuset is already the
operator's placement.

Everything is read from sysfs and ``/proc/stat``, before the process touches a GPU.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Set

SYS = "/sys"
MODES = ("none", "numa", "numa-cores", "auto")


def parse_cpulist(text: str) -> List[int]:
    """``0-3,8,10-11`` → [0, 1, 2, 3, 8, 10, 11]."""
    out: List[int] = []
    for part in text.strip().split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-", 1)
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return out


def _read(path: str) -> Optional[str]:
    try:
        with open(path) as f:
            return f.read()
    except OSError:
        return None


def amd_gpu_nodes(sys_root: str = SYS) -> List[int]:
    """NUMA node of each AMD GPU / accelerator (PCI vendor 0x1002, display or processing-
    accelerator class), in PCI address order (the order HIP enumerates them)."""
    base = os.path.join(sys_root, "bus", "pci", "devices")
    try:
        bdfs = sorted(os.listdir(base))
    except OSError:
        return []
    nodes = []
    for bdf in bdfs:
        d = os.path.join(base, bdf)
        vendor = (_read(os.path.join(d, "vendor")) or "").strip()
        cls = (_read(os.path.join(d, "class")) or "").strip()
        if vendor != "0x1002" or not (cls.startswith("0x0380") or cls.startswith("0x0300") or cls.startswith("0x1200")):
            continue
        n = (_read(os.path.join(d, "numa_node")) or "-1").strip()
        nodes.append(int(n) if n.lstrip("-").isdigit() else -1)
    return nodes


def node_cpus(node: int, sys_root: str = SYS) -> List[int]:
    text = _read(os.path.join(sys_root, "devices", "system", "node", f"node{node}", "cpulist"))
    return parse_cpulist(text) if text else []


def first_threads(cpus: List[int], sys_root: str = SYS) -> List[int]:
    """One hardware thread per physical core: a CPU is kept when it is the lowest of its
    ``thread_siblings_list`` (no SMT sibling of the set's own CPUs)."""
    out = []
    for c in cpus:
        sib = _read(os.path.join(sys_root, "devices", "system", "cpu", f"cpu{c}", "topology", "thread_siblings_list"))
        if sib is None or min(parse_cpulist(sib)) == c:
            out.append(c)
    return out


def cpu_busy(interval: float = 0.25, proc_root: str = "/proc") -> Dict[int, float]:
    """Each CPU's busy share over ``interval`` seconds (``/proc/stat``: everything but idle
    and iowait) — what other tenants of a shared host are running where."""
    import time

    def snap() -> Dict[int, tuple]:
        out = {}
        text = _read(os.path.join(proc_root, "stat")) or ""
        for line in text.splitlines():
            if line.startswith("cpu") and line[3:4].isdigit():
                parts = line.split()
                v = [int(x) for x in parts[1:]]
                idle = v[3] + (v[4] if len(v) > 4 else 0)
                out[int(parts[0][3:])] = (sum(v) - idle, sum(v))
        return out

    a = snap()
    time.sleep(interval)
    b = snap()
    busy = {}
    for c, (bb, bt) in b.items():
        ab, at = a.get(c, (bb, bt))
        busy[c] = (bb - ab) / (bt - at) if bt > at else 0.0
    return busy


def _siblings(c: int, sys_root: str) -> List[int]:
    sib = _read(os.path.join(sys_root, "devices", "system", "cpu", f"cpu{c}", "topology", "thread_siblings_list"))
    return parse_cpulist(sib) if sib else [c]


def plan(mode: str = "auto", gpu_index: int = 0, allowed: Optional[Set[int]] = None, min_cpus: int = 16,
         sys_root: str = SYS, busy: Optional[Dict[int, float]] = None,
         busy_max: float = 0.5) -> Optional[Dict[str, object]]:
    """The CPU set for ``mode`` (None: leave placement alone).  ``auto`` is ``numa-cores``
    when that leaves at least ``min_cpus`` CPUs, else ``numa``, else nothing.

    With ``busy`` (:func:`cpu_busy`, a shared host's current load per CPU), ``numa-cores``
    leaves out the physical cores another tenant keeps busy (both threads together at or
    over ``busy_max``) while ``min_cpus`` remain: those cores would run the replica at SMT
    speed.  The summary records how many were left out."""
    if mode not in MODES:
        raise ValueError(f"cpu affinity mode must be one of {MODES}, not {mode!r}")
    if mode == "none":
        return None
    if allowed is None:
        allowed = set(os.sched_getaffinity(0))
    gpus = amd_gpu_nodes(sys_root)
    node = gpus[gpu_index] if 0 <= gpu_index < len(gpus) and gpus[gpu_index] >= 0 else 0
    cpus = [c for c in node_cpus(node, sys_root) if c in allowed]
    if not cpus:
        return None
    tries = ["numa-cores", "numa"] if mode == "auto" else [mode]
    for m in tries:
        sel = first_threads(cpus, sys_root) if m == "numa-cores" else cpus
        if len(sel) < min_cpus:
            continue
        out: Dict[str, object] = {"mode": m, "node": node, "cpus": sel}
        if busy is not None and m == "numa-cores":
            quiet = [c for c in sel if sum(busy.get(x, 0.0) for x in _siblings(c, sys_root)) < busy_max]
            if len(quiet) >= min_cpus:
                out["cpus"] = quiet
                out["busy_cores_skipped"] = len(sel) - len(quiet)
        return out
    return None


def apply(p: Optional[Dict[str, object]]) -> Optional[Dict[str, object]]:
    """Restrict this process (and what it starts from now on) to the plan's CPUs; returns
    the summary recorded in the bench line (mode, node, CPU count), or None."""
    if not p:
        return None
    cpus = list(p["cpus"])  # type: ignore[arg-type]
    os.sched_setaffinity(0, cpus)
    out = {"mode": p["mode"], "node": p["node"], "cpus": len(cpus)}
    if "busy_cores_skipped" in p:
        out["busy_cores_skipped"] = p["busy_cores_skipped"]
    return out
