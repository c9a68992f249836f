"""GPU-local CPU placement for one process group per GPU-job slot.

An MI355X node hangs its eight OAM GPUs off two (or more) NUMA nodes.  A benchmark rank
(``bench.py``: one supervisor replica per GPU-job slot, with its shard workers, watch
hub and the harness's API-server / CQL simulators) is a dozen processes that talk to
each other over sockets all the time: left to the scheduler they spread over the whole
machine — both sockets, every CCD — and every hand-off crosses an L3 (or the socket
interconnect).  :func:`plan` gives each rank a compact block of physical cores on its
own GPU's NUMA node (``/sys/bus/pci/devices/<bdf>/local_cpulist``), sized to the rank's
CPU share and disjoint from the blocks of the other local ranks on that node; children
inherit the mask from the process that spawns them.

Measured (``profiles/r3_placement_ab``, MI355X box: 2 × EPYC 9575F, 8-core CCDs with
32 MB L3 each, cgroup quota 16 CPUs): pinning one rank to 16 GPU-local cores made it
20-25 % *slower* (31.6-33.6k vs 41.1k failures/s, 157-185 vs 139 µs of replica CPU per
failure) — the rank's Python processes, each with a large heap, then share two CCDs'
L3 instead of getting most of one each, which outweighs the shorter socket hand-offs.
So ``bench.py`` leaves placement off by default (``--cpu-placement gpu-local`` opts in).

There is no reference counterpart: the reference is one Go process with no placement
(``/root/reference/services/supervisor.go:69-135``).
"""
from __future__ import annotations

import os
from typing import Dict, Iterable, List, Optional, Sequence

SYS_PCI = "/sys/bus/pci/devices"
SYS_CPU = "/sys/devices/system/cpu"


def parse_cpulist(text: str) -> List[int]:
    """``"0-3,8,10-11"`` → ``[0, 1, 2, 3, 8, 10, 11]`` (the kernel's cpulist format)."""
    out: List[int] = []
    for part in (text or "").strip().split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            lo, hi = part.split("-", 1)
            out.extend(range(int(lo), int(hi) + 1))
        else:
            out.append(int(part))
    return sorted(set(out))


def format_cpulist(cpus: Iterable[int]) -> str:
    """Inverse of :func:`parse_cpulist` (compact ranges)."""
    cs = sorted(set(cpus))
    parts: List[str] = []
    i = 0
    while i < len(cs):
        j = i
        while j + 1 < len(cs) and cs[j + 1] == cs[j] + 1:
            j += 1
        parts.append(str(cs[i]) if i == j else f"{cs[i]}-{cs[j]}")
        i = j + 1
    return ",".join(parts)


def _read(path: str) -> Optional[str]:
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def pci_bdf(domain: int, bus: int, device: int, function: int = 0) -> str:
    return f"{domain:04x}:{bus:02x}:{device:02x}.{function:x}"


def device_locality(bdf: str, sys_pci: str = SYS_PCI) -> Dict[str, object]:
    """NUMA node and local CPUs of a PCI device (``numa_node`` -1 when the firmware
    does not say)."""
    base = os.path.join(sys_pci, bdf)
    node = _read(os.path.join(base, "numa_node"))
    cpus = _read(os.path.join(base, "local_cpulist"))
    return {"bdf": bdf, "numa_node": int(node) if node not in (None, "") else -1,
            "local_cpus": parse_cpulist(cpus) if cpus else []}


def primary_threads(cpus: Sequence[int], sys_cpu: str = SYS_CPU) -> List[int]:
    """The first SMT thread of every core among ``cpus`` (a block of *cores*, not of
    hyperthread siblings competing for one core's pipelines).  CPUs whose topology is
    unreadable are kept."""
    cores: Dict[object, int] = {}
    for c in sorted(cpus):
        sib = _read(os.path.join(sys_cpu, f"cpu{c}", "topology", "thread_siblings_list"))
        core = parse_cpulist(sib)[0] if sib else ("cpu", c)
        cores.setdefault(core, c)  # the lowest allowed thread stands for its core
    return sorted(cores.values())


def plan(local_rank: int, local_world: int, gpu_bdfs: Sequence[str], allowed: Sequence[int], per_rank: int,
         sys_pci: str = SYS_PCI, sys_cpu: str = SYS_CPU) -> Dict[str, object]:
    """CPU block of ``local_rank`` (of ``local_world`` ranks on this host) given the local
    ranks' GPUs (``gpu_bdfs[i]`` is rank i's GPU; missing or empty = unknown) and the CPUs
    this process may use.

    Ranks whose GPUs share a NUMA node split that node's allowed cores in local-rank
    order, ``per_rank`` cores each; a node too small for all of them gives every rank an
    equal share (at least one core).  Falls back to an even split of ``allowed`` when
    the GPU's locality is unknown or none of its CPUs are allowed.  Returns ``cpus``
    (empty = leave the mask alone) and how it was chosen."""
    allowed_set = set(allowed)
    per_rank = max(1, int(per_rank))
    unknown = {"numa_node": -1, "local_cpus": []}
    bdfs = list(gpu_bdfs)[:local_world] + [""] * max(0, local_world - len(gpu_bdfs))
    loc = [device_locality(b, sys_pci) if b else unknown for b in bdfs]
    me = loc[local_rank] if local_rank < len(loc) else unknown
    node = me["numa_node"]
    local = [c for c in me["local_cpus"] if c in allowed_set]
    how = "gpu-local"
    if node < 0 or not local:
        # unknown locality: an even, contiguous split of what we may use
        peers = list(range(max(local_world, local_rank + 1)))
        pool = primary_threads(sorted(allowed_set), sys_cpu)
        how = "split"
    else:
        peers = [i for i, l in enumerate(loc) if l["numa_node"] == node] or [local_rank]
        pool = primary_threads(local, sys_cpu)
    if not pool:
        return {"cpus": [], "how": "none", "numa_node": node}
    j = peers.index(local_rank) if local_rank in peers else 0
    n = min(per_rank, max(1, len(pool) // max(1, len(peers))))
    cpus = pool[j * n:(j + 1) * n] or pool[-n:]
    return {"cpus": cpus, "how": how, "numa_node": node, "pool": len(pool), "peers": len(peers)}


def apply(cpus: Sequence[int]) -> bool:
    """Pin the calling thread (and so every child it spawns from now on)."""
    if not cpus:
        return False
    try:
        os.sched_setaffinity(0, set(cpus))
        return True
    except (AttributeError, OSError, ValueError):
        return False
