"""RCCL / xGMI rank topology of a supervised job, read from its pod (north star:
"the RCCL/xGMI rank topology of the supervised job read from pod env and
written into the trace row").

The reference caches pods (``/root/reference/services/supervisor.go:74``) but
never inspects them beyond labels.  Here the pod's literal container env
(torchrun / RCCL variables), its ``amd.com/gpu`` request and its node are
folded into one JSON-able record.  Per-process truth (which rank actually sits
on which GPU) comes from the node agent (:mod:`.agent`) reading
``/proc/<pid>/environ`` of the processes amd-smi reports on each GPU; the two
views are merged by :func:`merge_process_ranks`.
"""
from __future__ import annotations

from typing import Any, Dict, Iterable, List, Optional, Tuple

from ..models import kube

RANK_VARS = ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "NODE_RANK", "NNODES",
             "ROLE_RANK", "ROLE_WORLD_SIZE", "JOB_COMPLETION_INDEX", "MASTER_ADDR", "MASTER_PORT")
DEVICE_VARS = ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "GPU_DEVICE_ORDINAL")
COLLECTIVE_PREFIXES = kube.ENV_PREFIXES  # the decoder keeps exactly these env families
# MI355X node: 8 OAM GPUs, every pair joined by xGMI (7 links per GPU)
GPUS_PER_NODE = 8
XGMI_LINKS_PER_GPU = 7


_INT_VARS = (("RANK", "rank"), ("WORLD_SIZE", "world_size"), ("LOCAL_RANK", "local_rank"),
             ("LOCAL_WORLD_SIZE", "local_world_size"), ("GROUP_RANK", "group_rank"), ("NODE_RANK", "node_rank"),
             ("NNODES", "nnodes"), ("JOB_COMPLETION_INDEX", "completion_index"), ("MASTER_PORT", "master_port"))


def _int(v) -> Optional[int]:
    try:
        return int(str(v).strip())
    except (TypeError, ValueError):
        return None


def parse_visible_devices(value: Optional[str]) -> List[str]:
    """``"0,1,2"`` → ``["0","1","2"]``; UUID entries (``GPU-…``) are kept verbatim."""
    if not value:
        return []
    return [v.strip() for v in str(value).split(",") if v.strip()]


# HIP device selection is layered: ROCr filters the node's agents first, then HIP
# indexes into what ROCr left (CUDA_VISIBLE_DEVICES is HIP's alias when HIP_* is unset).
_DEVICE_CHAIN = (("ROCR_VISIBLE_DEVICES",), ("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"))


# torchrun arguments given as env (``PET_<ARG>``: the Kubeflow training operator's PyTorchJob,
# or a pod that runs torchrun itself) → the topology keys they imply; the RANK family is set
# by torchrun in its child processes only, so from the pod spec these are all there is
_PET_VARS = ("PET_NNODES", "PET_NPROC_PER_NODE", "PET_NODE_RANK", "PET_MASTER_ADDR", "PET_MASTER_PORT",
             "PET_RDZV_ENDPOINT", "PET_RDZV_BACKEND")

# every variable _topology_from_env reads (besides the collective prefixes)
_READ_VARS = frozenset([v for v, _k in _INT_VARS] + [v for names in _DEVICE_CHAIN for v in names]
                       + ["GPU_DEVICE_ORDINAL"] + list(_PET_VARS))


def _launcher_env(env: Dict[str, str], topo: Dict[str, Any], gpus_requested: int) -> None:
    """Fold torchrun's ``PET_*`` arguments into ``topo`` where the direct variables are
    absent: nodes, processes per node (``gpu`` / ``auto`` = the pod's GPUs), this node's
    rank, the rendezvous endpoint, and the world size they imply.  An elastic range
    (``PET_NNODES=1:4``) is kept as ``nnodes_range``: the world size is then unknown."""
    if not any(v in env for v in _PET_VARS):
        return
    topo["launcher"] = "torchrun"
    nn = (env.get("PET_NNODES") or "").strip()
    if nn and "nnodes" not in topo:
        if ":" in nn:
            lo, _sep, hi = nn.partition(":")
            if _int(lo) is not None and _int(hi) is not None:
                topo["nnodes_range"] = [_int(lo), _int(hi)]
                if _int(lo) == _int(hi):
                    topo["nnodes"] = _int(lo)
        elif _int(nn) is not None:
            topo["nnodes"] = _int(nn)
    npp = (env.get("PET_NPROC_PER_NODE") or "").strip()
    if npp and "local_world_size" not in topo:
        n = _int(npp)
        if n is None and npp in ("gpu", "auto") and gpus_requested:
            n = gpus_requested  # torchrun: one process per visible GPU
        if n is not None:
            topo["local_world_size"] = n
    nr = _int(env.get("PET_NODE_RANK"))
    if nr is not None and "node_rank" not in topo:
        topo["node_rank"] = nr
    addr, port = env.get("PET_MASTER_ADDR"), _int(env.get("PET_MASTER_PORT"))
    ep = env.get("PET_RDZV_ENDPOINT") or ""
    if not addr and ep:
        host, _sep, p = ep.rpartition(":")
        addr, port = (host, _int(p)) if host and _int(p) is not None else (ep, port)
    if addr and "master_addr" not in topo:
        topo["master_addr"] = addr
    if port is not None and "master_port" not in topo:
        topo["master_port"] = port
    if env.get("PET_RDZV_BACKEND"):
        topo["rdzv_backend"] = env["PET_RDZV_BACKEND"]
    if "world_size" not in topo and topo.get("nnodes") and topo.get("local_world_size"):
        topo["world_size"] = topo["nnodes"] * topo["local_world_size"]
_ENV_MEMO: Dict[Tuple, Dict[str, Any]] = {}


def topology_from_env(env: Dict[str, str], gpus_requested: int = 0, node: str = "") -> Dict[str, Any]:
    """:func:`_topology_from_env`, memoised on the variables it reads except ``MASTER_ADDR``
    (unique per run; re-attached to a shallow copy).  Every run of a job template on a
    node folds the same rank/device/collective env: the fold is done once.  The result
    is shared and must not be mutated (callers build new dicts, as everywhere here).

    The memo key is the env's items in document order (C-level copy, no sort or filter:
    one job template always lists its variables in the same order, and a variable the
    fold does not read only splits the memo, it cannot change a result)."""
    addr = env.get("MASTER_ADDR")
    if addr is not None:
        env = env.copy()
        del env["MASTER_ADDR"]
    key = (tuple(env.items()), gpus_requested, node)
    topo = _ENV_MEMO.get(key)
    if topo is None:
        if len(_ENV_MEMO) > 4096:
            _ENV_MEMO.clear()
        topo = _ENV_MEMO[key] = _topology_from_env(
            {k: v for k, v in key[0] if k in _READ_VARS or k.startswith(COLLECTIVE_PREFIXES)}, gpus_requested, node)
    if addr:
        return dict(topo, master_addr=addr) if topo else _topology_from_env({"MASTER_ADDR": addr}, gpus_requested, node)
    return topo


def _topology_from_env(env: Dict[str, str], gpus_requested: int = 0, node: str = "") -> Dict[str, Any]:
    """Fold torchrun / RCCL env into a topology record (only non-empty keys).

    ``visible_devices`` is the *composed* device list in the container's numbering
    (ROCR_VISIBLE_DEVICES, then HIP/CUDA_VISIBLE_DEVICES indexing into it): entry ``i`` is
    what a process's HIP ordinal ``i`` (torch's ``GPU i``) opens.  ``device_chain`` keeps
    each layer.  The container numbering equals the node's physical numbering only when
    the container sees every GPU; :func:`resolve_devices` applies the device-plugin
    allocation when the node agent reported one."""
    topo: Dict[str, Any] = {}
    for var, key in _INT_VARS:
        raw = env.get(var)
        if raw is not None:
            v = _int(raw)
            if v is not None:
                topo[key] = v
    if env.get("MASTER_ADDR"):
        topo["master_addr"] = env["MASTER_ADDR"]
    if "rank" not in topo and "completion_index" in topo:
        topo["rank"] = topo["completion_index"]  # indexed Job → rank
    _launcher_env(env, topo, gpus_requested)
    chain = []
    for names in _DEVICE_CHAIN:
        for var in names:
            devs = parse_visible_devices(env.get(var))
            if devs:
                chain.append([var, devs])
                break
    if chain:
        topo["device_chain"] = chain
        topo["visible_devices"] = device_map(chain)
        topo["visible_devices_var"] = chain[-1][0]
    elif env.get("GPU_DEVICE_ORDINAL"):
        topo["visible_devices"] = parse_visible_devices(env["GPU_DEVICE_ORDINAL"])
        topo["visible_devices_var"] = "GPU_DEVICE_ORDINAL"
    coll = {k: v for k, v in env.items() if k.startswith(COLLECTIVE_PREFIXES)}
    if coll:
        topo["collective_env"] = dict(sorted(coll.items()))
    if gpus_requested:
        topo["gpus_requested"] = gpus_requested
    if node:
        topo["node"] = node
    if topo:
        topo["backend"] = "rccl"
        n_local = topo.get("local_world_size") or gpus_requested or len(topo.get("visible_devices", []))
        if n_local:
            # Platform default only (MI355X: 8 OAM GPUs, all pairs xGMI-connected).  The
            # measured fabric replaces this in :func:`xgmi_from_evidence` when telemetry
            # reported link metrics.
            topo["xgmi"] = {
                "source": "platform-default",
                "local_gpus": n_local,
                "links_per_gpu": min(XGMI_LINKS_PER_GPU, max(n_local - 1, 0)),
                "fully_connected": n_local <= GPUS_PER_NODE,
            }
        gpu = expected_gpu(topo)
        if gpu is not None:
            topo["expected_gpu"] = gpu
    return topo


def device_map(chain: List, allocated: Optional[List[int]] = None) -> List[str]:
    """Physical device of each logical HIP ordinal: the allocation (the GPUs a device
    plugin exposed to the container, in node order) narrowed by each env layer; entries
    are physical index strings or GPU UUIDs.  Empty = identity (nothing restricts)."""
    base: Optional[List[str]] = [str(i) for i in allocated] if allocated else None
    for _var, sel in chain:
        if base is None:
            base = list(sel)
            continue
        out = []
        for x in sel:
            if x.isdigit():
                i = int(x)
                if i < len(base):
                    out.append(base[i])
            else:
                out.append(x)  # a UUID names a device absolutely
        base = out
    return base or []


def physical_gpu(topo: Dict[str, Any], logical: Optional[int], gpus: Iterable[Dict[str, Any]] = (),
                 allocated: Optional[List[int]] = None) -> Optional[int]:
    """Physical GPU index behind a process's logical HIP ordinal (torch ``GPU N``).
    UUID entries resolve against telemetry records (``uuid`` / ``hip_uuid``)."""
    if logical is None:
        return None
    m = device_map(topo.get("device_chain") or [], allocated)
    if not m:
        return int(logical)
    if not 0 <= logical < len(m):
        return None
    ent = m[logical]
    if ent.isdigit():
        return int(ent)
    for g in gpus:
        if ent in (g.get("uuid"), g.get("hip_uuid")):
            return g.get("index")
    return None


def resolve_devices(topo: Dict[str, Any], gpu_evidence: Optional[Dict[str, Any]]) -> Dict[str, Any]:
    """Topology with the node's *physical* view applied: the device-plugin allocation the
    node agent reported (``gpu_evidence["allocated"]``) and UUID entries resolved against
    its GPU records.  Adds ``physical_devices`` and turns ``expected_gpu`` into the
    physical index (``expected_gpu_logical`` keeps the rank's ordinal).  Returns a new
    dict; the per-version memo of :func:`topology_from_pod` is never mutated."""
    alloc = list((gpu_evidence or {}).get("allocated") or [])
    gpus = (gpu_evidence or {}).get("gpus") or []
    chain = topo.get("device_chain") or []
    if not alloc and not any(not str(x).isdigit() for _v, sel in chain for x in sel):
        return topo
    out = dict(topo)
    m = device_map(chain, alloc)
    phys = []
    for ent in m:
        if ent.isdigit():
            phys.append(int(ent))
        else:
            hit = [g.get("index") for g in gpus if ent in (g.get("uuid"), g.get("hip_uuid"))]
            phys.append(hit[0] if hit else ent)
    if alloc:
        out["allocated_gpus"] = alloc
    if phys:
        out["physical_devices"] = phys
    lr = topo.get("local_rank")
    logical = lr if lr is not None and 0 <= lr < len(phys) else (0 if len(phys) == 1 else None)
    if logical is not None:
        out["expected_gpu_logical"] = logical
        out["expected_gpu"] = str(phys[logical])
    return out


_XGMI_MEMO: Dict[Tuple, Dict[str, Any]] = {}


def xgmi_from_evidence(topo: Dict[str, Any], gpu_evidence: Optional[Dict[str, Any]]) -> Dict[str, Any]:
    """Replace the platform-default xGMI block with the measured fabric of the pod's GPUs
    (link metrics the native monitor read from amd-smi: peers, rates, link status).  The
    block depends only on the GPUs' link records, which one telemetry snapshot shares
    between every pod's evidence: it is built once per snapshot and GPU set (shared,
    never mutated)."""
    gpus = [g for g in (gpu_evidence or {}).get("gpus", []) if g.get("links") is not None]
    if not gpus:
        return topo
    key = (gpu_evidence.get("source"),) + tuple((g.get("index"), id(g["links"]), g.get("xgmi_links_up"),
                                                 g.get("xgmi_links_down"), g.get("xgmi_hive_id")) for g in gpus)
    hit = _XGMI_MEMO.get(key)
    if hit is not None and all(h is g["links"] for h, g in zip(hit["_links"], gpus)):
        out = dict(topo)
        out["xgmi"] = hit["rec"]
        return out
    out = _xgmi_from_evidence(topo, gpu_evidence, gpus)
    if len(_XGMI_MEMO) > 256:
        _XGMI_MEMO.clear()
    _XGMI_MEMO[key] = {"rec": out["xgmi"], "_links": [g["links"] for g in gpus]}  # keeps the ids alive
    return out


def _xgmi_from_evidence(topo: Dict[str, Any], gpu_evidence: Dict[str, Any], gpus: List[Dict[str, Any]]) -> Dict[str, Any]:
    """The measured fabric as a compact, bounded block (the trace row has a size cap): per GPU the
    peers its xGMI ports reach — resolved to the peer's index when the peer is one of the
    node's enumerated GPUs (matched by PCI BDF in the native monitor), else its BDF — the
    link rate, and the port counts.  ``links_listed`` / ``links_up`` count those peer links
    (so they agree with the peers listed), ``ports_total`` / ``ports_up`` are amd-smi's
    link-status view of every port (it includes ports without a peer).  No cumulative
    traffic counters: they grow without bound and say nothing about the failure.
    ``fully_connected`` is None for fewer than two GPUs (nothing to connect)."""
    idx = {g.get("index") for g in gpus}
    hive = set()
    per_gpu = []
    pairs = set()
    for g in gpus:
        if g.get("xgmi_hive_id"):
            hive.add(g["xgmi_hive_id"])
        peers, rates, maxes = [], set(), set()
        up = 0
        for l in g["links"]:
            peer = l.get("peer")
            peers.append(peer if peer is not None else l.get("peer_bdf"))
            if l.get("gbps"):
                up += 1
                rates.add(l["gbps"])
            if l.get("max_gbps"):
                maxes.add(l["max_gbps"])
            if peer in idx and peer != g.get("index"):
                pairs.add(tuple(sorted((g.get("index"), peer))))
        rec_g: Dict[str, Any] = {"gpu": g.get("index"), "peers": peers, "links_listed": len(peers), "links_up": up}
        if rates:
            rec_g["gbps"] = rates.pop() if len(rates) == 1 else sorted(rates)
        if maxes:
            rec_g["max_gbps"] = maxes.pop() if len(maxes) == 1 else sorted(maxes)
        if g.get("xgmi_links_total") is not None:
            rec_g["ports_total"] = g.get("xgmi_links_total")
            rec_g["ports_up"] = g.get("xgmi_links_up")
            rec_g["ports_down"] = g.get("xgmi_links_down") or 0
        per_gpu.append(rec_g)
    n = len(idx)
    rec: Dict[str, Any] = {
        "source": gpu_evidence.get("source", "telemetry"),
        "gpus": sorted(idx),
        "per_gpu": per_gpu,
        "pairs_connected": [list(p) for p in sorted(pairs)],
        "fully_connected": (len(pairs) == n * (n - 1) // 2) if n >= 2 else None,
        "links_listed": sum(r["links_listed"] for r in per_gpu),
        "links_up": sum(r["links_up"] for r in per_gpu),
    }
    if hive:
        rec["hive_ids"] = sorted(hive)
    if any("ports_total" in r for r in per_gpu):
        rec["ports_total"] = sum(r.get("ports_total") or 0 for r in per_gpu)
        rec["ports_up"] = sum(r.get("ports_up") or 0 for r in per_gpu)
        rec["ports_down"] = sum(r.get("ports_down") or 0 for r in per_gpu)
    out = dict(topo)
    out["xgmi"] = rec
    return out


def expected_gpu(topo: Dict[str, Any]) -> Optional[str]:
    """The device a one-GPU-per-process rank should be on: ``visible[local_rank]``."""
    devs = topo.get("visible_devices") or []
    lr = topo.get("local_rank")
    if devs and lr is not None and 0 <= lr < len(devs):
        return devs[lr]
    if len(devs) == 1:
        return devs[0]
    return None


def topology_from_pod(pod: Dict[str, Any], gpu_resource: str = "amd.com/gpu") -> Dict[str, Any]:
    """Topology of one pod version, memoised on the (immutable, per-version) object."""
    rv = kube.resource_version(pod)
    cache = pod.get("_topo")
    if cache is not None and cache[0] == gpu_resource and cache[1] == rv and rv:
        return cache[2]
    topo = _topology_from_pod(pod, gpu_resource)
    pod["_topo"] = (gpu_resource, rv, topo)
    return topo


def _topology_from_pod(pod: Dict[str, Any], gpu_resource: str) -> Dict[str, Any]:
    env = kube.pod_env(pod)
    ann = kube.annotations_of(pod)
    idx = ann.get("batch.kubernetes.io/job-completion-index")
    if idx is not None and "JOB_COMPLETION_INDEX" not in env:
        env = dict(env, JOB_COMPLETION_INDEX=idx)
    node = (pod.get("spec") or {}).get("nodeName", "")
    return topology_from_env(env, kube.gpu_request(pod, gpu_resource), node)


def merge_process_ranks(topo: Dict[str, Any], gpu_evidence: Optional[Dict[str, Any]]) -> Dict[str, Any]:
    """Attach the agent's per-GPU rank map to ``topo``: one entry per (rank, GPU) —
    ``{"rank", "local_rank", "gpu", "pid", "procs"}`` with ``pid`` the rank's process with
    the largest VRAM peak and ``procs`` how many of its processes used that GPU (a
    dataloader's helpers must not multiply the trace)."""
    if not gpu_evidence:
        return topo
    groups: Dict[Tuple, Dict[str, Any]] = {}
    for g in gpu_evidence.get("gpus", []):
        for p in g.get("procs", []):
            key = (p.get("rank"), g.get("index"))
            e = groups.get(key)
            if e is None:
                e = groups[key] = {"gpu": g.get("index"), "pid": p.get("pid"), "procs": 0, "_peak": -1}
                for k in ("rank", "local_rank"):
                    if p.get(k) is not None:
                        e[k] = p[k]
                if p.get("world_size") is not None and "world_size" not in topo:
                    e["world_size"] = p["world_size"]
            e["procs"] += 1
            peak = p.get("peak_vram_bytes") or 0
            if peak > e["_peak"]:
                e["_peak"], e["pid"] = peak, p.get("pid")
    if groups:
        ranks = [{k: v for k, v in e.items() if k != "_peak"} for e in groups.values()]
        topo = dict(topo, rank_map=sorted(ranks, key=lambda e: (e.get("rank", 1 << 30), e.get("gpu") or 0)))
    penv = gpu_evidence.get("collective_env")
    if penv:
        # the RCCL / NCCL settings the ranks actually ran with (a launcher can pass them to
        # its children only: mpirun -x, a wrapper script): the pod spec's own values win
        mine = topo.get("collective_env") or {}
        extra = {k: v for k, v in penv.items() if k not in mine}
        if extra:
            topo = dict(topo, collective_env=dict(sorted({**mine, **extra}.items())))
            if mine:
                topo["collective_env_from_processes"] = sorted(extra)
    return topo


def rank_env_from_environ(environ: Iterable[str]) -> Dict[str, str]:
    """Pick rank/device vars out of a NUL-split ``/proc/<pid>/environ``."""
    out: Dict[str, str] = {}
    for item in environ:
        k, sep, v = item.partition("=")
        if sep and (k in RANK_VARS or k in DEVICE_VARS):
            out[k] = v
    return out
