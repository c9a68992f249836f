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

from typing import Any, Dict, Iterable, List, Optional

from ..models import kube

RANK_VARS = ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "NODE_RANK", "NNODES",
             "ROLE_RANK", "ROLE_WORLD_SIZE", "JOB_COMPLETION_INDEX", "MASTER_ADDR", "MASTER_PORT")
DEVICE_VARS = ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "GPU_DEVICE_ORDINAL")
COLLECTIVE_PREFIXES = ("NCCL_", "RCCL_", "TORCH_NCCL_", "HSA_", "MSCCL", "UCX_")
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


def topology_from_env(env: Dict[str, str], gpus_requested: int = 0, node: str = "") -> Dict[str, Any]:
    """Fold torchrun / RCCL env into a topology record (only non-empty keys)."""
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
    for var in DEVICE_VARS:
        devs = parse_visible_devices(env.get(var))
        if devs:
            topo.setdefault("visible_devices", devs)
            topo.setdefault("visible_devices_var", var)
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
            # single-node GPUs on an MI355X platform are all-to-all xGMI connected
            topo["xgmi"] = {
                "local_gpus": n_local,
                "links_per_gpu": min(XGMI_LINKS_PER_GPU, max(n_local - 1, 0)),
                "fully_connected": n_local <= GPUS_PER_NODE,
            }
        gpu = expected_gpu(topo)
        if gpu is not None:
            topo["expected_gpu"] = gpu
    return topo


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
    """Attach the agent's per-GPU rank map (``{"gpu": idx, "rank": r, "pid": p}``) to ``topo``."""
    if not gpu_evidence:
        return topo
    ranks = []
    for g in gpu_evidence.get("gpus", []):
        for p in g.get("procs", []):
            entry = {"gpu": g.get("index"), "pid": p.get("pid")}
            for k in ("rank", "local_rank", "world_size"):
                if p.get(k) is not None:
                    entry[k] = p[k]
            ranks.append(entry)
    if ranks:
        topo = dict(topo, rank_map=sorted(ranks, key=lambda e: (e.get("rank", 1 << 30), e.get("gpu") or 0)))
    return topo


def rank_env_from_environ(environ: Iterable[str]) -> Dict[str, str]:
    """Pick rank/device vars out of a NUL-split ``/proc/<pid>/environ``."""
    out: Dict[str, str] = {}
    for item in environ:
        k, sep, v = item.partition("=")
        if sep and (k in RANK_VARS or k in DEVICE_VARS):
            out[k] = v
    return out
