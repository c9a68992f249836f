"""Per-node GPU attribution agent (DaemonSet on MI355X nodes).

The cluster supervisor runs anywhere; GPU facts live on the node.  This agent
runs next to the GPUs (``hostPID`` so amd-smi PIDs match ``/proc``), keeps the
native amd-smi monitor running (:mod:`.telemetry`), watches the Nexus pods
scheduled on its node, and — the moment one of them fails or is hit by a GPU
fault — publishes an evidence record as the pod annotation
``nexus.amd.com/gpu-evidence`` (merge-PATCH).  The supervisor's classifier reads
it when deciding HBM-OOM vs host-OOM (:mod:`.oom`) and copies it into the
checkpoint trace column.

GPU ↔ pod mapping, strongest first: cgroup pod UID of the processes amd-smi saw
on each GPU (needs hostPID); the kubelet pod-resources allocation (device BDFs,
:mod:`.podresources`); the pod's ``HIP_VISIBLE_DEVICES``/``LOCAL_RANK`` env.

No counterpart in the reference (it has no node component).
"""
from __future__ import annotations

import asyncio
import json
import logging
import time
from typing import Any, Dict, List, Optional, Set, Tuple

from ..informer import InformerFactory
from ..models import kube
from .podresources import PodResourcesClient, gpu_allocations, normalize_bdf
from .telemetry import ATTRIBUTION_EVENTS, FAULT_EVENTS, GpuTelemetry, _pod_gpus, evidence_for
from .topology import topology_from_pod

log = logging.getLogger("nexus_supervisor_amd.agent")



def pod_failed(pod: Dict[str, Any]) -> bool:
    st = pod.get("status") or {}
    if st.get("phase") == "Failed" or st.get("reason") == "Evicted":
        return True
    for t in kube.terminated_states(pod):
        if t.get("which") == "state" and (t.get("exitCode") or 0) != 0:
            return True
    return False


class NodeAgent:
    def __init__(self, kube_client, telemetry: GpuTelemetry, node_name: str, namespace: str, *,
                 label_selector: str = "", annotation: str = "nexus.amd.com/gpu-evidence",
                 gpu_resource: str = "amd.com/gpu", pod_resources: Optional[PodResourcesClient] = None,
                 event_poll: float = 0.1, lookback: float = 600.0, factory: Optional[InformerFactory] = None):
        self.kube = kube_client
        self.tel = telemetry
        self.node = node_name
        self.namespace = namespace
        self.annotation = annotation
        self.gpu_resource = gpu_resource
        self.podres = pod_resources
        self.event_poll = event_poll
        self.lookback = lookback
        if factory is None:
            from ..kube.client import KubeListWatch

            factory = InformerFactory(lambda kind: KubeListWatch(kube_client, kind, namespace, label_selector=label_selector,
                                                                 field_selector=f"spec.nodeName={node_name}"), resync_period=0)
        self.factory = factory
        self.pods = factory.informer("Pod")
        self.published: Dict[str, str] = {}  # pod uid -> reason published
        self.faults: List[Dict[str, Any]] = []
        self._tasks: List[asyncio.Task] = []
        self._bdf_index: Dict[str, int] = {}
        self.patches = 0

    # ------------------------------------------------------------ lifecycle
    async def start(self) -> None:
        self.tel.start()
        self._bdf_index = {normalize_bdf(d.get("bdf", "")): d["index"] for d in self.tel.devices() if d.get("bdf")}
        self.pods.add_event_handler(on_add=lambda p: self._on_pod(None, p), on_update=self._on_pod)
        self.factory.start()
        self._tasks.append(asyncio.create_task(self._event_loop(), name="agent-gpu-events"))

    async def stop(self) -> None:
        for t in self._tasks:
            t.cancel()
        await asyncio.gather(*self._tasks, return_exceptions=True)
        await self.factory.stop()
        self.tel.stop()
        if self.podres is not None:
            self.podres.close()

    # ------------------------------------------------------------ mapping
    def allocation(self, pod: Dict[str, Any]) -> List[int]:
        """Physical GPU indices the device plugin allocated to ``pod`` (kubelet
        pod-resources, by PCI BDF), sorted: what the container enumerates as HIP
        ordinals 0..k-1 before any *_VISIBLE_DEVICES narrowing.  Empty when unknown."""
        if self.podres is None:
            return []
        try:
            alloc = gpu_allocations(self.podres.list(), self.gpu_resource)
        except Exception as exc:  # noqa: BLE001 - kubelet socket optional
            log.debug("pod-resources lookup failed: %s", exc)
            return []
        ids = alloc.get((kube.namespace_of(pod), kube.name_of(pod)), [])
        return sorted(self._bdf_index[normalize_bdf(i)] for i in ids if normalize_bdf(i) in self._bdf_index)

    def gpus_for(self, pod: Dict[str, Any], allocated: Optional[List[int]] = None) -> List[int]:
        """Physical GPU indices of ``pod``: the allocation, else its env's devices
        (logical ordinals mapped through ROCR/HIP_VISIBLE_DEVICES)."""
        alloc = self.allocation(pod) if allocated is None else allocated
        if alloc:
            return alloc
        topo = topology_from_pod(pod, self.gpu_resource)
        return _pod_gpus(topo, self.tel.devices())

    def evidence(self, pod: Dict[str, Any]) -> Optional[Dict[str, Any]]:
        alloc = self.allocation(pod)
        return evidence_for(self.tel, pod_uid=kube.uid_of(pod), gpu_indices=self.gpus_for(pod, alloc),
                            lookback=self.lookback, node=self.node, allocated=alloc)

    # ------------------------------------------------------------ publishing
    async def publish(self, pod: Dict[str, Any], reason: str) -> bool:
        ev = self.evidence(pod)
        if ev is None:
            return False
        ev["reason"] = reason
        body = {"metadata": {"annotations": {self.annotation: json.dumps(ev, separators=(",", ":"), sort_keys=True)}}}
        try:
            await self.kube.patch_merge("Pod", kube.namespace_of(pod), kube.name_of(pod), body)
        except Exception as exc:  # noqa: BLE001
            log.warning("annotating pod %s failed: %s", kube.name_of(pod), exc)
            return False
        self.published[kube.uid_of(pod)] = reason
        self.patches += 1
        return True

    def _on_pod(self, old, pod) -> None:
        uid = kube.uid_of(pod)
        if uid in self.published or not pod_failed(pod):
            return
        if kube.annotations_of(pod).get(self.annotation):
            self.published[uid] = "present"
            return
        self.published[uid] = "pending"
        asyncio.ensure_future(self.publish(pod, "pod-failed"))

    async def _event_loop(self) -> None:
        while True:
            await asyncio.sleep(self.event_poll)
            try:
                events = self.tel.drain_events()
            except Exception:  # noqa: BLE001
                continue
            faults = [e for e in events if e.get("type") in FAULT_EVENTS]
            if not faults:
                continue
            self.faults.extend(faults)
            hit: Set[int] = {e["gpu"] for e in faults}
            for pod in self.pods.indexer.values():
                if (pod.get("status") or {}).get("phase") not in ("Running", "Pending"):
                    continue
                if hit & set(self.gpus_for(pod)):
                    await self.publish(pod, "gpu-fault:" + ",".join(sorted({e["type"] for e in faults})))


async def run_agent(cfg, node_name: str) -> None:  # pragma: no cover - process entry
    from ..kube.client import KubeClient, KubeConfig
    from .podresources import SOCKET
    from .telemetry import make_telemetry
    import os

    kc = KubeClient(KubeConfig.load(cfg.kube_config_path))
    tel = make_telemetry("amdsmi" if cfg.gpu.backend == "auto" else cfg.gpu.backend, cfg.gpu.sample_interval)
    if tel is None:
        raise RuntimeError("no GPU telemetry backend on this node")
    pr = PodResourcesClient() if os.path.exists(SOCKET) else None
    sel = f"{cfg.labels.nexus_component_label}={cfg.labels.algorithm_run_value}"
    agent = NodeAgent(kc, tel, node_name, cfg.resource_namespace, label_selector=sel,
                      annotation=cfg.gpu.evidence_annotation, gpu_resource=cfg.gpu.gpu_resource_name, pod_resources=pr)
    await agent.start()
    stop = asyncio.Event()
    import signal

    loop = asyncio.get_running_loop()
    for s in (signal.SIGTERM, signal.SIGINT):
        loop.add_signal_handler(s, stop.set)
    await stop.wait()
    await agent.stop()
    await kc.close()
