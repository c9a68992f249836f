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

Container logs: for every failed container whose termination message is empty (the
default ``terminationMessagePolicy: File`` — PyTorch prints its HBM-OOM to stderr and
exits 1) the agent reads the tail of ``/var/log/pods/<ns>_<pod>_<uid>/<container>/<n>.log``
(read-only hostPath) and publishes the allocation-failure lines it finds (``logs``,
:mod:`.logtail`).

Delivery: an annotation PATCH that fails is retried with capped exponential backoff for
as long as the pod exists; the per-pod bookkeeping is dropped when the pod is deleted
(and by TTL), fault history is bounded, and every publish task is tracked and cancelled
on stop.

No counterpart in the reference (it has no node component).
"""
from __future__ import annotations

import asyncio
import collections
import json
import logging
import time
from typing import Any, Deque, Dict, List, Optional, Set, Tuple

from ..informer import InformerFactory
from ..models import kube
from . import logtail
from .podresources import PodResourcesClient, allocatable_ids, gpu_allocations, normalize_bdf
from .telemetry import ATTRIBUTION_EVENTS, FAULT_EVENTS, GpuTelemetry, _pod_gpus, admission_evidence, evidence_for
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


# capabilities a non-root agent would need (CapEff bits, linux/capability.h): ptrace-read
# access to other users' /proc/<pid>/{fd,fdinfo,environ}, and reading root-owned 0640 logs
_CAPS = {"CAP_DAC_OVERRIDE": 1, "CAP_DAC_READ_SEARCH": 2, "CAP_SYS_PTRACE": 19}


def process_privileges(status_path: str = "/proc/self/status") -> Dict[str, Any]:
    """euid and effective capabilities of this process, and whether they suffice for the
    agent: root (uid 0 in a privileged container has every capability), or
    CAP_SYS_PTRACE + CAP_DAC_READ_SEARCH.  A non-root UID in a ``privileged: true``
    container has an empty effective set — Kubernetes adds capabilities to the bounding
    set, the kernel gives a non-root process none of them."""
    import os

    eff = 0
    try:
        with open(status_path) as f:
            for line in f:
                if line.startswith("CapEff:"):
                    eff = int(line.split()[1], 16)
                    break
    except OSError:
        pass
    have = {k for k, bit in _CAPS.items() if eff >> bit & 1}
    need = {"CAP_SYS_PTRACE"} | ({"CAP_DAC_READ_SEARCH"} if "CAP_DAC_OVERRIDE" not in have else set())
    missing = sorted(need - have)
    return {"euid": os.geteuid(), "cap_eff": f"{eff:016x}", "caps": sorted(have), "missing": missing,
            "sufficient": not missing}


class NodeAgent:
    def __init__(self, kube_client, telemetry: GpuTelemetry, node_name: str, namespace: str, *,
                 label_selector: str = "", annotation: str = "nexus.amd.com/gpu-evidence",
                 gpu_resource: str = "amd.com/gpu", pod_resources: Optional[PodResourcesClient] = None,
                 event_poll: float = 0.1, lookback: float = 600.0, factory: Optional[InformerFactory] = None,
                 log_root: Optional[str] = logtail.LOG_ROOT, log_tail_bytes: int = logtail.TAIL_BYTES,
                 retry_base: float = 0.2, retry_max: float = 10.0, published_ttl: float = 3600.0,
                 max_faults: int = 1024):
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
        self.log_root = log_root
        self.log_tail_bytes = log_tail_bytes
        self.retry_base, self.retry_max = retry_base, retry_max
        self.published_ttl = published_ttl
        # pod uid -> (state, monotonic time): "pending" while a publish task runs, then the
        # reason published ("present": an annotation was already there)
        self.published: Dict[str, Tuple[str, float]] = {}
        self.faults: Deque[Dict[str, Any]] = collections.deque(maxlen=max_faults)
        self._tasks: List[asyncio.Task] = []
        self._publishing: Dict[str, asyncio.Task] = {}  # pod uid -> publish-with-retry task
        self._bdf_index: Dict[str, int] = {}
        self.patches = 0
        self.patch_failures = 0
        from ..obs.metrics import Metrics

        # agent_proc_scan_denied{source} / agent_log_read_denied / agent_podresources_denied:
        # attribution that silently degrades for lack of privileges is counted and logged once
        self.metrics = Metrics("nexus_gpu_agent", {"node": node_name})
        self._denied_seen: Dict[str, int] = {}
        self._vanished_seen = 0
        self._warned: Set[str] = set()
        self.privileges: Dict[str, Any] = {}

    # ------------------------------------------------------------ lifecycle
    async def start(self) -> None:
        self.privileges = process_privileges()
        self.metrics.set("agent_privileged", 1.0 if self.privileges.get("sufficient") else 0.0)
        if not self.privileges.get("sufficient"):
            self._warn_once("privileges", "node agent runs without the privileges per-process GPU attribution needs "
                            "(uid %s, missing %s): other users' /proc/<pid>/fdinfo and environ, root-owned container "
                            "logs and the kubelet pod-resources socket will be refused — run it as root "
                            "(the chart's gpu-agent securityContext)", self.privileges.get("euid"),
                            ",".join(self.privileges.get("missing") or []) or "-")
        check = getattr(self.podres, "check", None)
        if check is not None and check() == "denied":
            self._denied("podresources")
        self.tel.start()
        self._bdf_index = {normalize_bdf(d.get("bdf", "")): d["index"] for d in self.tel.devices() if d.get("bdf")}
        self.pods.add_event_handler(on_add=lambda p: self._on_pod(None, p), on_update=self._on_pod,
                                    on_delete=self._on_pod_delete)
        self.factory.start()
        self._tasks.append(asyncio.create_task(self._event_loop(), name="agent-gpu-events"))

    async def stop(self) -> None:
        tasks = self._tasks + list(self._publishing.values())
        for t in tasks:
            t.cancel()
        await asyncio.gather(*tasks, return_exceptions=True)
        self._publishing.clear()
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

    def allocatable_bdfs(self) -> Optional[List[str]]:
        """PCI addresses of the GPUs the kubelet's device manager offers for allocation
        (pod-resources ``GetAllocatableResources``), None when unknown."""
        fn = getattr(self.podres, "allocatable", None)
        if fn is None:
            return None
        try:
            return allocatable_ids(fn(), self.gpu_resource)
        except Exception as exc:  # noqa: BLE001 - kubelet socket optional / older kubelet
            log.debug("pod-resources allocatable lookup failed: %s", exc)
            return None

    def evidence(self, pod: Dict[str, Any]) -> Optional[Dict[str, Any]]:
        if kube.admission_rejection(pod) is not None:
            # the kubelet refused the pod before allocating it a GPU: what the supervisor
            # needs is which of this node's GPUs are unhealthy (classify: gpu-admission)
            return admission_evidence(self.tel, pod, node=self.node, lookback=self.lookback,
                                      allocatable_bdfs=self.allocatable_bdfs())
        alloc = self.allocation(pod)
        ev = evidence_for(self.tel, pod_uid=kube.uid_of(pod), gpu_indices=self.gpus_for(pod, alloc),
                          lookback=self.lookback, node=self.node, allocated=alloc)
        logs = self.log_evidence(pod)
        if logs:
            if ev is None:
                ev = {"source": self.tel.name, "t": round(time.time(), 3), "gpus": [], "node": self.node,
                      "pod_uid": kube.uid_of(pod)}
            ev["logs"] = logs
        return ev

    def log_evidence(self, pod: Dict[str, Any]) -> List[Dict[str, Any]]:
        """Allocation-failure lines from the tails of the pod's failed containers' logs."""
        if not self.log_root:
            return []
        try:
            recs = logtail.node_log_evidence(self.log_root, pod, self.log_tail_bytes)
        except Exception as exc:  # noqa: BLE001 - logs are evidence, never a reason to skip the GPU record
            log.debug("log tail of %s failed: %s", kube.name_of(pod), exc)
            return []
        for r in recs:
            if r.get("denied"):
                self._denied("log")
            elif not r.get("error"):
                # agent_log_reads{match}: container log tails read from the node's /var/log/pods
                self.metrics.inc("agent_log_reads", labels={"match": r.get("match") or "none"})
        return recs

    # ------------------------------------------------------------ privileges
    def _warn_once(self, key: str, msg: str, *args) -> None:
        if key not in self._warned:
            self._warned.add(key)
            log.warning(msg, *args)

    def _denied(self, what: str, n: int = 1) -> None:
        """A read the kernel refused: ``log`` (container log tail), ``podresources`` (the
        kubelet socket)."""
        name = {"log": "agent_log_read_denied", "podresources": "agent_podresources_denied"}[what]
        self.metrics.inc(name, n)
        self._warn_once(name, "node agent: %s refused (permission denied) — %s", what,
                        "container log tails come from the pods/log API instead (through the supervisor's "
                        "kube-qps budget)" if what == "log" else
                        "GPU allocations are unknown; devices fall back to the pod's *_VISIBLE_DEVICES env")

    def check_denials(self) -> Dict[str, int]:
        """Fold the native monitor's refused /proc and sysfs reads into
        ``agent_proc_scan_denied{source}``; returns the new ones by source."""
        try:
            cur = self.tel.denials()
        except Exception:  # noqa: BLE001 - diagnostics only
            return {}
        van = self.tel.process_vanished() if hasattr(self.tel, "process_vanished") else 0
        if van > self._vanished_seen:
            # processes that exited while amd-smi listed them (its stderr noise, counted)
            self.metrics.inc("gpu_process_vanished", van - self._vanished_seen)
            self._vanished_seen = van
        new = {}
        for src, n in cur.items():
            d = int(n) - self._denied_seen.get(src, 0)
            if d > 0:
                new[src] = d
                self.metrics.inc("agent_proc_scan_denied", d, labels={"source": src})
            self._denied_seen[src] = int(n)
        if new:
            self._warn_once("agent_proc_scan_denied", "node agent: /proc and sysfs reads refused (permission denied, "
                            "by source: %s) — per-process VRAM and rank env of other users' processes are not "
                            "attributed; run the agent as root", new)
        return new

    # ------------------------------------------------------------ publishing
    async def publish(self, pod: Dict[str, Any], reason: str) -> Optional[bool]:
        """One annotation PATCH; True when it landed, False when it failed, None when there
        is no evidence to publish (no GPU matched, no log read)."""
        ev = self.evidence(pod)
        if ev is None:
            return None
        ev["reason"] = reason
        body = {"metadata": {"annotations": {self.annotation: json.dumps(ev, separators=(",", ":"), sort_keys=True)}}}
        try:
            await self.kube.patch_merge("Pod", kube.namespace_of(pod), kube.name_of(pod), body, want_body=False)
        except Exception as exc:  # noqa: BLE001
            self.patch_failures += 1
            self.metrics.inc("agent_annotation_failures")
            log.warning("annotating pod %s failed: %s", kube.name_of(pod), exc)
            return False
        self.published[kube.uid_of(pod)] = (reason, time.monotonic())
        self.patches += 1
        self.metrics.inc("agent_annotations")
        return True

    async def _publish_with_retry(self, uid: str, key: str, pod: Dict[str, Any], reason: str) -> None:
        """Retry the PATCH with capped exponential backoff while the pod still exists (the
        evidence is rebuilt from the latest cached pod each attempt); the pod's entry is
        dropped when it goes away, so nothing is lost for good to one apiserver 5xx."""
        delay = self.retry_base
        try:
            while True:
                cur = self.pods.indexer.get(key) if key else pod
                if cur is None or kube.uid_of(cur) != uid:
                    self.published.pop(uid, None)
                    return
                ok = await self.publish(cur, reason)
                if ok is None:
                    self.published[uid] = ("no-evidence", time.monotonic())
                    return
                if ok:
                    return
                await asyncio.sleep(delay)
                delay = min(self.retry_max, delay * 2)
        finally:
            self._publishing.pop(uid, None)
            if self.published.get(uid, ("",))[0] == "pending":
                self.published.pop(uid, None)  # cancelled (stop) or gone: nothing is claimed

    def _spawn_publish(self, pod: Dict[str, Any], reason: str) -> None:
        uid = kube.uid_of(pod)
        if uid in self._publishing:
            return
        self.published[uid] = ("pending", time.monotonic())
        self._publishing[uid] = asyncio.ensure_future(
            self._publish_with_retry(uid, kube.object_key(pod), pod, reason))

    def _on_pod(self, old, pod) -> None:
        uid = kube.uid_of(pod)
        if uid in self.published or not pod_failed(pod):
            return
        if kube.annotations_of(pod).get(self.annotation):
            self.published[uid] = ("present", time.monotonic())
            return
        self._spawn_publish(pod, "admission-rejected" if kube.admission_rejection(pod) is not None else "pod-failed")

    def _on_pod_delete(self, pod) -> None:
        uid = kube.uid_of(pod)
        self.published.pop(uid, None)
        t = self._publishing.pop(uid, None)
        if t is not None:
            t.cancel()

    def _prune(self, now: float) -> None:
        """TTL for published entries whose pod deletion was missed (e.g. across a re-list)."""
        if not self.published:
            return
        cutoff = now - self.published_ttl
        for uid, (state, t) in list(self.published.items()):
            if t < cutoff and state != "pending":
                del self.published[uid]

    async def _event_loop(self) -> None:
        next_prune = time.monotonic() + 60.0
        next_check = time.monotonic() + 1.0
        while True:
            await asyncio.sleep(self.event_poll)
            now = time.monotonic()
            if now >= next_prune:
                self._prune(now)
                next_prune = now + 60.0
            if now >= next_check:
                self.check_denials()
                next_check = now + 5.0
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
                    ok = await self.publish(pod, "gpu-fault:" + ",".join(sorted({e["type"] for e in faults})))
                    if ok is False and kube.uid_of(pod) not in self._publishing:
                        self._spawn_publish(pod, "gpu-fault:" + ",".join(sorted({e["type"] for e in faults})))


async def run_agent(cfg, node_name: str) -> None:  # pragma: no cover - process entry
    from ..kube.client import KubeClient, KubeConfig
    from .podresources import SOCKET
    from .telemetry import make_telemetry
    import os

    kc = KubeClient.for_config(cfg)
    tel = make_telemetry("amdsmi" if cfg.gpu.backend == "auto" else cfg.gpu.backend, cfg.gpu.sample_interval)
    if tel is None:
        raise RuntimeError("no GPU telemetry backend on this node")
    pr = PodResourcesClient() if os.path.exists(SOCKET) else None
    sel = f"{cfg.labels.nexus_component_label}={cfg.labels.algorithm_run_value}"
    log_root = os.environ.get("NEXUS_AGENT_LOG_ROOT", logtail.LOG_ROOT)
    agent = NodeAgent(kc, tel, node_name, cfg.resource_namespace, label_selector=sel,
                      annotation=cfg.gpu.evidence_annotation, gpu_resource=cfg.gpu.gpu_resource_name, pod_resources=pr,
                      log_root=log_root if cfg.gpu.log_tail != "off" and os.path.isdir(log_root) else None,
                      log_tail_bytes=cfg.gpu.log_tail_bytes)
    await agent.start()
    sampler = None
    prof_out = os.environ.get("NEXUS_AGENT_PPROF", "")
    if prof_out:  # diagnostics: CPU profile of the agent's loop, written at exit
        from ..obs.pprof import Sampler

        sampler = Sampler(hz=199).start()
    runner = None
    port = int(os.environ.get("NEXUS_AGENT_METRICS_PORT", "0") or 0)
    if port:
        runner = await serve_metrics(agent, port)
    stop = asyncio.Event()
    import signal

    loop = asyncio.get_running_loop()
    for s in (signal.SIGTERM, signal.SIGINT):
        loop.add_signal_handler(s, stop.set)
    await stop.wait()
    if sampler is not None:
        prof = sampler.stop()
        with open(prof_out, "wb") as f:
            f.write(prof.encode_gz())
        with open(prof_out + ".top.txt", "w") as f:
            f.write(prof.top(40))
    if runner is not None:
        await runner.cleanup()
    await agent.stop()
    await kc.close()


async def serve_metrics(agent: NodeAgent, port: int, host: str = "0.0.0.0"):
    """``/metrics`` (Prometheus text) and ``/healthz`` of the node agent."""
    from aiohttp import web

    async def h_metrics(_req):
        agent.check_denials()
        return web.Response(text=agent.metrics.prometheus_text(), content_type="text/plain", charset="utf-8")

    async def h_healthz(_req):
        # ready once the node's pods are listed: a failure before that is seen at the list
        if all(i.has_synced() for i in agent.factory.informers.values()):
            return web.Response(text="ok")
        return web.Response(text="syncing", status=503)

    app = web.Application()
    app.router.add_get("/metrics", h_metrics)
    app.router.add_get("/healthz", h_healthz)
    runner = web.AppRunner(app, access_log=None)
    await runner.setup()
    await web.TCPSite(runner, host, port).start()
    return runner
