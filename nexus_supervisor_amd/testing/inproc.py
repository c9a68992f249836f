"""In-process harness: a supervisor wired to in-memory list/watch sources, a
memory (or any) store and a recording Job client — no sockets.  Used by the
parity suite and as the zero-I/O end of the benchmark."""
from __future__ import annotations

import asyncio
from typing import Any, Dict, Iterable, List, Optional

from ..config.schema import SupervisorConfig
from ..informer import ADDED, InformerFactory, QueueListWatch
from ..kube.errors import NotFound
from ..models.decisions import Decision
from ..obs.logging import KLogger
from ..store.base import CheckpointStore
from ..supervisor import JobClient, Supervisor


class RecordingJobs(JobClient):
    """Job client backed by a set of existing job names; records deletes."""

    def __init__(self, existing: Iterable[str] = (), latency: float = 0.0):
        self.existing = set(existing)
        self.deleted: List[str] = []
        self.latency = latency
        self.fail_next = 0
        self.logs: Dict[Any, bytes] = {}  # (namespace, pod, container) → pods/log text

    async def pod_log(self, namespace, name, container, *, previous=False, tail_lines=200, limit_bytes=65536,
                      timeout=2.0):
        text = self.logs.get((namespace, name, container))
        if text is None:
            return 400, b'{"kind":"Status","code":400}'
        return 200, text[-limit_bytes:]

    async def delete_job(self, namespace, name, propagation_policy="Background"):
        if self.latency:
            await asyncio.sleep(self.latency)
        if self.fail_next:
            self.fail_next -= 1
            raise RuntimeError("injected delete failure")
        self.deleted.append(name)
        if name not in self.existing:
            raise NotFound(404, "NotFound", f'jobs.batch "{name}" not found')
        self.existing.discard(name)


class InProcCluster:
    def __init__(self, cfg: SupervisorConfig, store: CheckpointStore, objects: Iterable[Dict[str, Any]] = (),
                 jobs: Optional[JobClient] = None, logger: Optional[KLogger] = None):
        self.sources: Dict[str, QueueListWatch] = {k: QueueListWatch(k) for k in ("Event", "Pod", "Job")}
        for o in objects:
            self.sources[o["kind"]].items.append(o)
        self.jobs = jobs or RecordingJobs(o["metadata"]["name"] for o in objects if o["kind"] == "Job")
        self.factory = InformerFactory(lambda kind: self.sources[kind], resync_period=0.0)
        self.supervisor = Supervisor(cfg, store, self.jobs, self.factory, logger=logger)
        self.decisions: List[Decision] = []
        self.supervisor.decision_hooks.append(self.decisions.append)

    async def start(self):
        self.supervisor.init()
        await self.supervisor.start(wait_sync_timeout=5)

    def push(self, obj: Dict[str, Any], etype: str = ADDED):
        self.sources[obj["kind"]].push(etype, obj)

    async def settle(self, timeout: float = 5.0) -> bool:
        # let watch queues drain into informers, then wait for the pipeline to go idle
        for _ in range(3):
            for _ in range(50):
                if all(s.queue.empty() for s in self.sources.values()):
                    break
                await asyncio.sleep(0.001)
            await asyncio.sleep(0)
            ok = await self.supervisor.pipeline.join(timeout)
            if not ok:
                return False
            if self.supervisor._deletes:  # background Job DELETEs issued after the writes
                await asyncio.wait(list(self.supervisor._deletes), timeout=timeout)
        return True

    async def stop(self):
        await self.supervisor.stop(drain=True, timeout=2)
