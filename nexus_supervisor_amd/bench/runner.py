"""Per-rank benchmark driver (see ``bench.py``)."""
from __future__ import annotations

import asyncio
import gc
import time
from dataclasses import dataclass
from typing import Any, Callable, Dict, List, Optional

from ..config.schema import SupervisorConfig
from ..models.decisions import Decision
from .workload import DEFAULT_HIP_OOM, Workload


@dataclass
class BenchConfig:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    jobs: int = 10_000
    events: int = 1000
    steps: int = 10
    warmup: int = 2
    transport: str = "wire"
    profile: str = "uncapped"
    workers: int = 256
    seed: int = 0
    hip_oom_message: Optional[str] = None
    telemetry: str = "fake"
    workdir: str = "/tmp"
    step_timeout: float = 120.0


def supervisor_config(cfg: BenchConfig) -> SupervisorConfig:
    sc = SupervisorConfig()
    sc.cql_store_type = "memory"
    sc.resource_namespace = "nexus"
    if cfg.profile == "reference":
        sc.workers, sc.rate_limit_elements_per_second, sc.rate_limit_elements_burst = 2, 10, 100
    else:
        sc.workers, sc.rate_limit_elements_per_second, sc.rate_limit_elements_burst = cfg.workers, 0, 1_000_000
    sc.sharding.shards = cfg.world
    sc.sharding.shard_index = cfg.rank
    sc.resync_period = 0.0
    sc.rules.stale_event_grace = 5.0
    sc.observability.stage_timestamps = True
    return sc


class _Tracker:
    """Decision hook: pod-fail push time → checkpoint ack latency per run."""

    def __init__(self):
        self.pushed: Dict[str, float] = {}
        self.waiting: set = set()
        self.latencies: List[float] = []
        self.errors = 0
        self.done = asyncio.Event()
        self.record = False

    def arm(self, rids: List[str], t: float):
        for r in rids:
            self.pushed[r] = t
        self.waiting = set(rids)
        self.done.clear()

    def __call__(self, d: Decision):
        rid = d.result.request_id
        if rid not in self.waiting:
            return
        t = time.perf_counter()
        self.waiting.discard(rid)
        if d.outcome != "applied":
            self.errors += 1
        elif self.record:
            self.latencies.append((t - self.pushed.pop(rid)) * 1000.0)
        if not self.waiting:
            self.done.set()


async def run_rank(cfg: BenchConfig, barrier_sync: Callable[[], None]) -> Dict[str, Any]:
    from ..gpu.telemetry import FakeTelemetry, make_telemetry, pod_evidence_provider

    sc = supervisor_config(cfg)
    wl = Workload(cfg.jobs, rank=cfg.rank, world=cfg.world, seed=cfg.seed,
                  hip_oom_message=cfg.hip_oom_message or DEFAULT_HIP_OOM, shards=cfg.world, shard_index=cfg.rank)
    objs, rows = wl.initial()
    telemetry = make_telemetry(cfg.telemetry) if cfg.telemetry != "fake" else FakeTelemetry()
    telemetry.start()

    if cfg.transport == "inproc":
        from ..store.memory import MemoryStore
        from ..testing.inproc import InProcCluster

        store = MemoryStore(rows)
        cluster = InProcCluster(sc, store, objs)
        harness = _InProcHarness(cluster, store)
    else:
        from .wire import WireHarness

        harness = WireHarness(sc, objs, rows, cfg.workdir)
    tracker = _Tracker()
    await harness.start()
    sup = harness.supervisor
    sup.classifier.evidence_provider = pod_evidence_provider(telemetry)
    sup.decision_hooks.append(tracker)

    async def one_step() -> None:
        failed, traffic, new_rows = wl.step(cfg.events)
        await harness.add_rows(new_rows)
        tracker.arm(failed, time.perf_counter())
        await harness.push(traffic)
        try:
            await asyncio.wait_for(tracker.done.wait(), cfg.step_timeout)
        except asyncio.TimeoutError:
            tracker.errors += len(tracker.waiting)
            tracker.waiting.clear()

    try:
        for _ in range(cfg.warmup):
            await one_step()
        gc.collect()
        tracker.errors = 0
        tracker.record = True
        barrier_sync()
        t0 = time.perf_counter()
        for _ in range(cfg.steps):
            await one_step()
        barrier_sync()
        elapsed = time.perf_counter() - t0
    finally:
        await harness.stop()
        telemetry.stop()
    return {"elapsed": elapsed, "events": cfg.events * cfg.steps, "errors": tracker.errors,
            "latencies_ms": tracker.latencies, "store": harness.store_name, "workers": sc.workers,
            "eps": sc.rate_limit_elements_per_second, "telemetry": telemetry.name}


class _InProcHarness:
    store_name = "memory"

    def __init__(self, cluster, store):
        self.cluster = cluster
        self.store = store
        self.supervisor = cluster.supervisor

    async def start(self):
        await self.cluster.start()

    async def add_rows(self, rows):
        for r in rows:
            self.store.rows[r.key] = r

    async def push(self, traffic):
        for etype, obj in traffic:
            self.cluster.push(obj, etype)

    async def stop(self):
        await self.cluster.stop()
