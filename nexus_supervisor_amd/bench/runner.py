"""Per-rank benchmark driver (see ``bench.py``).

Harness protocol: ``start()``, ``step(events) -> (failed run ids, push time)``,
``supervisor``, ``stop()``.  Times are ``time.monotonic()`` (CLOCK_MONOTONIC —
comparable across the rank and cluster processes on one host).
"""
from __future__ import annotations

import asyncio
import gc
import time
from dataclasses import dataclass
from typing import Any, Callable, Dict, List, Optional, Tuple

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
    step_timeout: float = 300.0
    cql_latency_us: int = 0
    pprof_out: str = ""
    kube_connections: int = 256


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
    sc.scylla_cql_store.connections_per_host = 2
    return sc


class Tracker:
    """Decision hook: checkpoint-ack time per run; latency = ack − pod-fail push."""

    def __init__(self):
        self.acks: Dict[str, Tuple[float, str]] = {}
        self.waiting: set = set()
        self.t_push = 0.0
        self.latencies: List[float] = []
        self.errors = 0
        self.done = asyncio.Event()
        self.record = False
        self.stage_sums: Dict[str, float] = {}

    def __call__(self, d: Decision):
        rid = d.result.request_id
        t = time.monotonic()
        self.acks[rid] = (t, d.outcome)
        if rid in self.waiting:
            self._settle(rid, t, d.outcome)

    def _settle(self, rid: str, t: float, outcome: str) -> None:
        self.waiting.discard(rid)
        if outcome != "applied":
            self.errors += 1
        elif self.record:
            self.latencies.append((t - self.t_push) * 1000.0)
        if not self.waiting:
            self.done.set()

    def arm(self, rids: List[str], t_push: float) -> None:
        self.t_push = t_push
        self.waiting = set(rids)
        self.done.clear()
        for rid in rids:
            a = self.acks.get(rid)
            if a is not None:
                self._settle(rid, *a)
        if not self.waiting:
            self.done.set()

    def reset_step(self) -> None:
        self.acks.clear()


class InProcHarness:
    store_name = "memory (in-process)"

    def __init__(self, sc: SupervisorConfig, cfg: BenchConfig):
        from ..store.memory import MemoryStore
        from ..testing.inproc import InProcCluster

        self.wl = Workload(cfg.jobs, rank=cfg.rank, world=cfg.world, seed=cfg.seed,
                           hip_oom_message=cfg.hip_oom_message or DEFAULT_HIP_OOM, shards=cfg.world, shard_index=cfg.rank)
        objs, rows = self.wl.initial()
        self.store = MemoryStore(rows)
        self.cluster = InProcCluster(sc, self.store, objs)
        self.supervisor = self.cluster.supervisor

    async def start(self):
        await self.cluster.start()

    async def step(self, events: int):
        failed, traffic, rows = self.wl.step(events)
        for r in rows:
            self.store.rows[r.key] = r
        t = time.monotonic()
        for etype, obj in traffic:
            self.cluster.push(obj, etype)
        return failed, t

    async def stop(self):
        await self.cluster.stop()


async def run_rank(cfg: BenchConfig, barrier_sync: Callable[[], None]) -> Dict[str, Any]:
    from ..gpu.telemetry import FakeTelemetry, make_telemetry, pod_evidence_provider

    sc = supervisor_config(cfg)
    telemetry = make_telemetry(cfg.telemetry) if cfg.telemetry != "fake" else FakeTelemetry()
    telemetry.start()
    if cfg.transport == "inproc":
        harness = InProcHarness(sc, cfg)
    else:
        from .wire import WireHarness

        harness = WireHarness(sc, cfg, cfg.workdir)
    tracker = Tracker()
    sampler = None
    try:
        await harness.start()
        sup = harness.supervisor
        sup.classifier.evidence_provider = pod_evidence_provider(telemetry)
        sup.decision_hooks.append(tracker)

        async def one_step() -> None:
            tracker.reset_step()
            failed, t_push = await harness.step(cfg.events)
            tracker.arm(failed, t_push)
            try:
                await asyncio.wait_for(tracker.done.wait(), cfg.step_timeout)
            except asyncio.TimeoutError:
                tracker.errors += len(tracker.waiting)
                tracker.waiting.clear()

        for _ in range(cfg.warmup):
            await one_step()
        gc.collect()
        tracker.errors = 0
        tracker.record = True
        if cfg.pprof_out:
            from ..obs.pprof import Sampler

            sampler = Sampler(hz=199).start()
        barrier_sync()
        t0 = time.perf_counter()
        for _ in range(cfg.steps):
            await one_step()
        barrier_sync()
        elapsed = time.perf_counter() - t0
        if sampler is not None:
            prof = sampler.stop()
            sampler = None
            with open(cfg.pprof_out, "wb") as f:
                f.write(prof.encode_gz())
            with open(cfg.pprof_out + ".top.txt", "w") as f:
                f.write(prof.top(40))
        stages = _stage_breakdown(sup)
    finally:
        if sampler is not None:
            sampler.stop()
        await harness.stop()
        telemetry.stop()
    return {"elapsed": elapsed, "events": cfg.events * cfg.steps, "errors": tracker.errors,
            "latencies_ms": tracker.latencies, "store": harness.store_name, "workers": sc.workers,
            "eps": sc.rate_limit_elements_per_second, "telemetry": telemetry.name, "stages": stages}


def _stage_breakdown(sup) -> Dict[str, Any]:
    m = sup.metrics
    out = {}
    for name in ("receive_to_checkpoint",):
        h = m.histogram(name)
        if h is not None:
            out[name] = {k: round(v / 1000.0, 3) for k, v in h.summary().items()}
    return out
