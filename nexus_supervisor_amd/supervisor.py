"""The supervisor domain service: informers → classify → keyed pipeline → actuate.

Parity map to ``/root/reference/services/supervisor.go``:

==========================  ===================================================
reference                   here
==========================  ===================================================
``NewSupervisor`` :69-103   :class:`Supervisor` ``__init__`` (namespaced factory,
                            Event/Pod/Job informers, injectable sync predicate)
``Init`` :106-135           :meth:`Supervisor.init` (pipeline + handlers)
``onEvent`` :137-259        :meth:`Supervisor._on_event_add` → :class:`Classifier`
``superviseAction`` :261    :meth:`Supervisor.supervise_action`
``Start`` :376-388          :meth:`Supervisor.start` (workers, then informers +
                            cache sync as the post-start hook)
==========================  ===================================================

Beyond the reference: pod/job status rules, Event Update handling (repeat
counts), parking of events whose object is not cached yet, per-run-key
serialization, NotFound-tolerant deletes, owned-columns writes, a
decided-stage cache that suppresses duplicate work, sharding/leader gating and
per-stage timestamps for the pod-fail → checkpoint latency metric.
"""
from __future__ import annotations

import asyncio
import datetime as _dt
import functools
import time
from collections import OrderedDict
from typing import Any, Callable, Dict, List, Optional, Tuple

from .classify import DECIDED, STALE, Classifier, ObjectLookup, render_trace
from .classify import reference_rules as R
from .config.schema import SupervisorConfig
from .informer import InformerFactory, label_index
from .kube.errors import NotFound
from .models import kube
from .models import checkpoint as _cp
from .models.checkpoint import LifecycleStage
from .gpu.telemetry import FAULT_EVENTS
from .models.decisions import Decision, DecisionAction as A, RunStatusAnalysisResult
from .models.decisions import FailureClass as F
from .obs.logging import KLogger
from .obs.metrics import Metrics
from .parallel.pipeline import PipelineStage
from .parallel.sharding import ShardSet
from .obs.delivery import CURRENT as _DELIVERY
from .store.base import CheckpointStore, NotSent, is_availability_error
from .utils.gctune import GcTuner

STAGE_FOR_ACTION = {
    A.TO_FAIL_STUCK_IN_PENDING: lambda: LifecycleStage.SCHEDULING_FAILED,
    A.TO_FAIL_FATAL_ERROR: lambda: LifecycleStage.FAILED,
    A.TO_FAIL_DEADLINE_EXCEEDED: lambda: LifecycleStage.DEADLINE_EXCEEDED,
    A.TO_RUNNING: lambda: LifecycleStage.RUNNING,
}


_GPU_CLASSES = frozenset((F.HBM_OOM, F.GPU_FAULT, F.COLLECTIVE, F.GPU_ADMISSION))
# Job event / condition reasons that imply one of the Job's pods has already failed
_POD_FAILED_REASONS = frozenset(("BackoffLimitExceeded", "PodFailurePolicy"))


def _pod_failed(pod) -> bool:
    """The pod shows a failure: phase Failed, evicted, or a container terminated non-zero."""
    st = pod.get("status") or {}
    if st.get("phase") == "Failed" or st.get("reason") == "Evicted":
        return True
    for t in kube.terminated_states(pod):
        if t.get("exitCode") not in (None, 0) or t.get("reason") == "OOMKilled":
            return True
    return False


def failed_gpu(r: RunStatusAnalysisResult) -> Tuple[str, Optional[Any]]:
    """(node, physical GPU index) a GPU-class decision is attributed to, best evidence
    first: the OOM verdict's GPU, a GPU with fault events in the node agent's evidence,
    then the rank's expected device (physical once the agent reported the allocation)."""
    ev = r.evidence
    topo = ev.get("topology") or {}
    gev = ev.get("gpu") or {}
    node = topo.get("node") or gev.get("node") or (ev.get("admission") or {}).get("node") or ""
    health = gev.get("node_health")
    if health is not None:
        # refused at kubelet admission: no GPU was allocated — the one unhealthy GPU of the
        # node, when the node agent's health record names exactly one
        bad = health.get("unhealthy") or ()
        return node, bad[0].get("index") if len(bad) == 1 else None
    oom = ev.get("oom") or {}
    if oom.get("gpu_index") is not None:
        return node, oom["gpu_index"]
    for g in gev.get("gpus") or ():
        if any(e.get("type") in FAULT_EVENTS for e in g.get("events") or ()):
            return node, g.get("index")
    return node, topo.get("expected_gpu")


def _wake(waiter: asyncio.Future, *_args) -> None:
    if not waiter.done():
        waiter.set_result(None)


def _consume_exception(fut: asyncio.Future) -> None:
    """A prefetched read that failed or was dropped: the decision reads on its own."""
    if not fut.cancelled():
        fut.exception()


def running_fused_actuation(cfg: SupervisorConfig) -> bool:
    """Is a ``ToRunning`` decision ONE conditional write (no read first)?  Whenever its write
    is conditional anyway (``compat.conditional-update`` auto / always) and the write is the
    owned-columns UPDATE (the full-row upsert needs the row read)."""
    c = cfg.compat
    return not c.full_row_upsert and c.conditional_update != "never"


def fused_actuation(cfg: SupervisorConfig) -> bool:
    """Is a decision ONE conditional write (``compat.fused-write``)?  ``auto``: only when
    a deposed owner may still hold decisions — leader election or shard leases — where
    the LWT's atomic stage check is what keeps a finished row final; a lone replica takes
    the reference's cheaper read + plain write (an LWT is a Paxos round)."""
    c = cfg.compat
    if c.full_row_upsert or c.conditional_update == "never":
        return False
    if c.fused_write == "true":
        return True
    if c.fused_write == "false":
        return False
    return cfg.leader_election.enabled or cfg.sharding.mode == "lease"


def _FAILED_STAGES():
    return (LifecycleStage.FAILED, LifecycleStage.SCHEDULING_FAILED, LifecycleStage.DEADLINE_EXCEEDED)


class JobClient:
    """What the actuator needs from the K8s API."""

    async def delete_job(self, namespace: str, name: str, propagation_policy: str = "Background") -> None:  # pragma: no cover
        raise NotImplementedError


class CasConflict(Exception):
    """Conditional write lost a race; the item is retried (re-read + re-decide)."""


class Fenced(Exception):
    """This replica lost its lease (or its shard) after the decision was dequeued."""


def parse_k8s_time(ts: Optional[str]) -> Optional[float]:
    """RFC3339 / MicroTime → epoch seconds."""
    if not ts:
        return None
    try:
        if ts.endswith("Z"):
            ts = ts[:-1] + "+00:00"
        return _dt.datetime.fromisoformat(ts).timestamp()
    except ValueError:
        return None


class _Lookup(ObjectLookup):
    __slots__ = ("sup",)

    def __init__(self, sup: "Supervisor"):
        self.sup = sup

    def get(self, kind, name):
        inf = self.sup.pod_informer if kind == "Pod" else self.sup.job_informer if kind == "Job" else None
        if inf is None:
            return None
        return inf.indexer.get_by_name(self.sup.namespace, name)

    def pods_of_job(self, job_name):
        return self.sup.pod_informer.indexer.by_index("job-name", job_name)


class _StageHists:
    """The unlabelled stage histograms of :meth:`Supervisor._observe`, each created on its
    first sample (fused mode never has a ``stage_read``)."""

    __slots__ = ("_m", "_names", "_h")

    def __init__(self, metrics: Metrics, names: Tuple[str, ...]):
        self._m = metrics
        self._names = names
        self._h: List[Any] = [None] * len(names)

    def rec(self, i: int, seconds: float) -> None:
        h = self._h[i]
        if h is None:
            h = self._h[i] = self._m.hist0(self._names[i])
        h.record(seconds * 1e6)


class Supervisor:
    def __init__(
        self,
        cfg: SupervisorConfig,
        store: CheckpointStore,
        jobs: JobClient,
        factory: InformerFactory,
        logger: Optional[KLogger] = None,
        metrics: Optional[Metrics] = None,
        sync_state: Optional[Callable[[], bool]] = None,
        wall: Callable[[], float] = time.time,
    ):
        self.cfg = cfg
        cfg.stages.apply()  # process-wide stage strings / finished set (stages: section)
        self.namespace = cfg.resource_namespace
        self.store = store
        self.jobs = jobs
        self.factory = factory
        self.log = logger or KLogger()
        self.metrics = metrics or Metrics(cfg.observability.statsd_name)
        self.wall = wall
        self.sync_state = sync_state
        self.classifier = Classifier(cfg.labels, cfg.rules, cfg.gpu)
        self.classifier.lazy_enrich = True  # enriched in supervise_action (finish), once per written decision
        self.event_informer = factory.informer("Event")
        self.pod_informer = factory.informer("Pod", indexers={"job-name": label_index(cfg.labels.job_name_label)})
        self.job_informer = factory.informer("Job")
        self.lookup = _Lookup(self)
        self.pipeline: Optional[PipelineStage] = None
        self.breaker = None  # store circuit breaker (init)
        self._event_tasks: set = set()  # observability.record-events posts in flight
        self._applied: "OrderedDict[Tuple[str, str], str]" = OrderedDict()
        self._applied_cap = 200_000
        self._hists: Optional["_StageHists"] = None  # _observe: the stage histograms, once looked up
        # one conditional write per decision instead of read + write (compat.fused-write);
        # conditional-update: never (the reference's unconditional writes) turns it off
        self._fused = fused_actuation(cfg)
        # ToRunning is a conditional write whenever conditional-update is not "never": its
        # not-applied answer already says "no row" / "finished" / "already RUNNING", so the
        # reference's read before it (supervisor.go:264) is one round trip that decides
        # nothing — the one-call path serves it even when failures take the read + write
        self._fused_running = self._fused or (running_fused_actuation(cfg))
        self._guards: Dict[Any, Any] = {}
        self._parked: Dict[Tuple[str, str], List[Tuple[float, Dict[str, Any], float]]] = {}
        self._gpu_wait: Dict[str, float] = {}  # pod key -> deadline (waiting for node-agent GPU evidence)
        # pod key -> a Job decision waiting for that pod's GPU evidence wait to end
        self._gpu_waiters: Dict[str, asyncio.Future] = {}
        self._log_fetches: Dict[str, asyncio.Future] = {}  # pod key -> in-flight pods/log tail fetch
        # run -> checkpoint stage read started while its deferred GPU failure waits (for its
        # log tail or the node agent's evidence): the decision that follows takes it instead
        # of a round trip of its own (two-step owned-columns actuation only)
        self._prefetch: "OrderedDict[Tuple[str, str], Tuple[asyncio.Future, float]]" = OrderedDict()
        self._prefetch_reads = not self._fused and not cfg.compat.full_row_upsert
        # a prefetched read is taken only by a decision that follows its wait: one that
        # outlived the longest wait it can overlap (a deferral that decided nothing) is
        # dropped, never used for a later decision of the run
        self._prefetch_ttl = max(cfg.gpu.log_tail_timeout, cfg.gpu.evidence_wait) + 2.0
        self._settle: Dict[str, asyncio.Future] = {}  # job name -> a Job decision waiting for its pod's failure
        # shards whose cached pods may be stale while the Pod informer re-lists (set when the list is in)
        self._pod_relist: Optional[Tuple[asyncio.Event, frozenset]] = None
        self._settle_wait = float(cfg.rules.job_pod_settle)
        self._job_label = cfg.labels.job_name_label
        # pod key -> (first receive, watch-batch delivery stamps) of a deferred pod failure:
        # its decision's stages start where the failure arrived, not at the re-classification
        self._deferred_at: Dict[str, Tuple[float, Any]] = {}
        self._log_sem: Optional[asyncio.Semaphore] = None  # gpu.log-tail-concurrency
        self._log_inflight = 0
        self.log_tail_inflight_max = 0
        g = cfg.gpu
        self._log_fetch = (g.attribution_enabled and g.log_tail in ("auto", "api")
                           and callable(getattr(jobs, "pod_log", None)))
        self._deletes: Dict[Any, str] = {}  # in-flight asynchronous Job DELETEs → request id
        self._bg: set = set()  # housekeeping tasks (post-re-list replays)
        self._sweeper: Optional[asyncio.Task] = None
        self.decision_hooks: List[Callable[[Decision], None]] = []
        # leader gating flips this; with shard leases ownership is per shard (self.shards)
        self.active = not cfg.leader_election.enabled or cfg.sharding.mode == "lease"
        # fencing epoch: bumped on every loss of leadership; a decision dequeued under an
        # older epoch never writes or deletes (see set_active)
        self.epoch = 0
        # leader lease hold deadline (CLOCK_MONOTONIC seconds, LeaderElector.valid_until):
        # past it this replica acts on nothing, even before the elector's step-down lands
        self.active_until = float("inf")
        self._label_check_at = 0.0
        self.label_mismatch = False
        self._unfinished_cache: Optional[Tuple[str, ...]] = None
        self.gc_tuner = GcTuner.from_config(cfg.runtime, self.metrics)
        # replica shards owned right now (sharding.*), with a fencing epoch per shard
        self.shards = ShardSet.from_config(cfg)
        self.worker_shard = None
        self.hub_fed = all(type(i.lw).__name__ == "HubListWatch"
                           for i in (self.event_informer, self.pod_informer, self.job_informer))
        if cfg.runtime.worker_processes > 1 or self.shards.enabled:
            from .parallel.workers import WorkerShard

            self.worker_shard = WorkerShard(cfg.runtime.worker_index, cfg.runtime.worker_processes,
                                            cfg.labels.job_name_label, shards=self.shards)
            self.worker_shard.install(self, routed_upstream=self.hub_fed)
        m = self.metrics
        m.describe("event_to_checkpoint", "Latency from K8s event creation to checkpoint write ack")
        m.describe("receive_to_checkpoint", "Latency from watch receive to checkpoint write ack")
        m.describe("stage_classify", "Watch receive to pipeline enqueue (classification)")
        m.describe("stage_hub", "Watch hub read of the API chunk to the shard worker's frame read")
        m.describe("stage_feed", "Shard worker frame read to decoded batch (queue wait + native decode)")
        m.describe("stage_dispatch", "Decoded batch to the supervisor's handler (informer dispatch)")
        m.describe("stage_queue", "Pipeline enqueue to worker dequeue (rate limit + queueing)")
        m.describe("stage_read", "Checkpoint read round trip (read + write actuation)")
        m.describe("stage_prepare", "Dequeue to conditional write sent: enrichment + trace (fused actuation)")
        m.describe("stage_write", "Checkpoint write round trip (fused: the conditional write)")
        m.describe("stage_delete", "Checkpoint ack to Job DELETE accepted")

    # ------------------------------------------------------------------ Init
    def init(self) -> None:
        c = self.cfg
        cb = c.circuit_breaker
        self.breaker = None
        processor = self.supervise_action
        if cb.enabled:
            from .parallel.breaker import CircuitBreaker

            self.breaker = CircuitBreaker(cb.failure_threshold, cb.open_duration, cb.max_open_duration, self.metrics)
            processor = self._guarded_action
        self.pipeline = PipelineStage(
            "supervisor",
            processor,
            gate=self.breaker,
            workers=c.workers,
            elements_per_second=c.rate_limit_elements_per_second,
            burst=c.rate_limit_elements_burst,
            base_delay=c.failure_rate_base_delay,
            max_delay=c.failure_rate_max_delay,
            max_retries=c.max_retries,
            key_fn=lambda r: (r.algorithm, r.request_id),
            coalesce_key=lambda r: r.action,
            on_dead_letter=self._dead_letter,
            on_done=self._done,
            tags={},
        )
        self.event_informer.add_event_handler(on_add=self._on_event_add, on_update=self._on_event_update)
        self.pod_informer.add_event_handler(on_add=self._on_pod_add, on_update=self._on_pod_update)
        self.job_informer.add_event_handler(on_add=self._on_job_add, on_update=self._on_job_update)

    # ------------------------------------------------------------------ Start / stop
    async def start(self, wait_sync_timeout: Optional[float] = None) -> None:
        if self.pipeline is None:
            self.init()

        async def post_start():
            self.factory.start()
            if self.sync_state is not None:
                ok = self.sync_state()
            else:
                ok = await self.factory.wait_for_cache_sync(wait_sync_timeout)
            if not ok:
                raise RuntimeError("failed to wait for pod informer caches to sync")
            self.log.info("resource informers synced")
            self.gc_tuner.after_sync()
            if self.cfg.rules.running_sweep_rate > 0:
                t = asyncio.ensure_future(self._running_sweep())
                self._bg.add(t)
                t.add_done_callback(self._bg.discard)

        await self.pipeline.start(post_start)
        self._sweeper = asyncio.create_task(self._sweep_parked(), name="stale-event-sweeper")

    async def _running_sweep(self) -> None:
        """After a restart, a run whose Started Event expired while the supervisor was down
        (the API server keeps Events about an hour) and whose pod was already running at the
        initial LIST would never be moved to RUNNING: the pod-status backup rule fires only
        on a transition to Running.  Once, ``rules.running-sweep-delay`` after the caches
        synced, every running Nexus pod of this replica with no Started Event in the Event
        cache gets a ``ToRunning`` decision — at most ``running-sweep-rate`` a second and
        only while no decision is queued, so a failure backlog is never held up.  A row
        already RUNNING or finished costs a read (the conditional ToRunning writes nothing)."""
        r = self.cfg.rules
        await asyncio.sleep(r.running_sweep_delay)
        started = set()
        for ev in list(self.event_informer.indexer.values()):
            if ev.get("reason") == "Started":
                inv = ev.get("involvedObject") or {}
                if inv.get("kind") == "Pod":
                    started.add(inv.get("name", ""))
        keys = [kube.object_key(p) for p in list(self.pod_informer.indexer.values())
                if kube.name_of(p) not in started and (p.get("status") or {}).get("phase") == "Running"]
        interval = 1.0 / r.running_sweep_rate
        n = 0
        for key in keys:
            while self.pipeline.busy():
                await asyncio.sleep(interval)
            pod = self.pod_informer.indexer.get(key)
            if pod is None or not self.active:
                continue
            res = self.classifier.running_result(pod)
            if res is None:
                continue
            now = self.wall()
            self._submit(res, now, now, "Pod")
            n += 1
            self.metrics.inc("running_sweep_decisions")
            await asyncio.sleep(interval)
        if n:
            self.log.info("running sweep: runs without a Started Event re-checked", runs=n)

    async def stop(self, drain: bool = True, timeout: float = 10.0) -> None:
        self.gc_tuner.stop()
        for t in list(self._bg) + list(self._log_fetches.values()):
            t.cancel()
        if self._sweeper:
            self._sweeper.cancel()
            try:
                await self._sweeper
            except (asyncio.CancelledError, Exception):
                pass
        await self.factory.stop()
        if self.pipeline is not None:
            await self.pipeline.stop(drain=drain, timeout=timeout)
        if self._deletes:
            pending = list(self._deletes)
            if drain:
                await asyncio.wait(pending, timeout=timeout)
            for t in pending:
                t.cancel()
            await asyncio.gather(*pending, return_exceptions=True)
        if self._event_tasks:  # decision Events still being posted (best effort, short)
            pending = list(self._event_tasks)
            await asyncio.wait(pending, timeout=min(timeout, 2.0))
            for t in pending:
                t.cancel()
            await asyncio.gather(*pending, return_exceptions=True)

    def set_active(self, active: bool) -> None:
        """Leader gating.  On gaining leadership replay the caches (idempotent) so nothing
        decided while standby is lost (SURVEY §5.3 'replay on restart').  On losing it,
        *fence*: bump the epoch (in-flight decisions check it right before their write
        and their Job DELETE), drop every queued and backing-off decision, cancel the
        background DELETEs and forget the decided-stage cache — the new leader owns those
        runs now, and a deposed leader must not race it.  The conditional write
        (``compat.conditional-update``) covers a write already on the wire."""
        was = self.active
        self.active = active
        if active and not was:
            self.replay()
        elif was and not active:
            self.fence()

    def fence(self) -> int:
        self.epoch += 1
        dropped = self.pipeline.clear() if self.pipeline is not None else 0
        for t in list(self._deletes):
            t.cancel()
        self._deletes.clear()
        self._gpu_wait.clear()
        for key in list(self._gpu_waiters):
            self._gpu_wait_over(key)
        self._parked.clear()
        self._applied.clear()
        self._drop_prefetch(lambda rid: True)
        self.metrics.inc("fenced_decisions_dropped", dropped)
        self.metrics.inc("fencings")
        self.log.info("leadership lost: fenced in-flight work", dropped=dropped, epoch=self.epoch)
        return dropped

    def _token(self, request_id: str) -> Tuple[int, int]:
        """Fencing token of a run: the replica epoch and its shard's epoch."""
        return self.epoch, self.shards.token(request_id)

    def _fenced(self, token: Tuple[int, int], request_id: str) -> bool:
        """True when this replica must not write or delete for ``request_id``: leadership or
        the run's shard lost since the decision was dequeued (epoch), not held now, or the
        lease's hold lapsed (time-bounded: a stalled apiserver cannot extend it)."""
        if not self.active or token[0] != self.epoch or time.monotonic() >= self.active_until:
            return True
        sh = self.shards
        if sh.owned is None:  # unsharded: the shard epoch is constant
            return False
        return token[1] != sh.token(request_id) or not sh.owns(request_id)

    def set_lease_deadline(self, until: float) -> None:
        self.active_until = until

    def _narrow_watches(self) -> bool:
        """``sharding.shard-label``: point the Pod/Job watches at the shards owned now (the
        caller re-lists); False when the watches are not this process's to narrow."""
        if not self.cfg.sharding.shard_label or self.hub_fed:
            return False
        from .parallel.sharding import watch_selector

        changed = False
        for kind, inf in (("Pod", self.pod_informer), ("Job", self.job_informer)):
            lw = getattr(inf, "lw", None)
            if lw is not None and hasattr(lw, "label_selector"):
                lw.label_selector = watch_selector(self.cfg, kind, self.shards.owned)
                changed = True
        return changed

    def set_shards(self, owned) -> Tuple[frozenset, frozenset]:
        """New owned replica-shard set (lease mode: a shard lease won or lost).  Lost shards
        are fenced like a lost leadership, but only for their runs: their queued and
        backing-off decisions are dropped, their background DELETEs cancelled and their
        objects purged from the caches (so a later regain re-adds them).  Gained shards
        are replayed from whatever the caches hold, and informers that filter at ingest
        re-list to pick up the runs they used to drop (the watch hub re-lists upstream)."""
        gained, lost = self.shards.update(owned)
        if self.worker_shard is not None:
            self.worker_shard.sync_replica()
        if lost:
            self.fence_shards(lost)
            if not gained and self._narrow_watches():
                before = self.pod_informer.relists
                for inf in (self.pod_informer, self.job_informer):
                    inf.relist()  # stop receiving the lost shards' objects
                self._pod_list_pending(self.shards.owned or (), before)
        if gained:
            self.metrics.inc("shards_gained", len(gained))
            self.replay(lambda rid: self.shards.of(rid) in gained)
            infs = (self.event_informer, self.pod_informer, self.job_informer)
            before = [inf.relists for inf in infs]
            narrowed = self._narrow_watches()
            relisted = False
            if self.worker_shard is not None and not self.hub_fed:
                for inf in infs:
                    inf.relist()
                relisted = True
            elif narrowed:
                for inf in (self.pod_informer, self.job_informer):
                    inf.relist()
                relisted = True
            # the pod informer's own re-list takes its watch down for every shard it holds;
            # the hub's upstream re-list only concerns the gained ones
            relist = self._pod_list_pending(self.shards.owned if relisted else gained, None)
            # the three kinds re-list independently: an Event of a gained run can be applied
            # before its Job and parked; replay the gained shards once more after every
            # informer took its new list (or the hub's fresh snapshot), so no ordering of
            # the re-lists can strand a decision
            t = asyncio.ensure_future(self._replay_after_relist(infs, before, gained, relist))
            self._bg.add(t)
            t.add_done_callback(self._bg.discard)
        self.metrics.set("shards_owned", float(len(self.shards.owned or ())))
        if gained or lost:
            self.log.info("replica shards changed", owned=sorted(self.shards.owned or ()), gained=sorted(gained),
                          lost=sorted(lost))
        return gained, lost

    def _pod_list_pending(self, shards, before: Optional[int]):
        """The pod list of ``shards`` is being re-taken: until it lands, a cached pod of
        theirs may be as old as this call (the pod watch is down while its informer
        re-lists), so :meth:`_await_pod_failure` waits for the list instead of the settle
        time alone.  ``before``: the pod informer's re-list count now, to clear the mark by
        itself (else :meth:`_replay_after_relist` does)."""
        prev = self._pod_relist
        keep = prev[1] if prev is not None and not prev[0].is_set() else frozenset()
        # an older mark's waiters are released by its own watcher: the re-list that replaced
        # its list bumps the same counter when it lands
        relist = self._pod_relist = (asyncio.Event(), frozenset(shards or ()) | keep)
        if before is not None:
            t = asyncio.ensure_future(self._pod_list_landed(relist, before))
            self._bg.add(t)
            t.add_done_callback(self._bg.discard)
        return relist

    async def _pod_list_landed(self, relist, before: int, timeout: float = 30.0) -> None:
        deadline = time.monotonic() + timeout
        while self.pod_informer.relists == before and time.monotonic() < deadline:
            await asyncio.sleep(0.05)
        self._end_pod_relist(relist)

    def _end_pod_relist(self, relist) -> None:
        relist[0].set()
        if self._pod_relist is relist:
            self._pod_relist = None

    async def _replay_after_relist(self, infs, before, gained, relist=None, timeout: float = 30.0) -> None:
        deadline = time.monotonic() + timeout
        while any(inf.relists == b for inf, b in zip(infs, before)) and time.monotonic() < deadline:
            if relist is not None and infs[1].relists != before[1] and not relist[0].is_set():
                self._end_pod_relist(relist)  # the pods are in
            await asyncio.sleep(0.05)
        if relist is not None:
            self._end_pod_relist(relist)
        owned = self.shards.owned or frozenset()
        still = frozenset(gained) & owned
        if still and self.active:
            self.metrics.inc("shard_replays")
            self.replay(lambda rid: self.shards.of(rid) in still)

    def fence_shards(self, lost) -> int:
        of = self.shards.of
        dropped = self.pipeline.clear(lambda key: of(key[1]) in lost) if self.pipeline is not None else 0
        for t, rid in list(self._deletes.items()):
            if of(rid) in lost:
                t.cancel()
                self._deletes.pop(t, None)
        for key in [k for k in self._applied if of(k[1]) in lost]:
            del self._applied[key]
        self._drop_prefetch(lambda rid: of(rid) in lost)
        self._purge(lambda rid: of(rid) in lost)
        self.metrics.inc("fenced_decisions_dropped", dropped)
        self.metrics.inc("shards_lost", len(lost))
        return dropped

    def _purge(self, lost_run: Callable[[str], bool]) -> None:
        """Forget cached objects of runs this replica no longer owns (no handlers fire)."""
        label = self.cfg.labels.job_name_label
        ns = self.namespace
        lost_pods = set()
        for pod in list(self.pod_informer.indexer.values()):
            rid = ((pod.get("metadata") or {}).get("labels") or {}).get(label)
            if rid and lost_run(rid):
                lost_pods.add(kube.name_of(pod))
                self.pod_informer.indexer.delete(pod)
        for job in list(self.job_informer.indexer.values()):
            if lost_run(kube.name_of(job)):
                self.job_informer.indexer.delete(job)
        for ev in list(self.event_informer.indexer.values()):
            inv = ev.get("involvedObject") or {}
            if (inv.get("kind") == "Job" and lost_run(inv.get("name", ""))) or \
                    (inv.get("kind") == "Pod" and inv.get("name") in lost_pods):
                self.event_informer.indexer.delete(ev)
        for key in [k for k in self._parked if k[0] == "Job" and lost_run(k[1])]:
            del self._parked[key]
        for key in [k for k in self._gpu_wait if self._gpu_wait_run(k, ns, lost_run)]:
            del self._gpu_wait[key]
            self._gpu_wait_over(key)

    def _gpu_wait_run(self, key, ns, lost_run) -> bool:
        pod = self.pod_informer.indexer.get(key)
        rid = ((pod or {}).get("metadata") or {}).get("labels", {}).get(self.cfg.labels.job_name_label) if pod else None
        return pod is None or (rid is not None and lost_run(rid))

    def replay(self, run_filter: Optional[Callable[[str], bool]] = None) -> None:
        """Re-decide every cached object (``run_filter``: only runs it accepts)."""
        if run_filter is None:
            for ev in list(self.event_informer.indexer.values()):
                self._on_event_add(ev)
            for job in list(self.job_informer.indexer.values()):
                self._on_job_add(job)
            for pod in list(self.pod_informer.indexer.values()):
                self._on_pod_add(pod)
            return
        label = self.cfg.labels.job_name_label
        for ev in list(self.event_informer.indexer.values()):
            inv = ev.get("involvedObject") or {}
            name = inv.get("name", "")
            if inv.get("kind") == "Pod":
                pod = self.pod_informer.indexer.get_by_name(self.namespace, name)
                name = ((pod or {}).get("metadata") or {}).get("labels", {}).get(label, "") if pod else ""
            if name and run_filter(name):
                self._on_event_add(ev)
        for job in list(self.job_informer.indexer.values()):
            if run_filter(kube.name_of(job)):
                self._on_job_add(job)
        for pod in list(self.pod_informer.indexer.values()):
            rid = ((pod.get("metadata") or {}).get("labels") or {}).get(label)
            if rid and run_filter(rid):
                self._on_pod_add(pod)

    # ------------------------------------------------------------------ ownership
    def owns(self, key: Tuple[str, str]) -> bool:
        ws = self.worker_shard
        if ws is not None and ws.count > 1 and ws.of(key[1]) != ws.index:
            return False
        return self.shards.owns(key[1])

    # ------------------------------------------------------------------ handlers
    def _on_event_add(self, ev: Dict[str, Any]) -> None:
        recv = self.wall()
        if self.log.enabled(4):
            self.log.v(4).info("event received", object=kube.object_key(ev), reason=ev.get("reason"))
        self.metrics.inc("events_received")
        if not self.active:
            return
        status, results = self.classifier.classify_event(ev, self.lookup)
        if status == STALE:
            self._park(ev, recv)
            return
        if status != DECIDED:
            if status == "noop":
                self.log.v(1).info("no-op event, ignoring", reason=ev.get("reason"), message=ev.get("message"))
            return
        origin = parse_k8s_time(ev.get("eventTime")) or parse_k8s_time(ev.get("lastTimestamp")) or recv
        for r in results:
            if r.action != A.TO_RUNNING:
                self.log.info("Algorithm run failed", requestId=r.request_id, algorithm=r.algorithm, reason=r.reason,
                              message=r.run_status_trace)
            self._submit(r, origin, recv, "Event")

    def _on_event_update(self, old: Dict[str, Any], new: Dict[str, Any]) -> None:
        if not self.cfg.rules.handle_event_updates or old is new:
            return
        if kube.resource_version(old) == kube.resource_version(new):
            return
        if old.get("count") == new.get("count") and old.get("reason") == new.get("reason") and old.get("series") == new.get("series"):
            return
        self._on_event_add(new)

    def _on_pod_add(self, pod):
        if self._parked:
            self._unpark("Pod", kube.name_of(pod))
        self._on_pod_update(None, pod)

    def _on_pod_update(self, old, pod, waited: bool = False):
        if not self.active or old is pod:
            return
        if self._settle:
            fut = self._settle.pop(((pod.get("metadata") or {}).get("labels") or {}).get(self._job_label), None)
            if fut is not None and not fut.done():
                fut.set_result(None)
        st = pod.get("status")
        if (not self._gpu_wait and (not st or not (st.get("containerStatuses") or st.get("initContainerStatuses")
                                                   or st.get("conditions") or st.get("phase") == "Failed"))):
            return  # a new (pending, unscheduled) pod: no pod-status rule can match it yet
        recv = self.wall()
        wait = self.cfg.gpu.evidence_wait
        results = self.classifier.classify_pod(pod, old, allow_wait=wait > 0 and not waited,
                                               allow_log_fetch=self._log_fetch)
        if not results and not self._gpu_wait and not self.classifier.deferred:
            return  # the common case (a new or unchanged pod): nothing to submit or un-defer
        key = kube.object_key(pod)
        if self.classifier.deferred:
            if key not in self._deferred_at:
                if len(self._deferred_at) >= 4096:  # a deferred pod deleted before its decision
                    del self._deferred_at[next(iter(self._deferred_at))]
                self._deferred_at[key] = (recv, _DELIVERY.get("Pod"))
            if self.classifier.deferred_log:
                # failed GPU container, empty termination message: its OOM text (if any) is in
                # the container log — fetch the tail, then decide (gpu.log-tail)
                if self._gpu_wait.pop(key, None) is not None:
                    self._gpu_wait_over(key)
                self._start_log_fetch(key, pod, self.classifier.deferred_log, waited)
                return
            # failed GPU pod without node-agent evidence yet: give the annotation time to land
            if key not in self._gpu_wait:
                self._gpu_wait[key] = time.monotonic() + wait
                self.metrics.inc("decisions_deferred_for_gpu_evidence")
                if self._prefetch_reads:
                    self._prefetch_read(pod)
            return
        if self._gpu_wait.pop(key, None) is not None and self._gpu_waiters:
            self._gpu_wait_over(key)
        first = self._deferred_at.pop(key, None) if self._deferred_at else None
        if first is not None:
            recv, delivery = first
            for r in results:
                self._submit(r, recv, recv, "Pod", delivery)
            return
        for r in results:
            self._submit(r, recv, recv, "Pod")

    def _start_log_fetch(self, key: str, pod: Dict[str, Any], want: List[Dict[str, Any]], waited: bool) -> None:
        if key in self._log_fetches:
            return
        self.metrics.inc("decisions_deferred_for_log_tail")
        t = asyncio.ensure_future(self._fetch_log_tail(key, pod, want, waited))
        self._log_fetches[key] = t
        if self._prefetch_reads:
            self._prefetch_read(pod)

    def _prefetch_read(self, pod: Dict[str, Any]) -> None:
        """Start the checkpoint stage read of a deferred GPU failure's run now, overlapped
        with the wait (the log tail's GET, the agent's annotation).  Only the finished /
        missing checks read it: a decision of this process that wrote the row since is
        caught by ``_applied`` before the read is taken, as with a read of its own."""
        labels = kube.labels_of(pod)
        rid = labels.get(self._job_label)
        if not rid:
            return
        key = (labels.get(self.cfg.labels.job_template_name_key, ""), rid)
        if key in self._applied:
            return
        now = time.monotonic()
        old = self._prefetch.get(key)
        if old is not None:
            if now - old[1] <= self._prefetch_ttl:
                return
            del self._prefetch[key]  # a stale one: read again
            old[0].cancel()
        while self._prefetch:  # deferrals that never became a decision (oldest first)
            k0, (f0, t0) = next(iter(self._prefetch.items()))
            if now - t0 <= self._prefetch_ttl and len(self._prefetch) < 4096:
                break
            del self._prefetch[k0]
            f0.cancel()
        fut = asyncio.ensure_future(self.store.read_status(*key))
        fut.add_done_callback(_consume_exception)
        self._prefetch[key] = (fut, now)
        self.metrics.inc("checkpoint_reads_prefetched")

    def _take_prefetch(self, key: Tuple[str, str]) -> Optional[asyncio.Future]:
        """The prefetched read of ``key`` if it is fresh and did not fail, else None."""
        entry = self._prefetch.pop(key, None)
        if entry is None:
            return None
        fut, t0 = entry
        if time.monotonic() - t0 > self._prefetch_ttl or fut.cancelled() or (fut.done() and fut.exception() is not None):
            fut.cancel()
            return None
        return fut

    def _drop_prefetch(self, lost: Callable[[str], bool]) -> None:
        for key in [k for k in self._prefetch if lost(k[1])]:
            self._prefetch.pop(key)[0].cancel()

    async def _fetch_log_tail(self, key: str, pod: Dict[str, Any], want: List[Dict[str, Any]], waited: bool) -> None:
        from .gpu.logtail import fetch_api_tail

        g = self.cfg.gpu
        sem = self._log_sem
        if sem is None:
            sem = self._log_sem = asyncio.Semaphore(g.log_tail_concurrency)

        async def one(w):
            # pods/log is proxied through the kubelet: a GPU failure wave reads at most
            # gpu.log-tail-concurrency tails at once per process, the rest queue here
            if sem.locked():
                self.metrics.inc("log_tail_queued")
            async with sem:
                self._log_inflight += 1
                self.log_tail_inflight_max = max(self.log_tail_inflight_max, self._log_inflight)
                self.metrics.set("log_tail_inflight", self._log_inflight)
                try:
                    return await fetch_api_tail(self.jobs, self.namespace, kube.name_of(pod), w["container"],
                                                previous=w["previous"], limit_bytes=g.log_tail_bytes,
                                                timeout=g.log_tail_timeout)
                finally:
                    self._log_inflight -= 1
                    self.metrics.set("log_tail_inflight", self._log_inflight)

        try:
            # one failed container (the common case): no gather, no Task per read
            recs = [await one(want[0])] if len(want) == 1 else await asyncio.gather(*(one(w) for w in want))
            for r, w in zip(recs, want):
                r["restart"] = w["restart"]
                if r.get("error"):
                    self.metrics.inc("log_tail_errors")
                elif r.get("match"):
                    self.metrics.inc("log_tail_hits", labels={"match": r["match"]})
            self.metrics.inc("log_tail_fetches", len(recs))
            self.classifier.store_logs(pod, list(recs))
        finally:
            self._log_fetches.pop(key, None)
        latest = self.pod_informer.indexer.get(key)
        if latest is not None and self.active:
            self._on_pod_update(None, latest, waited=waited)
        self._end_deferral(key)

    def _end_deferral(self, key: str) -> None:
        """A deferred failure was re-classified: unless it is waiting again, forget its
        arrival stamps (no decision came of it, or the decision took them) — a later
        failure of the same pod starts its own clock."""
        if key not in self._gpu_wait and key not in self._log_fetches:
            self._deferred_at.pop(key, None)

    def _expire_gpu_waits(self) -> None:
        now = time.monotonic()
        for key, deadline in list(self._gpu_wait.items()):
            if deadline > now:
                continue
            del self._gpu_wait[key]
            pod = self.pod_informer.indexer.get(key)
            if pod is not None:
                self.metrics.inc("gpu_evidence_wait_expired")
                self._on_pod_update(None, pod, waited=True)
            self._gpu_wait_over(key)
            self._end_deferral(key)

    def _gpu_wait_over(self, key: str) -> None:
        """A pod's GPU evidence wait ended (the annotation landed, the wait expired, the
        pod left this replica): release the Job decision waiting for it, if any."""
        fut = self._gpu_waiters.pop(key, None)
        if fut is not None and not fut.done():
            fut.set_result(None)

    def _on_job_add(self, job):
        if self._parked:
            self._unpark("Job", kube.name_of(job))
        self._on_job_update(None, job)

    def _on_job_update(self, old, job):
        if not self.active or old is job:
            return
        recv = self.wall()
        for r in self.classifier.classify_job(job, old, self.lookup):
            self._submit(r, recv, recv, "Job")

    # ------------------------------------------------------------------ stale-event parking
    def _park(self, ev, recv):
        inv = ev.get("involvedObject") or {}
        grace = self.cfg.rules.stale_event_grace
        if grace <= 0:
            if self.cfg.informer_label_selector:
                self.metrics.inc("events_unmatched")
                self.log.v(2).info("event object not in the Nexus caches, dropped", requestId=inv.get("name"))
            else:
                self.log.info("Algorithm object not found - stale event", requestId=inv.get("name"),
                              reason=ev.get("reason"), message=ev.get("message"))
                self.metrics.inc("events_stale")
            return
        key = (inv.get("kind", ""), inv.get("name", ""))
        lst = self._parked.setdefault(key, [])
        lst.append((time.monotonic() + grace, ev, recv))
        self.metrics.inc("events_parked")

    def _unpark(self, kind, name):
        if not self._parked:
            return
        lst = self._parked.pop((kind, name), None)
        if lst:
            for _deadline, ev, _recv in lst:
                self._on_event_add(ev)

    def drop_parked(self, kind, name):
        """Another shard worker owns this object: forget events parked waiting for it."""
        if self._parked:
            self._parked.pop((kind, name), None)

    async def _sweep_parked(self):
        tick = max(0.02, min(1.0, self.cfg.rules.stale_event_grace / 4 or 1.0,
                             self.cfg.gpu.evidence_wait / 4 if self.cfg.gpu.evidence_wait > 0 else 1.0))
        selected = self.cfg.informer_label_selector
        while True:
            await asyncio.sleep(tick)
            if self._gpu_wait:
                self._expire_gpu_waits()
            now = time.monotonic()
            if now >= self._label_check_at:
                self._check_labels(now)
            ws = self.worker_shard
            for key in list(self._parked):
                lst = [p for p in self._parked[key] if p[0] > now]
                dropped = len(self._parked[key]) - len(lst)
                if dropped and ws is not None and key[0] == "Pod":
                    owner = ws.owner_of_pod(key[1])
                    if owner not in (None, ws.index):
                        dropped = 0  # another shard worker (or replica) owns that pod: not stale, just not ours
                    elif owner is None and self.hub_fed and ws.index != 0:
                        # the hub broadcast an event about a pod it had not routed yet to every
                        # worker: only worker 0 accounts for it, so it is counted once
                        dropped = 0
                if dropped:
                    if selected:
                        # label-selected caches hold only Nexus runs: an event whose object never
                        # showed up is almost always about a non-Nexus Pod/Job of the namespace —
                        # counted, logged at V(2) only (not a stale-cache symptom)
                        self.metrics.inc("events_unmatched", dropped)
                        self.log.v(2).info("event object not in the Nexus caches, dropped", kind=key[0], name=key[1])
                    else:
                        self.metrics.inc("events_stale", dropped)
                        self.log.info("Algorithm object not found - stale event", kind=key[0], requestId=key[1])
                if lst:
                    self._parked[key] = lst
                else:
                    del self._parked[key]

    def _check_labels(self, now: float) -> None:
        """Loud startup check for a label-key mismatch: the label keys
        are unverifiable offline guesses, and with server-side selectors a wrong guess
        leaves the Pod/Job caches empty so every decision is silently dropped.  Events
        naming Pods/Jobs while both caches stay empty means the selector matches nothing."""
        synced = all(i.has_synced() for i in (self.event_informer, self.pod_informer, self.job_informer))
        if not synced or not self.cfg.informer_label_selector or not self.active:
            self._label_check_at = now + 5.0
            return
        self._label_check_at = now + 60.0
        owned = self.shards.owned
        if (owned is not None and not owned) or self.pod_informer.rejected or self.job_informer.rejected:
            # a shard replica holding no shard, or objects that matched the selector and were
            # filtered as another replica's / worker's: empty caches are by design here
            return
        if len(self.pod_informer.indexer) or len(self.job_informer.indexer):
            if self.label_mismatch:
                self.label_mismatch = False
                self.metrics.set("label_selector_mismatch", 0.0)
            return
        named = sum(1 for ev in self.event_informer.indexer.values()
                    if (ev.get("involvedObject") or {}).get("kind") in ("Pod", "Job"))
        if named < 3:
            return
        self.label_mismatch = True
        self.metrics.set("label_selector_mismatch", 1.0)
        lb = self.cfg.labels
        self.log.warning("LABEL MISMATCH: the namespace has Events about Pods/Jobs but no Pod or Job matches the "
                         "Nexus label selector - every decision would be dropped. Check labels.nexus-component / "
                         "labels.algorithm-run-value against the labels your Nexus runs carry.",
                         selector=f"{lb.nexus_component_label}={lb.algorithm_run_value}", events=named,
                         namespace=self.namespace)

    # ------------------------------------------------------------------ submit
    def _submit(self, r: RunStatusAnalysisResult, origin: float, recv: float, kind: str = "",
                delivery: Optional[Tuple[float, float, float]] = None) -> None:
        key = (r.algorithm, r.request_id)
        if not r.request_id:
            self.metrics.inc("decisions_unkeyed")
            return
        if not self.owns(key):
            return
        applied = self._applied.get(key)
        if applied is not None and (applied in _cp.FINISHED_STAGES
                                    or (r.action == A.TO_RUNNING and applied == LifecycleStage.RUNNING)):
            self.metrics.inc("decisions_suppressed")
            return
        if self.cfg.observability.stage_timestamps:
            st = r.stamps
            st["origin"] = origin
            st["receive"] = recv
            st["enqueue"] = self.wall()
            # the watch batch being dispatched (hub read / worker feed / decoded), or the one
            # that carried a deferred failure
            d = delivery if delivery is not None else _DELIVERY.get(kind)
            if d is not None:
                st["delivery"] = d
        self.metrics.inc("decisions", labels={"action": r.action})
        self.pipeline.receive(r)

    # ------------------------------------------------------------------ actuate
    def _conditional(self, running: bool) -> bool:
        mode = self.cfg.compat.conditional_update
        if mode == "always":
            return True
        if mode == "never":
            return False
        # HA: a single lease or shard leases (a deposed owner may still hold a decision)
        return running or self.cfg.leader_election.enabled or self.cfg.sharding.mode == "lease"

    async def _delete_job(self, name: str) -> bool:
        try:
            await self.jobs.delete_job(self.namespace, name, "Background")
            self.metrics.inc("jobs_deleted")
            return True
        except NotFound:
            if self.cfg.compat.delete_not_found_ok:
                return False
            raise

    async def _guarded_action(self, r: RunStatusAnalysisResult) -> Decision:
        """:meth:`supervise_action` reporting to the store circuit breaker: an
        availability error (no host, connection lost, client timeout, Unavailable /
        Overloaded / IsBootstrapping) counts against the store; a decision whose store call
        returned counts for it — even when the Job DELETE after the write then fails; one
        that never reached the store (fenced) or was refused as a request (Invalid, one
        partition's WriteTimeout, LWT contention) for neither."""
        br = self.breaker
        try:
            d = await self.supervise_action(r)
        except BaseException as exc:
            if is_availability_error(exc):
                br.failure()
            elif r.answered == r.attempts:
                br.success()  # the store answered (the Job DELETE after the write failed)
            else:
                br.neutral()  # never reached the store, or a request-level refusal: says nothing about its health
            raise
        if d.outcome == "fenced":
            br.neutral()
        else:
            br.success()
        return d

    async def supervise_action(self, r: RunStatusAnalysisResult) -> Decision:
        """Reference ``superviseAction`` (``supervisor.go:261-374``) with the fixes of SURVEY §7.5."""
        wall = self.wall
        compat = self.cfg.compat
        r.attempts += 1
        stamps = r.stamps
        if stamps is not None and "dequeue" not in stamps:
            stamps["dequeue"] = wall()
        failing = r.action in A.FAILING
        rid = r.request_id
        epoch = self._token(rid)
        if r.action not in STAGE_FOR_ACTION:
            raise ValueError(f"unknown analysis result action: {r.action}")
        if self._fenced(epoch, rid):
            self.metrics.inc("decisions_fenced")
            return Decision(r, "fenced", None, False)
        applied = self._applied.get((r.algorithm, rid))
        if applied is not None and not r.pending_delete:
            # queued behind the decision that wrote this row (a run's Started Event and its
            # pod's Running transition; a pod's OOM and its Job's PodFailurePolicy): its stage
            # is known, so the read is skipped — the outcome is what reading it would give
            if applied in _cp.FINISHED_STAGES:
                self.metrics.inc("decisions_suppressed")
                return await self._skip_finished(r, epoch, failing, applied)
            if r.action == A.TO_RUNNING and applied == LifecycleStage.RUNNING:
                self.metrics.inc("decisions_suppressed")
                return Decision(r, "skipped-already-running", applied, False)
        if failing and r.object_kind == "Job" and r.reason in _POD_FAILED_REASONS and self._settle_wait > 0:
            await self._await_pod_failure(r)
        if failing:
            # a Job-level failure can overtake its pod's (deferred) log-tail read: wait for it,
            # then re-enrich — an OOM found now also fixes the action (BackoffLimitExceeded of
            # an OOM-killed run is FAILED, not DEADLINE_EXCEEDED), so it must precede the stage
            if self._gpu_wait and r.object_kind == "Job":
                await self._await_gpu_evidence(r)
            if self._log_fetches and r.object_kind == "Job":
                await self._await_pod_logs(r)
            self.classifier.finish(r, self.lookup)
        if self._fused or (self._fused_running and not failing):
            d = await self._fused_action(r, epoch, failing)
            if d is not None:
                return d
        try:
            # the owned-columns write needs only the stage; the full-row upsert (reference
            # UpsertCheckpoint of the deep copy) needs every column
            pre = self._take_prefetch((r.algorithm, r.request_id)) if self._prefetch else None
            if pre is not None:
                cp = await pre  # started while the failure waited for its log tail / evidence
                self.metrics.inc("checkpoint_reads_prefetch_used")
            else:
                read = self.store.read_checkpoint if compat.full_row_upsert else self.store.read_status
                cp = await read(r.algorithm, r.request_id)
            r.answered = r.attempts
        except Exception as exc:
            self.log.error(exc, "no checkpoint exists for the provided request, job will be deleted without metadata saved",
                           requestId=r.request_id, algorithm=r.algorithm)
            if compat.delete_on_read_error and failing:
                try:
                    await self._delete_job(r.request_id)
                except Exception as del_exc:  # noqa: BLE001 - the read error is what is retried
                    self.log.error(del_exc, "failed to delete an algorithm submission after a checkpoint read error",
                                   requestId=r.request_id, algorithm=r.algorithm)
            raise
        stamps["read"] = wall()
        key = (r.algorithm, r.request_id)
        if cp is None:
            return await self._skip_missing(r, failing)
        if cp.is_finished():
            return await self._skip_finished(r, epoch, failing, cp.lifecycle_stage)
        stage = STAGE_FOR_ACTION[r.action]()
        now_dt = _dt.datetime.fromtimestamp(wall(), _dt.timezone.utc)
        if r.action == A.TO_RUNNING:
            if cp.lifecycle_stage == LifecycleStage.RUNNING and not compat.full_row_upsert:
                self._remember(key, stage)
                return Decision(r, "skipped-already-running", stage, False)
            if self._fenced(epoch, rid):
                self.metrics.inc("decisions_fenced")
                return Decision(r, "fenced", None, False)
            if not await self._write(cp, stage, None, None, now_dt, set_failure=False, running=True):
                return await self._lost_race(r, key)
            stamps["ack"] = wall()
            stamps["ack_mono"] = time.monotonic()
            self._observe(r)
            self._remember(key, stage)
            return Decision(r, "applied", stage, False)
        cause = R.failure_cause(r.action, r.run_status_message, compat.doubled_fatal_cause)
        details = render_trace(r, self.cfg.rules.trace_format, self.cfg.rules.trace_max_bytes)
        # The reference deletes the Job, then upserts the row (supervisor.go:289-301).  This
        # build writes first: deleting first (or concurrently) lets a crash between the two
        # lose the decision for good — the Job's pods are garbage-collected, so the replay
        # after failover has nothing to re-decide from.  Written-then-crashed instead leaves
        # a failed row whose Job still exists, which the replay finishes (finished path).
        if self._fenced(epoch, rid):
            self.metrics.inc("decisions_fenced")
            return Decision(r, "fenced", None, False)
        try:
            written = await self._write(cp, stage, cause, details, now_dt, set_failure=True)
        except Exception as exc:
            self.log.error(exc, "failed to update algorithm submission status", requestId=r.request_id, algorithm=r.algorithm)
            raise
        if not written:
            return await self._lost_race(r, key)
        stamps["ack"] = wall()
        stamps["ack_mono"] = time.monotonic()
        self._observe(r)
        self._remember(key, stage)
        self.metrics.inc("decisions_applied", labels={"stage": stage, "class": r.failure_class or "none"})
        if r.failure_class in _GPU_CLASSES:
            self._count_gpu_failure(r)
        if self.cfg.observability.record_events and not self.cfg.dry_run:
            self._record_event(r, stage)
        if self._fenced(epoch, rid):  # durable, but the Job now belongs to the new leader's replay
            return Decision(r, "applied", stage, False)
        if self.cfg.async_job_delete:
            # the decision is durable; the Job DELETE must not hold a worker (and with it
            # every later decision) hostage to API-server latency
            self._spawn_delete(r)
            return Decision(r, "applied", stage, False)
        try:
            deleted = await self._delete_job(r.request_id)
        except Exception as exc:
            self.log.error(exc, "failed to delete an algorithm submission", requestId=r.request_id, algorithm=r.algorithm)
            r.pending_delete = True  # the retry sees the finished row and only deletes
            raise
        return Decision(r, "applied", stage, deleted)

    async def _await_pod_failure(self, r: RunStatusAnalysisResult) -> None:
        """A Job's BackoffLimitExceeded / PodFailurePolicy means a pod of it failed.  When
        no cached pod shows that yet (or none is cached), the pod's update is still on its
        own watch stream:
        wait for it (``rules.job-pod-settle``) so the cause found by late enrichment (OOM,
        eviction, GPU) does not depend on which stream delivered first."""
        deadline = time.monotonic() + self._settle_wait
        waited = False
        while True:
            # no pod cached at all counts as "not seen yet": a replica that just gained the
            # run's shard re-lists Jobs and Pods concurrently
            pods = self.lookup.pods_of_job(r.request_id)
            if any(_pod_failed(p) for p in pods):
                break
            relist = self._pod_relist
            if relist is not None and not relist[0].is_set() and self.shards.of(r.request_id) in relist[1]:
                # its shard was just gained and the pod list is not in yet: until it is, the
                # pod watch is down and a cached pod may be as old as the gain (a 10k-pod list
                # behind a kube-qps bucket shared with the replay's DELETEs took 18 s in
                # config 5s) — wait for the list, not the settle time alone
                waited = True
                self.metrics.inc("job_pod_settle_relist_waits")
                try:
                    await asyncio.wait_for(relist[0].wait(), 30.0)
                except asyncio.TimeoutError:
                    pass
                deadline = max(deadline, time.monotonic() + self._settle_wait)
                continue
            left = deadline - time.monotonic()
            if left <= 0:
                self.metrics.inc("job_pod_settle_expired")
                self.log.info("no failed pod of the job seen within the settle time; deciding from the job",
                              requestId=r.request_id, reason=r.reason,
                              pods=[f"{kube.name_of(p)}:{(p.get('status') or {}).get('phase')}" for p in pods][:4])
                break
            loop = asyncio.get_running_loop()
            fut = self._settle.get(r.request_id)
            if fut is None or fut.done():
                fut = self._settle[r.request_id] = loop.create_future()
            waited = True
            # a plain waiter woken by the pod's update or the settle timer: most Job
            # decisions of a pod failure wait here once (the two watch streams race), and
            # wait_for(shield(...)) costs a Task and two futures per wait
            waiter = loop.create_future()
            wake = functools.partial(_wake, waiter)
            fut.add_done_callback(wake)
            timer = loop.call_later(left, wake)
            try:
                await waiter
            finally:
                timer.cancel()
                fut.remove_done_callback(wake)
        if waited:
            self.metrics.inc("job_pod_settle_waits")

    async def _await_gpu_evidence(self, r: RunStatusAnalysisResult) -> None:
        """A Job-level failure whose pod is held for the node agent's evidence annotation
        (``gpu.evidence-wait``): wait for that wait to end, so the Job decision is enriched
        with the same GPU evidence (an HBM-OOM found there also fixes the stage) instead of
        writing the row without it ahead of the annotation."""
        keys = [k for k in (kube.object_key(p) for p in self.lookup.pods_of_job(r.request_id)) if k in self._gpu_wait]
        if not keys:
            return
        self.metrics.inc("decisions_awaited_gpu_evidence")
        loop = asyncio.get_running_loop()
        futs = []
        for k in keys:
            fut = self._gpu_waiters.get(k)
            if fut is None or fut.done():
                fut = self._gpu_waiters[k] = loop.create_future()
            futs.append(fut)
        await asyncio.wait(futs, timeout=self.cfg.gpu.evidence_wait + 0.5)

    async def _await_pod_logs(self, r: RunStatusAnalysisResult) -> None:
        keys = [kube.object_key(p) for p in self.lookup.pods_of_job(r.request_id)]
        tasks = [self._log_fetches[k] for k in keys if k in self._log_fetches]
        if tasks:
            self.metrics.inc("decisions_awaited_log_tail")
            await asyncio.wait(tasks, timeout=self.cfg.gpu.log_tail_timeout + 0.5)

    async def _skip_missing(self, r: RunStatusAnalysisResult, failing: bool) -> Decision:
        self.log.info("no checkpoint exists for the provided request, skipping", requestId=r.request_id, algorithm=r.algorithm)
        deleted = False
        if self.cfg.compat.delete_on_read_error and failing:
            deleted = await self._delete_job(r.request_id)
        self.metrics.inc("decisions_missing_checkpoint")
        return Decision(r, "skipped-missing", None, deleted)

    async def _skip_finished(self, r: RunStatusAnalysisResult, epoch, failing: bool, current: str) -> Decision:
        self.log.info("algorithm run completed, skipping action", algorithm=r.algorithm, requestId=r.request_id)
        deleted = False
        # a failing decision on a run already in a failed stage: the Job may have survived
        # a crash between write and delete (or a failed delete) — finish the delete
        if r.pending_delete or (failing and current in _FAILED_STAGES()
                                and self.job_informer.indexer.get_by_name(self.namespace, r.request_id) is not None):
            if self._fenced(epoch, r.request_id):
                return Decision(r, "fenced", current, False)
            if self.cfg.async_job_delete and not r.pending_delete:
                # the row is final: like a fresh decision's, the Job DELETE must not hold a
                # worker — behind a kube-qps bucket full of DELETEs (a new leader finishing its
                # predecessor's) it would stall the whole pipeline for seconds
                self._spawn_delete(r)
            else:
                deleted = await self._delete_job(r.request_id)
            r.pending_delete = False
        self._remember((r.algorithm, r.request_id), current)
        self.metrics.inc("decisions_skipped_finished")
        return Decision(r, "skipped-finished", current, deleted)

    async def _fused_action(self, r: RunStatusAnalysisResult, epoch, failing: bool) -> Optional[Decision]:
        """``compat.fused-write``: the decision is ONE conditional write
        (``UPDATE … IF lifecycle_stage IN (<unfinished stages>)``) instead of the reference's
        read followed by a write (``supervisor.go:264-301``).  The store checks the stage
        inside a Paxos round, so a row finished by another *conditional* writer (a new
        leader's or shard owner's FAILED) is never overwritten, nor is one whose plain write
        was committed before the round's read phase.  A plain (non-LWT) write racing with the
        round — other Nexus components write the row without conditions — is not ordered
        against it: Cassandra / Scylla only linearise LWTs among themselves, so that window
        stays as narrow as, not narrower than, the reference's read→write window.  A
        not-applied answer carries the row's stage, which drives the reference's skip paths
        (no row / finished / ToRunning on a RUNNING row).  The price is a Paxos round (~4
        replica round trips, serialised per partition; ``compat.fused-write: auto`` uses it
        only under HA — docs/ARCHITECTURE.md "Pricing the LWT").  Returns None for a stage
        outside the known set (custom stage strings): the two-step path then decides with
        that stage in its guard."""
        wall = self.wall
        compat = self.cfg.compat
        stamps = r.stamps
        rid = r.request_id
        stage = STAGE_FOR_ACTION[r.action]()
        running = r.action == A.TO_RUNNING
        only_if = self._unfinished_guard(running)
        if running:
            cause = details = None
        else:
            cause = R.failure_cause(r.action, r.run_status_message, compat.doubled_fatal_cause)
            details = render_trace(r, self.cfg.rules.trace_format, self.cfg.rules.trace_max_bytes)
        if self._fenced(epoch, rid):
            self.metrics.inc("decisions_fenced")
            return Decision(r, "fenced", None, False)
        t = wall()
        stamps["prepare"] = t  # no read in this path: dequeue → here is local work, here → ack the CAS
        now_dt = _dt.datetime.fromtimestamp(t, _dt.timezone.utc)
        try:
            applied, current = await self.store.cas_update(r.algorithm, rid, stage, cause, details, now_dt,
                                                           only_if, set_failure=not running)
            r.answered = r.attempts
        except Exception as exc:
            self.log.error(exc, "failed to update algorithm submission status", requestId=rid, algorithm=r.algorithm)
            # the reference deletes on a failed checkpoint *read* (supervisor.go:265-273); here
            # the one store call is the write itself, so delete only when it provably never
            # reached the store — a timed-out write may have landed, and deleting then could
            # leave an unfinished row with nothing left to replay from
            if compat.delete_on_read_error and failing and isinstance(exc, NotSent):
                try:
                    await self._delete_job(rid)
                except Exception as del_exc:  # noqa: BLE001 - the store error is what is retried
                    self.log.error(del_exc, "failed to delete an algorithm submission after a checkpoint store error",
                                   requestId=rid, algorithm=r.algorithm)
            raise
        key = (r.algorithm, rid)
        if not applied:
            if current is not None:
                self.metrics.inc("conditional_write_rejected")
            if current is None:
                return await self._skip_missing(r, failing)
            if current in _cp.FINISHED_STAGES:
                return await self._skip_finished(r, epoch, failing, current)
            if running and current == LifecycleStage.RUNNING:
                self._remember(key, current)
                return Decision(r, "skipped-already-running", current, False)
            self.metrics.inc("fused_write_fallbacks")
            return None
        stamps["ack"] = wall()
        stamps["ack_mono"] = time.monotonic()
        self._observe(r)
        self._remember(key, stage)
        if running:
            return Decision(r, "applied", stage, False)
        self.metrics.inc("decisions_applied", labels={"stage": stage, "class": r.failure_class or "none"})
        if r.failure_class in _GPU_CLASSES:
            self._count_gpu_failure(r)
        if self.cfg.observability.record_events and not self.cfg.dry_run:
            self._record_event(r, stage)
        if self._fenced(epoch, rid):
            return Decision(r, "applied", stage, False)
        if self.cfg.async_job_delete:
            self._spawn_delete(r)
            return Decision(r, "applied", stage, False)
        try:
            deleted = await self._delete_job(rid)
        except Exception as exc:
            self.log.error(exc, "failed to delete an algorithm submission", requestId=rid, algorithm=r.algorithm)
            r.pending_delete = True  # the retry sees the finished row and only deletes
            raise
        return Decision(r, "applied", stage, deleted)

    def _unfinished_guard(self, running: bool) -> Tuple[str, ...]:
        """``IF lifecycle_stage IN (...)`` of a fused write, memoised per stage configuration
        (stage strings are configurable: ``stages:``).  ToRunning leaves RUNNING out, so a
        RUNNING row answers "not applied, RUNNING" (the reference's skip) without a write."""
        fin = _cp.FINISHED_STAGES
        hit = self._guards.get((running, id(fin)))
        if hit is not None and hit[0] is fin:
            return hit[1]
        g = _cp.unfinished_stages()
        if running:
            g = tuple(x for x in g if x != LifecycleStage.RUNNING)
        self._guards[(running, id(fin))] = (fin, g)
        return g

    def _spawn_delete(self, r: RunStatusAnalysisResult) -> None:
        nowait = getattr(self.jobs, "delete_job_nowait", None)
        if nowait is not None:
            # fast path: the request goes straight onto an open pipelined connection and a
            # callback settles it (no coroutine / Task per decision); failures fall back to
            # the retrying coroutine below
            fut = nowait(self.namespace, r.request_id, "Background")
            if fut is not None:
                self._deletes[fut] = r.request_id
                fut.add_done_callback(lambda f, r=r: self._delete_settled(r, f))
                return
        t = asyncio.ensure_future(self._delete_with_retry(r))
        self._deletes[t] = r.request_id
        t.add_done_callback(self._delete_done)

    def _delete_done(self, t) -> None:
        self._deletes.pop(t, None)

    def _delete_settled(self, r: RunStatusAnalysisResult, fut) -> None:
        self._deletes.pop(fut, None)
        if fut.cancelled():
            return
        exc = fut.exception()
        if exc is None:
            try:
                self.jobs.check_delete(fut.result())
            except NotFound as e:
                if self.cfg.compat.delete_not_found_ok:
                    return  # already gone (reference retried this forever: SURVEY §2.9.2)
                exc = e
            except Exception as e:  # noqa: BLE001 - API error: retried below
                exc = e
        if exc is None:
            self.metrics.inc("jobs_deleted")
            ack = r.stamps.get("ack") if r.stamps else None
            if ack is not None:
                self.metrics.observe_seconds("stage_delete", self.wall() - ack)
            return
        if not self.active or not self.shards.owns(r.request_id):
            return  # fenced: the new leader's (shard owner's) replay owns this Job
        self.metrics.inc("job_delete_retries")
        # a throttled DELETE (429) waits at least for the server's Retry-After hint
        first = max(self.cfg.failure_rate_base_delay, getattr(exc, "retry_after", None) or 0.0)
        t = asyncio.ensure_future(self._delete_with_retry(r, first_delay=first))
        self._deletes[t] = r.request_id
        t.add_done_callback(self._delete_done)

    async def _delete_with_retry(self, r: RunStatusAnalysisResult, first_delay: float = 0.0) -> None:
        """Background Job DELETE after a durable failure write.  The key is already marked
        finished, so a later failing decision would be suppressed: this loop is the only
        thing left that removes the Job (and frees its amd.com/gpu) — it never gives up
        while this replica leads and the Job is still cached.
        After ``max-retries`` attempts the backoff keeps doubling up to 60 s."""
        c = self.cfg
        delay = c.failure_rate_base_delay or 0.05
        cap = c.failure_rate_max_delay
        attempt = 0
        rid = r.request_id
        epoch = self._token(rid)
        if first_delay > 0:
            attempt = 1
            await asyncio.sleep(first_delay)
            delay = min(delay * 2, cap)
        while True:
            if self._fenced(epoch, rid):
                return
            if attempt and self.job_informer.indexer.get_by_name(self.namespace, r.request_id) is None \
                    and self.job_informer.has_synced():
                return  # gone from the cache: deleted by someone else (or our earlier attempt landed)
            attempt += 1
            try:
                await self._delete_job(r.request_id)
                ack = r.stamps.get("ack") if r.stamps else None
                if ack is not None:
                    self.metrics.observe_seconds("stage_delete", self.wall() - ack)
                return
            except asyncio.CancelledError:
                raise
            except Exception as exc:  # noqa: BLE001 - retried with backoff
                if c.max_retries and attempt == c.max_retries:
                    self.metrics.inc("job_deletes_slow")
                    self.log.error(exc, "algorithm submission still not deleted; retrying with a longer backoff",
                                   requestId=r.request_id, algorithm=r.algorithm, attempts=attempt)
                if c.max_retries and attempt >= c.max_retries:
                    cap = max(cap, 60.0)
                self.metrics.inc("job_delete_retries")
                await asyncio.sleep(max(delay, getattr(exc, "retry_after", None) or 0.0))
                delay = min(delay * 2, cap)

    async def _write(self, cp, stage, cause, details, now_dt, set_failure, running=False) -> bool:
        """Write the decision; False when the conditional write found the row already
        moved to a finished stage (by another leader, shard owner or component)."""
        compat = self.cfg.compat
        if compat.full_row_upsert:
            clone = cp.deep_copy()
            clone.lifecycle_stage = stage
            if set_failure:
                clone.algorithm_failure_cause = cause
                clone.algorithm_failure_details = details
            clone.last_modified = now_dt
            await self.store.upsert_checkpoint(clone)
            return True
        only_if = None
        if self._conditional(running) and cp.lifecycle_stage is not None:
            only_if = _cp.unfinished_stages()
            if cp.lifecycle_stage not in only_if:
                only_if = only_if + (cp.lifecycle_stage,)
        applied = await self.store.update_status(cp.algorithm, cp.id, stage, cause, details, now_dt,
                                                 only_if_stages=only_if, set_failure=set_failure)
        return bool(applied) or only_if is None

    async def _lost_race(self, r: RunStatusAnalysisResult, key) -> Decision:
        """The conditional write was not applied: re-read; a finished row is final (another
        writer got there first), anything else is retried through the pipeline backoff."""
        self.metrics.inc("conditional_write_rejected")
        cp = await self.store.read_status(r.algorithm, r.request_id)
        if cp is not None and cp.is_finished():
            self._remember(key, cp.lifecycle_stage)
            return Decision(r, "skipped-finished", cp.lifecycle_stage, False)
        raise CasConflict(f"checkpoint {r.algorithm}/{r.request_id} changed concurrently")

    def _remember(self, key, stage):
        self._applied[key] = stage
        self._applied.move_to_end(key)
        if len(self._applied) > self._applied_cap:
            self._applied.popitem(last=False)

    _STAGE_HISTS = ("event_to_checkpoint", "receive_to_checkpoint", "stage_classify", "stage_queue",
                    "stage_prepare", "stage_write", "stage_read", "stage_hub", "stage_feed", "stage_dispatch")

    def _record_event(self, r: RunStatusAnalysisResult, stage: str) -> None:
        """``observability.record-events``: a Warning Event on the run's Job, so ``kubectl
        describe job`` says what the supervisor decided and why (the reference records none).
        Fire-and-forget: an API error costs the Event, never the decision.  Its reason
        (``NexusRunFailed``) matches no rule, so the supervisor's own Event informer ignores it."""
        create = getattr(self.jobs, "create", None)
        if create is None:
            return
        node, gpu = failed_gpu(r) if r.failure_class in _GPU_CLASSES else ("", None)
        where = f", GPU {gpu}" + (f" on {node}" if node else "") if gpu is not None else ""
        cause = R.failure_cause(r.action, r.run_status_message, self.cfg.compat.doubled_fatal_cause)
        now = _dt.datetime.now(_dt.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")
        ev = {"apiVersion": "v1", "kind": "Event",
              "metadata": {"generateName": f"{r.request_id}.", "namespace": self.namespace},
              "involvedObject": {"apiVersion": "batch/v1", "kind": "Job", "name": r.request_id,
                                 "namespace": self.namespace},
              "reason": "NexusRunFailed", "type": "Warning", "count": 1,
              "message": f"{stage} ({r.failure_class or 'none'}{where}): {cause}"[:1024],
              "source": {"component": "nexus-supervisor"}, "firstTimestamp": now, "lastTimestamp": now}

        async def go():
            try:
                await create("Event", self.namespace, ev)
                self.metrics.inc("kube_events_recorded")
            except Exception as exc:  # noqa: BLE001 - best effort
                self.metrics.inc("kube_event_errors")
                self.log.v(1).info("recording a decision Event failed", requestId=r.request_id, err=str(exc))

        t = asyncio.ensure_future(go())
        self._event_tasks.add(t)
        t.add_done_callback(self._event_tasks.discard)

    def _count_gpu_failure(self, r: RunStatusAnalysisResult) -> None:
        """``gpu_failures{node,gpu,class}``: GPU-attributed failures per physical GPU.  The
        supervisor is the one place that sees every run's attribution; a GPU whose count
        keeps rising (VM faults, xGMI link loss, resets) is hardware to drain — an alert on
        ``increase(nexus_supervisor_gpu_failures_total{class="gpu-fault"}[1h]) >= 3`` finds
        it across replicas and shard workers (docs/OPERATIONS.md)."""
        node, gpu = failed_gpu(r)
        self.metrics.inc("gpu_failures", labels={"node": node or "unknown",
                                                 "gpu": "unknown" if gpu is None else str(gpu),
                                                 "class": r.failure_class})

    def _observe(self, r: RunStatusAnalysisResult):
        s = r.stamps
        ack = s.get("ack")
        if ack is None:
            return
        if self.metrics.statsd is None:
            # six records per decision straight into the histograms (no name lookups); a
            # series exists once it has a sample (fused mode has no stage_read)
            hs = self._hists
            if hs is None:
                hs = self._hists = _StageHists(self.metrics, self._STAGE_HISTS)
            origin = s.get("origin")
            if origin is not None:
                hs.rec(0, ack - origin)
            recv = s.get("receive")
            if recv is not None:
                hs.rec(1, ack - recv)
                dl = s.get("delivery")
                if dl is not None:  # hub read → worker feed → decoded → handler (obs/delivery.py)
                    hs.rec(7, dl[1] - dl[0])
                    hs.rec(8, dl[2] - dl[1])
                    hs.rec(9, s["ack_mono"] - (ack - recv) - dl[2])
                enq, deq, rd, prep = s.get("enqueue"), s.get("dequeue"), s.get("read"), s.get("prepare")
                if enq is not None and deq is not None and (rd is not None or prep is not None):
                    hs.rec(2, enq - recv)
                    hs.rec(3, deq - enq)
                    if prep is not None:
                        hs.rec(4, prep - deq)
                        hs.rec(5, ack - prep)
                    else:
                        hs.rec(6, rd - deq)
                        hs.rec(5, ack - rd)
            return
        if "origin" in s:
            self.metrics.observe_seconds("event_to_checkpoint", ack - s["origin"])
        if "receive" in s:
            obs = self.metrics.observe_seconds
            obs("receive_to_checkpoint", ack - s["receive"])
            dl = s.get("delivery")
            if dl is not None:
                obs("stage_hub", dl[1] - dl[0])
                obs("stage_feed", dl[2] - dl[1])
                obs("stage_dispatch", s["ack_mono"] - (ack - s["receive"]) - dl[2])
            # stage decomposition: classify → queue wait → CQL read → CQL write
            enq, deq, rd = s.get("enqueue"), s.get("dequeue"), s.get("read")
            prep = s.get("prepare")
            if enq is not None and deq is not None and (rd is not None or prep is not None):
                obs("stage_classify", enq - s["receive"])
                obs("stage_queue", deq - enq)
                if prep is not None:  # fused: no read; the write stage is the conditional write's round trip
                    obs("stage_prepare", prep - deq)
                    obs("stage_write", ack - prep)
                else:
                    obs("stage_read", rd - deq)
                    obs("stage_write", ack - rd)

    def _done(self, r: RunStatusAnalysisResult, decision: Decision) -> None:
        for h in self.decision_hooks:
            h(decision)

    def _dead_letter(self, r: RunStatusAnalysisResult, exc: BaseException) -> None:
        self.metrics.inc("decisions_dead_lettered")
        self.log.error(exc, "giving up on decision", requestId=r.request_id, algorithm=r.algorithm, action=r.action)
        d = Decision(r, "dead-letter", None, False)
        for h in self.decision_hooks:
            h(d)
