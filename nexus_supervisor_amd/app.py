"""Composition root: config → store, kube client, informers, supervisor, GPU
telemetry, leader election, HTTP observability.

Mirrors the reference's process entry and DI builder
(``/root/reference/main.go:12-43``; ``/root/reference/app/app_dependencies.go:12-85``):
store selection by ``cql-store-type`` (unknown → exit 1, ``main.go:28-36``),
kube client from ``kube-config-path`` (empty → in-cluster), supervisor wiring,
then ``Init`` + ``Start``.  Added: SIGTERM drain (the reference has none,
SURVEY §3E), leader election / sharding gating, GPU attribution and the
``/metrics`` ``/healthz`` ``/readyz`` ``/debug/pprof`` endpoints.
"""
from __future__ import annotations

import asyncio
import os
import signal
import socket
import sys
import time
from typing import Optional

from . import __build__, __version__
from .config import load_config, redacted
from .config.schema import CQL_STORE_MEMORY, SupervisorConfig
from .informer import InformerFactory
from .obs.logging import KLogger, configure_logging, shutdown_logging
from .obs.metrics import DogStatsd, Metrics
from .store.base import CheckpointStore
from .supervisor import JobClient, Supervisor


def build_store(cfg: SupervisorConfig) -> CheckpointStore:
    if cfg.cql_store_type == CQL_STORE_MEMORY:
        from .store.memory import MemoryStore

        return MemoryStore()
    from .store.cql import CqlCheckpointStore

    return CqlCheckpointStore.from_config(cfg)


def _identity(cfg: SupervisorConfig) -> str:
    le = cfg.leader_election
    return le.identity or os.environ.get("POD_NAME") or f"{socket.gethostname()}-{os.getpid()}"


def make_shard_leases(cfg: SupervisorConfig, kube, on_change, metrics, on_renewed=None):
    """``sharding.mode: lease``: the replica's :class:`~.ha.shards.ShardLeaseManager`."""
    from .ha.shards import ShardLeaseManager

    le, sh = cfg.leader_election, cfg.sharding
    return ShardLeaseManager(kube, cfg.resource_namespace, le.lease_name, _identity(cfg), sh.shards,
                             replicas=sh.replicas, lease_duration=le.lease_duration, renew_deadline=le.renew_deadline,
                             retry_period=le.retry_period, on_change=on_change, metrics=metrics, on_renewed=on_renewed)


def build_factory(cfg: SupervisorConfig, client) -> InformerFactory:
    from .kube.client import KubeListWatch
    from .parallel.sharding import ShardSet, watch_field_selector, watch_selector

    ns = cfg.resource_namespace
    owned = ShardSet.from_config(cfg).owned  # static: {shard-index}; lease: none until a lease is won

    def lw(kind: str):
        return KubeListWatch(client, kind, ns, label_selector=watch_selector(cfg, kind, owned),
                             field_selector=watch_field_selector(cfg, kind), watch_timeout=int(cfg.watch_timeout))

    return InformerFactory(lw, resync_period=cfg.resync_period)


def _shard_label_keeper(cfg, kube, metrics, log, owned):
    """The ``sharding.shard-label`` audit + repair and re-label passes
    (:class:`~.admission.ShardLabelKeeper`), in the process that owns the replica's API
    client (a single-process replica, or a sharded replica's parent — not its workers);
    ``owned``: callable → the replica's current shards."""
    s = cfg.sharding
    if (not s.shard_label or s.shards <= 1 or kube is None or not hasattr(kube, "request")
            or not hasattr(kube, "patch_merge") or os.environ.get("NEXUS_WORKER_CONFIG")):
        return None
    from .admission import ShardLabelKeeper

    keeper = ShardLabelKeeper(cfg, kube, metrics, log, owned)
    keeper.start()
    return keeper


async def _start_webhook(cfg, metrics, kube=None, log=None):
    if not cfg.sharding.webhook_port or os.environ.get("NEXUS_WORKER_CONFIG"):
        return None
    from .admission import WebhookServer

    ws = WebhookServer(cfg, metrics)
    boot = None
    if cfg.sharding.webhook_cert_bootstrap and kube is not None:
        from .webhook_certs import WebhookCertBootstrap

        # the serving pair exists before the server starts; renewals are picked up by its reload
        boot = WebhookCertBootstrap.from_config(cfg, kube, metrics, log)
        await boot.sync()
    await ws.start(cfg.observability.http_host, cfg.sharding.webhook_port, cfg.sharding.webhook_cert_dir)
    if boot is not None:
        boot.start(on_change=ws.check_cert)
        ws.bootstrap = boot
    return ws


class Application:
    def __init__(self, cfg: SupervisorConfig, *, kube=None, store: Optional[CheckpointStore] = None,
                 jobs: Optional[JobClient] = None, factory: Optional[InformerFactory] = None, telemetry=None,
                 logger: Optional[KLogger] = None, metrics: Optional[Metrics] = None):
        self.cfg = cfg
        self.log = logger or KLogger()
        self.metrics = metrics or Metrics(cfg.observability.statsd_name, {"version": __version__})
        if kube is None and (factory is None or jobs is None):
            from .kube.client import KubeClient

            kube = KubeClient.for_config(cfg, self.metrics)
        elif kube is not None and hasattr(kube, "apply_config") and not getattr(kube, "flow_configured", False):
            kube.apply_config(cfg, self.metrics)
        self.kube = kube
        self.store = store if store is not None else build_store(cfg)
        self.factory = factory if factory is not None else build_factory(cfg, kube)
        jobs = jobs if jobs is not None else kube
        if cfg.dry_run:
            from .dryrun import DryRunJobs, DryRunStore

            self.store = DryRunStore(self.store, self.log, self.metrics)
            jobs = DryRunJobs(jobs, self.log, self.metrics)
        self.supervisor = Supervisor(cfg, self.store, jobs, self.factory, logger=self.log, metrics=self.metrics)
        self.telemetry = telemetry
        self.elector = None
        self.shard_leases = None
        self.http = None
        self._stopped = asyncio.Event()

    async def start(self) -> None:
        cfg = self.cfg
        self.log.info("Starting Nexus Supervisor", version=__version__, build=__build__, namespace=cfg.resource_namespace,
                      store=cfg.cql_store_type)
        if cfg.dry_run:
            self.log.warning("dry run: checkpoints are read but never written, Jobs are never deleted")
        await self.store.connect()
        if self.telemetry is None and cfg.gpu.attribution_enabled and cfg.gpu.local_telemetry:
            from .gpu.telemetry import make_telemetry

            self.telemetry = make_telemetry(cfg.gpu.backend, cfg.gpu.sample_interval, cfg.gpu.telemetry_events)
        if self.telemetry is not None:
            from .gpu.telemetry import pod_evidence_provider

            self.telemetry.start()
            self.supervisor.classifier.evidence_provider = pod_evidence_provider(
                self.telemetry, cfg.gpu.gpu_resource_name, node=os.environ.get("NODE_NAME", ""))
        self.supervisor.init()
        if cfg.observability.http_port:
            from .obs.http import ObsServer

            self.http = ObsServer(self)
            await self.http.start(cfg.observability.http_host, cfg.observability.http_port)
        if cfg.sharding.mode == "lease":
            # one Lease per shard replaces the single leader lease (ha/shards.py)
            self.shard_leases = make_shard_leases(cfg, self.kube, self._set_shards, self.metrics,
                                                  on_renewed=self.supervisor.shards.set_deadlines)
        elif cfg.leader_election.enabled:
            from .ha.leader import LeaderElector, LeaseLock

            le = cfg.leader_election
            self.supervisor.active = False
            self.elector = LeaderElector(
                LeaseLock(self.kube, cfg.resource_namespace, le.lease_name, _identity(cfg)),
                lease_duration=le.lease_duration, renew_deadline=le.renew_deadline, retry_period=le.retry_period,
                on_started_leading=lambda: self.supervisor.set_active(True),
                on_stopped_leading=lambda: self.supervisor.set_active(False), metrics=self.metrics,
                on_renewed=self.supervisor.set_lease_deadline)
            self.supervisor.active_until = float("-inf")  # nothing until the first hold
        if self.shard_leases is not None:
            # before the cache sync: with shard leases the informers cache only owned shards,
            # so a replica that synced first would list nothing and reach the lease race last
            self.shard_leases.start()
        await self.supervisor.start()
        if self.elector is not None:
            self.elector.start()
        self.labels = _shard_label_keeper(cfg, self.kube, self.metrics, self.log,
                                          lambda: self.supervisor.shards.owned)
        self.webhook = await _start_webhook(cfg, self.metrics, self.kube, self.log)
        if cfg.sharding.mode != "lease" and self.labels is not None and self.supervisor.shards.owned:
            self.labels.request_relabel(self.supervisor.shards.owned)

    def _set_shards(self, owned):
        gained, lost = self.supervisor.set_shards(owned)
        if gained and getattr(self, "labels", None) is not None:
            self.labels.request_relabel(gained)  # their runs may carry labels of another shard count
        return gained, lost

    def ready(self) -> bool:
        return self.factory is not None and all(i.has_synced() for i in self.factory.informers.values())

    async def wait_for_cache_sync(self, timeout: Optional[float] = None) -> bool:
        return await self.factory.wait_for_cache_sync(timeout)

    async def stop(self, drain_timeout: float = 10.0) -> None:
        if getattr(self, "labels", None) is not None:
            await self.labels.stop()
        if getattr(self, "webhook", None) is not None:
            await self.webhook.stop()
        if self.elector is not None:
            await self.elector.stop(release=True)
        if self.shard_leases is not None:
            await self.shard_leases.stop(release=True)
        await self.supervisor.stop(drain=True, timeout=drain_timeout)
        if self.http is not None:
            await self.http.stop()
        if self.telemetry is not None:
            self.telemetry.stop()
        await self.store.close()
        if self.kube is not None:
            await self.kube.close()
        self._stopped.set()

    async def run(self, stop: asyncio.Event) -> None:
        await self.start()
        await stop.wait()
        self.log.info("shutting down: draining in-flight decisions")
        await self.stop()


class _SupervisorFacade:
    """What in-process callers (bench, tests) use of a supervisor, backed by worker processes."""

    def __init__(self, app: "ShardedApplication"):
        self._app = app
        self.namespace = app.cfg.resource_namespace
        self.decision_hooks = app.pool.decision_hooks
        # (request_id, outcome, ack_mono, stage) per reported decision, without building the
        # result/decision objects (the bench tracker: harness work stays out of the parent's CPU)
        self.report_hooks = app.pool.report_hooks
        self.classifier = type("RemoteClassifier", (), {"evidence_provider": None})()

    @property
    def active(self) -> bool:
        return self._app.pool.active

    def set_active(self, active: bool) -> None:
        self._app.pool.set_active(active)

    @property
    def metrics(self) -> Metrics:
        return self._app.merged_metrics


class ShardedApplication:
    """A replica of ``runtime.worker-processes`` shard-worker processes
    (:mod:`.parallel.workers`): this process holds the lease, relays active/standby,
    serves the merged ``/metrics`` and supervises the workers (a worker that dies is
    restarted with backoff; ``/healthz`` reports it until it is back)."""

    def __init__(self, cfg: SupervisorConfig, *, kube=None, logger: Optional[KLogger] = None,
                 metrics: Optional[Metrics] = None, report_decisions: bool = False, log_dir: str = "",
                 telemetry=None):
        from .parallel.workers import WorkerPool

        self.cfg = cfg
        self.log = logger or KLogger()
        self.metrics = metrics or Metrics(cfg.observability.statsd_name, {"version": __version__})
        self.kube = kube
        self.pool = WorkerPool(cfg, report_decisions=report_decisions, log_dir=log_dir)
        if kube is not None and hasattr(kube, "apply_config") and not getattr(kube, "flow_configured", False):
            kube.apply_config(cfg, self.metrics, self.pool.qps_schedule)
        self.supervisor = _SupervisorFacade(self)
        self.merged_metrics = self.metrics
        self.store = None
        self.elector = None
        self.shard_leases = None
        self.http = None
        self.hub = None
        from .parallel.sharding import ShardSet

        self.shards = ShardSet.from_config(cfg)
        self.telemetry = telemetry
        self._owns_telemetry = telemetry is None
        self._gpu_task: Optional[asyncio.Task] = None
        self._gc_task: Optional[asyncio.Task] = None
        from .utils.gctune import GcTuner

        # the parent's loop runs the watch hub: a generation-1/2 collection of its heap (the
        # whole import graph, ~1 ms a pass) is a watch line waiting — the same freeze as the
        # workers' informer caches, once every worker has synced
        self.gc_tuner = GcTuner.from_config(cfg.runtime, self.metrics)
        self._stopped = asyncio.Event()

    async def _tune_gc(self) -> None:
        if await self.pool.wait_synced(None):
            self.gc_tuner.after_sync()

    async def _publish_gpu(self) -> None:
        """Mirror the replica's one GPU monitor into every worker (``RemoteTelemetry``)."""
        from .gpu.telemetry import telemetry_message

        since: dict = {}
        interval = max(0.05, self.cfg.gpu.sample_interval)
        last_snap = None
        while True:
            try:
                t0 = time.perf_counter()
                msg = telemetry_message(self.telemetry, since)
                if msg["snap"] == last_snap:
                    # an unchanged snapshot (GPU processes, events) is not re-sent: the workers
                    # keep theirs (RemoteTelemetry.update); only the new VRAM samples travel.
                    # This runs on the watch hub's loop: every millisecond here is a watch line
                    # waiting (the delivery tail, obs/delivery.py)
                    del msg["snap"]
                else:
                    last_snap = msg["snap"]
                self.pool.broadcast(dict(msg, op="gpu"))
                self.metrics.observe_seconds("gpu_mirror_publish", time.perf_counter() - t0)
            except Exception as exc:  # noqa: BLE001 - telemetry must never stop the replica
                self.log.error(exc, "GPU telemetry publish failed")
            await asyncio.sleep(interval)

    async def start(self) -> None:
        cfg = self.cfg
        self.log.info("Starting Nexus Supervisor", version=__version__, build=__build__, namespace=cfg.resource_namespace,
                      store=cfg.cql_store_type, worker_processes=self.pool.count)
        le = cfg.leader_election
        lease_mode = cfg.sharding.mode == "lease"
        from .obs.loopwatch import install_from_env

        install_from_env(self.metrics, "parent")  # diagnostic: NEXUS_SLOW_CALLBACK_MS (the watch hub's loop)
        if lease_mode:
            self.pool.owned_shards = []  # nothing until a shard lease is won
        await self.pool.start(active=lease_mode or not le.enabled)
        if self.pool.remote_gpu:
            if self.telemetry is None:
                from .gpu.telemetry import make_telemetry

                self.telemetry = make_telemetry(cfg.gpu.backend, cfg.gpu.sample_interval, cfg.gpu.telemetry_events)
                if self.telemetry is not None:
                    self.telemetry.start()
            if self.telemetry is not None:
                self._gpu_task = asyncio.create_task(self._publish_gpu(), name="gpu-telemetry-mirror")
        if self.pool.hub:
            from .parallel.watchhub import WatchHub

            if self.kube is None:
                from .kube.client import KubeClient

                self.kube = KubeClient.for_config(cfg, self.metrics, schedule=self.pool.qps_schedule)
            self.hub = WatchHub(cfg, self.kube, self.pool.count, self.pool.send_data, self.pool.data_buffered,
                                self.pool.data_drain, metrics=self.metrics)
            self.pool.on_restart = lambda _index: self.hub.resync()
            self.hub.start()
        self._gc_task = asyncio.create_task(self._tune_gc(), name="gc-tune")
        if cfg.observability.http_port:
            from .obs.http import ObsServer

            self.http = ObsServer(self)
            await self.http.start(cfg.observability.http_host, cfg.observability.http_port)
        if lease_mode or le.enabled:
            if self.kube is None:
                from .kube.client import KubeClient

                self.kube = KubeClient.for_config(cfg, self.metrics, schedule=self.pool.qps_schedule)
        if lease_mode:
            self.shard_leases = make_shard_leases(cfg, self.kube, self.set_shards, self.metrics,
                                                  on_renewed=self._shard_holds)
            self.shard_leases.start()
        elif le.enabled:
            from .ha.leader import LeaderElector, LeaseLock

            self.elector = LeaderElector(
                LeaseLock(self.kube, cfg.resource_namespace, le.lease_name, _identity(cfg)),
                lease_duration=le.lease_duration, renew_deadline=le.renew_deadline, retry_period=le.retry_period,
                on_started_leading=lambda: self.pool.set_active(True, until=self.elector.valid_until),
                on_stopped_leading=lambda: self.pool.set_active(False), metrics=self.metrics,
                on_renewed=self.pool.set_lease_deadline)
            self.elector.start()
        if self.kube is None and cfg.sharding.shard_label and cfg.sharding.shards > 1:
            from .kube.client import KubeClient

            self.kube = KubeClient.for_config(cfg, self.metrics, schedule=self.pool.qps_schedule)
        self.labels = _shard_label_keeper(cfg, self.kube, self.metrics, self.log, lambda: self.shards.owned)
        self.webhook = await _start_webhook(cfg, self.metrics, self.kube, self.log)
        if not lease_mode and self.labels is not None and self.shards.owned:
            self.labels.request_relabel(self.shards.owned)

    def _shard_holds(self, until) -> None:
        """Shard hold deadlines renewed: the workers self-fence on them (no parent round trip)."""
        self.shards.set_deadlines(until)
        self.pool.set_shard_deadlines(until)

    def set_shards(self, owned) -> None:
        """Shard leases won / lost: the workers fence and replay, the hub re-routes and
        re-lists so the workers receive the runs of gained shards."""
        gained, lost = self.shards.update(owned)
        if gained and getattr(self, "labels", None) is not None:
            self.labels.request_relabel(gained)
        self.pool.set_shards(owned, self.shard_leases.deadlines() if self.shard_leases is not None else None)
        if self.hub is not None:
            self.hub.set_shards(self.shards)
            if gained or lost:
                asyncio.ensure_future(self.hub.resync())
        self.metrics.set("shards_owned", float(len(self.shards.owned or ())))

    def ready(self) -> bool:
        return self.pool.all_synced()

    async def wait_for_cache_sync(self, timeout: Optional[float] = None) -> bool:
        return await self.pool.wait_synced(timeout)

    async def refresh_metrics(self) -> Metrics:
        await self.pool.refresh_metrics()
        self.merged_metrics = self.pool.merged_metrics(self.metrics)
        return self.merged_metrics

    async def stop(self, drain_timeout: float = 10.0) -> None:
        if getattr(self, "labels", None) is not None:
            await self.labels.stop()
        if getattr(self, "webhook", None) is not None:
            await self.webhook.stop()
        if self.elector is not None:
            await self.elector.stop(release=True)
        if self.shard_leases is not None:
            await self.shard_leases.stop(release=True)
        if self.hub is not None:
            await self.hub.stop()
        if self._gc_task is not None:
            self._gc_task.cancel()
        self.gc_tuner.stop()
        if self._gpu_task is not None:
            self._gpu_task.cancel()
            try:
                await self._gpu_task
            except (asyncio.CancelledError, Exception):
                pass
        await self.pool.stop(drain_timeout)
        if self.telemetry is not None and self._owns_telemetry:
            self.telemetry.stop()
        self.merged_metrics = self.pool.merged_metrics(self.metrics)
        if self.http is not None:
            await self.http.stop()
        if self.kube is not None:
            await self.kube.close()
        self._stopped.set()

    async def run(self, stop: asyncio.Event) -> None:
        await self.start()
        await stop.wait()
        self.log.info("shutting down: draining worker processes")
        await self.stop()


def make_application(cfg: SupervisorConfig, **kw):
    """``Application`` or, with ``runtime.worker-processes`` > 1, ``ShardedApplication``."""
    if cfg.runtime.worker_processes > 1:
        return ShardedApplication(cfg, logger=kw.get("logger"), metrics=kw.get("metrics"), kube=kw.get("kube"))
    return Application(cfg, **kw)


def main(argv=None) -> int:
    """Process entry (``/root/reference/main.go:12-43``)."""
    cfg = load_config()
    log = configure_logging(cfg.log_level, static={"service": "nexus-supervisor"})
    metrics = Metrics(cfg.observability.statsd_name, {"version": __version__})
    metrics.statsd = DogStatsd.from_env(cfg.observability.statsd_name)
    log.v(1).info("configuration", config=redacted(cfg))
    rt = cfg.runtime
    if rt.cpu_affinity != "none":
        from .utils import affinity

        try:  # before any worker process starts: they inherit it
            placed = affinity.apply(affinity.plan(rt.cpu_affinity, 0, min_cpus=rt.worker_processes + 1,
                                                  busy=affinity.cpu_busy(0.25)))
        except OSError as exc:
            log.error(exc, "cpu placement not applied")
        else:
            log.info("cpu placement", **(placed or {"mode": "none (too few CPUs allowed)"}))

    async def amain() -> int:
        stop = asyncio.Event()
        loop = asyncio.get_running_loop()
        for sig in (signal.SIGTERM, signal.SIGINT):
            loop.add_signal_handler(sig, stop.set)
        if metrics.statsd is not None:
            metrics.statsd.attach(loop)
        try:
            app = make_application(cfg, logger=log, metrics=metrics)
        except Exception as exc:  # noqa: BLE001 - fatal init (klog.FlushAndExit analog)
            log.error(exc, "failed to initialise application services")
            return 1
        try:
            await app.run(stop)
        except Exception as exc:  # noqa: BLE001
            log.error(exc, "supervisor failed")
            return 1
        return 0

    try:
        return asyncio.run(amain())
    finally:
        if metrics.statsd is not None:
            metrics.statsd.close()
        shutdown_logging()


if __name__ == "__main__":
    sys.exit(main())
