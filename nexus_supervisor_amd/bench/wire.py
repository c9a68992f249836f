"""Wire-mode benchmark harness: supervisor (this process) ↔ fake kube-apiserver over
HTTP watch (cluster process) and ↔ native CQL server over TCP.

Process layout per rank::

    nexus-cqlsrv  ◄── CQL v4 ──  supervisor (rank process)  ── HTTP list/watch/DELETE ──►  cluster_proc
         ▲                                                                                  (apiserver +
         └──────────────────────────── CQL v4 (receiver inserts new rows) ───────────────── workload)

``cluster="per-rank"``: every rank runs its own CQL server and cluster process holding
only its shard's runs (N independent copies).  ``cluster="shared"`` (``bench.py``'s
default for N>1): rank 0 starts ONE CQL server and ONE cluster process (one apiserver)
holding every shard's runs; every rank's replica watches the whole namespace with
``sharding.shards = N`` and its hub drops the other replicas' runs — the cost of a
sharded replica filtering the shared stream is inside the measurement.
"""
from __future__ import annotations

import asyncio
import json
import os
import subprocess
import sys
import time
from typing import Any, Callable, Dict, List, Optional, Tuple

import aiohttp

from ..app import Application, ShardedApplication
from ..config.schema import SupervisorConfig
from ..kube.client import KubeClient, KubeConfig
from ..models.checkpoint import create_index_cql, create_table_cql
from ..store.cql import CqlCheckpointStore, CqlSession
from ..testing.cqlsrv import CqlServer
from ..utils.proc import die_with_parent


def schema_statements(ks: str = "nexus", table: str = "checkpoints") -> List[str]:
    return ([f"CREATE KEYSPACE IF NOT EXISTS {ks} WITH replication = {{'class': 'SimpleStrategy', 'replication_factor': 1}}",
             create_table_cql(ks, table)] + list(create_index_cql(ks, table)))


class WireHarness:
    store_name = "cql (nexus-cqlsrv over TCP)"
    # latency probe: the cluster answers a step this long after applying it (runner._latency_probe)
    probe_hold_ms = 10.0

    def __init__(self, sc: SupervisorConfig, cfg, workdir: str, telemetry=None,
                 share: Optional[Callable[[Any], Any]] = None, barrier: Optional[Callable[[], None]] = None):
        self.sc = sc
        self.telemetry = telemetry
        self.cfg = cfg
        self.workdir = workdir
        self.cql: CqlServer = None
        self.proc: subprocess.Popen = None
        self.app: Application = None
        self.ctl = ""
        self.http: aiohttp.ClientSession = None
        # node mode: ONE replica (this rank's) supervises every GPU slot of the node; the
        # cluster holds one workload per slot (slot k's pods on GPU k)
        self.node = getattr(cfg, "slot_mode", "replica") == "node" and cfg.world > 1
        self.shared = cfg.cluster == "shared" and cfg.world > 1 and not self.node
        self.share = share or (lambda obj: obj)
        self.barrier = barrier or (lambda: None)
        self.owner = not self.shared or cfg.rank == 0  # this rank runs the harness servers
        self.cql_port = 0
        self.readback: Optional[CqlCheckpointStore] = None

    async def _start_cluster(self) -> dict:
        cfg = self.cfg
        # a Scylla node is sharded (one shard per core): the store runs as a sharded node and
        # the replicas route every request to the owning shard (shard-aware driver); the
        # shared cluster gets a shard per rank, up to 8
        shards = max(2, min(8, cfg.world)) if self.shared else 2
        self.cql_shards = shards
        self.cql = CqlServer(exec_statements=schema_statements(), latency_us=cfg.cql_latency_us, shards=shards,
                             lwt_latency_us=cfg.cql_lwt_latency_us).start()
        ready = os.path.join(self.workdir, "cluster.ready")
        if os.path.exists(ready):
            os.unlink(ready)
        env = dict(os.environ, PYTHONPATH=os.pathsep.join(p for p in sys.path if p))
        self._log = open(os.path.join(self.workdir, "cluster.log"), "ab")
        # the apiserver's watch cache scales with the traffic it must hold (every shard's)
        history = 50_000 * (cfg.world if self.shared or self.node else 1)
        # the node agent process reads default pods' HIP OOM text from a kubelet-style
        # /var/log/pods the simulator writes (its LOG lines as CRI files)
        self.log_root = ""
        if cfg.gpu_evidence == "agent" and cfg.hbm_shape == "default-pod":
            self.log_root = os.path.join(self.workdir, "var-log-pods")
            os.makedirs(self.log_root, exist_ok=True)
        self.proc = subprocess.Popen([sys.executable, "-m", "nexus_supervisor_amd.bench.cluster_proc", "--cql",
                                      f"127.0.0.1:{self.cql.port}", "--ready-file", ready, "--history", str(history),
                                      # every rank's replica watches the shared namespace: fan out in parallel
                                      "--flush-threads", str(min(8, cfg.world) if self.shared else 3),
                                      "--api-latency-us", str(int(cfg.api_latency_us)),
                                      "--write-qps", str(float(cfg.api_write_qps)),
                                      "--log-root", self.log_root],
                                     env=env, stdout=self._log, stderr=self._log, start_new_session=True,
                                     preexec_fn=die_with_parent())
        deadline = time.monotonic() + 120
        while not os.path.exists(ready):
            if self.proc.poll() is not None or time.monotonic() > deadline:
                raise RuntimeError(f"cluster process failed to start (rc={self.proc.poll()})")
            await asyncio.sleep(0.05)
        with open(ready) as f:
            info = json.load(f)
        info["cql_port"] = self.cql.port
        async with aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=900)) as http:
            async with http.post(info["ctl"] + "/bench/init", json={
                    "jobs": cfg.jobs, "seed": cfg.seed, "rank": cfg.rank, "world": cfg.world, "shards": cfg.world,
                    "shard_indexes": list(range(cfg.world)) if self.shared else [cfg.rank],
                    "hip_oom_message": cfg.hip_oom_message,
                    "shard_label": self.sc.sharding.shard_label if self.shared else "",
                    "hbm_shape": cfg.hbm_shape, "run_starts": cfg.run_starts,
                    "node_slots": cfg.world if self.node else 0,
                    "pregen": cfg.warmup + cfg.steps if cfg.pregen else 0, "events": cfg.events}) as r:
                r.raise_for_status()
                await r.json()
        return info

    async def start(self) -> None:
        info = await self._start_cluster() if self.owner else None
        # diagnostic: start the replica this long after the harness (which of the two a
        # time-since-start effect follows)
        delay = float(os.environ.get("NEXUS_BENCH_DIAG_REPLICA_DELAY_S", "0") or 0)
        if delay > 0:
            await asyncio.sleep(delay)
        if self.shared:
            info = self.share(info)  # rank 0's harness addresses to every rank
        self.ctl = info["ctl"]
        self.api = info["api"]
        self.cql_port = info["cql_port"]
        self.sim_pid = info.get("sim_pid") if self.owner else None
        self.http = aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=600))
        sc = self.sc
        sc.cql_store_type = "scylla"
        sc.scylla_cql_store.hosts = [f"127.0.0.1:{self.cql_port}"]
        sc.scylla_cql_store.consistency = "LOCAL_QUORUM"
        if self.cfg.procs > 1:
            # process-per-core replica: the workers build their own clients from the config
            kcfg = os.path.join(self.workdir, "kubeconfig.yaml")
            with open(kcfg, "w") as f:
                json.dump({"apiVersion": "v1", "kind": "Config", "current-context": "bench",
                           "clusters": [{"name": "bench", "cluster": {"server": info["api"]}}],
                           "contexts": [{"name": "bench", "context": {"cluster": "bench", "user": "bench"}}],
                           "users": [{"name": "bench", "user": {}}]}, f)
            sc.kube_config_path = kcfg
            sc.runtime.worker_processes = self.cfg.procs
            via_agent = self.cfg.gpu_evidence == "agent"
            if not via_agent:
                # the rank's GPU monitor (owned by the runner) is mirrored into every worker
                sc.gpu.local_telemetry = True
                sc.gpu.backend = self.cfg.telemetry
            self.app = ShardedApplication(sc, report_decisions=True, log_dir=self.workdir,
                                          telemetry=None if via_agent else self.telemetry)
        else:
            kube = KubeClient(KubeConfig(info["api"]), max_connections=self.cfg.kube_connections)
            store = CqlCheckpointStore(CqlSession([("127.0.0.1", self.cql_port)],
                                                  connections_per_host=sc.scylla_cql_store.connections_per_host))
            self.app = Application(sc, kube=kube, store=store)
        await self.app.start()
        ok = await self.app.wait_for_cache_sync(120)
        if not ok:
            raise RuntimeError("informer caches did not sync")

    @property
    def supervisor(self):
        return self.app.supervisor

    async def step(self, events: int, respond_after_ms: float = 0.0, shard: Optional[int] = None):
        """One step: ``{"rids", "t_push", "expected", "started", "start_expected"}`` — in node
        mode one per GPU slot (a list), the slots' steps pushed concurrently."""
        if self.node and shard is None:
            return list(await asyncio.gather(*(self.step(events, respond_after_ms, k) for k in range(self.cfg.world))))
        body = {"events": events, "shard": self.cfg.rank if shard is None else shard}
        if respond_after_ms:
            body["respond_after_ms"] = respond_after_ms
        async with self.http.post(self.ctl + "/bench/step", json=body) as r:
            r.raise_for_status()
            return await r.json()

    async def oom(self, slot: int, message: Optional[str]) -> Dict[str, Any]:
        """A run of GPU slot ``slot`` dies of an HBM-OOM with the real ``message`` of that GPU."""
        async with self.http.post(self.ctl + "/bench/oom", json={"slot": slot, "message": message}) as r:
            r.raise_for_status()
            return await r.json()

    async def read_rows(self, algorithm: str, rids: List[str]) -> Dict[str, Any]:
        """Full rows (stage, cause, trace) of ``rids`` as the CQL server holds them."""
        if self.readback is None:
            self.readback = CqlCheckpointStore(CqlSession([("127.0.0.1", self.cql_port)], connections_per_host=2))
            await self.readback.connect()
        return {rid: await self.readback.read_checkpoint(algorithm, rid) for rid in rids}

    async def probe(self, n: int, rate_per_min: float, seed: int) -> List[Dict[str, Any]]:
        """The open-loop probe played by the cluster process (one request for all ``n``
        arrivals): each arrival's ``{"rids", "t_push", "expected"}``."""
        body = {"n": n, "rate_per_min": rate_per_min, "seed": seed, "shard": self.cfg.rank}
        budget = aiohttp.ClientTimeout(total=n / max(rate_per_min / 60.0, 1e-3) * 3 + 120)
        async with self.http.post(self.ctl + "/bench/probe", json=body, timeout=budget) as r:
            r.raise_for_status()
            doc = await r.json()
        return doc["steps"]

    algorithm = "bench-algorithm"

    async def read_stages(self, algorithm: str, rids: List[str]) -> Dict[str, Optional[str]]:
        """Rows as the CQL server holds them (the bench's read-back check)."""
        if self.readback is None:
            self.readback = CqlCheckpointStore(CqlSession([("127.0.0.1", self.cql_port)], connections_per_host=2))
            await self.readback.connect()
        out: Dict[str, Optional[str]] = {}

        async def one(rid):
            row = await self.readback.read_status(algorithm, rid)
            out[rid] = row.lifecycle_stage if row else None

        for i in range(0, len(rids), 512):
            await asyncio.gather(*(one(r) for r in rids[i:i + 512]))
        return out

    def replica_rss_mb(self) -> Dict[str, float]:
        """Resident memory of the replica: this (parent) process plus its shard workers."""
        def rss(pid):
            try:
                with open(f"/proc/{pid}/status") as f:
                    for line in f:
                        if line.startswith("VmRSS:"):
                            return int(line.split()[1]) / 1024.0
            except OSError:
                pass
            return 0.0
        pool = getattr(self.app, "pool", None)
        workers = sum(rss(p) for p in pool.pids()) if pool is not None else 0.0
        return {"replica_rss_mb": round(rss(os.getpid()) + workers, 1), "workers_rss_mb": round(workers, 1)}

    async def sync_metrics(self) -> None:
        refresh = getattr(self.app, "refresh_metrics", None)
        if refresh is not None:
            await refresh()

    def external_cpu(self):
        """CPU seconds used so far by the harness processes (utilisation diagnostics)."""
        out = {}
        procs = [("cluster", self.proc), ("cqlsrv", self.cql.proc if self.cql else None)]
        if getattr(self, "sim_pid", None):
            procs.append(("kubesim", type("P", (), {"pid": self.sim_pid})()))
        pool = getattr(self.app, "pool", None)
        if pool is not None:
            procs += [(f"worker{w.index}", w.proc) for w in pool.workers]
        for name, proc in procs:
            try:
                with open(f"/proc/{proc.pid}/stat") as f:
                    parts = f.read().rsplit(")", 1)[1].split()
                out[name] = (int(parts[11]) + int(parts[12])) / os.sysconf("SC_CLK_TCK")
                if name in ("kubesim", "cqlsrv"):  # kernel share: the native servers are syscall-bound
                    out[name + "_sys"] = int(parts[12]) / os.sysconf("SC_CLK_TCK")
            except (OSError, AttributeError, IndexError):
                pass
        return out

    async def sim_stats(self):
        """The apiserver simulator's counters (requests, event-loop iterations, send calls)."""
        try:
            async with self.http.get(self.api + "/sim/stats") as r:
                return await r.json(content_type=None)
        except Exception:  # noqa: BLE001 - diagnostics only
            return None

    async def stop(self) -> None:
        try:
            if self.app is not None:
                await self.app.stop(drain_timeout=5)
        finally:
            if self.readback is not None:
                await self.readback.close()
            if self.http is not None:
                await self.http.close()
            if self.shared:
                self.barrier()  # every rank's replica is down before the shared servers go
            if self.proc is not None and self.proc.poll() is None:
                self.proc.terminate()
                try:
                    self.proc.wait(10)
                except subprocess.TimeoutExpired:
                    self.proc.kill()
            if self.cql is not None:
                self.cql.stop()
            if getattr(self, "_log", None):
                self._log.close()
