"""Wire-mode benchmark harness: supervisor (this process) ↔ fake kube-apiserver over
HTTP watch (cluster process) and ↔ native CQL server over TCP.

Process layout per rank::

    nexus-cqlsrv  ◄── CQL v4 ──  supervisor (rank process)  ── HTTP list/watch/DELETE ──►  cluster_proc
         ▲                                                                                  (apiserver +
         └──────────────────────────── CQL v4 (receiver inserts new rows) ───────────────── workload)
"""
from __future__ import annotations

import asyncio
import json
import os
import subprocess
import sys
import time
from typing import List, Tuple

import aiohttp

from ..app import Application, ShardedApplication
from ..config.schema import SupervisorConfig
from ..kube.client import KubeClient, KubeConfig
from ..models.checkpoint import create_index_cql, create_table_cql
from ..store.cql import CqlCheckpointStore, CqlSession
from ..testing.cqlsrv import CqlServer


def schema_statements(ks: str = "nexus", table: str = "checkpoints") -> List[str]:
    return ([f"CREATE KEYSPACE IF NOT EXISTS {ks} WITH replication = {{'class': 'SimpleStrategy', 'replication_factor': 1}}",
             create_table_cql(ks, table)] + list(create_index_cql(ks, table)))


class WireHarness:
    store_name = "cql (nexus-cqlsrv over TCP)"

    def __init__(self, sc: SupervisorConfig, cfg, workdir: str, telemetry=None):
        self.sc = sc
        self.telemetry = telemetry
        self.cfg = cfg
        self.workdir = workdir
        self.cql: CqlServer = None
        self.proc: subprocess.Popen = None
        self.app: Application = None
        self.ctl = ""
        self.http: aiohttp.ClientSession = None

    async def start(self) -> None:
        self.cql = CqlServer(exec_statements=schema_statements(), latency_us=self.cfg.cql_latency_us).start()
        ready = os.path.join(self.workdir, "cluster.ready")
        if os.path.exists(ready):
            os.unlink(ready)
        env = dict(os.environ, PYTHONPATH=os.pathsep.join(p for p in sys.path if p))
        self._log = open(os.path.join(self.workdir, "cluster.log"), "ab")
        self.proc = subprocess.Popen([sys.executable, "-m", "nexus_supervisor_amd.bench.cluster_proc", "--cql",
                                      f"127.0.0.1:{self.cql.port}", "--ready-file", ready], env=env,
                                     stdout=self._log, stderr=self._log, start_new_session=True)
        deadline = time.monotonic() + 120
        while not os.path.exists(ready):
            if self.proc.poll() is not None or time.monotonic() > deadline:
                raise RuntimeError(f"cluster process failed to start (rc={self.proc.poll()})")
            await asyncio.sleep(0.05)
        with open(ready) as f:
            info = json.load(f)
        self.ctl = info["ctl"]
        self.api = info["api"]
        self.sim_pid = info.get("sim_pid")
        self.http = aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=600))
        async with self.http.post(self.ctl + "/bench/init", json={
                "jobs": self.cfg.jobs, "seed": self.cfg.seed, "rank": self.cfg.rank, "world": self.cfg.world,
                "shards": self.cfg.world, "shard_index": self.cfg.rank,
                "hip_oom_message": self.cfg.hip_oom_message,
                "pregen": self.cfg.warmup + self.cfg.steps if self.cfg.pregen else 0, "events": self.cfg.events}) as r:
            r.raise_for_status()
            await r.json()
        sc = self.sc
        sc.cql_store_type = "scylla"
        sc.scylla_cql_store.hosts = [f"127.0.0.1:{self.cql.port}"]
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
            # the rank's GPU monitor (owned by the runner) is mirrored into every worker
            sc.gpu.local_telemetry = True
            sc.gpu.backend = self.cfg.telemetry
            self.app = ShardedApplication(sc, report_decisions=True, log_dir=self.workdir, telemetry=self.telemetry)
        else:
            kube = KubeClient(KubeConfig(info["api"]), max_connections=self.cfg.kube_connections)
            store = CqlCheckpointStore(CqlSession([("127.0.0.1", self.cql.port)],
                                                  connections_per_host=sc.scylla_cql_store.connections_per_host))
            self.app = Application(sc, kube=kube, store=store)
        await self.app.start()
        ok = await self.app.wait_for_cache_sync(120)
        if not ok:
            raise RuntimeError("informer caches did not sync")

    @property
    def supervisor(self):
        return self.app.supervisor

    async def step(self, events: int) -> Tuple[List[str], float]:
        async with self.http.post(self.ctl + "/bench/step", json={"events": events}) as r:
            r.raise_for_status()
            doc = await r.json()
        return doc["rids"], doc["t_push"]

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
            if self.http is not None:
                await self.http.close()
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
