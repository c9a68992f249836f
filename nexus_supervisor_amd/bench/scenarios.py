"""BASELINE.json's five measurement configurations, each run at the reference's
processing limits (Helm defaults: 10 eps, burst 100, 2 workers — ``/root/reference/
.helm/values.yaml:153-161``) and uncapped.

====  =================================================================  =====================================
cfg   BASELINE.json config                                                here
====  =================================================================  =====================================
1     single OOMKilled pod → one checkpoint row (CPU plumbing)            HTTP watch + native CQL server; 20
                                                                          sequential single failures, latency
2     100 synthetic failing pods (OOMKilled/ImagePullBackOff mix),        one burst of 100, latency + drain rate
      1 replica
3     1×MI355X: 8 ROCm stress pods, HBM-OOM injected, per-GPU             GPU only (``--gpu``): 7 VRAM-holding
      attribution in the checkpoint                                       pods + 1 driven to a real HBM-OOM on
                                                                          the box's GPU; attribution + latency
3a    config 3 through the deployed path                                  no local telemetry; the node agent
                                                                          process (amd-smi, /var/log/pods) PATCHes
                                                                          the evidence annotation, the supervisor
                                                                          waits ``gpu.evidence-wait`` for it
4     1000 pod-fail events/min over 10k concurrent jobs, informer→CQL    open-loop at 1000/min for ``--seconds``
      p99                                                                 (1 slot here; 1/2/4/8 slots: bench.py)
5     2 replicas + leader election + 10k concurrent jobs + chaos          1000/min churn with a CQL node restart,
      (evictions, Scylla node restart)                                    an eviction storm and the leader dying
                                                                          without releasing its lease; failover
                                                                          time, p50/p99, every run's final stage
====  =================================================================  =====================================

Latency = failure pushed into the apiserver → checkpoint write acknowledged
(``stamps["ack_mono"]``), both ``time.monotonic()`` in this process.

    python -m nexus_supervisor_amd.bench.scenarios [--only 1,2,3a,4,5] [--gpu] [--json-out F]
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import sys
import time
from typing import Any, Dict, List, Optional

from ..app import Application
from ..config import load_config
from ..kube.client import KubeClient, KubeConfig
from ..models.decisions import Decision
from ..store.cql import CqlCheckpointStore, CqlSession
from ..testing.cqlsrv import CqlServer
from ..testing.fake_apiserver import FakeApiServer
from .wire import schema_statements
from .workload import Workload

PROFILES = {
    "reference": {"workers": 2, "rate-limit-elements-per-second": 10, "rate-limit-elements-burst": 100,
                  "kube-qps": 5, "kube-burst": 10},
    "uncapped": {"workers": 256, "rate-limit-elements-per-second": 0, "rate-limit-elements-burst": 1_000_000,
                 "kube-qps": 1_000_000, "kube-burst": 1_000_000},
}


def _pct(xs: List[float], p: float) -> Optional[float]:
    if not xs:
        return None
    s = sorted(xs)
    return round(s[min(len(s) - 1, int(round(p / 100.0 * (len(s) - 1))))], 3)


class AckClock:
    """First checkpoint ack of each pushed failure (any replica), as a decision hook; a
    run's start (ToRunning) is not its failure."""

    def __init__(self):
        self.pushed: Dict[str, float] = {}
        self.acked: Dict[str, float] = {}
        self.outcomes: Dict[str, str] = {}

    def __call__(self, d: Decision) -> None:
        rid = d.result.request_id
        if rid in self.acked or rid not in self.pushed:
            return
        if d.result.action == "ToRunning":
            return  # the run's start (lifecycle traffic), not the failure being timed
        if d.outcome in ("applied", "skipped-finished"):
            self.acked[rid] = d.result.stamps.get("ack_mono") or time.monotonic()
            self.outcomes[rid] = d.outcome

    def latencies_ms(self, rids=None) -> List[float]:
        rids = self.pushed.keys() if rids is None else rids
        return [(self.acked[r] - self.pushed[r]) * 1000.0 for r in rids if r in self.acked]

    async def wait(self, rids, timeout: float) -> bool:
        deadline = time.monotonic() + timeout
        while time.monotonic() < deadline:
            if all(r in self.acked for r in rids):
                return True
            await asyncio.sleep(0.01)
        return False


class Cluster:
    """Fake apiserver (HTTP) + native CQL server + ``replicas`` supervisor applications."""

    def __init__(self, jobs: int, profile: str, replicas: int = 1, leader_election: bool = False, seed: int = 0,
                 persist: bool = False, telemetry=None, shards: int = 0, gpu: Optional[Dict[str, Any]] = None):
        self.jobs, self.profile, self.replicas, self.le = jobs, profile, replicas, leader_election
        self.gpu = gpu or {}  # gpu.* overrides (the node-agent path: evidence-wait, no local telemetry)
        self.shards = shards  # > 0: runs split over this many shards held through per-shard Leases
        self.wl = Workload(concurrent_jobs=jobs, seed=seed)
        self.clock = AckClock()
        self.persist = persist
        self.telemetry = telemetry
        self.apps: List[Application] = []

    def _cfg(self, ident: str):
        over = {"cql-store-type": "scylla", "resync-period": "0s", "failure-rate-base-delay": "20ms",
                "failure-rate-max-delay": "500ms", "max-retries": 0,
                "scylla-cql-store": {"hosts": [f"127.0.0.1:{self.srv.port}"], "request-timeout": "1s"}}
        over.update(PROFILES[self.profile])
        if self.gpu:
            over["gpu"] = dict(self.gpu)
        if self.le or self.shards:
            over["leader-election"] = {"enabled": bool(self.le and not self.shards), "identity": ident,
                                       "lease-duration": "2s", "renew-deadline": "1500ms", "retry-period": "200ms"}
        if self.shards:
            over["sharding"] = {"shards": self.shards, "mode": "lease", "replicas": self.replicas}
        return load_config(path=None, env={}, overrides=over)

    async def start(self) -> None:
        self.srv = CqlServer(persist=self.persist, exec_statements=schema_statements()).start()
        self.api = FakeApiServer(bookmark_interval=0.5)
        self.url = await self.api.start()
        self.store = CqlCheckpointStore(CqlSession([self.srv.address], request_timeout=1.0))
        await self.store.connect()
        objs, rows = self.wl.initial()
        await self._write_rows(rows)
        for o in objs:
            self.api.create(o, copy_obj=False)
        for i in range(self.replicas):
            await self.add_replica(f"replica-{i}")

    async def add_replica(self, ident: str) -> Application:
        app = Application(self._cfg(ident), kube=KubeClient(KubeConfig(self.url)),
                          store=CqlCheckpointStore(CqlSession([self.srv.address], request_timeout=1.0)),
                          telemetry=self.telemetry)
        app.supervisor.decision_hooks.append(self.clock)
        await app.start()
        if not self.le and not self.shards:
            await app.supervisor.factory.wait_for_cache_sync(60)
        self.apps.append(app)
        return app

    async def _write_rows(self, rows) -> None:
        sem = asyncio.Semaphore(256)

        async def one(r):
            async with sem:
                for _ in range(100):
                    try:
                        await self.store.upsert_checkpoint(r)
                        return
                    except Exception:  # noqa: BLE001 - CQL node restarting (chaos)
                        await asyncio.sleep(0.05)

        await asyncio.gather(*(one(r) for r in rows))

    async def push(self, n: int, kinds=None) -> List[str]:
        failed, traffic, rows = self.wl.step(n, kinds)
        await self._write_rows(rows)
        t = time.monotonic()
        for rid in failed:
            self.clock.pushed[rid] = t
        for etype, obj in traffic:
            self.api.apply(etype, obj, copy_obj=False)
        return failed

    async def prime(self, n: int) -> None:
        """``n`` runs created and pending, so the next :meth:`push` can fail starting runs
        (image-pull, gpu-admission: a start failure needs a run that has not started)."""
        st = self.wl.create(n)
        await self._write_rows(st.rows)
        for etype, obj in st.traffic:
            self.api.apply(etype, obj, copy_obj=False)

    async def final_stages(self, rids) -> Dict[str, Any]:
        bad = []
        for rid in rids:
            row = await self.store.read_checkpoint(self.wl.algorithm, rid)
            if row is None or row.lifecycle_stage != self.wl.expected[rid]:
                bad.append([rid, row.lifecycle_stage if row else None, self.wl.expected[rid],
                            self.wl.kind_of.get(rid)])
        out: Dict[str, Any] = {"checked": len(rids), "wrong_stage": len(bad)}
        if bad:
            out["wrong_examples"] = bad[:5]
        return out

    def leader(self) -> Optional[Application]:
        act = [a for a in self.apps if a.supervisor.active]
        return act[0] if act else None

    def shard_owners(self) -> Dict[int, List[str]]:
        return {k: [a.cfg.leader_election.identity for a in self.apps if a.shard_leases and k in a.shard_leases.owned]
                for k in range(self.shards)}

    async def stop(self) -> None:
        for a in self.apps:
            await a.stop(drain_timeout=1.0)
        await self.store.close()
        await self.api.stop()
        self.srv.stop()


def _summary(name: str, profile: str, lat: List[float], events: int, seconds: float, **extra) -> Dict[str, Any]:
    out = {"config": name, "profile": profile, "events": events, "acked": len(lat),
           "p50_ms": _pct(lat, 50), "p99_ms": _pct(lat, 99), "max_ms": round(max(lat), 3) if lat else None,
           "events_per_s": round(len(lat) / seconds, 2) if seconds > 0 else None}
    out.update(extra)
    return out


async def cfg1_single(profile: str, n: int = 20) -> Dict[str, Any]:
    c = Cluster(jobs=50, profile=profile)
    await c.start()
    try:
        t0 = time.monotonic()
        for _ in range(n):
            rids = await c.push(1, kinds=["host-oom"])
            await c.clock.wait(rids, 30)
        dt = time.monotonic() - t0
        return _summary("1: single OOMKilled pod -> row", profile, c.clock.latencies_ms(), n, dt,
                        **(await c.final_stages(list(c.clock.pushed))))
    finally:
        await c.stop()


async def cfg2_burst(profile: str, n: int = 100) -> Dict[str, Any]:
    c = Cluster(jobs=1000, profile=profile)
    await c.start()
    try:
        # the start failures (image pulls, GPU admission rejections) need starting runs
        await c.prime(n)
        await asyncio.sleep(0.5)
        t0 = time.monotonic()
        # OOMKilled and ImagePullBackOff as the config names them, plus a share of pods the
        # kubelet refused because the device plugin could not allocate an amd.com/gpu
        kinds = ["host-oom"] * 9 + ["image-pull"] * 9 + ["gpu-admission"] * 2
        rids = await c.push(n, kinds=kinds)
        await c.clock.wait(rids, 120)
        dt = max(c.clock.acked.values()) - t0 if c.clock.acked else 0.0
        mix: Dict[str, int] = {}
        for r in rids:
            mix[c.wl.kind_of.get(r, "?")] = mix.get(c.wl.kind_of.get(r, "?"), 0) + 1
        return _summary("2: 100 failing pods (OOMKilled/ImagePullBackOff + GPU admission), 1 replica", profile,
                        c.clock.latencies_ms(), n, dt, kinds=mix, **(await c.final_stages(rids)))
    finally:
        await c.stop()


async def _open_loop(c: Cluster, rate_per_min: float, seconds: float, chaos=None) -> List[str]:
    interval = 60.0 / rate_per_min
    t0 = time.monotonic()
    rids: List[str] = []
    i = 0
    while True:
        due = t0 + i * interval
        if due - t0 >= seconds:
            break
        d = due - time.monotonic()
        if d > 0:
            await asyncio.sleep(d)
        if chaos is not None:
            await chaos(time.monotonic() - t0)
        rids += await c.push(1)
        i += 1
    return rids


async def cfg4_rate(profile: str, seconds: float = 30.0, rate: float = 1000.0, jobs: int = 10_000) -> Dict[str, Any]:
    c = Cluster(jobs=jobs, profile=profile)
    await c.start()
    try:
        t0 = time.monotonic()
        rids = await _open_loop(c, rate, seconds)
        ok = await c.clock.wait(rids, 120)
        dt = time.monotonic() - t0
        return _summary(f"4: {int(rate)} pod-fail/min, {jobs} concurrent jobs, 1 slot", profile, c.clock.latencies_ms(rids),
                        len(rids), dt, drained=ok, **(await c.final_stages(rids)))
    finally:
        await c.stop()


async def cfg5_chaos(profile: str, seconds: float = 30.0, rate: float = 1000.0, jobs: int = 10_000) -> Dict[str, Any]:
    c = Cluster(jobs=jobs, profile=profile, replicas=2, leader_election=True, persist=True)
    await c.start()
    marks: Dict[str, Any] = {}
    try:
        deadline = time.monotonic() + 30
        while c.leader() is None and time.monotonic() < deadline:
            await asyncio.sleep(0.05)

        async def chaos(t: float) -> None:
            if t >= seconds * 0.2 and "cql_restart" not in marks:
                marks["cql_restart"] = round(t, 2)
                c.srv.restart()
            if t >= seconds * 0.4 and "storm" not in marks:
                marks["storm"] = round(t, 2)
                await c.push(50, kinds=["evicted"])
            if t >= seconds * 0.6 and "leader_crash" not in marks:
                marks["leader_crash"] = round(t, 2)
                old = c.leader()
                if old is not None:
                    t_crash = time.monotonic()
                    await old.elector.stop(release=False)  # dies holding the lease
                    old.supervisor.active = False
                    c.apps.remove(old)
                    await old.stop(drain_timeout=0.2)
                    asyncio.ensure_future(_failover(t_crash))

        async def _failover(t_crash: float) -> None:
            while c.leader() is None:
                await asyncio.sleep(0.01)
            marks["failover_s"] = round(time.monotonic() - t_crash, 3)

        t0 = time.monotonic()
        rids = await _open_loop(c, rate, seconds, chaos)
        rids = list(c.clock.pushed)
        ok = await c.clock.wait(rids, 180)
        dt = time.monotonic() - t0
        return _summary(f"5: 2 replicas + leader election, {jobs} jobs, chaos", profile, c.clock.latencies_ms(rids),
                        len(rids), dt, drained=ok, chaos=marks, **(await c.final_stages(rids)))
    finally:
        await c.stop()


async def cfg5s_sharded_chaos(profile: str, seconds: float = 30.0, rate: float = 1000.0, jobs: int = 10_000,
                              replicas: int = 3, shards: int = 6) -> Dict[str, Any]:
    """Config 5 with horizontal scale: ``replicas`` replicas split the runs over ``shards``
    shard Leases (fair share ``ceil(shards / replicas)``); chaos = CQL node restart, an
    eviction storm, and a replica dying holding its shard Leases — its shards must move to
    the survivors, the replica's return must win its share back (rebalancing), and every
    run must still end in its expected stage."""
    c = Cluster(jobs=jobs, profile=profile, replicas=replicas, persist=True, shards=shards)
    await c.start()
    marks: Dict[str, Any] = {}
    try:
        deadline = time.monotonic() + 30

        def settled() -> bool:  # every shard owned once, and the shares balanced (rebalancing)
            own = c.shard_owners()
            per = [sum(1 for v in own.values() if a.cfg.leader_election.identity in v) for a in c.apps]
            return all(len(v) == 1 for v in own.values()) and max(per) - min(per) <= 1

        while not settled() and time.monotonic() < deadline:
            await asyncio.sleep(0.05)
        marks["initial_owners"] = c.shard_owners()

        async def chaos(t: float) -> None:
            if t >= seconds * 0.2 and "cql_restart" not in marks:
                marks["cql_restart"] = round(t, 2)
                c.srv.restart()
            if t >= seconds * 0.4 and "storm" not in marks:
                marks["storm"] = round(t, 2)
                await c.push(50, kinds=["evicted"])
            if t >= seconds * 0.6 and "replica_crash" not in marks:
                marks["replica_crash"] = round(t, 2)
                victim = next(a for a in c.apps if a.shard_leases.owned)
                lost = sorted(victim.shard_leases.owned)
                marks["crashed"] = {"replica": victim.cfg.leader_election.identity, "shards": lost}
                await victim.shard_leases.stop(release=False)  # dies holding its leases
                c.apps.remove(victim)
                await victim.stop(drain_timeout=0.2)
                asyncio.ensure_future(_failover(time.monotonic(), lost))
            if t >= seconds * 0.8 and "failover_s" in marks and "replica_return" not in marks:
                await _return(t)

        async def _return(t: float) -> None:
            # the crashed replica comes back (pod restarted): rebalancing hands it its share
            marks["replica_return"] = round(t, 2)
            marks["t_return"] = time.monotonic()
            await c.add_replica(marks["crashed"]["replica"])

        async def _failover(t_crash: float, lost) -> None:
            while any(not c.shard_owners()[k] for k in lost):
                await asyncio.sleep(0.01)
            marks["failover_s"] = round(time.monotonic() - t_crash, 3)
            marks["final_owners"] = c.shard_owners()

        t0 = time.monotonic()
        await _open_loop(c, rate, seconds, chaos)
        if "crashed" in marks and "replica_return" not in marks:
            deadline = time.monotonic() + 30
            while "failover_s" not in marks and time.monotonic() < deadline:
                await asyncio.sleep(0.05)
            await _return(round(time.monotonic() - t0, 2))
        rids = list(c.clock.pushed)
        ok = await c.clock.wait(rids, 180)
        dt = time.monotonic() - t0
        if "t_return" in marks:
            deadline = time.monotonic() + 30
            while not settled() and time.monotonic() < deadline:
                await asyncio.sleep(0.05)
            marks["rebalanced"] = settled()
            marks["rebalanced_owners"] = c.shard_owners()
            marks["rebalance_s"] = round(time.monotonic() - marks.pop("t_return"), 3)
        return _summary(f"5s: {replicas} replicas x {shards} shard leases, {jobs} jobs, chaos", profile,
                        c.clock.latencies_ms(rids), len(rids), dt, drained=ok, chaos=marks,
                        **(await c.final_stages(rids)))
    finally:
        await c.stop()


async def cfg3_gpu(profile: str, holders: int = 7, hold_gib: float = 30.0) -> Dict[str, Any]:
    """Real MI355X: ``holders`` pods keep ``hold_gib`` each resident on the GPU while one
    more pod allocates until HIP reports out-of-memory; its failure is pushed with the
    real termination message and must be checkpointed as hbm-oom on GPU 0."""
    import subprocess
    import tempfile

    from .._build import binary
    from ..gpu.telemetry import AmdSmiTelemetry

    exe = binary("gpu_stress")
    tel = AmdSmiTelemetry(interval=0.05)
    tel.start()
    c = Cluster(jobs=holders + 1, profile=profile, telemetry=tel)
    procs = []
    try:
        await c.start()
        runs = list(c.wl.live)
        env = dict(os.environ, HIP_VISIBLE_DEVICES="0")
        for _ in range(holders):
            procs.append(subprocess.Popen([exe, "hold", "--gib", str(hold_gib), "--seconds", "20"], env=env,
                                          stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL))
        await asyncio.sleep(4.0)  # holders resident
        log = os.path.join(tempfile.mkdtemp(prefix="cfg3-"), "termination.log")
        p = await asyncio.get_running_loop().run_in_executor(None, lambda: subprocess.run(
            [exe, "hbm-oom", "--chunk-gib", "4", "--linger", "0.5", "--termination-log", log, "--max-gib", "400"],
            env=env, capture_output=True, text=True, timeout=180))
        msg = open(log).read().strip() if os.path.exists(log) else ""
        victim = runs[-1]
        c.wl.hip_oom_message = msg or c.wl.hip_oom_message
        # fail exactly the victim run with the real termination message
        c.wl.live = [victim]
        failed, traffic, rows = c.wl.step(1, kinds=["hbm-oom"])
        t = time.monotonic()
        c.clock.pushed[victim] = t
        # (workload pods are local rank 0 of an 8-way job: expected GPU = visible device 0)
        for etype, obj in traffic:
            c.api.apply(etype, obj, copy_obj=False)
        await c.clock.wait([victim], 30)
        row = await c.store.read_checkpoint(c.wl.algorithm, victim)
        trace = json.loads(row.algorithm_failure_details) if row and (row.algorithm_failure_details or "").startswith("{") else {}
        g = ((trace.get("gpu") or {}).get("gpus") or [{}])[0]
        return _summary("3: 1xMI355X, 8 stress pods, real HBM-OOM", profile, c.clock.latencies_ms([victim]), 1, 1.0,
                        oom_rc=p.returncode, trace_class=trace.get("class"), gpu_index=g.get("index"),
                        vram_peak_mb=g.get("vram_peak_mb"), vram_total_mb=g.get("vram_total_mb"),
                        stage=row.lifecycle_stage if row else None)
    finally:
        for pr in procs:
            pr.kill()
            pr.wait(10)
        await c.stop()
        tel.stop()


async def cfg3_agent(profile: str, runs: int = 20, gpu: bool = True, evidence_wait: float = 2.0,
                     sample_interval: float = 0.5) -> Dict[str, Any]:
    """Config 3 through the production attribution path (the chart's deployment): the
    supervisor has **no** local GPU telemetry and holds a failed GPU pod's decision up to
    ``gpu.evidence-wait`` for the node agent's annotation; the agent is its own process
    (``python -m nexus_supervisor_amd agent``, amd-smi monitor at the production 0.5 s
    sample interval, ``/var/log/pods`` reader), watching the apiserver for its node's pods
    and merge-PATCHing ``nexus.amd.com/gpu-evidence``.

    ``runs`` default pods (``terminationMessagePolicy: File``: empty termination message,
    the HIP OOM text on stderr only) fail one after another; with ``gpu`` each is preceded
    by a real HIP OOM on the box's MI355X (``gpu_stress hbm-oom``) whose stderr becomes the
    pod's container log.  Latency: the pod's failure pushed into the apiserver → checkpoint
    write acknowledged, through watch → defer → agent watch → evidence → PATCH → watch →
    decision → CQL.  Reported with the share of decisions whose wait expired
    (``gpu_evidence_wait_expired``: written without the agent's evidence) and the pods/log
    reads the supervisor made (0: the agent read the log)."""
    import subprocess
    import tempfile

    from ..testing.fakelogs import write_cri_log
    from .agentproc import AgentProcess

    work = tempfile.mkdtemp(prefix="cfg3a-")
    logroot = os.path.join(work, "pods")
    os.makedirs(logroot)
    c = Cluster(jobs=runs + 8, profile=profile, gpu={
        "evidence-wait": f"{evidence_wait}s", "local-telemetry": False, "backend": "none"})
    c.wl.visible_devices = "0"  # the device plugin gave each pod GPU 0
    c.wl.hbm_shape = "default-pod"
    agent = None
    exe = None
    if gpu:
        from .._build import binary

        exe = binary("gpu_stress")
    try:
        await c.start()
        agent = await AgentProcess(c.url, work, c.wl._templates()[4], namespace=c.wl.ns,
                                   backend="amdsmi" if gpu else "fake", sample_interval=sample_interval,
                                   log_root=logroot).start()
        sup = c.apps[0].supervisor
        m0 = {k: sup.metrics.counter(k) for k in ("gpu_evidence_wait_expired", "decisions_deferred_for_gpu_evidence",
                                                    "decisions_awaited_gpu_evidence")}
        loop = asyncio.get_running_loop()
        rids, rcs, wrong, ooms = [], [], [], []
        t_start = time.monotonic()
        for i in range(runs):
            if gpu:
                p = await loop.run_in_executor(None, lambda: subprocess.run(
                    [exe, "hbm-oom", "--chunk-gib", "4", "--no-termination-log", "--linger", "0", "--max-gib", "400"],
                    env=dict(os.environ, HIP_VISIBLE_DEVICES="0"), capture_output=True, text=True, timeout=180))
                rcs.append(p.returncode)
                text = p.stderr
            else:
                text = f"epoch 3 step 1200 loss 0.412\n{c.wl.hip_oom_message}\n"
            rid = c.wl.live[-1]
            pod = c.wl.pods[rid]
            write_cri_log(logroot, c.wl.ns, pod["metadata"]["name"], pod["metadata"]["uid"], "algorithm", 0,
                          [("stderr", text)])
            st = c.wl.fail_with("hbm-oom", rid=rid)
            await c._write_rows(st.rows)
            c.clock.pushed[rid] = time.monotonic()
            for etype, obj in st.traffic:
                c.api.apply(etype, obj, copy_obj=False)
            await c.clock.wait([rid], evidence_wait + 30)
            rids.append(rid)
            row = await c.store.read_checkpoint(c.wl.algorithm, rid)
            trace = json.loads(row.algorithm_failure_details) if row and (row.algorithm_failure_details or "").startswith("{") else {}
            oom = trace.get("oom") or {}
            ooms.append(((trace.get("gpu") or {}).get("gpus") or [{}])[0])
            if not (row and row.lifecycle_stage == "FAILED" and trace.get("class") == "hbm-oom"
                    and oom.get("gpu_index") == 0 and any("node-log tail" in x for x in oom.get("signals") or ())):
                wrong.append({"rid": rid, "stage": row.lifecycle_stage if row else None, "class": trace.get("class"),
                              "oom": oom})
        dt = time.monotonic() - t_start
        m = {k: sup.metrics.counter(k) - v for k, v in m0.items()}
        am = await agent.metrics()
        return _summary(f"3a: 1xMI355X via the node agent, {runs} default pods, real HBM-OOM" if gpu else
                        f"3a: node agent (fake GPU backend), {runs} default pods", profile, c.clock.latencies_ms(rids),
                        runs, dt, via="node-agent", evidence_wait_s=evidence_wait, sample_interval_s=sample_interval,
                        oom_rcs=sorted(set(rcs)), wrong=len(wrong), wrong_examples=wrong[:3],
                        evidence_wait_expired=int(m["gpu_evidence_wait_expired"]),
                        evidence_wait_expired_share=round(m["gpu_evidence_wait_expired"] / max(1, runs), 4),
                        deferred_for_gpu_evidence=int(m["decisions_deferred_for_gpu_evidence"]),
                        job_decisions_awaited_evidence=int(m["decisions_awaited_gpu_evidence"]),
                        supervisor_pod_log_reads=len(c.api.log_requests),
                        agent_annotations=int(sum(v for k, v in am.items() if k.endswith("agent_annotations_total"))),
                        agent_cpu_s=round(agent.cpu_s(), 2),
                        rows_with_gpu_record=sum(1 for g in ooms if g.get("index") == 0),
                        vram_peak_mb=max((g.get("vram_peak_mb") or 0) for g in ooms) if ooms else None,
                        vram_total_mb=max((g.get("vram_total_mb") or 0) for g in ooms) if ooms else None)
    finally:
        if agent is not None:
            agent.stop()
        await c.stop()


CONFIGS = {"1": cfg1_single, "2": cfg2_burst, "3": cfg3_gpu, "3a": cfg3_agent, "4": cfg4_rate, "5": cfg5_chaos,
           "5s": cfg5s_sharded_chaos}


async def run_all(only: List[str], profiles: List[str], seconds: float, jobs: int, gpu: bool = False
                  ) -> List[Dict[str, Any]]:
    out = []
    for k in only:
        for prof in profiles:
            fn = CONFIGS[k]
            kw = {"seconds": seconds, "jobs": jobs} if k in ("4", "5", "5s") else {}
            if k == "3a":
                kw = {"gpu": gpu}  # without --gpu: the agent on the fake GPU backend
            t0 = time.monotonic()
            res = await fn(prof, **kw)
            res["wall_s"] = round(time.monotonic() - t0, 2)
            print(json.dumps(res), flush=True)
            out.append(res)
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--only", default="1,2,4,5,5s")
    ap.add_argument("--gpu", action="store_true", help="include config 3 (needs an MI355X)")
    ap.add_argument("--profiles", default="reference,uncapped")
    ap.add_argument("--seconds", type=float, default=30.0, help="duration of the open-loop configs 4 and 5")
    ap.add_argument("--jobs", type=int, default=10_000)
    ap.add_argument("--json-out", default="")
    args = ap.parse_args(argv)
    only = [x for x in args.only.split(",") if x]
    if args.gpu and "3" not in only:
        only.insert(2, "3")
    if args.gpu and "3a" not in only:
        only.insert(only.index("3") + 1, "3a")
    res = asyncio.run(run_all(only, args.profiles.split(","), args.seconds, args.jobs, args.gpu))
    if args.json_out:
        with open(args.json_out, "w") as f:
            json.dump(res, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
