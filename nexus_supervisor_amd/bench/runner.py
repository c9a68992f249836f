"""Per-rank benchmark driver (see ``bench.py``).

Harness protocol: ``start()``, ``step(events) -> {"rids", "t_push", "expected", "started",
"start_expected"}``, ``supervisor``, ``stop()``.  Times are ``time.monotonic()`` (CLOCK_MONOTONIC —
comparable across the rank and cluster processes on one host).
"""
from __future__ import annotations

import asyncio
import gc
import json
import os
import resource
import time
from dataclasses import dataclass
from typing import Any, Callable, Dict, List, Optional, Tuple

from ..config.schema import SupervisorConfig
from ..models.decisions import Decision
from ..obs.delivery import record as delivery_record
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
    step_timeout: float = float(os.environ.get("NEXUS_BENCH_STEP_TIMEOUT", "300"))
    cql_latency_us: int = 0
    api_latency_us: int = 0  # simulated apiserver answer latency of object requests (kubesim)
    api_write_qps: float = 0.0  # APF-like cap on the simulator's mutating requests (429 + Retry-After)
    cql_lwt_latency_us: int = -1  # extra latency of a conditional write (Paxos); -1 = 3 x cql_latency_us
    fused_write: str = "auto"  # compat.fused-write: auto | true | false (the reference's read + write)
    conditional_update: str = "auto"  # compat.conditional-update
    pprof_out: str = ""
    kube_connections: int = 256
    inflight: int = 2
    probe_events: int = 600
    probe_rate_per_min: float = 1000.0
    probe_timeline: bool = False  # diagnostic: CPU of every process (and the host) per second of the probe
    step_timeline: bool = False  # diagnostic: the same over the timed steps, and which process paced them
    procs: int = 1  # supervisor shard-worker processes (runtime.worker-processes)
    pregen: bool = True  # cluster pre-generates the synthetic steps' traffic before the timed region
    cluster: str = "per-rank"  # per-rank | shared (one apiserver + one CQL server for all ranks)
    pprof_hz: int = 199
    # client-side API bucket (kube-qps; the uncapped profile sets it high so the limiter's
    # path runs without pacing, the reference profile uses client-go's 5 / 10)
    kube_qps: float = 1_000_000.0
    # shared cluster: the runs carry their shard as a label and every replica watches only
    # its shard's Pods / Jobs (sharding.shard-label); "" = every replica gets the whole stream
    shard_label: str = "nexus.amd.com/shard"
    # how the synthetic HBM-OOMs look: "default-pod" (empty termination message, the HIP text
    # in the container log: the supervisor reads pods/log) or "termination-message"
    hbm_shape: str = "default-pod"
    # new runs go Pending -> Running with the kubelet's Events (a ToRunning decision each);
    # False: the failure-only shape of round 4
    run_starts: bool = True
    # "replica": one replica (and GPU monitor) per GPU slot, each with its own shard; "node":
    # ONE replica and ONE monitor on rank 0 supervise every slot of the node (the production
    # shape: an HA supervisor and one node agent), the other ranks only run their GPU's work
    slot_mode: str = "replica"
    # "local": the supervisor reads the rank's GPU monitor in-process; "agent": the node agent
    # process annotates failed pods and the supervisor waits gpu.evidence-wait for it
    gpu_evidence: str = "local"
    evidence_wait: float = 2.0

    @property
    def node(self) -> bool:
        return self.slot_mode == "node" and self.world > 1


def supervisor_config(cfg: BenchConfig) -> SupervisorConfig:
    sc = SupervisorConfig()
    sc.cql_store_type = "memory"
    sc.resource_namespace = "nexus"
    if cfg.profile == "reference":
        sc.workers, sc.rate_limit_elements_per_second, sc.rate_limit_elements_burst = 2, 10, 100
        sc.kube_qps, sc.kube_burst = 5.0, 10
    else:
        sc.workers, sc.rate_limit_elements_per_second, sc.rate_limit_elements_burst = cfg.workers, 0, 1_000_000
        sc.kube_qps, sc.kube_burst = cfg.kube_qps, max(1, int(min(cfg.kube_qps, 1_000_000)))
    sc.sharding.shards = 1 if cfg.node else cfg.world
    sc.sharding.shard_index = 0 if cfg.node else cfg.rank
    if cfg.cluster == "shared" and cfg.world > 1:
        sc.sharding.shard_label = cfg.shard_label
    sc.resync_period = 0.0
    sc.rules.stale_event_grace = 5.0
    sc.observability.stage_timestamps = True
    sc.scylla_cql_store.connections_per_host = 2
    sc.compat.fused_write = cfg.fused_write
    sc.compat.conditional_update = cfg.conditional_update
    if cfg.gpu_evidence == "agent":
        sc.gpu.evidence_wait = cfg.evidence_wait
        sc.gpu.local_telemetry = False
        sc.gpu.backend = "none"
    return sc


_RUNNING = "RUNNING"
# supervisor counters of the node-agent evidence path (the timed region's growth)
_EVIDENCE_COUNTERS = ("decisions_deferred_for_gpu_evidence", "gpu_evidence_wait_expired", "decisions_awaited_gpu_evidence")


class Tracker:
    """Decision hook: checkpoint-ack time per run; latency = ack − push.

    Two decisions are tracked per step: each failed run's failure decision (the north-star
    latency, pod-fail → checkpoint) and each started run's ``ToRunning`` (Started →
    ``RUNNING``).  A report is matched to one or the other by the stage it wrote, so a run
    started in one step and failed in a later one — both possibly in flight — is tracked
    twice.  Several steps may be in flight at once (the generator runs ahead of the
    supervisor, as a live cluster would); each step completes when every decision it
    carries has been acknowledged by the store.  Every acknowledged decision is checked
    against the stage the workload expects (``wrong_stage``), and the timed runs are
    remembered for the read-back check against the store afterwards."""

    def __init__(self):
        self.acks: Dict[Tuple[str, bool], Tuple[float, str, Optional[str], Any]] = {}
        self.owner: Dict[Tuple[str, bool], "StepState"] = {}
        self.latencies: List[float] = []        # failures: pod-fail push → checkpoint ack
        self.start_latencies: List[float] = []  # starts: Started push → RUNNING ack
        self.errors = 0
        self.wrong_stage = 0
        self.wrong_examples: List[Tuple[str, Optional[str], str]] = []
        self.checked: Dict[str, str] = {}  # timed run → expected final stage (read-back)
        self.record = False
        self.failures = 0  # recorded decisions acknowledged
        self.starts = 0
        self.superseded = 0  # starts whose run's failure was decided first
        self.failed_rids: set = set()
        # recorded decisions' push→ack decomposition (ms): api (push → hub read), hub (→ worker
        # frame), feed (→ decoded), dispatch (→ handler), classify (handler → enqueue, with any
        # log-tail wait), queue (→ dequeue), actuate (→ checkpoint ack)
        self.parts: List[Tuple[float, ...]] = []
        self.pushed_at: List[Tuple[float, str]] = []  # (push time, run) of each entry of ``latencies``
        self.part_of: Dict[str, Tuple[float, ...]] = {}  # run -> its entry of ``parts`` (by-kind report)
        self.by_rid = False  # fill part_of (the latency probe only)

    def __call__(self, d: Decision):
        s = d.result.stamps
        x = None
        dl = s.get("delivery")
        if dl is not None and "ack" in s and "receive" in s:
            x = delivery_record(s, dl)
        self.report(d.result.request_id, d.outcome, s.get("ack_mono"), d.new_stage, x)

    def report(self, rid: str, outcome: str, ack: Optional[float], stage: Optional[str], x=None) -> None:
        # the metric is pod-fail → checkpoint *write ack* (the Job DELETE follows the write)
        t = ack or time.monotonic()
        key = (rid, stage == _RUNNING)
        if not key[1]:
            # the run's failure was decided: a start still waiting for its ToRunning is
            # superseded (a finished row suppresses a later ToRunning — IsFinished, as in the
            # reference — when the failure overtook the Started Event on another stream)
            self.failed_rids.add(rid)
            sst = self.owner.pop((rid, True), None)
            if sst is not None:
                sst.supersede(self, (rid, True))
        st = self.owner.pop(key, None)
        if st is None:
            # raced ahead of the step response (or a duplicate: the pod-status rule's ToRunning
            # behind the Started Event's) — keep the applied one
            prev = self.acks.get(key)
            if prev is None or prev[1] != "applied":
                self.acks[key] = (t, outcome, stage, x)
            return
        st.settle(self, key, t, outcome, stage, x)

    def arm(self, rids: List[str], t_push: float, expected: Optional[Dict[str, str]] = None,
            started: Optional[List[str]] = None, start_expected: Optional[Dict[str, str]] = None) -> "StepState":
        expected = dict(expected or {})
        keys = [(r, False) for r in rids]
        for r in started or ():
            keys.append((r, True))
            expected.setdefault(r, (start_expected or {}).get(r, _RUNNING))
        st = StepState(set(keys), t_push, self.record, expected or {})
        if self.record:
            for r in started or ():
                self.checked[r] = _RUNNING
            for r in rids:
                if r in expected:
                    self.checked[r] = expected[r]
        for key in keys:
            a = self.acks.pop(key, None)
            if a is not None:
                st.settle(self, key, *a)
            elif key[1] and key[0] in self.failed_rids:
                st.supersede(self, key)
            else:
                self.owner[key] = st
        if not st.waiting:
            st.done.set()
        return st

    def abandon(self, st: "StepState") -> None:
        import sys

        print(f"[bench] step abandoned: {len(st.waiting)} decisions never acknowledged, e.g. "
              f"{sorted(st.waiting)[:5]}", file=sys.stderr, flush=True)
        self.errors += len(st.waiting)
        for key in st.waiting:
            self.owner.pop(key, None)
        st.waiting.clear()
        st.done.set()


class StepState:
    __slots__ = ("waiting", "t_push", "record", "done", "expected")

    def __init__(self, waiting, t_push, record, expected):
        self.waiting = waiting
        self.t_push = t_push
        self.record = record
        self.expected = expected
        self.done = asyncio.Event()

    def supersede(self, tr: Tracker, key) -> None:
        self.waiting.discard(key)
        tr.superseded += 1
        if not self.waiting:
            self.done.set()

    def settle(self, tr: Tracker, key, t: float, outcome: str, stage: Optional[str] = None, x=None) -> None:
        self.waiting.discard(key)
        rid, start = key
        want = _RUNNING if start else self.expected.get(rid)
        if outcome != "applied":
            tr.errors += 1
        else:
            if want is not None and stage != want:
                tr.wrong_stage += 1
                if len(tr.wrong_examples) < 5:
                    tr.wrong_examples.append((rid, stage, want))
            if self.record:
                total = (t - self.t_push) * 1000.0
                if start:
                    tr.starts += 1
                    tr.start_latencies.append(total)
                else:
                    tr.failures += 1
                    tr.latencies.append(total)
                    tr.pushed_at.append((self.t_push, rid))
                    if x is not None and len(x) >= 6:
                        hub, feed, dec, cls, que, r2c = x[:6]
                        part = (total, (hub - self.t_push) * 1e3, (feed - hub) * 1e3, (dec - feed) * 1e3,
                                (t - r2c - dec) * 1e3, cls * 1e3, que * 1e3, (r2c - cls - que) * 1e3)
                        tr.parts.append(part)
                        if tr.by_rid:
                            tr.part_of[rid] = part
        if not self.waiting:
            self.done.set()


class InProcHarness:
    store_name = "memory (in-process)"

    def __init__(self, sc: SupervisorConfig, cfg: BenchConfig):
        from ..store.memory import MemoryStore
        from ..testing.inproc import InProcCluster

        self.wl = Workload(cfg.jobs, rank=cfg.rank, world=cfg.world, seed=cfg.seed,
                           hip_oom_message=cfg.hip_oom_message or DEFAULT_HIP_OOM, shards=cfg.world, shard_index=cfg.rank,
                           run_starts=cfg.run_starts)
        objs, rows = self.wl.initial()
        self.store = MemoryStore(rows)
        self.cluster = InProcCluster(sc, self.store, objs)
        self.supervisor = self.cluster.supervisor

    async def start(self):
        await self.cluster.start()

    async def step(self, events: int):
        st = self.wl.step(events)
        for r in st.rows:
            self.store.rows[r.key] = r
        t = time.monotonic()
        for etype, obj in st.traffic:
            if etype != "LOG":
                self.cluster.push(obj, etype)
        return st.doc(t)

    async def read_stages(self, algorithm: str, rids: List[str]) -> Dict[str, Optional[str]]:
        out = {}
        for rid in rids:
            row = self.store.get(algorithm, rid)
            out[rid] = row.lifecycle_stage if row else None
        return out

    @property
    def algorithm(self) -> str:
        return self.wl.algorithm

    async def stop(self):
        await self.cluster.stop()

    def external_cpu(self):
        return {}


def _dump_tasks_on_sigusr2() -> None:
    """Diagnostics: ``kill -USR2 <rank pid>`` prints every pending asyncio task's stack."""
    import signal
    import sys

    def dump():
        for t in asyncio.all_tasks():
            print(f"--- task {t.get_name()}", file=sys.stderr)
            t.print_stack(limit=8, file=sys.stderr)

    try:
        asyncio.get_running_loop().add_signal_handler(signal.SIGUSR2, dump)
    except (NotImplementedError, RuntimeError):  # pragma: no cover - non-Unix / no loop
        pass


def monitor_cost(telemetry, seconds: float = 2.0) -> Optional[Dict[str, Any]]:
    """CPU of the GPU monitor per sample (this process otherwise idle): what one node
    agent's sampling of every local GPU costs."""
    s0 = getattr(telemetry, "samples", None)
    if not isinstance(s0, int):
        return None
    c0 = time.process_time()
    time.sleep(seconds)
    n = telemetry.samples - s0
    if n <= 0:
        return None
    return {"gpus": len(telemetry.devices()), "samples": n, "interval_ms": round(1000 * telemetry.interval, 1),
            "cpu_us_per_sample": round((time.process_time() - c0) * 1e6 / n, 1)}


async def run_slot(cfg: BenchConfig, barrier_sync: Callable[[], None],
                   oom_phase: Optional[Callable[[], Any]] = None) -> Dict[str, Any]:
    """Node mode, ranks > 0: the GPU slot's own work only (its real HBM-OOM in the
    attribution phase); the collectives mirror rank 0's :func:`run_rank`."""
    barrier_sync()  # timed region starts
    barrier_sync()  # ... and ends
    if oom_phase is not None:
        await asyncio.get_running_loop().run_in_executor(None, oom_phase)
    return {"elapsed": 0.0, "events": 0, "errors": 0, "failures": 0, "starts": 0, "start_latencies_ms": [],
            "watch_objects_per_failure": None, "wrong_stage": 0, "wrong_examples": [], "readback": {"checked": 0},
            "latencies_ms": [], "store": None, "workers": 0, "actuation": None, "eps": None, "kube_qps": None,
            "telemetry": None, "stages": {}, "cpu": {}, "probe": None, "step_done_ms": []}


async def _node_attribution(harness, tracker: "Tracker", telemetry, ooms: List[Dict[str, Any]],
                            cfg: "BenchConfig") -> Dict[str, Any]:
    """Every slot's GPU ran out of HBM at about the same time (a real OOM on an MI355X, or the
    synthetic text on CPU); one run per slot dies with its slot's message.  The single
    replica must write each as hbm-oom on the *physical* GPU of that slot."""
    from ..gpu.telemetry import FakeTelemetry

    if isinstance(telemetry, FakeTelemetry):  # CPU: each slot's GPU filled for the monitor
        for o in ooms:
            telemetry.set_vram(o["slot"], int(telemetry.devices()[o["slot"]]["vram_total_mb"] * 0.99))
    saved, tracker.latencies = tracker.latencies, []
    states, slot_of = [], {}
    for o in sorted(ooms, key=lambda x: x["slot"]):
        d = await harness.oom(o["slot"], o.get("message"))
        for rid in d["rids"]:
            slot_of[rid] = o["slot"]
        states.append(tracker.arm(d["rids"], d["t_push"], d.get("expected")))
    for st in states:
        try:
            await asyncio.wait_for(st.done.wait(), cfg.step_timeout)
        except asyncio.TimeoutError:
            tracker.abandon(st)
    lat = tracker.latencies
    tracker.latencies = saved
    rows = await harness.read_rows(harness.algorithm, list(slot_of))
    per = []
    for rid, slot in sorted(slot_of.items(), key=lambda kv: kv[1]):
        row = rows.get(rid)
        trace = {}
        try:
            trace = json.loads(row.algorithm_failure_details) if row is not None else {}
        except ValueError:
            pass
        g = (trace.get("oom") or {}).get("gpu_index")
        per.append({"slot": slot, "stage": row.lifecycle_stage if row else None, "class": trace.get("class"),
                    "gpu_index": g, "correct": g == slot and trace.get("class") == "hbm-oom",
                    "real_oom": bool(next((o for o in ooms if o["slot"] == slot), {}).get("real"))})
    out = {"slots": len(per), "correct": sum(1 for p in per if p["correct"]), "per_slot": per}
    if lat:
        ls = sorted(lat)
        out["p50_ms"] = round(ls[len(ls) // 2], 3)
        out["max_ms"] = round(ls[-1], 3)
    return out


async def run_rank(cfg: BenchConfig, barrier_sync: Callable[[], None],
                   share: Optional[Callable[[Any], Any]] = None,
                   oom_phase: Optional[Callable[[], Any]] = None) -> Dict[str, Any]:
    """One rank of the bench.  ``share(obj)`` returns rank 0's ``obj`` on every rank (the
    shared-cluster rendezvous); ``barrier_sync`` brackets the timed region.  Node mode
    (``cfg.node``): rank 0 runs the one replica and monitor for every slot; ``oom_phase``
    (a collective: each rank's real OOM on its GPU) feeds the per-GPU attribution check."""
    from ..gpu.telemetry import FakeTelemetry, make_telemetry, pod_evidence_provider

    _dump_tasks_on_sigusr2()
    if cfg.node and cfg.rank != 0:
        return await run_slot(cfg, barrier_sync, oom_phase)
    sc = supervisor_config(cfg)
    via_agent = cfg.gpu_evidence == "agent"
    # agent mode: the real monitor is the agent's (its own process); the runner's is a stand-in
    telemetry = make_telemetry(cfg.telemetry) if cfg.telemetry != "fake" and not via_agent else FakeTelemetry()
    telemetry.start()
    monitor = await asyncio.get_running_loop().run_in_executor(None, monitor_cost, telemetry)
    if cfg.transport == "inproc":
        harness = InProcHarness(sc, cfg)
    else:
        from .wire import WireHarness

        harness = WireHarness(sc, cfg, cfg.workdir, telemetry=telemetry, share=share, barrier=barrier_sync)
    tracker = Tracker()
    sampler = None
    agent = None
    beat = None
    try:
        await harness.start()
        sup = harness.supervisor
        if via_agent:
            from .agentproc import AgentProcess

            agent = await AgentProcess(harness.api, cfg.workdir, f"mi355x-{cfg.rank // 8:03d}", namespace=sc.resource_namespace,
                                       backend="amdsmi" if cfg.telemetry == "amdsmi" else "fake",
                                       kube_qps=sc.kube_qps, kube_burst=sc.kube_burst,
                                       log_root=getattr(harness, "log_root", "") or None).start()
            ev0 = {k: sup.metrics.counter(k) for k in _EVIDENCE_COUNTERS}
        else:
            sup.classifier.evidence_provider = pod_evidence_provider(telemetry)
        if hasattr(sup, "report_hooks"):  # worker processes: their decision reports as plain tuples
            sup.report_hooks.append(tracker.report)
        else:
            sup.decision_hooks.append(tracker)

        done_at: List[float] = []  # completion time of each timed step (diagnostics)

        async def run_steps(n: int) -> None:
            """Push ``n`` steps with at most ``cfg.inflight`` unacknowledged at a time."""
            pending: List[StepState] = []

            async def finish(st: StepState) -> None:
                try:
                    await asyncio.wait_for(st.done.wait(), cfg.step_timeout)
                except asyncio.TimeoutError:
                    tracker.abandon(st)
                if tracker.record:
                    done_at.append(time.perf_counter())

            for _ in range(n):
                while len(pending) >= cfg.inflight:
                    for st in pending.pop(0):
                        await finish(st)
                docs = await harness.step(cfg.events)
                pending.append([tracker.arm(d["rids"], d["t_push"], d.get("expected"), d.get("started"),
                                            d.get("start_expected")) for d in (docs if isinstance(docs, list) else [docs])])
            for sts in pending:
                for st in sts:
                    await finish(st)

        phase = {"name": "warmup", "t0": time.monotonic()}

        async def heartbeat() -> None:
            # a progress line every 15 s on stderr: long runs (a soak of hundreds of steps, a
            # read-back of a million rows) stay visibly alive to whatever supervises them
            import sys as _sys

            while True:
                await asyncio.sleep(15.0)
                print(f"[bench] {phase['name']} {time.monotonic() - phase['t0']:.0f}s: {len(done_at)} timed steps "
                      f"done, {tracker.failures} failures acked", file=_sys.stderr, flush=True)

        beat = asyncio.ensure_future(heartbeat())
        await run_steps(cfg.warmup)
        phase.update(name="timed", t0=time.monotonic())
        gc.collect()
        tracker.errors = tracker.wrong_stage = 0
        tracker.wrong_examples.clear()
        tracker.record = True
        if cfg.pprof_out:
            from ..obs.pprof import Sampler

            sampler = Sampler(hz=cfg.pprof_hz).start()
            pool = getattr(getattr(harness, "app", None), "pool", None)
            if pool is not None:  # shard workers profile themselves over the same window
                pool.broadcast({"op": "pprof", "on": True, "hz": cfg.pprof_hz})
        barrier_sync()
        pool = getattr(getattr(harness, "app", None), "pool", None)
        r0 = getattr(pool, "report_cpu_s", 0.0)
        t0 = time.perf_counter()
        c0 = time.process_time()
        a0 = agent.cpu_s() if agent is not None else 0.0
        x0 = harness.external_cpu()
        sim_stats = getattr(harness, "sim_stats", None)
        s0 = await sim_stats() if sim_stats is not None else None
        step_tl = (_CpuTimeline(harness, interval=0.2, sim=True)
                   if cfg.step_timeline and hasattr(harness, "external_cpu") else None)
        if step_tl is not None:
            step_tl.start()
        await run_steps(cfg.steps)
        if step_tl is not None:
            await step_tl.stop()
        barrier_sync()
        elapsed = time.perf_counter() - t0
        timed = (tracker.failures, tracker.starts, list(tracker.start_latencies))
        step_done_ms = [round(1000.0 * (t - t0), 1) for t in done_at]
        step_timeline = None
        if step_tl is not None:
            # t0 of the rows: the timed region's start on the monotonic clock
            mono0 = time.monotonic() - (time.perf_counter() - t0)
            rows = step_tl.report(mono0)
            step_timeline = {"rows": rows, "steady": steady_util(rows, step_done_ms)}
        cpu = {"supervisor_util": round((time.process_time() - c0) / elapsed, 3),
               "supervisor_max_rss_mb": round(resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1024.0, 1)}
        x1 = harness.external_cpu()
        if agent is not None:  # the node agent: product code, not harness
            cpu["agent_util"] = round((agent.cpu_s() - a0) / elapsed, 3)
            cpu["agent_cpu_us_per_event"] = round((agent.cpu_s() - a0) * 1e6 / max(1, cfg.events * cfg.steps), 1)
        for k in x1:
            cpu[f"{k}_util"] = round((x1[k] - x0.get(k, 0.0)) / elapsed, 3)
        s1 = await sim_stats() if s0 else None
        if os.environ.get("NEXUS_BENCH_DEBUG"):
            print("[bench] sim stats", s0, s1, file=__import__("sys").stderr)
        watch_objects = None
        if s0 and s1:
            # shared cluster: the simulator serves every rank's failures
            # shared cluster / node mode: the simulator serves every slot's failures
            n_ev = max(cfg.events * cfg.steps * (cfg.world if getattr(harness, "shared", False) or cfg.node else 1), 1)
            for k in ("requests", "loops", "sends"):
                cpu[f"kubesim_{k}_per_event"] = round((s1.get(k, 0) - s0.get(k, 0)) / n_ev, 3)
            # every committed change (ADDED / MODIFIED / DELETED of an Event, Pod or Job — the
            # supervisor's own Job DELETEs and their pod GC included) bumps the resourceVersion:
            # the watch objects the namespace carried per pod failure
            if "rv" in s1 and "rv" in s0:
                watch_objects = (s1["rv"] - s0["rv"]) / n_ev
            # event-loop phases (µs per pod failure): busy = everything but epoll_wait;
            # request includes apply (the synthetic traffic injection)
            for k in ("busy", "apply", "prepare", "request", "recv", "flush"):
                if f"{k}_ns" in s1:
                    cpu[f"kubesim_{k}_us_per_event"] = round((s1[f"{k}_ns"] - s0.get(f"{k}_ns", 0)) / 1000.0 / n_ev, 2)
            if "busy_ns" in s1:
                # the simulator's serial parts over the timed region: its event loop's busy share,
                # its apply port's, and the store lock's hold time (the loop and the apply port
                # both commit under it) — the largest is what saturates first
                share = {k: round((s1.get(f"{k}_ns", 0) - s0.get(f"{k}_ns", 0)) / 1e9 / elapsed, 3)
                         for k in _SIM_SERIAL if k != "gc" or "gc_ns" in s1}
                c0, c1 = s0.get("apply_conn_ns"), s1.get("apply_conn_ns")
                if c1:
                    # each apply connection is one thread: the busiest one is the serial part
                    # (node mode has one generator connection per slot; their sum is not)
                    share["apply_thread"] = round(max(v - (c0 or {}).get(k, 0) for k, v in c1.items()) / 1e9 / elapsed, 3)
                cpu["kubesim_loop_util"] = share["busy"]
                cpu["kubesim_apply_port_util"] = share["apply_thread"]
                cpu["kubesim_store_util"] = share["store"]
                if "gc" in share:  # --async-gc: the GC thread deleting the Jobs' pods
                    cpu["kubesim_gc_util"] = share["gc"]
                cpu["kubesim_serial_util"] = max(share.values())
        if getattr(harness, "cql_shards", None):
            cpu["cqlsrv_shards"] = harness.cql_shards
        workers = [v for k, v in cpu.items() if k.startswith("worker")]
        if workers:
            cpu["workers_util_sum"] = round(sum(workers), 3)
        # supervisor CPU per pod failure: the replica's processes (coordinating parent — here
        # also the bench driver — plus its shard workers), whole-run CPU seconds ÷ failures.
        # The decision-report channel (workers → parent → tracker; it exists only so the bench
        # can time every decision) is measured in the parent and reported on its own line
        n_ev = max(cfg.events * cfg.steps * (cfg.world if cfg.node else 1), 1)  # node mode: every slot's
        report_s = getattr(pool, "report_cpu_s", 0.0) - r0
        cpu["bench_report_cpu_us_per_event"] = round(report_s * 1e6 / n_ev, 1)
        sup_cpu = cpu["supervisor_util"] * elapsed - report_s + sum(workers) * elapsed
        cpu["supervisor_cpu_us_per_event"] = round(sup_cpu * 1e6 / n_ev, 1)
        if workers:
            cpu["worker_cpu_us_per_event"] = round(sum(workers) * elapsed * 1e6 / n_ev, 1)
        rss = getattr(harness, "replica_rss_mb", None)
        if rss is not None:
            cpu.update(rss())
        if sampler is not None:
            prof = sampler.stop()
            sampler = None
            with open(cfg.pprof_out, "wb") as f:
                f.write(prof.encode_gz())
            with open(cfg.pprof_out + ".top.txt", "w") as f:
                f.write(prof.top(40))
            pool = getattr(getattr(harness, "app", None), "pool", None)
            if pool is not None:
                pool.broadcast({"op": "pprof", "on": False, "path": cfg.pprof_out})
                want = [f"{cfg.pprof_out}.w{w.index}.top.txt" for w in pool.workers]
                for _ in range(100):
                    if all(os.path.exists(x) for x in want):
                        break
                    await asyncio.sleep(0.05)
        sync = getattr(harness, "sync_metrics", None)
        if sync is not None:
            await sync()
        stages = _stage_breakdown(sup)
        # the replica parent's periodic GPU-telemetry mirror (it shares the watch hub's loop)
        mirror = _stage_breakdown(sup, ("gpu_mirror_publish", "worker_gpu_update"))
        if mirror.get("gpu_mirror_publish"):
            cpu["gpu_mirror_publish_ms"] = mirror["gpu_mirror_publish"]
        if mirror.get("worker_gpu_update"):  # ... and each worker applying it
            cpu["worker_gpu_update_ms"] = mirror["worker_gpu_update"]
            sizes = (sup.metrics.gauges.get("worker_gpu_update_bytes") or {}).values()
            cpu["worker_gpu_update_bytes_max"] = max(sizes, default=None)
        gpu_evidence = {"via": "local-monitor"}
        if agent is not None:
            am = await agent.metrics()
            ev = {k: int(sup.metrics.counter(k) - ev0[k]) for k in _EVIDENCE_COUNTERS}
            deferred = ev["decisions_deferred_for_gpu_evidence"]
            gpu_evidence = {"via": "node-agent", "evidence_wait_s": cfg.evidence_wait, "counted_over": "warmup+timed",
                            "agent_annotations": int(sum(v for k, v in am.items() if k.endswith("agent_annotations_total"))),
                            "agent_util": cpu.get("agent_util"), "agent_cpu_us_per_event": cpu.get("agent_cpu_us_per_event"),
                            "deferred": deferred, "wait_expired": ev["gpu_evidence_wait_expired"],
                            "wait_expired_share": round(ev["gpu_evidence_wait_expired"] / deferred, 4) if deferred else None,
                            "job_decisions_awaited": ev["decisions_awaited_gpu_evidence"],
                            # default pods: the agent read their OOM text from the node's logs
                            "agent_log_reads": int(sum(v for k, v in am.items() if k.endswith("agent_log_reads_total"))),
                            "supervisor_log_fetches": int(sup.metrics.counter("decisions_deferred_for_log_tail"))}
        phase.update(name="readback", t0=time.monotonic())
        readback = await _read_back(harness, tracker)
        attribution = None
        if cfg.node and oom_phase is not None:
            ooms = await asyncio.get_running_loop().run_in_executor(None, oom_phase)
            attribution = await _node_attribution(harness, tracker, telemetry, ooms, cfg)
        probe = None
        if cfg.probe_events > 0:
            before = _stage_counts(sup)
            slow0 = _slow_snapshot(sup)
            phase.update(name="probe", t0=time.monotonic())
            probe = await _latency_probe(harness, tracker, cfg)
            if sync is not None:
                await sync()
            if probe.get("events"):
                # where the open-loop latency goes: the stage histograms' growth over the probe
                probe["stages_ms"] = _stage_delta(before, _stage_counts(sup))
                slow = _slow_callbacks(slow0, _slow_snapshot(sup))
                if slow:  # NEXUS_SLOW_CALLBACK_MS: what held a loop during the probe
                    probe["slow_callbacks"] = slow
    finally:
        if beat is not None:
            beat.cancel()
        if sampler is not None:
            sampler.stop()
        if agent is not None:
            agent.stop()
        await harness.stop()
        telemetry.stop()
        if monitor is not None:
            # libamd_smi's "Unable to open queues directory" lines, counted instead of printed
            monitor["process_vanished"] = telemetry.process_vanished()
    return {"elapsed": elapsed, "events": cfg.events * cfg.steps * (cfg.world if cfg.node else 1), "errors": tracker.errors,
            "failures": timed[0], "starts": timed[1], "start_latencies_ms": timed[2],
            "starts_superseded": tracker.superseded,
            "watch_objects_per_failure": watch_objects,
            "wrong_stage": tracker.wrong_stage, "wrong_examples": tracker.wrong_examples, "readback": readback,
            "latencies_ms": tracker.latencies, "store": harness.store_name, "workers": sc.workers,
            "actuation": _actuation(sc),
            "eps": sc.rate_limit_elements_per_second, "kube_qps": sc.kube_qps, "telemetry": telemetry.name, "stages": stages, "cpu": cpu,
            "probe": probe, "step_done_ms": step_done_ms, "monitor": monitor, "attribution": attribution,
            "gpu_evidence": gpu_evidence, "step_timeline": step_timeline}


async def _latency_probe(harness, tracker: "Tracker", cfg: "BenchConfig") -> Dict[str, Any]:
    """Open-loop latency at a pod-failure rate (BASELINE config 4: 1000 pod-fail events/min):
    single failures arriving as a Poisson process of that mean rate (seeded: the same
    schedule every run), each timed from push to checkpoint ack — the latency a run sees
    when the supervisor is not saturated, including the occasional near-simultaneous pair."""
    import random

    saved, tracker.latencies = tracker.latencies, []
    saved_parts, tracker.parts = tracker.parts, []
    saved_starts, tracker.start_latencies = tracker.start_latencies, []
    saved_pushed, tracker.pushed_at = tracker.pushed_at, []
    if cfg.run_starts:
        # the last timed step's new runs start now, before the first arrival: thousands of
        # starts in one burst are the saturated workload's, not the north-star churn's
        docs = await harness.step(0)
        for d in (docs if isinstance(docs, list) else [docs]):
            st = tracker.arm(d["rids"], d["t_push"], d.get("expected"), d.get("started"), d.get("start_expected"))
            try:
                await asyncio.wait_for(st.done.wait(), cfg.step_timeout)
            except asyncio.TimeoutError:
                tracker.abandon(st)
        tracker.latencies, tracker.parts, tracker.start_latencies, tracker.pushed_at = [], [], [], []
    tracker.by_rid, tracker.part_of = True, {}
    rate = cfg.probe_rate_per_min / 60.0
    rng = random.Random(0x5EED + cfg.seed + cfg.rank)
    loop = asyncio.get_running_loop()
    start = loop.time()
    states = []
    pending = []
    at = 0.0
    hold = getattr(harness, "probe_hold_ms", 0.0)

    kinds: Dict[str, str] = {}  # probe run -> failure kind (the tail report)

    async def one():
        # the harness answers after the failure is delivered (hold): the driver's own work on
        # the answer stays out of the replica parent's loop while the line is in flight; the
        # decision's ack may arrive first (Tracker.report keeps it until the step is armed)
        doc = await (harness.step(1, hold) if hold else harness.step(1))
        kinds.update(doc.get("kinds") or {})
        states.append(tracker.arm(doc["rids"], doc["t_push"], doc.get("expected"), doc.get("started"),
                                  doc.get("start_expected")))

    timeline = _CpuTimeline(harness) if cfg.probe_timeline and hasattr(harness, "external_cpu") else None
    if timeline is not None:
        timeline.start()
    played = getattr(harness, "probe", None)
    if played is not None:
        # the cluster process plays the schedule (same seed, same arrivals): one request for
        # the whole probe, every decision's ack kept by the tracker until its step is armed
        for doc in await played(cfg.probe_events, cfg.probe_rate_per_min, 0x5EED + cfg.seed + cfg.rank):
            kinds.update(doc.get("kinds") or {})
            states.append(tracker.arm(doc["rids"], doc["t_push"], doc.get("expected"), doc.get("started"),
                                      doc.get("start_expected")))
    for i in range(cfg.probe_events if played is None else 0):
        at += rng.expovariate(rate)
        delay = start + at - loop.time()
        if delay > 0:
            await asyncio.sleep(delay)
        if hold:
            pending.append(asyncio.ensure_future(one()))  # open loop: the next arrival does not wait
        else:
            await one()
    if pending:
        await asyncio.gather(*pending)
    for st in states:
        try:
            await asyncio.wait_for(st.done.wait(), cfg.step_timeout)
        except asyncio.TimeoutError:
            tracker.abandon(st)
    if timeline is not None:
        await timeline.stop()
    timed = [(t, rid, v) for (t, rid), v in zip(tracker.pushed_at, tracker.latencies)]
    lat = sorted(tracker.latencies)
    starts = sorted(tracker.start_latencies)
    parts = tracker.parts
    tracker.latencies, tracker.parts, tracker.start_latencies = saved, saved_parts, saved_starts
    tracker.pushed_at = saved_pushed
    if not lat:
        return {"events": 0}
    q = lambda p, v=lat: v[min(len(v) - 1, int(round(p * (len(v) - 1))))]  # noqa: E731
    out = {"rate_per_min": cfg.probe_rate_per_min, "arrivals": "poisson", "events": len(lat),
           "p50_ms": round(q(0.5), 3), "p90_ms": round(q(0.9), 3), "p99_ms": round(q(0.99), 3),
           "max_ms": round(lat[-1], 3)}
    if timed:
        # when the tail arrived: seconds from the first arrival of every failure at or over p99
        t0 = min(t for t, _, _ in timed)
        out["t0_monotonic"] = round(t0, 4)  # the first arrival's push (CLOCK_MONOTONIC)
        out["tail_arrival_s"] = sorted(round(t - t0, 2) for t, _, v in timed if v >= q(0.99))
        if kinds:
            # which failure kinds the tail is, against the probe's mix
            out["tail_kinds"] = sorted(kinds.get(rid, "?") for _, rid, v in timed if v >= q(0.99))
            mix: Dict[str, int] = {}
            for _, rid, _ in timed:
                mix[kinds.get(rid, "?")] = mix.get(kinds.get(rid, "?"), 0) + 1
            out["kinds"] = mix
            out["by_kind"] = _by_kind(timed, kinds, tracker.part_of)
        if timeline is not None:
            out["cpu_timeline"] = timeline.report(t0)
    tracker.by_rid, tracker.part_of = False, {}
    if starts:  # the replacement runs' Started → RUNNING at the same rate
        out["starts"] = len(starts)
        out["start_p50_ms"] = round(q(0.5, starts), 3)
        out["start_p99_ms"] = round(q(0.99, starts), 3)
    if parts:
        out["delivery"] = decompose(parts)
    return out


PART_NAMES = ("api", "hub", "feed", "dispatch", "classify", "queue", "actuate")


def _by_kind(timed, kinds: Dict[str, str], part_of: Dict[str, Tuple[float, ...]]) -> Dict[str, Any]:
    """Probe latency per failure kind: count, p50 / p99 / max, and the mean of each
    delivery stage — does one kind (an hbm-oom's log-tail read, an eviction's Job settle)
    carry the tail?"""
    by: Dict[str, List[Tuple[float, str]]] = {}
    for _t, rid, v in timed:
        by.setdefault(kinds.get(rid, "?"), []).append((v, rid))
    out: Dict[str, Any] = {}
    for kind, vs in sorted(by.items()):
        lat = sorted(v for v, _ in vs)
        q = lambda p: lat[min(len(lat) - 1, int(round(p * (len(lat) - 1))))]  # noqa: E731
        rec: Dict[str, Any] = {"n": len(lat), "p50_ms": round(q(0.5), 3), "p99_ms": round(q(0.99), 3),
                               "max_ms": round(lat[-1], 3)}
        parts = [part_of[rid] for _, rid in vs if rid in part_of]
        if parts:
            rec["stage_mean_ms"] = {name: round(sum(p[i + 1] for p in parts) / len(parts), 3)
                                    for i, name in enumerate(PART_NAMES)}
        out[kind] = rec
    return out


_SIM_SERIAL = ("busy", "apply_thread", "store", "gc")  # the simulator's single-thread parts (/sim/stats)
_PACING_KEYS = ("parent", "cluster", "cqlsrv", "kubesim") + tuple(f"kubesim_{k}" for k in _SIM_SERIAL)


def steady_util(rows: List[Dict[str, Any]], step_done_ms: List[float]) -> Dict[str, Any]:
    """Each process's CPU (cores) over the *steady* part of the timed steps — from the
    second step's completion to the second-to-last's, when every in-flight slot is full —
    as its median and 90th percentile over the timeline's intervals, and the process closest
    to a full core there (``pacing``: the stage the line waits on).  ``kubesim`` is the
    simulator's whole CPU, threads included; its single-thread parts are ``kubesim_busy``
    (event loop), ``kubesim_apply_thread`` (apply port) and ``kubesim_store`` (store lock
    held)."""
    if len(step_done_ms) >= 4:
        lo, hi = step_done_ms[1] / 1000.0, step_done_ms[-2] / 1000.0
    else:
        lo, hi = float("-inf"), float("inf")
    sel = [r for r in rows if lo <= r["t"] <= hi] or rows
    if not sel:
        return {}
    keys = [k for k in sel[0] if k.startswith("worker") or k in _PACING_KEYS]
    out: Dict[str, Any] = {"window_s": [round(lo, 2), round(hi, 2)] if lo != float("-inf") else None,
                           "intervals": len(sel), "median": {}, "p90": {}}
    for k in keys:
        v = sorted(r.get(k, 0.0) for r in sel)
        out["median"][k] = v[len(v) // 2]
        out["p90"][k] = v[min(len(v) - 1, int(0.9 * len(v)))]
    single = {k: v for k, v in out["median"].items() if k != "kubesim"}  # one-thread processes / parts
    if single:
        top = max(single, key=single.get)
        out["pacing"] = {"process": top, "median_util": single[top]}
    return out


class _CpuTimeline:
    """``--diag-probe-timeline``: every second of the probe, the CPU share of each bench
    process (simulator, CQL server, cluster process, shard workers, this replica parent),
    the host's busy CPUs (``/proc/stat``: other tenants included) and the cgroup's CFS
    throttling (``cpu.stat``) — to tell a stall of one process from contention for the box."""

    def __init__(self, harness, interval: float = 0.25, sim: bool = False):
        self.harness = harness
        self.interval = interval
        self.rows: List[Dict[str, Any]] = []
        self._task: Optional[asyncio.Task] = None
        # the simulator's serial parts too (its /sim/stats busy counters): event loop, apply
        # port, store lock — each a single thread of the multi-threaded process
        self.sim = getattr(harness, "sim_stats", None) if sim else None

    @staticmethod
    def _host() -> Tuple[float, float]:
        try:
            with open("/proc/stat") as f:
                v = [int(x) for x in f.readline().split()[1:]]
            return float(sum(v) - v[3] - (v[4] if len(v) > 4 else 0)), float(sum(v))
        except (OSError, ValueError, IndexError):
            return 0.0, 0.0

    @staticmethod
    def _throttled() -> Tuple[float, float]:
        for path in ("/sys/fs/cgroup/cpu.stat", "/sys/fs/cgroup/cpu/cpu.stat"):
            try:
                with open(path) as f:
                    kv = dict(line.split() for line in f if line.strip())
                us = float(kv.get("throttled_usec", 0.0)) or float(kv.get("throttled_time", 0.0)) / 1000.0
                return float(kv.get("nr_throttled", 0.0)), us
            except (OSError, ValueError):
                continue
        return 0.0, 0.0

    def _pids(self) -> Dict[str, int]:
        h = self.harness
        out = {"parent": os.getpid()}
        for name, proc in (("cluster", getattr(h, "proc", None)), ("cqlsrv", getattr(getattr(h, "cql", None), "proc", None))):
            if proc is not None:
                out[name] = proc.pid
        if getattr(h, "sim_pid", None):
            out["kubesim"] = h.sim_pid
        pool = getattr(getattr(h, "app", None), "pool", None)
        if pool is not None:
            out.update({f"worker{w.index}": w.proc.pid for w in pool.workers})
        return out

    @staticmethod
    def _faults(pid: int) -> Tuple[int, int]:
        try:
            with open(f"/proc/{pid}/stat") as f:
                parts = f.read().rsplit(")", 1)[1].split()
            return int(parts[7]), int(parts[9])  # minflt, majflt
        except (OSError, ValueError, IndexError):
            return 0, 0

    def _sample(self) -> Dict[str, Any]:
        cpu = dict(self.harness.external_cpu())
        t = os.times()
        cpu["parent"] = t.user + t.system
        busy, total = self._host()
        n, us = self._throttled()
        flt = {k: self._faults(pid) for k, pid in self._pids().items()}
        return {"t": time.monotonic(), "cpu": cpu, "host_busy": busy, "host_total": total, "thr_n": n, "thr_us": us,
                "flt": flt}

    async def _sim(self, row: Dict[str, Any]) -> None:
        try:
            st = await self.sim()
        except Exception:  # noqa: BLE001 - a diagnostic: a missed sample is a gap
            return
        if st:
            row["cpu"].update({f"kubesim_{k}": st.get(f"{k}_ns", 0) / 1e9 for k in _SIM_SERIAL})
            conns = st.get("apply_conn_ns")
            if conns:  # one thread per apply connection: the busiest one (see run_rank)
                row["cpu"]["kubesim_apply_thread"] = max(conns.values()) / 1e9

    async def _run(self) -> None:
        while True:
            row = self._sample()
            if self.sim is not None:
                await self._sim(row)
            self.rows.append(row)
            await asyncio.sleep(self.interval)

    def start(self) -> None:
        self._task = asyncio.ensure_future(self._run())

    async def stop(self) -> None:
        if self._task is not None:
            self._task.cancel()
            try:
                await self._task
            except asyncio.CancelledError:
                pass
        row = self._sample()
        if self.sim is not None:
            await self._sim(row)
        self.rows.append(row)

    def report(self, t0: float) -> List[Dict[str, Any]]:
        """One entry per interval: seconds from ``t0`` (the first arrival), each process's
        cores, the host's busy cores and the cgroup's throttled periods / milliseconds."""
        ncpu = os.cpu_count() or 1
        out = []
        for a, b in zip(self.rows, self.rows[1:]):
            dt = b["t"] - a["t"]
            if dt <= 0:
                continue
            row = {"t": round(a["t"] - t0, 1)}
            row.update({k: round((b["cpu"][k] - a["cpu"].get(k, 0.0)) / dt, 2) for k in b["cpu"]
                        if not k.endswith("_sys") and k in a["cpu"]})
            if b["host_total"] > a["host_total"]:
                row["host_busy_cpus"] = round(ncpu * (b["host_busy"] - a["host_busy"]) / (b["host_total"] - a["host_total"]), 1)
            row["throttled"] = int(b["thr_n"] - a["thr_n"])
            row["throttled_ms"] = round((b["thr_us"] - a["thr_us"]) / 1000.0, 1)
            # page faults in the interval, all bench processes: minor, major
            row["minflt"] = sum(v[0] - a["flt"].get(k, (0, 0))[0] for k, v in b["flt"].items())
            row["majflt"] = sum(v[1] - a["flt"].get(k, (0, 0))[1] for k, v in b["flt"].items())
            out.append(row)
        return out


def _slow_callbacks(before: Dict[str, Dict[Any, float]], after: Dict[str, Dict[Any, float]],
                    top: int = 15) -> List[Dict[str, Any]]:
    """Growth of the ``slow_callbacks`` / ``slow_callback_seconds`` /
    ``slow_callback_gc_seconds`` counters ``{name, where}`` (:mod:`..obs.loopwatch`) between
    two snapshots, longest total first."""
    n0, s0 = before.get("slow_callbacks") or {}, before.get("slow_callback_seconds") or {}
    n1, s1 = after.get("slow_callbacks") or {}, after.get("slow_callback_seconds") or {}
    g0, g1 = before.get("slow_callback_gc_seconds") or {}, after.get("slow_callback_gc_seconds") or {}
    rows = []
    for k, v in n1.items():
        n = v - n0.get(k, 0.0)
        if n > 0:
            lab = dict(k)
            rows.append({"where": lab.get("where", ""), "name": lab.get("name", ""), "count": int(n),
                         "total_ms": round((s1.get(k, 0.0) - s0.get(k, 0.0)) * 1e3, 3),
                         "gc_ms": round((g1.get(k, 0.0) - g0.get(k, 0.0)) * 1e3, 3)})
    rows.sort(key=lambda r: -r["total_ms"])
    return rows[:top]


def _slow_snapshot(sup) -> Dict[str, Dict[Any, float]]:
    c = sup.metrics.counters
    return {n: dict(c.get(n) or {}) for n in ("slow_callbacks", "slow_callback_seconds", "slow_callback_gc_seconds")}


def decompose(parts) -> Dict[str, Any]:
    """Per-decision push→ack decomposition: every stage's p50 / p99, and the mean of each
    stage over the median band (p45–p55) and the tail (≥ p99) of the *total* — those means
    sum to the band's mean total, so the tail is explained stage by stage."""
    ps = sorted(parts)
    n = len(ps)

    def qs(vals, p):
        v = sorted(vals)
        return round(v[min(len(v) - 1, int(round(p * (len(v) - 1))))], 3)

    out: Dict[str, Any] = {"events": n, "stages": {}}
    for i, name in enumerate(PART_NAMES, start=1):
        col = [p[i] for p in ps]
        out["stages"][name] = {"p50": qs(col, 0.5), "p99": qs(col, 0.99)}

    def band(lo, hi):
        sel = ps[int(lo * (n - 1)):max(int(lo * (n - 1)) + 1, int(round(hi * (n - 1))) + 1)]
        m = {name: round(sum(p[i] for p in sel) / len(sel), 3) for i, name in enumerate(PART_NAMES, start=1)}
        m["total"] = round(sum(p[0] for p in sel) / len(sel), 3)
        m["events"] = len(sel)
        return m

    out["median_band_mean_ms"] = band(0.45, 0.55)
    out["tail_p99_mean_ms"] = band(0.99, 1.0)
    return out


async def _read_back(harness, tracker: "Tracker") -> Dict[str, Any]:
    """After the timed steps: read every timed run's row back from the store and compare
    its lifecycle stage with the stage the workload expects (the decision reports say
    what the supervisor *meant* to write; this checks what the store *holds*)."""
    read = getattr(harness, "read_stages", None)
    if read is None or not tracker.checked:
        return {"checked": 0}
    rids = list(tracker.checked)
    got = await read(harness.algorithm, rids)
    wrong = [(r, got.get(r), tracker.checked[r]) for r in rids if got.get(r) != tracker.checked[r]]
    return {"checked": len(rids), "wrong": len(wrong), "examples": wrong[:5]}


def _actuation(sc: SupervisorConfig) -> str:
    from ..supervisor import fused_actuation

    if fused_actuation(sc):
        return "fused conditional write"
    cu = sc.compat.conditional_update
    return "read+write" + (" (ToRunning: one conditional write)" if cu == "auto" else " (conditional)" if cu == "always"
                           else "")


STAGES = ("receive_to_checkpoint", "stage_classify", "stage_queue", "stage_read", "stage_prepare", "stage_write",
          "stage_delete", "stage_hub", "stage_feed", "stage_dispatch")


def _stage_counts(sup) -> Dict[str, Tuple[Dict[int, int], int, int]]:
    """Bucket counts, total and sum of every stage histogram (cumulative, merged over workers)."""
    out = {}
    for name in STAGES:
        h = sup.metrics.histogram(name)
        if h is not None:
            out[name] = ({int(i): int(c) for i, c in h.sparse()}, int(h.total), int(h.sum))
    return out


def _stage_delta(before, after) -> Dict[str, Any]:
    """Stage summaries (ms) of what was recorded between two :func:`_stage_counts`
    snapshots; min / max are the bounds of the outermost non-empty buckets."""
    from ..obs.histogram import PyLatencyHistogram

    out = {}
    for name, (counts, total, hsum) in after.items():
        b_counts, b_total, b_sum = before.get(name, ({}, 0, 0))
        h = PyLatencyHistogram()
        for i, c in counts.items():
            d = c - b_counts.get(i, 0)
            if d > 0 and i < len(h.counts):
                h.counts[i] = d
        nz = [i for i, c in enumerate(h.counts) if c]
        h.total = sum(h.counts)
        if not nz or total - b_total <= 0:
            continue
        h.sum = hsum - b_sum
        h.min = h._bounds(nz[0])[0]
        h.max = h._bounds(nz[-1])[1] - 1
        out[name] = {k: (int(v) if k == "count" else round(v / 1000.0, 3)) for k, v in h.summary().items()}
    return out


def _stage_breakdown(sup, names=None) -> Dict[str, Any]:
    m = sup.metrics
    out = {}
    for name in names or STAGES:
        h = m.histogram(name)
        if h is not None:
            out[name] = {k: (int(v) if k == "count" else round(v / 1000.0, 3)) for k, v in h.summary().items()}
    return out
