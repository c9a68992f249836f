"""Process-per-core runtime: one supervisor replica as K shard-worker processes.

The reference is a Go binary, so its informer goroutines, the nexus-core actor's
``Workers`` goroutines and the client libraries spread over every core of the pod
(``/root/reference/services/supervisor.go:73-75,107-117``).  A CPython event loop
uses one core, so this build scales a replica *out* across processes instead of
threads:

* each worker process is a complete :class:`~..app.Application` (own informers,
  own CQL session, own pipelined Job-DELETE connections, own GPU telemetry);
* runs are partitioned by the Job name (= request id), the one key every Job,
  Pod (``batch.kubernetes.io/job-name`` label) and Job Event carries, so a run's
  Job, its Pods and their Events all land in the same worker and per-run
  ordering (the pipeline's per-key FIFO) is preserved without cross-process
  coordination;
* the filter runs at ingest (:attr:`SharedInformer.accept`): a worker neither
  caches nor classifies another worker's objects, so cache memory and classify
  CPU divide by K (only the watch-stream decode is repeated);
* a Pod Event names the Pod, not the Job: every worker keeps a name → owner map
  of all Pods it has seen (cheap) and an Event for a Pod nobody has seen yet is
  parked by every worker until the Pod arrives, then dropped by the non-owners;
* the coordinating parent holds the leader-election lease, relays
  active/standby to the workers, merges their metrics for ``/metrics`` and, when
  asked (benchmarks, tests), relays their decisions to in-process hooks.

Control channel: one ``socketpair`` per worker, newline-delimited JSON.
Parent → worker: ``{"op": "active", "v": bool}``, ``{"op": "metrics", "seq": n}``,
``{"op": "shards", "owned": [k, ...]}`` (replica shard leases won / lost),
``{"op": "stop", "drain": seconds}``.  Worker → parent: ``{"op": "synced"}``,
``{"op": "dec", "d": [[request_id, algorithm, outcome, ack_mono, stage], ...]}``,
``{"op": "metrics", "seq": n, "s": state}``, ``{"op": "exit"}``.  A worker whose
channel hits EOF (parent gone) drains and exits; ``PR_SET_PDEATHSIG`` backs that
up if the parent is killed outright.
"""
from __future__ import annotations

import asyncio
import collections
import copy
import json
import os
import signal
import socket
import subprocess
import sys
import time
import zlib
from typing import Any, Callable, Deque, Dict, List, Optional, Tuple

from ..models import kube
from ..models.decisions import Decision, RunStatusAnalysisResult
from ..obs.delivery import record as delivery_record

try:
    from .._kube_native import dumps as _native_dumps
except ImportError:  # pragma: no cover - the json module path
    _native_dumps = None
from ..obs.histogram import LatencyHistogram
from ..obs.metrics import Metrics

_SEED = 0x2545F491  # decorrelates worker placement from replica sharding (sharding.SHARD_SEED)
_FOREIGN = -2  # pod owner: another replica's run (native router OWNER_NONE)
# how long a deleted pod's owner is remembered for Pod Events still in flight: at tens of
# thousands of pod failures per second every second of window is ~100k map entries in the
# router (profiles/r2_pprof_*: a 120 s window held millions in the hub parent); an Event
# later than this is parked by every worker and dropped as unmatched — harmless
POD_FORGET_AFTER = 30.0
_LINE_LIMIT = 64 << 20


def worker_of(request_id: str, count: int) -> int:
    """Owner worker of a run (its Job name)."""
    if count <= 1:
        return 0
    return zlib.crc32(request_id.encode(), _SEED) % count


class WorkerShard:
    """Ingest filter of worker ``index`` of ``count`` (installed on the Event/Pod/Job informers),
    and of the replica's shard set (``shards``: runs of other replicas are dropped)."""

    def __init__(self, index: int, count: int, job_name_label: str, forget_after: float = POD_FORGET_AFTER,
                 clock: Callable[[], float] = time.monotonic, shards=None):
        from .sharding import ShardSet

        self.index = index
        self.count = count
        self.job_name_label = job_name_label
        self.forget_after = forget_after
        self.clock = clock
        self.shards = shards if shards is not None else ShardSet(1)
        self.pod_owner: Dict[str, Tuple[int, str]] = {}  # pod name → (worker, run)
        self._gone: Deque[Tuple[float, str]] = collections.deque()
        try:  # native pre-decode filter (csrc/kube/watch_decoder.cpp ShardRouter)
            from .._kube_native import ShardRouter

            self.native = ShardRouter(index, count, _SEED, job_name_label, forget_after)
        except ImportError:  # pragma: no cover - pure-Python fallback filters after decode
            self.native = None
        self.sync_replica()

    def sync_replica(self) -> None:
        """Push the replica's current shard set into the native router."""
        if self.native is not None and self.shards.enabled:
            from .sharding import SHARD_SEED

            self.native.set_replica(self.shards.shards, SHARD_SEED, sorted(self.shards.owned))

    def of(self, request_id: str) -> int:
        return zlib.crc32(request_id.encode(), _SEED) % self.count

    def _owner(self, request_id: str) -> int:
        return self.of(request_id) if self.shards.owns(request_id) else _FOREIGN

    def accept_job(self, obj: Dict[str, Any], etype: str) -> bool:
        return self._owner(kube.name_of(obj)) == self.index

    def accept_pod(self, obj: Dict[str, Any], etype: str) -> bool:
        meta = obj.get("metadata") or {}
        rid = (meta.get("labels") or {}).get(self.job_name_label)
        worker = self.of(rid) if rid else 0
        name = meta.get("name", "")
        if etype == "DELETED":
            # events about a deleted pod may still be in flight on the event watch
            self._gone.append((self.clock() + self.forget_after, name))
        self.pod_owner[name] = (worker, rid or "")
        if self.native is not None:
            self.native.note_pod(name, worker, etype == "DELETED", rid)
        if self._gone:
            self._expire()
        return (worker if not rid or self.shards.owns(rid) else _FOREIGN) == self.index

    def _expire(self) -> None:
        now = self.clock()
        gone = self._gone
        while gone and gone[0][0] <= now:
            _, name = gone.popleft()
            self.pod_owner.pop(name, None)

    def accept_event(self, obj: Dict[str, Any], etype: str) -> bool:
        inv = obj.get("involvedObject") or {}
        kind = inv.get("kind")
        if kind == "Job":
            return self._owner(inv.get("name", "")) == self.index
        if kind == "Pod":
            owner = self.owner_of_pod(inv.get("name", ""))
            return owner is None or owner == self.index  # unknown pod: park everywhere until it shows up
        return self.index == 0

    def owner_of_pod(self, name: str) -> Optional[int]:
        """Worker owning a pod seen so far; None = unknown, -2 = another replica's run."""
        seen = self.pod_owner.get(name)
        if seen is not None:
            worker, rid = seen
            return worker if not rid or self.shards.owns(rid) else _FOREIGN
        if self.native is not None:
            return self.native.pod_owner(name)  # pods dropped before decode are only known natively
        return None

    def install(self, sup, routed_upstream: bool = False) -> None:
        """Filter this worker's informers.  ``routed_upstream`` (watch hub): the parent
        already sends only this worker's objects, so no per-object filter is installed."""
        if routed_upstream:
            return
        if self.native is not None:
            for inf, role in ((sup.job_informer, "job"), (sup.pod_informer, "pod"), (sup.event_informer, "event")):
                if hasattr(inf.lw, "shard_router"):
                    inf.lw.shard_router = (self.native, role)
        sup.job_informer.accept = self.accept_job
        sup.pod_informer.accept = self.accept_pod
        sup.event_informer.accept = self.accept_event
        sup.pod_informer.on_reject = lambda pod: sup.drop_parked("Pod", kube.name_of(pod))
        sup.job_informer.on_reject = lambda job: sup.drop_parked("Job", kube.name_of(job))


# ---------------------------------------------------------------------- metrics hand-off
def metrics_state(m: Metrics) -> Dict[str, Any]:
    hists = []
    for name, series in m.hists.items():
        for k, h in series.items():
            hists.append([name, [list(p) for p in k], h.sparse(), h.total, h.sum, h.min, h.max])
    return {"c": [[n, [list(p) for p in k], v] for n, s in m.counters.items() for k, v in s.items()],
            "g": [[n, [list(p) for p in k], v] for n, s in m.gauges.items() for k, v in s.items()],
            "h": hists, "help": m.help}


def merge_metrics_state(dst: Metrics, st: Dict[str, Any], gauge_labels: Optional[Dict[str, str]] = None) -> None:
    """Add a worker's state into ``dst``: counters and histograms sum, gauges are kept per
    worker (``gauge_labels`` added) since a sum is not meaningful for every gauge."""
    for name, k, v in st.get("c", ()):
        key = tuple(tuple(p) for p in k)
        d = dst.counters.setdefault(name, {})
        d[key] = d.get(key, 0.0) + v
    extra = tuple(sorted((gauge_labels or {}).items()))
    for name, k, v in st.get("g", ()):
        key = tuple(sorted(tuple(tuple(p) for p in k) + extra))
        dst.gauges.setdefault(name, {})[key] = v
    for name, k, sparse, total, hsum, hmin, hmax in st.get("h", ()):
        key = tuple(tuple(p) for p in k)
        series = dst.hists.setdefault(name, {})
        h = series.get(key)
        if h is None:
            h = series[key] = LatencyHistogram()
        h.merge_state(sparse, total, hsum, hmin, hmax)
    for name, text in (st.get("help") or {}).items():
        dst.help.setdefault(name, text)


def collect_gauges(sup, m: Metrics) -> None:
    """Point-in-time gauges of one supervisor (queue, informer sizes, role)."""
    if sup.pipeline is not None:
        m.set("queue_depth", sup.pipeline.depth())
        m.set("in_flight", sup.pipeline.in_flight())
        for k, v in sup.pipeline.stats.as_dict().items():
            m.set(f"pipeline_{k}", v)
    for kind, inf in sup.factory.informers.items():
        m.set("informer_objects", len(inf.indexer), {"kind": kind})
        m.set("informer_relists", inf.relists, {"kind": kind})
        lw = inf.lw
        if hasattr(lw, "decode_seconds"):
            m.set("informer_decode_seconds", lw.decode_seconds, {"kind": kind})
            m.set("informer_decoded_lines", lw.decoded_lines, {"kind": kind})
    m.set("active", 1.0 if sup.active else 0.0)


# ---------------------------------------------------------------------- channel
class Channel:
    """Newline-delimited JSON over a connected stream socket."""

    def __init__(self, reader: asyncio.StreamReader, writer: asyncio.StreamWriter):
        self.reader = reader
        self.writer = writer

    @classmethod
    async def open(cls, sock: socket.socket) -> "Channel":
        reader, writer = await asyncio.open_connection(sock=sock, limit=_LINE_LIMIT)
        return cls(reader, writer)

    def send(self, msg: Dict[str, Any]) -> None:
        if not self.writer.is_closing():
            # the native compact encoder (the decision reports of a busy worker are ~1 % of its
            # CPU through the json module, profiles/r2_pprof_v18_procs6)
            try:
                data = _native_dumps(msg) if _native_dumps is not None else None
            except (TypeError, ValueError):
                data = None
            if data is None:
                data = json.dumps(msg, separators=(",", ":")).encode()
            self.writer.write(data + b"\n")

    async def recv_line(self) -> Optional[bytes]:
        try:
            line = await self.reader.readline()
        except (ConnectionError, asyncio.IncompleteReadError, ValueError):
            return None
        return line or None

    async def recv(self) -> Optional[Dict[str, Any]]:
        line = await self.recv_line()
        return json.loads(line) if line else None

    def close(self) -> None:
        try:
            self.writer.close()
        except Exception:  # noqa: BLE001
            pass


# ---------------------------------------------------------------------- parent side
class _Worker:
    __slots__ = ("index", "proc", "chan", "synced", "state", "reader", "exited", "sock", "data")

    def __init__(self, index: int):
        self.index = index
        self.proc: Optional[subprocess.Popen] = None
        self.chan: Optional[Channel] = None
        self.synced = asyncio.Event()
        self.state: Dict[str, Any] = {}
        self.reader: Optional[asyncio.Task] = None
        self.exited = asyncio.Event()
        self.sock: Optional[socket.socket] = None
        self.data: Optional[asyncio.StreamWriter] = None  # watch-hub frames to this worker


class WorkerPool:
    """Spawns and supervises the shard-worker processes of one replica."""

    def __init__(self, cfg, *, report_decisions: bool = False, python: str = sys.executable,
                 env: Optional[Dict[str, str]] = None, log_dir: str = ""):
        from ..config import to_mapping

        self.cfg = cfg
        self.count = cfg.runtime.worker_processes
        self.report_decisions = report_decisions
        self.python = python
        self.env = env
        self.log_dir = log_dir
        self.workers: List[_Worker] = [_Worker(i) for i in range(self.count)]
        self.decision_hooks: List[Callable[[Decision], None]] = []
        self.report_hooks: List[Callable[[str, str, Optional[float], Optional[str]], None]] = []
        # parent CPU spent on the decision-report channel (benchmarks / tests only: decode +
        # hooks); the bench reports it apart from the supervisor's own CPU
        self.report_cpu_s = 0.0
        self.active = True
        self._mapping = to_mapping(cfg)
        self._metrics_seq = 0
        self._metrics_waiters: Dict[int, Tuple[asyncio.Future, set]] = {}
        self.restarts = 0
        self.restart_backoff = (0.2, 10.0)  # base, max seconds between restarts of one worker
        self.hub = bool(cfg.runtime.watch_hub)
        # node-local GPU telemetry: the parent owns the one amd-smi session and mirrors it
        # into every worker (RemoteTelemetry) instead of K monitors per replica
        self.remote_gpu = bool(cfg.gpu.attribution_enabled and cfg.gpu.local_telemetry)
        self.on_restart: Optional[Callable[[int], Any]] = None  # async callback (watch hub resync)
        self.owned_shards: Optional[List[int]] = None  # lease mode: shards held right now
        # lease hold deadlines (CLOCK_MONOTONIC, one clock for the host's processes): the
        # workers fence themselves on them without waiting for the parent
        self.shard_until: Dict[str, float] = {}
        self.active_until: Optional[float] = None  # leader lease
        self._stopping = False
        self._watchdog: Optional[asyncio.Task] = None
        # the replica's kube-qps / kube-burst as one shared budget for the parent and every
        # worker (kube/flowcontrol.py SharedSchedule; None = a fixed 1/(K+1) split)
        from ..kube.flowcontrol import replica_schedule

        self.qps_schedule = replica_schedule(cfg, create=self.count > 1)

    def _child_mapping(self, index: int) -> Dict[str, Any]:
        m = copy.deepcopy(self._mapping)
        m["runtime"]["worker-index"] = index
        # admission knobs are per replica (reference semantics): split them over the workers
        k = self.count
        m["workers"] = max(1, -(-int(m["workers"]) // k))
        if m["rate-limit-elements-per-second"]:
            m["rate-limit-elements-per-second"] = float(m["rate-limit-elements-per-second"]) / k
        m["rate-limit-elements-burst"] = max(1, int(m["rate-limit-elements-burst"]) // k)
        m["leader-election"]["enabled"] = False  # the parent holds the lease
        m["observability"]["http-port"] = 0      # the parent serves /metrics
        return m

    async def start(self, active: bool = True) -> None:
        self.active = active
        self._stopping = False
        for w in self.workers:
            await self._spawn(w)
        self._watchdog = asyncio.create_task(self._watch(), name="worker-watchdog")

    async def _watch(self) -> None:
        """Restart a worker that exited on its own (crash, OOM kill) with exponential backoff;
        the new process re-lists and replays, which is idempotent (finished rows are skipped).
        Its siblings keep running: one bad run cannot take the whole replica down."""
        base, cap = self.restart_backoff
        delay = {w.index: base for w in self.workers}
        while not self._stopping:
            await asyncio.sleep(0.1)
            for w in self.workers:
                if self._stopping or w.proc is None or w.proc.poll() is None:
                    continue
                rc = w.proc.returncode
                await asyncio.sleep(delay[w.index])
                if self._stopping:
                    return
                self.restarts += 1
                delay[w.index] = min(cap, delay[w.index] * 2)
                import logging

                logging.getLogger("nexus_supervisor_amd.workers").warning(
                    "worker %d exited rc=%s; restarting (restart #%d)", w.index, rc, self.restarts)
                if w.reader is not None:
                    w.reader.cancel()
                if w.chan is not None:
                    w.chan.close()
                if w.data is not None:
                    w.data.close()
                await self._spawn(w)
                if self.on_restart is not None:
                    await self.on_restart(w.index)

    async def _spawn(self, w: _Worker) -> None:
        parent, child = socket.socketpair()
        dparent = dchild = None
        if self.hub:
            dparent, dchild = socket.socketpair()
        from .. import compiled

        pkg_root = os.path.dirname(compiled.PKG_DIR)  # (this module may run compiled: no __file__ walk)
        env = dict(self.env if self.env is not None else os.environ)
        env["PYTHONPATH"] = os.pathsep.join(p for p in [pkg_root, env.get("PYTHONPATH", "")] if p)
        env["NEXUS_WORKER_CONFIG"] = json.dumps(self._child_mapping(w.index))
        env["NEXUS_WORKER_CTL_FD"] = str(child.fileno())
        env["NEXUS_WORKER_START_ACTIVE"] = "1" if self.active else "0"
        env["NEXUS_WORKER_REPORT"] = "1" if self.report_decisions else "0"
        env["NEXUS_WORKER_REMOTE_GPU"] = "1" if self.remote_gpu else "0"
        fds = [child.fileno()]
        if self.qps_schedule is not None:
            env["NEXUS_WORKER_QPS_FD"] = str(self.qps_schedule.fd)
            fds.append(self.qps_schedule.fd)
        else:
            env.pop("NEXUS_WORKER_QPS_FD", None)
        if dchild is not None:
            env["NEXUS_WORKER_DATA_FD"] = str(dchild.fileno())
            fds.append(dchild.fileno())
        else:
            env.pop("NEXUS_WORKER_DATA_FD", None)
        out = None
        if self.log_dir:
            out = open(os.path.join(self.log_dir, f"worker-{w.index}.log"), "ab")
        try:
            w.proc = subprocess.Popen([self.python, "-m", "nexus_supervisor_amd", "worker"], env=env,
                                      pass_fds=tuple(fds), stdout=out, stderr=out)
        finally:
            child.close()
            if dchild is not None:
                dchild.close()
            if out is not None:
                out.close()
        w.sock = parent
        w.chan = await Channel.open(parent)
        if dparent is not None:
            _r, w.data = await asyncio.open_connection(sock=dparent)
        w.synced.clear()
        w.exited.clear()
        w.reader = asyncio.create_task(self._read(w), name=f"worker-{w.index}-ctl")
        if self.owned_shards is not None:  # lease mode: the shards this replica holds right now
            w.chan.send({"op": "shards", "owned": self.owned_shards, "until": self.shard_until})
        if self.active_until is not None:
            w.chan.send({"op": "lease", "active_until": self.active_until})

    async def _read(self, w: _Worker) -> None:
        while True:
            line = await w.chan.recv_line()
            if line is None:
                break
            t0 = time.thread_time()
            msg = json.loads(line)
            op = msg.get("op")
            if op == "dec":
                for h in self.report_hooks:
                    for d in msg["d"]:
                        h(d[0], d[2], d[3], d[4], d[5] if len(d) > 5 else None)
                if self.decision_hooks:
                    for rid, alg, outcome, ack, stage, *_x in msg["d"]:
                        r = RunStatusAnalysisResult("", "", "", request_id=rid, algorithm=alg)
                        if ack is not None:
                            r.stamps["ack_mono"] = ack
                        d = Decision(r, outcome, stage)
                        for h in self.decision_hooks:
                            h(d)
                self.report_cpu_s += time.thread_time() - t0
            elif op == "metrics":
                w.state = msg.get("s") or {}
                waiter = self._metrics_waiters.get(msg.get("seq", -1))
                if waiter is not None:
                    fut, pending = waiter
                    pending.discard(w.index)
                    if not pending and not fut.done():
                        fut.set_result(None)
            elif op == "synced":
                w.synced.set()
            elif op == "exit":
                break
        w.exited.set()
        for fut, pending in list(self._metrics_waiters.values()):
            pending.discard(w.index)
            if not pending and not fut.done():
                fut.set_result(None)

    # ---- watch-hub data path (parallel/watchhub.py)
    def send_data(self, index: int, ftype: int, kind: int, payload: bytes) -> None:
        from .watchhub import HEADER

        d = self.workers[index].data
        if d is not None and not d.is_closing():
            head = HEADER.pack(ftype, kind, len(payload))
            if len(payload) <= 1 << 16:
                # one send: written apart, an idle socket sends the 6-byte header at once and
                # the worker wakes for it, then again for the payload (a watch frame is small)
                d.write(head + payload)
            else:  # a LIST snapshot: no copy of megabytes
                d.write(head)
                d.write(payload)

    def data_buffered(self, index: int) -> int:
        d = self.workers[index].data
        return d.transport.get_write_buffer_size() if d is not None and not d.is_closing() else 0

    async def data_drain(self, index: int) -> None:
        d = self.workers[index].data
        if d is not None and not d.is_closing():
            try:
                await d.drain()
            except ConnectionError:
                pass

    def broadcast(self, msg: Dict[str, Any]) -> None:
        """Control message to every live worker (e.g. the GPU telemetry mirror)."""
        for w in self.workers:
            if w.chan is not None and not w.exited.is_set():
                w.chan.send(msg)

    def set_active(self, active: bool, until: Optional[float] = None) -> None:
        self.active = active
        msg: Dict[str, Any] = {"op": "active", "v": active}
        if until is not None:
            self.active_until = msg["until"] = until
        for w in self.workers:
            if w.chan is not None:
                w.chan.send(msg)

    def set_lease_deadline(self, until: float) -> None:
        """Leader lease renewed: the workers' hold deadline moves with it."""
        self.active_until = until
        self.broadcast({"op": "lease", "active_until": until})

    def set_shard_deadlines(self, until: Dict[int, float]) -> None:
        self.shard_until = {str(k): t for k, t in until.items()}
        self.broadcast({"op": "lease", "until": self.shard_until})

    def set_shards(self, owned, until: Optional[Dict[int, float]] = None) -> None:
        """Relay the replica's owned shard set (with the holds' deadlines); a worker
        restarted later gets it at spawn."""
        self.owned_shards = sorted(owned)
        if until is not None:
            self.shard_until = {str(k): t for k, t in until.items()}
        for w in self.workers:
            if w.chan is not None:
                w.chan.send({"op": "shards", "owned": self.owned_shards, "until": self.shard_until})

    def all_synced(self) -> bool:
        return all(w.synced.is_set() for w in self.workers)

    def alive(self) -> bool:
        return all(w.proc is not None and w.proc.poll() is None for w in self.workers)

    async def wait_synced(self, timeout: Optional[float] = None) -> bool:
        async def one(w):
            done, _ = await asyncio.wait([asyncio.ensure_future(w.synced.wait()), asyncio.ensure_future(w.exited.wait())],
                                         return_when=asyncio.FIRST_COMPLETED)
            for t in _:
                t.cancel()
            return w.synced.is_set()
        try:
            res = await asyncio.wait_for(asyncio.gather(*(one(w) for w in self.workers)), timeout)
        except asyncio.TimeoutError:
            return False
        return all(res)

    async def refresh_metrics(self, timeout: float = 5.0) -> None:
        """Ask every live worker for a fresh metrics state and wait for the answers."""
        self._metrics_seq += 1
        seq = self._metrics_seq
        live = {w.index for w in self.workers if not w.exited.is_set() and w.chan is not None}
        if not live:
            return
        fut = asyncio.get_running_loop().create_future()
        self._metrics_waiters[seq] = (fut, set(live))
        for w in self.workers:
            if w.index in live:
                w.chan.send({"op": "metrics", "seq": seq})
        try:
            await asyncio.wait_for(fut, timeout)
        except asyncio.TimeoutError:
            pass
        finally:
            self._metrics_waiters.pop(seq, None)

    def merged_metrics(self, base: Optional[Metrics] = None) -> Metrics:
        m = Metrics(base.namespace if base else "nexus_supervisor", base.static_tags if base else None)
        if base is not None:
            merge_metrics_state(m, metrics_state(base))
        for w in self.workers:
            if w.state:
                merge_metrics_state(m, w.state, {"worker": str(w.index)})
        return m

    def pids(self) -> List[int]:
        return [w.proc.pid for w in self.workers if w.proc is not None]

    async def stop(self, drain_timeout: float = 10.0) -> None:
        self._stopping = True
        if self._watchdog is not None:
            self._watchdog.cancel()
            try:
                await self._watchdog
            except (asyncio.CancelledError, Exception):
                pass
            self._watchdog = None
        for w in self.workers:
            if w.chan is not None:
                w.chan.send({"op": "stop", "drain": drain_timeout})
        deadline = time.monotonic() + drain_timeout + 5.0
        for w in self.workers:
            if w.proc is None:
                continue
            while w.proc.poll() is None and time.monotonic() < deadline:
                await asyncio.sleep(0.02)
            if w.proc.poll() is None:
                w.proc.terminate()
                try:
                    await asyncio.get_running_loop().run_in_executor(None, w.proc.wait, 5)
                except subprocess.TimeoutExpired:
                    w.proc.kill()
                    w.proc.wait()
        for w in self.workers:
            if w.reader is not None:
                w.reader.cancel()
                try:
                    await w.reader
                except (asyncio.CancelledError, Exception):
                    pass
            if w.chan is not None:
                w.chan.close()
            if w.data is not None:
                w.data.close()


# ---------------------------------------------------------------------- worker side
def _set_pdeathsig() -> None:
    try:
        import ctypes

        libc = ctypes.CDLL(None, use_errno=True)
        libc.prctl(1, signal.SIGTERM)  # PR_SET_PDEATHSIG
    except Exception:  # noqa: BLE001 - best effort (non-Linux)
        pass


async def run_worker(cfg, sock: socket.socket, *, start_active: bool = True, report: bool = False,
                     logger=None, metrics: Optional[Metrics] = None, app_factory=None,
                     data_sock: Optional[socket.socket] = None, remote_gpu: bool = False) -> int:
    """Body of one shard-worker process (also callable in-process by tests)."""
    from ..app import Application

    chan = await Channel.open(sock)
    feed = None
    extra: Dict[str, Any] = {}
    remote_tel = None
    if remote_gpu:
        from ..gpu.telemetry import RemoteTelemetry

        remote_tel = extra["telemetry"] = RemoteTelemetry(cfg.gpu.sample_interval)
    if data_sock is not None:
        # watch-hub mode: informers are fed by the parent's routed stream; the worker still
        # talks to the API server itself for Job DELETEs
        from ..informer import InformerFactory
        from ..kube.client import KubeClient
        from .watchhub import KINDS, HubFeed

        feed = HubFeed()
        await feed.start(data_sock)
        kube = KubeClient.for_config(cfg, metrics)
        factory = InformerFactory(lambda kind: feed.list_watch(kind) if kind in KINDS else None,
                                  resync_period=cfg.resync_period)
        app = (app_factory or Application)(cfg, kube=kube, factory=factory, logger=logger, metrics=metrics, **extra)
    else:
        app = (app_factory or Application)(cfg, logger=logger, metrics=metrics, **extra)
    sup = app.supervisor
    sup.active = start_active
    batch: List[list] = []
    loop = asyncio.get_running_loop()

    def flush():
        if batch:
            chan.send({"op": "dec", "d": batch[:]})
            batch.clear()

    def reporter(d: Decision):
        r = d.result
        if not batch:
            loop.call_soon(flush)
        st = r.stamps
        rec = [r.request_id, r.algorithm, d.outcome, st.get("ack_mono") if st else None, d.new_stage]
        dl = st.get("delivery") if st else None
        if dl is not None and "ack" in st and "receive" in st:
            # delivery stamps + receive→ack split at enqueue and dequeue: the bench decomposes
            # push→ack per decision
            rec.append(delivery_record(st, dl))
        batch.append(rec)

    if report:
        sup.decision_hooks.append(reporter)

    def send_metrics(seq: int) -> None:
        flush()
        collect_gauges(sup, app.metrics)
        chan.send({"op": "metrics", "seq": seq, "s": metrics_state(app.metrics)})

    from ..obs.loopwatch import install_from_env

    install_from_env(app.metrics, "worker")  # diagnostic: NEXUS_SLOW_CALLBACK_MS
    await app.start()

    async def announce_sync():
        if await app.wait_for_cache_sync(None):
            chan.send({"op": "synced"})

    sync_task = asyncio.create_task(announce_sync())
    drain = 10.0
    profiler = None
    try:
        while True:
            line = await chan.recv_line()
            if line is None:
                break
            t_msg = time.perf_counter()
            msg = json.loads(line)
            op = msg.get("op")
            if op == "active":
                if msg.get("until") is not None:
                    sup.set_lease_deadline(float(msg["until"]))
                sup.set_active(bool(msg.get("v")))
            elif op == "metrics":
                send_metrics(int(msg.get("seq", 0)))
            elif op == "shards":
                sup.shards.set_deadlines(msg.get("until") or {})
                sup.set_shards(msg.get("owned") or ())
            elif op == "lease":
                if msg.get("until"):
                    sup.shards.set_deadlines(msg["until"])
                if msg.get("active_until") is not None:
                    sup.set_lease_deadline(float(msg["active_until"]))
            elif op == "gpu" and remote_tel is not None:
                remote_tel.update(msg)
                # the mirror runs on the worker's loop too: a watch frame arriving meanwhile waits
                app.metrics.observe_seconds("worker_gpu_update", time.perf_counter() - t_msg)
                app.metrics.set("worker_gpu_update_bytes", float(len(line)))
            elif op == "pprof":
                profiler = _pprof_op(msg, profiler, cfg.runtime.worker_index)
            elif op == "stop":
                drain = float(msg.get("drain", drain))
                break
    finally:
        sync_task.cancel()
        await app.stop(drain_timeout=drain)
        if feed is not None:
            await feed.close()
        flush()
        send_metrics(-1)
        chan.send({"op": "exit"})
        try:
            await chan.writer.drain()
        except Exception:  # noqa: BLE001
            pass
        chan.close()
    return 0


def _pprof_op(msg: Dict[str, Any], profiler, index: int):
    """``{"op": "pprof", "on": true}`` starts the CPU sampler (SIGPROF, this event loop);
    ``{"on": false, "path": P}`` stops it and writes ``P.w<index>.pb.gz`` + ``.top.txt``."""
    from ..obs.pprof import Sampler

    if msg.get("on"):
        if profiler is None:
            profiler = Sampler(hz=int(msg.get("hz", 199))).start()
        return profiler
    if profiler is not None:
        prof = profiler.stop()
        path = msg.get("path")
        if path:
            with open(f"{path}.w{index}.pb.gz", "wb") as f:
                f.write(prof.encode_gz())
            with open(f"{path}.w{index}.top.txt", "w") as f:
                f.write(prof.top(40))
    return None


def worker_main() -> int:
    """``python -m nexus_supervisor_amd worker`` (spawned by :class:`WorkerPool`)."""
    from .. import __version__
    from ..config import from_mapping
    from ..obs.logging import configure_logging
    from ..obs.metrics import DogStatsd

    _set_pdeathsig()
    cfg = from_mapping(json.loads(os.environ["NEXUS_WORKER_CONFIG"]))
    sock = socket.socket(fileno=int(os.environ["NEXUS_WORKER_CTL_FD"]))
    idx = str(cfg.runtime.worker_index)
    log = configure_logging(cfg.log_level, static={"service": "nexus-supervisor", "worker": idx})
    metrics = Metrics(cfg.observability.statsd_name, {"version": __version__})
    sd = DogStatsd.from_env(cfg.observability.statsd_name)
    if sd is not None:
        sd.tags["worker"] = idx
    metrics.statsd = sd

    async def amain() -> int:
        loop = asyncio.get_running_loop()
        for sig in (signal.SIGTERM, signal.SIGINT):
            loop.add_signal_handler(sig, sock.shutdown, socket.SHUT_RD)  # → EOF → drain and exit
        if sd is not None:
            sd.attach(loop)
        dfd = os.environ.get("NEXUS_WORKER_DATA_FD")
        return await run_worker(cfg, sock, start_active=os.environ.get("NEXUS_WORKER_START_ACTIVE", "1") == "1",
                                report=os.environ.get("NEXUS_WORKER_REPORT", "0") == "1", logger=log, metrics=metrics,
                                data_sock=socket.socket(fileno=int(dfd)) if dfd else None,
                                remote_gpu=os.environ.get("NEXUS_WORKER_REMOTE_GPU", "0") == "1")

    def finish() -> None:
        from ..obs.logging import shutdown_logging

        if sd is not None:
            sd.close()
        shutdown_logging()

    prof_path = os.environ.get("NEXUS_WORKER_CPROFILE")
    if not prof_path:
        try:
            return asyncio.run(amain())
        finally:
            finish()
    import cProfile
    import pstats

    prof = cProfile.Profile()
    prof.enable()
    try:
        return asyncio.run(amain())
    finally:
        prof.disable()
        prof.dump_stats(f"{prof_path}.{idx}.prof")  # raw, for callers/callees analysis
        with open(f"{prof_path}.{idx}.txt", "w") as f:
            pstats.Stats(prof, stream=f).sort_stats("tottime").print_stats(45)
