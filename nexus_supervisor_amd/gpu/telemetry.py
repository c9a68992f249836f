"""GPU telemetry backends and the per-pod evidence record.

:class:`AmdSmiTelemetry` wraps the native monitor (``csrc/amdsmi/gpu_monitor.cpp``
→ ``_amdsmi_monitor``): amd-smi VRAM/process sampling + the GPU event listener,
all in native threads.  :class:`FakeTelemetry` is the programmable stand-in used
on CPU-only hosts and in tests (the sandbox has no ``/dev/kfd``).

:func:`evidence_for` folds a telemetry snapshot into the JSON record the
classifier consumes (``nexus.amd.com/gpu-evidence``, see
:mod:`nexus_supervisor_amd.gpu.oom`): the GPUs the pod's processes ran on, each
with the device-wide VRAM peak *while those processes lived*, the processes'
ranks (from their environment) and GPU events (VM faults, queue evictions,
resets) in that window.

The reference has no GPU awareness (``/root/reference/services/supervisor.go``
classifies on event reasons only); this is the north-star extension.
"""
from __future__ import annotations

import bisect
import os
import threading
import time
from typing import Any, Dict, Iterable, List, Optional

from ..models import kube
from .topology import COLLECTIVE_PREFIXES as _COLLECTIVE_PREFIXES
from .topology import _int, physical_gpu, topology_from_pod

ATTRIBUTION_EVENTS = ("VMFAULT", "QUEUE_EVICTION", "GPU_PRE_RESET", "GPU_POST_RESET", "THERMAL_THROTTLE",
                      "ECC_UNCORRECTABLE", "XGMI_LINK_DOWN", "XGMI_ERROR")
# events that by themselves explain a job failure (hardware / driver faults)
FAULT_EVENTS = ("VMFAULT", "GPU_PRE_RESET", "GPU_POST_RESET", "ECC_UNCORRECTABLE", "XGMI_LINK_DOWN", "XGMI_ERROR")


class TelemetryUnavailable(RuntimeError):
    pass


class GpuTelemetry:
    """Backend protocol. All methods are cheap and non-blocking (snapshots of native state)."""

    name = "none"
    interval = 0.25

    def start(self) -> None:  # pragma: no cover - interface
        raise NotImplementedError

    def stop(self) -> None:  # pragma: no cover - interface
        raise NotImplementedError

    def devices(self) -> List[Dict[str, Any]]:  # pragma: no cover - interface
        raise NotImplementedError

    def snapshot(self, include_exited: bool = True) -> List[Dict[str, Any]]:  # pragma: no cover - interface
        raise NotImplementedError

    def drain_events(self) -> List[Dict[str, Any]]:  # pragma: no cover - interface
        raise NotImplementedError

    def peak_between(self, gpu_index: int, t0: float, t1: float) -> int:  # pragma: no cover - interface
        raise NotImplementedError

    def denials(self) -> Dict[str, int]:
        """Process / sysfs reads the kernel refused so far, by source (``fd``, ``fdinfo``,
        ``environ``, ``proc``, ``sysfs``): non-zero means per-process attribution is
        degraded for lack of privileges."""
        return {}

    def process_vanished(self) -> int:
        """Processes that exited while amd-smi listed them (libamd_smi's "Unable to open
        queues directory" — kept off stderr and counted, ``csrc/amdsmi/stderr_filter.hpp``)."""
        return 0


def native_monitor_module(stub: bool = False):
    """Import the native monitor (``stub``: the build over the stub amd-smi, for CPU
    tests); raises :class:`TelemetryUnavailable` with the build hint."""
    try:
        if stub:
            from .. import _amdsmi_monitor_stub  # type: ignore

            return _amdsmi_monitor_stub
        from .. import _amdsmi_monitor  # type: ignore

        return _amdsmi_monitor
    except ImportError as exc:  # pragma: no cover - exercised on hosts without the build
        raise TelemetryUnavailable(
            "native amd-smi monitor not built: run `python -m nexus_supervisor_amd._build`") from exc


class AmdSmiTelemetry(GpuTelemetry):
    name = "amdsmi"

    def __init__(self, interval: float = 0.25, events: bool = True, retain: float = 600.0, read_proc: bool = True,
                 proc_source: str = "auto", proc_root: str = "/proc", sys_root: str = "/sys", stub: bool = False):
        """``proc_source``: where per-process GPU use comes from — ``auto`` (amd-smi with KFD
        sysfs fill-in when this process shares the host PID namespace, else DRM fdinfo of
        our own /proc), or forced ``amdsmi`` / ``kfd`` / ``drm``."""
        mod = native_monitor_module(stub)
        self._mod = mod
        self.interval = interval
        self._m = mod.GpuMonitor(int(interval * 1000), events, retain, read_proc, proc_source, proc_root, sys_root)
        self._started = False

    def start(self) -> None:
        if not self._started:
            self._m.start()
            self._started = True

    def stop(self) -> None:
        if self._started:
            self._m.stop()
            self._started = False

    def devices(self):
        return self._m.devices()

    def snapshot(self, include_exited: bool = True):
        return self._m.snapshot(include_exited)

    def drain_events(self):
        return self._m.drain_events()

    def inject_event(self, gpu: int, etype: str, message: str = "") -> None:
        self._m.inject_event(gpu, etype, message)

    def peak_between(self, gpu_index: int, t0: float, t1: float) -> int:
        return int(self._m.peak_between(gpu_index, t0, t1))

    def history(self, gpu_index: int, since: float = 0.0):
        return self._m.history(gpu_index, since)

    def denials(self) -> Dict[str, int]:
        fn = getattr(self._mod, "denials", None)
        return dict(fn()) if fn is not None else {}

    def process_vanished(self) -> int:
        return int(getattr(self._m, "process_vanished", 0))

    @property
    def samples(self) -> int:
        return self._m.samples

    @property
    def proc_mode(self) -> str:
        """Per-process source in use (``amdsmi`` / ``kfd`` / ``drm``), known after start()."""
        return self._m.proc_mode


class RemoteTelemetry(GpuTelemetry):
    """Telemetry mirrored from another process's monitor (a shard worker's view of the one
    amd-smi session its replica's parent owns): :meth:`update` applies the parent's
    periodic message — the latest snapshot plus the VRAM samples taken since the last one —
    and every query answers from that mirror."""

    name = "remote"

    def __init__(self, interval: float = 0.5, retain: float = 600.0):
        self.interval = interval
        self.retain = retain
        self._snap: List[Dict[str, Any]] = []
        self._hist: Dict[int, _PeakSeries] = {}
        self.source = ""
        self.updates = 0

    def start(self) -> None:
        return None

    def stop(self) -> None:
        return None

    def update(self, msg: Dict[str, Any]) -> None:
        self.updates += 1
        self.source = msg.get("source", self.source)
        if msg.get("snap") is not None:
            self._snap = msg["snap"]
        horizon = (msg.get("t") or time.time()) - self.retain
        for gi, samples in (msg.get("hist") or {}).items():
            h = self._hist.get(int(gi))
            if h is None:
                h = self._hist[int(gi)] = _PeakSeries()
            h.extend(samples)
            h.trim(horizon)

    def devices(self):
        return [{k: g.get(k) for k in ("index", "uuid", "hip_uuid", "bdf", "vram_total_mb", "links")} for g in self._snap]

    def snapshot(self, include_exited: bool = True):
        if include_exited:
            return self._snap
        return [dict(g, procs=[p for p in g.get("procs", []) if p.get("alive")]) for g in self._snap]

    def drain_events(self):
        return []

    def peak_between(self, gpu_index: int, t0: float, t1: float) -> int:
        h = self._hist.get(int(gpu_index))
        return h.peak(t0, t1) if h is not None else 0


class _PeakSeries:
    """Time-ordered VRAM samples with per-block maxima: a window peak costs a bisect plus
    at most two partial blocks, not a scan of the retained history (the supervisor asks
    for a 300 s lookback peak per failed GPU pod)."""

    B = 64

    def __init__(self):
        self.t: List[float] = []
        self.v: List[int] = []
        self.bmax: List[int] = []

    def __len__(self) -> int:
        return len(self.t)

    def extend(self, samples) -> None:
        t, v, bmax, B = self.t, self.v, self.bmax, self.B
        for ts, mb in samples:
            ts, mb = float(ts), int(mb)
            if t and ts < t[-1]:
                continue  # out of order (a resent sample): the series stays sorted
            if len(t) % B == 0:
                bmax.append(mb)
            elif mb > bmax[-1]:
                bmax[-1] = mb
            t.append(ts)
            v.append(mb)

    def trim(self, horizon: float) -> None:
        i = bisect.bisect_left(self.t, horizon)
        if i >= self.B:  # drop whole blocks only (keeps the block alignment)
            cut = (i // self.B) * self.B
            del self.t[:cut]
            del self.v[:cut]
            del self.bmax[:cut // self.B]

    def peak(self, t0: float, t1: float) -> int:
        lo = bisect.bisect_left(self.t, t0)
        hi = bisect.bisect_right(self.t, t1)
        if lo >= hi:
            return 0
        B, v = self.B, self.v
        b0, b1 = -(-lo // B), hi // B  # whole blocks [b0, b1)
        if b0 >= b1:
            return max(v[lo:hi])
        best = max(self.bmax[b0:b1])
        if lo < b0 * B:
            best = max(best, max(v[lo:b0 * B]))
        if b1 * B < hi:
            best = max(best, max(v[b1 * B:hi]))
        return best


def telemetry_message(tel: GpuTelemetry, since: Dict[int, float]) -> Dict[str, Any]:
    """What a telemetry owner forwards to its mirrors (:class:`RemoteTelemetry`): the snapshot
    and each GPU's VRAM samples newer than ``since`` (advanced in place)."""
    snap = tel.snapshot(True)
    hist: Dict[str, List] = {}
    hist_fn = getattr(tel, "history", None)
    for g in snap:
        gi = g["index"]
        if hist_fn is not None:
            samples = hist_fn(gi, since.get(gi, 0.0))
        else:  # backends without a history: the current reading as one sample
            samples = [(time.time(), g.get("vram_used_mb", 0))]
        if samples:
            since[gi] = samples[-1][0]
            hist[str(gi)] = [[t, mb] for t, mb in samples]
    return {"source": tel.name, "t": time.time(), "snap": snap, "hist": hist}


class FakeTelemetry(GpuTelemetry):
    """In-memory node model: N MI355X GPUs (288 GB HBM3E each), programmable processes,
    VRAM usage and events — same snapshot format as the native monitor."""

    name = "fake"

    def __init__(self, n_gpus: int = 8, vram_total_mb: int = 294896, clock=time.time):
        self.clock = clock
        self._lock = threading.Lock()
        bdf = [f"0000:{0x0a + i:02x}:00.0" for i in range(n_gpus)]
        # MI355X node fabric: every GPU pair joined by one xGMI link (7 per GPU on 8 GPUs)
        self._gpus = [{"index": i, "uuid": f"fake-{i:04d}", "hip_uuid": f"GPU-fake{i:012d}", "bdf": bdf[i],
                       "vram_total_mb": vram_total_mb, "vram_used_mb": 0, "vram_peak_mb": 0,
                       "ecc_correctable": 0, "ecc_uncorrectable": 0, "xgmi_hive_id": 0x5A7E,
                       "links": [{"peer_bdf": bdf[j], "peer_index": j, "type": "xgmi", "bit_rate_gbps": 38,
                                  "max_bandwidth_gbps": 608, "read_kb": 0, "write_kb": 0}
                                 for j in range(n_gpus) if j != i]} for i in range(n_gpus)]
        self._hist: List[List] = [[] for _ in range(n_gpus)]
        self._procs: Dict[tuple, Dict[str, Any]] = {}
        self._events: List[Dict[str, Any]] = []
        self._pending: List[Dict[str, Any]] = []

    def start(self):
        return None

    def stop(self):
        return None

    def devices(self):
        with self._lock:
            return [{k: g[k] for k in ("index", "uuid", "hip_uuid", "bdf", "vram_total_mb", "links")} | {"hip_id": g["index"],
                    "market_name": "AMD Instinct MI355X (fake)", "events": True} for g in self._gpus]

    # ---- programming API
    def set_vram(self, gpu: int, used_mb: int, t: Optional[float] = None) -> None:
        with self._lock:
            g = self._gpus[gpu]
            g["vram_used_mb"] = used_mb
            g["vram_peak_mb"] = max(g["vram_peak_mb"], used_mb)
            self._hist[gpu].append((self.clock() if t is None else t, used_mb))

    def add_process(self, pid: int, gpu: int, vram_bytes: int = 0, env: Optional[Dict[str, str]] = None,
                    pod_uid: str = "", name: str = "python3") -> None:
        now = self.clock()
        with self._lock:
            self._procs[(gpu, pid)] = {"pid": pid, "name": name, "source": "fake", "vram_bytes": vram_bytes,
                                       "peak_vram_bytes": vram_bytes,
                                       "cu_occupancy": 0, "alive": True, "first_seen": now, "last_seen": now,
                                       "pod_uid": pod_uid, "env": dict(env or {}), "gpu": gpu}

    def update_process(self, pid: int, gpu: int, vram_bytes: int) -> None:
        with self._lock:
            p = self._procs[(gpu, pid)]
            p["vram_bytes"] = vram_bytes
            p["peak_vram_bytes"] = max(p["peak_vram_bytes"], vram_bytes)
            p["last_seen"] = self.clock()

    def end_process(self, pid: int, gpu: int) -> None:
        with self._lock:
            p = self._procs[(gpu, pid)]
            p["alive"] = False
            p["last_seen"] = self.clock()
        self.inject_event(gpu, "PROCESS_END", f"pid {pid}")

    def set_xgmi(self, gpu: int, total: int = 7, down: int = 0, error: int = 0) -> None:
        """Link / fabric health as the native monitor reports it (events on degradation)."""
        with self._lock:
            g = self._gpus[gpu]
            prev_down, prev_err = g.get("xgmi_links_down", 0), g.get("xgmi_error", 0)
            g.update(xgmi_links_total=total, xgmi_links_up=total - down, xgmi_links_down=down, xgmi_error=error)
        if down > prev_down:
            self.inject_event(gpu, "XGMI_LINK_DOWN", f"{down}/{total} xGMI links down")
        if error and not prev_err:
            self.inject_event(gpu, "XGMI_ERROR", f"xGMI error status {error}")

    def set_ecc(self, gpu: int, uncorrectable: int, correctable: int = 0) -> None:
        with self._lock:
            g = self._gpus[gpu]
            prev = g["ecc_uncorrectable"]
            g["ecc_uncorrectable"], g["ecc_correctable"] = uncorrectable, correctable
        if uncorrectable > prev:
            self.inject_event(gpu, "ECC_UNCORRECTABLE", f"{uncorrectable - prev} new uncorrectable ECC error(s)")

    def inject_event(self, gpu: int, etype: str, message: str = "") -> None:
        e = {"gpu": gpu, "type": etype, "message": message, "t": self.clock()}
        with self._lock:
            self._events.append(e)
            self._pending.append(e)

    # ---- protocol
    def snapshot(self, include_exited: bool = True):
        with self._lock:
            out = []
            for g in self._gpus:
                d = dict(g)
                d["procs"] = [{k: v for k, v in p.items() if k != "gpu"} for p in self._procs.values()
                              if p["gpu"] == g["index"] and (p["alive"] or include_exited)]
                d["events"] = [dict(e) for e in self._events if e["gpu"] == g["index"]][-256:]
                out.append(d)
            return out

    def drain_events(self):
        with self._lock:
            out, self._pending = self._pending, []
            return out

    def peak_between(self, gpu_index: int, t0: float, t1: float) -> int:
        with self._lock:
            return max((u for t, u in self._hist[gpu_index] if t0 <= t <= t1), default=0)

    def history(self, gpu_index: int, since: float = 0.0):
        with self._lock:
            return [(t, u) for t, u in self._hist[gpu_index] if t > since]


def has_amd_gpu() -> bool:
    return os.path.exists("/dev/kfd")


def make_telemetry(backend: str = "auto", interval: float = 0.25, events: bool = True) -> Optional[GpuTelemetry]:
    """``auto``: native amd-smi when a GPU is present (fails loudly if the extension is
    missing there), else none; ``amdsmi``/``fake``/``none`` force a backend.  ``events``
    False skips the amd-smi event listener (VRAM/process sampling only)."""
    if backend == "none":
        return None
    if backend == "fake":
        return FakeTelemetry()
    if backend == "amdsmi" or (backend == "auto" and has_amd_gpu()):
        return AmdSmiTelemetry(interval=interval, events=events)
    return None


def _rank_fields(env: Dict[str, str]) -> Dict[str, Any]:
    out: Dict[str, Any] = {}
    for var, key in (("RANK", "rank"), ("LOCAL_RANK", "local_rank"), ("WORLD_SIZE", "world_size"),
                     ("LOCAL_WORLD_SIZE", "local_world_size")):
        v = _int(env.get(var))
        if v is not None:
            out[key] = v
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES"):
        if env.get(var):
            out["visible_devices"] = env[var]
            break
    return out


def _links_of(g: Dict[str, Any]) -> Optional[List[Dict[str, Any]]]:
    """Connected xGMI ports of one GPU (disabled ports report an all-ones peer BDF)."""
    raw = g.get("links")
    if raw is None:
        return None
    out = []
    for l in raw:
        peer = l.get("peer_bdf") or ""
        if not peer or peer.startswith("ffff") or l.get("type") not in ("xgmi", None):
            continue
        # no cumulative read/write counters: they grow without bound and say nothing about
        # a failure, and the trace row is bounded
        out.append({"peer_bdf": peer, "peer": l.get("peer_index") if (l.get("peer_index") or 0) >= 0 else None,
                    "gbps": l.get("bit_rate_gbps"), "max_gbps": l.get("max_bandwidth_gbps")})
    return out


class _LazyLinks(dict):
    """GPU index → :func:`_links_of`, computed on first use per snapshot: a failure asks for
    the links of the one or two GPUs its pod used, not all eight (at a low failure rate
    every decision meets a fresh snapshot, and the eager table was most of its cost)."""

    __slots__ = ("_by_index",)

    def __init__(self, snap: Iterable[Dict[str, Any]]):
        super().__init__()
        self._by_index = {g["index"]: g for g in snap}

    def __missing__(self, index: int):
        g = self._by_index.get(index)
        v = self[index] = _links_of(g) if g is not None else None
        return v


def evidence_for(telemetry: GpuTelemetry, pod_uid: str = "", gpu_indices: Iterable[int] = (), pids: Iterable[int] = (),
                 lookback: float = 300.0, now: Optional[float] = None, node: str = "",
                 snapshot: Optional[List[Dict[str, Any]]] = None,
                 allocated: Optional[List[int]] = None,
                 links: Optional[Dict[int, Any]] = None) -> Optional[Dict[str, Any]]:
    """Evidence record for one pod (matched by cgroup pod UID, PIDs or explicit GPU indices).

    Per GPU: the device-wide VRAM peak over the window the pod's processes lived (or the
    lookback when none matched), the pod's own processes with their per-process VRAM and
    peak (``source``: amdsmi / kfd / drm-fdinfo), the measured xGMI links, GPU events in
    the window and usage by processes of other PID namespaces.  ``allocated`` (physical
    indices from the kubelet pod-resources API) is recorded so the supervisor can map the
    pod's logical HIP ordinals to physical GPUs (:func:`..topology.resolve_devices`)."""
    snap = snapshot if snapshot is not None else telemetry.snapshot(True)
    now = time.time() if now is None else now
    pids = set(pids)
    wanted = set(int(i) for i in gpu_indices)
    grace = 2 * max(telemetry.interval, 0.05)
    gpus = []
    for g in snap:
        procs = [p for p in g.get("procs", [])
                 if (pod_uid and p.get("pod_uid") == pod_uid) or (p.get("pid") in pids)]
        if not procs and g["index"] not in wanted:
            continue
        if procs:
            t0 = min(p["first_seen"] for p in procs) - grace
            t1 = max(p["last_seen"] for p in procs) + grace
        else:
            t0, t1 = now - lookback, now
        peak = telemetry.peak_between(g["index"], t0, t1) or 0
        rec: Dict[str, Any] = {"index": g["index"], "uuid": g.get("hip_uuid") or g.get("uuid"),
                               "bdf": g.get("bdf"), "vram_total_mb": g.get("vram_total_mb"),
                               "vram_used_mb": g.get("vram_used_mb"), "vram_peak_mb": peak,
                               "window": [round(t0, 3), round(t1, 3)], "matched": bool(procs)}
        if g.get("ecc_uncorrectable"):
            rec["ecc_uncorrectable"] = g["ecc_uncorrectable"]
        if g.get("xgmi_links_total") is not None:
            rec["xgmi_links_up"] = g.get("xgmi_links_up")
            rec["xgmi_links_down"] = g.get("xgmi_links_down") or 0
            rec["xgmi_links_total"] = g.get("xgmi_links_total")
        if g.get("xgmi_error"):
            rec["xgmi_error"] = g["xgmi_error"]
        if g.get("xgmi_hive_id"):
            rec["xgmi_hive_id"] = g["xgmi_hive_id"]
        glinks = (links[g["index"]] if links is not None and (type(links) is _LazyLinks or g["index"] in links)
                  else _links_of(g))
        if glinks is not None:
            rec["links"] = glinks
        if g.get("foreign_procs"):
            rec["foreign_procs"] = g["foreign_procs"]
            rec["foreign_vram_bytes"] = g.get("foreign_vram_bytes", 0)
        holders = _holders(g.get("procs", ()), procs, t0 - grace, t1 + grace)
        if holders:
            rec["holders"] = holders
        rec["procs"] = [dict({"pid": p["pid"], "vram_bytes": p.get("vram_bytes", 0),
                              "peak_vram_bytes": p.get("peak_vram_bytes", 0), "alive": p.get("alive", False),
                              "source": p.get("source", "")},
                             **_rank_fields(p.get("env") or {})) for p in procs]
        if procs:
            rec["proc_peak_vram_bytes"] = sum(p.get("peak_vram_bytes", 0) for p in procs)
        evs = [{"type": e["type"], "t": round(e["t"], 3), "message": (e.get("message") or "")[:200]}
               for e in g.get("events", []) if e["type"] in ATTRIBUTION_EVENTS and t0 <= e["t"] <= t1 + grace]
        if evs:
            rec["events"] = evs
        gpus.append(rec)
    if not gpus:
        return None
    out: Dict[str, Any] = {"source": telemetry.name, "t": round(now, 3), "gpus": gpus}
    coll: Dict[str, str] = {}
    for g in snap:
        for p in g.get("procs", ()):
            if (pod_uid and p.get("pod_uid") == pod_uid) or p.get("pid") in pids:
                for k, v in (p.get("env") or {}).items():
                    if k.startswith(_COLLECTIVE_PREFIXES) and k not in coll:
                        coll[k] = v
    if coll:
        # the RCCL / NCCL env of the pod's processes (/proc/<pid>/environ), once per pod
        out["collective_env"] = dict(sorted(coll.items()))
    if allocated:
        out["allocated"] = sorted(int(i) for i in allocated)
    if node:
        out["node"] = node
    if pod_uid:
        out["pod_uid"] = pod_uid
    return out


def node_gpu_health(telemetry: GpuTelemetry, lookback: float = 600.0, now: Optional[float] = None,
                    snapshot: Optional[List[Dict[str, Any]]] = None,
                    allocatable_bdfs: Optional[Iterable[str]] = None) -> Dict[str, Any]:
    """Health of every GPU of the node, for a pod the kubelet refused at admission (it never
    got a GPU, so no per-GPU record of its own exists): the GPUs amd-smi sees, and per
    unhealthy GPU what is wrong — uncorrectable ECC errors, xGMI links down or in error,
    resets / VM faults / ECC / xGMI events in the ``lookback`` window.  With the kubelet's
    allocatable device set (pod-resources ``GetAllocatableResources``, by PCI BDF) the GPUs
    amd-smi sees but the device plugin no longer offers are listed too
    (``not_allocatable``): the usual shape of "the device plugin marked a GPU unhealthy"."""
    from .podresources import normalize_bdf

    snap = snapshot if snapshot is not None else telemetry.snapshot(False)
    now = time.time() if now is None else now
    alloc = None if allocatable_bdfs is None else {normalize_bdf(b) for b in allocatable_bdfs}
    unhealthy: List[Dict[str, Any]] = []
    not_alloc: List[int] = []
    for g in snap:
        problems: List[str] = []
        if g.get("ecc_uncorrectable"):
            problems.append(f"ecc_uncorrectable={g['ecc_uncorrectable']}")
        if g.get("xgmi_links_down"):
            problems.append(f"xgmi_links_down={g['xgmi_links_down']}/{g.get('xgmi_links_total')}")
        if g.get("xgmi_error"):
            problems.append(f"xgmi_error={g['xgmi_error']}")
        evs = [{"type": e["type"], "t": round(e["t"], 3), "message": (e.get("message") or "")[:200]}
               for e in g.get("events", ()) if e.get("type") in FAULT_EVENTS and e.get("t", 0) >= now - lookback]
        if evs:
            problems.append("events=" + ",".join(sorted({e["type"] for e in evs})))
        if alloc is not None and g.get("bdf") and normalize_bdf(g["bdf"]) not in alloc:
            not_alloc.append(g["index"])
            problems.append("not in the kubelet's allocatable set")
        if problems:
            rec: Dict[str, Any] = {"index": g["index"], "uuid": g.get("hip_uuid") or g.get("uuid"), "bdf": g.get("bdf"),
                                   "problems": problems}
            if evs:
                rec["events"] = evs[-TRACE_EVENTS:]
            unhealthy.append(rec)
    out: Dict[str, Any] = {"gpus_seen": len(snap), "healthy": sorted(g["index"] for g in snap
                                                                      if g["index"] not in {u["index"] for u in unhealthy}),
                           "unhealthy": unhealthy}
    if alloc is not None:
        out["allocatable"] = len(alloc)
        out["not_allocatable"] = not_alloc
    return out


TRACE_EVENTS = 4  # fault events per unhealthy GPU in a node-health record


def admission_evidence(telemetry: GpuTelemetry, pod: Dict[str, Any], node: str = "", lookback: float = 600.0,
                       allocatable_bdfs: Optional[Iterable[str]] = None) -> Dict[str, Any]:
    """Evidence record (same envelope as :func:`evidence_for`) for a pod refused at kubelet
    admission: no per-GPU records, the node's GPU health instead."""
    out: Dict[str, Any] = {"source": telemetry.name, "t": round(time.time(), 3), "gpus": [],
                           "node_health": node_gpu_health(telemetry, lookback, allocatable_bdfs=allocatable_bdfs)}
    n = node or (pod.get("spec") or {}).get("nodeName", "")
    if n:
        out["node"] = n
    uid = kube.uid_of(pod)
    if uid:
        out["pod_uid"] = uid
    return out


HOLDERS_MAX = 4  # other processes listed per GPU, largest VRAM peak first


def _holders(all_procs, own, t0: float, t1: float) -> List[Dict[str, Any]]:
    """The *other* processes that held memory on a GPU while the pod's processes lived (or
    in the lookback when none of them was seen): what filled a GPU a pod then ran out of,
    or crashed on at init — a zombie of a previous tenant, another job, a host process.
    Each names its pod (cgroup pod UID) or ``host``; largest peak first, at most
    :data:`HOLDERS_MAX`."""
    mine = {id(p) for p in own}
    out = []
    for p in all_procs:
        if id(p) in mine:
            continue
        peak = p.get("peak_vram_bytes") or p.get("vram_bytes") or 0
        if not peak or p.get("first_seen", t0) > t1 or p.get("last_seen", t1) < t0:
            continue
        out.append((peak, p))
    if not out:
        return []
    out.sort(key=lambda x: (-x[0], x[1].get("pid") or 0))
    return [{"pid": p.get("pid"), "vram_bytes": peak, "owner": p.get("pod_uid") or "host",
             "name": p.get("name") or "", "alive": bool(p.get("alive"))} for peak, p in out[:HOLDERS_MAX]]


def pod_evidence_provider(telemetry: GpuTelemetry, gpu_resource: str = "amd.com/gpu", node: str = "",
                          lookback: float = 300.0):
    """Classifier hook (``Classifier.evidence_provider``): live evidence for a pod from a
    co-located telemetry backend, matched by pod UID (cgroup) or the pod's expected GPU
    (``visible_devices[local_rank]`` from its env)."""
    cache: Dict[str, Any] = {"t": -1.0, "snap": None, "by_uid": {}, "by_index": {}, "memo": {}}
    ttl = max(0.005, telemetry.interval / 2)  # the native sampler cannot have anything newer

    def refresh(now: float) -> None:
        snap = telemetry.snapshot(True)
        if snap is cache["snap"]:
            # a mirror (RemoteTelemetry) hands back the same list until its owner's next
            # update, which also carries the new VRAM samples: tables and memo stay exact
            cache["t"] = now
            return
        by_uid: Dict[str, set] = {}
        for g in snap:
            for p in g.get("procs", ()):
                u = p.get("pod_uid")
                if u:
                    by_uid.setdefault(u, set()).add(g["index"])
        cache.update(t=now, wall=time.time(), snap=snap, by_uid=by_uid, by_index={g["index"]: g for g in snap},
                     links=_LazyLinks(snap), memo={})

    def provider(pod: Dict[str, Any]) -> Optional[Dict[str, Any]]:
        if kube.admission_rejection(pod) is not None:
            # refused by the kubelet before any GPU was allocated: the node's GPU health
            return admission_evidence(telemetry, pod, node=node, lookback=lookback)
        topo = topology_from_pod(pod, gpu_resource)
        now = time.monotonic()
        if cache["snap"] is None or now - cache["t"] > ttl:
            refresh(now)
        gpus = _pod_gpus(topo, cache["snap"])
        uid = kube.uid_of(pod)
        pod_node = node or (pod.get("spec") or {}).get("nodeName", "")
        mine = cache["by_uid"].get(uid)
        by_index = cache["by_index"]
        if not mine:
            # no process of this pod on any GPU: its evidence is the expected devices' records
            # of this snapshot, the same for every such pod — built once per snapshot (a burst
            # of failures on one node shares them; the per-GPU records are never mutated)
            key = (tuple(gpus), pod_node)
            hit = cache["memo"].get(key)
            if hit is None:
                sub = [by_index[i] for i in sorted(set(gpus)) if i in by_index]
                hit = cache["memo"][key] = (evidence_for(telemetry, gpu_indices=gpus, lookback=lookback, node=pod_node,
                                                         snapshot=sub, links=cache["links"], now=cache["wall"]),)
            if hit[0] is None:
                return None
            out = dict(hit[0])
            if uid:
                out["pod_uid"] = uid
            return out
        # only the GPUs this pod could have used: its expected devices + where its processes ran
        relevant = set(gpus) | mine
        sub = [by_index[i] for i in sorted(relevant) if i in by_index]
        return evidence_for(telemetry, pod_uid=uid, gpu_indices=gpus, lookback=lookback, node=pod_node, snapshot=sub,
                            links=cache["links"])

    return provider


_POD_GPUS_MEMO: Dict[Any, List[int]] = {}


def _pod_gpus(topo: Dict[str, Any], snap: Iterable[Dict[str, Any]] = ()) -> List[int]:
    """Physical GPUs a pod's env points at: the rank's expected device, else every visible
    device; UUID entries resolved against the telemetry snapshot.  Memoised when the device
    chain is plain indices (then the snapshot plays no part): every rank of a template on
    a node asks the same question."""
    lr = topo.get("local_rank")
    devs = topo.get("visible_devices") or []
    chain = topo.get("device_chain")
    key = None
    if chain is not None and all(x.isdigit() for _v, sel in chain for x in sel):
        key = (lr, tuple(tuple(sel) for _v, sel in chain))
        hit = _POD_GPUS_MEMO.get(key)
        if hit is not None:
            return hit
    out = _pod_gpus_of(topo, lr, devs, snap)
    if key is not None:
        if len(_POD_GPUS_MEMO) > 1024:
            _POD_GPUS_MEMO.clear()
        _POD_GPUS_MEMO[key] = out
    return out


def _pod_gpus_of(topo, lr, devs, snap) -> List[int]:
    out = []
    if devs and lr is not None and 0 <= lr < len(devs):
        p = physical_gpu(topo, lr, snap)
        if p is not None:
            out.append(p)
    elif devs:
        for i in range(len(devs)):
            p = physical_gpu(topo, i, snap)
            if p is not None:
                out.append(p)
    return out
