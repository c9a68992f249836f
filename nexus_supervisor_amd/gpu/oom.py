"""HBM-OOM vs host-OOM attribution (north star).

Scored-evidence model — every signal adds weight to one hypothesis and is
recorded, so the trace row says *why*:

host-OOM
  * container ``terminated.reason == "OOMKilled"`` (cgroup OOM, exit 137)  +1.0
  * bare exit 137 (SIGKILL) without reason                                  +0.35
  * in-process host allocation failure (Python ``MemoryError``, numpy
    ``_ArrayMemoryError`` / ``Unable to allocate … for an array``, ``std::bad_alloc``,
    ``java.lang.OutOfMemoryError``, Go ``runtime: out of memory``, V8 ``heap out of
    memory``, ``Cannot allocate memory``)                                   +0.6
HBM-OOM (288 GB HBM3E per MI355X)
  * HIP OOM signature in the termination / event message or in the container's log
    tail (``hipErrorOutOfMemory``, ``HIP out of memory``, torch ``OutOfMemoryError``,
    RCCL/hipMalloc allocation failures; :mod:`.logtail` reads the tail from the node's
    ``/var/log/pods`` or the ``pods/log`` API, because a default pod's termination
    message is empty — PyTorch prints its OOM to stderr and exits 1)           +1.0
  * the pod's OWN processes (cgroup pod UID / PID match) peaked at
    ≥ ``hbm_oom_fraction`` × capacity and the container exited non-zero       +0.75
  * agent-sampled device-wide VRAM peak ≥ ``hbm_oom_fraction`` × capacity    +0.5
  * VM-fault / queue-eviction event on that GPU                             +0.25

A verdict needs ≥0.5 **and** at least one OOM *signature* (an allocation-failure message
or log line, OOMKilled or exit 137).  VRAM numbers — even the pod's own processes filling
the GPU — and GPU events corroborate and attribute, they never make a plain crash an OOM
on their own: PyTorch's caching allocator routinely holds nearly all of a GPU, so an
exit-1 from a NaN assert or an RCCL timeout on a full GPU is *not* an HBM-OOM, and a GPU
left full by a previous tenant must not bypass the Job's retry policy either (the
classifier reads the container log tail first, :class:`..classify.Classifier`).

HBM needs a GPU.  ``gpu_involved=False`` (the pod requests no ``amd.com/gpu`` and no GPU
process of its own was seen) turns every HBM signal into a recorded non-verdict: a
CPU-only pod whose JVM runs out of heap is never written as "ran out of GPU memory" (the
reference writes a plain fatal error and never claims a device,
``/root/reference/services/supervisor.go:194-204,310-335``).  ``None`` = unknown (no pod
in the cache): only the anchored HIP/torch texts count.

The larger score wins; a cgroup OOMKill (a hard kernel fact
about *host* memory) is beaten only by HIP's own words, never by VRAM numbers.  Every
signal names its source (termination message, node-log / pods/log tail, own-process
peak, device peak).

GPU index.  torch's ``GPU N`` is the *logical* HIP ordinal inside the process, after
ROCR/HIP_VISIBLE_DEVICES and the device plugin's allocation narrowed the node's GPUs.
With the pod's topology the verdict records both ``gpu_logical_index`` (N) and
``gpu_index`` (the physical GPU, :func:`..topology.physical_gpu`), and only the physical
GPU's telemetry is read.  Per-process VRAM (the pod's own processes on that GPU) is
preferred over the device-wide peak for ``peak_vram_bytes``.
"""
from __future__ import annotations

import re
from dataclasses import dataclass, field
from typing import Any, Dict, Iterable, List, Optional, Tuple

from .topology import physical_gpu

HBM_PATTERNS = [
    re.compile(r"hipErrorOutOfMemory", re.I),
    re.compile(r"\bHIP out of memory", re.I),
    re.compile(r"\bCUDA out of memory", re.I),  # torch wording on some ROCm builds
    # torch's exception class only: a bare "OutOfMemoryError" is also Java's heap OOM
    re.compile(r"\btorch(?:\.cuda)?\.OutOfMemoryError\b"),
    re.compile(r"hipMalloc(?:Managed|Async)?\b[^\n]{0,80}(?:fail|out of memory|error)", re.I),
    re.compile(r"(?:NCCL|RCCL)[^\n]{0,120}out of memory", re.I),
    re.compile(r"HSA_STATUS_ERROR_OUT_OF_RESOURCES", re.I),
    re.compile(r"\bGPU\b[^\n]{0,40}out of memory", re.I),
    re.compile(r"RESOURCE_EXHAUSTED: Out of memory while trying to allocate", re.I),
    # runtime-check wordings: torch's C10_HIP_CHECK / C10_CUDA_CHECK ("HIP error: out of
    # memory") when the HIP context, a hipBLAS handle or RCCL cannot allocate on a full GPU
    re.compile(r"\b(?:HIP|CUDA) error: out of memory", re.I),
    re.compile(r"hipErrorMemoryAllocation"),
    # math-library allocation failures: hipBLAS(Lt) / cuBLAS workspace, rocBLAS, MIOpen
    re.compile(r"\b(?:HIPBLAS|CUBLAS)(?:LT)?_STATUS_ALLOC_FAILED\b"),
    re.compile(r"\brocblas_status_memory_error\b"),
    re.compile(r"\bmiopenStatusAllocFailed\b"),
]
HOST_PATTERNS = [
    re.compile(r"\bMemoryError\b"),
    re.compile(r"\b_ArrayMemoryError\b"),                                  # numpy
    re.compile(r"Unable to allocate [\d.]+ [KMGTP]?i?B for an array", re.I),  # numpy's message
    re.compile(r"std::bad_alloc"),
    re.compile(r"\bjava\.lang\.OutOfMemoryError\b"),
    re.compile(r"\bruntime: out of memory"),                                # Go
    re.compile(r"JavaScript heap out of memory"),                           # Node / V8
    re.compile(r"Cannot allocate memory", re.I),
    re.compile(r"Memory cgroup out of memory", re.I),
    re.compile(r"\bOOMKilled\b"),
    # torch's CPU allocator ("[enforce fail at alloc_cpu.cpp] . DefaultCPUAllocator: not
    # enough memory: you tried to allocate N bytes")
    re.compile(r"DefaultCPUAllocator: (?:not enough memory|can't allocate memory)", re.I),
]

# Literal keywords every pattern of a list contains (lower-cased): a substring scan of the
# lower-cased text rejects the common no-match message in well under a microsecond, where
# the case-insensitive regex list costs ~10 µs per message.
_HBM_KEYS = ("out of memory", "outofmemory", "hipmalloc", "out_of_resources", "memoryallocation",
             "alloc_failed", "memory_error", "allocfailed")
_HOST_KEYS = ("memoryerror", "bad_alloc", "cannot allocate memory", "out of memory", "oomkilled",
              "unable to allocate", "outofmemoryerror", "defaultcpuallocator")
_TORCH_KEYS = ("total capacity", "tried to allocate")


def _mentions(text: str, keys) -> bool:
    low = text.lower()
    for k in keys:
        if k in low:
            return True
    return False

# "someone else filled the GPU": the device at or above this share of its HBM in the
# window while the pod's own processes held under OWN_SHARE_MAX of it
FOREIGN_FULL_FRACTION = 0.95
OWN_SHARE_MAX = 0.10

_TORCH_GPU = re.compile(r"GPU (\d+) has a total capacity of ([\d.]+) (GiB|MiB|GB|MB)", re.I)
_TORCH_REQ = re.compile(r"Tried to allocate ([\d.]+) (GiB|MiB|GB|MB|KiB)", re.I)
_UNIT = {"gib": 1 << 30, "gb": 1 << 30, "mib": 1 << 20, "mb": 1 << 20, "kib": 1 << 10}


@dataclass
class OomVerdict:
    kind: Optional[str] = None  # "hbm" | "host" | None
    hbm_score: float = 0.0
    host_score: float = 0.0
    signals: List[str] = field(default_factory=list)
    gpu_index: Optional[int] = None
    gpu_logical_index: Optional[int] = None
    requested_bytes: Optional[int] = None
    capacity_bytes: Optional[int] = None
    peak_vram_bytes: Optional[int] = None
    device_peak_vram_bytes: Optional[int] = None
    signature: bool = False
    oomkilled: bool = False
    hbm_text: bool = False
    host_text: bool = False
    # the GPU was full of someone else's memory (:data:`FOREIGN_FULL_FRACTION`, the pod's own
    # share under :data:`OWN_SHARE_MAX`): who held it — recorded whatever the verdict
    foreign: Optional[Dict[str, Any]] = None

    @property
    def text_signature(self) -> bool:
        """Backed by an allocation-failure text or a cgroup OOMKill (not only exit codes
        and VRAM numbers): nothing a container log could still overrule."""
        return self.hbm_text or self.host_text or self.oomkilled

    def as_dict(self) -> Dict[str, Any]:
        d: Dict[str, Any] = {"kind": self.kind, "hbm_score": round(self.hbm_score, 3),
                             "host_score": round(self.host_score, 3), "signals": self.signals}
        for k in ("gpu_index", "gpu_logical_index", "requested_bytes", "capacity_bytes", "peak_vram_bytes",
                  "device_peak_vram_bytes"):
            v = getattr(self, k)
            if v is not None:
                d[k] = v
        if self.foreign is not None:
            d["foreign_occupancy"] = True
        return d


# text -> (hbm signature, host signature): failures of one job template repeat the same
# termination message (a torch OOM line, an OOMKilled reason) run after run, and the
# keyword scan + up to ten regexes cost ~5-20 µs per text; a hit is one dict lookup
_SIG_MEMO: Dict[str, Tuple[Optional[str], Optional[str]]] = {}
_SIG_MEMO_MAX = 4096
_SIG_MEMO_TEXT = 4096  # longer texts (log tails) are scanned, not memoised


def _scan(text: str, keys, patterns) -> Optional[str]:
    if not _mentions(text, keys):
        return None
    for p in patterns:
        m = p.search(text)
        if m:
            return m.group(0)
    return None


def signatures(text: str) -> Tuple[Optional[str], Optional[str]]:
    """``(hbm_signature(text), host_signature(text))``, memoised for short texts."""
    hit = _SIG_MEMO.get(text)
    if hit is not None:
        return hit
    got = (_scan(text, _HBM_KEYS, HBM_PATTERNS), _scan(text, _HOST_KEYS, HOST_PATTERNS))
    if len(text) <= _SIG_MEMO_TEXT:
        if len(_SIG_MEMO) >= _SIG_MEMO_MAX:
            _SIG_MEMO.clear()
        _SIG_MEMO[text] = got
    return got


def hbm_signature(text: str) -> Optional[str]:
    return signatures(text)[0]


def host_signature(text: str) -> Optional[str]:
    return signatures(text)[1]


def gpu_involved(gpus_requested: int, gpu_evidence: Optional[Dict[str, Any]]) -> bool:
    """Did the pod use a GPU: it requests one, or the evidence matched its own processes
    on one (a pod that reaches /dev/kfd without requesting amd.com/gpu)."""
    if gpus_requested > 0:
        return True
    for g in (gpu_evidence or {}).get("gpus") or ():
        if g.get("matched") or g.get("proc_peak_vram_bytes") or g.get("procs"):
            return True
    return False


def analyze(
    texts: Iterable[Any] = (),
    terminated: Iterable[Dict[str, Any]] = (),
    gpu_evidence: Optional[Dict[str, Any]] = None,
    expected_gpu: Optional[str] = None,
    hbm_capacity_gb: float = 288.0,
    hbm_oom_fraction: float = 0.97,
    topo: Optional[Dict[str, Any]] = None,
    gpu_involved: Optional[bool] = None,
) -> OomVerdict:
    """``texts``: strings (a termination / event / condition message) or ``(source, text)``
    pairs (container log tails, :mod:`.logtail`) — every signal names where it was found.
    ``gpu_involved``: see the module docstring (False = no HBM verdict possible)."""

    v = OomVerdict()
    sourced: List[Tuple[str, str]] = []
    for t in texts:
        if isinstance(t, tuple):
            if t[1]:
                sourced.append((t[0], t[1]))
        elif t:
            sourced.append(("message", t))
    failed_exit = False
    for t in terminated:
        reason = t.get("reason") or ""
        code = t.get("exitCode")
        if code not in (None, 0) or reason == "OOMKilled":
            failed_exit = True
        if reason == "OOMKilled":
            v.host_score += 1.0
            v.signature = True
            v.oomkilled = True
            v.signals.append(f"container {t.get('container', '')!s} OOMKilled (cgroup, exit {code})")
        elif code == 137:
            v.host_score += 0.35
            v.signature = True
            v.signals.append(f"container {t.get('container', '')!s} exit 137 (SIGKILL)")
        if t.get("message"):
            sourced.append((f"termination message of container {t.get('container', '')}", t["message"]))
    hbm_hit = host_hit = False
    logical = None
    for source, text in sourced:
        s, h = signatures(text)
        if h and not host_hit and h != "OOMKilled":
            host_hit = True
            v.signature = True
            v.host_text = True
            v.host_score += 0.6
            v.signals.append(f"host allocation failure in {source}: {h!r}")
        if s and not hbm_hit:
            hbm_hit = True
            if gpu_involved is False:
                v.signals.append(f"HIP OOM text in {source} ({s!r}) on a pod with no GPU (no GPU request, no GPU "
                                 f"process of its own): not an HBM verdict")
            else:
                v.signature = True
                v.hbm_text = True
                v.hbm_score += 1.0
                v.signals.append(f"HIP OOM signature in {source}: {s!r}")
        if not _mentions(text, _TORCH_KEYS):
            continue
        m = _TORCH_GPU.search(text)
        if m and logical is None:
            logical = int(m.group(1))
            v.capacity_bytes = int(float(m.group(2)) * _UNIT[m.group(3).lower()])
        r = _TORCH_REQ.search(text)
        if r and v.requested_bytes is None:
            v.requested_bytes = int(float(r.group(1)) * _UNIT[r.group(2).lower()])
    if logical is not None and gpu_involved is not False:
        v.gpu_logical_index = logical
        if topo is not None:
            ev = gpu_evidence or {}
            v.gpu_index = physical_gpu(topo, logical, ev.get("gpus") or (), ev.get("allocated"))
        else:
            v.gpu_index = logical  # no topology: the process saw the node's numbering
    if gpu_evidence and gpu_involved is not False:
        cap = int(hbm_capacity_gb * (1 << 30))
        own_sig = False
        for g in _candidate_gpus(gpu_evidence, expected_gpu, v.gpu_index):
            total = int(g.get("vram_total_mb") or 0) * (1 << 20) or cap
            peak = int(g.get("vram_peak_mb") or g.get("vram_used_mb") or 0) * (1 << 20)
            own = int(g.get("proc_peak_vram_bytes") or 0)
            if own and own >= hbm_oom_fraction * total and failed_exit and not own_sig:
                # the pod's OWN processes (matched by cgroup pod UID / PID) filled the GPU and
                # the container then failed: strong corroboration (and the attribution), but
                # not a signature — the caching allocator holds a full GPU in healthy runs too
                own_sig = True
                v.hbm_score += 0.75
                v.signals.append(f"own-process VRAM peak: the pod's processes on GPU {g.get('index')} peaked at "
                                 f"{own / (1 << 30):.1f} GiB of {total / (1 << 30):.1f} GiB, then the container "
                                 f"exited non-zero")
                v.peak_vram_bytes = own
                if v.gpu_index is None:
                    v.gpu_index = g.get("index")
            if peak and peak >= hbm_oom_fraction * total:
                v.hbm_score += 0.5
                share = f"; the pod's own processes peaked at {own / (1 << 30):.1f} GiB" if own else ""
                v.signals.append(f"GPU {g.get('index')} VRAM peak {peak / (1 << 30):.1f} GiB of "
                                 f"{total / (1 << 30):.1f} GiB{share} (device-wide: corroboration only)")
                v.device_peak_vram_bytes = peak
                v.peak_vram_bytes = own or peak
                if v.gpu_index is None:
                    v.gpu_index = g.get("index")
            if (v.foreign is None and peak and peak >= FOREIGN_FULL_FRACTION * total and own < OWN_SHARE_MAX * total):
                # full, but not of the pod's doing: name who held it (the stage stays what the
                # evidence says — an HBM-OOM is still one, a crash still a crash)
                holders = g.get("holders") or []
                v.foreign = {"gpu": g.get("index"), "device_peak_bytes": peak, "own_peak_bytes": own,
                             "total_bytes": total, "holders": holders}
                if g.get("foreign_vram_bytes"):
                    v.foreign["other_namespace_bytes"] = g["foreign_vram_bytes"]
                top = holders[0] if holders else None
                who = (f"; largest holder pid {top.get('pid')} ({top.get('owner')}) "
                       f"{(top.get('vram_bytes') or 0) / (1 << 30):.1f} GiB" if top else "")
                v.signals.append(f"foreign occupancy: GPU {g.get('index')} was {peak / total:.0%} full while the pod's "
                                 f"own processes held {own / (1 << 30):.1f} GiB{who}")
            faults = [e for e in g.get("events", []) if e.get("type") in ("VMFAULT", "QUEUE_EVICTION", "GPU_PRE_RESET")]
            if faults:
                v.hbm_score += 0.25
                v.signals.append(f"GPU {g.get('index')} events: {sorted({e['type'] for e in faults})}")
                if v.gpu_index is None:
                    v.gpu_index = g.get("index")
            if v.capacity_bytes is None and g.get("vram_total_mb"):
                v.capacity_bytes = int(g["vram_total_mb"]) * (1 << 20)
    if v.signature and (v.hbm_score >= 0.5 or v.host_score >= 0.5):
        if v.oomkilled and not v.hbm_text:
            v.kind = "host"  # a cgroup OOMKill is a kernel fact about host memory: only HIP's own words beat it
        elif v.host_score >= 1.0 and v.host_score >= v.hbm_score:
            v.kind = "host"
        elif v.hbm_score >= v.host_score:
            v.kind = "hbm"
        else:
            v.kind = "host"
    elif v.hbm_score >= 0.5:
        v.signals.append("no OOM signature (allocation-failure message or log line, OOMKilled or exit 137): "
                         "VRAM numbers alone are not an OOM verdict")
    return v


def _candidate_gpus(ev: Dict[str, Any], expected: Optional[str], idx: Optional[int]):
    gpus = ev.get("gpus") or []
    if idx is not None:
        # the failing process named its GPU: never read another GPU's evidence for it
        return [g for g in gpus if g.get("index") == idx]
    if expected is not None:
        sel = [g for g in gpus if str(g.get("index")) == str(expected) or g.get("uuid") == expected]
        if sel:
            return sel
    return gpus
