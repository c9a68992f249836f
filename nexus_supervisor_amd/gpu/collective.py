"""Root cause of a multi-rank job's failure: which rank failed first, and which ranks only
died of its collateral (RCCL / collective errors).

A distributed MI355X job is one Job with a pod per rank (indexed Job) or per node: when
rank 3 runs out of HBM, every other rank blocks in its next all-reduce and fails a few
seconds (or a watchdog timeout) later with an RCCL error — ``Watchdog caught collective
operation timeout``, ``NCCL communicator was aborted``, ``DistBackendError``,
``ncclRemoteError``.  The Job's terminal condition (``BackoffLimitExceeded`` /
``PodFailurePolicy``) names none of this; the reference writes the Job event's message
and nothing else (``/root/reference/services/supervisor.go:183-204``).  The supervisor
instead ranks the failed pods:

=====  ============================================  ==============================
score  pod failure                                   meaning
=====  ============================================  ==============================
3      HIP / host OOM text, OOMKilled                a resource ran out on this rank
2      GPU fault evidence, or a non-zero exit whose  this rank failed on its own
       messages carry no collective error
1      only collective / RCCL errors                 collateral of another rank
=====  ============================================  ==============================

The highest score is the *culprit* (ties: the earliest ``finishedAt``, then the name); its
topology and GPU evidence attribute the decision (a torch ``GPU 0`` in rank 3's message is
rank 3's device, not the last pod's), and the trace lists the ranks with their failure
kinds (``ranks``).  When every failed rank shows only collective errors, the run failed in
the fabric or the collective layer itself (failure class ``collective``).
"""
from __future__ import annotations

import re
from typing import Any, Dict, Iterable, List, Optional, Tuple

COLLECTIVE_PATTERNS = [
    re.compile(r"Watchdog caught collective operation timeout[^\n]{0,160}"),
    re.compile(r"(?:NCCL|RCCL) communicator was aborted[^\n]{0,120}"),
    re.compile(r"\bDistBackendError\b[^\n]{0,160}"),
    re.compile(r"\bnccl(?:RemoteError|SystemError|InternalError|UnhandledCudaError|InvalidUsage)\b[^\n]{0,120}"),
    re.compile(r"ProcessGroupNCCL[^\n]{0,160}(?:timed? ?out|abort)[^\n]{0,80}", re.I),
    re.compile(r"(?:NCCL|RCCL) (?:error|WARN)\b[^\n]{0,160}"),
    re.compile(r"\bcollective operation timeout\b[^\n]{0,120}", re.I),
]
_KEYS = ("NCCL", "RCCL", "ollective", "DistBackend", "nccl")

TRACE_MAX_RANKS = 8  # pods listed in a trace (the culprit first); the rest are counted


def collective_signature(text: Optional[str]) -> Optional[str]:
    """The first collective / RCCL error in ``text`` (clipped), or None."""
    if not text or not any(k in text for k in _KEYS):
        return None
    for p in COLLECTIVE_PATTERNS:
        m = p.search(text)
        if m:
            return m.group(0)[:200]
    return None


def pod_failure(pod_name: str, terms: Iterable[Dict[str, Any]], texts: Iterable[Tuple[str, str]],
                oom_kind: Optional[str], gpu_fault: bool, rank: Optional[int]) -> Optional[Dict[str, Any]]:
    """One failed pod's record (None when none of its containers failed).  ``terms``: its
    terminated states; ``texts``: (source, text) of its termination messages and log
    tails; ``oom_kind``: "hbm" / "host" when its own evidence makes it an OOM."""
    failed = [t for t in terms if t.get("exitCode", 0) != 0 or t.get("reason") == "OOMKilled"]
    if not failed:
        return None
    coll = None
    for _src, txt in texts:
        coll = collective_signature(txt)
        if coll:
            break
    if oom_kind:
        kind, score = f"{oom_kind}-oom", 3
    elif gpu_fault:
        kind, score = "gpu-fault", 2
    elif coll:
        kind, score = "collective", 1
    else:
        kind, score = "error", 2
    t0 = min(failed, key=lambda t: str(t.get("finishedAt") or "~"))
    rec: Dict[str, Any] = {"pod": pod_name, "kind": kind, "exit_code": t0.get("exitCode"),
                           "reason": t0.get("reason") or "", "finished": t0.get("finishedAt") or ""}
    if rank is not None:
        rec["rank"] = rank
    if coll and kind != "collective":
        rec["collective"] = coll  # it also reported a collective error, after its own
    elif coll:
        rec["signature"] = coll
    rec["_score"] = score
    return rec


def rank_summary(records: List[Dict[str, Any]]) -> Tuple[Optional[Dict[str, Any]], Dict[str, Any]]:
    """(culprit record, trace block) over the failed pods' records."""
    if not records:
        return None, {}
    ordered = sorted(records, key=lambda r: (-r["_score"], r.get("finished") or "~", r["pod"]))
    culprit = ordered[0]
    clean = [{k: v for k, v in r.items() if k != "_score"} for r in ordered]
    block: Dict[str, Any] = {"culprit": clean[0], "failed": len(records),
                             "collateral": sum(1 for r in records if r["kind"] == "collective"),
                             "all_collective": all(r["kind"] == "collective" for r in records)}
    if len(clean) > 1:
        block["pods"] = clean[1:TRACE_MAX_RANKS]
        if len(clean) > TRACE_MAX_RANKS:
            block["pods_total"] = len(clean)
    return culprit, block
