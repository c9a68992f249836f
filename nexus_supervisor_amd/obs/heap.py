"""Heap census of a replica process (``/debug/heap``; Go's ``/debug/pprof/heap`` plays
this part for the reference).

What a long-lived supervisor holds is dominated by a few structures — the informer caches,
the decision / evidence / topology memos, the CQL routing caches — so the census reports
their sizes next to a live-object count by type (dicts by their key set: a Pod, a Job, a
topology block), the process RSS, and, when ``PYTHONTRACEMALLOC`` tracing is on, the top
allocation sites.  ``tools/replica_memory.py`` uses it to find what grows with churn.
"""
from __future__ import annotations

import collections
import gc
import os
from typing import Any, Dict, Optional


def _rss_mb() -> Optional[float]:
    try:
        with open(f"/proc/{os.getpid()}/status") as f:
            for ln in f:
                if ln.startswith("VmRSS:"):
                    return int(ln.split()[1]) / 1024.0
    except OSError:
        pass
    return None


def _sizes(sup) -> Dict[str, Any]:
    out: Dict[str, Any] = {}
    if sup is None:
        return out
    for name, inf in getattr(getattr(sup, "factory", None), "informers", {}).items():
        out[f"informer.{name}"] = len(inf.indexer)
    for attr in ("_applied", "_parked", "_gpu_wait", "_gpu_waiters", "_log_fetches", "_deletes", "_bg", "_event_tasks"):
        v = getattr(sup, attr, None)
        if v is not None:
            out[f"supervisor.{attr}"] = len(v)
    clf = getattr(sup, "classifier", None)
    if clf is not None:
        out["classifier.evidence"] = len(clf.evidence)
        out["classifier._ctx_cache"] = len(clf._ctx_cache)
        out["classifier.log_cache"] = len(clf.log_cache)
    pipe = getattr(sup, "pipeline", None)
    if pipe is not None:
        out["pipeline.pending_keys"] = len(pipe._pending)
        out["pipeline.backoff_keys"] = len(getattr(pipe.backoff, "_failures", {}) or {})
    sess = getattr(getattr(sup, "store", None), "session", None)
    if sess is not None:
        out["cql._tokens"] = len(getattr(sess, "_tokens", {}) or {})
        out["cql._routes"] = len(getattr(sess, "_routes", {}) or {})
    return out


def _desc(o) -> str:
    t = type(o)
    if t is dict:
        return "dict{" + ",".join(sorted(map(str, o.keys()))[:6]) + "}"
    if t in (list, tuple, set):
        return f"{t.__name__}[{len(o)}]"
    if t.__name__ == "frame":
        return f"frame {o.f_code.co_filename.rsplit('/', 2)[-1]}:{o.f_lineno} {o.f_code.co_name}"
    if t.__name__ == "cell":
        return "cell"
    return t.__qualname__


def retainers(sup, kind: str, samples: int = 3, depth: int = 4) -> list:
    """For up to ``samples`` live objects of ``kind`` (``Pod`` / ``Job`` / ``Event``) that
    are *not* in the informer caches: the chain of what references them (first referrer
    at each level), to find what keeps a deleted object alive."""
    cached = set()
    for inf in getattr(getattr(sup, "factory", None), "informers", {}).values():
        cached.update(id(o) for o in inf.indexer._items.values())
    stray = [o for o in gc.get_objects() if type(o) is dict and o.get("kind") == kind and id(o) not in cached
             and isinstance(o.get("metadata"), dict)]
    out = []
    skip = {id(stray)}
    for o in stray[:samples]:
        chain = []
        cur = o
        seen = {id(o)}
        for _ in range(depth):
            refs = [r for r in gc.get_referrers(cur) if id(r) not in skip and id(r) not in seen
                    and type(r).__name__ != "frame" or (type(r).__name__ == "frame" and r.f_code.co_name != "retainers")]
            refs = [r for r in refs if id(r) not in skip and r is not stray]
            if not refs:
                break
            chain.append([_desc(r) for r in refs[:4]])
            cur = refs[0]
            seen.add(id(cur))
        out.append({"name": o["metadata"].get("name"), "rv": o["metadata"].get("resourceVersion"), "chain": chain})
    return [{"stray": len(stray)}] + out


def malloc_trim() -> bool:
    """Hand the C heap's free pages back to the kernel (glibc ``malloc_trim``)."""
    try:
        import ctypes

        return bool(ctypes.CDLL("libc.so.6").malloc_trim(0))
    except (OSError, AttributeError):
        return False


def census(sup=None, top: int = 25, trim: bool = False) -> Dict[str, Any]:
    gc.collect()
    if trim:
        before = _rss_mb()
        malloc_trim()
        trimmed = {"rss_before_trim_mb": before, "rss_after_trim_mb": _rss_mb()}
    else:
        trimmed = {}
    types: "collections.Counter[str]" = collections.Counter()
    shapes: "collections.Counter[str]" = collections.Counter()
    for o in gc.get_objects():
        t = type(o)
        if t is dict:
            keys = sorted(map(str, o.keys()))
            shapes[",".join(keys[:6]) + (",…" if len(keys) > 6 else "")] += 1
        types[t.__name__] += 1
    doc: Dict[str, Any] = {"rss_mb": _rss_mb(), "gc_objects": sum(types.values()),
                           "gc_frozen": gc.get_freeze_count(),
                           "types": dict(types.most_common(top)), "dict_shapes": dict(shapes.most_common(top)),
                           "structures": _sizes(sup), **trimmed}
    import tracemalloc

    if tracemalloc.is_tracing():
        global _LAST
        snap = tracemalloc.take_snapshot()
        doc["tracemalloc_mb"] = round(sum(st.size for st in snap.statistics("filename")) / 2**20, 2)
        doc["tracemalloc_top"] = [str(st) for st in snap.statistics("lineno")[:top]]
        if _LAST is not None:
            # growth since the previous /debug/heap call, by allocating call stack
            doc["tracemalloc_growth"] = [
                {"size_kb": round(st.size_diff / 1024, 1), "count": st.count_diff,
                 "stack": [f"{f.filename.rsplit('/', 2)[-1]}:{f.lineno}" for f in st.traceback][-6:]}
                for st in snap.compare_to(_LAST, "traceback")[:top]]
        _LAST = snap
    return doc


_LAST = None
