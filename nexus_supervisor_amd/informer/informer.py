"""List+watch informers (client-go ``SharedIndexInformer`` equivalent, asyncio).

The reference builds one namespaced ``SharedInformerFactory`` with Event, Pod
and Job informers (``/root/reference/services/supervisor.go:70-75``) and only
attaches an ``AddFunc`` to events (``:124-128``).  Here every informer:

* lists, then watches from the list's ``resourceVersion`` with bookmarks;
* on ``410 Gone`` / expired RV re-lists and emits synthetic Add/Update/Delete
  for the diff (so nothing is lost across a watch gap);
* slims objects before caching (``models.kube.SLIMMERS``);
* dispatches Add/Update/Delete synchronously on the event-loop thread (the
  classifier is pure, so dispatch never blocks on I/O);
* optionally resyncs (Update(obj, obj) for every cached object).

``ListWatch`` is the transport seam: :class:`..kube.client.KubeListWatch` speaks
the real REST/watch protocol, tests can use :class:`QueueListWatch`.
"""
from __future__ import annotations

import asyncio
import logging
import os
import random
import time
from typing import Any, AsyncIterator, Callable, Dict, List, Optional, Tuple

from ..models import kube
from .store import IndexFunc, Indexer

log = logging.getLogger("nexus_supervisor_amd.informer")

ADDED, MODIFIED, DELETED, BOOKMARK, ERROR = "ADDED", "MODIFIED", "DELETED", "BOOKMARK", "ERROR"


class WatchGone(Exception):
    """The watch's resourceVersion is too old (HTTP 410) — re-list required."""


class ListWatch:
    kind: str = ""

    async def list(self) -> Tuple[List[Dict[str, Any]], str]:  # pragma: no cover - interface
        raise NotImplementedError

    def watch(self, resource_version: str) -> AsyncIterator[Tuple[str, Dict[str, Any]]]:  # pragma: no cover
        raise NotImplementedError


class Handler:
    __slots__ = ("on_add", "on_update", "on_delete")

    def __init__(self, on_add=None, on_update=None, on_delete=None):
        self.on_add = on_add
        self.on_update = on_update
        self.on_delete = on_delete


class SharedInformer:
    def __init__(self, kind: str, lw: ListWatch, *, resync_period: float = 0.0,
                 indexers: Optional[Dict[str, IndexFunc]] = None, transform: Optional[Callable] = None,
                 stamp: Optional[Callable[[], float]] = None):
        self.kind = kind
        self.lw = lw
        self.resync_period = resync_period
        self.indexer = Indexer(indexers)
        if transform is None:
            # a ListWatch that already projects objects (native decode) supplies its own finisher
            transform = getattr(lw, "transform", kube.SLIMMERS.get(kind)) if hasattr(lw, "transform") else kube.SLIMMERS.get(kind)
        self.transform = transform
        self.handlers: List[Handler] = []
        self._synced = asyncio.Event() if _has_loop() else None
        self._rv = ""
        self._task: Optional[asyncio.Task] = None
        self._resync_task: Optional[asyncio.Task] = None
        self.stamp = stamp or time.monotonic
        self.relists = 0
        self.watch_events = 0
        self.last_receive = 0.0
        # ingest filter (shard workers): ``accept(obj, etype)`` false → the object is neither
        # cached nor dispatched; ``on_reject(obj)`` is told about it instead
        self.accept: Optional[Callable[[Dict[str, Any], str], bool]] = None
        self.on_reject: Optional[Callable[[Dict[str, Any]], None]] = None
        self.rejected = 0

    # ------------------------------------------------------------------ API
    def add_event_handler(self, on_add=None, on_update=None, on_delete=None) -> Handler:
        h = Handler(on_add, on_update, on_delete)
        self.handlers.append(h)
        if self.has_synced():  # late registration: replay current state as adds
            for obj in self.indexer.values():
                if on_add:
                    on_add(obj)
        return h

    def has_synced(self) -> bool:
        return self._synced is not None and self._synced.is_set()

    async def wait_synced(self, timeout: Optional[float] = None) -> bool:
        self._ensure_event()
        try:
            await asyncio.wait_for(self._synced.wait(), timeout)
            return True
        except asyncio.TimeoutError:
            return False

    def get(self, name: str, namespace: str = "") -> Optional[Dict[str, Any]]:
        return self.indexer.get_by_name(namespace, name)

    def start(self) -> asyncio.Task:
        self._ensure_event()
        if self._task is None:
            self._task = asyncio.create_task(self._run(), name=f"informer-{self.kind}")
            if self.resync_period > 0:
                self._resync_task = asyncio.create_task(self._resync_loop(), name=f"resync-{self.kind}")
        return self._task

    def relist(self) -> None:
        """Restart list+watch now (a changed ingest filter: objects it used to drop must be
        listed again; the re-list diff dispatches them as adds)."""
        if self._task is None:
            return
        self._task.cancel()
        self._task = asyncio.create_task(self._run(), name=f"informer-{self.kind}")

    async def stop(self) -> None:
        for t in (self._task, self._resync_task):
            if t is not None:
                t.cancel()
        for t in (self._task, self._resync_task):
            if t is not None:
                try:
                    await t
                except (asyncio.CancelledError, Exception):
                    pass
        self._task = self._resync_task = None

    # ------------------------------------------------------------------ direct feed (tests / in-proc)
    def inject(self, etype: str, obj: Dict[str, Any]) -> None:
        """Apply one watch event as if it came from the server."""
        self._apply(etype, obj)

    def mark_synced(self) -> None:
        self._ensure_event()
        self._synced.set()

    # ------------------------------------------------------------------ internals
    def _ensure_event(self):
        if self._synced is None:
            self._synced = asyncio.Event()

    def _dispatch_add(self, obj):
        for h in self.handlers:
            if h.on_add:
                try:
                    h.on_add(obj)
                except Exception:  # handler bugs must not kill the informer
                    log.exception("%s add handler failed", self.kind)

    def _dispatch_update(self, old, new):
        for h in self.handlers:
            if h.on_update:
                try:
                    h.on_update(old, new)
                except Exception:
                    log.exception("%s update handler failed", self.kind)

    def _dispatch_delete(self, obj):
        for h in self.handlers:
            if h.on_delete:
                try:
                    h.on_delete(obj)
                except Exception:
                    log.exception("%s delete handler failed", self.kind)

    def _apply(self, etype: str, raw: Dict[str, Any]) -> None:
        self.watch_events += 1
        self.last_receive = self.stamp()
        if etype == BOOKMARK:
            rv = kube.resource_version(raw)
            if rv:
                self._rv = rv
            return
        obj = self.transform(raw) if self.transform else raw
        rv = kube.resource_version(obj)
        if rv:
            self._rv = rv
        if self.accept is not None and not self.accept(obj, etype):
            self._reject(obj)
            return
        if etype == DELETED:
            old = self.indexer.delete(obj)
            self._dispatch_delete(old or obj)
            return
        old = self.indexer.upsert(obj)
        if old is None:
            self._dispatch_add(obj)
        else:
            self._dispatch_update(old, obj)

    def _reject(self, obj) -> None:
        self.rejected += 1
        if self.on_reject is not None:
            try:
                self.on_reject(obj)
            except Exception:
                log.exception("%s reject handler failed", self.kind)

    def _relist_apply(self, items: List[Dict[str, Any]]) -> None:
        objs = [self.transform(o) if self.transform else o for o in items]
        if self.accept is not None:
            kept = []
            for o in objs:
                if self.accept(o, ADDED):
                    kept.append(o)
                else:
                    self._reject(o)
            objs = kept
        old = self.indexer.replace(objs)
        for o in objs:
            k = kube.object_key(o)
            prev = old.pop(k, None)
            if prev is None:
                self._dispatch_add(o)
            elif kube.resource_version(prev) != kube.resource_version(o):
                self._dispatch_update(prev, o)
        for prev in old.values():
            self._dispatch_delete(prev)

    async def _run(self):
        backoff = 0.2
        while True:
            try:
                items, rv = await self.lw.list()
                self.relists += 1
                self._relist_apply(items)
                # this frame lives as long as the watch: holding the LIST's list would keep every
                # listed object alive after the watch replaced it (a second copy of the cache)
                del items
                self._rv = rv
                self._synced.set()
                backoff = 0.2
                while True:
                    try:
                        await self._watch_once()
                    except WatchGone:
                        log.info("%s watch expired (410) at rv=%s, re-listing", self.kind, self._rv)
                        break
                    # clean end of a watch (server timeout): resume from last RV
                    await asyncio.sleep(0)
            except asyncio.CancelledError:
                raise
            except Exception as exc:  # connection errors: back off and re-list
                # a throttled list / watch (429) waits at least the server's Retry-After
                wait = max(backoff * (1 + random.random() * 0.2), getattr(exc, "retry_after", None) or 0.0)
                log.warning("%s list/watch failed: %s; retrying in %.1fs", self.kind, exc, wait)
                await asyncio.sleep(wait)
                backoff = min(backoff * 2, 30.0)

    def _watch_error(self, obj) -> None:
        if (obj or {}).get("code") == 410:
            raise WatchGone()
        log.warning("%s watch error object: %s", self.kind, obj)

    async def _watch_once(self) -> None:
        """One watch stream from the last resourceVersion: returns on a clean end or an error
        object, raises :class:`WatchGone` on 410.  A transport with ``watch_batches`` (the
        watch hub's per-worker feed) hands over one list per received frame, applied in one
        loop instead of one async-generator step per line; either way the loop yields to the
        pipeline every 64 lines."""
        batches = getattr(self.lw, "watch_batches", None)
        if batches is None:
            async for etype, obj in self.lw.watch(self._rv):
                if etype == ERROR:
                    return self._watch_error(obj)
                self._apply(etype, obj)
            return
        apply = self._apply
        async for batch in batches(self._rv):
            if self.accept is not None or self.transform is not None:
                n = 0
                for etype, obj in batch:
                    if etype == ERROR:
                        return self._watch_error(obj)
                    apply(etype, obj)
                    n += 1
                    if not n & 63:
                        await asyncio.sleep(0)
                continue
            for i in range(0, len(batch), 64):
                err = self._apply_lines(batch, i, i + 64)
                if err is not None:
                    return self._watch_error(err)
                if i + 64 < len(batch):
                    await asyncio.sleep(0)

    def _apply_lines(self, batch, start: int, end: int):
        """:meth:`_apply` for ``batch[start:end]`` of a projecting transport (no transform,
        no ingest filter), with the per-line lookups hoisted out of the loop; returns the
        ERROR event's object if one is met (the lines before it are applied)."""
        self.last_receive = self.stamp()
        indexer = self.indexer
        adds = [h.on_add for h in self.handlers if h.on_add]
        updates = [h.on_update for h in self.handlers if h.on_update]
        deletes = [h.on_delete for h in self.handlers if h.on_delete]
        kind = self.kind
        native = _native_apply()
        if native is not None and (indexer._labels is not None or not indexer._indexers):
            # the same loop in C (csrc/kube/informer_apply.cpp): store, label index, handlers
            err, seen, rv = native(batch, start, end, indexer._items, indexer._labels, indexer._indices,
                                   adds, updates, deletes, _handler_failed, kind)
            self.watch_events += seen
            if rv:
                self._rv = rv
            return err
        upsert, delete = indexer.upsert, indexer.delete
        rv = None
        seen = 0
        try:
            for etype, obj in batch[start:end]:
                if etype == ERROR:
                    return obj
                seen += 1
                m = obj.get("metadata")
                if m:
                    v = m.get("resourceVersion")
                    if v:
                        rv = v
                if etype == BOOKMARK:
                    continue
                if etype == DELETED:
                    old = delete(obj) or obj
                    for f in deletes:
                        try:
                            f(old)
                        except Exception:
                            log.exception("%s delete handler failed", kind)
                    continue
                old = upsert(obj)
                if old is None:
                    for f in adds:
                        try:
                            f(obj)
                        except Exception:  # handler bugs must not kill the informer
                            log.exception("%s add handler failed", kind)
                else:
                    for f in updates:
                        try:
                            f(old, obj)
                        except Exception:
                            log.exception("%s update handler failed", kind)
        finally:
            self.watch_events += seen
            if rv:
                self._rv = rv
        return None

    async def _resync_loop(self):
        while True:
            await asyncio.sleep(self.resync_period)
            if not self.has_synced():
                continue
            for obj in self.indexer.values():
                self._dispatch_update(obj, obj)


_NATIVE_APPLY: List[Any] = []


def _native_apply():
    """``_kube_native.apply_lines`` (None without the native build, or with
    ``NEXUS_PY_INFORMER_APPLY=1``: the Python loop below, for A/B runs)."""
    if not _NATIVE_APPLY:
        fn = None
        if os.environ.get("NEXUS_PY_INFORMER_APPLY") != "1":
            try:
                from .. import _kube_native

                fn = getattr(_kube_native, "apply_lines", None)
            except ImportError:
                fn = None
        _NATIVE_APPLY.append(fn)
    return _NATIVE_APPLY[0]


def _handler_failed(kind: str, exc: BaseException) -> None:
    log.error("%s handler failed", kind, exc_info=(type(exc), exc, exc.__traceback__))


def _has_loop() -> bool:
    try:
        asyncio.get_running_loop()
        return True
    except RuntimeError:
        return False


class QueueListWatch(ListWatch):
    """In-memory ListWatch: a seeded object list plus an asyncio queue of watch events."""

    def __init__(self, kind: str, items: Optional[List[Dict[str, Any]]] = None):
        self.kind = kind
        self.items = list(items or [])
        self.queue: "asyncio.Queue[Tuple[str, Dict[str, Any]]]" = asyncio.Queue()
        self.rv = 1

    async def list(self):
        return list(self.items), str(self.rv)

    async def watch(self, resource_version: str):
        while True:
            etype, obj = await self.queue.get()
            yield etype, obj

    def push(self, etype: str, obj: Dict[str, Any]) -> None:
        self.queue.put_nowait((etype, obj))


class InformerFactory:
    """One namespaced factory (``kubeinformers.NewSharedInformerFactoryWithOptions``,
    ``/root/reference/services/supervisor.go:71``)."""

    def __init__(self, list_watch_for: Callable[[str], ListWatch], resync_period: float = 30.0):
        self._lw_for = list_watch_for
        self.resync_period = resync_period
        self.informers: Dict[str, SharedInformer] = {}

    def informer(self, kind: str, indexers: Optional[Dict[str, IndexFunc]] = None, resync: Optional[float] = None) -> SharedInformer:
        inf = self.informers.get(kind)
        if inf is None:
            inf = SharedInformer(kind, self._lw_for(kind), resync_period=self.resync_period if resync is None else resync,
                                 indexers=indexers)
            self.informers[kind] = inf
        elif indexers:
            for n, fn in indexers.items():
                inf.indexer.add_indexer(n, fn)
        return inf

    def start(self) -> None:
        for inf in self.informers.values():
            inf.start()

    async def wait_for_cache_sync(self, timeout: Optional[float] = None) -> bool:
        res = await asyncio.gather(*(i.wait_synced(timeout) for i in self.informers.values()))
        return all(res)

    async def stop(self) -> None:
        await asyncio.gather(*(i.stop() for i in self.informers.values()))
