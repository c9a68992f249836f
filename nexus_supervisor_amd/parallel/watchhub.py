"""One watch per replica, demultiplexed to the shard workers.

With ``runtime.worker-processes`` = K and no hub, every worker would hold its own
Event/Pod/Job LIST+WATCH: the API server serialises and sends every change K times per
replica, and every worker scans every line.  The reference's single Go process holds
one watch per kind (``/root/reference/services/supervisor.go:73-75``); so does this
replica.  The parent process runs the hub:

* per kind, LIST then WATCH from the list's resourceVersion against the API server
  (same label selectors and timeouts as the informers would use);
* the native :class:`_kube_native.WatchSplitter` routes each LIST item and each watch
  line to the worker that owns it (``crc32(job name)``, the same placement as
  :mod:`.workers`), consuming bookmarks and handing errors back; a chunk costs one C
  call however many lines it holds;
* routed bytes go to the worker over a per-worker data socket as length-prefixed
  frames: ``SNAPSHOT`` (resourceVersion + the worker's items as a JSON array) and
  ``LINES`` (NDJSON watch lines); the hub pauses reading the API server while any
  worker's socket buffer is above a high-water mark (back-pressure end to end);
* Events whose reason no rule reads (``Scheduled``, ``Pulling``, ``Pulled``, ``Created``,
  ``Killing``, ``SuccessfulCreate``, … — most of a namespace's Events) are dropped by the
  splitter before any worker decodes them (:data:`..classify.classifier.EVENT_REASONS_READ`;
  ``watch_events_unread`` counts them);
* on ``410 Gone`` / stream errors the hub re-lists and sends every worker a fresh
  snapshot; a worker's :class:`HubListWatch` turns that into the informer's 410 →
  re-list path, so the informer's diff logic is unchanged.  A restarted worker gets a
  fresh snapshot the same way (:meth:`WatchHub.resync`).

Frame: ``!BBI`` (type, kind index, payload length) + payload.  ``LINES_T`` is ``LINES``
with an ``!d`` prefix: the CLOCK_MONOTONIC time the hub read the chunk from the API server
(:mod:`..obs.delivery` — the delivery-latency stages).
"""
from __future__ import annotations

import asyncio
import logging
import os
import struct
import sys
import time
from time import thread_time as _thread_time
from typing import Any, Callable, Dict, List, Optional, Tuple

from ..informer.informer import ListWatch
from ..obs import delivery as _delivery
from ..models.kube import PROJECTIONS, watch_projection

log = logging.getLogger("nexus_supervisor_amd.watchhub")

KINDS: Tuple[str, ...] = ("Event", "Pod", "Job")
ROLES = {"Event": "event", "Pod": "pod", "Job": "job"}
SNAPSHOT, LINES, LINES_T = 1, 2, 3
HEADER = struct.Struct("!BBI")
STAMP = struct.Struct("!d")
HIGH_WATER = 32 << 20


_CHUNK_LOG = os.environ.get("NEXUS_SLOW_CALLBACK_LOG", "") not in ("", "0")


class _Gone(Exception):
    pass


def _is_gone(line: bytes) -> bool:
    import json

    try:
        return (json.loads(line).get("object") or {}).get("code") == 410
    except ValueError:
        return False


class WatchHub:
    """Parent side: ``send(worker, frame_type, kind_index, payload)`` delivers a frame and
    ``buffered(worker)`` reports the bytes still queued for it."""

    def __init__(self, cfg, kube, count: int, send: Callable[[int, int, int, bytes], None],
                 buffered: Callable[[int], int], drain: Callable[[int], Any], metrics=None):
        from .. import _kube_native
        from .workers import _SEED, POD_FORGET_AFTER

        self.cfg = cfg
        self.kube = kube
        self.count = count
        self.send = send
        self.buffered = buffered
        self.drain = drain
        self.metrics = metrics
        self.router = _kube_native.ShardRouter(0, count, _SEED, cfg.labels.job_name_label, POD_FORGET_AFTER)
        from ..classify.classifier import event_reasons_read

        # an Event no rule reads decides nothing: no worker decodes, caches or dispatches it
        self.router.set_event_reasons(sorted(event_reasons_read(cfg.gpu.gpu_resource_name)))
        self._unread_seen = 0
        from .sharding import ShardSet

        self.tasks: Dict[str, asyncio.Task] = {}
        self.relists = 0
        self.bytes_routed = 0
        self.owned = None  # the replica's shards (sharding.shard-label narrows the Pod/Job watches)
        self.set_shards(ShardSet.from_config(cfg))  # static mode: the owned set is final here

    def set_shards(self, shards) -> None:
        """Replica shard set: lines of runs this replica does not own are dropped in the
        splitter (before any decode, in any worker).  A change takes effect for lines
        routed from now on; :meth:`resync` re-lists so gained runs reach the workers."""
        from .sharding import SHARD_SEED

        if shards.enabled:
            self.router.set_replica(shards.shards, SHARD_SEED, sorted(shards.owned))
        else:
            self.router.set_replica(1, SHARD_SEED, [0])
        self.owned = shards.owned

    def start(self) -> None:
        for i, kind in enumerate(KINDS):
            if kind not in self.tasks:
                self.tasks[kind] = asyncio.create_task(self._pump(i, kind), name=f"watchhub-{kind}")

    async def stop(self) -> None:
        tasks = list(self.tasks.values())
        self.tasks.clear()
        for t in tasks:
            t.cancel()
        for t in tasks:
            try:
                await t
            except (asyncio.CancelledError, Exception):
                pass

    async def resync(self) -> None:
        """Re-list every kind and send every worker a fresh snapshot (a restarted worker
        has an empty cache; the others apply the relist diff, which is idempotent)."""
        await self.stop()
        self.start()

    def _path_params(self, kind: str) -> Tuple[str, Dict[str, str]]:
        from ..kube.client import resource_path

        from .sharding import watch_field_selector, watch_selector

        params: Dict[str, str] = {}
        sel = watch_selector(self.cfg, kind, self.owned)
        if sel:
            params["labelSelector"] = sel
        fsel = watch_field_selector(self.cfg, kind)
        if fsel:
            params["fieldSelector"] = fsel
        return resource_path(kind, self.cfg.resource_namespace), params

    async def _route(self, ki: int, outs: List[bytes], ftype: int, prefix: bytes = b"") -> None:
        for w, b in enumerate(outs):
            if b or ftype == SNAPSHOT:
                payload = prefix + b if prefix else b
                self.send(w, ftype, ki, payload)
                self.bytes_routed += len(payload)
        for w in range(self.count):
            if self.buffered(w) > HIGH_WATER:
                await self.drain(w)

    async def _pump(self, ki: int, kind: str) -> None:
        from .. import _kube_native

        splitter = _kube_native.WatchSplitter(self.router, ROLES[kind])
        path, base = self._path_params(kind)
        backoff = 0.2
        rv = ""
        while True:
            try:
                status, body = await self.kube.get_raw(path, base)
                if status >= 400:
                    raise RuntimeError(f"LIST {kind}: HTTP {status}")
                rv, parts = splitter.split_list(body)
                self.relists += 1
                if self.metrics is not None:
                    self.metrics.inc("watchhub_relists", labels={"kind": kind})
                await self._route(ki, parts, SNAPSHOT, rv.encode() + b"\n")
                # this frame lives as long as the watch: do not pin the LIST body and its
                # per-worker parts (tens of MB at 10k jobs) for the watch's lifetime
                del body, parts
                backoff = 0.2
                while True:
                    params = dict(base, watch="1", resourceVersion=rv, allowWatchBookmarks="true",
                                  timeoutSeconds=str(int(self.cfg.watch_timeout)))
                    splitter.reset()
                    async with self.kube.stream(path, params, timeout=self.cfg.watch_timeout + 30) as resp:
                        if resp.status == 410:
                            raise _Gone()
                        if resp.status >= 400:
                            from ..kube.flowcontrol import retry_after

                            err = RuntimeError(f"WATCH {kind}: HTTP {resp.status}")
                            err.retry_after = retry_after(resp.headers.get("Retry-After"))  # 429: APF's hint
                            raise err
                        async for chunk in resp.content.iter_any():
                            t_read = time.monotonic()
                            outs, last, errors = splitter.feed(chunk)
                            t_split = time.monotonic()
                            if last:
                                rv = last
                            if any(outs):
                                await self._route(ki, outs, LINES_T, STAMP.pack(t_read))
                            if _CHUNK_LOG and time.monotonic() - t_read > 0.001:
                                # diagnostic (NEXUS_SLOW_CALLBACK_LOG): a chunk that held the
                                # loop: its size, the bytes routed to workers, split / route time
                                sys.stderr.write(f"HUBCHUNK {t_read:.4f} {kind} in={len(chunk)} "
                                                 f"out={sum(len(o) for o in outs if o)} "
                                                 f"split={(t_split - t_read) * 1e3:.2f}ms "
                                                 f"route={(time.monotonic() - t_split) * 1e3:.2f}ms\n")
                            if ki == 0 and self.metrics is not None:
                                unread = self.router.stats["unread"]
                                if unread != self._unread_seen:
                                    self.metrics.inc("watch_events_unread", unread - self._unread_seen)
                                    self._unread_seen = unread
                            if errors:
                                if any(_is_gone(e) for e in errors):
                                    raise _Gone()
                                log.warning("%s watch error: %s", kind, errors[0][:300])
                                break
            except asyncio.CancelledError:
                raise
            except _Gone:
                log.info("%s watch expired at rv=%s: re-listing", kind, rv)
                continue
            except Exception as exc:  # noqa: BLE001 - connection errors: back off and re-list
                wait = max(backoff, getattr(exc, "retry_after", None) or 0.0)
                log.warning("%s hub list/watch failed: %s; retrying in %.1fs", kind, exc, wait)
                await asyncio.sleep(wait)
                backoff = min(backoff * 2, 30.0)


class HubFeed:
    """Worker side: reads the parent's frames and queues them per kind in arrival order.

    A protocol parses every complete frame of a socket read in one pass, and the LINES frames
    of one kind that arrive together are joined into one queue item: with 12 shard workers a
    hub frame carries about one line per worker, so per-frame reads, queue wake-ups and
    decoder calls were paid per watch line (profiles/r2_pprof_v11_fused: ~15 % of a worker's
    CPU in the feed and the informer's per-batch loop)."""

    def __init__(self):
        self.queues: Dict[int, asyncio.Queue] = {i: asyncio.Queue() for i in range(len(KINDS))}
        self._transport = None
        self.frames = 0
        self.reads = 0

    async def start(self, sock) -> None:
        loop = asyncio.get_running_loop()
        self._transport, _ = await loop.create_connection(lambda: _FeedProtocol(self), sock=sock)

    def _frames(self, buf: bytearray) -> int:
        """Queue every complete frame in ``buf``; returns the bytes consumed."""
        hs = HEADER.size
        n = len(buf)
        pos = 0
        pending: Dict[int, List[bytes]] = {}
        stamped: Dict[int, Tuple[float, float]] = {}  # kind -> (hub read time of its oldest lines, now)
        queues = self.queues
        view = memoryview(buf)
        t_feed = 0.0

        def lines_item(ki, parts):
            payload = b"".join(parts) if len(parts) > 1 else parts[0]
            st = stamped.pop(ki, None)
            return (LINES, payload) if st is None else (LINES, payload, st)

        try:
            while n - pos >= hs:
                ftype, ki, ln = HEADER.unpack_from(buf, pos)
                end = pos + hs + ln
                if end > n:
                    break
                if ftype == LINES_T and ln >= 8:
                    if not t_feed:
                        t_feed = time.monotonic()
                    if ki not in stamped:
                        stamped[ki] = (STAMP.unpack_from(buf, pos + hs)[0], t_feed)
                    payload = bytes(view[pos + hs + 8:end])
                    ftype = LINES
                else:
                    payload = bytes(view[pos + hs:end])
                pos = end
                self.frames += 1
                q = queues.get(ki)
                if q is None:
                    continue
                if ftype == LINES:
                    pending.setdefault(ki, []).append(payload)
                    continue
                parts = pending.pop(ki, None)  # this kind's earlier lines go first
                if parts:
                    q.put_nowait(lines_item(ki, parts))
                q.put_nowait((ftype, payload))
        finally:
            view.release()
        for ki, parts in pending.items():
            queues[ki].put_nowait(lines_item(ki, parts))
        return pos

    def _closed(self) -> None:
        for q in self.queues.values():
            q.put_nowait((0, b""))  # parent gone: informers stop on the closed feed

    def list_watch(self, kind: str) -> "HubListWatch":
        return HubListWatch(kind, self.queues[KINDS.index(kind)])

    async def close(self) -> None:
        t = self._transport
        if t is not None:
            self._transport = None
            t.close()


class _FeedProtocol(asyncio.Protocol):
    def __init__(self, feed: HubFeed):
        self.feed = feed
        self.buf = bytearray()

    def data_received(self, data: bytes) -> None:
        buf = self.buf
        buf += data
        self.feed.reads += 1
        used = self.feed._frames(buf)
        if used:
            del buf[:used]

    def connection_lost(self, exc) -> None:
        self.feed._closed()


class HubListWatch(ListWatch):
    """Informer transport fed by the parent's hub: ``list()`` returns the next snapshot,
    ``watch()`` yields routed lines until a newer snapshot arrives (then reports 410 so
    the informer re-lists, i.e. takes that snapshot)."""

    def __init__(self, kind: str, queue: asyncio.Queue):
        from .. import _kube_native

        self.kind = kind
        self.queue = queue
        proj = PROJECTIONS.get(kind)
        self._list_decoder = _kube_native.ProjectedDecoder(True if proj is None else ["list", proj])
        self._watch_proj = watch_projection(kind)
        self._pending: Optional[bytes] = None
        self.transform = None
        # native decode cost of the watch lines (thread CPU seconds, lines): the
        # informer_decode_* gauges, so a profile's decode share can be checked directly
        self.decode_seconds = 0.0
        self.decoded_lines = 0

    async def list(self) -> Tuple[List[Dict[str, Any]], str]:
        while self._pending is None:
            item = await self.queue.get()
            ftype, payload = item[0], item[1]
            if ftype == SNAPSHOT:
                self._pending = payload
            elif ftype == 0:
                raise ConnectionError("watch hub closed")
            # LINES before a snapshot belong to the stream it replaces: dropped
        payload, self._pending = self._pending, None
        nl = payload.index(b"\n")
        rv = payload[:nl].decode()
        items = self._list_decoder.decode(payload[nl + 1:])
        for it in items:
            it.setdefault("kind", self.kind)
        return items, rv

    async def watch_batches(self, resource_version: str):
        """The :meth:`watch` stream as one list of ``(type, object)`` per hub frame (the
        informer's batched path: no async-generator step per line)."""
        from .. import _kube_native

        decoder = _kube_native.ProjectedDecoder(self._watch_proj)
        kind = self.kind
        current = _delivery.CURRENT
        while True:
            item = await self.queue.get()
            ftype, payload = item[0], item[1]
            if ftype == SNAPSHOT:
                self._pending = payload
                yield [("ERROR", {"kind": "Status", "code": 410, "reason": "Expired", "message": "hub re-listed"})]
                return
            if ftype == 0:
                raise ConnectionError("watch hub closed")
            stamp = item[2] if len(item) > 2 else None  # the oldest joined frame's (hub, feed)
            # lines queued behind this frame while the worker was busy join it: one decode call
            # and one informer batch for all of them (a snapshot or close stays queued first)
            q = self.queue
            parts = None
            while q._queue and q._queue[0][0] == LINES:  # type: ignore[attr-defined]
                if parts is None:
                    parts = [payload]
                nxt = q.get_nowait()
                parts.append(nxt[1])
                if stamp is None and len(nxt) > 2:
                    stamp = nxt[2]
            if parts is not None:
                payload = b"".join(parts)
            # (type, object) pairs with the object's kind defaulted, built by the decoder itself
            t0 = _thread_time()
            batch = decoder.feed_events(payload, kind)
            self.decode_seconds += _thread_time() - t0
            self.decoded_lines += len(batch)
            if batch:
                if stamp is not None:
                    current[kind] = (stamp[0], stamp[1], time.monotonic())
                yield batch
                if stamp is not None:
                    current.pop(kind, None)  # dispatched: later (timer) handler calls get no stamps

    async def watch(self, resource_version: str):
        from .. import _kube_native

        decoder = _kube_native.ProjectedDecoder(self._watch_proj)
        kind = self.kind
        n = 0
        while True:
            item = await self.queue.get()
            ftype, payload = item[0], item[1]
            if ftype == SNAPSHOT:
                self._pending = payload
                yield "ERROR", {"kind": "Status", "code": 410, "reason": "Expired", "message": "hub re-listed"}
                return
            if ftype == 0:
                raise ConnectionError("watch hub closed")
            for ev in decoder.feed(payload):
                obj = ev.get("object") or {}
                if obj.get("kind") is None:
                    obj["kind"] = kind
                yield ev.get("type", ""), obj
                n += 1
                if n % 64 == 0:
                    await asyncio.sleep(0)
