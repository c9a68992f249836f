"""Keyed, rate-limited, retrying work pipeline (asyncio).

This is the supervisor's equivalent of nexus-core's
``pipeline.NewDefaultPipelineStageActor`` (constructed at
``/root/reference/services/supervisor.go:107-117``, fed by ``Receive`` at
``:174-252``, started at ``:376-388``), redesigned around the two hazards
SURVEY §2.7/§5.2 found in the reference:

* **per-key serialization** — items with the same run key ``(algorithm, id)``
  are processed one at a time, in arrival order, by whichever worker holds the
  key; a failing item blocks later items of its key until it succeeds or is
  dead-lettered (so "pod Failed then BackOff" is deterministic);
* **coalescing** — an item equal (by ``coalesce_key``) to one already pending
  for the key is dropped;
* **bounded retries** — per-key exponential backoff, then a dead-letter
  callback instead of retrying forever.

Admission is a token bucket taken per dequeued item (rate 0 = uncapped).
``workers`` is the number of concurrently processed keys; because the
processor is a coroutine, a worker waiting on CQL/K8s I/O costs nothing, so
hundreds of workers are cheap.
"""
from __future__ import annotations

import asyncio
import collections
import logging
import time
from typing import Any, Awaitable, Callable, Deque, Dict, Hashable, Optional

from .ratelimit import ExponentialBackoff, TokenBucket

log = logging.getLogger("nexus_supervisor_amd.pipeline")


class PipelineStats:
    __slots__ = ("received", "coalesced", "processed", "failed_attempts", "retries", "dead_lettered", "dropped_closed")

    def __init__(self):
        self.received = self.coalesced = self.processed = 0
        self.failed_attempts = self.retries = self.dead_lettered = self.dropped_closed = 0

    def as_dict(self) -> Dict[str, int]:
        return {k: getattr(self, k) for k in self.__slots__}


class _Entry:
    __slots__ = ("item", "ckey")

    def __init__(self, item, ckey):
        self.item = item
        self.ckey = ckey


class PipelineStage:
    def __init__(
        self,
        name: str,
        processor: Callable[[Any], Awaitable[Any]],
        *,
        workers: int = 2,
        elements_per_second: float = 10,
        burst: int = 100,
        base_delay: float = 0.1,
        max_delay: float = 1.0,
        max_retries: int = 16,
        key_fn: Callable[[Any], Hashable] = lambda x: x.key,
        coalesce_key: Optional[Callable[[Any], Hashable]] = None,
        on_dead_letter: Optional[Callable[[Any, BaseException], None]] = None,
        on_done: Optional[Callable[[Any, Any], None]] = None,
        tags: Optional[Dict[str, str]] = None,
        clock: Callable[[], float] = time.monotonic,
        gate=None,
    ):
        if workers < 1:
            raise ValueError("workers must be >= 1")
        self.name = name
        self.tags = dict(tags or {})
        self.processor = processor
        self.n_workers = workers
        self.bucket = TokenBucket(elements_per_second, burst, clock)
        self.backoff = ExponentialBackoff(base_delay, max_delay)
        self.max_retries = max_retries
        # optional admission gate before every attempt (``is_closed()`` / ``await wait()``:
        # the store circuit breaker, parallel/breaker.py) — an item waiting there keeps its
        # key's place and its retry budget
        self.gate = gate
        self.key_fn = key_fn
        self.coalesce_key = coalesce_key
        self.on_dead_letter = on_dead_letter
        self.on_done = on_done
        self.stats = PipelineStats()
        self._pending: Dict[Hashable, Deque[_Entry]] = {}
        self._ready: Deque[Hashable] = collections.deque()
        self._active: set = set()       # keys held by a worker or waiting out a backoff
        self._running: set = set()      # keys a worker is processing right now
        # idle workers park on their own future; a signal wakes exactly one (a shared
        # Event would wake every idle worker per item: 256 wakeups for one decision)
        self._waiters: Deque[asyncio.Future] = collections.deque()
        self._tasks = []
        self._timers: Dict[Hashable, asyncio.TimerHandle] = {}  # backoff retries by key
        self._closed = False
        self._idle: Optional[asyncio.Event] = None
        self._loop: Optional[asyncio.AbstractEventLoop] = None

    # ---------------------------------------------------------------- intake
    def receive(self, item: Any) -> bool:
        """Enqueue ``item`` (nexus-core ``actor.Receive``). Must be called on the loop thread."""
        if self._closed:
            self.stats.dropped_closed += 1
            return False
        self.stats.received += 1
        key = self.key_fn(item)
        ckey = self.coalesce_key(item) if self.coalesce_key else None
        q = self._pending.get(key)
        if q is None:
            q = self._pending[key] = collections.deque()
        elif ckey is not None and any(e.ckey == ckey for e in q):
            self.stats.coalesced += 1
            return True
        q.append(_Entry(item, ckey))
        if key not in self._active and len(q) == 1:
            self._ready.append(key)
            self._signal()
        if self._idle is not None:
            self._idle.clear()
        return True

    def receive_threadsafe(self, item: Any) -> None:
        assert self._loop is not None, "pipeline not started"
        self._loop.call_soon_threadsafe(self.receive, item)

    def _signal(self):
        waiters = self._waiters
        while waiters:
            w = waiters.popleft()
            if not w.done():
                w.set_result(None)
                return

    # ---------------------------------------------------------------- workers
    async def _next_key(self) -> Optional[Hashable]:
        while True:
            if self._ready:
                return self._ready.popleft()
            if self._closed and not self._pending and not self._active:
                return None
            self._check_idle()
            fut = self._loop.create_future()
            self._waiters.append(fut)
            try:
                await fut
            except asyncio.CancelledError:
                if fut.done() and not fut.cancelled():
                    self._signal()  # woken, then cancelled: hand the wakeup on
                raise

    def busy(self) -> bool:
        """Any decision queued, waiting out a backoff or being processed."""
        return bool(self._pending or self._active or self._ready)

    def _check_idle(self):
        if self._idle is not None and not self._pending and not self._active and not self._ready:
            self._idle.set()

    async def _worker(self, wid: int):
        while True:
            key = await self._next_key()
            if key is None:
                self._signal()  # let siblings observe shutdown
                return
            q = self._pending.get(key)
            if not q:
                self._pending.pop(key, None)
                continue
            self._active.add(key)
            self._running.add(key)
            entry = q[0]
            delay = self.bucket.reserve()
            if delay > 0:
                await asyncio.sleep(delay)
            gate = self.gate
            gated = False
            try:
                if gate is not None and not gate.is_closed():
                    await gate.wait()
                    gated = True
                out = await self.processor(entry.item)
            except asyncio.CancelledError:
                self._running.discard(key)
                raise
            except BaseException as exc:  # noqa: BLE001 - every failure is retried / dead-lettered
                self._running.discard(key)
                self.stats.failed_attempts += 1
                if gated and getattr(gate, "state", None) == "open":
                    # a probe through the open gate failed and the gate is shut again: that is
                    # the store's verdict, not this item's — it keeps its retry budget and
                    # waits at the gate again (which item probes is the scheduler's choice)
                    self.stats.retries += 1
                    self._schedule_retry(key, 0.0)
                    continue
                nfail = self.backoff.failures(key) + 1
                if self.max_retries and nfail > self.max_retries:
                    self.stats.dead_lettered += 1
                    self.backoff.forget(key)
                    q.popleft()
                    log.error("%s: dead-lettering item for key %s after %d attempts: %s", self.name, key, nfail, exc)
                    if self.on_dead_letter:
                        try:
                            self.on_dead_letter(entry.item, exc)
                        except Exception:  # pragma: no cover
                            log.exception("dead-letter hook failed")
                    self._release(key)
                    continue
                wait = self.backoff.when(key)
                self.stats.retries += 1
                log.debug("%s: retry key %s in %.3fs (%s)", self.name, key, wait, exc)
                self._schedule_retry(key, wait)
                continue
            self._running.discard(key)
            self.stats.processed += 1
            self.backoff.forget(key)
            q.popleft()
            if self.on_done:
                try:
                    self.on_done(entry.item, out)
                except Exception:  # pragma: no cover
                    log.exception("on_done hook failed")
            self._release(key)

    def _release(self, key):
        self._active.discard(key)
        q = self._pending.get(key)
        if q:
            self._ready.append(key)
            self._signal()
        else:
            self._pending.pop(key, None)
            self._check_idle()

    def _schedule_retry(self, key, wait):
        # key stays in _active: later items of the same key cannot overtake the retried one
        def fire():
            self._timers.pop(key, None)
            self._active.discard(key)
            if self._pending.get(key):
                self._ready.appendleft(key)
                self._signal()
            else:
                self._pending.pop(key, None)
                self._check_idle()

        self._timers[key] = self._loop.call_later(wait, fire)

    # ---------------------------------------------------------------- lifecycle
    async def start(self, post_start: Optional[Callable[[], Awaitable[None]]] = None) -> None:
        """Spawn workers, then run ``post_start`` (e.g. start informers + wait for sync;
        ``/root/reference/services/supervisor.go:377-387``)."""
        self._loop = asyncio.get_running_loop()
        self._idle = asyncio.Event()
        self._tasks = [asyncio.create_task(self._worker(i), name=f"{self.name}-w{i}") for i in range(self.n_workers)]
        if self._ready:
            self._signal()
        if post_start is not None:
            await post_start()

    async def join(self, timeout: Optional[float] = None) -> bool:
        """Wait until nothing is pending, in flight or waiting on a backoff."""
        self._check_idle()
        try:
            await asyncio.wait_for(self._idle.wait(), timeout)
            return True
        except asyncio.TimeoutError:
            return False

    async def stop(self, drain: bool = True, timeout: float = 10.0) -> None:
        """Stop intake; with ``drain`` let workers finish queued items first (SIGTERM drain —
        the reference has none)."""
        self._closed = True
        if drain:
            await self.join(timeout)
        for h in list(self._timers.values()):
            h.cancel()
        self._timers.clear()
        self._pending.clear()
        self._active.clear()
        self._ready.clear()
        self._signal()
        for t in self._tasks:
            t.cancel()
        await asyncio.gather(*self._tasks, return_exceptions=True)
        self._tasks = []

    def clear(self, predicate: Optional[Callable[[Hashable], bool]] = None) -> int:
        """Drop every queued item and every backoff retry (fencing on lost leadership),
        or only those of keys ``predicate`` accepts (a lost replica shard); items a worker
        is processing right now finish (their processor checks the fence itself).
        Returns the number of items dropped."""
        dropped = 0
        gone = set()
        for key, q in list(self._pending.items()):
            if predicate is not None and not predicate(key):
                continue
            if key in self._running:
                while len(q) > 1:
                    q.pop()
                    dropped += 1
                continue
            dropped += len(q)
            del self._pending[key]
            gone.add(key)
            h = self._timers.pop(key, None)
            if h is not None:
                h.cancel()
            self._active.discard(key)
            self.backoff.forget(key)
        if predicate is None:
            self._ready.clear()
        elif gone:
            # a dropped key re-received later is queued afresh: no stale duplicate may stay
            self._ready = collections.deque(k for k in self._ready if k not in gone)
        self.stats.dropped_closed += dropped
        self._check_idle()
        return dropped

    # ---------------------------------------------------------------- introspection
    def depth(self) -> int:
        return sum(len(q) for q in self._pending.values())

    def in_flight(self) -> int:
        return len(self._active)
