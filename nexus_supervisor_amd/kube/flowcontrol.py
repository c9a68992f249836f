"""Client-side API flow control: what client-go gives the reference for free.

The reference builds its clientset with ``clientcmd.BuildConfigFromFlags`` +
``kubernetes.NewForConfig`` and sets no QPS (``/root/reference/app/app_dependencies.go:
39-45``), so every request passes client-go's default token bucket (``rest.Config``
QPS 5, burst 10: ``flowcontrol.NewTokenBucketRateLimiter``), and a ``429 Too Many
Requests`` (or a 5xx) carrying ``Retry-After`` is retried after the server's hint, up to
10 times (``rest.Request`` ``checkWait`` / ``maxRetries``).  A real kube-apiserver with
API Priority and Fairness answers a burst of Job DELETEs or a wave of ``pods/log`` reads
with exactly those 429s.

Here:

* :class:`TokenBucket` — ``kube-qps`` / ``kube-burst``, shared by every request of one
  process.  Waiters are released at ``qps`` (never in a burst larger than ``burst``) by
  weighted round robin over request classes (reads, mutations, Events), in arrival order
  within a class.  ``qps <= 0`` = no limit.
* :class:`SharedSchedule` — a replica split into shard-worker processes draws from one
  budget in shared memory (GCRA word), so a skewed wave is not capped at ``qps / K``.
* :func:`retry_after` — the server's hint (integer seconds, as client-go reads it; an
  HTTP-date is honoured too), bounded by ``cap``.
* :class:`RetryPolicy` — which answers are retried and how long to wait: 429 always (1 s
  when the server gave no hint), 5xx only with a ``Retry-After`` (client-go's rule), never
  earlier than the hint.
"""
from __future__ import annotations

import asyncio
import email.utils
import heapq
import time
from typing import Callable, Optional

# the reference's effective limits (client-go rest.Config defaults, app_dependencies.go:39-45)
CLIENT_GO_QPS, CLIENT_GO_BURST, CLIENT_GO_MAX_RETRIES = 5.0, 10, 10


# request classes of the bucket: the reads a waiting decision needs (pods/log tails, LIST /
# WATCH), mutations (background Job DELETEs that free a failed job's GPUs, agent PATCHes),
# and the supervisor's own decision Events
READ, MUTATE, EVENT = 0, 1, 2
# weighted round robin over the classes that have waiters: with all three queued, reads and
# DELETEs get 2/5 of the tokens each and Events 1/5; an idle class's share goes to the others
CLASS_WEIGHTS = (2, 2, 1)


def _wrr_cycle(weights) -> tuple:
    """Smooth weighted round robin order of the classes (nginx's algorithm): (2, 2, 1) ->
    (0, 1, 2, 0, 1) — no class waits more than one turn of the others between tokens."""
    cur = [0] * len(weights)
    total = sum(weights)
    out = []
    for _ in range(total):
        for i, w in enumerate(weights):
            cur[i] += w
        best = max(range(len(weights)), key=lambda i: (cur[i], -i))
        cur[best] -= total
        out.append(best)
    return tuple(out)


class SharedSchedule:
    """A replica's ``kube-qps`` / ``kube-burst`` as one GCRA word in a shared mapping
    (``csrc/kube/shared_bucket.cpp``): the parent's watch hub and every shard worker draw
    from it, so together they never exceed the replica's budget and a worker holding most
    of a wave gets most of the tokens instead of a fixed 1/K."""

    __slots__ = ("fd", "buf", "interval_ns", "tolerance_ns", "_k")

    SIZE = 64

    def __init__(self, qps: float, burst: int, fd: Optional[int] = None):
        import mmap
        import os

        from .. import _kube_native

        self._k = _kube_native
        if fd is None:
            fd = os.memfd_create("nexus-kube-qps", 0)  # inherited by the workers (pass_fds)
            os.ftruncate(fd, self.SIZE)
        self.fd = fd
        self.buf = mmap.mmap(fd, self.SIZE)
        self.interval_ns = max(1, int(1e9 / float(qps)))
        self.tolerance_ns = max(0, int(burst) - 1) * self.interval_ns

    def reserve(self) -> float:
        return self._k.bucket_reserve(self.buf, self.interval_ns, self.tolerance_ns) / 1e9

    def try_take(self) -> bool:
        return self._k.bucket_try_take(self.buf, self.interval_ns, self.tolerance_ns)

    def give_back(self) -> None:
        self._k.bucket_give_back(self.buf, self.interval_ns, self.tolerance_ns)

    def backlog(self) -> float:
        return self._k.bucket_backlog(self.buf) / 1e9


class TokenBucket:
    """Token bucket rate limiter (``qps`` tokens per second, at most ``burst`` banked) whose
    waiters are served by weighted round robin over request classes, in arrival order
    within a class.

    client-go has one FIFO bucket; a failure wave on default GPU pods needs both a
    ``pods/log`` read per failure (to classify it) and a Job DELETE per failure (which
    frees the job's GPUs — its other ranks otherwise hang in an all-reduce until the
    watchdog).  Strict priority for reads starved the DELETEs for the whole wave (at 50 qps
    a 1,000-pod wave is 20 s of reads); a FIFO puts each read behind every DELETE queued
    before it.  With :data:`CLASS_WEIGHTS` each class that has waiters is guaranteed its
    share and no class waits for another to drain.

    ``shared``: a :class:`SharedSchedule` replaces the local tokens (a replica's processes
    draw from one budget); the class scheduling stays per process."""

    __slots__ = ("qps", "burst", "tokens", "last", "clock", "waits", "waited_s", "_queues", "_cycle", "_pos",
                 "_timer", "shared", "_held", "served", "max_wait", "_nq")

    def __init__(self, qps: float, burst: int, clock: Callable[[], float] = time.monotonic,
                 weights=CLASS_WEIGHTS, shared: Optional[SharedSchedule] = None):
        import collections

        self.qps = float(qps)
        self.burst = max(1, int(burst))
        self.tokens = float(self.burst)
        self.clock = clock
        self.last = clock()
        self.waits = 0        # requests that had to wait for a token
        self.waited_s = 0.0   # total time they waited
        self._queues = [collections.deque() for _ in weights]  # per class: (enqueued_at, future)
        self._nq = 0          # futures in the queues (cancelled ones included until popped)
        self._cycle = _wrr_cycle(weights)
        self._pos = 0
        self._timer = None
        self.shared = shared if self.qps > 0 else None
        self._held = False    # shared mode: a committed reservation waits for its timer
        self.served = [0] * len(weights)       # waiters released per class
        self.max_wait = [0.0] * len(weights)   # longest wait per class

    @property
    def unlimited(self) -> bool:
        return self.qps <= 0

    @property
    def queued(self) -> int:
        return sum(1 for q in self._queues for w in q if not w[1].done())

    def _refill(self) -> float:
        now = self.clock()
        if now > self.last:
            self.tokens = min(float(self.burst), self.tokens + (now - self.last) * self.qps)
            self.last = now
        return now

    def _take_now(self) -> bool:
        if self.shared is not None:
            return self.shared.try_take()
        self._refill()
        if self.tokens >= 1.0:
            self.tokens -= 1.0
            return True
        return False

    def try_accept(self) -> bool:
        """Take a token if one is banked right now and nobody is queued (client-go
        ``TryAccept``; a caller that gets False falls back to :meth:`wait`)."""
        if self.qps <= 0:
            return True
        if self._nq:
            return False
        return self._take_now()

    def give_back(self) -> None:
        """Return a token taken by :meth:`try_accept` that was not used (the request could
        not be sent and goes through :meth:`wait` instead)."""
        if self.qps <= 0:
            return
        if self.shared is not None:
            self.shared.give_back()
        else:
            self.tokens = min(float(self.burst), self.tokens + 1.0)
        if self._nq:
            self._kick()

    async def wait(self, priority: int = MUTATE, timeout: Optional[float] = None) -> float:
        """client-go ``Wait``: block until this request may go; returns the time waited.
        ``timeout``: give up after that long (``asyncio.TimeoutError``; no token taken)."""
        if self.qps <= 0:
            return 0.0
        if not self._nq and self._take_now():
            return 0.0
        cls = min(max(0, int(priority)), len(self._queues) - 1)
        loop = asyncio.get_running_loop()
        fut = loop.create_future()
        t0 = self.clock()
        self._queues[cls].append((t0, fut))
        self._nq += 1
        self._kick()
        try:
            if timeout is None:
                await fut
            else:
                await asyncio.wait_for(asyncio.shield(fut), timeout)
        except (asyncio.TimeoutError, asyncio.CancelledError):
            # timed out, or the caller was cancelled (a log fetch on fence or shard loss): a
            # token released to us in the same tick goes back, a queued wait is withdrawn —
            # in shared mode a stranded token is the whole replica's budget
            if fut.done() and not fut.cancelled():
                self.give_back()
            else:
                fut.cancel()
            raise
        d = self.clock() - t0
        self.waits += 1
        self.waited_s += d
        return d

    def _next(self):
        """Pop the next live waiter by weighted round robin, or None."""
        if not self._nq:
            return None
        qs = self._queues
        cyc = self._cycle
        n = len(cyc)
        for _ in range(2):
            for step in range(n):
                c = cyc[(self._pos + step) % n]
                q = qs[c]
                while q and q[0][1].done():  # cancelled / timed out
                    q.popleft()
                    self._nq -= 1
                if q:
                    self._pos = (self._pos + step + 1) % n
                    t0, fut = q.popleft()
                    self._nq -= 1
                    d = self.clock() - t0
                    self.served[c] += 1
                    if d > self.max_wait[c]:
                        self.max_wait[c] = d
                    return fut
        return None

    def _kick(self) -> None:
        if self._timer is not None:
            return
        try:
            loop = asyncio.get_running_loop()
        except RuntimeError:
            loop = asyncio.get_event_loop()
        if self.shared is not None:
            self._release_shared(loop)
        else:
            self._refill()
            self._timer = loop.call_later(max(0.0, (1.0 - self.tokens) / self.qps), self._release)

    def _release(self) -> None:
        self._timer = None
        self._refill()
        while self._nq and self.tokens >= 1.0:
            fut = self._next()
            if fut is None:
                break
            self.tokens -= 1.0
            fut.set_result(None)
        if self._nq:
            self._kick()

    def _release_shared(self, loop) -> None:
        """Shared mode: commit a reservation for the head waiter; release it now when the
        slot is due, else when the timer fires (one reservation held per process)."""
        sh = self.shared
        while self._nq:
            if not self._held:
                d = sh.reserve()
                self._held = True
                if d > 0:
                    self._timer = loop.call_later(d, self._fire_shared)
                    return
            fut = self._next()
            self._held = False
            if fut is None:
                sh.give_back()
                return
            fut.set_result(None)
        if self._held and not self._nq:
            self._held = False
            sh.give_back()

    def _fire_shared(self) -> None:
        self._timer = None
        try:
            loop = asyncio.get_running_loop()
        except RuntimeError:
            loop = asyncio.get_event_loop()
        self._release_shared(loop)


_WORKER_SCHEDULE: list = []  # [SharedSchedule or None] once looked up in a shard worker


def replica_schedule(cfg, create: bool = False) -> Optional[SharedSchedule]:
    """The replica's shared API budget: in a shard worker the one its parent passed
    (``NEXUS_WORKER_QPS_FD``); in a parent with ``create`` a new one when the replica runs
    more than one process and ``kube-qps`` limits it.  None = a per-process bucket."""
    import os

    qps, burst = float(cfg.kube_qps), int(cfg.kube_burst)
    if qps <= 0:
        return None
    fd = os.environ.get("NEXUS_WORKER_QPS_FD")
    if fd:
        if not _WORKER_SCHEDULE:
            try:
                _WORKER_SCHEDULE.append(SharedSchedule(qps, burst, fd=int(fd)))
            except (ImportError, OSError, ValueError):
                _WORKER_SCHEDULE.append(None)
        return _WORKER_SCHEDULE[0]
    if create and int(getattr(cfg.runtime, "worker_processes", 1) or 1) > 1:
        try:
            return SharedSchedule(qps, burst)
        except (ImportError, OSError, AttributeError):
            return None
    return None


def split(qps: float, burst: int, parts: int):
    """A replica's ``kube-qps`` / ``kube-burst`` divided over ``parts`` processes (each
    holds its own bucket; together they never exceed the replica's).  Used only when the
    replica has no :class:`SharedSchedule`."""
    parts = max(1, int(parts))
    if qps <= 0 or parts == 1:
        return qps, burst
    return qps / parts, max(1, int(burst) // parts)


def retry_after(value: Optional[str], cap: float = 60.0, now: Optional[float] = None) -> Optional[float]:
    """Seconds from a ``Retry-After`` header value (delta-seconds or HTTP-date), bounded
    to ``[0, cap]``; None when absent or unparsable."""
    if value is None:
        return None
    if isinstance(value, (bytes, bytearray)):
        value = value.decode("latin-1")
    v = value.strip()
    if not v:
        return None
    try:
        secs = float(int(v))
    except ValueError:
        try:
            dt = email.utils.parsedate_to_datetime(v)
        except (TypeError, ValueError):
            return None
        if dt is None:
            return None
        secs = dt.timestamp() - (time.time() if now is None else now)
    return min(max(0.0, secs), cap)


class RetryPolicy:
    """When to retry an API answer and after how long (client-go ``checkWait``)."""

    __slots__ = ("max_retries", "cap", "default_429")

    def __init__(self, max_retries: int = CLIENT_GO_MAX_RETRIES, cap: float = 60.0, default_429: float = 1.0):
        self.max_retries = max(0, int(max_retries))
        self.cap = cap
        self.default_429 = default_429

    def delay(self, status: int, hint: Optional[float]) -> Optional[float]:
        """Seconds to wait before retrying an answer with ``status`` and ``Retry-After``
        hint ``hint`` (already parsed); None = not retryable."""
        if status == 429:
            return min(self.cap, hint if hint is not None else self.default_429)
        if status >= 500 and hint is not None:
            return min(self.cap, hint)
        return None
