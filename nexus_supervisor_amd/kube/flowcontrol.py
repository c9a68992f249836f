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
  process (a replica split into shard workers divides them, ``split``).  Waiters are
  released at ``qps`` (never in a burst larger than ``burst``) by priority, then in arrival
  order: decision reads first, background Job DELETEs next, Events last.  ``qps <= 0`` = no
  limit.
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


class TokenBucket:
    """Token bucket rate limiter (``qps`` tokens per second, at most ``burst`` banked) whose
    waiters are served by priority, then in arrival order.

    client-go has one FIFO bucket; here a failure wave's background Job DELETEs (priority 1)
    must not delay the ``pods/log`` reads (priority 0) that the waiting decisions need — a
    FIFO reservation would put a read behind every DELETE queued before it (at 50 qps, a
    1,000-pod wave is 20 s of DELETEs).  Decision Events are priority 2."""

    __slots__ = ("qps", "burst", "tokens", "last", "clock", "waits", "waited_s", "_waiters", "_seq", "_timer")

    def __init__(self, qps: float, burst: int, clock: Callable[[], float] = time.monotonic):
        self.qps = float(qps)
        self.burst = max(1, int(burst))
        self.tokens = float(self.burst)
        self.clock = clock
        self.last = clock()
        self.waits = 0        # requests that had to wait for a token
        self.waited_s = 0.0   # total time they waited
        self._waiters: list = []  # heap of (priority, seq, future)
        self._seq = 0
        self._timer = None

    @property
    def unlimited(self) -> bool:
        return self.qps <= 0

    @property
    def queued(self) -> int:
        return sum(1 for w in self._waiters if not w[2].done())

    def _refill(self) -> float:
        now = self.clock()
        if now > self.last:
            self.tokens = min(float(self.burst), self.tokens + (now - self.last) * self.qps)
            self.last = now
        return now

    def try_accept(self) -> bool:
        """Take a token if one is banked right now and nobody is queued (client-go
        ``TryAccept``; a caller that gets False falls back to :meth:`wait`)."""
        if self.qps <= 0:
            return True
        if self._waiters:
            return False
        self._refill()
        if self.tokens >= 1.0:
            self.tokens -= 1.0
            return True
        return False

    async def wait(self, priority: int = 1) -> float:
        """client-go ``Wait``: block until this request may go; returns the time waited."""
        if self.qps <= 0:
            return 0.0
        self._refill()
        if not self._waiters and self.tokens >= 1.0:
            self.tokens -= 1.0
            return 0.0
        loop = asyncio.get_running_loop()
        fut = loop.create_future()
        self._seq += 1
        heapq.heappush(self._waiters, (priority, self._seq, fut))
        self._arm(loop)
        t0 = self.clock()
        await fut
        d = self.clock() - t0
        self.waits += 1
        self.waited_s += d
        return d

    def _arm(self, loop) -> None:
        if self._timer is None and self._waiters:
            self._refill()
            self._timer = loop.call_later(max(0.0, (1.0 - self.tokens) / self.qps), self._release)

    def _release(self) -> None:
        self._timer = None
        self._refill()
        ws = self._waiters
        while ws and self.tokens >= 1.0:
            _p, _s, fut = heapq.heappop(ws)
            if fut.done():  # the waiter was cancelled
                continue
            self.tokens -= 1.0
            fut.set_result(None)
        while ws and ws[0][2].done():
            heapq.heappop(ws)
        if ws:
            self._arm(asyncio.get_event_loop())


def split(qps: float, burst: int, parts: int):
    """A replica's ``kube-qps`` / ``kube-burst`` divided over ``parts`` shard-worker
    processes (each holds its own bucket; together they never exceed the replica's)."""
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
