"""Admission control and retry backoff for the work pipeline.

Replaces the nexus-core actor's limiter pair (call site
``/root/reference/services/supervisor.go:107-117``): a token bucket of
``rate-limit-elements-per-second`` / ``rate-limit-elements-burst``
(``golang.org/x/time/rate`` in the reference, ``go.mod:80``) and a per-key
exponential failure backoff ``failure-rate-base-delay`` → ``failure-rate-max-delay``.
"""
from __future__ import annotations

import asyncio
import time
from typing import Callable, Dict, Hashable


class TokenBucket:
    """Token bucket; ``rate <= 0`` disables limiting (extension: "uncapped")."""

    def __init__(self, rate: float, burst: int, clock: Callable[[], float] = time.monotonic):
        self.rate = float(rate)
        self.burst = max(1, int(burst))
        self.clock = clock
        self._tokens = float(self.burst)
        self._last = clock()

    @property
    def unlimited(self) -> bool:
        return self.rate <= 0

    def _refill(self) -> None:
        now = self.clock()
        if now > self._last:
            self._tokens = min(self.burst, self._tokens + (now - self._last) * self.rate)
        self._last = now

    def reserve(self) -> float:
        """Take one token; return how long the caller must wait before using it."""
        if self.unlimited:
            return 0.0
        self._refill()
        self._tokens -= 1.0
        if self._tokens >= 0:
            return 0.0
        return -self._tokens / self.rate

    async def acquire(self) -> None:
        delay = self.reserve()
        if delay > 0:
            await asyncio.sleep(delay)


class ExponentialBackoff:
    """Per-key ``base * 2**failures`` capped at ``max_delay`` (client-go
    ``ItemExponentialFailureRateLimiter`` semantics)."""

    def __init__(self, base_delay: float, max_delay: float):
        self.base = max(0.0, float(base_delay))
        self.max = max(self.base, float(max_delay))
        self._failures: Dict[Hashable, int] = {}

    def when(self, key: Hashable) -> float:
        n = self._failures.get(key, 0)
        self._failures[key] = n + 1
        if self.base == 0:
            return 0.0
        # avoid float overflow on huge n
        if n > 62:
            return self.max
        return min(self.max, self.base * (2 ** n))

    def failures(self, key: Hashable) -> int:
        return self._failures.get(key, 0)

    def forget(self, key: Hashable) -> None:
        self._failures.pop(key, None)

    def __len__(self) -> int:
        return len(self._failures)
