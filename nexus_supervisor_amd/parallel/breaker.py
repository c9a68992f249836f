"""Circuit breaker in front of the checkpoint store ("Missing: … circuit
breaker on CQL").

Without it a store outage turns into retries: every queued decision is attempted,
fails, backs off (``failure-rate-base-delay`` → ``failure-rate-max-delay``) and is
attempted again, each attempt costing a request against a store that is down, until
``max-retries`` dead-letters it — a Scylla restart longer than ~16 × 1 s loses every
decision queued behind it (until a restart replays it).  The reference has the same
retry loop and nothing else (nexus-core actor, ``/root/reference/services/supervisor.go:
107-117``).

Here the pipeline's workers pass a gate before each attempt:

* **closed** — normal operation; ``failure-threshold`` store failures in a row open it;
* **open** — attempts wait at the gate (queued decisions keep their place and their
  retry budget) for ``open-duration``, doubled on every re-open up to
  ``max-open-duration``;
* **half-open** — exactly one attempt (the probe) goes through; its success closes the
  breaker and releases everyone, its failure re-opens it; an attempt that never reached
  the store (a fenced decision) hands the probe to the next waiter.
"""
from __future__ import annotations

import asyncio
import logging
import time
from typing import Callable, Optional

log = logging.getLogger("nexus_supervisor_amd.breaker")

CLOSED, OPEN, HALF_OPEN = "closed", "open", "half-open"


class CircuitBreaker:
    def __init__(self, failure_threshold: int = 5, open_duration: float = 1.0, max_open_duration: float = 30.0,
                 metrics=None, clock: Callable[[], float] = time.monotonic):
        self.failure_threshold = max(1, int(failure_threshold))
        self.open_duration = max(0.001, float(open_duration))
        self.max_open_duration = max(self.open_duration, float(max_open_duration))
        self.metrics = metrics
        self.clock = clock
        self.state = CLOSED
        self.failures = 0           # consecutive store failures (closed state)
        self.until = 0.0            # open: when the next probe may go
        self._span = self.open_duration
        self._probing = False       # half-open: the probe is out
        self._changed: Optional[asyncio.Event] = None
        self.trips = 0
        self._gauge()

    # ------------------------------------------------------------------ gate
    def is_closed(self) -> bool:
        return self.state is CLOSED

    async def wait(self) -> None:
        """Return when this attempt may go to the store (the caller then reports its
        outcome with :meth:`success`, :meth:`failure` or :meth:`neutral`)."""
        while self.state is not CLOSED:
            now = self.clock()
            if self.state is OPEN and now >= self.until:
                self.state = HALF_OPEN
                self._gauge()
            if self.state is HALF_OPEN and not self._probing:
                self._probing = True
                return
            ev = self._event()
            timeout = max(0.001, self.until - now) if self.state is OPEN else None
            try:
                await asyncio.wait_for(ev.wait(), timeout)
            except asyncio.TimeoutError:
                pass

    # ------------------------------------------------------------------ outcomes
    def success(self) -> None:
        self.failures = 0
        if self.state is not CLOSED:
            log.info("checkpoint store answered again: circuit closed after %d trip(s)", self.trips)
            self.state = CLOSED
            self._probing = False
            self._span = self.open_duration
            self._gauge()
            self._notify()

    def failure(self) -> None:
        if self.state is CLOSED:
            self.failures += 1
            if self.failures >= self.failure_threshold:
                self._open()
        elif self.state is HALF_OPEN:
            self._span = min(self._span * 2, self.max_open_duration)
            self._open()
        # open: a straggler that was already in flight changes nothing

    def neutral(self) -> None:
        """The attempt never reached the store: if it was the probe, the next waiter probes."""
        if self.state is HALF_OPEN and self._probing:
            self._probing = False
            self._notify()

    # ------------------------------------------------------------------ internals
    def _open(self) -> None:
        if self.state is not OPEN:
            self.trips += 1
            if self.metrics is not None:
                self.metrics.inc("store_circuit_trips")
            log.warning("checkpoint store failing: circuit open for %.3gs (decisions wait in the queue)", self._span)
        self.state = OPEN
        self._probing = False
        self.failures = 0
        self.until = self.clock() + self._span
        self._gauge()
        self._notify()

    def _event(self) -> asyncio.Event:
        if self._changed is None:
            self._changed = asyncio.Event()
        return self._changed

    def _notify(self) -> None:
        ev, self._changed = self._changed, None
        if ev is not None:
            ev.set()

    def _gauge(self) -> None:
        if self.metrics is not None:
            self.metrics.set("store_circuit_open", 0.0 if self.state is CLOSED else 1.0)
