"""Lease-based leader election (``coordination.k8s.io/v1`` Lease).

The reference has no leader election: every replica processes every event
(``/root/reference/.helm/values.yaml:124-125`` "Increase to support higher
(1000+) pod numbers").  BASELINE config 5 asks for a
2-replica supervisor with leader election, so this module implements the
client-go ``leaderelection`` contract:

* the holder renews ``spec.renewTime`` every ``retry_period``; a renewal that
  cannot be completed within ``renew_deadline`` steps down;
* a candidate takes over once ``renewTime + leaseDurationSeconds`` has passed
  (optimistic concurrency on ``metadata.resourceVersion`` — a lost race is a
  409 and the candidate stays standby);
* ``leaseTransitions`` counts holder changes; ``release`` on shutdown clears the
  holder so a standby takes over immediately instead of after a full lease.

Time comparisons use the local clock on *observed* record changes (as client-go
does): a candidate measures expiry from when it last saw the record change,
so skew between nodes does not matter.

Ownership is time-bounded at write time, not only by renewal progress: a renewal that
*started* at ``t0`` (before its GET) and succeeded makes this replica the holder until
``t0 + renew_deadline`` (:attr:`LeaderElector.valid_until`, reported through
``on_renewed``).  Any other candidate can only take over ``lease_duration`` after it
*observed* that renewal, i.e. after ``t0 + lease_duration`` > ``valid_until``.  Every
renewal attempt is bounded by the time left to ``valid_until`` and the holder steps down
the moment it passes, so a stalled or partitioned apiserver can never leave a deposed
leader acting after its successor started (the supervisor also checks ``valid_until``
before each write and Job DELETE).
"""
from __future__ import annotations

import asyncio
import datetime as _dt
import logging
import time
from typing import Callable, Optional, Tuple

from ..kube.errors import ApiError, Conflict, NotFound

log = logging.getLogger("nexus_supervisor_amd.leader")


def _micro(t: Optional[float] = None) -> str:
    d = _dt.datetime.fromtimestamp(time.time() if t is None else t, _dt.timezone.utc)
    return d.strftime("%Y-%m-%dT%H:%M:%S.%fZ")


class LeaseLock:
    """Read/create/update one Lease object through a :class:`KubeClient`-like API."""

    def __init__(self, client, namespace: str, name: str, identity: str, labels: Optional[dict] = None):
        self.client = client
        self.namespace = namespace
        self.name = name
        self.identity = identity
        self.labels = dict(labels or {})

    async def get(self):
        try:
            return await self.client.get("Lease", self.namespace, self.name)
        except NotFound:
            return None

    async def create(self, spec):
        md = {"name": self.name, "namespace": self.namespace}
        if self.labels:
            md["labels"] = dict(self.labels)
        body = {"apiVersion": "coordination.k8s.io/v1", "kind": "Lease", "metadata": md, "spec": spec}
        return await self.client.create("Lease", self.namespace, body)

    async def update(self, lease, spec):
        body = dict(lease)
        body["spec"] = spec
        return await self.client.replace("Lease", self.namespace, self.name, body)


class LeaderElector:
    def __init__(self, lock: LeaseLock, *, lease_duration: float = 15.0, renew_deadline: float = 10.0,
                 retry_period: float = 2.0, on_started_leading: Optional[Callable[[], None]] = None,
                 on_stopped_leading: Optional[Callable[[], None]] = None, metrics=None,
                 clock: Callable[[], float] = time.monotonic,
                 on_renewed: Optional[Callable[[float], None]] = None):
        if not lease_duration > renew_deadline > retry_period > 0:
            raise ValueError("lease_duration > renew_deadline > retry_period > 0 required")
        self.lock = lock
        self.lease_duration = lease_duration
        self.renew_deadline = renew_deadline
        self.retry_period = retry_period
        self.on_started = on_started_leading
        self.on_stopped = on_stopped_leading
        self.on_renewed = on_renewed
        self.metrics = metrics
        self.clock = clock
        self.leader = False
        self.valid_until = float("-inf")  # clock time this replica's hold expires locally
        self.observed_holder = ""
        self._observed_record = None
        self._observed_at = 0.0
        self._task: Optional[asyncio.Task] = None
        self.transitions_seen = 0

    @property
    def identity(self) -> str:
        return self.lock.identity

    def start(self) -> asyncio.Task:
        if self._task is None:
            self._task = asyncio.create_task(self._run(), name=f"leader-{self.identity}")
        return self._task

    async def stop(self, release: bool = True) -> None:
        if self._task is not None:
            self._task.cancel()
            try:
                await self._task
            except (asyncio.CancelledError, Exception):
                pass
            self._task = None
        if release and self.leader:
            try:
                await self._release()
            except Exception as exc:  # noqa: BLE001
                log.warning("lease release failed: %s", exc)
        self._set_leader(False)

    def _renewed(self, t0: float) -> None:
        self.valid_until = t0 + self.renew_deadline
        if self.on_renewed is not None:
            try:
                self.on_renewed(self.valid_until)
            except Exception:  # pragma: no cover
                log.exception("lease renewal callback failed")

    async def acquire_or_renew_bounded(self, budget: float) -> Tuple[bool, float]:
        """:meth:`try_acquire_or_renew` bounded by ``budget`` seconds; returns (ok, t0) with
        ``t0`` the clock before the request went out — the start of the new hold."""
        t0 = self.clock()
        if budget <= 0:
            return False, t0
        ok = await asyncio.wait_for(self.try_acquire_or_renew(), budget)
        return ok, t0

    def _set_leader(self, v: bool) -> None:
        if v == self.leader:
            return
        self.leader = v
        if self.metrics is not None:
            self.metrics.set("leader", 1.0 if v else 0.0)
            self.metrics.inc("leader_transitions")
        log.info("%s %s leadership of lease %s/%s", self.identity, "acquired" if v else "lost",
                 self.lock.namespace, self.lock.name)
        cb = self.on_started if v else self.on_stopped
        if cb is not None:
            try:
                cb()
            except Exception:  # pragma: no cover
                log.exception("leadership callback failed")

    def _spec(self, lease) -> dict:
        prev = (lease or {}).get("spec") or {}
        now = _micro()
        transitions = int(prev.get("leaseTransitions") or 0)
        acquire = prev.get("acquireTime") or now
        if prev.get("holderIdentity") != self.identity:
            transitions += 1 if prev.get("holderIdentity") else 0
            acquire = now
        return {"holderIdentity": self.identity, "leaseDurationSeconds": int(round(self.lease_duration)),
                "acquireTime": acquire, "renewTime": now, "leaseTransitions": transitions}

    async def try_acquire_or_renew(self) -> bool:
        lease = await self.lock.get()
        now = self.clock()
        if lease is None:
            try:
                await self.lock.create(self._spec(None))
            except (Conflict, ApiError) as exc:
                if isinstance(exc, Conflict) or getattr(exc, "status", 0) == 409:
                    return False
                raise
            self._observe({"holderIdentity": self.identity}, now)
            return True
        spec = lease.get("spec") or {}
        record = (spec.get("holderIdentity"), spec.get("renewTime"), spec.get("leaseTransitions"))
        if record != self._observed_record:
            self._observe(spec, now, record)
        holder = spec.get("holderIdentity") or ""
        duration = float(spec.get("leaseDurationSeconds") or self.lease_duration)
        if holder and holder != self.identity and now < self._observed_at + duration:
            return False  # someone else holds a live lease
        try:
            await self.lock.update(lease, self._spec(lease))
        except Conflict:
            return False
        self._observe({"holderIdentity": self.identity}, now)
        return True

    async def observe(self) -> bool:
        """Read the lease without competing for it (caller does not hold it); True when
        nobody holds a live lease (never created, released, or not renewed for a full lease
        duration as observed locally — the same expiry rule :meth:`try_acquire_or_renew`
        applies)."""
        lease = await self.lock.get()
        now = self.clock()
        if lease is None:
            return True
        spec = lease.get("spec") or {}
        record = (spec.get("holderIdentity"), spec.get("renewTime"), spec.get("leaseTransitions"))
        if record != self._observed_record:
            self._observe(spec, now, record)
        holder = spec.get("holderIdentity") or ""
        duration = float(spec.get("leaseDurationSeconds") or self.lease_duration)
        # our own identity on a lease we do not hold any more (renewal timed out): ours to retake
        return not holder or holder == self.identity or now >= self._observed_at + duration

    def _observe(self, spec, now, record=None):
        self._observed_record = record
        self._observed_at = now
        holder = spec.get("holderIdentity") or ""
        if holder != self.observed_holder:
            self.transitions_seen += 1
        self.observed_holder = holder

    async def _release(self) -> None:
        lease = await self.lock.get()
        if lease is None or (lease.get("spec") or {}).get("holderIdentity") != self.identity:
            return
        spec = dict(lease.get("spec") or {})
        spec.update(holderIdentity="", leaseDurationSeconds=1, renewTime=_micro(), acquireTime=_micro())
        try:
            await self.lock.update(lease, spec)
        except Conflict:
            pass

    async def _run(self) -> None:
        while True:
            if not self.leader:
                try:
                    ok, t0 = await self.acquire_or_renew_bounded(self.renew_deadline)
                except Exception as exc:  # noqa: BLE001 - API errors / timeouts: keep trying
                    log.warning("leader election: acquire failed: %r", exc)
                    ok = False
                if ok:
                    self._renewed(t0)
                    if self.clock() < self.valid_until:
                        self._set_leader(True)
                        continue
                await asyncio.sleep(self.retry_period)
                continue
            # leading: renew every retry_period; every attempt is bounded by the time left on
            # the current hold, and the hold ends at valid_until whatever the API does
            left = self.valid_until - self.clock()
            await asyncio.sleep(max(0.0, min(self.retry_period, left)))
            try:
                ok, t0 = await self.acquire_or_renew_bounded(self.valid_until - self.clock())
            except Exception as exc:  # noqa: BLE001 - incl. the wait_for timeout at valid_until
                log.warning("leader election: renew failed: %r", exc)
                ok = False
            if ok:
                self._renewed(t0)
            elif self.observed_holder and self.observed_holder != self.identity:
                self.valid_until = float("-inf")  # somebody else holds it now: step down at once
            if self.clock() >= self.valid_until:
                if self.metrics is not None:
                    self.metrics.inc("lease_expired_locally")
                self._set_leader(False)
