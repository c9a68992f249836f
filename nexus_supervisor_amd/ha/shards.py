"""Per-shard Lease ownership (``sharding.mode: lease``).

The reference scales out by running more replicas that all do all the work
(``/root/reference/.helm/values.yaml:124-125``); a single leader lease (``leader.py``)
makes that safe but leaves every replica but one idle.  Here the runs are split into
``sharding.shards`` shards (``parallel/sharding.py``) and each shard has its own
``coordination.k8s.io/v1`` Lease, ``<lease-name>-shard-<k>``:

* a replica renews the shard leases it holds every ``retry-period``; a shard whose
  renewal has not succeeded for ``renew-deadline`` is dropped (fenced) before anybody
  else can take it (``lease-duration`` > ``renew-deadline``, as in client-go);
* it competes for free shards (never created, released, or expired as observed
  locally) while it holds fewer than its fair share ``ceil(shards / replicas)``
  (``sharding.replicas``, the Helm replica count; 0 = take everything);
* a shard whose lease *expired* under a holder (that replica crashed) is taken by anyone
  after a short grace (two retry periods, so replicas below their share win the race),
  and a shard *never held or released* after a full ``lease-duration`` — so N−1 survivors
  cover all shards, a crash costs about one lease duration, and a cold start or rolling
  restart still spreads the shards before anyone exceeds its share;
* candidates walk the shards in an order rotated by their identity hash, so replicas
  starting together rarely collide on the same lease (a collision is a 409 anyway);
* on shutdown the held leases are released so survivors take over within a retry
  period instead of a lease duration.

Changes of the held set are reported through ``on_change(frozenset)``: the replica
fences lost shards and replays gained ones (``Supervisor.set_shards``).
"""
from __future__ import annotations

import asyncio
import logging
import time
import zlib
from typing import Callable, Dict, FrozenSet, List, Optional

from .leader import LeaderElector, LeaseLock

log = logging.getLogger("nexus_supervisor_amd.shards")


def shard_lease_name(base: str, k: int) -> str:
    return f"{base}-shard-{k}"


class ShardLeaseManager:
    def __init__(self, client, namespace: str, base_name: str, identity: str, shards: int, *,
                 replicas: int = 0, lease_duration: float = 15.0, renew_deadline: float = 10.0,
                 retry_period: float = 2.0, on_change: Optional[Callable[[FrozenSet[int]], None]] = None,
                 metrics=None, clock: Callable[[], float] = time.monotonic):
        if shards < 1:
            raise ValueError("shards must be >= 1")
        self.identity = identity
        self.shards = shards
        self.lease_duration = lease_duration
        self.renew_deadline = renew_deadline
        self.retry_period = retry_period
        self.on_change = on_change
        self.metrics = metrics
        self.clock = clock
        self.target = -(-shards // replicas) if replicas > 0 else shards
        self.electors: List[LeaderElector] = [
            LeaderElector(LeaseLock(client, namespace, shard_lease_name(base_name, k), identity),
                          lease_duration=lease_duration, renew_deadline=renew_deadline, retry_period=retry_period,
                          clock=clock)
            for k in range(shards)]
        start = zlib.crc32(identity.encode()) % shards
        self.order = [(start + i) % shards for i in range(shards)]
        self.held: Dict[int, float] = {}       # shard → clock of the last successful renewal
        self.free_since: Dict[int, float] = {}  # shard → clock it was first seen free
        self._task: Optional[asyncio.Task] = None
        self.acquisitions = 0

    @property
    def owned(self) -> FrozenSet[int]:
        return frozenset(self.held)

    def start(self) -> asyncio.Task:
        if self._task is None:
            self._task = asyncio.create_task(self._run(), name=f"shard-leases-{self.identity}")
        return self._task

    async def stop(self, release: bool = True) -> None:
        if self._task is not None:
            self._task.cancel()
            try:
                await self._task
            except (asyncio.CancelledError, Exception):
                pass
            self._task = None
        held = sorted(self.held)
        self.held.clear()
        if held:
            self._changed()
        if release:
            for k in held:
                try:
                    await self.electors[k]._release()  # noqa: SLF001 - same package
                except Exception as exc:  # noqa: BLE001
                    log.warning("shard %d lease release failed: %s", k, exc)

    async def _run(self) -> None:
        while True:
            try:
                await self.tick()
            except asyncio.CancelledError:
                raise
            except Exception as exc:  # noqa: BLE001 - API errors: keep going
                log.warning("shard leases: %s", exc)
            await asyncio.sleep(self.retry_period)

    async def tick(self) -> None:
        """One round: renew what is held, then compete for free shards."""
        changed = False
        for k in sorted(self.held):
            try:
                ok = await asyncio.wait_for(self.electors[k].try_acquire_or_renew(), self.renew_deadline)
            except asyncio.CancelledError:
                raise
            except Exception as exc:  # noqa: BLE001
                log.warning("shard %d lease renew failed: %s", k, exc)
                ok = False
            now = self.clock()
            if ok:
                self.held[k] = now
            elif now - self.held[k] >= self.renew_deadline:
                del self.held[k]
                changed = True
                log.info("%s lost shard %d", self.identity, k)
        for k in self.order:
            if k in self.held:
                continue
            e = self.electors[k]
            try:
                free = await e.observe()
            except Exception as exc:  # noqa: BLE001
                log.warning("shard %d lease read failed: %s", k, exc)
                continue
            now = self.clock()
            if not free:
                self.free_since.pop(k, None)
                continue
            since = self.free_since.setdefault(k, now)
            # expired under a holder (crash): short grace; never held / released: a lease duration
            grace = 2 * self.retry_period if e.observed_holder and e.observed_holder != self.identity \
                else self.lease_duration
            orphaned = now - since >= grace
            if len(self.held) >= self.target and not orphaned:
                continue
            try:
                ok = await e.try_acquire_or_renew()
            except Exception as exc:  # noqa: BLE001
                log.warning("shard %d lease acquire failed: %s", k, exc)
                ok = False
            if ok:
                self.held[k] = self.clock()
                self.free_since.pop(k, None)
                self.acquisitions += 1
                changed = True
                log.info("%s acquired shard %d%s", self.identity, k, " (orphaned)" if orphaned else "")
        if changed:
            self._changed()

    def _changed(self) -> None:
        if self.metrics is not None:
            self.metrics.set("shard_leases_held", float(len(self.held)))
            self.metrics.inc("shard_lease_changes")
        if self.on_change is not None:
            try:
                self.on_change(self.owned)
            except Exception:  # pragma: no cover
                log.exception("shard ownership callback failed")
