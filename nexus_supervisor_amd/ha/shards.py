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
  period instead of a lease duration;
* every replica also renews a *membership* Lease (``<lease-name>-member-<identity>``,
  labelled with the group) and lists the group each round: the fair share is computed
  over ``max(sharding.replicas, live members)``, and when a live member holds fewer
  than ``shards // members`` shards the richest replica (ties: highest identity) fences
  and releases one shard per round — so a replica that starts late, or comes back after
  its shards failed over, gets its share back instead of idling until the next restart
  (the taker is below its share and acquires a released shard on its next round).

Changes of the held set are reported through ``on_change(frozenset)``: the replica
fences lost shards and replays gained ones (``Supervisor.set_shards``).
"""
from __future__ import annotations

import asyncio
import logging
import re
import time
import zlib
from typing import Callable, Dict, FrozenSet, List, Optional, Tuple

from .leader import LeaderElector, LeaseLock

log = logging.getLogger("nexus_supervisor_amd.shards")


MEMBER_LABEL = "nexus.sneaksanddata.com/shard-lease-group"
STALE_MEMBER_LEASES = 10  # lease durations without a renewal before a membership Lease is garbage


def shard_lease_name(base: str, k: int) -> str:
    return f"{base}-shard-{k}"


def member_lease_name(base: str, identity: str) -> str:
    """DNS-1123 subdomain name of a replica's membership Lease."""
    ident = re.sub(r"[^a-z0-9.-]+", "-", identity.lower()).strip("-.") or "replica"
    name = f"{base}-member-{ident}"
    if len(name) > 253:
        name = f"{name[:240]}-{zlib.crc32(identity.encode()):08x}"
    return name


class ShardLeaseManager:
    def __init__(self, client, namespace: str, base_name: str, identity: str, shards: int, *,
                 replicas: int = 0, lease_duration: float = 15.0, renew_deadline: float = 10.0,
                 retry_period: float = 2.0, on_change: Optional[Callable[[FrozenSet[int]], None]] = None,
                 metrics=None, clock: Callable[[], float] = time.monotonic):
        if shards < 1:
            raise ValueError("shards must be >= 1")
        self.client = client
        self.namespace = namespace
        self.base_name = base_name
        self.identity = identity
        self.shards = shards
        self.lease_duration = lease_duration
        self.renew_deadline = renew_deadline
        self.retry_period = retry_period
        self.on_change = on_change
        self.metrics = metrics
        self.clock = clock
        self.replicas = replicas
        self.target = -(-shards // replicas) if replicas > 0 else shards
        self.member = LeaderElector(LeaseLock(client, namespace, member_lease_name(base_name, identity), identity,
                                              labels={MEMBER_LABEL: base_name}),
                                    lease_duration=lease_duration, renew_deadline=renew_deadline,
                                    retry_period=retry_period, clock=clock)
        self._seen: Dict[str, Tuple[str, float]] = {}  # member → (last renewTime seen, local clock it changed)
        self.members: FrozenSet[str] = frozenset({identity})
        self.counts: Dict[str, int] = {}  # live holder → shards it holds (as last observed)
        self._last_release = float("-inf")
        self._member_warned = float("-inf")
        self._released: Dict[int, float] = {}  # shard → clock this replica handed it back
        self.rebalances = 0
        self.stale_members_deleted = 0
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
            try:  # a pod name is not reused: its membership Lease goes with it
                await self.client.delete("Lease", self.namespace, self.member.lock.name)
            except Exception as exc:  # noqa: BLE001 - e.g. no `delete` verb: leave it released
                log.debug("membership lease delete failed (%s); releasing", exc)
                try:
                    await self.member._release()  # noqa: SLF001
                except Exception as exc2:  # noqa: BLE001
                    log.warning("membership lease release failed: %s", exc2)

    async def _run(self) -> None:
        while True:
            try:
                await self.tick()
            except asyncio.CancelledError:
                raise
            except Exception as exc:  # noqa: BLE001 - API errors: keep going
                log.warning("shard leases: %s", exc)
            await asyncio.sleep(self.retry_period)

    async def _refresh_members(self) -> None:
        """Renew this replica's membership Lease and list the group's: a member is live
        while its ``renewTime`` keeps changing within a lease duration (observed locally,
        as for the shard leases — no cross-node clock comparison)."""
        try:
            await self.member.try_acquire_or_renew()
            items, _ = await self.client.list("Lease", self.namespace, label_selector=f"{MEMBER_LABEL}={self.base_name}")
        except Exception as exc:  # noqa: BLE001 - keep the last view; the fair share falls back to `replicas`
            # e.g. RBAC without `list` on leases after an upgrade: say so once per lease
            # duration, not every retry period
            now = self.clock()
            if now - self._member_warned >= self.lease_duration:
                self._member_warned = now
                log.warning("shard membership unavailable (fair share from sharding.replicas): %s", exc)
            if self.metrics is not None:
                self.metrics.inc("shard_membership_errors")
            return
        now = self.clock()
        live = {self.identity}
        stale = []
        for it in items:
            spec = it.get("spec") or {}
            holder = spec.get("holderIdentity") or ""
            renew = str(spec.get("renewTime") or "")
            key = holder or (it.get("metadata") or {}).get("name", "")
            prev = self._seen.get(key)
            if prev is None or prev[0] != renew:
                self._seen[key] = (renew, now)
            quiet = now - self._seen[key][1]
            if holder and quiet < self.lease_duration:
                live.add(holder)
            elif holder != self.identity and quiet >= STALE_MEMBER_LEASES * self.lease_duration:
                stale.append((it.get("metadata") or {}).get("name", ""))
        self.members = frozenset(live)
        # a replica killed without a clean shutdown (or a release without delete) leaves its
        # membership Lease behind; one per pod ever started would pile up across rollouts
        for name in stale[:4]:
            if not name or name == self.member.lock.name:
                continue
            try:
                await self.client.delete("Lease", self.namespace, name)
                self.stale_members_deleted += 1
            except Exception as exc:  # noqa: BLE001 - another replica got it first, or no `delete` verb
                log.debug("stale membership lease %s not deleted: %s", name, exc)
        denom = max(self.replicas, len(live))
        self.target = -(-self.shards // denom) if (self.replicas > 0 or len(live) > 1) else self.shards

    def _rebalance_pick(self) -> Optional[int]:
        """A shard to hand back: only when some live member holds fewer than the floor of
        the fair share and this replica is the richest (ties → highest identity), at most
        one per two retry periods so observations catch up between moves."""
        members = self.members
        if len(members) < 2 or not self.held:
            return None
        floor = self.shards // max(self.replicas, len(members))
        counts = {m: self.counts.get(m, 0) for m in members}
        counts[self.identity] = len(self.held)
        if len(self.held) <= floor or not any(c < floor for m, c in counts.items() if m != self.identity):
            return None
        richest = max(counts.items(), key=lambda kv: (kv[1], kv[0]))[0]
        if richest != self.identity or self.clock() - self._last_release < 2 * self.retry_period:
            return None
        return max(self.held, key=self.order.index)  # the shard this replica would take last

    async def tick(self) -> None:
        """One round: membership, renew what is held, compete for free shards, rebalance."""
        changed = False
        await self._refresh_members()
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
        counts: Dict[str, int] = {}
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
                counts[e.observed_holder] = counts.get(e.observed_holder, 0) + 1
                continue
            since = self.free_since.setdefault(k, now)
            # expired under a holder (crash): short grace; never held / released: a lease duration
            grace = 2 * self.retry_period if e.observed_holder and e.observed_holder != self.identity \
                else self.lease_duration
            orphaned = now - since >= grace
            # a shard this replica just handed back is for the member below its share (the
            # releaser itself may dip below the ceiling share): retaken only once orphaned
            given = now - self._released.get(k, float("-inf")) < self.lease_duration
            if (len(self.held) >= self.target or given) and not orphaned:
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
        self.counts = counts
        give = self._rebalance_pick()
        if give is not None:
            # fence first (the supervisor drops the shard's queued work), then hand the lease over
            del self.held[give]
            self._changed()
            changed = False
            self._last_release = self._released[give] = self.clock()
            self.rebalances += 1
            if self.metrics is not None:
                self.metrics.inc("shard_rebalances")
            log.info("%s released shard %d to rebalance (members=%d, share=%d)", self.identity, give,
                     len(self.members), self.target)
            try:
                await self.electors[give]._release()  # noqa: SLF001 - same package
            except Exception as exc:  # noqa: BLE001 - expires after a lease duration instead
                log.warning("shard %d lease release failed: %s", give, exc)
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
