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

Ownership is time-bounded, so a replica never acts on a shard it may have lost: a shard
renewal that *started* at ``t0`` and succeeded is good until ``t0 + renew-deadline``;
every API call (membership, renewals, observations, acquisitions) runs under a
``wait_for`` bounded by the time it may take, held shards are renewed concurrently, and
a watchdog task drops a shard the moment its hold lapses — whatever the apiserver is
doing — so a partitioned replica stops acting on a shard strictly before any other
replica can take it (``lease-duration`` after observing the last renewal).  The hold
deadlines are published through ``on_renewed({shard: valid_until})`` so the supervisor
(and its worker processes) check them before every write and Job DELETE.
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
                 metrics=None, clock: Callable[[], float] = time.monotonic,
                 on_renewed: Optional[Callable[[Dict[int, float]], None]] = None):
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
        self.on_renewed = on_renewed
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
        self.held: Dict[int, float] = {}       # shard → clock the last successful renewal STARTED
        self.free_since: Dict[int, float] = {}  # shard → clock it was first seen free
        self._task: Optional[asyncio.Task] = None
        self._watchdog: Optional[asyncio.Task] = None
        self._wake: Optional[asyncio.Event] = None
        self.acquisitions = 0
        self.expired_locally = 0
        self._gc: Dict[str, asyncio.Future] = {}  # stale membership Lease deletes in flight

    def valid_until(self, k: int) -> float:
        t = self.held.get(k)
        return float("-inf") if t is None else t + self.renew_deadline

    def deadlines(self) -> Dict[int, float]:
        return {k: t + self.renew_deadline for k, t in self.held.items()}

    def _publish_deadlines(self) -> None:
        if self.on_renewed is not None and self.held:
            try:
                self.on_renewed(self.deadlines())
            except Exception:  # pragma: no cover
                log.exception("shard renewal callback failed")

    @property
    def owned(self) -> FrozenSet[int]:
        return frozenset(self.held)

    def start(self) -> asyncio.Task:
        if self._task is None:
            self._wake = asyncio.Event()
            self._task = asyncio.create_task(self._run(), name=f"shard-leases-{self.identity}")
            self._watchdog = asyncio.create_task(self._expire_loop(), name=f"shard-expiry-{self.identity}")
        return self._task

    async def stop(self, release: bool = True) -> None:
        for t in list(self._gc.values()):
            t.cancel()
        for attr in ("_task", "_watchdog"):
            t = getattr(self, attr)
            if t is not None:
                t.cancel()
                try:
                    await t
                except (asyncio.CancelledError, Exception):
                    pass
                setattr(self, attr, None)
        held = sorted(self.held)
        self.held.clear()
        if held:
            self._changed()
        if release:
            for k in held:
                try:
                    await asyncio.wait_for(self.electors[k]._release(), self.renew_deadline)  # noqa: SLF001
                except Exception as exc:  # noqa: BLE001
                    log.warning("shard %d lease release failed: %s", k, exc)
            try:  # a pod name is not reused: its membership Lease goes with it
                await asyncio.wait_for(self.client.delete("Lease", self.namespace, self.member.lock.name),
                                       self.renew_deadline)
            except Exception as exc:  # noqa: BLE001 - e.g. no `delete` verb: leave it released
                log.debug("membership lease delete failed (%s); releasing", exc)
                try:
                    await asyncio.wait_for(self.member._release(), self.renew_deadline)  # noqa: SLF001
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

    async def _expire_loop(self) -> None:
        """Watchdog: drop every shard whose hold lapsed, at the moment it lapses — it does
        not wait for a renewal round (which may be stuck on a slow apiserver)."""
        while True:
            now = self.clock()
            expired = [k for k, t in self.held.items() if now >= t + self.renew_deadline]
            if expired:
                for k in expired:
                    del self.held[k]
                    log.warning("%s: hold on shard %d lapsed (no renewal within renew-deadline): fenced", self.identity, k)
                self.expired_locally += len(expired)
                if self.metrics is not None:
                    self.metrics.inc("shard_leases_expired_locally", len(expired))
                self._changed()
            nxt = min((t + self.renew_deadline for t in self.held.values()), default=now + self.retry_period)
            self._wake.clear()
            try:
                await asyncio.wait_for(self._wake.wait(), max(0.001, min(nxt - now, self.retry_period)))
            except asyncio.TimeoutError:
                pass

    async def _delete_stale(self, name: str) -> None:
        try:
            await self._bounded(self.client.delete("Lease", self.namespace, name), self.lease_duration)
            self.stale_members_deleted += 1
        except Exception as exc:  # noqa: BLE001 - another replica got it first, or no `delete` verb
            log.debug("stale membership lease %s not deleted: %r", name, exc)

    async def _bounded(self, coro, budget: Optional[float] = None):
        return await asyncio.wait_for(coro, self.renew_deadline if budget is None else max(0.001, budget))

    async def _refresh_members(self) -> None:
        """Renew this replica's membership Lease and list the group's: a member is live
        while its ``renewTime`` keeps changing within a lease duration (observed locally,
        as for the shard leases — no cross-node clock comparison).  Each call is bounded by
        ``renew-deadline`` and runs next to (never in front of) the shard renewals."""
        try:
            await self._bounded(self.member.try_acquire_or_renew())
            items, _ = await self._bounded(self.client.list("Lease", self.namespace,
                                                            label_selector=f"{MEMBER_LABEL}={self.base_name}"))
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
            if not name or name == self.member.lock.name or name in self._gc:
                continue
            # housekeeping, not ownership: off the renewal path, bounded by a lease duration
            t = asyncio.ensure_future(self._delete_stale(name))
            self._gc[name] = t
            t.add_done_callback(lambda _t, n=name: self._gc.pop(n, None))
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

    async def _renew(self, k: int) -> Optional[bool]:
        """Renew one held shard within the time left on its hold.  True: renewed (the hold
        now runs from this attempt's start); False: failed; None: dropped meanwhile."""
        t0 = self.clock()
        left = self.valid_until(k) - t0
        try:
            ok = await self._bounded(self.electors[k].try_acquire_or_renew(), left) if left > 0 else False
        except asyncio.CancelledError:
            raise
        except Exception as exc:  # noqa: BLE001 - incl. the wait_for timeout at the hold's end
            log.warning("shard %d lease renew failed: %r", k, exc)
            ok = False
        if k not in self.held:
            return None  # the watchdog fenced it while the call was out: regained by acquisition
        if ok:
            self.held[k] = t0
            return True
        return False

    async def tick(self) -> None:
        """One round: membership (concurrently), renew every held shard (concurrently,
        each bounded by its hold), compete for free shards, rebalance."""
        changed = False
        members = asyncio.ensure_future(self._refresh_members())
        try:
            held = sorted(self.held)
            if held:
                await asyncio.gather(*(self._renew(k) for k in held))
                self._publish_deadlines()
                now = self.clock()
                for k in held:
                    if k in self.held and now >= self.held[k] + self.renew_deadline:
                        del self.held[k]
                        changed = True
                        log.info("%s lost shard %d", self.identity, k)
            await members
        finally:
            if not members.done():
                members.cancel()
        counts: Dict[str, int] = {}
        free_keys = [k for k in self.order if k not in self.held]
        observed = await asyncio.gather(*(self._bounded(self.electors[k].observe()) for k in free_keys),
                                        return_exceptions=True)
        for k, free in zip(free_keys, observed):
            e = self.electors[k]
            if isinstance(free, BaseException):
                if isinstance(free, asyncio.CancelledError):
                    raise free
                log.warning("shard %d lease read failed: %r", k, free)
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
            t0 = self.clock()
            try:
                ok = await self._bounded(e.try_acquire_or_renew())
            except asyncio.CancelledError:
                raise
            except Exception as exc:  # noqa: BLE001
                log.warning("shard %d lease acquire failed: %r", k, exc)
                ok = False
            if ok and self.clock() < t0 + self.renew_deadline:
                self.held[k] = t0
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
                await self._bounded(self.electors[give]._release())  # noqa: SLF001 - same package
            except Exception as exc:  # noqa: BLE001 - expires after a lease duration instead
                log.warning("shard %d lease release failed: %r", give, exc)
        if changed:
            self._changed()
        if self._wake is not None:
            self._wake.set()  # holds moved: let the watchdog re-arm on the new deadlines

    def _changed(self) -> None:
        if self.metrics is not None:
            self.metrics.set("shard_leases_held", float(len(self.held)))
            self.metrics.inc("shard_lease_changes")
        self._publish_deadlines()  # gained shards' holds before the ownership change lands
        if self.on_change is not None:
            try:
                self.on_change(self.owned)
            except Exception:  # pragma: no cover
                log.exception("shard ownership callback failed")
