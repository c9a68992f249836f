"""Replica sharding (``parallel/sharding.py``) and per-shard leases (``ha/shards.py``).

Horizontal scale that can actually be deployed with HA —
one Lease per shard, a dead owner's shard moves within the lease duration, and no
run is lost or written twice.  The reference scales by running more replicas that
all process everything (``/root/reference/.helm/values.yaml:124-125``)."""
import asyncio
import collections
import json
import time

from nexus_supervisor_amd import _kube_native
from nexus_supervisor_amd.app import Application
from nexus_supervisor_amd.bench.workload import Workload
from nexus_supervisor_amd.config import load_config
from nexus_supervisor_amd.kube.client import KubeClient, KubeConfig
from nexus_supervisor_amd.parallel.pipeline import PipelineStage
from nexus_supervisor_amd.parallel.sharding import SHARD_SEED, ShardSet, shard_of
from nexus_supervisor_amd.parallel.workers import _SEED
from nexus_supervisor_amd.store.memory import MemoryStore
from nexus_supervisor_amd.testing.fake_apiserver import FakeApiServer
from conftest import TIME_SCALE

LABEL = "batch.kubernetes.io/job-name"


def _ids(n_per_shard, shards=2):
    out = collections.defaultdict(list)
    i = 0
    while any(len(out[k]) < n_per_shard for k in range(shards)):
        rid = f"run-{i:05d}"
        i += 1
        k = shard_of(rid, shards)
        if len(out[k]) < n_per_shard:
            out[k].append(rid)
    return out


def _line(etype, obj):
    return (json.dumps({"type": etype, "object": obj}) + "\n").encode()


def test_shard_set_epochs_and_hash():
    s = ShardSet(4, [1, 2])
    rid = next(r for r in (f"x{i}" for i in range(100)) if shard_of(r, 4) == 2)
    assert s.owns(rid) and s.token(rid) == 0
    gained, lost = s.update([0, 1])
    assert gained == {0} and lost == {2}
    assert not s.owns(rid) and s.token(rid) == 1  # a decision holding token 0 is fenced
    assert ShardSet(1).owns("anything") and not ShardSet(1).enabled
    assert all(0 <= shard_of(f"r{i}", 3) < 3 for i in range(50))


def test_native_router_drops_other_replicas_runs_before_decode():
    ids = _ids(3)
    router = _kube_native.ShardRouter(0, 2, _SEED, LABEL)
    router.set_replica(2, SHARD_SEED, [0])
    jobs = _kube_native.WatchSplitter(router, "job")
    pods = _kube_native.WatchSplitter(router, "pod")
    events = _kube_native.WatchSplitter(router, "event")
    body = b"".join(_line("ADDED", {"kind": "Job", "metadata": {"name": r, "resourceVersion": "1"}})
                    for k in (0, 1) for r in ids[k])
    outs, _rv, errors = jobs.feed(body)
    text = b"".join(outs).decode()
    assert not errors
    assert all(r in text for r in ids[0]) and not any(r in text for r in ids[1])
    # each owned run goes to exactly one worker (the in-replica placement)
    for r in ids[0]:
        assert sum(r.encode() in o for o in outs) == 1
    pod_body = b"".join(_line("ADDED", {"kind": "Pod", "metadata": {"name": f"{r}-w0", "resourceVersion": "2",
                                                                   "labels": {LABEL: r}}})
                        for k in (0, 1) for r in ids[k])
    outs, _rv, _e = pods.feed(pod_body)
    assert not any(r.encode() in b"".join(outs) for r in ids[1])
    foreign_pod = f"{ids[1][0]}-w0"
    assert router.pod_owner(foreign_pod) == -2
    # a Pod Event follows its pod's owner: another replica's pod → dropped everywhere
    ev = {"kind": "Event", "metadata": {"name": "e1", "resourceVersion": "3"},
          "involvedObject": {"kind": "Pod", "name": foreign_pod}, "reason": "OOMKilling"}
    outs, _rv, _e = events.feed(_line("ADDED", ev))
    assert not any(outs)
    # unknown pod: every worker parks it until the pod shows up
    ev2 = dict(ev, involvedObject={"kind": "Pod", "name": "never-seen"})
    outs, _rv, _e = events.feed(_line("ADDED", ev2))
    assert all(outs)
    assert router.stats["foreign"] >= 5
    # gaining the shard re-evaluates what the router already knows about its pods
    router.set_replica(2, SHARD_SEED, [0, 1])
    assert router.pod_owner(foreign_pod) in (0, 1)
    outs, _rv, _e = events.feed(_line("ADDED", ev))
    assert sum(bool(o) for o in outs) == 1
    # LIST bodies are split the same way
    router.set_replica(2, SHARD_SEED, [1])
    listing = json.dumps({"metadata": {"resourceVersion": "9"}, "items": [
        {"kind": "Job", "metadata": {"name": r}} for k in (0, 1) for r in ids[k]]}).encode()
    rv, parts = jobs.split_list(listing)
    items = [it["metadata"]["name"] for p in parts for it in json.loads(p)]
    assert rv == "9" and sorted(items) == sorted(ids[1])


def test_pipeline_clear_with_predicate_keeps_other_keys(arun):
    async def go():
        done = []
        release = asyncio.Event()

        async def proc(item):
            await release.wait()
            done.append(item)

        p = PipelineStage("t", proc, workers=1, elements_per_second=0, burst=10, key_fn=lambda x: x)
        await p.start()
        for k in ("a", "b", "c", "d"):
            p.receive(k)
        await asyncio.sleep(0.01)  # "a" is running, the rest queued
        dropped = p.clear(lambda key: key in ("b", "d"))
        assert dropped == 2
        p.receive("b")  # re-received after the drop: queued once
        release.set()
        assert await p.join(2)
        assert sorted(done) == ["a", "b", "c"] and done.count("b") == 1
        await p.stop()

    arun(go())


def _cfg(ident, extra=None):
    over = {"cql-store-type": "memory", "workers": 8, "rate-limit-elements-per-second": 0, "resync-period": "0s",
            "rules": {"stale-event-grace": "2s"},
            "leader-election": {"identity": ident, "lease-duration": _ms(800), "renew-deadline": _ms(500),
                                "retry-period": _ms(100)}}
    over.update(extra or {})
    return load_config(path=None, env={}, overrides=over)


def _ms(v: float) -> str:
    return f"{int(v * TIME_SCALE)}ms"


async def _wait(pred, timeout):
    deadline = time.monotonic() + timeout * TIME_SCALE
    while time.monotonic() < deadline:
        if pred():
            return True
        await asyncio.sleep(0.05)
    return pred()


def _push(api, wl, store, n, expected):
    failed, traffic, rows = wl.step(n)
    for r in rows:
        store.rows[r.key] = r.deep_copy()
    for etype, obj in traffic:
        api.apply(etype, obj)
    for rid in failed:
        expected[rid] = wl.expected[rid]


def _check_exactly_once(store, wl, expected):
    stages = {rid: store.get(wl.algorithm, rid).lifecycle_stage for rid in expected}
    wrong = {rid: (s, expected[rid]) for rid, s in stages.items() if s != expected[rid]}
    # each failure written once; a run started before it failed also has its RUNNING write
    # (one at most: the Started Event's and the pod's Running transition are one decision)
    writes = collections.Counter(key[1] for key, stage in store.write_log if stage != "RUNNING")
    running = collections.Counter(key[1] for key, stage in store.write_log if stage == "RUNNING")
    twice = {rid: writes[rid] for rid in expected if writes[rid] != 1}
    twice.update({rid: ("RUNNING", n) for rid, n in running.items() if n > 1})
    return wrong, twice


def test_static_shards_split_the_namespace_and_write_each_run_once(arun):
    """Two replicas with ``sharding.shards: 2`` over one namespace: each caches and decides
    only its own half (ingest filter), and every failed run is written exactly once."""
    async def go():
        api = FakeApiServer(bookmark_interval=0.1)
        url = await api.start()
        wl = Workload(concurrent_jobs=120, seed=3)
        objs, rows = wl.initial()
        store = MemoryStore(rows)
        for o in objs:
            api.create(o)
        apps = []
        for i in range(2):
            cfg = _cfg(f"s{i}", {"sharding": {"shards": 2, "shard-index": i}})
            app = Application(cfg, kube=KubeClient(KubeConfig(url)), store=store)
            await app.start()
            apps.append(app)
        for a in apps:
            assert await a.wait_for_cache_sync(10)
        jobs = [len(a.supervisor.job_informer.indexer) for a in apps]
        assert sum(jobs) == 120 and all(j > 20 for j in jobs), jobs
        expected = {}
        _push(api, wl, store, 60, expected)
        assert await _wait(lambda: not _check_exactly_once(store, wl, expected)[0], 15)
        await asyncio.sleep(0.3)  # late duplicates would land now
        wrong, twice = _check_exactly_once(store, wl, expected)
        assert not wrong and not twice, (wrong, twice)
        for a in apps:
            await a.stop(drain_timeout=1)
        await api.stop()

    arun(go(), timeout=60)


def test_shard_leases_fail_over_individually_without_loss_or_double_writes(arun):
    """Three replicas, two shards (fair share 1 each, one standby).  Killing a shard owner
    (no lease release) moves exactly that shard to the standby within the lease duration;
    runs failing during the gap are decided by the new owner; nothing is written twice."""
    async def go():
        api = FakeApiServer(bookmark_interval=0.1)
        url = await api.start()
        wl = Workload(concurrent_jobs=200, seed=11)
        objs, rows = wl.initial()
        store = MemoryStore(rows)
        for o in objs:
            api.create(o)
        apps = {}
        for ident in ("rep-a", "rep-b", "rep-c"):
            cfg = _cfg(ident, {"sharding": {"shards": 2, "mode": "lease", "replicas": 3}})
            app = Application(cfg, kube=KubeClient(KubeConfig(url)), store=store)
            await app.start()
            apps[ident] = app

        def owners():
            return {k: [i for i, a in apps.items() if k in a.shard_leases.owned] for k in (0, 1)}

        assert await _wait(lambda: all(len(v) == 1 for v in owners().values()), 5), owners()
        own = owners()
        assert own[0] != own[1]  # fair share: one shard each, the third replica stands by
        standby = next(i for i in apps if i not in own[0] + own[1])
        expected = {}
        _push(api, wl, store, 40, expected)
        assert await _wait(lambda: not _check_exactly_once(store, wl, expected)[0], 15)
        # the owner of shard 1 dies holding its lease
        victim_id = own[1][0]
        victim = apps.pop(victim_id)
        await victim.shard_leases.stop(release=False)
        await victim.stop(drain_timeout=0.2)
        t0 = time.monotonic()
        _push(api, wl, store, 40, expected)  # failures of both shards during the gap
        assert await _wait(lambda: owners()[1] == [standby], 5), owners()
        took = time.monotonic() - t0
        # lease duration (0.8 s) + up to two retry periods of observation
        assert took < (0.8 + 0.5) * TIME_SCALE, took
        assert owners()[0] == own[0]  # the surviving owner kept its shard throughout
        assert await _wait(lambda: not _check_exactly_once(store, wl, expected)[0], 15)
        await asyncio.sleep(0.3)
        wrong, twice = _check_exactly_once(store, wl, expected)
        assert not wrong and not twice, (wrong, twice)
        lease = api.get("Lease", "nexus", "nexus-supervisor-leader-shard-1")
        assert lease["spec"]["holderIdentity"] == standby
        for a in apps.values():
            await a.stop(drain_timeout=1)
        await api.stop()

    arun(go(), timeout=60)


def test_last_survivor_takes_orphaned_shards(arun):
    """With the fair share at one shard, a lone survivor still takes a shard nobody renews
    for a full lease duration (orphaned), so the namespace is never left uncovered."""
    async def go():
        api = FakeApiServer(bookmark_interval=0.1)
        url = await api.start()
        wl = Workload(concurrent_jobs=60, seed=5)
        objs, rows = wl.initial()
        store = MemoryStore(rows)
        for o in objs:
            api.create(o)
        cfg = _cfg("lonely", {"sharding": {"shards": 2, "mode": "lease", "replicas": 2}})
        app = Application(cfg, kube=KubeClient(KubeConfig(url)), store=store)
        await app.start()
        assert await _wait(lambda: len(app.shard_leases.owned) == 1, 3)
        assert await _wait(lambda: len(app.shard_leases.owned) == 2, 4)  # after a lease duration
        expected = {}
        _push(api, wl, store, 30, expected)
        assert await _wait(lambda: not _check_exactly_once(store, wl, expected)[0], 15)
        await app.stop(drain_timeout=1)
        # released on shutdown
        for k in (0, 1):
            assert api.get("Lease", "nexus", f"nexus-supervisor-leader-shard-{k}")["spec"]["holderIdentity"] == ""
        await api.stop()

    arun(go(), timeout=60)


def test_late_replica_gets_its_share_back_by_rebalancing(arun):
    """Six shards, three replicas configured, only two running: after a lease duration they
    cover the orphaned shards (3 + 3 or 2 + 4).  When the third replica joins (its membership Lease
    appears), the richest replica fences and hands back one shard per round until every
    replica holds its share of 2 — failures pushed throughout are written exactly once."""
    async def go():
        api = FakeApiServer(bookmark_interval=0.1)
        url = await api.start()
        wl = Workload(concurrent_jobs=300, seed=23)
        objs, rows = wl.initial()
        store = MemoryStore(rows)
        for o in objs:
            api.create(o)
        sharding = {"sharding": {"shards": 6, "mode": "lease", "replicas": 3}}
        apps = {}

        async def start(ident):
            app = Application(_cfg(ident, sharding), kube=KubeClient(KubeConfig(url)), store=store)
            await app.start()
            apps[ident] = app

        def counts():
            return sorted(len(a.shard_leases.owned) for a in apps.values())

        def covered():
            held = [k for a in apps.values() for k in a.shard_leases.owned]
            return sorted(held) == list(range(6))

        await start("rep-a")
        await start("rep-b")
        assert await _wait(lambda: covered() and counts() in ([3, 3], [2, 4]), 6), counts()
        expected = {}
        _push(api, wl, store, 40, expected)
        await start("rep-c")
        _push(api, wl, store, 40, expected)  # during the hand-over
        assert await _wait(lambda: covered() and counts() == [2, 2, 2], 10), counts()
        _push(api, wl, store, 40, expected)
        assert await _wait(lambda: not _check_exactly_once(store, wl, expected)[0], 15)
        await asyncio.sleep(0.3)
        wrong, twice = _check_exactly_once(store, wl, expected)
        assert not wrong and not twice, (wrong, twice)
        # 3+3 → 2+2+2 or 4+2 → 2+2+2: two hand-backs; one when a slow round (a loaded CI box,
        # the coverage tracer) let a lease lapse and the newcomer took that shard unheld
        assert 1 <= sum(a.shard_leases.rebalances for a in apps.values()) <= 2
        assert all(a.shard_leases.members == frozenset(apps) for a in apps.values())
        for a in apps.values():
            await a.stop(drain_timeout=1)
        for ident in apps:  # membership Leases deleted on shutdown
            assert api.get("Lease", "nexus", f"nexus-supervisor-leader-member-{ident}") is None
        await api.stop()

    arun(go(), timeout=90)


def test_member_lease_names_are_dns_safe():
    from nexus_supervisor_amd.ha.shards import member_lease_name

    assert member_lease_name("nexus-supervisor-leader", "Pod_Name.x") == "nexus-supervisor-leader-member-pod-name.x"
    long = member_lease_name("base", "x" * 400)
    assert len(long) <= 253 and long.startswith("base-member-")


def test_shard_leases_with_worker_processes_and_watch_hub(arun, tmp_path):
    """Lease mode on process-per-core replicas: the parent holds the shard leases, its
    watch hub drops the other replica's runs before decode, and when the other replica
    dies the survivor's hub re-lists and its workers decide the orphaned shard's runs."""
    from nexus_supervisor_amd.app import ShardedApplication
    from nexus_supervisor_amd.bench.wire import schema_statements
    from nexus_supervisor_amd.store.cql import CqlCheckpointStore, CqlSession
    from nexus_supervisor_amd.testing.cqlsrv import CqlServer

    srv = CqlServer(exec_statements=schema_statements()).start()

    async def go():
        api = FakeApiServer(bookmark_interval=0.1)
        url = await api.start()
        kc = tmp_path / "kubeconfig"
        kc.write_text(json.dumps({"clusters": [{"name": "c", "cluster": {"server": url}}],
                                  "contexts": [{"name": "x", "context": {"cluster": "c"}}], "current-context": "x"}))
        wl = Workload(concurrent_jobs=120, seed=21)
        objs, rows = wl.initial()
        st = CqlCheckpointStore(CqlSession([srv.address]))
        await st.connect()
        await st.upsert_many(rows)
        for o in objs:
            api.create(o)
        apps = {}
        try:
            for ident in ("hub-a", "hub-b"):
                cfg = _cfg(ident, {"cql-store-type": "scylla", "kube-config-path": str(kc),
                                   "scylla-cql-store": {"hosts": f"127.0.0.1:{srv.port}"},
                                   "runtime": {"worker-processes": 2},
                                   "sharding": {"shards": 2, "mode": "lease", "replicas": 2},
                                   # leases long enough that a loaded host (the worker processes
                                   # and xdist peers) does not lapse them mid-test: each lapse
                                   # re-lists both hubs and the runs wait on the new owner
                                   "leader-election": {"identity": ident, "lease-duration": _ms(2400),
                                                       "renew-deadline": _ms(1600), "retry-period": _ms(200)}})
                app = ShardedApplication(cfg)
                await app.start()
                apps[ident] = app
            for a in apps.values():
                assert await a.wait_for_cache_sync(30)
            assert await _wait(lambda: sorted(k for a in apps.values() for k in a.shards.owned or ()) == [0, 1], 5)
            expected = {}

            async def decided():
                got = {}
                for rid, stage in expected.items():
                    row = await st.read_checkpoint(wl.algorithm, rid)
                    got[rid] = row.lifecycle_stage if row else None
                return {r: (g, expected[r]) for r, g in got.items() if g != expected[r]}

            async def wait_decided(timeout):
                deadline = time.monotonic() + timeout
                bad = await decided()
                while bad and time.monotonic() < deadline:
                    await asyncio.sleep(0.1)
                    bad = await decided()
                return bad

            async def push(n):
                failed, traffic, new_rows = wl.step(n)
                await st.upsert_many(new_rows)
                for etype, obj in traffic:
                    api.apply(etype, obj)
                for rid in failed:
                    expected[rid] = wl.expected[rid]

            await push(30)
            assert not await wait_decided(20)
            # each hub routed only its own shard's runs to its workers
            for a in apps.values():
                assert a.hub.router.stats["foreign"] > 0
            victim = apps.pop("hub-a")
            survivor = apps["hub-b"]
            await victim.shard_leases.stop(release=False)
            await victim.stop(drain_timeout=0.5)
            await push(30)
            assert await _wait(lambda: survivor.shards.owned == {0, 1}, 6), survivor.shards.owned
            bad = await wait_decided(30)
            assert not bad, list(bad.items())[:3]
        finally:
            for a in apps.values():
                await a.stop(drain_timeout=1)
            await st.close()
            await api.stop()

    try:
        arun(go(), timeout=120)
    finally:
        srv.stop()


def test_replica_shard_is_independent_of_worker_placement():
    """CRC32 is affine in its seed: the replica hash must not correlate with the worker
    placement inside a replica, or one worker would get all of a replica's runs."""
    import random
    import zlib

    rng = random.Random(1)
    counts = collections.Counter()
    for _ in range(4000):
        rid = "%08x-%04x-4%03x-8%03x-%012x" % (rng.getrandbits(32), rng.getrandbits(16), rng.getrandbits(12),
                                              rng.getrandbits(12), rng.getrandbits(48))
        counts[(shard_of(rid, 2), zlib.crc32(rid.encode(), _SEED) % 2)] += 1
    assert len(counts) == 4 and min(counts.values()) > 800, counts
    # the native router agrees with the Python hash
    router = _kube_native.ShardRouter(0, 1, _SEED, LABEL)
    router.set_replica(3, SHARD_SEED, [1])
    split = _kube_native.WatchSplitter(router, "job")
    ids = [f"job-{i}" for i in range(60)]
    outs, _rv, _e = split.feed(b"".join(_line("ADDED", {"metadata": {"name": r}}) for r in ids))
    kept = {json.loads(x)["object"]["metadata"]["name"] for x in outs[0].splitlines()}
    assert kept == {r for r in ids if shard_of(r, 3) == 1}


def test_membership_list_failure_falls_back_to_configured_share(arun):
    """Without `list` on leases (an upgraded deployment whose RBAC lags), the fair share
    stays ``ceil(shards / sharding.replicas)`` and nothing is rebalanced away."""
    from nexus_supervisor_amd.ha.shards import ShardLeaseManager
    from nexus_supervisor_amd.kube.errors import ApiError

    class NoList:
        def __init__(self):
            self.leases = {}

        async def get(self, kind, ns, name):
            from nexus_supervisor_amd.kube.errors import NotFound
            if name not in self.leases:
                raise NotFound(404, "NotFound", name)
            return self.leases[name]

        async def create(self, kind, ns, body):
            self.leases[body["metadata"]["name"]] = dict(body, metadata=dict(body["metadata"], resourceVersion="1"))
            return self.leases[body["metadata"]["name"]]

        async def replace(self, kind, ns, name, body):
            self.leases[name] = body
            return body

        async def list(self, *a, **kw):
            raise ApiError(403, "Forbidden", "leases is forbidden: cannot list")

    async def go():
        m = ShardLeaseManager(NoList(), "nexus", "lease", "solo", 4, replicas=2, lease_duration=0.8,
                              renew_deadline=0.5, retry_period=0.1)
        await m.tick()
        assert m.target == 2 and len(m.owned) == 2 and m.members == frozenset({"solo"})
        await m.tick()
        assert len(m.owned) == 2 and m.rebalances == 0

    arun(go())


def test_stale_membership_leases_are_garbage_collected(arun):
    """A replica killed without a clean shutdown leaves its membership Lease; after ten
    lease durations without a renewal a live replica deletes it (one Lease per pod ever
    started would otherwise pile up across rollouts), and never deletes a live one."""
    from nexus_supervisor_amd.ha.shards import ShardLeaseManager

    async def go():
        api = FakeApiServer(bookmark_interval=0.1)
        url = await api.start()
        kw = dict(replicas=2, lease_duration=0.2, renew_deadline=0.15, retry_period=0.05)
        dead = ShardLeaseManager(KubeClient(KubeConfig(url)), "nexus", "grp", "dead-pod", 2, **kw)
        await dead.tick()  # registers, then dies without releasing anything
        live = ShardLeaseManager(KubeClient(KubeConfig(url)), "nexus", "grp", "live-pod", 2, **kw)
        other = ShardLeaseManager(KubeClient(KubeConfig(url)), "nexus", "grp", "other-pod", 2, **kw)
        live.start()
        other.start()
        assert api.get("Lease", "nexus", "grp-member-dead-pod") is not None
        assert await _wait(lambda: api.get("Lease", "nexus", "grp-member-dead-pod") is None, 6)
        assert await _wait(lambda: live.stale_members_deleted + other.stale_members_deleted >= 1, 2)
        assert live.stale_members_deleted + other.stale_members_deleted == 1
        assert api.get("Lease", "nexus", "grp-member-live-pod") is not None
        assert live.members == frozenset({"live-pod", "other-pod"})
        await live.stop()
        await other.stop()
        assert api.get("Lease", "nexus", "grp-member-live-pod") is None
        await api.stop()

    arun(go(), timeout=30)


class _Tagged:
    """Per-replica view of the shared store / Job client recording when each write and
    DELETE was *issued* (monotonic) and by whom."""

    def __init__(self, inner, ident, log):
        self.inner, self.ident, self.log = inner, ident, log

    def __getattr__(self, name):
        return getattr(self.inner, name)

    async def cas_update(self, algorithm, request_id, *a, **kw):
        self.log.append((time.monotonic(), self.ident, "write", request_id))
        return await self.inner.cas_update(algorithm, request_id, *a, **kw)

    async def update_status(self, algorithm, request_id, *a, **kw):
        self.log.append((time.monotonic(), self.ident, "write", request_id))
        return await self.inner.update_status(algorithm, request_id, *a, **kw)

    async def delete_job(self, namespace, name, propagation_policy="Background"):
        self.log.append((time.monotonic(), self.ident, "delete", name))
        return await self.inner.delete_job(namespace, name, propagation_policy)


def test_partitioned_shard_owner_stops_acting_before_anyone_takes_over(arun):
    """Replica A is cut off from the apiserver (every request
    stalls) while it still has a backlog of decisions for its shard.  Its hold lapses
    ``renew-deadline`` after its last renewal started: A issues no write and no Job DELETE
    after that, B acquires the shard only later (a lease duration after it last saw A
    renew), finishes the runs, and no run is written twice."""
    from nexus_supervisor_amd.testing.netproxy import PausableProxy

    async def go():
        api = FakeApiServer(bookmark_interval=0.1)
        url = await api.start()
        host, port = url.rsplit(":", 1)
        proxy = PausableProxy(host.split("//")[1], int(port))
        purl = await proxy.start()
        wl = Workload(concurrent_jobs=400, seed=31)
        objs, rows = wl.initial()
        store = MemoryStore(rows, latency=0.03 * TIME_SCALE)  # a slow store: A keeps a backlog past its hold
        for o in objs:
            api.create(o)
        events = []
        apps = {}
        # twice the production ratios' minimum: a loaded CI box (the suite under xdist) must not
        # turn a scheduling delay into a lapsed hold
        lease = {"lease-duration": _ms(2400), "renew-deadline": _ms(1600), "retry-period": _ms(300)}
        for ident, u in (("rep-a", purl), ("rep-b", url)):
            cfg = _cfg(ident, {"workers": 2, "sharding": {"shards": 2, "mode": "lease", "replicas": 2},
                               "leader-election": dict(lease, identity=ident)})
            kc = KubeClient(KubeConfig(u))
            app = Application(cfg, kube=kc, store=_Tagged(store, ident, events), jobs=_Tagged(kc, ident, events))
            await app.start()
            apps[ident] = app
        a, b = apps["rep-a"], apps["rep-b"]
        assert await _wait(lambda: len(a.shard_leases.owned) == 1 and len(b.shard_leases.owned) == 1, 6)
        ka = next(iter(a.shard_leases.owned))
        expected = {}
        failed, traffic, new_rows = wl.step(300)
        for r in new_rows:
            store.rows[r.key] = r.deep_copy()
        for etype, obj in traffic:
            api.apply(etype, obj)
        for rid in failed:
            expected[rid] = wl.expected[rid]
        mine = [rid for rid in failed if shard_of(rid, 2) == ka]
        # A has received (most of) its shard's failures and is working through them
        assert await _wait(lambda: a.supervisor.pipeline.depth() >= 20, 5), a.supervisor.pipeline.depth()
        t_cut = time.monotonic()
        proxy.pause()
        hold_end = a.shard_leases.valid_until(ka)
        assert hold_end <= t_cut + 1.6 * TIME_SCALE + 0.01
        assert await _wait(lambda: ka in b.shard_leases.owned, 10), "B never took A's shard"
        t_b = time.monotonic()
        assert await _wait(lambda: not _check_exactly_once(store, wl, expected)[0], 20)
        a_acts = [t for t, who, _kind, rid in events if who == "rep-a" and shard_of(rid, 2) == ka]
        assert a_acts and max(a_acts) < hold_end, (max(a_acts) - hold_end)
        assert max(a_acts) < t_b
        b_acts = [t for t, who, _kind, rid in events if who == "rep-b" and shard_of(rid, 2) == ka]
        assert b_acts and min(b_acts) > hold_end
        assert a.shard_leases.expired_locally >= 1 and ka not in a.supervisor.shards.owned
        wrong, twice = _check_exactly_once(store, wl, expected)
        assert not wrong and not twice, (wrong, twice)
        assert len(mine) > 20
        proxy.resume()
        for x in apps.values():
            await x.stop(drain_timeout=1)
        await proxy.stop()
        await api.stop()

    arun(go(), timeout=90)


def test_single_shard_lease_mode_gates_the_whole_namespace(arun):
    """``mode: lease`` with one shard is one Lease for the
    namespace — a replica that loses the race for it acts on nothing (it used to own
    "every shard" and run with leader election silently off)."""
    async def go():
        api = FakeApiServer(bookmark_interval=0.1)
        url = await api.start()
        wl = Workload(concurrent_jobs=60, seed=9)
        objs, rows = wl.initial()
        store = MemoryStore(rows)
        for o in objs:
            api.create(o)
        events = []
        apps = []
        for ident in ("solo-a", "solo-b"):
            cfg = _cfg(ident, {"sharding": {"shards": 1, "mode": "lease"}})
            kc = KubeClient(KubeConfig(url))
            app = Application(cfg, kube=kc, store=_Tagged(store, ident, events))
            await app.start()
            apps.append(app)
        assert await _wait(lambda: sum(len(x.shard_leases.owned) for x in apps) == 1, 5)
        assert not any(not x.supervisor.shards.owned and x.supervisor.shards.owns("anything") for x in apps)
        holder = next(x for x in apps if x.shard_leases.owned)
        expected = {}
        _push(api, wl, store, 30, expected)
        assert await _wait(lambda: not _check_exactly_once(store, wl, expected)[0], 10)
        writers = {who for _t, who, _k, _r in events}
        assert writers == {holder.cfg.leader_election.identity}, writers
        for x in apps:
            await x.stop(drain_timeout=1)
        await api.stop()

    arun(go(), timeout=60)
