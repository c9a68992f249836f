"""Leader election (BASELINE config 5: 2 replicas, exactly one active, failover
< lease duration, no lost decisions), pprof profiles and the HTTP endpoints."""
import asyncio
import gzip
import json
import time

import aiohttp
import pytest

from nexus_supervisor_amd.app import Application
from nexus_supervisor_amd.config import load_config
from nexus_supervisor_amd.ha.leader import LeaderElector, LeaseLock
from nexus_supervisor_amd.kube.client import KubeClient, KubeConfig
from nexus_supervisor_amd.obs.pprof import Profile, Sampler, decode_profile
from nexus_supervisor_amd.store.memory import MemoryStore
from nexus_supervisor_amd.testing.fake_apiserver import FakeApiServer
from nexus_supervisor_amd.testing.seed import ALGORITHM, make_event, make_job, seed_rows


def _elector(url, ident, **kw):
    c = KubeClient(KubeConfig(url))
    return LeaderElector(LeaseLock(c, "nexus", "nexus-supervisor-leader", ident), **kw), c


def test_exactly_one_leader_and_failover(arun):
    async def go():
        api = FakeApiServer()
        url = await api.start()
        kw = dict(lease_duration=0.6, renew_deadline=0.4, retry_period=0.1)
        a, ca = _elector(url, "a", **kw)
        b, cb = _elector(url, "b", **kw)
        a.start()
        await asyncio.sleep(0.3)
        b.start()
        for _ in range(10):
            await asyncio.sleep(0.1)
            assert a.leader + b.leader == 1
        assert a.leader
        # crash without releasing: b takes over after the lease expires
        t0 = time.monotonic()
        await a.stop(release=False)
        while not b.leader and time.monotonic() - t0 < 5:
            await asyncio.sleep(0.02)
        took = time.monotonic() - t0
        assert b.leader and took < 0.6 + 0.9, took  # lease duration + observation (CPU-loaded CI slack)
        lease = api.get("Lease", "nexus", "nexus-supervisor-leader")
        assert lease["spec"]["holderIdentity"] == "b" and lease["spec"]["leaseTransitions"] >= 1
        # graceful release: a fresh candidate gets it within ~one retry period
        c, cc = _elector(url, "c", **kw)
        c.start()
        await asyncio.sleep(0.2)
        assert not c.leader
        t0 = time.monotonic()
        await b.stop(release=True)
        while not c.leader and time.monotonic() - t0 < 5:
            await asyncio.sleep(0.02)
        assert c.leader and time.monotonic() - t0 < 1.0  # a few retry periods (CPU-loaded CI slack)
        await c.stop()
        for x in (ca, cb, cc):
            await x.close()
        await api.stop()

    arun(go())


def test_standby_replica_takes_over_without_losing_decisions(arun):
    """Two supervisor replicas with leader election over one apiserver; the leader dies
    mid-stream; every run still ends in its decided stage (replay on gaining leadership)."""
    async def go():
        api = FakeApiServer(bookmark_interval=0.2)
        url = await api.start()
        store = MemoryStore(seed_rows())
        apps = []
        for ident in ("r0", "r1"):
            cfg = load_config(path=None, env={}, overrides={
                "cql-store-type": "memory", "workers": 4, "rate-limit-elements-per-second": 0, "resync-period": "0s",
                "leader-election": {"enabled": True, "identity": ident, "lease-duration": "600ms",
                                    "renew-deadline": "400ms", "retry-period": "100ms"}})
            app = Application(cfg, kube=KubeClient(KubeConfig(url)), store=store)
            await app.start()
            apps.append(app)
        await asyncio.sleep(0.4)
        leaders = [a for a in apps if a.supervisor.active]
        assert len(leaders) == 1
        leader = leaders[0]
        standby = apps[1] if leader is apps[0] else apps[0]
        rows = seed_rows()
        labels = leader.cfg.labels
        api.create(make_job(rows[0].id, labels))
        api.create(make_event("Job", rows[0].id, "FailedCreate"))
        await asyncio.sleep(0.3)
        # leader crashes (no lease release); events keep arriving
        await leader.elector.stop(release=False)
        leader.supervisor.active = False
        await leader.stop()
        api.create(make_job(rows[1].id, labels))
        api.create(make_event("Job", rows[1].id, "DeadlineExceeded"))
        for _ in range(100):
            if standby.supervisor.active and store.get(ALGORITHM, rows[1].id).lifecycle_stage == "DEADLINE_EXCEEDED":
                break
            await asyncio.sleep(0.05)
        assert standby.supervisor.active
        assert store.get(ALGORITHM, rows[0].id).lifecycle_stage == "SCHEDULING_FAILED"
        assert store.get(ALGORITHM, rows[1].id).lifecycle_stage == "DEADLINE_EXCEEDED"
        await standby.stop()
        await api.stop()

    arun(go(), timeout=60)


def test_pprof_profile_roundtrip():
    p = Profile(period_ns=10_000_000)
    p.add((("a.py", "leaf", 1, 3), ("a.py", "root", 1, 9)), 5)
    p.add((("b.py", "other", 2, 4), ("a.py", "root", 1, 9)), 2)
    d = decode_profile(p.encode_gz())
    assert d["samples"] == 2 and d["sample_count"] == 7 and d["functions"] == 3 and d["locations"] == 3
    assert d["strings"][0] == "" and "leaf" in d["strings"] and "cpu" in d["strings"] and d["period"] == 10_000_000
    assert "leaf" in p.top()


def test_sampler_sees_busy_function():
    def busy_loop_marker(t_end):
        x = 0
        while time.monotonic() < t_end:
            x += 1
        return x

    s = Sampler(hz=400).start()
    busy_loop_marker(time.monotonic() + 0.3)
    prof = s.stop()
    assert any(fr[1] == "busy_loop_marker" for st in prof.stacks for fr in st)


def test_http_endpoints(arun):
    async def go():
        api = FakeApiServer()
        url = await api.start()
        cfg = load_config(path=None, env={}, overrides={"cql-store-type": "memory", "resync-period": "0s"})
        app = Application(cfg, kube=KubeClient(KubeConfig(url)), store=MemoryStore(seed_rows()))
        from nexus_supervisor_amd.obs.http import ObsServer

        await app.start()
        obs = ObsServer(app)
        port = await obs.start("127.0.0.1", 0)
        base = f"http://127.0.0.1:{port}"
        await app.factory.wait_for_cache_sync(5)
        async with aiohttp.ClientSession() as s:
            async with s.get(base + "/healthz") as r:
                assert r.status == 200
            async with s.get(base + "/readyz") as r:
                assert r.status == 200 and "leader" in await r.text()
            async with s.get(base + "/metrics") as r:
                text = await r.text()
                assert "nexus_supervisor_queue_depth" in text and 'kind="Pod"' in text
            async def fetch():
                async with s.get(base + "/debug/pprof/profile?seconds=0.3&hz=200") as r:
                    return await r.read()

            t = asyncio.ensure_future(fetch())
            await asyncio.sleep(0.05)
            t_end = time.monotonic() + 0.15  # CPU on the loop thread while the profile runs
            while time.monotonic() < t_end:
                pass
            d = decode_profile(await t)
            assert d["samples"] >= 1
            async with s.get(base + "/debug/vars") as r:
                doc = json.loads(await r.text())
                assert doc["active"] is True and "pipeline" in doc
            async with s.get(base + "/debug/heap?top=5&trim=1") as r:
                heap = json.loads(await r.text())
                assert heap["rss_mb"] > 0 and len(heap["types"]) == 5
                assert heap["structures"]["informer.Pod"] >= 0 and "supervisor._applied" in heap["structures"]
                assert heap["rss_after_trim_mb"] > 0
        await obs.stop()
        await app.stop()
        await api.stop()

    arun(go())


def test_signal_sampler_is_cpu_time_based():
    """SIGPROF mode (main thread): CPU-bound code is sampled, time blocked in a syscall
    is not (the thread sampler over-counts such frames)."""
    def cpu_marker(t_end):
        x = 0
        while time.monotonic() < t_end:
            x += 1
        return x

    def sleep_marker():
        time.sleep(0.3)

    s = Sampler(hz=500)
    assert s.mode == "signal"
    s.start()
    cpu_marker(time.monotonic() + 0.3)
    sleep_marker()
    prof = s.stop()
    leaf = {}
    for st, n in prof.stacks.items():
        leaf[st[0][1]] = leaf.get(st[0][1], 0) + n
    assert leaf.get("cpu_marker", 0) >= 20, leaf
    assert leaf.get("sleep_marker", 0) <= 3, leaf
    import signal as _signal

    assert _signal.getsignal(_signal.SIGPROF) in (_signal.SIG_DFL, None) or callable(_signal.getsignal(_signal.SIGPROF))


def test_profile_decode_and_merge_roundtrip():
    from nexus_supervisor_amd.obs.pprof import load_profile, merge_profiles

    p = Profile(5_000_000)
    p.add((("a.py", "leaf", 1, 3), ("a.py", "root", 10, 12)), 7)
    p.add((("b.py", "other", 2, 5),), 3)
    q = load_profile(p.encode_gz())
    assert q.stacks == p.stacks and q.period_ns == p.period_ns
    m = merge_profiles([q, load_profile(p.encode())])
    assert sum(m.stacks.values()) == 20 and "leaf (a.py)" in m.top(5)


def test_partitioned_leader_steps_down_at_its_hold_deadline(arun):
    """The leader is cut off from the apiserver (requests stall): it steps down no later
    than ``renew-deadline`` after its last renewal *started* — before the standby can take
    the lease (a lease duration after it last saw a renewal) — and reports each hold's
    deadline (``on_renewed``) so the supervisor fences writes on the clock."""
    from nexus_supervisor_amd.testing.netproxy import PausableProxy

    async def go():
        api = FakeApiServer()
        url = await api.start()
        host, port = url.rsplit(":", 1)
        proxy = PausableProxy(host.split("//")[1], int(port))
        purl = await proxy.start()
        kw = dict(lease_duration=0.8, renew_deadline=0.5, retry_period=0.1)
        holds = []
        a, ca = _elector(purl, "a", on_renewed=holds.append, **kw)
        b, cb = _elector(url, "b", **kw)
        a.start()
        await asyncio.sleep(0.3)
        b.start()
        await asyncio.sleep(0.3)
        assert a.leader and not b.leader and holds and holds[-1] == a.valid_until
        t_cut = time.monotonic()
        proxy.pause()
        end = a.valid_until
        assert end <= t_cut + 0.5 + 0.01
        while a.leader and time.monotonic() - t_cut < 5:
            await asyncio.sleep(0.005)
        t_down = time.monotonic()
        while not b.leader and time.monotonic() - t_cut < 5:
            await asyncio.sleep(0.005)
        t_b = time.monotonic()
        assert not a.leader and t_down <= end + 0.05, (t_down - end)
        assert b.leader and t_b > end, (t_b - end)
        proxy.resume()
        await a.stop(release=False)
        await b.stop()
        for x in (ca, cb):
            await x.close()
        await proxy.stop()
        await api.stop()

    arun(go(), timeout=30)


def test_supervisor_fences_on_the_hold_deadline():
    from nexus_supervisor_amd.supervisor import Supervisor
    from nexus_supervisor_amd.testing.inproc import InProcCluster

    cfg = load_config(path=None, env={}, overrides={"cql-store-type": "memory", "leader-election": {"enabled": True}})
    c = InProcCluster(cfg, MemoryStore(), [])
    sup: Supervisor = c.supervisor
    sup.active = True
    tok = sup._token("r1")
    sup.set_lease_deadline(time.monotonic() + 60)
    assert not sup._fenced(tok, "r1")
    sup.set_lease_deadline(time.monotonic() - 0.001)  # the hold lapsed: nothing is written any more
    assert sup._fenced(tok, "r1")
