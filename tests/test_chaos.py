"""Chaos suite — BASELINE config 5 analog, scaled to CPU: two supervisor replicas with
leader election over one apiserver, hundreds of concurrent runs, and during the
failure stream: a CQL node crash + restart (WAL replay), watch-history compaction
(410 Gone → re-list), the leader dying without releasing its lease, and an
eviction storm.  Every failed run must still end in its expected lifecycle stage.
(The reference has no fault injection at all — SURVEY §4, §5.3.)"""
import asyncio
import time

import pytest

from nexus_supervisor_amd.app import Application
from nexus_supervisor_amd.bench.wire import schema_statements
from nexus_supervisor_amd.bench.workload import Workload
from nexus_supervisor_amd.config import load_config
from nexus_supervisor_amd.kube.client import KubeClient, KubeConfig
from nexus_supervisor_amd.store.cql import CqlCheckpointStore, CqlSession
from nexus_supervisor_amd.testing.cqlsrv import CqlServer
from nexus_supervisor_amd.testing.fake_apiserver import FakeApiServer
from conftest import TIME_SCALE

pytestmark = pytest.mark.slow


def _cfg(ident, port):
    cfg = load_config(path=None, env={}, overrides={
        "cql-store-type": "scylla", "workers": 32, "rate-limit-elements-per-second": 0, "resync-period": "0s",
        "failure-rate-base-delay": "20ms", "failure-rate-max-delay": "200ms", "max-retries": 0,
        "scylla-cql-store": {"hosts": [f"127.0.0.1:{port}"], "request-timeout": "1s"},
        "leader-election": {"enabled": True, "identity": ident, "lease-duration": "800ms",
                            "renew-deadline": "500ms", "retry-period": "100ms"}})
    return cfg


async def _wait_stages(store, algorithm, expected, timeout):
    deadline = time.monotonic() + timeout
    missing = dict(expected)
    while missing and time.monotonic() < deadline:
        for rid, stage in list(missing.items()):
            try:
                row = await store.read_checkpoint(algorithm, rid)
            except Exception:  # noqa: BLE001 - server restarting
                await asyncio.sleep(0.05)
                continue
            if row is not None and row.lifecycle_stage == stage:
                del missing[rid]
        if missing:
            await asyncio.sleep(0.1)
    return missing


def test_two_replicas_survive_cql_restart_410_leader_crash_and_evictions(arun):
    async def go():
        srv = CqlServer(persist=True, exec_statements=schema_statements()).start()
        api = FakeApiServer(bookmark_interval=0.1)
        url = await api.start()
        wl = Workload(concurrent_jobs=300, seed=7)
        objs, rows = wl.initial()
        seed_store = CqlCheckpointStore(CqlSession([srv.address], request_timeout=1.0))
        await seed_store.connect()
        await asyncio.gather(*(seed_store.upsert_checkpoint(r) for r in rows))
        for o in objs:
            api.create(o)
        apps = []
        for ident in ("replica-a", "replica-b"):
            app = Application(_cfg(ident, srv.port), kube=KubeClient(KubeConfig(url)),
                              store=CqlCheckpointStore(CqlSession([srv.address], request_timeout=1.0)))
            await app.start()
            apps.append(app)
        await asyncio.sleep(0.5)
        assert sum(a.supervisor.active for a in apps) == 1
        expected = {}

        async def push(n, kinds=None):
            failed, traffic, new_rows = wl.step(n, kinds)
            for r in new_rows:
                for _ in range(50):
                    try:
                        await seed_store.upsert_checkpoint(r)
                        break
                    except Exception:  # noqa: BLE001
                        await asyncio.sleep(0.05)
            for etype, obj in traffic:
                api.apply(etype, obj)
            for rid in failed:
                expected[rid] = wl.expected[rid]

        # round 1: CQL node crash mid-stream (acknowledged writes survive through the WAL)
        await push(60)
        await asyncio.sleep(0.05)
        srv.restart()
        await push(60)
        # round 2: watch history compacted (410 → re-list) and the leader dies holding its lease
        api.expire()
        leader = next(a for a in apps if a.supervisor.active)
        await leader.elector.stop(release=False)
        leader.supervisor.active = False
        await leader.stop(drain_timeout=0.5)
        apps.remove(leader)
        await push(60)
        # round 3: eviction storm (pods evicted, Jobs then fail with BackoffLimitExceeded)
        await push(60, kinds=["evicted"])
        missing = await _wait_stages(seed_store, wl.algorithm, expected, timeout=40 * TIME_SCALE)
        assert not missing, f"{len(missing)} runs never reached their stage, e.g. {list(missing.items())[:3]}"
        survivor = apps[0]
        assert survivor.supervisor.active
        # every failed run's Job was deleted through the API (paced by the client-side
        # kube-qps bucket: 50/s by default, so the deletes trail the checkpoint writes)
        for _ in range(int(200 * TIME_SCALE)):
            deleted = {n for k, _ns, n, _p in api.deleted if k == "Job"}
            if set(expected) <= deleted:
                break
            await asyncio.sleep(0.05)
        assert set(expected) <= deleted
        # evicted runs were enriched with the eviction history (the Pod and Job watches are
        # separate streams, so a Job's failure can occasionally be decided before its pod's
        # eviction arrives: require the enrichment for most, not all)
        import json

        storm = list(expected)[-60:]
        classes = []
        for rid in storm:
            row = await seed_store.read_checkpoint(wl.algorithm, rid)
            classes.append(json.loads(row.algorithm_failure_details).get("class") if row.algorithm_failure_details.startswith("{") else None)
        assert classes.count("evicted") >= len(storm) // 2, classes
        for a in apps:
            await a.stop(drain_timeout=1)
        await seed_store.close()
        await api.stop()
        srv.stop()

    arun(go(), timeout=120 * TIME_SCALE)


def test_sharded_replicas_survive_cql_restart_storm_and_a_replica_crash(arun):
    """BASELINE config 5 with horizontal scale: 3 replicas over 6 shard Leases; a CQL node
    restart, an eviction storm and a replica dying with its leases mid-stream.  Its shards
    move to the survivors, its return wins its share back, and every failed run ends in
    its expected stage."""
    from nexus_supervisor_amd.bench.scenarios import cfg5s_sharded_chaos

    async def go():
        r = await cfg5s_sharded_chaos("uncapped", seconds=8, rate=3000, jobs=600)
        assert r["drained"] and r["acked"] == r["events"] and r["wrong_stage"] == 0, r
        ch = r["chaos"]
        lost = ch["crashed"]["shards"]
        assert lost and all(ch["final_owners"][k] and ch["final_owners"][k] != [ch["crashed"]["replica"]] for k in lost)
        assert ch["failover_s"] < 2.0 + 1.5  # lease duration + grace + observation
        # the crashed replica came back and got its fair share (2 of 6) handed back
        assert ch["rebalanced"], ch
        back = ch["crashed"]["replica"]
        assert sum(1 for v in ch["rebalanced_owners"].values() if back in v) == 2, ch

    arun(go(), timeout=120 * TIME_SCALE)
