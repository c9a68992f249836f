"""Scylla shard-aware routing.  The reference pins the
scylladb/gocql fork (``/root/reference/go.mod:93``), which keeps one connection per
Scylla shard and sends each request to the shard owning its token.  ``nexus-cqlsrv
--shards N`` emulates a sharded node (shard threads, ``SCYLLA_*`` SUPPORTED keys, the
shard-aware port) and counts, per EXECUTE, whether it arrived on the owning shard."""
import asyncio
import uuid

import pytest

from nexus_supervisor_amd.bench.wire import schema_statements
from nexus_supervisor_amd.models.checkpoint import CheckpointedRequest, LifecycleStage
from nexus_supervisor_amd.store.cql import CqlCheckpointStore, CqlSession, scylla_shard_of
from nexus_supervisor_amd.testing.cqlsrv import CqlServer


def test_biased_token_round_robin():
    # ignore_msb 0, 2 shards: the lower half of the (biased) ring is shard 0
    assert scylla_shard_of(-(1 << 63), 2, 0) == 0
    assert scylla_shard_of(-1, 2, 0) == 0
    assert scylla_shard_of(0, 2, 0) == 1
    assert scylla_shard_of((1 << 63) - 1, 2, 0) == 1
    import random

    rng = random.Random(3)
    shards = {scylla_shard_of(rng.randrange(-(1 << 63), 1 << 63), 8, 12) for _ in range(400)}
    assert shards == set(range(8))
    # ignore_msb: the top bits do not move a token between shards
    t = 0x123456789ABCDEF
    assert scylla_shard_of(t, 8, 12) == scylla_shard_of(t ^ (0x7FF << 52), 8, 12)


async def _stats(store):
    rows = await store.session.query("SELECT * FROM system.cqlsrv_stats")
    return rows.dicts()[0]


def _rows(n):
    return [CheckpointedRequest(algorithm="alg", id=str(uuid.uuid4()), lifecycle_stage=LifecycleStage.RUNNING)
            for _ in range(n)]


@pytest.mark.parametrize("aware_port", [0, -1], ids=["shard-aware-port", "reconnect-until-covered"])
def test_every_request_lands_on_the_owning_shard(arun, aware_port):
    srv = CqlServer(exec_statements=schema_statements(), shards=4, shard_aware_port=aware_port).start()

    async def go():
        store = CqlCheckpointStore(CqlSession([srv.address], connections_per_host=1))
        await store.connect()
        h = next(iter(store.session.hosts.values()))
        assert h.nr_shards == 4 and h.ignore_msb == 12
        assert [len(c) >= 1 for c in h.shard_conns] == [True] * 4
        for k, conns in enumerate(h.shard_conns):
            assert all(int(c.scylla("SCYLLA_SHARD")) == k for c in conns)
        before = await _stats(store)
        rows = _rows(300)
        await asyncio.gather(*(store.upsert_checkpoint(r) for r in rows))
        got = await asyncio.gather(*(store.read_status(r.algorithm, r.id) for r in rows))
        assert all(g.lifecycle_stage == LifecycleStage.RUNNING for g in got)
        await asyncio.gather(*(store.update_status(r.algorithm, r.id, LifecycleStage.FAILED, "c", "d", None)
                               for r in rows[:100]))
        after = await _stats(store)
        hits = after["shard_hits"] - before["shard_hits"]
        misses = after["shard_misses"] - before["shard_misses"]
        assert misses == 0 and hits >= 700, (hits, misses)
        assert store.session.stats["shard_routed"] >= 700
        await store.close()

    try:
        arun(go())
    finally:
        srv.stop()


def test_shard_unaware_client_pays_cross_shard_hops(arun):
    """Control: with shard-awareness off the same traffic lands on the wrong shard ~3/4
    of the time on a 4-shard node — the hop the shard-aware driver avoids."""
    srv = CqlServer(exec_statements=schema_statements(), shards=4).start()

    async def go():
        store = CqlCheckpointStore(CqlSession([srv.address], connections_per_host=1, shard_aware=False))
        await store.connect()
        rows = _rows(200)
        await asyncio.gather(*(store.upsert_checkpoint(r) for r in rows))
        st = await _stats(store)
        assert st["shard_misses"] > 100, st
        await store.close()

    try:
        arun(go())
    finally:
        srv.stop()


def _closed_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_unreachable_shard_aware_port_falls_back_without_leaks(arun):
    """A node advertises SCYLLA_SHARD_AWARE_PORT but the port is
    refused (e.g. a Service exposing only 9042).  The host still comes up — every shard
    reached by reconnecting to the regular port — and nothing is left open but the
    per-shard connections."""
    srv = CqlServer(exec_statements=schema_statements(), shards=4, shard_aware_port=-1,
                    extra_args=["--advertise-shard-aware-port", str(_closed_port())]).start()

    async def go():
        store = CqlCheckpointStore(CqlSession([srv.address], connections_per_host=1))
        await store.connect()
        h = next(iter(store.session.hosts.values()))
        assert h.up and h.nr_shards == 4
        assert store.session.stats.get("shard_port_fallbacks", 0) >= 1
        assert all(len(c) == 1 for c in h.shard_conns), [len(c) for c in h.shard_conns]
        assert len(h.conns) == 4
        rows = _rows(50)
        await asyncio.gather(*(store.upsert_checkpoint(r) for r in rows))
        stats = await _stats(store)
        assert stats["shard_misses"] == 0
        # connections accepted in total: the regular port hands each new connection the
        # least-loaded shard, so the fallback needs exactly one per shard (the refused
        # aware-port attempts never reach the server)
        assert stats["connections"] == 4, stats
        await store.close()

    try:
        arun(go())
    finally:
        srv.stop()


def test_failed_host_open_closes_what_it_opened(arun, monkeypatch):
    """A host whose open fails half-way (here: the 3rd shard connection raises) leaves no
    connection behind — every reconnect attempt used to leak the ones already opened."""
    from nexus_supervisor_amd.store import cql as cql_mod

    srv = CqlServer(exec_statements=schema_statements(), shards=4).start()
    made = []
    real = cql_mod.CqlConnection.connect

    async def flaky(self, keyspace=None):
        made.append(self)
        if len(made) == 3:
            raise OSError(111, "injected refusal")
        return await real(self, keyspace)

    async def go():
        sess = CqlSession([srv.address], connections_per_host=1, discover=False)
        h = cql_mod.Host(address=srv.address)
        sess.shard_aware_port = False  # regular-port mode: an OSError is fatal for this open
        monkeypatch.setattr(cql_mod.CqlConnection, "connect", flaky)
        try:
            await sess._open_host(h)
        except OSError:
            pass
        else:
            raise AssertionError("open should have failed")
        assert made and all(c.closed for c in made)
        assert not h.up and h.conns == []

    try:
        arun(go())
    finally:
        srv.stop()


def test_conditional_writes_never_skip_metadata(arun):
    """A conditional write prepares with result metadata
    ``[applied]`` alone (as Cassandra), while its not-applied answer carries the row's
    stage.  The client must not execute it with skip_metadata, or the finished-row skip
    and the unknown-stage fallback would silently stop working."""
    from nexus_supervisor_amd.store.cql import is_conditional

    assert is_conditional("UPDATE t SET a=? WHERE k=? IF a IN (?)")
    assert is_conditional("insert into t (k) values (?) if not exists")
    assert not is_conditional("SELECT lifecycle_stage FROM t WHERE k=?")
    assert not is_conditional("UPDATE t SET a=? WHERE k=?")
    srv = CqlServer(exec_statements=schema_statements()).start()

    async def go():
        store = CqlCheckpointStore(CqlSession([srv.address], connections_per_host=1))
        await store.connect()
        row = _rows(1)[0]
        row.lifecycle_stage = LifecycleStage.CANCELLED
        await store.upsert_checkpoint(row)
        unfinished = ("NEW", "BUFFERED", "RUNNING")
        applied, current = await store.cas_update(row.algorithm, row.id, LifecycleStage.FAILED, "c", "d", None,
                                                  unfinished)
        assert (applied, current) == (False, LifecycleStage.CANCELLED)
        ps = next(p for q, p in store.session._prepared.items() if " IF " in q)
        assert ps.conditional and ps.result_names == ("[applied]",)  # the prepared shape is [applied] only
        missing = await store.cas_update(row.algorithm, "no-such-run", LifecycleStage.FAILED, "c", "d", None, unfinished)
        assert missing == (False, None)
        await store.close()

    try:
        arun(go())
    finally:
        srv.stop()
