"""CQL v4 codec (native), the asyncio client and the checkpoint store against the
native CQL server — the Scylla leg of the reference integration test
(``/root/reference/services/supervisor_test.go:36-39``; schema + seed
``/root/reference/test-resources/checkpoints.cql``)."""
import asyncio
import datetime as dt
import uuid

import pytest

from nexus_supervisor_amd import _cql_native as N
from nexus_supervisor_amd.models.checkpoint import LifecycleStage
from nexus_supervisor_amd.store.cql import (CONSISTENCY, CqlCheckpointStore, CqlError, CqlSession, StoreError)
from nexus_supervisor_amd.testing.cqlsrv import CqlServer
from nexus_supervisor_amd.testing.seed import ALGORITHM, seed_cql_statements, seed_rows

UTC = dt.timezone.utc


# ---------------------------------------------------------------- codec
def test_murmur3_public_driver_vectors():
    # vectors published with the DataStax python-driver murmur3 tests
    assert N.murmur3_token(b"123") == -7468325962851647638
    assert N.murmur3_token(b"\x00\xff\x10\xfa\x99" * 10) == 5837342703291459765
    assert N.murmur3_token(b"\xfe" * 8) == -8927430733708461935
    assert N.murmur3_token(b"\x10" * 8) == 1446172840243228796
    assert N.murmur3_token(b"9223372036854775807") == 7162290910810015547


def test_composite_routing_key_layout():
    k = N.routing_key([b"algo", b"id-1"])
    assert k == b"\x00\x04algo\x00\x00\x04id-1\x00"
    assert N.routing_key([b"only"]) == b"only"
    assert N.token_for(["algo", "id-1"]) == N.murmur3_token(k)


@pytest.mark.parametrize("typ,value", [
    (0x0D, "héllo ✓"), (0x02, -(2 ** 62)), (0x09, -12345), (0x04, True), (0x04, False), (0x07, 2.5),
    (0x03, b"\x00\x01\xff"), (0x0C, "6ba7b810-9dad-11d1-80b4-00c04fd430c8"), (0x13, -7), (0x14, 5),
    ((0x22, 0x0D), ["a", "b"]), ((0x20, 0x09), [1, 2, 3]), ((0x21, 0x0D, 0x02), {"x": 1, "y": 2}),
])
def test_value_roundtrip(typ, value):
    assert N.deserialize(N.serialize(value, typ), typ) == value


def test_timestamp_roundtrip_ms_precision():
    t = dt.datetime(2023, 10, 2, 10, 0, 0, 123000, tzinfo=UTC)
    raw = N.serialize(t, 0x0B)
    assert raw == int(t.timestamp() * 1000).to_bytes(8, "big", signed=True)
    assert N.deserialize(raw, 0x0B) == t


def test_frame_reader_handles_split_frames():
    # a READY frame (opcode 2, empty body) and an ERROR frame, fed one byte at a time
    ready = bytes([0x84, 0, 0, 7, 0x02, 0, 0, 0, 0])
    msg = b"boom"
    body = (0x2200).to_bytes(4, "big") + len(msg).to_bytes(2, "big") + msg
    err = bytes([0x84, 0, 0, 9, 0x00]) + len(body).to_bytes(4, "big") + body
    r = N.FrameReader()
    out = []
    for b in ready + err:
        out += r.feed(bytes([b]))
    assert out == [(7, 2, ("ready",)), (9, 0, ("error", 0x2200, "boom", {}))]
    assert r.buffered == 0


def test_encode_query_frame_layout():
    f = N.encode_query(5, "SELECT 1", None, None, CONSISTENCY["ONE"])
    assert f[:5] == bytes([0x04, 0x00, 0x00, 0x05, 0x07])
    assert int.from_bytes(f[5:9], "big") == len(f) - 9
    assert f[9:13] == len("SELECT 1").to_bytes(4, "big") and f[13:21] == b"SELECT 1"


# ---------------------------------------------------------------- store against nexus-cqlsrv
@pytest.fixture
def seeded():
    with CqlServer(exec_statements=seed_cql_statements()) as srv:
        yield srv


async def _store(srv, **kw):
    st = CqlCheckpointStore(CqlSession([srv.address], **kw))
    await st.connect()
    return st


def test_seed_rows_byte_compatible(seeded, arun):
    async def go():
        st = await _store(seeded)
        try:
            for row in seed_rows():
                got = await st.read_checkpoint(ALGORITHM, row.id)
                assert got == row
            assert await st.read_checkpoint(ALGORITHM, "missing") is None
            cnt = await st.session.query("SELECT COUNT(*) FROM nexus.checkpoints")
            assert cnt.rows[0][0] == 8
            idx = await st.session.query("SELECT id FROM nexus.checkpoints WHERE lifecycle_stage = 'CANCELLED'")
            assert [r[0] for r in idx.rows] == ["df1b6e8d-cc3c-fb5b-a3f6-5d7b9e2c7f2b"]
        finally:
            await st.close()

    arun(go())


def test_owned_columns_update_keeps_other_columns(seeded, arun):
    async def go():
        st = await _store(seeded)
        row = seed_rows()[0]
        now = dt.datetime(2026, 1, 1, 12, 0, 0, 500000, tzinfo=UTC)
        assert await st.update_status(ALGORITHM, row.id, LifecycleStage.FAILED, "cause", "details", now)
        got = await st.read_checkpoint(ALGORITHM, row.id)
        assert (got.lifecycle_stage, got.algorithm_failure_cause, got.algorithm_failure_details) == ("FAILED", "cause", "details")
        assert got.last_modified == now
        assert got.payload_uri == row.payload_uri and got.received_at == row.received_at and got.tag == row.tag
        # stage-only write leaves the failure columns alone
        await st.update_status(ALGORITHM, row.id, LifecycleStage.RUNNING, None, None, now, set_failure=False)
        got = await st.read_checkpoint(ALGORITHM, row.id)
        assert got.lifecycle_stage == "RUNNING" and got.algorithm_failure_cause == "cause"
        # projected stage read (owned-columns path): key + stage only
        lite = await st.read_status(ALGORITHM, row.id)
        assert (lite.algorithm, lite.id, lite.lifecycle_stage) == (ALGORITHM, row.id, "RUNNING")
        assert lite.payload_uri is None and not lite.is_finished()
        assert await st.read_status(ALGORITHM, "missing") is None
        await st.close()

    arun(go())


def test_conditional_update_lwt(seeded, arun):
    async def go():
        st = await _store(seeded)
        rid = seed_rows()[0].id  # BUFFERED
        now = dt.datetime.now(UTC)
        assert not await st.update_status(ALGORITHM, rid, "FAILED", "c", "d", now, only_if_stages=["RUNNING"])
        assert (await st.read_checkpoint(ALGORITHM, rid)).lifecycle_stage == "BUFFERED"
        assert await st.update_status(ALGORITHM, rid, "FAILED", "c", "d", now, only_if_stages=["NEW", "BUFFERED"])
        assert (await st.read_checkpoint(ALGORITHM, rid)).lifecycle_stage == "FAILED"
        await st.close()

    arun(go())


def test_full_row_upsert(seeded, arun):
    async def go():
        st = await _store(seeded)
        row = seed_rows()[1].deep_copy()
        row.id = str(uuid.uuid4())
        row.result_uri = None
        await st.upsert_checkpoint(row)
        assert await st.read_checkpoint(ALGORITHM, row.id) == row
        await st.close()

    arun(go())


def test_password_authenticator():
    async def go(srv):
        with pytest.raises(CqlError) as ei:
            await _store(srv, user="nexus", password="wrong")
        assert ei.value.code == 0x0100
        st = await _store(srv, user="nexus", password="s3cret")
        assert await st.read_checkpoint(ALGORITHM, seed_rows()[0].id) is not None
        await st.close()

    with CqlServer(user="nexus", password="s3cret", exec_statements=seed_cql_statements()) as srv:
        asyncio.run(asyncio.wait_for(go(srv), 30))


def test_restart_with_wal_reprepares_and_keeps_rows(arun):
    srv = CqlServer(persist=True, exec_statements=seed_cql_statements()).start()
    try:
        async def go():
            st = await _store(srv, request_timeout=2.0)
            rid = seed_rows()[2].id
            now = dt.datetime.now(UTC).replace(microsecond=0)
            await st.update_status(ALGORITHM, rid, "DEADLINE_EXCEEDED", "x", "y", now)
            srv.restart()  # SIGKILL + start: prepared statements gone, rows replayed from the WAL
            for _ in range(100):
                try:
                    got = await st.read_checkpoint(ALGORITHM, rid)
                    break
                except StoreError:
                    await asyncio.sleep(0.05)
            assert got.lifecycle_stage == "DEADLINE_EXCEEDED" and got.last_modified == now
            assert st.session.stats["reprepares"] >= 1
            assert await st.read_checkpoint(ALGORITHM, seed_rows()[0].id) == seed_rows()[0]
            await st.close()

        arun(go())
    finally:
        srv.stop()


def test_dropped_connections_are_retried(seeded, arun):
    async def go():
        st = await _store(seeded, request_timeout=2.0)
        seeded.drop_connections()
        await asyncio.sleep(0.1)
        got = None
        for _ in range(50):
            try:
                got = await st.read_checkpoint(ALGORITHM, seed_rows()[0].id)
                break
            except StoreError:
                await asyncio.sleep(0.05)
        assert got is not None
        await st.close()

    arun(go())


def test_overloaded_errors_retried(arun):
    with CqlServer(error_rate=0.3, exec_statements=seed_cql_statements()) as srv:
        async def go():
            st = await _store(srv, max_retries=8)
            for _ in range(30):
                assert (await st.read_checkpoint(ALGORITHM, seed_rows()[0].id)) is not None
            assert st.session.stats["retries"] > 0
            await st.close()

        arun(go())


def test_token_aware_routing_two_nodes(arun):
    # node A owns (-inf, 0], node B owns (0, +inf); each advertises the other as a peer
    stmts = ["CREATE KEYSPACE ks WITH replication = {'class': 'SimpleStrategy', 'replication_factor': 1}",
             "CREATE TABLE ks.t (algorithm text, id text, v text, PRIMARY KEY ((algorithm, id)))"]
    a = CqlServer(tokens=[0], exec_statements=stmts).start()
    b = CqlServer(tokens=[9223372036854775807], exec_statements=stmts).start()
    a.stop(); b.stop()
    a.peers = [f"127.0.0.1:{b.port}:9223372036854775807"]
    b.peers = [f"127.0.0.1:{a.port}:0"]
    a.port, b.port = a.port, b.port
    a.start(); b.start()
    try:
        async def go():
            s = CqlSession([a.address], consistency="ONE")
            await s.connect()
            assert len(s.hosts) == 2
            keys = [("algo", f"id-{i}") for i in range(40)]
            for k in keys:
                await s.execute("INSERT INTO ks.t (algorithm, id, v) VALUES (?, ?, ?)", (k[0], k[1], "x"))
            owner_a = [k for k in keys if N.token_for(list(k)) <= 0]
            ca = await s._query_on(s.hosts[a.address], "SELECT COUNT(*) FROM ks.t")
            cb = await s._query_on(s.hosts[b.address], "SELECT COUNT(*) FROM ks.t")
            assert ca.rows[0][0] == len(owner_a) and cb.rows[0][0] == len(keys) - len(owner_a)
            assert 0 < len(owner_a) < len(keys)
            assert s.stats["token_routed"] >= len(keys)
            await s.close()

        arun(go())
    finally:
        a.stop()
        b.stop()


def test_server_rejects_bad_cql(seeded, arun):
    async def go():
        s = CqlSession([seeded.address])
        await s.connect()
        with pytest.raises(CqlError) as ei:
            await s.query("SELEKT * FROM nexus.checkpoints")
        assert ei.value.code == 0x2000
        with pytest.raises(CqlError) as ei:
            await s.query("SELECT nope FROM nexus.checkpoints WHERE algorithm = 'a' AND id = 'b'")
        assert ei.value.code == 0x2200
        await s.close()

    arun(go())


def test_bulk_upsert_as_unlogged_batches(arun):
    """Receiver-style bulk load: ``upsert_many`` sends one BATCH frame per 64 rows."""
    from nexus_supervisor_amd.bench.wire import schema_statements
    from nexus_supervisor_amd.bench.workload import Workload

    async def go():
        srv = CqlServer(exec_statements=schema_statements()).start()
        st = CqlCheckpointStore(CqlSession([srv.address]))
        try:
            await st.connect()
            _, rows = Workload(200).initial()
            before = st.session.stats["requests"]
            await st.upsert_many(rows)
            assert st.session.stats["requests"] - before == 4  # ceil(200 / 64) batches
            for r in (rows[0], rows[77], rows[-1]):
                got = await st.read_checkpoint(r.algorithm, r.id)
                assert got.id == r.id and got.lifecycle_stage == r.lifecycle_stage and got.payload_uri == r.payload_uri
            cnt = await st.session.query("SELECT COUNT(*) FROM nexus.checkpoints")
            assert cnt.rows[0][0] == 200
        finally:
            await st.close()
            srv.stop()

    arun(go())
