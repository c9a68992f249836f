"""Fused actuation (``compat.fused-write``, the default): one conditional write per decision
instead of the reference's read followed by a write (``/root/reference/services/supervisor.go:264-301``).

The not-applied answer of ``UPDATE … IF lifecycle_stage IN (<unfinished>)`` carries the row's
stage, so the reference's skip paths (no row, finished row, ToRunning on a RUNNING row) are
taken without a read — and a row finished between the reference's read and write (another
component's CANCELLED, a new leader's FAILED) cannot be overwritten even without HA."""
import asyncio
import datetime as dt

from nexus_supervisor_amd.config import load_config
from nexus_supervisor_amd.models import checkpoint as cp_mod
from nexus_supervisor_amd.models.checkpoint import LifecycleStage
from nexus_supervisor_amd.store.cql import CqlCheckpointStore, CqlSession
from nexus_supervisor_amd.store.memory import MemoryStore
from nexus_supervisor_amd.testing.cqlsrv import CqlServer
from nexus_supervisor_amd.testing.inproc import InProcCluster, RecordingJobs
from nexus_supervisor_amd.testing.seed import ALGORITHM, make_event, make_job, make_pod, seed_cql_statements, seed_rows

UTC = dt.timezone.utc
ROWS = seed_rows()
BUFFERED_ROW, RUNNING_ROW, CANCELLED_ROW = ROWS[0], ROWS[1], ROWS[7]


class CountingStore(MemoryStore):
    """Memory store that counts reads and can hold the fused write 'on the wire'."""

    def __init__(self, rows):
        super().__init__(rows)
        self.status_reads = 0
        self.cas_calls = 0
        self.gate = None
        self.at_gate = asyncio.Event()

    async def read_checkpoint(self, algorithm, request_id):
        self.status_reads += 1
        return await super().read_checkpoint(algorithm, request_id)

    async def cas_update(self, *a, **kw):
        self.cas_calls += 1
        if self.gate is not None:
            self.at_gate.set()
            await self.gate.wait()
        return await super().cas_update(*a, **kw)


def _cfg(**over):
    """These tests pin the fused actuation (``compat.fused-write: true``); its ``auto``
    default (fused only under HA) is covered by test_fused_default_follows_ha."""
    base = {"cql-store-type": "memory", "rate-limit-elements-per-second": 0, "resync-period": "0s",
            "failure-rate-base-delay": "10ms", "failure-rate-max-delay": "50ms", "compat": {"fused-write": True}}
    over = dict(over)
    if "compat" in over:
        over["compat"] = dict(base["compat"], **over["compat"])
    base.update(over)
    return load_config(path=None, env={}, overrides=base)


def test_fused_default_follows_ha():
    """An LWT is a Paxos round (~4 replica round trips, serialised per
    partition), so the default fuses the decision into one conditional write only where
    its atomic stage check is needed — a deposed leader or shard owner may still hold a
    decision — and a lone replica keeps the reference's read + plain write."""
    from nexus_supervisor_amd.supervisor import fused_actuation

    def cfg(**over):
        return load_config(path=None, env={}, overrides=dict({"cql-store-type": "memory"}, **over))

    assert cfg().compat.fused_write == "auto" and not fused_actuation(cfg())
    assert fused_actuation(cfg(**{"leader-election": {"enabled": True}}))
    assert fused_actuation(cfg(sharding={"shards": 2, "mode": "lease"}))
    assert not fused_actuation(cfg(sharding={"shards": 2, "shard-index": 1}))  # static shards: no deposed owner
    assert fused_actuation(cfg(compat={"fused-write": True}))
    assert not fused_actuation(cfg(compat={"fused-write": False}, **{"leader-election": {"enabled": True}}))
    assert cfg(compat={"fused-write": "yes"}).compat.fused_write == "true"


def test_fused_is_the_default_and_reference_mode_turns_it_off():
    assert _cfg().compat.fused_write == "true"
    from nexus_supervisor_amd.supervisor import Supervisor  # noqa: F401 - import check
    cfg = _cfg(compat={"conditional-update": "never"})
    c = InProcCluster(cfg, MemoryStore(ROWS), [])
    assert c.supervisor._fused is False
    c2 = InProcCluster(_cfg(compat={"full-row-upsert": True}), MemoryStore(ROWS), [])
    assert c2.supervisor._fused is False
    assert InProcCluster(_cfg(), MemoryStore(ROWS), []).supervisor._fused is True


def test_failure_decision_is_one_store_request_and_deletes_the_job(arun):
    async def go():
        cfg = _cfg()
        store = CountingStore([RUNNING_ROW])
        jobs = RecordingJobs([RUNNING_ROW.id])
        c = InProcCluster(cfg, store, [make_job(RUNNING_ROW.id, cfg.labels)], jobs=jobs)
        await c.start()
        c.push(make_event("Job", RUNNING_ROW.id, "DeadlineExceeded", "Job was active longer than specified deadline"))
        assert await c.settle(5)
        row = store.get(ALGORITHM, RUNNING_ROW.id)
        assert row.lifecycle_stage == LifecycleStage.DEADLINE_EXCEEDED
        assert row.algorithm_failure_details  # the trace rendered before the write
        assert store.status_reads == 0 and store.cas_calls == 1
        assert [d.outcome for d in c.decisions] == ["applied"]
        for _ in range(100):
            if jobs.deleted:
                break
            await asyncio.sleep(0.01)
        assert jobs.deleted == [RUNNING_ROW.id]
        await c.stop()

    arun(go())


def test_third_party_cancelled_wins_without_ha(arun):
    """No leader election, failure write on the wire when another component cancels the run:
    the two-step path (read RUNNING, then an unconditional write) would overwrite CANCELLED
    with FAILED; the fused write is refused and reports the finished stage."""
    async def go():
        cfg = _cfg()
        store = CountingStore([RUNNING_ROW])
        jobs = RecordingJobs([RUNNING_ROW.id])
        c = InProcCluster(cfg, store, [make_job(RUNNING_ROW.id, cfg.labels)], jobs=jobs)
        await c.start()
        store.gate = asyncio.Event()
        c.push(make_event("Job", RUNNING_ROW.id, "PodFailurePolicy", "exit 137"))
        await asyncio.wait_for(store.at_gate.wait(), 5)
        store.rows[(ALGORITHM, RUNNING_ROW.id)].lifecycle_stage = LifecycleStage.CANCELLED
        store.gate.set()
        assert await c.settle(5)
        assert store.get(ALGORITHM, RUNNING_ROW.id).lifecycle_stage == LifecycleStage.CANCELLED
        assert [(d.outcome, d.new_stage) for d in c.decisions] == [("skipped-finished", LifecycleStage.CANCELLED)]
        assert jobs.deleted == []  # CANCELLED is not a failed stage: the Job is not this decision's to delete
        await c.stop()

    arun(go())


def test_missing_row_and_finished_row_skip_without_a_read(arun):
    async def go():
        cfg = _cfg()
        store = CountingStore([CANCELLED_ROW])
        c = InProcCluster(cfg, store, [make_job("no-such-run", cfg.labels), make_job(CANCELLED_ROW.id, cfg.labels)])
        await c.start()
        c.push(make_event("Job", "no-such-run", "DeadlineExceeded", "deadline"))
        c.push(make_event("Job", CANCELLED_ROW.id, "DeadlineExceeded", "deadline"))
        assert await c.settle(5)
        got = sorted((d.result.request_id, d.outcome) for d in c.decisions)
        assert got == sorted([("no-such-run", "skipped-missing"), (CANCELLED_ROW.id, "skipped-finished")])
        assert store.status_reads == 0 and store.write_log == []
        assert store.get(ALGORITHM, CANCELLED_ROW.id).lifecycle_stage == LifecycleStage.CANCELLED
        assert c.supervisor.metrics.counter("decisions_missing_checkpoint") == 1
        await c.stop()

    arun(go())


def test_finished_failed_row_with_surviving_job_finishes_the_delete(arun):
    """A crash between the durable write and the Job DELETE: the replay's fused write is refused
    with FAILED, and the Job still in the cache is deleted (the two-step path's rule) — in the
    background, like a fresh decision's DELETE (``async-job-delete``): the worker does not
    wait for it."""
    async def go():
        cfg = _cfg()
        failed = RUNNING_ROW.deep_copy()
        failed.lifecycle_stage = LifecycleStage.FAILED
        store = CountingStore([failed])
        jobs = RecordingJobs([failed.id])
        c = InProcCluster(cfg, store, [make_job(failed.id, cfg.labels)], jobs=jobs)
        await c.start()
        c.push(make_event("Job", failed.id, "PodFailurePolicy", "exit 137"))
        assert await c.settle(5)
        assert [d.outcome for d in c.decisions] == ["skipped-finished"]
        for _ in range(100):
            if jobs.deleted:
                break
            await asyncio.sleep(0.01)
        assert jobs.deleted == [failed.id] and store.write_log == []
        await c.stop()

    arun(go())


def test_to_running_on_running_row_is_not_written(arun):
    async def go():
        cfg = _cfg()
        store = CountingStore([RUNNING_ROW, BUFFERED_ROW])
        objs = []
        c = InProcCluster(cfg, store, objs)
        await c.start()
        for row in (RUNNING_ROW, BUFFERED_ROW):
            pod = make_pod(row.id, cfg.labels, status={"phase": "Pending"})
            c.push(pod)
            c.push(make_event("Pod", pod["metadata"]["name"], "Started", "Started container algorithm"))
        assert await c.settle(5)
        out = {d.result.request_id: d.outcome for d in c.decisions}
        assert out == {RUNNING_ROW.id: "skipped-already-running", BUFFERED_ROW.id: "applied"}
        assert store.write_log == [((ALGORITHM, BUFFERED_ROW.id), LifecycleStage.RUNNING)]
        assert store.status_reads == 0
        await c.stop()

    arun(go())


def test_unknown_stage_string_falls_back_to_the_two_step_path(arun):
    """A row in a stage outside the configured set is neither finished nor in the guard:
    the fused write is refused and the two-step path decides with that stage in its guard."""
    async def go():
        cfg = _cfg()
        odd = RUNNING_ROW.deep_copy()
        odd.lifecycle_stage = "PAUSED_BY_OPERATOR"
        store = CountingStore([odd])
        c = InProcCluster(cfg, store, [make_job(odd.id, cfg.labels)])
        await c.start()
        c.push(make_event("Job", odd.id, "DeadlineExceeded", "deadline"))
        assert await c.settle(5)
        assert [d.outcome for d in c.decisions] == ["applied"]
        assert store.get(ALGORITHM, odd.id).lifecycle_stage == LifecycleStage.DEADLINE_EXCEEDED
        assert c.supervisor.metrics.counter("fused_write_fallbacks") == 1
        assert store.status_reads == 1
        await c.stop()

    arun(go())


def test_guard_follows_configured_stages(arun):
    """Remapped stage strings (``stages:``) reach the fused guard."""
    try:
        cp_mod.configure_lifecycle_stages({"FAILED": "FAILED_V2"})
        cfg = _cfg()
        c = InProcCluster(cfg, MemoryStore(ROWS), [])
        g = c.supervisor._unfinished_guard(False)
        assert "FAILED_V2" not in g and "FAILED" not in g and LifecycleStage.RUNNING in g
        assert LifecycleStage.RUNNING not in c.supervisor._unfinished_guard(True)
    finally:
        cp_mod.configure_lifecycle_stages(None)


def test_cql_cas_update_against_native_server(arun):
    """The store's fused write over the wire: applied; refused with the finished stage;
    refused on a missing row (no stage); the row's other columns untouched."""
    async def go():
        with CqlServer(exec_statements=seed_cql_statements()) as srv:
            st = CqlCheckpointStore(CqlSession([srv.address]))
            await st.connect()
            try:
                now = dt.datetime(2026, 1, 1, 12, 0, 0, 250000, tzinfo=UTC)
                guard = cp_mod.unfinished_stages()
                assert await st.cas_update(ALGORITHM, RUNNING_ROW.id, "FAILED", "cause", "details", now, guard) == (True, None)
                got = await st.read_checkpoint(ALGORITHM, RUNNING_ROW.id)
                assert (got.lifecycle_stage, got.algorithm_failure_cause, got.last_modified) == ("FAILED", "cause", now)
                assert got.payload_uri == RUNNING_ROW.payload_uri
                assert await st.cas_update(ALGORITHM, RUNNING_ROW.id, "DEADLINE_EXCEEDED", "c", "d", now, guard) \
                    == (False, "FAILED")
                assert await st.cas_update(ALGORITHM, CANCELLED_ROW.id, "FAILED", "c", "d", now, guard) \
                    == (False, "CANCELLED")
                assert await st.cas_update(ALGORITHM, "missing", "FAILED", "c", "d", now, guard) == (False, None)
                assert await st.read_checkpoint(ALGORITHM, "missing") is None  # no upsert of a phantom row
                run_guard = tuple(s for s in guard if s != "RUNNING")
                assert await st.cas_update(ALGORITHM, BUFFERED_ROW.id, "RUNNING", None, None, now, run_guard,
                                           set_failure=False) == (True, None)
                assert await st.cas_update(ALGORITHM, BUFFERED_ROW.id, "RUNNING", None, None, now, run_guard,
                                           set_failure=False) == (False, "RUNNING")
            finally:
                await st.close()

    arun(go())


def test_base_store_fallback_cas_is_read_then_conditional_write(arun):
    """A store without an atomic ``cas_update`` gets the protocol's read + conditional write."""
    from nexus_supervisor_amd.store.base import CheckpointStore

    class TwoStep(CheckpointStore):
        def __init__(self, rows):
            self.inner = MemoryStore(rows)
            self.race = None  # stage another writer sets between the read and the write

        async def read_checkpoint(self, algorithm, request_id):
            return await self.inner.read_checkpoint(algorithm, request_id)

        async def update_status(self, algorithm, request_id, *a, **kw):
            if self.race is not None:
                self.inner.rows[(algorithm, request_id)].lifecycle_stage = self.race
                self.race = None
            return await self.inner.update_status(algorithm, request_id, *a, **kw)

    async def go():
        st = TwoStep([RUNNING_ROW, CANCELLED_ROW])
        now = dt.datetime.now(UTC)
        guard = cp_mod.unfinished_stages()
        assert await st.cas_update(ALGORITHM, "missing", "FAILED", "c", "d", now, guard) == (False, None)
        assert await st.cas_update(ALGORITHM, CANCELLED_ROW.id, "FAILED", "c", "d", now, guard) == (False, "CANCELLED")
        st.race = "CANCELLED"  # lost the race after the read: the conditional write refuses, re-read reports it
        assert await st.cas_update(ALGORITHM, RUNNING_ROW.id, "FAILED", "c", "d", now, guard) == (False, "CANCELLED")
        st.inner.rows[(ALGORITHM, RUNNING_ROW.id)].lifecycle_stage = "RUNNING"
        assert await st.cas_update(ALGORITHM, RUNNING_ROW.id, "FAILED", "c", "d", now, guard) == (True, None)
        assert st.inner.get(ALGORITHM, RUNNING_ROW.id).lifecycle_stage == "FAILED"

    arun(go())


class FailingCas(MemoryStore):
    """Fused write that fails once with ``exc`` (then works)."""

    def __init__(self, rows, exc):
        super().__init__(rows)
        self.exc = exc

    async def cas_update(self, *a, **kw):
        if self.exc is not None:
            exc, self.exc = self.exc, None
            raise exc
        return await super().cas_update(*a, **kw)


def test_fused_delete_on_store_error_only_when_the_write_never_left(arun):
    """With ``compat.delete-on-read-error`` the fused path used
    to delete the Job whenever its conditional write failed — also on a timeout after which
    the write may have landed.  Now only a write that provably never reached the store
    (:class:`NotSent`) deletes; otherwise the retry (which sees the finished row) does."""
    from nexus_supervisor_amd.store.base import NotSent, StoreError

    async def case(exc):
        cfg = _cfg(compat={"delete-on-read-error": True})
        jobs = RecordingJobs([RUNNING_ROW.id])
        store = FailingCas([RUNNING_ROW], exc)
        c = InProcCluster(cfg, store, [make_job(RUNNING_ROW.id, cfg.labels)], jobs=jobs)
        await c.start()
        c.push(make_event("Job", RUNNING_ROW.id, "DeadlineExceeded", "deadline"))
        assert await c.settle(5)
        deleted_first = list(jobs.deleted)
        await c.stop()
        return deleted_first, store.get(ALGORITHM, RUNNING_ROW.id).lifecycle_stage

    async def go():
        # a timed-out write: no delete on the error; the retry writes, then deletes once
        deleted, stage = await case(StoreError("request timed out"))
        assert stage == LifecycleStage.DEADLINE_EXCEEDED and deleted == [RUNNING_ROW.id]
        # never sent: the reference's delete-on-error happens (and the retry's delete is NotFound-tolerant)
        deleted, stage = await case(NotSent("no CQL host available"))
        assert stage == LifecycleStage.DEADLINE_EXCEEDED and deleted[0] == RUNNING_ROW.id

    arun(go())
