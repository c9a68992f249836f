"""Failover safety, configurable
lifecycle stages (weak #5) and the label-mismatch warning (weak #13).

The reference runs every replica on every event with unconditional full-row upserts
(``/root/reference/services/supervisor.go:264-301``): a deposed or duplicate replica can
write a stale stage over a newer one.  Here a replica that loses its lease fences itself
(queued work dropped, in-flight work checks the epoch before writing, background DELETEs
cancelled) and writes are conditional (``IF lifecycle_stage IN (<unfinished>)``), so a
finished row — FAILED by the new leader, CANCELLED by another component — stays final."""
import asyncio
import datetime as dt

from nexus_supervisor_amd.config import load_config
from nexus_supervisor_amd.config.loader import from_mapping, to_mapping
from nexus_supervisor_amd.models import checkpoint as cp_mod
from nexus_supervisor_amd.models.checkpoint import LifecycleStage
from nexus_supervisor_amd.store.memory import MemoryStore
from nexus_supervisor_amd.testing.inproc import InProcCluster, RecordingJobs
from nexus_supervisor_amd.testing.seed import ALGORITHM, make_event, make_job, make_pod, seed_rows

BUFFERED_ROW = seed_rows()[0]  # BUFFERED
RUNNING_ROW = seed_rows()[1]   # RUNNING


class GatedStore(MemoryStore):
    """Memory store whose reads / writes can be held at a gate (a request 'on the wire')."""

    def __init__(self, rows):
        super().__init__(rows)
        self.read_gate = None
        self.write_gate = None
        self.at_read = asyncio.Event()
        self.at_write = asyncio.Event()

    async def read_checkpoint(self, algorithm, request_id):
        row = await super().read_checkpoint(algorithm, request_id)
        if self.read_gate is not None:
            self.at_read.set()
            await self.read_gate.wait()
        return row

    async def update_status(self, *a, **kw):
        if self.write_gate is not None:
            self.at_write.set()
            await self.write_gate.wait()
        return await super().update_status(*a, **kw)

    async def cas_update(self, *a, **kw):  # a ToRunning is one conditional write (no read first)
        if self.write_gate is not None:
            self.at_write.set()
            await self.write_gate.wait()
        return await super().cas_update(*a, **kw)


def _cfg(**over):
    """These tests pin the two-step (read, then write) actuation: the fused single-write path
    is covered by tests/test_fused_write.py."""
    base = {"cql-store-type": "memory", "rate-limit-elements-per-second": 0, "resync-period": "0s",
            "failure-rate-base-delay": "10ms", "failure-rate-max-delay": "50ms",
            "leader-election": {"enabled": True}, "compat": {"fused-write": False},
            # pod-less Job failures here: no wait for a pod update (tests/test_pod_rules.py covers it)
            "rules": {"job-pod-settle": "0s"}}
    over = dict(over)
    if "compat" in over:
        over["compat"] = dict(base["compat"], **over["compat"])
    base.update(over)
    return load_config(path=None, env={}, overrides=base)


def _started(cfg, row):
    pod = make_pod(row.id, cfg.labels, status={"phase": "Pending"})
    return pod, make_event("Pod", pod["metadata"]["name"], "Started", "Started container algorithm")


def _new_leader_writes(store, row, stage):
    store.rows[(row.algorithm, row.id)].lifecycle_stage = stage


def test_deposed_leader_in_flight_write_cannot_overwrite_new_leaders_failed(arun):
    """Old leader read BUFFERED for a ToRunning and its write is on the wire when the lease
    is lost; the new leader writes FAILED; the old write lands afterwards and is refused by
    the conditional write.  Row stays FAILED."""
    async def go():
        cfg = _cfg()
        store = GatedStore([BUFFERED_ROW])
        pod, ev = _started(cfg, BUFFERED_ROW)
        c = InProcCluster(cfg, store, [pod, make_job(BUFFERED_ROW.id, cfg.labels)])
        await c.start()
        c.supervisor.set_active(True)
        store.write_gate = asyncio.Event()
        c.push(ev)
        await asyncio.wait_for(store.at_write.wait(), 5)
        c.supervisor.set_active(False)  # lease lost while the write is on the wire
        _new_leader_writes(store, BUFFERED_ROW, LifecycleStage.FAILED)
        store.write_gate.set()
        assert await c.settle(5)
        assert store.get(ALGORITHM, BUFFERED_ROW.id).lifecycle_stage == LifecycleStage.FAILED
        assert c.decisions[-1].outcome == "skipped-finished"
        assert c.supervisor.metrics.counter("conditional_write_rejected") == 1
        await c.stop()

    arun(go())


def test_deposed_leader_dequeued_decision_is_fenced_before_write(arun):
    """The lease is lost while the old leader's decision sits between read and write: the
    epoch check stops it before any write or DELETE is issued."""
    async def go():
        cfg = _cfg()
        store = GatedStore([RUNNING_ROW])
        jobs = RecordingJobs([RUNNING_ROW.id])
        job = make_job(RUNNING_ROW.id, cfg.labels)
        c = InProcCluster(cfg, store, [job], jobs=jobs)
        await c.start()
        c.supervisor.set_active(True)
        store.read_gate = asyncio.Event()
        c.push(make_event("Job", RUNNING_ROW.id, "DeadlineExceeded", "Job was active longer than specified deadline"))
        await asyncio.wait_for(store.at_read.wait(), 5)
        c.supervisor.set_active(False)
        _new_leader_writes(store, RUNNING_ROW, LifecycleStage.CANCELLED)
        store.read_gate.set()
        assert await c.settle(5)
        assert store.get(ALGORITHM, RUNNING_ROW.id).lifecycle_stage == LifecycleStage.CANCELLED
        assert store.writes == 0 and jobs.deleted == []
        assert [d.outcome for d in c.decisions] == ["fenced"]
        await c.stop()

    arun(go())


def test_fencing_drops_queued_and_backing_off_decisions_and_cancels_deletes(arun):
    async def go():
        cfg = _cfg(workers=1)
        rows = seed_rows()
        store = GatedStore(rows)
        jobs = RecordingJobs([r.id for r in rows], latency=0.2)
        objs = [make_job(r.id, cfg.labels) for r in rows]
        c = InProcCluster(cfg, store, objs, jobs=jobs)
        await c.start()
        c.supervisor.set_active(True)
        sup = c.supervisor
        # first decision: written, its background DELETE in flight (0.2 s)
        c.push(make_event("Job", rows[1].id, "DeadlineExceeded", "deadline"))
        for _ in range(200):
            if sup._deletes:
                break
            await asyncio.sleep(0.005)
        assert sup._deletes
        # the single worker is held on a read; two more decisions queue behind it
        store.read_gate = asyncio.Event()
        for r in (rows[2], rows[4]):
            c.push(make_event("Job", r.id, "PodFailurePolicy", "exit 137"))
        await asyncio.wait_for(store.at_read.wait(), 5)
        await asyncio.sleep(0.05)
        assert sup.pipeline.depth() >= 2
        sup.active = False
        dropped = sup.fence()  # what set_active(False) does
        store.read_gate.set()
        await asyncio.sleep(0.3)
        assert dropped >= 1 and sup.pipeline.depth() == 0 and not sup._deletes
        assert jobs.deleted == []  # the in-flight DELETE was cancelled before the API saw it
        assert store.get(ALGORITHM, rows[2].id).lifecycle_stage == "RUNNING"
        assert store.get(ALGORITHM, rows[4].id).lifecycle_stage == "RUNNING"
        assert sup.metrics.counter("fenced_decisions_dropped") == dropped
        await c.stop()

    arun(go())


def test_third_party_cancelled_wins_over_in_flight_to_running(arun):
    """No failover at all (a single active replica): CANCELLED written by another Nexus
    component while a ToRunning is on the wire stays CANCELLED (ToRunning is conditional
    by default)."""
    async def go():
        cfg = _cfg(**{"leader-election": {"enabled": False}})
        store = GatedStore([BUFFERED_ROW])
        pod, ev = _started(cfg, BUFFERED_ROW)
        c = InProcCluster(cfg, store, [pod])
        await c.start()
        store.write_gate = asyncio.Event()
        c.push(ev)
        await asyncio.wait_for(store.at_write.wait(), 5)
        _new_leader_writes(store, BUFFERED_ROW, LifecycleStage.CANCELLED)
        store.write_gate.set()
        assert await c.settle(5)
        assert store.get(ALGORITHM, BUFFERED_ROW.id).lifecycle_stage == LifecycleStage.CANCELLED
        await c.stop()

    arun(go())


def test_reference_mode_never_conditional():
    cfg = _cfg(compat={"conditional-update": "false"})
    assert cfg.compat.conditional_update == "never"
    assert _cfg(compat={"conditional-update": True}).compat.conditional_update == "always"


def test_background_delete_outlives_the_retry_budget(arun):
    """An API outage longer than max-retries must not leak the Job — the key is
    marked finished, so the background DELETE is the only thing left that removes it."""
    async def go():
        cfg = _cfg(**{"leader-election": {"enabled": False}, "max-retries": 3})
        store = MemoryStore([RUNNING_ROW])
        jobs = RecordingJobs([RUNNING_ROW.id])
        jobs.fail_next = 8  # > max-retries
        c = InProcCluster(cfg, store, [make_job(RUNNING_ROW.id, cfg.labels)], jobs=jobs)
        await c.start()
        c.push(make_event("Job", RUNNING_ROW.id, "DeadlineExceeded", "deadline"))
        for _ in range(300):
            if RUNNING_ROW.id in jobs.deleted:
                break
            await asyncio.sleep(0.02)
        assert store.get(ALGORITHM, RUNNING_ROW.id).lifecycle_stage == LifecycleStage.DEADLINE_EXCEEDED
        assert jobs.deleted == [RUNNING_ROW.id] and jobs.fail_next == 0
        assert c.supervisor.metrics.counter("job_deletes_slow") == 1
        await c.stop()

    arun(go(), timeout=30)


# ----------------------------------------------------------------------------- stages

def test_stage_strings_and_finished_set_from_yaml_and_env(tmp_path):
    p = tmp_path / "appconfig.yaml"
    p.write_text("cql-store-type: memory\nstages:\n  failed: FAILED_V2\n  finished: ''\n")
    try:
        cfg = load_config(path=str(p), env={"NEXUS__STAGES__CANCELLED": "ABORTED"})
        assert cfg.stages.failed == "FAILED_V2" and cfg.stages.cancelled == "ABORTED"
        cfg.stages.apply()
        assert LifecycleStage.FAILED == "FAILED_V2"
        # only the mapping given: the finished set follows the remapped strings
        assert cp_mod.finished_stages() == {"COMPLETED", "FAILED_V2", "SCHEDULING_FAILED", "DEADLINE_EXCEEDED", "ABORTED"}
        assert cp_mod.unfinished_stages() == ("NEW", "BUFFERED", "RUNNING")
        cfg2 = from_mapping(to_mapping(cfg))  # the hand-off to shard-worker processes keeps it
        assert cfg2.stages.failed == "FAILED_V2" and cfg2.stages.cancelled == "ABORTED"
    finally:
        load_config(path=None, env={}).stages.apply()
    assert LifecycleStage.FAILED == "FAILED" and "FAILED_V2" not in cp_mod.finished_stages()


def test_supervisor_honours_remapped_stages(arun):
    async def go():
        cfg = _cfg(**{"leader-election": {"enabled": False}},
                   stages={"failed": "FAILED_V2", "running": "IN_PROGRESS",
                           "finished": ["FAILED_V2", "CANCELLED", "COMPLETED", "SCHEDULING_FAILED", "DEADLINE_EXCEEDED",
                                        "ARCHIVED"]})
        try:
            rows = seed_rows()
            rows[1].lifecycle_stage = "IN_PROGRESS"
            rows[2].lifecycle_stage = "ARCHIVED"  # finished by config: never touched
            store = MemoryStore(rows)
            objs = [make_job(r.id, cfg.labels) for r in rows[1:3]]
            c = InProcCluster(cfg, store, objs)
            await c.start()
            c.push(make_event("Job", rows[1].id, "PodFailurePolicy", "exit 137"))
            c.push(make_event("Job", rows[2].id, "PodFailurePolicy", "exit 137"))
            assert await c.settle(5)
            assert store.get(ALGORITHM, rows[1].id).lifecycle_stage == "FAILED_V2"
            assert store.get(ALGORITHM, rows[2].id).lifecycle_stage == "ARCHIVED"
            await c.stop()
        finally:
            load_config(path=None, env={}).stages.apply()

    arun(go())


def test_stages_validation():
    import pytest

    from nexus_supervisor_amd.config.schema import ConfigError

    with pytest.raises(ConfigError):
        load_config(path=None, env={}, overrides={"stages": {"failed": "RUNNING"}})
    with pytest.raises(ConfigError):
        load_config(path=None, env={}, overrides={"stages": {"finished": ["RUNNING", "FAILED"]}})


def test_stages_across_worker_processes(arun, tmp_path):
    """Two shard-worker processes receive the stages section through the config hand-off
    and write the remapped strings."""
    from nexus_supervisor_amd.app import ShardedApplication
    from nexus_supervisor_amd.store.cql import CqlCheckpointStore, CqlSession
    from nexus_supervisor_amd.testing.cqlsrv import CqlServer
    from nexus_supervisor_amd.testing.fake_apiserver import FakeApiServer
    from nexus_supervisor_amd.testing.seed import seed_cql_statements

    srv = CqlServer(exec_statements=seed_cql_statements()).start()

    async def go():
        api = FakeApiServer(bookmark_interval=0.1)
        url = await api.start()
        rows = seed_rows()
        targets = [rows[1], rows[2], rows[4]]  # RUNNING rows
        import json

        kc = tmp_path / "kubeconfig"
        kc.write_text(json.dumps({"clusters": [{"name": "c", "cluster": {"server": url}}],
                                  "contexts": [{"name": "x", "context": {"cluster": "c"}}], "current-context": "x"}))
        cfg = load_config(path=None, env={}, overrides={
            "cql-store-type": "scylla", "rate-limit-elements-per-second": 0, "resync-period": "0s",
            "kube-config-path": str(kc), "scylla-cql-store": {"hosts": f"127.0.0.1:{srv.port}"},
            "runtime": {"worker-processes": 2}, "stages": {"deadline-exceeded": "TIMED_OUT"}})
        for r in targets:
            api.create(make_job(r.id, cfg.labels))
        app = ShardedApplication(cfg)
        try:
            await app.start()
            assert await app.wait_for_cache_sync(20)
            for r in targets:
                api.create(make_event("Job", r.id, "DeadlineExceeded", "deadline"))
            st = CqlCheckpointStore(CqlSession([srv.address]))
            await st.connect()
            got = {}
            for _ in range(200):
                got = {r.id: (await st.read_checkpoint(ALGORITHM, r.id)).lifecycle_stage for r in targets}
                if all(v == "TIMED_OUT" for v in got.values()):
                    break
                await asyncio.sleep(0.05)
            await st.close()
            assert all(v == "TIMED_OUT" for v in got.values()), got
            assert LifecycleStage.DEADLINE_EXCEEDED == "DEADLINE_EXCEEDED"  # the parent process is untouched
        finally:
            await app.stop()
            await api.stop()

    try:
        arun(go(), timeout=60)
    finally:
        srv.stop()


# ----------------------------------------------------------------------------- label mismatch

def test_label_mismatch_warning(arun):
    async def go():
        cfg = _cfg(**{"leader-election": {"enabled": False}})
        events = [make_event("Pod", f"other-{i}", "Started", "x") for i in range(4)]
        c = InProcCluster(cfg, MemoryStore(), events)
        await c.start()
        sup = c.supervisor
        sup._check_labels(0.0)
        assert sup.label_mismatch and sup.metrics.gauge("label_selector_mismatch") == 1.0
        c.push(make_job("x", cfg.labels))
        await asyncio.sleep(0.05)
        sup._check_labels(0.0)
        assert not sup.label_mismatch and sup.metrics.gauge("label_selector_mismatch") == 0.0
        await c.stop()

    arun(go())


def test_no_label_mismatch_alarm_for_a_shard_replica_holding_nothing(arun):
    """Lease-mode shard replica that holds no shard (yet): its Pod/Job caches are empty by
    design while the namespace's Events name Pods — not a selector mismatch (seen as a false
    alarm in the 3-replica chaos scenario)."""
    async def go():
        cfg = _cfg(**{"leader-election": {"enabled": False}, "sharding": {"shards": 4, "mode": "lease"}})
        events = [make_event("Pod", f"other-{i}", "Started", "x") for i in range(4)]
        c = InProcCluster(cfg, MemoryStore(), events)
        await c.start()
        sup = c.supervisor
        assert sup.shards.owned is not None and not sup.shards.owned
        sup._check_labels(0.0)
        assert not sup.label_mismatch
        await c.stop()

    arun(go())


def test_unknown_yaml_keys_are_tolerated_with_a_warning(tmp_path, caplog):
    """viper tolerates unknown keys (a reference appconfig with extra keys must start);
    this build logs them and refuses only in strict mode."""
    import logging

    import pytest

    from nexus_supervisor_amd.config.schema import ConfigError

    p = tmp_path / "appconfig.yaml"
    p.write_text("cql-store-type: memory\nsome-future-key: 1\ngpu:\n  not-a-knob: x\n")
    with caplog.at_level(logging.WARNING):
        cfg = load_config(path=str(p), env={})
    assert cfg.cql_store_type == "memory"
    assert "some-future-key" in caplog.text and "gpu.not-a-knob" in caplog.text
    with pytest.raises(ConfigError):
        load_config(path=str(p), env={"NEXUS_CONFIG_STRICT": "1"})
