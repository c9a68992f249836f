"""Pod/Job status rules beyond the reference event table (SURVEY §2.9.1 gaps, M4):
OOMKilled, HBM-OOM, ImagePullBackOff, CreateContainerConfigError, CrashLoopBackOff,
Evicted (fail / observe→enrich), Unschedulable timeout, lost-event Job conditions and
lost Started events, Event repeat-count updates, and per-run ordering."""
import json

import pytest

from nexus_supervisor_amd.config import load_config
from nexus_supervisor_amd.models import LifecycleStage as S
from nexus_supervisor_amd.store.memory import MemoryStore
from nexus_supervisor_amd.testing.inproc import InProcCluster
from nexus_supervisor_amd.testing.seed import ALGORITHM, make_event, make_job, make_pod, seed_rows

RUNNING_ROW = seed_rows()[1]          # RUNNING
BUFFERED_ROW = seed_rows()[0]         # BUFFERED
RID = RUNNING_ROW.id
BID = BUFFERED_ROW.id


def _cfg(**over):
    base = {"cql-store-type": "memory", "workers": 4, "rate-limit-elements-per-second": 0, "resync-period": "0s"}
    base.update(over)
    return load_config(path=None, env={}, overrides=base)


def _status(state, phase="Failed", **extra):
    st = {"phase": phase, "containerStatuses": [{"name": "algorithm", "restartCount": 0, "state": state}]}
    st.update(extra)
    return st


async def _run(cfg, objects, updates, rows=(RUNNING_ROW, BUFFERED_ROW)):
    store = MemoryStore(rows)
    c = InProcCluster(cfg, store, objects)
    await c.start()
    for etype, obj in updates:
        c.push(obj, etype)
        assert await c.settle(5)
    await c.stop()
    return store, c


def _failed_pod(labels, rid, status, rv="5", **kw):
    p = make_pod(rid, labels, rv=rv, **kw)
    p["status"] = status
    return p


def _trace(row):
    return json.loads(row.algorithm_failure_details)


def test_oomkilled_pod_is_host_oom(arun):
    cfg = _cfg()
    pod = make_pod(RID, cfg.labels, gpus=1, env={"RANK": "2", "WORLD_SIZE": "8", "LOCAL_RANK": "2"})
    upd = _failed_pod(cfg.labels, RID, _status({"terminated": {"reason": "OOMKilled", "exitCode": 137}}), gpus=1,
                      env={"RANK": "2", "WORLD_SIZE": "8", "LOCAL_RANK": "2"})
    store, c = arun(_run(cfg, [pod, make_job(RID, cfg.labels)], [("MODIFIED", upd)]))
    row = store.get(ALGORITHM, RID)
    assert row.lifecycle_stage == S.FAILED
    assert row.algorithm_failure_cause == ("Algorithm encountered a fatal error during execution: "
                                           "Algorithm container was OOMKilled: host memory limit exceeded.")
    t = _trace(row)
    assert t["class"] == "host-oom" and t["oom"]["kind"] == "host" and t["topology"]["rank"] == 2
    assert c.jobs.deleted == [RID]


def test_hip_oom_message_is_hbm_oom(arun):
    cfg = _cfg()
    msg = ("torch.OutOfMemoryError: HIP out of memory. Tried to allocate 12.00 GiB. GPU 3 has a total capacity of "
           "287.98 GiB of which 1.02 GiB is free.")
    upd = _failed_pod(cfg.labels, RID, _status({"terminated": {"reason": "Error", "exitCode": 1, "message": msg}}),
                      gpus=1)
    store, _ = arun(_run(cfg, [make_pod(RID, cfg.labels, gpus=1)], [("MODIFIED", upd)]))
    t = _trace(store.get(ALGORITHM, RID))
    assert t["class"] == "hbm-oom" and t["oom"]["gpu_index"] == 3 and t["oom"]["requested_bytes"] == 12 << 30


def test_gpu_failures_are_counted_per_physical_gpu(arun):
    """gpu_failures{node,gpu,class}: an HBM-OOM on node n7 GPU 3 and a GPU fault (VM fault
    in the node agent's evidence) on GPU 5 — the counters an alert finds a bad GPU with."""
    cfg = _cfg()
    msg = "torch.OutOfMemoryError: HIP out of memory. GPU 3 has a total capacity of 287.98 GiB"
    a = _failed_pod(cfg.labels, RID, _status({"terminated": {"reason": "Error", "exitCode": 1, "message": msg}}),
                    node="n7", gpus=1)
    ev = {"source": "agent", "node": "n7", "gpus": [{"index": 5, "vram_total_mb": 294896, "vram_peak_mb": 1000,
                                                     "events": [{"type": "VMFAULT", "t": 1.0}]}]}
    b = _failed_pod(cfg.labels, BID, _status({"terminated": {"reason": "Error", "exitCode": 134}}), node="n7",
                    gpus=1, annotations={"nexus.amd.com/gpu-evidence": json.dumps(ev)})
    store, c = arun(_run(cfg, [make_pod(RID, cfg.labels, node="n7", gpus=1), make_pod(BID, cfg.labels, node="n7", gpus=1)],
                         [("MODIFIED", a), ("MODIFIED", b)]))
    got = {dict(k)["gpu"] + "/" + dict(k)["class"]: v for k, v in c.supervisor.metrics.counters["gpu_failures"].items()}
    assert got == {"3/hbm-oom": 1, "5/gpu-fault": 1}
    assert {dict(k)["node"] for k in c.supervisor.metrics.counters["gpu_failures"]} == {"n7"}


@pytest.mark.parametrize("reason,stage,klass", [
    ("ImagePullBackOff", S.SCHEDULING_FAILED, "image-pull"),
    ("ErrImagePull", S.SCHEDULING_FAILED, "image-pull"),
    ("CreateContainerConfigError", S.SCHEDULING_FAILED, "config"),
    ("CrashLoopBackOff", S.FAILED, "crash-loop"),
])
def test_waiting_reasons(arun, reason, stage, klass):
    cfg = _cfg()
    upd = _failed_pod(cfg.labels, BID, _status({"waiting": {"reason": reason, "message": "back-off"}}, phase="Pending"))
    store, _ = arun(_run(cfg, [make_pod(BID, cfg.labels)], [("MODIFIED", upd)]))
    row = store.get(ALGORITHM, BID)
    assert row.lifecycle_stage == stage
    assert _trace(row)["class"] == klass


def test_evicted_fail_policy(arun):
    cfg = _cfg(**{"rules": {"evicted-policy": "fail"}})
    upd = make_pod(RID, cfg.labels, rv="5", status={"phase": "Failed", "reason": "Evicted",
                                                     "message": "The node was low on resource: memory."})
    store, _ = arun(_run(cfg, [make_pod(RID, cfg.labels)], [("MODIFIED", upd)]))
    row = store.get(ALGORITHM, RID)
    assert row.lifecycle_stage == S.FAILED and _trace(row)["class"] == "evicted"


def test_evicted_observe_then_backoff_limit_is_attributed(arun):
    cfg = _cfg()  # default evicted-policy: observe
    evicted = make_pod(RID, cfg.labels, rv="5", status={"phase": "Failed", "reason": "Evicted", "message": "low memory"})
    job = make_job(RID, cfg.labels, rv="6")
    job_failed = make_job(RID, cfg.labels, rv="7", conditions=[{"type": "Failed", "status": "True",
                                                                "reason": "BackoffLimitExceeded", "message": "limit"}])
    store, _ = arun(_run(cfg, [make_pod(RID, cfg.labels), job], [("MODIFIED", evicted)]))
    assert store.get(ALGORITHM, RID).lifecycle_stage == S.RUNNING  # eviction alone decides nothing
    store2, c = arun(_run(cfg, [make_pod(RID, cfg.labels), job], [("MODIFIED", evicted), ("MODIFIED", job_failed)]))
    row = store2.get(ALGORITHM, RID)
    # the same row evicted-policy "fail" writes (rules.oom-fails-backoff-job, default on)
    assert row.lifecycle_stage == S.FAILED
    assert row.algorithm_failure_cause == ("Algorithm encountered a fatal error during execution: "
                                           "Algorithm pod was evicted from its node.")
    t = _trace(row)
    assert t["class"] == "evicted" and t["history"][0]["kind"] == "evicted"
    # the compat switch off keeps the reference's stage for BackoffLimitExceeded
    cfg3 = _cfg(**{"rules": {"oom-fails-backoff-job": False}})
    store3, _ = arun(_run(cfg3, [make_pod(RID, cfg3.labels), job], [("MODIFIED", evicted), ("MODIFIED", job_failed)]))
    row3 = store3.get(ALGORITHM, RID)
    assert row3.lifecycle_stage == S.DEADLINE_EXCEEDED and _trace(row3)["class"] == "evicted"


def test_eviction_storm_rows_name_the_eviction(arun):
    """An eviction storm under both policies: every run's row ends FAILED with the eviction
    cause — at the eviction itself (fail) or at the Job's BackoffLimitExceeded (observe)."""
    rows = [type(RUNNING_ROW)(algorithm=ALGORITHM, id=f"storm-{i:02d}", lifecycle_stage="RUNNING") for i in range(20)]
    for policy in ("fail", "observe"):
        cfg = _cfg(**{"rules": {"evicted-policy": policy}})
        objs, upd = [], []
        for r in rows:
            objs += [make_pod(r.id, cfg.labels), make_job(r.id, cfg.labels, rv="6")]
            upd.append(("MODIFIED", make_pod(r.id, cfg.labels, rv="7", status={
                "phase": "Failed", "reason": "Evicted", "message": "The node was low on resource: memory."})))
            if policy == "observe":
                upd.append(("MODIFIED", make_job(r.id, cfg.labels, rv="8", conditions=[
                    {"type": "Failed", "status": "True", "reason": "BackoffLimitExceeded", "message": "limit"}])))
        store, _ = arun(_run(cfg, objs, upd, rows=rows))
        for r in rows:
            row = store.get(ALGORITHM, r.id)
            assert row.lifecycle_stage == S.FAILED, (policy, r.id, row.lifecycle_stage)
            assert row.algorithm_failure_cause.endswith("Algorithm pod was evicted from its node."), (policy, row)


def test_unschedulable_timeout(arun):
    cfg = _cfg(**{"rules": {"unschedulable-timeout": "1s"}})
    pod = make_pod(BID, cfg.labels, rv="5", status={"phase": "Pending", "conditions": [
        {"type": "PodScheduled", "status": "False", "reason": "Unschedulable",
         "message": "0/8 nodes are available: 8 Insufficient amd.com/gpu."}]})
    pod["metadata"]["creationTimestamp"] = "2020-01-01T00:00:00Z"
    store, _ = arun(_run(cfg, [make_pod(BID, cfg.labels)], [("MODIFIED", pod)]))
    row = store.get(ALGORITHM, BID)
    assert row.lifecycle_stage == S.SCHEDULING_FAILED and "amd.com/gpu" in _trace(row)["message"]
    store2, _ = arun(_run(_cfg(), [make_pod(BID, cfg.labels)], [("MODIFIED", pod)]))
    assert store2.get(ALGORITHM, BID).lifecycle_stage == S.BUFFERED  # timeout 0 = never


def test_job_failed_condition_without_event(arun):
    cfg = _cfg()
    job = make_job(RID, cfg.labels, rv="9", conditions=[{"type": "Failed", "status": "True", "reason": "DeadlineExceeded",
                                                         "message": "Job was active longer than specified deadline"}])
    store, _ = arun(_run(cfg, [make_job(RID, cfg.labels)], [("MODIFIED", job)]))
    row = store.get(ALGORITHM, RID)
    assert row.lifecycle_stage == S.DEADLINE_EXCEEDED
    assert row.algorithm_failure_cause == "Algorithm exceeded its max allowed run time limit or retry attempt count."


def test_running_status_without_started_event(arun):
    cfg = _cfg()
    upd = _failed_pod(cfg.labels, BID, _status({"running": {"startedAt": "2026-01-01T00:00:00Z"}}, phase="Running"))
    store, _ = arun(_run(cfg, [make_pod(BID, cfg.labels)], [("MODIFIED", upd)]))
    assert store.get(ALGORITHM, BID).lifecycle_stage == S.RUNNING


def test_failed_then_backoff_same_run_is_deterministic(arun):
    """Two reference pod events for one run (no per-key ordering in the
    reference) — the per-run FIFO makes the first decision win every time."""
    cfg = _cfg()
    pod = make_pod(BID, cfg.labels)
    failed = make_event("Pod", pod["metadata"]["name"], "Failed", "Error: ErrImagePull")
    backoff = make_event("Pod", pod["metadata"]["name"], "BackOff", "Back-off restarting failed container")
    for _ in range(5):
        store = MemoryStore([BUFFERED_ROW])
        c = InProcCluster(cfg, store, [pod, make_job(BID, cfg.labels)])

        async def go():
            await c.start()
            c.push(failed)
            c.push(backoff)
            assert await c.settle(5)
            await c.stop()

        arun(go())
        assert store.get(ALGORITHM, BID).lifecycle_stage == S.SCHEDULING_FAILED
        assert [d.outcome for d in c.decisions] in (["applied", "skipped-finished"], ["applied"])


def test_event_repeat_count_update_is_handled(arun):
    cfg = _cfg()
    ev = make_event("Job", RID, "Tagged", "noise")
    ev2 = json.loads(json.dumps(ev))
    ev2["reason"] = "DeadlineExceeded"
    ev2["count"] = 2
    ev2["metadata"]["resourceVersion"] = "99"
    store, _ = arun(_run(cfg, [make_job(RID, cfg.labels)], [("ADDED", ev), ("MODIFIED", ev2)]))
    assert store.get(ALGORITHM, RID).lifecycle_stage == S.DEADLINE_EXCEEDED
    store2, _ = arun(_run(_cfg(**{"rules": {"handle-event-updates": False}}), [make_job(RID, cfg.labels)],
                          [("ADDED", ev), ("MODIFIED", ev2)]))
    assert store2.get(ALGORITHM, RID).lifecycle_stage == S.RUNNING  # reference behaviour: AddFunc only


def test_running_sweep_after_restart_when_started_event_expired(arun):
    """a pod already running at the initial LIST whose Started Event expired
    while the supervisor was down (Event TTL) never produced ToRunning; the running sweep
    decides it after the caches synced — but not runs whose Started Event is cached (the
    replay decides those), pods being deleted, or pending pods."""
    cfg = _cfg(**{"rules": {"running-sweep-rate": 50, "running-sweep-delay": "0s"}})
    running = _status({"running": {"startedAt": "2026-01-01T00:00:00Z"}}, phase="Running")
    expired = make_pod(BID, cfg.labels, status=running)                       # no Started Event left
    rows = [BUFFERED_ROW] + [type(BUFFERED_ROW)(algorithm=ALGORITHM, id=f"sweep-{i}", lifecycle_stage="BUFFERED")
                             for i in range(3)]
    replayed = make_pod("sweep-0", cfg.labels, status=running)
    deleting = make_pod("sweep-1", cfg.labels, status=running)
    deleting["metadata"]["deletionTimestamp"] = "2026-01-01T00:00:00Z"
    pending = make_pod("sweep-2", cfg.labels, status={"phase": "Pending"})
    started_ev = make_event("Pod", replayed["metadata"]["name"], "Started", "Started container algorithm")

    async def go():
        store = MemoryStore(rows)
        c = InProcCluster(cfg, store, [expired, replayed, deleting, pending, started_ev])
        await c.start()
        for _ in range(100):
            if store.get(ALGORITHM, BID).lifecycle_stage == S.RUNNING:
                break
            await asyncio.sleep(0.02)
        await asyncio.sleep(0.2)
        await c.stop()
        return store, c

    import asyncio

    store, c = arun(go())
    assert store.get(ALGORITHM, BID).lifecycle_stage == S.RUNNING          # the sweep
    assert store.get(ALGORITHM, "sweep-0").lifecycle_stage == S.RUNNING    # the replayed Started Event
    assert store.get(ALGORITHM, "sweep-1").lifecycle_stage == "BUFFERED"   # being deleted
    assert store.get(ALGORITHM, "sweep-2").lifecycle_stage == "BUFFERED"   # not running
    assert c.supervisor.metrics.counter("running_sweep_decisions") == 1
    # off: the reference's behaviour (nothing moves the expired run)
    cfg0 = _cfg(**{"rules": {"running-sweep-rate": 0}})
    store0 = MemoryStore([BUFFERED_ROW])

    async def go0():
        c0 = InProcCluster(cfg0, store0, [make_pod(BID, cfg0.labels, status=running)])
        await c0.start()
        await asyncio.sleep(0.2)
        await c0.stop()

    arun(go0())
    assert store0.get(ALGORITHM, BID).lifecycle_stage == "BUFFERED"
