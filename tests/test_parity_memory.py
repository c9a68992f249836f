"""Reference parity suite, in-process.

Mirrors ``/root/reference/services/supervisor_test.go:542-580``: the same 8
runs, the same seeded stages, the same expected end stages — but with
deterministic settling instead of fixed sleeps.
"""
import pytest

from nexus_supervisor_amd.classify import reference_rules as R
from nexus_supervisor_amd.config import load_config
from nexus_supervisor_amd.models import LifecycleStage
from nexus_supervisor_amd.store.memory import MemoryStore
from nexus_supervisor_amd.testing.inproc import InProcCluster
from nexus_supervisor_amd.testing.seed import ALGORITHM, reference_scenarios, seed_rows


def _cfg(**over):
    # reference test processing config: 100ms/1s backoff, 10 eps, burst 10, 4 workers (supervisor_test.go:553-559)
    base = {"cql-store-type": "memory", "workers": 4, "rate-limit-elements-per-second": 10,
            "rate-limit-elements-burst": 10, "failure-rate-base-delay": "100ms", "failure-rate-max-delay": "1s"}
    base.update(over)
    return load_config(path=None, env={}, overrides=base)


async def _run_all(cfg, scenarios):
    store = MemoryStore(seed_rows())
    objs = [o for s in scenarios for o in s.objects]
    cluster = InProcCluster(cfg, store, objs)
    await cluster.start()
    assert await cluster.settle(10)
    await cluster.stop()
    return store, cluster


def test_reference_scenarios_end_stages(arun):
    scenarios = reference_scenarios()
    store, cluster = arun(_run_all(_cfg(), scenarios))
    for s in scenarios:
        for rid, stage in s.expected.items():
            row = store.get(ALGORITHM, rid)
            assert row is not None, rid
            assert row.lifecycle_stage == stage, (s.name, rid, row.lifecycle_stage)


def test_failure_cause_strings_byte_exact(arun):
    scenarios = reference_scenarios()
    store, cluster = arun(_run_all(_cfg(), scenarios))
    by = {s.name: s.request_ids for s in scenarios}
    fc = store.get(ALGORITHM, by["failed-create"][0])
    assert fc.algorithm_failure_cause == (
        "Algorithm submission was buffered, but failed to launch on the target cluster: "
        "Unable to launch a container for the algorithm - please review configuration and try again.")
    assert fc.algorithm_failure_details == ""
    oom = store.get(ALGORITHM, by["pod-failure-policy-oom"][0])
    # reference doubles the sentence (supervisor.go:198,325)
    assert oom.algorithm_failure_cause == (
        "Algorithm encountered a fatal error during execution: Algorithm encountered a fatal error during execution.")
    for rid in by["deadline-and-backoff"]:
        assert store.get(ALGORITHM, rid).algorithm_failure_cause == R.MSG_DEADLINE
    pb = store.get(ALGORITHM, by["pod-backoff"][0])
    assert pb.algorithm_failure_cause == "Algorithm encountered a fatal error during execution: BackOff"
    pf = store.get(ALGORITHM, by["pod-failed"][0])
    assert pf.algorithm_failure_cause.endswith(": Failed")


def test_jobs_deleted_only_for_failures(arun):
    scenarios = reference_scenarios()
    store, cluster = arun(_run_all(_cfg(), scenarios))
    by = {s.name: s.request_ids for s in scenarios}
    deleted = set(cluster.jobs.deleted)
    for name in ("failed-create", "deadline-and-backoff", "pod-failure-policy-oom", "pod-failed", "pod-backoff"):
        for rid in by[name]:
            assert rid in deleted, name
    assert by["pod-started"][0] not in deleted
    assert by["started-after-cancel"][0] not in deleted  # finished → skipped before delete


def test_cancelled_is_untouched(arun):
    scenarios = reference_scenarios()
    store, cluster = arun(_run_all(_cfg(), scenarios))
    cid = [s for s in scenarios if s.name == "started-after-cancel"][0].request_ids[0]
    before = [r for r in seed_rows() if r.id == cid][0]
    after = store.get(ALGORITHM, cid)
    assert after == before


def test_rerun_is_idempotent(arun):
    """The reference test re-runs without re-seeding: end states are stable."""
    scenarios = reference_scenarios()

    async def twice():
        store = MemoryStore(seed_rows())
        objs = [o for s in scenarios for o in s.objects]
        for _ in range(2):
            c = InProcCluster(_cfg(), store, objs)
            await c.start()
            assert await c.settle(10)
            await c.stop()
        return store

    store = arun(twice())
    for s in scenarios:
        for rid, stage in s.expected.items():
            assert store.get(ALGORITHM, rid).lifecycle_stage == stage


def test_full_row_upsert_compat_mode(arun):
    scenarios = reference_scenarios()
    store, _ = arun(_run_all(_cfg(compat={"full-row-upsert": True}), scenarios))
    for s in scenarios:
        for rid, stage in s.expected.items():
            assert store.get(ALGORITHM, rid).lifecycle_stage == stage


def test_owned_columns_update_preserves_other_columns(arun):
    scenarios = reference_scenarios()
    store, _ = arun(_run_all(_cfg(), scenarios))
    seeds = {r.id: r for r in seed_rows()}
    for s in scenarios:
        for rid in s.expected:
            after = store.get(ALGORITHM, rid)
            before = seeds[rid]
            for col in ("payload_uri", "received_by_host", "received_at", "content_hash", "tag", "job_uid", "payload_valid_for"):
                assert getattr(after, col) == getattr(before, col), (rid, col)


def test_unknown_reasons_are_noops(arun):
    from nexus_supervisor_amd.config.schema import LabelConfig
    from nexus_supervisor_amd.testing.seed import make_event, make_job, make_pod

    labels = LabelConfig()
    rid = seed_rows()[0].id
    objs = [make_job(rid, labels), make_pod(rid, labels), make_event("Job", rid, "SuccessfulCreate"),
            make_event("Pod", f"{rid}-acdey", "Pulling"), make_event("Pod", f"{rid}-acdey", "Killing")]

    async def go():
        store = MemoryStore(seed_rows())
        c = InProcCluster(_cfg(), store, objs)
        await c.start()
        assert await c.settle(5)
        await c.stop()
        return store

    store = arun(go())
    assert store.get(ALGORITHM, rid).lifecycle_stage == LifecycleStage.BUFFERED
