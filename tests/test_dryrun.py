"""Shadow mode (``dry-run: true``, :mod:`nexus_supervisor_amd.dryrun`): the reference
parity scenarios over HTTP watch + CQL decide exactly as they do live, but no row is
written and no Job is deleted; each would-be action is logged and counted."""
import datetime as dt
import io

from nexus_supervisor_amd.dryrun import DryRunJobs, DryRunStore
from nexus_supervisor_amd.obs.logging import KLogger
from nexus_supervisor_amd.obs.metrics import Metrics
from nexus_supervisor_amd.store.memory import MemoryStore
from nexus_supervisor_amd.testing.inproc import RecordingJobs
from nexus_supervisor_amd.testing.seed import ALGORITHM, reference_scenarios, seed_rows

from test_kube_wire import _cfg, _settle, _wire_cluster

NOW = dt.datetime(2026, 1, 1, tzinfo=dt.timezone.utc)


def _counter(m: Metrics, name: str) -> float:
    return sum((m.counters.get(name) or {}).values())


def test_dry_run_store_answers_like_the_store_without_writing(arun):
    async def go():
        inner = MemoryStore(seed_rows())
        m = Metrics("t")
        log = KLogger()  # (configure_logging would detach the package logger from caplog for later tests)
        s = DryRunStore(inner, log, m)
        running = next(r for r in seed_rows() if r.lifecycle_stage == "RUNNING")
        cancelled = next(r for r in seed_rows() if r.lifecycle_stage == "CANCELLED")
        assert await s.cas_update(ALGORITHM, running.id, "FAILED", "c", "d", NOW, ("RUNNING", "BUFFERED")) == (True, None)
        assert await s.cas_update(ALGORITHM, cancelled.id, "FAILED", "c", "d", NOW, ("RUNNING",)) == (False, "CANCELLED")
        assert await s.cas_update(ALGORITHM, "no-such-run", "FAILED", "c", "d", NOW, ("RUNNING",)) == (False, None)
        assert await s.update_status(ALGORITHM, running.id, "FAILED", "c", "d", NOW) is True
        assert await s.update_status(ALGORITHM, cancelled.id, "RUNNING", None, None, NOW, only_if_stages=("BUFFERED",)) is False
        assert inner.get(ALGORITHM, running.id).lifecycle_stage == "RUNNING"  # nothing written
        assert (await s.read_status(ALGORITHM, running.id)).lifecycle_stage == "RUNNING"
        assert s.writes == 2 and _counter(m, "dry_run_writes") == 2
        jobs = DryRunJobs(RecordingJobs(["j1"]), log, m)
        assert getattr(jobs, "delete_job_nowait", None) is None
        await jobs.delete_job("nexus", "j1")
        assert jobs.inner.deleted == [] and jobs.deletes == 1

    arun(go())


def test_reference_scenarios_in_dry_run_touch_nothing(arun):
    scenarios = reference_scenarios()

    async def go():
        objs = [o for s in scenarios for o in s.objects]
        cfg = _cfg(**{"dry-run": True})
        api, srv, app, store, decisions = await _wire_cluster(objs, cfg=cfg)
        try:
            await _settle(app, decisions, 8)
            before = {r.id: r.lifecycle_stage for r in seed_rows()}
            # the decisions are the live ones...
            decided = {d.result.request_id: d.new_stage for d in decisions if d.outcome == "applied"}
            for s in scenarios:
                for rid, stage in s.expected.items():
                    if before[rid] != stage:
                        assert decided.get(rid) == stage, (s.name, rid, decided.get(rid))
            # ...but the store still holds the seeded stages and no Job was deleted
            for rid, stage in before.items():
                assert (await store.read_checkpoint(ALGORITHM, rid)).lifecycle_stage == stage, rid
            assert not [d for d in api.deleted if d[0] == "Job"]
            m = app.supervisor.metrics
            assert _counter(m, "dry_run_writes") == len(decided)
            assert _counter(m, "dry_run_deletes") == sum(1 for s in decided.values() if s != "RUNNING")
        finally:
            await app.stop()
            srv.stop()
            await api.stop()

    arun(go(), timeout=60)


def test_shadow_report_compares_the_shadow_log_with_the_store(arun):
    """The shadow run's log lines against the rows the acting supervisor wrote: agreement,
    differences (with the shadow's failure class), runs the other side has not finished."""
    import logging

    from nexus_supervisor_amd.obs.logging import JsonFormatter
    from nexus_supervisor_amd.shadow import parse_shadow_log, report

    scenarios = reference_scenarios()
    buf = io.StringIO()
    h = logging.StreamHandler(buf)
    h.setFormatter(JsonFormatter())
    pkg = logging.getLogger("nexus_supervisor_amd")
    pkg.addHandler(h)
    level = pkg.level
    pkg.setLevel(logging.INFO)

    async def go():
        objs = [o for s in scenarios for o in s.objects]
        api, srv, app, store, decisions = await _wire_cluster(objs, cfg=_cfg(**{"dry-run": True}))
        try:
            await _settle(app, decisions, 8)
            shadow = parse_shadow_log(buf.getvalue().splitlines())
            expected = {rid: st for s in scenarios for rid, st in s.expected.items()}
            assert {rid for _a, rid in shadow} == {rid for rid, st in expected.items()
                                                   if st != next(r.lifecycle_stage for r in seed_rows() if r.id == rid)}
            # the "reference" acts: it agrees on all runs but one, which it marks differently,
            # and has not got to another yet
            keys = sorted(shadow)
            other, pending = keys[0], keys[1]
            for alg, rid in keys:
                if rid == pending[1]:
                    continue
                stage = shadow[(alg, rid)]["stage"]
                if rid == other[1]:
                    stage = "FAILED" if stage == "DEADLINE_EXCEEDED" else "DEADLINE_EXCEEDED"
                await store.update_status(alg, rid, stage, "c", "d", NOW)
            rep = await report(shadow, store)
            assert rep["runs"] == len(keys) and rep["differ"] == 1 and rep["missing"] == 0
            assert rep["agree"] + rep["unfinished"] == len(keys) - 1
            assert rep["differences"][0]["request_id"] == other[1]
            assert rep["agreement"] == round(rep["agree"] / (rep["agree"] + 1), 4)
        finally:
            await app.stop()
            srv.stop()
            await api.stop()

    try:
        arun(go(), timeout=60)
    finally:
        pkg.removeHandler(h)
        pkg.setLevel(level)
