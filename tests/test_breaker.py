"""Store circuit breaker (parallel/breaker.py): a store outage longer than the retry budget
loses no decision — they wait at the gate instead of burning retries — and the store sees
probes, not a retry storm."""
import asyncio

from nexus_supervisor_amd.config import load_config
from nexus_supervisor_amd.models import LifecycleStage as S
from nexus_supervisor_amd.models.checkpoint import CheckpointedRequest
from nexus_supervisor_amd.parallel.breaker import CLOSED, HALF_OPEN, OPEN, CircuitBreaker
from nexus_supervisor_amd.store.base import StoreError
from nexus_supervisor_amd.store.memory import MemoryStore
from nexus_supervisor_amd.testing.inproc import InProcCluster
from nexus_supervisor_amd.testing.seed import ALGORITHM, make_job, make_pod


def test_breaker_states(arun):
    async def go():
        b = CircuitBreaker(failure_threshold=2, open_duration=0.05, max_open_duration=0.2)
        assert b.is_closed()
        b.failure()
        assert b.state is CLOSED
        b.failure()
        assert b.state is OPEN and b.trips == 1
        t0 = asyncio.get_running_loop().time()
        await b.wait()  # the probe: released once the open period ends
        assert b.state is HALF_OPEN and asyncio.get_running_loop().time() - t0 >= 0.04
        second = asyncio.ensure_future(b.wait())
        await asyncio.sleep(0.02)
        assert not second.done()  # one probe at a time
        b.neutral()  # the probe never reached the store: the next waiter probes
        await asyncio.wait_for(second, 1)
        b.failure()  # failed probe: open again, for twice as long
        assert b.state is OPEN and b._span == 0.1
        third = asyncio.ensure_future(b.wait())
        await asyncio.sleep(0.12)
        assert third.done() and b.state is HALF_OPEN
        b.success()
        assert b.state is CLOSED and b._span == 0.05
        await asyncio.wait_for(b.wait(), 0.01)

    arun(go())


class FlakyStore(MemoryStore):
    """Every call fails while ``down``; counts the calls that reached it."""

    def __init__(self, rows):
        super().__init__(rows)
        self.down = False
        self.calls = 0

    async def _io(self):
        self.calls += 1
        if self.down:
            raise StoreError("store unavailable")
        await super()._io()


def _scenario(breaker: bool, n: int = 12, outage: float = 0.6, max_retries: int = 3):
    cfg = load_config(path=None, env={}, overrides={
        "cql-store-type": "memory", "workers": 16, "rate-limit-elements-per-second": 0, "resync-period": "0s",
        "failure-rate-base-delay": "10ms", "failure-rate-max-delay": "40ms", "max-retries": max_retries,
        "circuit-breaker": {"enabled": breaker, "failure-threshold": 3, "open-duration": "50ms",
                            "max-open-duration": "100ms"}})
    rids = [f"outage-run-{i}" for i in range(n)]
    store = FlakyStore([CheckpointedRequest(algorithm=ALGORITHM, id=r, lifecycle_stage=S.RUNNING) for r in rids])
    objs = [o for r in rids for o in (make_job(r, cfg.labels), make_pod(r, cfg.labels))]

    async def go():
        c = InProcCluster(cfg, store, objs)
        await c.start()
        store.down = True
        calls0 = store.calls
        for r in rids:
            p = make_pod(r, cfg.labels, rv="9")
            p["status"] = {"phase": "Failed", "containerStatuses": [{"name": "algorithm", "state": {
                "terminated": {"reason": "OOMKilled", "exitCode": 137}}}]}
            c.push(p, "MODIFIED")
        await asyncio.sleep(outage)
        during = store.calls - calls0
        store.down = False
        await c.settle(10)
        await c.stop()
        failed = sum(1 for r in rids if store.get(ALGORITHM, r).lifecycle_stage == S.FAILED)
        return failed, c.supervisor.pipeline.stats.dead_lettered, during, c.supervisor

    return go()


def test_failed_probes_do_not_spend_the_retry_budget(arun):
    """Whichever decision the scheduler lets through as the probe, a probe that fails and
    re-opens the circuit is the store's verdict: with one retry allowed and a 0.8 s outage
    (several failed probes), nothing is dead-lettered."""
    failed, dead, _during, sup = arun(_scenario(breaker=True, outage=0.8, max_retries=1), timeout=30)
    assert failed == 12 and dead == 0 and sup.breaker.trips >= 2


def test_outage_longer_than_the_retry_budget_loses_nothing(arun):
    failed, dead, during, sup = arun(_scenario(breaker=True), timeout=30)
    assert failed == 12 and dead == 0
    # the first attempts trip it (3), then one probe per open period (≤ 0.6 s / 50 ms)
    assert during <= 3 + 16 + 12, during
    assert sup.breaker.trips >= 1 and sup.breaker.state is CLOSED
    assert sup.metrics.counters["store_circuit_trips"]


def test_without_the_breaker_the_same_outage_dead_letters(arun):
    failed, dead, during, _ = arun(_scenario(breaker=False), timeout=30)
    assert dead > 0 and failed < 12


class RefusingStore(MemoryStore):
    """Every write is refused with the given CQL error (the read answers)."""

    def __init__(self, rows, code):
        super().__init__(rows)
        self.code = code
        self.refused = 0

    async def update_status(self, *a, **kw):
        from nexus_supervisor_amd.store.cql import CqlError
        self.refused += 1
        raise CqlError(self.code, "refused")


def _classified(code, async_delete=True, jobs=None):
    from nexus_supervisor_amd.testing.inproc import RecordingJobs

    cfg = load_config(path=None, env={}, overrides={
        "cql-store-type": "memory", "workers": 4, "rate-limit-elements-per-second": 0, "resync-period": "0s",
        "failure-rate-base-delay": "5ms", "failure-rate-max-delay": "10ms", "max-retries": 2,
        "async-job-delete": async_delete,
        "circuit-breaker": {"enabled": True, "failure-threshold": 2, "open-duration": "5s"}})
    rids = [f"refused-run-{i}" for i in range(6)]
    rows = [CheckpointedRequest(algorithm=ALGORITHM, id=r, lifecycle_stage=S.RUNNING) for r in rids]
    store = RefusingStore(rows, code) if code is not None else MemoryStore(rows)
    objs = [o for r in rids for o in (make_job(r, cfg.labels), make_pod(r, cfg.labels))]

    async def go():
        c = InProcCluster(cfg, store, objs, jobs=jobs(objs) if jobs else None)
        await c.start()
        for r in rids:
            p = make_pod(r, cfg.labels, rv="9")
            p["status"] = {"phase": "Failed", "containerStatuses": [{"name": "algorithm", "state": {
                "terminated": {"reason": "OOMKilled", "exitCode": 137}}}]}
            c.push(p, "MODIFIED")
        await c.settle(5)
        await c.stop()
        return c.supervisor, store

    return go()


def test_request_level_cql_errors_do_not_trip_the_breaker(arun):
    """One partition's WriteTimeout (0x1100) or an Invalid query (0x2200)
    is a refusal of that request, not a store outage: decisions dead-letter through their
    own retry budget and the breaker stays closed.  Unavailable (0x1000) trips it."""
    for code in (0x1100, 0x2200):
        sup, store = arun(_classified(code), timeout=20)
        assert sup.breaker.trips == 0 and sup.breaker.state is CLOSED, hex(code)
        assert store.refused >= 6
    sup, _ = arun(_classified(0x1000), timeout=20)
    assert sup.breaker.trips >= 1


def test_failed_job_delete_after_a_durable_write_counts_for_the_store(arun):
    """The write landed, then the synchronous Job DELETE failed — the store
    answered, so the breaker records a success (it never counts the API server's errors)."""
    from nexus_supervisor_amd.testing.inproc import RecordingJobs

    def failing_jobs(objs):
        j = RecordingJobs(o["metadata"]["name"] for o in objs if o["kind"] == "Job")
        j.fail_next = 100
        return j

    async def go():
        sup, store = await _classified(None, async_delete=False, jobs=failing_jobs)
        return sup, store

    sup, store = arun(go(), timeout=20)
    assert all(store.get(ALGORITHM, f"refused-run-{i}").lifecycle_stage == S.FAILED for i in range(6))
    assert sup.breaker.trips == 0 and sup.breaker.failures == 0
