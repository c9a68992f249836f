"""Client-side API flow control.

The reference's clientset runs on client-go's defaults (``/root/reference/app/
app_dependencies.go:39-45``): a QPS 5 / burst 10 token bucket, and ``429`` answers
retried after the server's ``Retry-After``.  Here: ``kube-qps`` / ``kube-burst`` shared by
every request of a process, 429 / hinted 5xx retried never earlier than the hint, and a
bound on concurrent ``pods/log`` reads.
"""
import asyncio
import json
import time

import pytest

from nexus_supervisor_amd.app import Application
from nexus_supervisor_amd.config import load_config
from nexus_supervisor_amd.config.schema import ConfigError
from nexus_supervisor_amd.kube.client import KubeClient, KubeConfig
from nexus_supervisor_amd.kube.errors import TooManyRequests
from nexus_supervisor_amd.kube.flowcontrol import RetryPolicy, TokenBucket, retry_after, split
from nexus_supervisor_amd.models.checkpoint import CheckpointedRequest
from nexus_supervisor_amd.store.memory import MemoryStore
from nexus_supervisor_amd.testing.fake_apiserver import FakeApiServer
from nexus_supervisor_amd.testing.seed import ALGORITHM, make_job, make_pod


def test_token_bucket_burst_then_qps_and_priorities(arun):
    """Burst tokens go at once, then one per 1/qps; a decision read (class 0) queued after
    ten background DELETEs (class 1) gets its weighted turn instead of waiting for all of
    them (it is first here: the round robin starts at the read class)."""
    async def go():
        b = TokenBucket(100, 2)
        assert b.try_accept() and b.try_accept() and not b.try_accept()  # the burst
        order = []

        async def one(tag, prio):
            await b.wait(prio)
            order.append(tag)

        t0 = time.monotonic()
        tasks = [asyncio.ensure_future(one(f"delete{i}", 1)) for i in range(10)]
        await asyncio.sleep(0)
        tasks.append(asyncio.ensure_future(one("log-read", 0)))
        await asyncio.gather(*tasks)
        took = time.monotonic() - t0
        assert order[0] == "log-read" and order[1:] == [f"delete{i}" for i in range(10)], order
        assert 0.09 <= took < 0.5, took  # 11 tokens at 100/s with the bank empty
        assert b.waits == 11 and b.queued == 0
        # a cancelled waiter gives its turn away
        w = asyncio.ensure_future(b.wait(1))
        await asyncio.sleep(0)
        w.cancel()
        assert await asyncio.wait_for(b.wait(0), 1.0) >= 0.0
        assert TokenBucket(0, 1).try_accept() and await TokenBucket(0, 1).wait() == 0.0

    arun(go(), timeout=10)


def test_split_over_shard_workers():
    assert split(50, 100, 1) == (50, 100)
    assert split(50, 100, 4) == (12.5, 25)
    assert split(0, 100, 4) == (0, 100)
    assert split(5, 10, 16) == (5 / 16, 1)


def test_retry_after_parsing_and_policy():
    assert retry_after("3") == 3.0 and retry_after(b"1") == 1.0
    assert retry_after("9999") == 60.0 and retry_after("-4") == 0.0
    assert retry_after(None) is None and retry_after("soon") is None
    assert retry_after("Wed, 21 Oct 2015 07:28:10 GMT", now=1445412480.0) == pytest.approx(10.0)
    p = RetryPolicy()
    assert p.delay(429, None) == 1.0 and p.delay(429, 4.0) == 4.0
    assert p.delay(503, 2.0) == 2.0 and p.delay(503, None) is None and p.delay(404, 1.0) is None


def test_config_keys_and_reference_defaults():
    cfg = load_config(path=None, env={})
    assert (cfg.kube_qps, cfg.kube_burst, cfg.kube_max_retries) == (50.0, 100, 10)
    cfg = load_config(path=None, env={"NEXUS__KUBE_QPS": "5", "NEXUS__KUBE_BURST": "10"})
    assert (cfg.kube_qps, cfg.kube_burst) == (5.0, 10)  # the reference's effective client-go limits
    with pytest.raises(ConfigError):
        load_config(path=None, env={}, overrides={"kube-burst": 0})
    with pytest.raises(ConfigError):
        load_config(path=None, env={}, overrides={"gpu": {"log-tail-concurrency": 0}})


def test_client_retries_429_after_the_hint(arun):
    async def go():
        api = FakeApiServer(bookmark_interval=0.1)
        url = await api.start()
        api.create(make_job("j1", load_config(path=None, env={}).labels))
        kc = KubeClient(KubeConfig(url))
        api.throttle_next[("GET", "Job")] = 2
        t0 = time.monotonic()
        got = await kc.get("Job", "nexus", "j1")
        assert got["metadata"]["name"] == "j1" and time.monotonic() - t0 >= 2.0
        assert kc.throttled == 2 and kc.retried == 2
        # out of retries: the 429 surfaces, typed, with the hint
        kc.retry = RetryPolicy(max_retries=0)
        api.throttle_next[("GET", "Job")] = 1
        with pytest.raises(TooManyRequests) as ei:
            await kc.get("Job", "nexus", "j1")
        assert ei.value.retry_after == 1.0
        await kc.close()
        await api.stop()

    arun(go(), timeout=20)


def test_client_side_bucket_paces_requests(arun):
    async def go():
        api = FakeApiServer(bookmark_interval=0.1)
        url = await api.start()
        kc = KubeClient(KubeConfig(url), qps=20, burst=2)
        t0 = time.monotonic()
        await asyncio.gather(*(kc.list("Job", "nexus") for _ in range(12)))
        took = time.monotonic() - t0
        assert took >= (12 - 2) / 20 * 0.9, took  # burst 2, then 20/s
        assert kc.limiter.waits >= 9
        # Lease calls bypass the bucket (leader election never starves behind a DELETE burst)
        kc.limiter = TokenBucket(0.5, 1)
        kc.limiter.try_accept()
        t0 = time.monotonic()
        try:
            await kc.get("Lease", "nexus", "none")
        except Exception:
            pass
        assert time.monotonic() - t0 < 1.0
        await kc.close()
        await api.stop()

    arun(go(), timeout=20)


def _app_cfg(**over):
    base = {"cql-store-type": "memory", "rate-limit-elements-per-second": 0, "resync-period": "0s",
            "failure-rate-base-delay": "20ms", "failure-rate-max-delay": "200ms"}
    base.update(over)
    return load_config(path=None, env={}, overrides=base)


def _oomkilled(pod):
    p = json.loads(json.dumps(pod))
    p["status"] = {"phase": "Failed", "containerStatuses": [
        {"name": "algorithm", "restartCount": 0, "state": {"terminated": {"reason": "OOMKilled", "exitCode": 137}}}]}
    p["metadata"]["resourceVersion"] = "2"
    return p


def test_throttled_job_deletes_all_land_and_honour_retry_after(arun):
    """Done-criterion: the first 50 Job DELETEs get ``429 Retry-After: 1``.  Every Job is
    deleted, no decision is dead-lettered, and no re-sent DELETE of a throttled Job comes
    earlier than 1 s after its 429."""
    n = 60

    async def go():
        api = FakeApiServer(bookmark_interval=0.1)
        url = await api.start()
        cfg = _app_cfg()
        rids = [f"throttled-{i:03d}" for i in range(n)]
        for r in rids:
            api.create(make_pod(r, cfg.labels, status={"phase": "Running"}))
            api.create(make_job(r, cfg.labels))
        store = MemoryStore([CheckpointedRequest(algorithm=ALGORITHM, id=r, lifecycle_stage="RUNNING") for r in rids])
        app = Application(cfg, kube=KubeClient(KubeConfig(url)), store=store)
        await app.start()
        await app.factory.wait_for_cache_sync(5)
        api.throttle_next[("DELETE", "Job")] = 50
        for r in rids:
            api.update(_oomkilled(api.get("Pod", "nexus", f"{r}-acdey")))
        for _ in range(400):
            if all(api.get("Job", "nexus", r) is None for r in rids):
                break
            await asyncio.sleep(0.02)
        assert all(api.get("Job", "nexus", r) is None for r in rids)
        assert all(store.get(ALGORITHM, r).lifecycle_stage == "FAILED" for r in rids)
        assert app.supervisor.pipeline.stats.dead_lettered == 0
        first_429 = {}
        for t, method, _kind, name, status in api.throttle_log:
            if status == 429:
                first_429.setdefault(name, t)
            else:
                assert t - first_429[name] >= 0.99, (name, t - first_429[name])
        assert len(first_429) == 50
        assert app.kube.throttled >= 50
        assert app.metrics.counters.get("kube_throttled")
        await app.stop()
        await api.stop()

    arun(go(), timeout=40)


def test_pods_log_wave_is_bounded(arun):
    """Done-criterion: a 500-pod GPU failure wave (default pods: empty termination
    messages, so every decision wants its container log) never has more than
    ``gpu.log-tail-concurrency`` pods/log GETs in flight; every run is still decided."""
    n, bound = 500, 8

    async def go():
        api = FakeApiServer(bookmark_interval=0.1)
        url = await api.start()
        cfg = _app_cfg(**{"kube-qps": 0, "gpu": {"log-tail-concurrency": bound}})
        rids = [f"wave-{i:03d}" for i in range(n)]
        for r in rids:
            api.create(make_pod(r, cfg.labels, gpus=1, status={"phase": "Running"}))
            api.create(make_job(r, cfg.labels))
            api.set_pod_log("nexus", f"{r}-acdey", "algorithm", "torch.OutOfMemoryError: HIP out of memory.\n")
        api.log_latency = 0.005
        store = MemoryStore([CheckpointedRequest(algorithm=ALGORITHM, id=r, lifecycle_stage="RUNNING") for r in rids])
        app = Application(cfg, kube=KubeClient(KubeConfig(url)), store=store)
        await app.start()
        await app.factory.wait_for_cache_sync(5)
        for r in rids:
            p = json.loads(json.dumps(api.get("Pod", "nexus", f"{r}-acdey")))
            p["status"] = {"phase": "Failed", "containerStatuses": [
                {"name": "algorithm", "restartCount": 0,
                 "state": {"terminated": {"reason": "Error", "exitCode": 1, "message": ""}}}]}
            api.update(p)
        for _ in range(1000):
            if all(store.get(ALGORITHM, r).lifecycle_stage == "FAILED" for r in rids):
                break
            await asyncio.sleep(0.02)
        assert all(store.get(ALGORITHM, r).lifecycle_stage == "FAILED" for r in rids)
        assert json.loads(store.get(ALGORITHM, rids[-1]).algorithm_failure_details)["class"] == "hbm-oom"
        assert len(api.log_requests) == n
        assert api.log_inflight_max <= bound and app.supervisor.log_tail_inflight_max <= bound
        assert app.supervisor.log_tail_inflight_max == bound  # the bound was reached, not idle
        assert app.metrics.counter("log_tail_queued") > 0
        await app.stop()
        await api.stop()

    arun(go(), timeout=60)


def test_log_reads_are_not_starved_by_a_delete_backlog(arun):
    """kube-qps 20: a wave of 80 OOMKilled runs queues 80 background Job DELETEs (4 s of
    tokens).  A GPU pod that fails right behind them with an empty termination message needs
    its pods/log tail before it can be decided: the read class has its own share of the
    tokens, so that run is decided within a second, not after the backlog drains."""
    async def go():
        api = FakeApiServer(bookmark_interval=0.1)
        url = await api.start()
        cfg = _app_cfg(**{"kube-qps": 20, "kube-burst": 5})
        rids = [f"wave-{i:03d}" for i in range(80)]
        for r in rids + ["gpu-run"]:
            api.create(make_pod(r, cfg.labels, gpus=1 if r == "gpu-run" else 0, status={"phase": "Running"}))
            api.create(make_job(r, cfg.labels))
        api.set_pod_log("nexus", "gpu-run-acdey", "algorithm", "torch.OutOfMemoryError: HIP out of memory.\n")
        store = MemoryStore([CheckpointedRequest(algorithm=ALGORITHM, id=r, lifecycle_stage="RUNNING")
                             for r in rids + ["gpu-run"]])
        app = Application(cfg, kube=KubeClient(KubeConfig(url)), store=store)
        await app.start()
        await app.factory.wait_for_cache_sync(5)
        for r in rids:
            api.update(_oomkilled(api.get("Pod", "nexus", f"{r}-acdey")))
        for _ in range(200):
            if all(store.get(ALGORITHM, r).lifecycle_stage == "FAILED" for r in rids):
                break
            await asyncio.sleep(0.01)
        assert app.kube.limiter.queued > 30  # the DELETE backlog is there
        p = json.loads(json.dumps(api.get("Pod", "nexus", "gpu-run-acdey")))
        p["status"] = {"phase": "Failed", "containerStatuses": [
            {"name": "algorithm", "restartCount": 0, "state": {"terminated": {"reason": "Error", "exitCode": 1}}}]}
        p["metadata"]["resourceVersion"] = "3"
        t0 = time.monotonic()
        api.update(p)
        for _ in range(300):
            if store.get(ALGORITHM, "gpu-run").lifecycle_stage == "FAILED":
                break
            await asyncio.sleep(0.01)
        took = time.monotonic() - t0
        assert store.get(ALGORITHM, "gpu-run").lifecycle_stage == "FAILED" and took < 1.0, took
        assert json.loads(store.get(ALGORITHM, "gpu-run").algorithm_failure_details)["class"] == "hbm-oom"
        assert app.kube.limiter.queued > 0  # ...while DELETEs were still waiting for tokens
        await app.stop()
        await api.stop()

    arun(go(), timeout=40)


def _wave(qps, burst, reads, shared=None):
    """A failure wave on default GPU pods: ``reads`` pods/log reads queued at once, and
    each decided read queues that run's Job DELETE.  Returns (read waits, delete waits)."""
    async def go():
        b = TokenBucket(qps, burst, shared=shared)
        read_w, del_w = [], []

        async def delete():
            t = time.monotonic()
            await b.wait(1)
            del_w.append(time.monotonic() - t)

        dels = []

        async def read():
            t = time.monotonic()
            await b.wait(0)
            read_w.append(time.monotonic() - t)
            dels.append(asyncio.ensure_future(delete()))

        await asyncio.gather(*[read() for _ in range(reads)])
        await asyncio.gather(*dels)
        return read_w, del_w, b

    return go()


def _p99(xs):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(0.99 * len(xs)))]


def test_delete_share_in_a_gpu_wave(arun):
    """1,000 default-pod GPU failures at once: 1,000 pods/log reads and, behind each decided
    read, its Job DELETE (which frees the job's GPUs).  The reference's bucket is one FIFO
    (client-go); strict read priority made every DELETE wait for the whole read wave (at
    kube-qps 50 that is 20 s, here scaled to qps 1000 = 1 s).  With the weighted round robin
    a DELETE waits about one token turn, and the reads finish within 2x the time their
    fair share (reads and DELETEs alternating) gives them."""
    qps, n = 1000.0, 1000
    read_w, del_w, b = arun(_wave(qps, 1, n), timeout=30)
    wave = n / qps  # the read wave alone, at full rate
    assert _p99(del_w) < 0.1 * wave, _p99(del_w)
    fair = n / (qps / 2)  # reads' completion time when they share the tokens with the DELETEs
    assert max(read_w) <= 2 * fair, (max(read_w), fair)
    assert b.served[0] >= n - 1 and b.served[1] > 0.9 * n  # (the first read took the banked token)


def test_wrr_cycle_and_idle_classes():
    from nexus_supervisor_amd.kube.flowcontrol import _wrr_cycle

    assert _wrr_cycle((2, 2, 1)) == (0, 1, 2, 0, 1)
    assert sorted(_wrr_cycle((3, 1))) == [0, 0, 0, 1]

    async def go():
        # an idle class's share goes to the others: only Events queued -> full rate
        b = TokenBucket(400, 1)
        t0 = time.monotonic()
        await asyncio.gather(*[b.wait(2) for _ in range(40)])
        return time.monotonic() - t0

    took = asyncio.run(go())
    assert took < 0.2, took


def test_bucket_wait_timeout_takes_no_token(arun):
    async def go():
        b = TokenBucket(10, 1)
        assert b.try_accept()
        with pytest.raises(asyncio.TimeoutError):
            await b.wait(0, timeout=0.02)
        assert b.queued == 0
        # the next waiter gets the token the timed-out one would have had
        d = await asyncio.wait_for(b.wait(0), 1.0)
        assert d < 0.15

    arun(go(), timeout=10)


def test_cancelled_wait_strands_no_token(arun):
    """a log fetch cancelled (fence, shard loss) while it waits with a timeout:
    its queued wait is withdrawn, so the next token goes to the next waiter instead of to
    nobody."""
    async def go():
        b = TokenBucket(10, 1)
        assert b.try_accept()
        t = asyncio.ensure_future(b.wait(0, timeout=5.0))
        await asyncio.sleep(0.01)
        t.cancel()
        with pytest.raises(asyncio.CancelledError):
            await t
        await asyncio.sleep(0)
        assert b.queued == 0
        d = await asyncio.wait_for(b.wait(0), 1.0)  # the token the cancelled wait would have had
        assert d < 0.15

    arun(go(), timeout=10)


def test_give_back_refunds_try_accept():
    b = TokenBucket(1, 1)
    assert b.try_accept() and not b.try_accept()
    b.give_back()
    assert b.try_accept()


def test_shared_schedule_adapts_to_skew(arun):
    """Two processes' buckets on one replica budget (SharedSchedule): alone, one of them
    gets the whole kube-qps (a fixed split would cap it at half); together they share it
    and never exceed it."""
    from nexus_supervisor_amd.kube.flowcontrol import SharedSchedule

    async def go():
        sh = SharedSchedule(500, 1)
        a, b = TokenBucket(500, 1, shared=sh), TokenBucket(500, 1, shared=sh)
        t0 = time.monotonic()
        await asyncio.gather(*[a.wait(0) for _ in range(100)])
        alone = time.monotonic() - t0
        t0 = time.monotonic()
        await asyncio.gather(*[a.wait(0) for _ in range(100)], *[b.wait(1) for _ in range(100)])
        both = time.monotonic() - t0
        return alone, both

    alone, both = arun(go(), timeout=20)
    assert 0.15 <= alone < 0.4, alone   # 100 tokens at 500/s, not at 250/s
    assert 0.35 <= both < 0.8, both     # 200 tokens: the budget is shared, never doubled


def test_shared_schedule_across_processes(tmp_path):
    """The parent's GCRA word is inherited by a child process (memfd + pass_fds, as a shard
    worker gets it): the child's takes count against the parent's budget."""
    import os
    import subprocess
    import sys

    from nexus_supervisor_amd.kube.flowcontrol import SharedSchedule

    sh = SharedSchedule(100, 10)
    code = ("import os,sys; from nexus_supervisor_amd.kube.flowcontrol import SharedSchedule as S; "
            "s=S(100,10,fd=int(os.environ['FD'])); print(sum(s.try_take() for _ in range(50)))")
    env = dict(os.environ, FD=str(sh.fd))
    out = subprocess.run([sys.executable, "-c", code], env=env, pass_fds=(sh.fd,), capture_output=True, text=True,
                         timeout=120)
    assert out.returncode == 0, out.stderr
    assert 10 <= int(out.stdout.strip()) <= 12  # the burst (plus what refilled meanwhile)
    assert not sh.try_take() or sh.backlog() >= 0  # the parent sees the spent burst
    assert sh.backlog() > 0.05
