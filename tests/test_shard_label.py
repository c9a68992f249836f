"""Shard-narrowed watches: with ``sharding.shard-label``
each replica watches only its shards' Pods and Jobs (``<label> in (owned…)``, filtered by
the API server), so N replicas on one namespace do not each receive — and the API server
does not serialise N times — the whole stream.  The reference's only scale knob is more
replicas that all see everything (``/root/reference/.helm/values.yaml:124-125``)."""
import asyncio
import json

from nexus_supervisor_amd.app import Application
from nexus_supervisor_amd.config import load_config
from nexus_supervisor_amd.kube.client import KubeClient, KubeConfig
from nexus_supervisor_amd.models.checkpoint import CheckpointedRequest
from nexus_supervisor_amd.parallel.sharding import shard_of, shard_selector, watch_selector
from nexus_supervisor_amd.store.memory import MemoryStore
from nexus_supervisor_amd.testing.fake_apiserver import FakeApiServer
from nexus_supervisor_amd.testing.kubesim import KubeSim, SimControl
from nexus_supervisor_amd.testing.seed import ALGORITHM, make_job, make_pod

LABEL = "nexus.amd.com/shard"


def _cfg(index, shards=2, **over):
    base = {"cql-store-type": "memory", "rate-limit-elements-per-second": 0, "resync-period": "0s",
            "sharding": {"shards": shards, "shard-index": index, "shard-label": LABEL}}
    base.update(over)
    return load_config(path=None, env={}, overrides=base)


def test_selectors():
    assert shard_selector(LABEL, {1, 3}, 4) == f"{LABEL} in (1,3)"
    assert shard_selector(LABEL, set(), 4) == f"{LABEL} in (none)"
    assert shard_selector(LABEL, {0, 1}, 2) == "" and shard_selector("", {1}, 4) == "" and shard_selector(LABEL, None, 4) == ""
    cfg = _cfg(1)
    assert watch_selector(cfg, "Pod", {1}) == (f"{cfg.labels.nexus_component_label}={cfg.labels.algorithm_run_value},"
                                               f"{LABEL} in (1)")
    assert watch_selector(cfg, "Event", {1}) == ""
    cfg.sharding.shard_label = ""
    assert LABEL not in watch_selector(cfg, "Job", {1})


def test_watchhub_static_mode_narrows_pod_and_job_watches():
    """A static-mode sharded replica's watch hub (worker-processes > 1) must send the shard
    selector on its Pod/Job LIST/WATCH: nothing calls ``set_shards`` after construction."""
    from nexus_supervisor_amd.parallel.watchhub import WatchHub

    cfg = _cfg(1, shards=4)
    hub = WatchHub(cfg, kube=None, count=2, send=lambda *a: None, buffered=lambda w: 0, drain=lambda w: None)
    assert hub.owned == frozenset({1})
    for kind in ("Pod", "Job"):
        _, params = hub._path_params(kind)
        assert f"{LABEL} in (1)" in params["labelSelector"], (kind, params)
    _, params = hub._path_params("Event")
    assert "labelSelector" not in params


def _labelled(rid, labels, shards=2, stamp=True):
    extra = {LABEL: str(shard_of(rid, shards))} if stamp else {}
    pod = make_pod(rid, labels, status={"phase": "Running"})
    pod["metadata"]["labels"].update(extra)
    job = make_job(rid, labels)
    job["metadata"]["labels"].update(extra)
    return pod, job


def _oomkilled(pod):
    p = json.loads(json.dumps(pod))
    p["status"] = {"phase": "Failed", "containerStatuses": [
        {"name": "algorithm", "restartCount": 0, "state": {"terminated": {"reason": "OOMKilled", "exitCode": 137}}}]}
    p["metadata"]["resourceVersion"] = str(int(p["metadata"]["resourceVersion"]) + 1)
    return p


def test_two_replicas_watch_only_their_shards(arun):
    async def go():
        api = FakeApiServer(bookmark_interval=0.1)
        url = await api.start()
        labels = _cfg(0).labels
        rids = [f"run-{i:02d}" for i in range(24)]
        for r in rids:
            for o in _labelled(r, labels):
                api.create(o)
        unlabelled_pod, unlabelled_job = _labelled("run-unlabelled", labels, stamp=False)
        api.create(unlabelled_pod)
        api.create(unlabelled_job)
        store = MemoryStore([CheckpointedRequest(algorithm=ALGORITHM, id=r, lifecycle_stage="RUNNING") for r in rids])
        apps = [Application(_cfg(k), kube=KubeClient(KubeConfig(url)), store=store) for k in (0, 1)]
        for a in apps:
            await a.start()
            await a.factory.wait_for_cache_sync(5)
        for k, a in enumerate(apps):
            mine = {r for r in rids if shard_of(r, 2) == k}
            pods = {p["metadata"]["labels"]["batch.kubernetes.io/job-name"] for p in a.supervisor.pod_informer.indexer.values()}
            jobs = {j["metadata"]["name"] for j in a.supervisor.job_informer.indexer.values()}
            assert pods == mine and jobs == mine, k  # the server filtered: nothing of the other shard arrived
            assert a.supervisor.pod_informer.rejected == 0
        for r in rids:
            api.update(_oomkilled(api.get("Pod", "nexus", f"{r}-acdey")))
        for _ in range(200):
            if all(store.get(ALGORITHM, r).lifecycle_stage == "FAILED" for r in rids):
                break
            await asyncio.sleep(0.02)
        assert all(store.get(ALGORITHM, r).lifecycle_stage == "FAILED" for r in rids)
        per = [a.metrics.counter("decisions_applied", {"stage": "FAILED", "class": "host-oom"}) for a in apps]
        assert sum(per) == len(rids) and all(per)
        # the audit finds the Nexus Job that lacks the label (invisible to both replicas)
        for _ in range(100):
            if apps[0].metrics.gauge("shard_label_missing") == 1.0:
                break
            await asyncio.sleep(0.02)
        assert apps[0].metrics.gauge("shard_label_missing") == 1.0
        for a in apps:
            await a.stop()
        await api.stop()

    arun(go(), timeout=30)


def test_lease_mode_rewatches_on_shard_change(arun):
    """A lease-mode replica watches nothing until it holds a shard; gaining shard 1 re-lists
    the Pod/Job watches with the new selector, losing it narrows them again."""
    async def go():
        api = FakeApiServer(bookmark_interval=0.1)
        url = await api.start()
        cfg = _cfg(0, **{"sharding": {"shards": 2, "shard-label": LABEL, "mode": "lease"},
                         "leader-election": {"lease-duration": "60s", "renew-deadline": "40s", "retry-period": "20s"}})
        rids = [f"lease-{i:02d}" for i in range(16)]
        for r in rids:
            for o in _labelled(r, cfg.labels):
                api.create(o)
        app = Application(cfg, kube=KubeClient(KubeConfig(url)), store=MemoryStore([]))
        sup = app.supervisor
        sup.init()
        await sup.start(wait_sync_timeout=5)
        assert len(sup.pod_informer.indexer) == 0  # owns nothing yet
        import time

        sup.shards.set_deadlines({0: time.monotonic() + 60, 1: time.monotonic() + 60})  # what the lease manager renews
        sup.set_shards({1})
        mine = {r for r in rids if shard_of(r, 2) == 1}
        for _ in range(200):
            if len(sup.pod_informer.indexer) == len(mine):
                break
            await asyncio.sleep(0.02)
        assert {p["metadata"]["labels"]["batch.kubernetes.io/job-name"] for p in sup.pod_informer.indexer.values()} == mine
        assert sup.pod_informer.lw.label_selector.endswith(f"{LABEL} in (1)")
        sup.set_shards(set())
        for _ in range(200):
            if len(sup.pod_informer.indexer) == 0:
                break
            await asyncio.sleep(0.02)
        assert len(sup.pod_informer.indexer) == 0
        await sup.stop(drain=False)
        await app.kube.close()
        await api.stop()

    arun(go(), timeout=30)


def test_kubesim_set_selectors(arun):
    async def go():
        labels = _cfg(0).labels
        with KubeSim() as sim:
            ctl = SimControl(sim.url)
            objs = []
            for i in range(12):
                pod, job = _labelled(f"k-{i:02d}", labels, shards=3)
                objs += [pod, job]
            await ctl.apply([("ADDED", o) for o in objs])
            kc = KubeClient(KubeConfig(sim.url))
            got, _ = await kc.list("Job", "nexus", label_selector=f"{LABEL} in (0, 2)")
            want = {o["metadata"]["name"] for o in objs if o["kind"] == "Job" and o["metadata"]["labels"][LABEL] in ("0", "2")}
            assert {j["metadata"]["name"] for j in got} == want
            got, _ = await kc.list("Job", "nexus", label_selector=f"{LABEL} notin (0,2)")
            assert {j["metadata"]["labels"][LABEL] for j in got} == {"1"}
            await kc.close()
            await ctl.close()

    arun(go(), timeout=20)


def test_job_decision_waits_for_the_pod_relist_of_a_shard_change(arun):
    """Gaining a shard re-lists the Pod watch: until the list lands the cached pods of EVERY
    owned shard are as old as the gain.  A Job's BackoffLimitExceeded seen meanwhile (its
    own watch is back first) must wait for that list, not just ``rules.job-pod-settle``:
    the cached pod still says Running, and deciding from the Job alone writes
    DEADLINE_EXCEEDED without the pod's OOMKilled (config 5s at reference limits, where a
    10k-pod list behind kube-qps 5 took 18 s)."""
    async def go():
        api = FakeApiServer(bookmark_interval=0.1)
        url = await api.start()
        cfg = _cfg(0, **{"sharding": {"shards": 2, "shard-label": LABEL, "mode": "lease"},
                         "rules": {"job-pod-settle": "200ms"},
                         "leader-election": {"lease-duration": "60s", "renew-deadline": "40s", "retry-period": "20s"}})
        rid = next(f"relist-{i:02d}" for i in range(64) if shard_of(f"relist-{i:02d}", 2) == 1)
        pod, job = _labelled(rid, cfg.labels)
        api.create(pod)
        api.create(job)
        store = MemoryStore([CheckpointedRequest(algorithm=ALGORITHM, id=rid, lifecycle_stage="RUNNING")])
        app = Application(cfg, kube=KubeClient(KubeConfig(url)), store=store)
        sup = app.supervisor
        sup.init()
        await sup.start(wait_sync_timeout=5)
        import time

        sup.shards.set_deadlines({0: time.monotonic() + 60, 1: time.monotonic() + 60})
        sup.set_shards({1})
        for _ in range(200):
            if sup.pod_informer.indexer.get_by_name("nexus", f"{rid}-acdey") is not None and sup._pod_relist is None:
                break
            await asyncio.sleep(0.02)
        assert sup.pod_informer.indexer.get_by_name("nexus", f"{rid}-acdey") is not None
        lw = sup.pod_informer.lw
        slow_list = lw.list

        async def list_late(*a, **kw):
            await asyncio.sleep(1.5)  # the pod list queued behind a kube-qps bucket
            return await slow_list(*a, **kw)

        lw.list = list_late
        sup.set_shards({0, 1})  # gains shard 0: the Pod watch is down until the list lands
        await asyncio.sleep(0.1)
        api.update(_oomkilled(api.get("Pod", "nexus", f"{rid}-acdey")))
        from test_logtail import _job_failed

        api.update(_job_failed(api.get("Job", "nexus", rid)))
        for _ in range(250):
            if store.get(ALGORITHM, rid).lifecycle_stage != "RUNNING":
                break
            await asyncio.sleep(0.02)
        row = store.get(ALGORITHM, rid)
        assert row.lifecycle_stage == "FAILED", (row.lifecycle_stage, row.algorithm_failure_details)
        assert app.metrics.counter("job_pod_settle_relist_waits") >= 1
        await sup.stop(drain=False)
        await app.kube.close()
        await api.stop()

    arun(go(), timeout=30)
