"""Process-per-core replica (``parallel/workers.py``): placement, the native pre-decode
shard router, ingest filtering, metrics hand-off, and a 2-worker replica running the
reference parity scenarios end to end over kubesim + the native CQL server."""
import asyncio
import json
import random
import zlib

import aiohttp
import pytest

from nexus_supervisor_amd import _kube_native
from nexus_supervisor_amd.app import ShardedApplication, make_application
from nexus_supervisor_amd.config import from_mapping, load_config, to_mapping
from nexus_supervisor_amd.config.schema import ConfigError, LabelConfig
from nexus_supervisor_amd.obs.metrics import Metrics
from nexus_supervisor_amd.parallel.workers import (_SEED, WorkerPool, WorkerShard, merge_metrics_state, metrics_state,
                                                   worker_of)
from nexus_supervisor_amd.store.cql import CqlCheckpointStore, CqlSession
from nexus_supervisor_amd.testing.cqlsrv import CqlServer
from nexus_supervisor_amd.testing.kubesim import KubeSim, SimControl
from nexus_supervisor_amd.testing.seed import ALGORITHM, make_event, make_job, make_pod, reference_scenarios, seed_cql_statements

JOB_LABEL = LabelConfig().job_name_label


def _line(etype, obj):
    return _kube_native.dumps({"type": etype, "object": obj}, newline=True)


def test_placement_native_matches_python():
    rng = random.Random(7)
    for count in (2, 3, 4, 8):
        routers = [_kube_native.ShardRouter(i, count, _SEED, JOB_LABEL) for i in range(count)]
        for _ in range(300):
            rid = "%032x" % rng.getrandbits(128)
            w = worker_of(rid, count)
            assert w == zlib.crc32(rid.encode(), _SEED) % count
            assert all(r.owner_of(rid) == w for r in routers)
    assert worker_of("anything", 1) == 0


def test_native_router_drops_other_workers_lines():
    labels = LabelConfig()
    rids = [f"run-{i}" for i in range(40)]
    pods = [make_pod(r, labels) for r in rids]
    jobs = [make_job(r, labels) for r in rids]
    job_events = [make_event("Job", r, "DeadlineExceeded") for r in rids]
    pod_events = [make_event("Pod", p["metadata"]["name"], "BackOff") for p in pods]
    unknown = make_event("Pod", "never-seen-pod", "Failed")
    got = {}
    for idx in range(2):
        router = _kube_native.ShardRouter(idx, 2, _SEED, JOB_LABEL)
        decs = {}
        for role in ("job", "pod", "event"):
            d = _kube_native.ProjectedDecoder(True)
            d.set_router(router, role)
            decs[role] = d
        out_jobs = decs["job"].feed(b"".join(_line("ADDED", j) for j in jobs))
        out_pods = decs["pod"].feed(b"".join(_line("ADDED", p) for p in pods))
        out_ev = decs["event"].feed(b"".join(_line("ADDED", e) for e in job_events + pod_events + [unknown])
                                    + b'{"type":"BOOKMARK","object":{"kind":"Event","metadata":{"resourceVersion":"9"}}}\n')
        got[idx] = (out_jobs, out_pods, out_ev)
        owned = {r for r in rids if worker_of(r, 2) == idx}
        assert {o["object"]["metadata"]["name"] for o in out_jobs} == owned
        assert {o["object"]["metadata"]["labels"][JOB_LABEL] for o in out_pods} == owned
        names = [(o["object"].get("involvedObject") or {}).get("name") for o in out_ev]
        assert names.count("never-seen-pod") == 1 and names[-1] is None  # unknown pod + bookmark pass everywhere
        ev_runs = {n if n in rids else n.rsplit("-", 1)[0] for n in names if n and n != "never-seen-pod"}
        assert ev_runs == owned
        assert router.pod_owner(pods[0]["metadata"]["name"]) == worker_of(rids[0], 2)
        assert router.stats["dropped"] > 0
    # the two workers partition the traffic
    assert len(got[0][0]) + len(got[1][0]) == len(jobs)
    assert len(got[0][1]) + len(got[1][1]) == len(pods)


def test_worker_shard_python_filter_and_pod_expiry():
    now = [0.0]
    shards = [WorkerShard(i, 3, JOB_LABEL, forget_after=10.0, clock=lambda: now[0]) for i in range(3)]
    labels = LabelConfig()
    pod = make_pod("r-1", labels)
    owner = worker_of("r-1", 3)
    assert [s.accept_pod(pod, "ADDED") for s in shards] == [i == owner for i in range(3)]
    assert [s.accept_job(make_job("r-1", labels), "ADDED") for s in shards] == [i == owner for i in range(3)]
    ev = make_event("Pod", pod["metadata"]["name"], "BackOff")
    assert [s.accept_event(ev, "ADDED") for s in shards] == [i == owner for i in range(3)]
    stray = make_event("Pod", "unknown-pod", "BackOff")
    assert all(s.accept_event(stray, "ADDED") for s in shards)  # parked everywhere until the pod shows up
    other = {"involvedObject": {"kind": "Node", "name": "n1"}}
    assert [s.accept_event(other, "ADDED") for s in shards] == [True, False, False]
    for s in shards:
        s.accept_pod(pod, "DELETED")
    now[0] = 5.0
    shards[0].accept_pod(make_pod("r-2", labels), "ADDED")
    assert shards[0].owner_of_pod(pod["metadata"]["name"]) == owner  # still remembered for late events
    now[0] = 11.0
    shards[0].accept_pod(make_pod("r-3", labels), "ADDED")
    assert shards[0].pod_owner.get(pod["metadata"]["name"]) is None


def test_metrics_state_merge():
    a, b = Metrics("ns"), Metrics("ns")
    a.inc("decisions", 3, {"action": "x"})
    b.inc("decisions", 4, {"action": "x"})
    a.observe_seconds("lat", 0.010)
    b.observe_seconds("lat", 0.030)
    b.set("queue_depth", 5)
    m = Metrics("ns")
    merge_metrics_state(m, json.loads(json.dumps(metrics_state(a))), {"worker": "0"})
    merge_metrics_state(m, json.loads(json.dumps(metrics_state(b))), {"worker": "1"})
    assert m.counter("decisions", {"action": "x"}) == 7
    h = m.histogram("lat")
    assert h.total == 2 and 9_000 <= h.min <= 10_100 and 29_000 <= h.max <= 30_100
    assert m.gauge("queue_depth", {"worker": "1"}) == 5
    assert "ns_lat_seconds_count 2" in m.prometheus_text()


def test_config_handoff_and_admission_split():
    cfg = load_config(path=None, env={}, overrides={"workers": 9, "rate-limit-elements-per-second": 10,
                                                    "rate-limit-elements-burst": 100, "cql-store-type": "scylla",
                                                    "scylla-cql-store": {"hosts": "a:1,b:2", "password": "s3cret"},
                                                    "runtime": {"worker-processes": 4}})
    m = to_mapping(cfg)
    assert from_mapping(json.loads(json.dumps(m))) == cfg
    pool = WorkerPool(cfg)
    child = from_mapping(pool._child_mapping(3))
    assert child.runtime.worker_index == 3 and child.workers == 3  # ceil(9 / 4)
    assert child.rate_limit_elements_per_second == 2.5 and child.rate_limit_elements_burst == 25
    assert not child.leader_election.enabled and child.observability.http_port == 0
    assert child.scylla_cql_store.password == "s3cret"
    assert isinstance(make_application(cfg), ShardedApplication)
    with pytest.raises(ConfigError):
        load_config(path=None, env={}, overrides={"runtime": {"worker-processes": 2, "worker-index": 2}})


def test_watch_splitter_routes_lines_and_list_items():
    labels = LabelConfig()
    router = _kube_native.ShardRouter(0, 3, _SEED, JOB_LABEL)
    rids = [f"job-{i}" for i in range(30)]
    pods = [make_pod(r, labels) for r in rids]
    sp_pod = _kube_native.WatchSplitter(router, "pod")
    sp_ev = _kube_native.WatchSplitter(router, "event")
    body = _kube_native.dumps({"kind": "PodList", "apiVersion": "v1", "metadata": {"resourceVersion": "4242"},
                               "items": pods})
    rv, parts = sp_pod.split_list(body)
    assert rv == "4242" and len(parts) == 3
    for w, part in enumerate(parts):
        names = {p["metadata"]["labels"][JOB_LABEL] for p in json.loads(part)}
        assert names == {r for r in rids if worker_of(r, 3) == w}
    # a chunk boundary in the middle of a line: the tail waits for the next feed
    stream = b"".join(_line("MODIFIED", p) for p in pods[:10])
    stream += b'{"type":"BOOKMARK","object":{"kind":"Pod","metadata":{"resourceVersion":"9999"}}}\n'
    outs1, last1, err1 = sp_pod.feed(stream[:-40])
    outs2, last2, err2 = sp_pod.feed(stream[-40:])
    assert last2 == "9999" and not err1 and not err2  # bookmark consumed, its RV reported
    got = [b"".join(x) for x in zip(outs1, outs2)]
    for w in range(3):
        lines = [json.loads(l) for l in got[w].splitlines()]
        assert {l["object"]["metadata"]["labels"][JOB_LABEL] for l in lines} == \
            {r for r in rids[:10] if worker_of(r, 3) == w}
    # Pod events follow their pod's owner; unknown pods go everywhere; errors come back
    evs = [make_event("Pod", pods[0]["metadata"]["name"], "BackOff"), make_event("Pod", "ghost", "Failed")]
    outs, last, errs = sp_ev.feed(b"".join(_line("ADDED", e) for e in evs)
                                  + b'{"type":"ERROR","object":{"kind":"Status","code":410}}\n')
    owner = worker_of(rids[0], 3)
    for w in range(3):
        names = [json.loads(l)["object"]["involvedObject"]["name"] for l in outs[w].splitlines()]
        assert names == ([pods[0]["metadata"]["name"], "ghost"] if w == owner else ["ghost"])
    assert len(errs) == 1 and json.loads(errs[0])["object"]["code"] == 410
    with pytest.raises(ValueError):
        sp_pod.split_list(b'{"kind":"Status"}')


def test_splitter_drops_events_no_rule_reads():
    """With the rules' reasons set, a Scheduled / Pulled / Created Event (most of a
    namespace's Events) reaches no worker — watch line or LIST item — and is counted as
    unread; a Started or BackOff Event is routed as before, and without the set everything
    passes."""
    from nexus_supervisor_amd.classify.classifier import EVENT_REASONS_READ

    labels = LabelConfig()
    router = _kube_native.ShardRouter(0, 2, _SEED, JOB_LABEL)
    sp_ev = _kube_native.WatchSplitter(router, "event")
    pods = [make_pod(f"job-{i}", labels) for i in range(4)]
    sp_pod = _kube_native.WatchSplitter(router, "pod")
    sp_pod.feed(b"".join(_line("ADDED", p) for p in pods))  # pod owners known
    names = [p["metadata"]["name"] for p in pods]
    evs = [make_event("Pod", n, r) for n, r in zip(names, ("Scheduled", "Started", "Pulled", "BackOff"))]
    evs.append(make_event("Job", "job-9", "SuccessfulCreate"))
    stream = b"".join(_line("ADDED", e) for e in evs)
    outs, _, _ = sp_ev.feed(stream)
    assert sum(len(o.splitlines()) for o in outs) == 5  # no reason set: everything routed
    router.set_event_reasons(sorted(EVENT_REASONS_READ))
    outs, _, _ = sp_ev.feed(stream)
    got = sorted(json.loads(l)["object"]["reason"] for o in outs for l in o.splitlines())
    assert got == ["BackOff", "Started"] and router.stats["unread"] == 3
    body = _kube_native.dumps({"kind": "EventList", "apiVersion": "v1", "metadata": {"resourceVersion": "7"},
                               "items": evs})
    _, parts = sp_ev.split_list(body)
    assert sorted(e["reason"] for p in parts for e in json.loads(p)) == ["BackOff", "Started"]
    assert router.stats["unread"] == 6
    router.set_event_reasons(None)
    outs, _, _ = sp_ev.feed(stream)
    assert sum(len(o.splitlines()) for o in outs) == 5


def test_hub_feed_batched_watch_matches_per_line(arun):
    """HubListWatch.watch_batches (one list per frame, the informer's path) yields the same
    (type, object) stream as the per-line watch(), and a newer snapshot ends both with a 410
    that leaves the snapshot pending for the informer's re-list."""
    from nexus_supervisor_amd.informer.informer import SharedInformer
    from nexus_supervisor_amd.parallel.watchhub import LINES, SNAPSHOT, HubListWatch

    labels = LabelConfig()
    pods = [make_pod(f"job-{i}", labels) for i in range(100)]
    frames = [(LINES, b"".join(_line("ADDED", p) for p in pods[:70])),
              (LINES, b"".join(_line("DELETED", p) for p in pods[70:])),
              (SNAPSHOT, b"77\n" + _kube_native.dumps([pods[0]]))]

    async def drain(batched):
        q = asyncio.Queue()
        for f in frames:
            q.put_nowait(f)
        lw = HubListWatch("Pod", q)
        got = []
        if batched:
            async for batch in lw.watch_batches("1"):
                got.extend(batch)
        else:
            async for item in lw.watch("1"):
                got.append(item)
        items, rv = await lw.list()
        return got, items, rv

    async def informer_run():
        q = asyncio.Queue()
        q.put_nowait((SNAPSHOT, b"5\n[]"))
        for f in frames:
            q.put_nowait(f)
        inf = SharedInformer("Pod", HubListWatch("Pod", q))
        task = inf.start()
        for _ in range(200):
            await asyncio.sleep(0.01)
            if inf.relists >= 2:
                break
        task.cancel()
        return inf

    per_line = arun(drain(False))
    batched = arun(drain(True))
    assert per_line == batched
    got, items, rv = batched
    assert [t for t, _ in got] == ["ADDED"] * 70 + ["DELETED"] * 30 + ["ERROR"]
    assert got[-1][1]["code"] == 410 and rv == "77" and len(items) == 1
    inf = arun(informer_run())
    assert inf.relists == 2 and inf.watch_events == 100  # frames applied, then the new snapshot
    assert len(inf.indexer.values()) == 1


@pytest.mark.slow
@pytest.mark.parametrize("hub", [True, False], ids=["watch-hub", "per-worker-watch"])
def test_two_worker_replica_reference_parity(arun, tmp_path, hub):
    scenarios = reference_scenarios()

    async def go():
        with KubeSim(bookmark_ms=200) as sim:
            ctl = SimControl(sim.url)
            await ctl.apply([("ADDED", o) for s in scenarios for o in s.objects])
            srv = CqlServer(exec_statements=seed_cql_statements()).start()
            kc = tmp_path / "kubeconfig"
            kc.write_text(json.dumps({"clusters": [{"name": "c", "cluster": {"server": sim.url}}],
                                      "contexts": [{"name": "x", "context": {"cluster": "c"}}], "current-context": "x"}))
            cfg = load_config(path=None, env={}, overrides={
                "cql-store-type": "scylla", "workers": 8, "rate-limit-elements-per-second": 0, "resync-period": "0s",
                "kube-config-path": str(kc), "scylla-cql-store": {"hosts": f"127.0.0.1:{srv.port}"},
                "runtime": {"worker-processes": 2, "watch-hub": hub}, "observability": {"http-port": 0}})
            app = ShardedApplication(cfg, report_decisions=True, log_dir=str(tmp_path))
            decisions = []
            app.supervisor.decision_hooks.append(decisions.append)
            store = CqlCheckpointStore(CqlSession([srv.address]))
            await store.connect()
            try:
                await app.start()
                assert await app.wait_for_cache_sync(30), [w.proc.poll() for w in app.pool.workers]
                assert app.ready() and app.pool.alive()
                for _ in range(500):
                    if sum(1 for d in decisions if d.outcome == "applied") >= 7:
                        break
                    await asyncio.sleep(0.02)
                for s in scenarios:
                    for rid, stage in s.expected.items():
                        row = await store.read_checkpoint(ALGORITHM, rid)
                        assert row.lifecycle_stage == stage, (s.name, rid, row.lifecycle_stage)
                applied = [d for d in decisions if d.outcome == "applied"]
                assert all(d.result.stamps.get("ack_mono") for d in applied)
                # each run was decided by exactly one worker
                assert len({d.result.request_id for d in applied}) == len(applied)
                m = await app.refresh_metrics()
                assert m.counter("decisions_applied", {"stage": "FAILED", "class": "fatal"}) >= 1 or \
                    sum(v for k, v in m.counters.get("decisions_applied", {}).items()) >= 7
                objs = {k: v for k, v in m.gauges.get("informer_objects", {}).items() if ("kind", "Job") in k}
                assert len(objs) == 2  # one gauge per worker: each caches only its own runs
                st = await ctl.stats()
                assert st["watch_requests"] == (3 if hub else 6)  # one watch per kind per replica with the hub
                # a compaction that overtakes the streams: 410 → (hub) re-list → fresh snapshots
                late = [make_job(f"late-{i}", cfg.labels) for i in range(6)]
                await ctl.apply([("ADDED", j) for j in late], expire=True)
                live = (await ctl.stats())["objects"]["Job"]
                for _ in range(300):
                    m = await app.refresh_metrics()
                    jobs = sum(v for k, v in m.gauges.get("informer_objects", {}).items() if ("kind", "Job") in k)
                    if jobs == live and (not hub or app.hub.relists >= 4):
                        break
                    await asyncio.sleep(0.05)
                assert jobs == live  # every live Job cached by exactly one worker after the re-list
                if hub:
                    assert app.hub.relists >= 4  # 3 initial LISTs + the Job 410 re-list
                assert live >= 6
            finally:
                await app.stop(drain_timeout=5)
                await store.close()
                srv.stop()
                await ctl.close()
            assert all(w.proc.poll() == 0 for w in app.pool.workers), [w.proc.poll() for w in app.pool.workers]

    arun(go(), timeout=90)


@pytest.mark.slow
def test_sharded_obs_endpoints(arun, tmp_path):
    async def go():
        with KubeSim() as sim:
            kc = tmp_path / "kubeconfig"
            kc.write_text(json.dumps({"clusters": [{"name": "c", "cluster": {"server": sim.url}}],
                                      "contexts": [{"name": "x", "context": {"cluster": "c"}}], "current-context": "x"}))
            cfg = load_config(path=None, env={}, overrides={
                "cql-store-type": "memory", "resync-period": "0s", "kube-config-path": str(kc),
                "runtime": {"worker-processes": 2}, "observability": {"http-port": 0}})
            app = ShardedApplication(cfg)
            await app.start()
            from nexus_supervisor_amd.obs.http import ObsServer

            obs = ObsServer(app)
            port = await obs.start("127.0.0.1", 0)
            try:
                assert await app.wait_for_cache_sync(30)
                async with aiohttp.ClientSession() as s:
                    async with s.get(f"http://127.0.0.1:{port}/metrics") as r:
                        text = await r.text()
                        assert r.status == 200 and 'worker="1"' in text
                        assert 'nexus_supervisor_worker_processes_alive{version="0.1.0"} 2' in text
                    async with s.get(f"http://127.0.0.1:{port}/healthz") as r:
                        assert r.status == 200
                    async with s.get(f"http://127.0.0.1:{port}/readyz") as r:
                        assert r.status == 200 and "leader" in await r.text()
                    async with s.get(f"http://127.0.0.1:{port}/debug/vars") as r:
                        doc = await r.json()
                        assert doc["worker_processes"] == 2 and all(w["alive"] for w in doc["workers"])
                app.supervisor.set_active(False)
                await app.pool.refresh_metrics()
                m = app.pool.merged_metrics()
                assert all(v == 0.0 for v in m.gauges["active"].values())
            finally:
                await obs.stop()
                await app.stop(drain_timeout=5)

    arun(go(), timeout=90)


@pytest.mark.slow
def test_crashed_worker_restarts_and_leader_gating(arun, tmp_path):
    """A killed worker is restarted and replays its shard; with leader election on, the
    workers stay standby until the parent holds the Lease (kubesim serves the Lease)."""
    import os
    import signal

    async def go():
        labels = LabelConfig()
        with KubeSim(bookmark_ms=200) as sim:
            ctl = SimControl(sim.url)
            srv = CqlServer(exec_statements=seed_cql_statements()).start()
            kc = tmp_path / "kubeconfig"
            kc.write_text(json.dumps({"clusters": [{"name": "c", "cluster": {"server": sim.url}}],
                                      "contexts": [{"name": "x", "context": {"cluster": "c"}}], "current-context": "x"}))
            cfg = load_config(path=None, env={}, overrides={
                "cql-store-type": "scylla", "workers": 8, "rate-limit-elements-per-second": 0, "resync-period": "0s",
                "kube-config-path": str(kc), "scylla-cql-store": {"hosts": f"127.0.0.1:{srv.port}"},
                "runtime": {"worker-processes": 2},
                "leader-election": {"enabled": True, "lease-duration": "3s", "renew-deadline": "2s",
                                    "retry-period": "200ms", "identity": "replica-a"}})
            app = ShardedApplication(cfg, report_decisions=True, log_dir=str(tmp_path))
            app.pool.restart_backoff = (0.1, 0.5)
            decisions = []
            app.supervisor.decision_hooks.append(decisions.append)
            try:
                await app.start()
                assert await app.wait_for_cache_sync(30)
                for _ in range(200):  # the parent acquires the Lease and activates the workers
                    if app.pool.active:
                        break
                    await asyncio.sleep(0.05)
                assert app.pool.active and app.elector.leader
                victim = app.pool.workers[1].proc
                os.kill(victim.pid, signal.SIGKILL)
                for _ in range(200):
                    w = app.pool.workers[1]
                    if app.pool.restarts >= 1 and w.proc is not victim and w.synced.is_set():
                        break
                    await asyncio.sleep(0.05)
                assert app.pool.restarts == 1 and app.pool.alive() and app.ready()
                # runs of both workers are still decided after the restart
                scen = reference_scenarios()
                await ctl.apply([("ADDED", o) for s in scen for o in s.objects])
                for _ in range(400):
                    if sum(1 for d in decisions if d.outcome == "applied") >= 7:
                        break
                    await asyncio.sleep(0.05)
                owners = {worker_of(d.result.request_id, 2) for d in decisions if d.outcome == "applied"}
                assert owners == {0, 1}, [(d.result.request_id, d.outcome) for d in decisions]
            finally:
                await app.stop(drain_timeout=5)
                srv.stop()
                await ctl.close()

    arun(go(), timeout=120)


def test_remote_telemetry_mirror_matches_owner():
    from nexus_supervisor_amd.gpu.telemetry import FakeTelemetry, RemoteTelemetry, telemetry_message

    import time

    owner = FakeTelemetry(n_gpus=2)
    mirror = RemoteTelemetry()
    since = {}
    t = time.time() - 10
    owner.set_vram(1, 1000, t=t)
    owner.add_process(7, 1, vram_bytes=5 << 30, pod_uid="pod-a")
    mirror.update(json.loads(json.dumps(telemetry_message(owner, since))))
    owner.set_vram(1, 290000, t=t + 1)
    owner.set_vram(0, 5, t=t + 1.5)
    mirror.update(json.loads(json.dumps(telemetry_message(owner, since))))  # only the new samples travel
    assert mirror.peak_between(1, t - 1, t + 2) == owner.peak_between(1, t - 1, t + 2) == 290000
    assert mirror.peak_between(1, t - 1, t + 0.5) == 1000 and mirror.peak_between(0, t, t + 5) == 5
    assert [p["pod_uid"] for p in mirror.snapshot()[1]["procs"]] == ["pod-a"]
    assert len(mirror._hist[1]) == 2 and mirror.updates == 2


def test_evidence_provider_reuses_an_unchanged_mirror_snapshot():
    """A mirror returns the same snapshot list until its owner's next update: the
    provider keeps its per-snapshot memo across ttl expiries, and an update (which
    brings new VRAM samples too) rebuilds it."""
    import time

    from nexus_supervisor_amd.gpu.telemetry import FakeTelemetry, RemoteTelemetry, pod_evidence_provider, telemetry_message

    owner = FakeTelemetry(n_gpus=2)
    mirror = RemoteTelemetry(interval=0.01)
    since = {}
    owner.set_vram(1, 1000, t=time.time() - 1)
    mirror.update(json.loads(json.dumps(telemetry_message(owner, since))))
    prov = pod_evidence_provider(mirror)
    pod = make_pod("r", LabelConfig(), env={"LOCAL_RANK": "1", "HIP_VISIBLE_DEVICES": "0,1"}, gpus=1)
    a = prov(pod)
    time.sleep(0.02)  # past the ttl, same snapshot object
    b = prov(pod)
    assert a["gpus"] is b["gpus"] and a["gpus"][0]["vram_peak_mb"] == 1000
    owner.set_vram(1, 290000)
    mirror.update(json.loads(json.dumps(telemetry_message(owner, since))))
    time.sleep(0.02)
    c = prov(pod)
    assert c["gpus"] is not a["gpus"] and c["gpus"][0]["vram_peak_mb"] == 290000


@pytest.mark.slow
def test_worker_gpu_evidence_from_parent_monitor(arun, tmp_path):
    """Node-local attribution with worker processes: one monitor in the parent, mirrored into
    the workers; an HBM-OOM pod's row carries the GPU and the VRAM peak of its window."""
    from nexus_supervisor_amd.gpu.telemetry import FakeTelemetry
    from nexus_supervisor_amd.models.checkpoint import CheckpointedRequest, LifecycleStage

    async def go():
        labels = LabelConfig()
        tel = FakeTelemetry(n_gpus=8)
        tel.set_vram(3, 294000)
        env = {"LOCAL_RANK": "3", "RANK": "3", "WORLD_SIZE": "8", "HIP_VISIBLE_DEVICES": "0,1,2,3,4,5,6,7"}
        rids = [f"hbm-run-{i}" for i in (0, 1, 4, 5)]  # two per worker
        with KubeSim(bookmark_ms=200) as sim:
            ctl = SimControl(sim.url)
            srv = CqlServer(exec_statements=seed_cql_statements()).start()
            store = CqlCheckpointStore(CqlSession([srv.address]))
            await store.connect()
            for rid in rids:
                await store.upsert_checkpoint(CheckpointedRequest(algorithm=ALGORITHM, id=rid,
                                                                  lifecycle_stage=LifecycleStage.RUNNING))
            await ctl.apply([("ADDED", o) for rid in rids for o in (make_job(rid, labels),
                                                                   make_pod(rid, labels, env=env, gpus=1))])
            kc = tmp_path / "kubeconfig"
            kc.write_text(json.dumps({"clusters": [{"name": "c", "cluster": {"server": sim.url}}],
                                      "contexts": [{"name": "x", "context": {"cluster": "c"}}], "current-context": "x"}))
            cfg = load_config(path=None, env={}, overrides={
                "cql-store-type": "scylla", "rate-limit-elements-per-second": 0, "resync-period": "0s",
                "kube-config-path": str(kc), "scylla-cql-store": {"hosts": f"127.0.0.1:{srv.port}"},
                "runtime": {"worker-processes": 2}, "gpu": {"local-telemetry": True, "sample-interval": "100ms"}})
            app = ShardedApplication(cfg, report_decisions=True, log_dir=str(tmp_path), telemetry=tel)
            decisions = []
            app.supervisor.decision_hooks.append(decisions.append)
            try:
                await app.start()
                assert await app.wait_for_cache_sync(30)
                await asyncio.sleep(0.3)  # a mirror update or two
                failed = []
                for rid in rids:
                    p = make_pod(rid, labels, env=env, gpus=1, rv="3", status={
                        "phase": "Failed", "containerStatuses": [{"name": "algorithm", "restartCount": 0, "state": {
                            "terminated": {"reason": "Error", "exitCode": 1,
                                           "message": "torch.OutOfMemoryError: HIP out of memory. Tried to allocate 8.00 GiB"}}}]})
                    failed.append(("MODIFIED", p))
                await ctl.apply(failed)
                for _ in range(300):
                    if sum(1 for d in decisions if d.outcome == "applied") >= len(rids):
                        break
                    await asyncio.sleep(0.05)
                assert {worker_of(r, 2) for r in rids} == {0, 1}  # both workers took part
                for rid in rids:
                    row = await store.read_checkpoint(ALGORITHM, rid)
                    assert row.lifecycle_stage == LifecycleStage.FAILED, (rid, row)
                    trace = json.loads(row.algorithm_failure_details)
                    assert trace["class"] == "hbm-oom", trace
                    g = trace["gpu"]["gpus"][0]
                    assert g["index"] == 3 and g["vram_peak_mb"] == 294000, g
            finally:
                await app.stop(drain_timeout=5)
                await store.close()
                srv.stop()
                await ctl.close()

    arun(go(), timeout=90)


def test_hub_feed_protocol_split_reads_join_lines_and_keep_order():
    """Frames cut at every byte boundary parse the same; one kind's LINES frames of a read are
    joined into one queue item, a SNAPSHOT stays behind that kind's earlier lines, and frames
    of other kinds keep their own queues."""
    from nexus_supervisor_amd.parallel.watchhub import HEADER, LINES, SNAPSHOT, HubFeed, _FeedProtocol

    def frame(ftype, ki, payload):
        return HEADER.pack(ftype, ki, len(payload)) + payload

    stream = (frame(LINES, 1, b'{"a":1}\n') + frame(LINES, 2, b'{"j":1}\n') + frame(LINES, 1, b'{"a":2}\n')
              + frame(SNAPSHOT, 1, b"9\n[]") + frame(LINES, 1, b'{"a":3}\n') + frame(LINES, 9, b"x\n"))

    def drain(feed):
        out = {}
        for ki, q in feed.queues.items():
            items = []
            while not q.empty():
                items.append(q.get_nowait())
            out[ki] = items
        return out

    async def run(chunks):
        feed = HubFeed()
        proto = _FeedProtocol(feed)
        for c in chunks:
            proto.data_received(c)
        assert not proto.buf  # everything consumed
        return feed, drain(feed)

    async def go():
        feed, whole = await run([stream])
        assert whole[1] == [(LINES, b'{"a":1}\n{"a":2}\n'), (SNAPSHOT, b"9\n[]"), (LINES, b'{"a":3}\n')]
        assert whole[2] == [(LINES, b'{"j":1}\n')] and whole[0] == []
        assert feed.frames == 6
        _, bytewise = await run([stream[i:i + 1] for i in range(len(stream))])
        joined = {ki: [(t, p) for t, p in items] for ki, items in bytewise.items()}
        # one byte per read: nothing to join, same bytes in the same order per kind
        assert b"".join(p for t, p in joined[1] if t == LINES) == b'{"a":1}\n{"a":2}\n{"a":3}\n'
        assert [t for t, _ in joined[1]] == [LINES, LINES, SNAPSHOT, LINES]
        proto_feed = HubFeed()
        _FeedProtocol(proto_feed).connection_lost(None)
        assert all(q.get_nowait() == (0, b"") for q in proto_feed.queues.values())

    asyncio.run(go())


def test_router_forgets_deleted_pods_by_generation():
    """A deleted pod's owner stays known for Pod Events still in flight, for forget_after
    to twice that, then is forgotten wholesale with its generation (no per-entry erase on
    the hub's hot path); a live pod is never forgotten, and arena blocks are reused."""
    import time

    labels = LabelConfig()
    router = _kube_native.ShardRouter(0, 3, _SEED, JOB_LABEL, 0.2)
    sp_pod = _kube_native.WatchSplitter(router, "pod")
    pods = [make_pod(f"gen-{i}", labels) for i in range(2000)]
    sp_pod.feed(b"".join(_line("ADDED", p) for p in pods))
    assert router.stats["pods"] == 2000 and router.stats["gone"] == 0
    sp_pod.feed(b"".join(_line("DELETED", p) for p in pods[:1500]))
    st = router.stats
    assert st["pods"] == 500 and st["gone"] == 1500
    name = pods[0]["metadata"]["name"]
    assert router.pod_owner(name) == worker_of("gen-0", 3)  # remembered after its DELETE
    time.sleep(0.25)
    router.note_pod("other-a", 1, True)  # next deletion rotates: the 1500 move to the old generation
    assert router.pod_owner(name) == worker_of("gen-0", 3) and router.stats["gone"] == 1501
    time.sleep(0.25)
    router.note_pod("other-b", 2, True)  # second rotation: the first generation is dropped
    assert router.pod_owner(name) is None
    assert router.pod_owner("other-a") == 1 and router.pod_owner("other-b") == 2
    assert router.stats["gone"] == 2 and router.stats["pool_bytes"] >= 0  # freed blocks are pooled for reuse
    assert router.pod_owner(pods[1999]["metadata"]["name"]) == worker_of("gen-1999", 3)  # live: kept
    # a re-created pod of the same name is live again
    sp_pod.feed(_line("ADDED", pods[1]))
    assert router.pod_owner(pods[1]["metadata"]["name"]) == worker_of("gen-1", 3)
