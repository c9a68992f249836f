"""Native kube-apiserver simulator (``csrc/kubesim``): the supervisor's own REST/watch
client and informers against it, the same contract the Python fake apiserver is
tested for in ``test_kube_wire.py``, and the reference parity suite over
kubesim + the native CQL server."""
import asyncio

import pytest

from nexus_supervisor_amd.app import Application
from nexus_supervisor_amd.config import load_config
from nexus_supervisor_amd.informer import InformerFactory
from nexus_supervisor_amd.kube.client import KubeClient, KubeConfig, KubeListWatch
from nexus_supervisor_amd.kube.errors import ApiError, Conflict, NotFound
from nexus_supervisor_amd.store.cql import CqlCheckpointStore, CqlSession
from nexus_supervisor_amd.testing.cqlsrv import CqlServer
from nexus_supervisor_amd.testing.kubesim import KubeSim, SimControl
from nexus_supervisor_amd.testing.seed import ALGORITHM, make_event, make_job, make_pod, reference_scenarios, seed_cql_statements


def _cfg(**over):
    base = {"cql-store-type": "scylla", "workers": 4, "rate-limit-elements-per-second": 0,
            "rate-limit-elements-burst": 100, "failure-rate-base-delay": "100ms", "failure-rate-max-delay": "1s",
            "resync-period": "0s"}
    base.update(over)
    return load_config(path=None, env={}, overrides=base)


def test_apply_port_commits_beside_the_loop(arun):
    """Bulk applies on the apply port (read and prepared on their own threads, committed
    under the store lock) reach watches and REST like loop-port applies; the port serves
    nothing else."""
    import aiohttp

    async def go():
        labels = _cfg().labels
        with KubeSim(apply_threads=4, flush_threads=2) as sim:
            assert sim.apply_url and sim.apply_url != sim.url
            ctl = SimControl(sim.url, sim.apply_url)
            c = KubeClient(KubeConfig(sim.url))
            rv = str((await ctl.stats())["rv"])
            seen = []

            async def watch():
                async for t, o in c.watch("Pod", "nexus", rv, timeout_seconds=10):
                    seen.append((t, o["metadata"]["name"]))

            task = asyncio.ensure_future(watch())
            await asyncio.sleep(0.2)
            pods = [make_pod(f"a{i}", labels) for i in range(200)]
            out = await ctl.apply([("ADDED", p) for p in pods])
            assert out["applied"] == 200
            await c.delete("Pod", "nexus", pods[0]["metadata"]["name"])
            for _ in range(100):
                if len(seen) >= 201:
                    break
                await asyncio.sleep(0.05)
            task.cancel()
            await asyncio.gather(task, return_exceptions=True)
            assert len([s for s in seen if s[0] == "ADDED"]) == 200 and seen[-1] == ("DELETED", pods[0]["metadata"]["name"])
            items, _ = await c.list("Pod", "nexus")
            assert len(items) == 199
            st = await ctl.stats()
            assert st["apply_thread_ns"] > 0 and st["store_ns"] > 0
            # busy time per apply connection (one thread each): a second generator connection
            # is a second serial part, not more load on the first
            ctl2 = SimControl(sim.url, sim.apply_url)
            await ctl2.apply([("ADDED", make_pod("b0", labels))])
            conns = (await ctl.stats())["apply_conn_ns"]
            assert len(conns) == 2 and all(v > 0 for v in conns.values())
            assert sum(conns.values()) == (await ctl.stats())["apply_thread_ns"]
            await ctl2.close()
            async with aiohttp.ClientSession() as s:
                async with s.get(sim.apply_url + "/sim/stats") as r:
                    assert r.status == 404
            await c.close()
            await ctl.close()

    arun(go(), timeout=60)


def test_rest_semantics(arun):
    async def go():
        labels = _cfg().labels
        with KubeSim(token="t0k") as sim:
            ctl = SimControl(sim.url)
            out = await ctl.apply([("ADDED", make_pod(f"r{i}", labels)) for i in range(7)])
            assert out["applied"] == 7 and out["t_push"] > 0
            c = KubeClient(KubeConfig(sim.url, token="t0k"))
            items, rv = await c.list("Pod", "nexus", limit=3)  # 3 pages over one snapshot
            assert len(items) == 7 and items[0]["kind"] == "Pod" and int(rv) == out["rv"]
            assert all(i["metadata"]["uid"] and i["metadata"]["creationTimestamp"] for i in items)
            items, _ = await c.list("Pod", "nexus", label_selector="batch.kubernetes.io/job-name=r3")
            assert [i["metadata"]["name"] for i in items] == ["r3-acdey"]
            items, _ = await c.list("Pod", "nexus", label_selector="batch.kubernetes.io/job-name!=r3")
            assert len(items) == 6
            items, _ = await c.list("Pod", "nexus", field_selector="metadata.name=r5-acdey")
            assert [i["metadata"]["name"] for i in items] == ["r5-acdey"]
            got = await c.get("Pod", "nexus", "r1-acdey")
            patched = await c.patch_merge("Pod", "nexus", "r1-acdey", {"metadata": {"annotations": {"a": "b"}}})
            assert patched["metadata"]["annotations"] == {"a": "b"}
            assert patched["metadata"]["uid"] == got["metadata"]["uid"]
            with pytest.raises(Conflict):
                await c.replace("Pod", "nexus", "r1-acdey", got)  # stale resourceVersion
            fresh = await c.replace("Pod", "nexus", "r1-acdey", patched)
            assert int(fresh["metadata"]["resourceVersion"]) > int(patched["metadata"]["resourceVersion"])
            ev = make_event("Job", "r1", "DeadlineExceeded")
            ev["metadata"] = {"generateName": "r1.", "namespace": "nexus"}
            created = await c.create("Event", "nexus", ev)
            assert created["metadata"]["name"].startswith("r1.") and len(created["metadata"]["name"]) == 8
            await c.create("Job", "nexus", make_job("r1", labels))
            with pytest.raises(ApiError) as ei:
                await c.create("Job", "nexus", make_job("r1", labels))
            assert ei.value.status == 409
            await c.delete_job("nexus", "r1")  # Background: the Job's pod is garbage-collected
            with pytest.raises(NotFound):
                await c.get("Pod", "nexus", "r1-acdey")
            with pytest.raises(NotFound):
                await c.delete_job("nexus", "r1")
            st = await ctl.stats()
            assert st["objects"]["Pod"] == 6 and st["objects"]["Job"] == 0 and st["deleted"] == 2
            bad = KubeClient(KubeConfig(sim.url, token="nope"))
            with pytest.raises(ApiError) as ei:
                await bad.list("Pod", "nexus")
            assert ei.value.status == 401
            await bad.close()
            await c.close()
            await ctl.close()

    arun(go())


def test_event_noise_selector_on_list_and_watch(arun):
    """``informer-event-noise-selector``: the Event list/watch of a replica (and of the
    parent's watch hub) carries ``reason!=…`` for the start/stop reasons no rule reads, so
    the server never sends them; every reason a rule reads still arrives."""
    from nexus_supervisor_amd.app import build_factory
    from nexus_supervisor_amd.classify.classifier import EVENT_NOISE_REASONS, event_field_selector, event_reasons_read
    from nexus_supervisor_amd.parallel.sharding import watch_field_selector
    from nexus_supervisor_amd.parallel.watchhub import WatchHub

    sel = event_field_selector()
    read = event_reasons_read()
    assert sel and all(f"reason!={r}" in sel.split(",") for r in EVENT_NOISE_REASONS if r not in read)
    assert not any(t.split("!=")[1] in read for t in sel.split(","))
    assert watch_field_selector(_cfg(), "Pod") == "" and watch_field_selector(_cfg(), "Event") == sel
    assert watch_field_selector(_cfg(**{"informer-event-noise-selector": False}), "Event") == ""
    hub = WatchHub(_cfg(), None, 1, send=lambda *a: None, buffered=lambda w: 0, drain=lambda w: None)
    assert hub._path_params("Event")[1]["fieldSelector"] == sel
    assert "fieldSelector" not in hub._path_params("Pod")[1]

    kept = ["Started", "BackOff", "Failed", "FailedScheduling", "OutOfamd.com/gpu", "Evicted", "SomethingNew"]
    noise = list(EVENT_NOISE_REASONS)

    async def go():
        with KubeSim() as sim:
            ctl = SimControl(sim.url)
            c = KubeClient(KubeConfig(sim.url))
            await ctl.apply([("ADDED", make_event("Pod", f"p{i}", r)) for i, r in enumerate(kept[:3] + noise[:4])])
            lw = build_factory(_cfg(), c)._lw_for("Event")  # the single-process replica's Event source
            assert isinstance(lw, KubeListWatch) and lw.field_selector == sel
            items, rv = await lw.list()
            assert sorted(i["reason"] for i in items) == sorted(kept[:3])
            seen = []

            async def watch():
                async for t, o in lw.watch(rv):
                    seen.append(o["reason"])

            task = asyncio.ensure_future(watch())
            await asyncio.sleep(0.2)
            await ctl.apply([("ADDED", make_event("Pod", f"q{i}", r)) for i, r in enumerate(noise + kept[3:])])
            for _ in range(100):
                if len(seen) >= len(kept) - 3:
                    break
                await asyncio.sleep(0.05)
            await asyncio.sleep(0.2)
            task.cancel()
            await asyncio.gather(task, return_exceptions=True)
            assert sorted(seen) == sorted(kept[3:])
            await c.close()
            await ctl.close()

    arun(go(), timeout=60)


def test_pipelined_applies_commit_in_order(arun):
    """``SimControl.apply_pipelined``: chunks sent ahead of their answers on one apply
    connection commit in the order given (a watch sees ADDED, MODIFIED, DELETED, ADDED of
    one pod in that order), and concurrent callers each get a connection of their own."""
    from nexus_supervisor_amd.testing.kubesim import encode_events

    async def go():
        labels = _cfg().labels
        with KubeSim(apply_threads=2) as sim:
            ctl = SimControl(sim.url, sim.apply_url)
            c = KubeClient(KubeConfig(sim.url))
            rv = str((await ctl.stats())["rv"])
            seen = []

            async def watch():
                async for t, o in c.watch("Pod", "nexus", rv, timeout_seconds=10):
                    seen.append((t, o["metadata"]["name"], (o.get("status") or {}).get("phase")))

            task = asyncio.ensure_future(watch())
            await asyncio.sleep(0.2)
            p = make_pod("x", labels)
            q = dict(p, status={"phase": "Failed"})
            others = [[encode_events([("ADDED", make_pod(f"o{k}-{i}", labels))]) for i in range(20)] for k in range(2)]
            bodies = [encode_events(b) for b in ([("ADDED", p)], [("MODIFIED", q)], [("DELETED", q)], [("ADDED", p)])]
            docs, *rest = await asyncio.gather(ctl.apply_pipelined(bodies, depth=3),
                                               *(ctl.apply_pipelined(o, depth=4) for o in others))
            assert [d["applied"] for d in docs] == [1, 1, 1, 1] and all(len(r) == 20 for r in rest)
            assert len(ctl._streams) >= 2  # the concurrent calls did not share a connection
            for _ in range(100):
                if len(seen) >= 4 + 40:
                    break
                await asyncio.sleep(0.05)
            task.cancel()
            await asyncio.gather(task, return_exceptions=True)
            mine = [(t, ph) for t, n, ph in seen if n == p["metadata"]["name"]]
            assert [t for t, _ in mine] == ["ADDED", "MODIFIED", "DELETED", "ADDED"]
            await c.close()
            await ctl.close()

    arun(go(), timeout=60)


def test_async_gc_deletes_a_jobs_pods_after_the_answer(arun):
    """``--async-gc``: a Background Job DELETE is answered at once and the Job's pods are
    deleted afterwards on the GC thread (watchers see their DELETED lines); Foreground still
    deletes the pods before the answer."""
    async def go():
        labels = _cfg().labels
        with KubeSim(async_gc=True) as sim:
            ctl = SimControl(sim.url)
            await ctl.apply([("ADDED", o) for r in ("g1", "g2") for o in (make_job(r, labels), make_pod(r, labels))])
            c = KubeClient(KubeConfig(sim.url))
            rv = str((await ctl.stats())["rv"])
            seen = []

            async def watch():
                async for t, o in c.watch("Pod", "nexus", rv, timeout_seconds=10):
                    seen.append((t, o["metadata"]["name"]))

            task = asyncio.ensure_future(watch())
            await asyncio.sleep(0.2)
            await c.delete_job("nexus", "g1")  # Background
            for _ in range(100):
                if ("DELETED", "g1-acdey") in seen:
                    break
                await asyncio.sleep(0.02)
            assert ("DELETED", "g1-acdey") in seen
            with pytest.raises(NotFound):
                await c.get("Pod", "nexus", "g1-acdey")
            st = await ctl.stats()
            assert st["gc_pods"] == 1 and st["gc_pending"] == 0 and st["gc_ns"] > 0
            await c.request("DELETE", "/apis/batch/v1/namespaces/nexus/jobs/g2",
                            body={"kind": "DeleteOptions", "apiVersion": "v1", "propagationPolicy": "Foreground"})
            with pytest.raises(NotFound):  # gone before the answer
                await c.get("Pod", "nexus", "g2-acdey")
            assert (await ctl.stats())["gc_pods"] == 1
            task.cancel()
            await asyncio.gather(task, return_exceptions=True)
            await c.close()
            await ctl.close()

    arun(go(), timeout=60)


def test_resource_versions_spliced_consistently(arun):
    """Fully-formed objects are stored by splicing the new resourceVersion into the client's
    text (no re-serialisation): every stored / streamed copy must still be valid JSON with
    the server's RV, through create, update and the GC'd delete."""
    async def go():
        labels = _cfg().labels
        with KubeSim() as sim:
            ctl = SimControl(sim.url)
            job, pod = make_job("s1", labels, rv="77"), make_pod("s1", labels, rv="77")
            pod["metadata"]["annotations"] = {"note": 'quote " and \\ backslash', "unicode": "h\u00e9"}
            r = await ctl.apply([("ADDED", job), ("ADDED", pod)])
            c = KubeClient(KubeConfig(sim.url))
            got = await c.get("Pod", "nexus", "s1-acdey")
            assert got["metadata"]["resourceVersion"] == str(r["rv"]) and got["metadata"]["annotations"] == pod["metadata"]["annotations"]
            lines = []

            async def watch():
                async for et, o in c.watch("Pod", "nexus", str(r["rv"]), timeout_seconds=2):
                    lines.append((et, o["metadata"]["resourceVersion"], o))
                    if et == "DELETED":
                        return
            t = asyncio.create_task(watch())
            pod2 = dict(pod, status={"phase": "Running"})
            r2 = await ctl.apply([("MODIFIED", pod2)])
            await c.delete_job("nexus", "s1")
            await asyncio.wait_for(t, 5)
            assert [e for e, _, _ in lines] == ["MODIFIED", "DELETED"]
            assert lines[0][1] == str(r2["rv"]) and int(lines[1][1]) > r2["rv"]
            assert lines[1][2]["status"] == {"phase": "Running"} and lines[1][2]["metadata"]["uid"] == pod["metadata"]["uid"]
            # a watch resumed from the history replays the same DELETED line (its RV is
            # spliced into the removed object's text on send, not stored as a copy)
            replay = []
            async for et, o in c.watch("Pod", "nexus", str(r2["rv"]), timeout_seconds=1):
                replay.append((et, o["metadata"]["resourceVersion"], o))
                if et == "DELETED":
                    break
            assert replay == lines[1:]
            # server-owned metadata missing: inserted into the client's text (uid, timestamp, RV)
            bare = {"apiVersion": "batch/v1", "kind": "Job", "metadata": {"name": "bare", "namespace": "nexus"}}
            r3 = await ctl.apply([("ADDED", bare)])
            got = await c.get("Job", "nexus", "bare")
            md = got["metadata"]
            assert md["resourceVersion"] == str(r3["rv"]) and len(md["uid"]) == 36 and md["creationTimestamp"].endswith("Z")
            upd = {"apiVersion": "batch/v1", "kind": "Job", "metadata": {"name": "bare", "namespace": "nexus"},
                   "status": {"active": 1}}
            await ctl.apply([("MODIFIED", upd)])
            got2 = await c.get("Job", "nexus", "bare")
            assert got2["metadata"]["uid"] == md["uid"] and got2["metadata"]["creationTimestamp"] == md["creationTimestamp"]
            assert got2["status"] == {"active": 1} and int(got2["metadata"]["resourceVersion"]) > r3["rv"]
            await c.close()
            await ctl.close()

    arun(go())


def test_watch_resume_bookmarks_and_410_relist(arun):
    async def go():
        labels = _cfg().labels
        with KubeSim(bookmark_ms=50) as sim:
            ctl = SimControl(sim.url)
            await ctl.apply([("ADDED", make_job("a", labels))])
            c = KubeClient(KubeConfig(sim.url))
            # raw stream: bookmarks while idle, resume from an RV replays history
            _, rv0 = await c.list("Job", "nexus")
            await ctl.apply([("ADDED", make_job("b", labels))])
            seen = []
            async for et, o in c.watch("Job", "nexus", rv0, timeout_seconds=1):
                seen.append(et)
                if et == "BOOKMARK":
                    break
            assert seen[0] == "ADDED" and "BOOKMARK" in seen
            f = InformerFactory(lambda kind: KubeListWatch(c, kind, "nexus", watch_timeout=5), resync_period=0)
            inf = f.informer("Job")
            log = []
            inf.add_event_handler(on_add=lambda o: log.append(("add", o["metadata"]["name"])),
                                  on_update=lambda o, n: log.append(("upd", n["metadata"]["name"])),
                                  on_delete=lambda o: log.append(("del", o["metadata"]["name"])))
            f.start()
            assert await f.wait_for_cache_sync(5)
            j = make_job("a", labels)
            j["status"] = {"active": 1}
            await ctl.apply([("MODIFIED", j), ("ADDED", make_job("c", labels))])
            for _ in range(200):
                if ("upd", "a") in log and ("add", "c") in log:
                    break
                await asyncio.sleep(0.02)
            assert ("upd", "a") in log and ("add", "c") in log
            relists = inf.relists
            # compaction: the stream is cut and the resume gets 410 → re-list emits the diff
            await ctl.apply([("DELETED", make_job("b", labels)), ("ADDED", make_job("d", labels))], expire=True)
            for _ in range(300):
                if ("add", "d") in log and ("del", "b") in log:
                    break
                await asyncio.sleep(0.02)
            assert ("add", "d") in log and ("del", "b") in log
            assert inf.relists > relists
            assert sorted(inf.indexer.keys()) == ["nexus/a", "nexus/c", "nexus/d"]
            await f.stop()
            await c.close()
            await ctl.close()

    arun(go(), timeout=60)


def test_reference_parity_over_kubesim_and_cql(arun):
    scenarios = reference_scenarios()

    async def go():
        with KubeSim(bookmark_ms=200) as sim:
            ctl = SimControl(sim.url)
            await ctl.apply([("ADDED", o) for s in scenarios for o in s.objects])
            srv = CqlServer(exec_statements=seed_cql_statements()).start()
            cfg = _cfg()
            kube = KubeClient(KubeConfig(sim.url))
            store = CqlCheckpointStore(CqlSession([srv.address]))
            app = Application(cfg, kube=kube, store=store)
            decisions = []
            app.supervisor.decision_hooks.append(decisions.append)
            try:
                await app.start()
                assert await app.wait_for_cache_sync(10)
                for _ in range(500):
                    if len(decisions) >= 8:
                        break
                    await asyncio.sleep(0.02)
                await app.supervisor.pipeline.join(10)
                if app.supervisor._deletes:
                    await asyncio.wait(list(app.supervisor._deletes), timeout=10)
                for s in scenarios:
                    for rid, stage in s.expected.items():
                        row = await store.read_checkpoint(ALGORITHM, rid)
                        assert row.lifecycle_stage == stage, (s.name, rid, row.lifecycle_stage)
                st = await ctl.stats()
                assert st["deleted"] >= 5  # failing decisions deleted their Jobs (+ GC'd pods)
            finally:
                await app.stop()
                srv.stop()
                await ctl.close()

    arun(go(), timeout=60)


async def _fanout(sim, watchers=8, pods=300):
    """``watchers`` concurrent watches of one namespace, a burst of pod traffic: every
    watcher must see every line, in resourceVersion order."""
    labels = _cfg().labels
    ctl = SimControl(sim.url)
    out = await ctl.apply([("ADDED", make_pod(f"f{i}", labels)) for i in range(5)])
    rv0 = str(out["rv"])
    clients = [KubeClient(KubeConfig(sim.url)) for _ in range(watchers)]
    seen = [[] for _ in range(watchers)]

    async def watch(k):
        async for et, o in clients[k].watch("Pod", "nexus", rv0, timeout_seconds=20):
            if et == "BOOKMARK":
                continue
            seen[k].append(int(o["metadata"]["resourceVersion"]))
            if len(seen[k]) == pods:
                return

    tasks = [asyncio.create_task(watch(k)) for k in range(watchers)]
    await asyncio.sleep(0.2)
    for i in range(0, pods, 50):
        await ctl.apply([("ADDED", make_pod(f"g{j}", labels)) for j in range(i, i + 50)])
    await asyncio.wait_for(asyncio.gather(*tasks), 30)
    for s in seen:
        assert len(s) == pods and s == sorted(s)
    assert seen.count(seen[0]) == watchers
    for c in clients:
        await c.close()
    await ctl.close()


def test_parallel_watch_fanout(arun):
    """``--flush-threads``: the dirty watch streams of one loop iteration are written by a
    thread pool (a sharded deployment has every replica watching the whole namespace)."""
    async def go():
        with KubeSim(flush_threads=4) as sim:
            await _fanout(sim)

    arun(go())


@pytest.mark.slow
def test_parallel_watch_fanout_under_tsan(arun, monkeypatch):
    import os

    from nexus_supervisor_amd import _build

    try:
        _build.build(only=["kubesim"], sanitize="thread")
    except RuntimeError as exc:  # pragma: no cover - toolchain without the runtime
        pytest.skip(f"TSan build unavailable: {exc}")
    monkeypatch.setenv("NEXUS_KUBESIM_BINARY", os.path.join(_build.BIN, "nexus-kubesim-thread"))
    holder = {}

    async def go():
        sim = KubeSim(flush_threads=4).start(timeout=30)
        holder["sim"] = sim
        try:
            await _fanout(sim, watchers=6, pods=200)
        finally:
            sim.stop()

    arun(go(), timeout=120)
    log = holder["sim"].log()
    assert "ThreadSanitizer" not in log, log[-3000:]


def test_priced_apiserver_latency_throttle_and_write_cap(arun):
    """The simulator prices the API server.  --api-latency-us holds
    object answers (in order on a pipelined connection; LIST unaffected), --throttle-deletes
    answers the first Job DELETEs 429 + Retry-After (the client re-sends after the hint), and
    --write-qps caps mutating requests the way APF rejects them."""
    import time

    async def go():
        labels = _cfg().labels
        with KubeSim(api_latency_us=30_000, throttle_deletes=2, retry_after=1) as sim:
            ctl = SimControl(sim.url)
            await ctl.apply([("ADDED", make_job(f"j{i}", labels)) for i in range(6)])
            c = KubeClient(KubeConfig(sim.url))
            t0 = time.monotonic()
            await c.list("Job", "nexus")
            assert time.monotonic() - t0 < 0.025  # LIST is not priced
            t0 = time.monotonic()
            await c.get("Job", "nexus", "j0")
            assert time.monotonic() - t0 >= 0.029
            # pipelined DELETEs: answers keep their order, each ≥ the latency
            t0 = time.monotonic()
            futs = [c.delete_job("nexus", f"j{i}") for i in range(3, 6)]
            await asyncio.gather(*futs)
            took = time.monotonic() - t0
            assert took >= 1.0  # the first two DELETEs were throttled: re-sent after Retry-After 1
            assert c.throttled == 2 and c.retried == 2
            st = await ctl.stats()
            assert st["throttled"] == 2 and st["deleted"] == 3 and st["delayed"] >= 4
            await c.close()
        with KubeSim(write_qps=5, write_burst=2, retry_after=1) as sim:
            ctl = SimControl(sim.url)
            await ctl.apply([("ADDED", make_job(f"k{i}", labels)) for i in range(4)])
            c = KubeClient(KubeConfig(sim.url), max_retries=0)
            res = await asyncio.gather(*(c.delete_job("nexus", f"k{i}") for i in range(4)), return_exceptions=True)
            codes = sorted(getattr(r, "status", 200) for r in res)
            assert codes == [200, 200, 429, 429], codes
            assert all(r.retry_after == 1.0 for r in res if isinstance(r, ApiError))
            await c.close()

    arun(go(), timeout=30)


def test_pod_log_endpoint(arun):
    """pods/{name}/log from the simulator: the bench's default-pod HBM-OOMs keep their HIP
    text in the container log (a LOG line in /sim/apply, never sent to watchers)."""
    async def go():
        labels = _cfg().labels
        with KubeSim() as sim:
            ctl = SimControl(sim.url)
            pod = make_pod("lg", labels)
            text = "".join(f"line {i}\n" for i in range(50)) + "HIP out of memory\n"
            await ctl.apply([("ADDED", pod), ("LOG", {"namespace": "nexus", "pod": pod["metadata"]["name"],
                                                      "container": "algorithm", "text": text})])
            kc = KubeClient(KubeConfig(sim.url))
            st, body = await kc.pod_log("nexus", pod["metadata"]["name"], "algorithm", tail_lines=2, limit_bytes=1000)
            assert st == 200 and body == b"line 49\nHIP out of memory\n"
            st, body = await kc.pod_log("nexus", pod["metadata"]["name"], "algorithm", tail_lines=100, limit_bytes=12)
            assert st == 200 and body == b"line 0\nline "
            st, _ = await kc.pod_log("nexus", pod["metadata"]["name"], "sidecar")
            assert st == 400
            st, _ = await kc.pod_log("nexus", "nope", "algorithm")
            assert st == 404
            items, _ = await kc.list("Pod", "nexus")
            assert len(items) == 1  # the LOG line made no object
            await ctl.apply([("DELETED", pod)])
            await ctl.apply([("ADDED", pod)])
            st, _ = await kc.pod_log("nexus", pod["metadata"]["name"], "algorithm")
            assert st == 400  # the log went with the deleted pod
            await kc.close()
            await ctl.close()

    arun(go(), timeout=20)
