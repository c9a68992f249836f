"""Kubernetes REST/watch client against the fake apiserver, and the reference parity
suite end to end over real protocols (HTTP watch + CQL over TCP) — the analog of
``/root/reference/services/supervisor_test.go:542-580`` with fake client-go
replaced by an HTTP apiserver and docker Scylla by the native CQL server."""
import asyncio
import os

import pytest

from nexus_supervisor_amd.app import Application
from nexus_supervisor_amd.config import load_config
from nexus_supervisor_amd.informer import InformerFactory
from nexus_supervisor_amd.kube.client import KubeClient, KubeConfig, KubeListWatch
from nexus_supervisor_amd.kube.errors import Conflict, NotFound
from nexus_supervisor_amd.models.decisions import Decision
from nexus_supervisor_amd.store.cql import CqlCheckpointStore, CqlSession
from nexus_supervisor_amd.testing.cqlsrv import CqlServer
from nexus_supervisor_amd.testing.fake_apiserver import FakeApiServer
from nexus_supervisor_amd.testing.seed import ALGORITHM, make_event, make_job, make_pod, reference_scenarios, seed_cql_statements, seed_rows


def _cfg(**over):
    base = {"cql-store-type": "scylla", "workers": 4, "rate-limit-elements-per-second": 10,
            "rate-limit-elements-burst": 10, "failure-rate-base-delay": "100ms", "failure-rate-max-delay": "1s",
            "resync-period": "0s"}
    base.update(over)
    return load_config(path=None, env={}, overrides=base)


# ---------------------------------------------------------------- client
def test_list_pagination_get_patch_put_delete(arun):
    async def go():
        api = FakeApiServer(token="t0k")
        url = await api.start()
        for i in range(7):
            api.create(make_pod(f"r{i}", _cfg().labels))
        c = KubeClient(KubeConfig(url, token="t0k"))
        items, rv = await c.list("Pod", "nexus", limit=3)
        assert len(items) == 7 and int(rv) == api.rv and items[0]["kind"] == "Pod"
        sel = f"batch.kubernetes.io/job-name=r3"
        items, _ = await c.list("Pod", "nexus", label_selector=sel)
        assert [i["metadata"]["name"] for i in items] == ["r3-acdey"]
        got = await c.get("Pod", "nexus", "r1-acdey")
        patched = await c.patch_merge("Pod", "nexus", "r1-acdey", {"metadata": {"annotations": {"a": "b"}}})
        assert patched["metadata"]["annotations"] == {"a": "b"}
        with pytest.raises(Conflict):
            await c.replace("Pod", "nexus", "r1-acdey", got)  # stale resourceVersion
        api.create(make_job("r1", _cfg().labels))
        await c.delete_job("nexus", "r1")
        assert api.get("Job", "nexus", "r1") is None and api.get("Pod", "nexus", "r1-acdey") is None  # GC'd
        assert ("Job", "nexus", "r1", "Background") in api.deleted
        with pytest.raises(NotFound):
            await c.delete_job("nexus", "r1")
        bad = KubeClient(KubeConfig(url, token="nope"))
        with pytest.raises(Exception) as ei:
            await bad.list("Pod", "nexus")
        assert getattr(ei.value, "status", 0) == 401
        await bad.close()
        await c.close()
        await api.stop()

    arun(go())


def test_watch_stream_and_410_relist_through_informer(arun):
    async def go():
        api = FakeApiServer(bookmark_interval=0.05)
        url = await api.start()
        labels = _cfg().labels
        api.create(make_job("a", labels))
        c = KubeClient(KubeConfig(url))
        f = InformerFactory(lambda kind: KubeListWatch(c, kind, "nexus", watch_timeout=5), resync_period=0)
        inf = f.informer("Job")
        seen = []
        inf.add_event_handler(on_add=lambda o: seen.append(("add", o["metadata"]["name"])),
                              on_update=lambda o, n: seen.append(("upd", n["metadata"]["name"])),
                              on_delete=lambda o: seen.append(("del", o["metadata"]["name"])))
        f.start()
        assert await f.wait_for_cache_sync(5)
        api.create(make_job("b", labels))
        j = dict(api.get("Job", "nexus", "a"))
        j["status"] = {"active": 1}
        api.update(j)
        for _ in range(100):
            if ("upd", "a") in seen:
                break
            await asyncio.sleep(0.02)
        assert ("add", "a") in seen and ("add", "b") in seen and ("upd", "a") in seen
        # compaction while watching: the stream is dropped, the resume gets 410, the informer re-lists
        api.expire("Job")
        api.delete("Job", "nexus", "b")
        api.create(make_job("c", labels))
        api.expire("Job")
        for _ in range(200):
            if ("add", "c") in seen and ("del", "b") in seen:
                break
            await asyncio.sleep(0.02)
        assert ("add", "c") in seen and ("del", "b") in seen
        assert inf.relists >= 2
        assert sorted(inf.indexer.keys()) == ["nexus/a", "nexus/c"]
        await f.stop()
        await c.close()
        await api.stop()

    arun(go())


def test_kubeconfig_and_in_cluster(tmp_path, monkeypatch):
    kc = tmp_path / "config"
    kc.write_text("""
apiVersion: v1
kind: Config
current-context: dev
clusters:
- name: c1
  cluster: {server: "https://10.0.0.1:6443", insecure-skip-tls-verify: true}
contexts:
- name: dev
  context: {cluster: c1, user: u1, namespace: nexus}
users:
- name: u1
  user: {token: abc}
""")
    cfg = KubeConfig.load(str(kc))
    assert cfg.server == "https://10.0.0.1:6443" and cfg.bearer() == "abc" and cfg.insecure and cfg.namespace == "nexus"
    assert cfg.ssl_context() is not None
    sa = tmp_path / "sa"
    sa.mkdir()
    (sa / "token").write_text("sa-token\n")
    (sa / "namespace").write_text("nexus")
    import nexus_supervisor_amd.kube.client as kc_mod

    monkeypatch.setattr(kc_mod, "SA_DIR", str(sa))
    monkeypatch.setenv("KUBERNETES_SERVICE_HOST", "10.96.0.1")
    monkeypatch.setenv("KUBERNETES_SERVICE_PORT", "443")
    ic = KubeConfig.load("")
    assert ic.server == "https://10.96.0.1:443" and ic.bearer() == "sa-token" and ic.namespace == "nexus"
    monkeypatch.delenv("KUBERNETES_SERVICE_HOST")
    with pytest.raises(Exception):
        KubeConfig.load("")


# ---------------------------------------------------------------- parity over the wire
async def _wire_cluster(objects, cfg=None, store_rows=True):
    api = FakeApiServer(bookmark_interval=0.2)
    url = await api.start()
    for o in objects:
        api.create(o)
    srv = CqlServer(exec_statements=seed_cql_statements() if store_rows else []).start()
    cfg = cfg or _cfg()
    cfg.scylla_cql_store.hosts = [f"127.0.0.1:{srv.port}"]
    kube = KubeClient(KubeConfig(url))
    store = CqlCheckpointStore(CqlSession([srv.address]))
    app = Application(cfg, kube=kube, store=store)
    decisions = []
    app.supervisor.decision_hooks.append(decisions.append)
    await app.start()
    assert await app.factory.wait_for_cache_sync(10)
    return api, srv, app, store, decisions


async def _settle(app, decisions, n, timeout=10.0):
    t = asyncio.get_running_loop().time()
    while len(decisions) < n and asyncio.get_running_loop().time() - t < timeout:
        await asyncio.sleep(0.02)
    await app.supervisor.pipeline.join(timeout)
    if app.supervisor._deletes:  # background Job DELETEs
        await asyncio.wait(list(app.supervisor._deletes), timeout=timeout)


def test_reference_parity_over_http_and_cql(arun):
    scenarios = reference_scenarios()

    async def go():
        objs = [o for s in scenarios for o in s.objects]
        api, srv, app, store, decisions = await _wire_cluster(objs)
        try:
            await _settle(app, decisions, 8)
            for s in scenarios:
                for rid, stage in s.expected.items():
                    row = await store.read_checkpoint(ALGORITHM, rid)
                    assert row.lifecycle_stage == stage, (s.name, rid, row.lifecycle_stage)
            # failing decisions deleted their Jobs through the API (Background propagation)
            deleted = {n for k, _, n, p in api.deleted if k == "Job" and p == "Background"}
            for s in scenarios:
                for rid, stage in s.expected.items():
                    if stage in ("FAILED", "SCHEDULING_FAILED", "DEADLINE_EXCEEDED") and any(o["kind"] == "Job" for o in s.objects):
                        assert rid in deleted, (s.name, rid)
            assert "df1b6e8d-cc3c-fb5b-a3f6-5d7b9e2c7f2b" not in deleted  # CANCELLED run untouched
        finally:
            await app.stop()
            srv.stop()
            await api.stop()

    arun(go(), timeout=60)


def test_restart_replay_is_idempotent(arun):
    """a restarted supervisor re-lists every live event; finished rows and
    RUNNING→RUNNING make the replay a no-op (no extra writes, no extra deletes)."""
    scenarios = reference_scenarios()

    async def go():
        objs = [o for s in scenarios for o in s.objects]
        api, srv, app, store, decisions = await _wire_cluster(objs)
        try:
            await _settle(app, decisions, 8)
            rows1 = {r.id: await store.read_checkpoint(ALGORITHM, r.id) for r in seed_rows()}
            await app.stop()
            n_deleted = len(api.deleted)
            store2 = CqlCheckpointStore(CqlSession([srv.address]))
            cfg = _cfg()
            cfg.scylla_cql_store.hosts = [f"127.0.0.1:{srv.port}"]
            app2 = Application(cfg, kube=KubeClient(KubeConfig(api.url)), store=store2)
            d2 = []
            app2.supervisor.decision_hooks.append(d2.append)
            await app2.start()
            await app2.factory.wait_for_cache_sync(10)
            await _settle(app2, d2, 1, timeout=2)
            rows2 = {r.id: await store2.read_checkpoint(ALGORITHM, r.id) for r in seed_rows()}
            assert rows1 == rows2
            assert all(d.outcome != "applied" for d in d2), [(d.result.request_id, d.outcome) for d in d2]
            assert len(api.deleted) == n_deleted
            await app2.stop()
        finally:
            srv.stop()
            await api.stop()

    arun(go(), timeout=60)


def test_late_event_then_object_is_not_lost(arun):
    """An Event whose Job is not cached yet is parked (the reference drops it as stale,
    supervisor.go:161-164) and decided once the Job arrives."""
    labels = _cfg().labels
    rid = seed_rows()[0].id

    async def go():
        api, srv, app, store, decisions = await _wire_cluster([])
        try:
            api.create(make_event("Job", rid, "FailedCreate", message="quota exceeded"))
            await asyncio.sleep(0.2)
            api.create(make_job(rid, labels))
            await _settle(app, decisions, 1)
            row = await store.read_checkpoint(ALGORITHM, rid)
            assert row.lifecycle_stage == "SCHEDULING_FAILED" and row.algorithm_failure_details == "quota exceeded"
        finally:
            await app.stop()
            srv.stop()
            await api.stop()

    arun(go(), timeout=60)


def test_kubeconfig_exec_credential_plugin(arun, tmp_path):
    """users[].user.exec (EKS/GKE style): the plugin's ExecCredential token authenticates,
    and is re-run once it expires."""
    import sys

    plugin = tmp_path / "cred.py"
    count = tmp_path / "count"
    plugin.write_text(
        "import json, os, sys\n"
        f"p = {str(count)!r}\n"
        "n = int(open(p).read()) + 1 if os.path.exists(p) else 1\n"
        "open(p, 'w').write(str(n))\n"
        "assert json.loads(os.environ['KUBERNETES_EXEC_INFO'])['kind'] == 'ExecCredential'\n"
        "print(json.dumps({'apiVersion': 'client.authentication.k8s.io/v1', 'kind': 'ExecCredential',\n"
        "                  'status': {'token': os.environ['TOK'], 'expirationTimestamp': '2000-01-01T00:00:00Z'}}))\n")
    kc = tmp_path / "config"

    async def go():
        api = FakeApiServer(token="s3cret")
        url = await api.start()
        kc.write_text(f"""apiVersion: v1
kind: Config
current-context: c
clusters: [{{name: k, cluster: {{server: "{url}"}}}}]
contexts: [{{name: c, context: {{cluster: k, user: u}}}}]
users:
- name: u
  user:
    exec:
      apiVersion: client.authentication.k8s.io/v1
      command: {sys.executable}
      args: ["{plugin}"]
      env: [{{name: TOK, value: s3cret}}]
""")
        cfg = KubeConfig.load(str(kc))
        c = KubeClient(cfg)
        api.create(make_pod("r1", _cfg().labels))
        items, _ = await c.list("Pod", "nexus")
        assert len(items) == 1
        await c.list("Pod", "nexus")  # already-expired credential: plugin runs again
        assert int(count.read_text()) >= 2
        await c.close()
        await api.stop()

    arun(go())


def test_background_job_delete_retries_on_api_errors(arun):
    """The Job DELETE after a durable write goes out on the pipelined connection without a
    task; a 500 from the API server falls back to the retrying path until it succeeds."""
    rows = [r for r in seed_rows() if r.lifecycle_stage in ("RUNNING", "BUFFERED")][:2]
    labels = _cfg().labels
    objs = []
    for r in rows:
        objs += [make_job(r.id, labels), make_pod(r.id, labels)]

    async def go():
        api, srv, app, store, decisions = await _wire_cluster(objs)
        try:
            def fail(rid, rv):
                p = make_pod(rid, labels, rv=rv)
                p["status"] = {"phase": "Failed", "containerStatuses": [
                    {"name": "algorithm", "state": {"terminated": {"reason": "OOMKilled", "exitCode": 137}}}]}
                api.update(p)

            fail(rows[0].id, "50")  # opens the pipelined write connections
            await _settle(app, decisions, 1)
            assert api.get("Job", "nexus", rows[0].id) is None
            api.fail_next[("DELETE", "Job")] = 2
            fail(rows[1].id, "51")
            await _settle(app, decisions, 2)
            for _ in range(100):
                if api.get("Job", "nexus", rows[1].id) is None:
                    break
                await asyncio.sleep(0.05)
            assert api.get("Job", "nexus", rows[1].id) is None
            m = app.supervisor.metrics
            assert m.counter("job_delete_retries") >= 1 and m.counter("jobs_deleted") >= 2
        finally:
            await app.stop()
            await api.stop()
            srv.stop()

    arun(go())


def test_record_events_puts_the_decision_on_the_job(arun):
    """observability.record-events: each failing decision leaves a Warning Event
    (NexusRunFailed) on its Job; the supervisor's own Event informer ignores it (no extra
    decisions), and a RUNNING transition records nothing."""
    scenarios = reference_scenarios()

    async def go():
        objs = [o for s in scenarios for o in s.objects]
        api, srv, app, store, decisions = await _wire_cluster(objs, cfg=_cfg(**{"observability": {"record-events": True}}))
        try:
            await _settle(app, decisions, 8)
            for _ in range(100):
                if not app.supervisor._event_tasks:
                    break
                await asyncio.sleep(0.02)
            evs = [e for e in api.objects["Event"].values() if e.get("reason") == "NexusRunFailed"]
            failing = {rid for s in scenarios for rid, st in s.expected.items()
                       if st in ("FAILED", "SCHEDULING_FAILED", "DEADLINE_EXCEEDED")}
            assert {e["involvedObject"]["name"] for e in evs} == failing
            assert all(e["type"] == "Warning" and e["involvedObject"]["kind"] == "Job" for e in evs)
            pfp = next(e for e in evs if e["involvedObject"]["name"] == "1d7b6e8d-cc3c-fb5b-a3f6-5d7b9e2c7f2b")
            assert pfp["message"].startswith("FAILED (fatal): Algorithm encountered a fatal error")
            await asyncio.sleep(0.3)  # the informer has seen them: still one decision per run
            assert len([d for d in decisions if d.outcome == "applied"]) == len(failing) + 1  # + the RUNNING run
        finally:
            await app.stop()
            srv.stop()
            await api.stop()

    arun(go(), timeout=60)


def _self_signed(tmp_path):
    """A throw-away CA-less server certificate for 127.0.0.1 (the openssl CLI)."""
    import shutil
    import subprocess

    if shutil.which("openssl") is None:
        pytest.skip("openssl CLI not available")
    key, crt = tmp_path / "tls.key", tmp_path / "tls.crt"
    subprocess.run(["openssl", "req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", str(key), "-out", str(crt),
                    "-days", "1", "-subj", "/CN=127.0.0.1", "-addext", "subjectAltName=IP:127.0.0.1"],
                   check=True, capture_output=True)
    return str(crt), str(key)


def test_tls_and_bearer_token_on_every_path(arun, tmp_path):
    """A real kube-apiserver answers only over TLS and wants the ServiceAccount token: the
    informers' LIST / WATCH (aiohttp), the pipelined Job DELETE and the keep-alive pods/log
    read (the fast client) all verify the server against the kubeconfig's CA and send the
    bearer token — a decision end to end over TLS, then the fast paths directly."""
    import ssl

    crt, key = _self_signed(tmp_path)
    server_ctx = ssl.create_default_context(ssl.Purpose.CLIENT_AUTH)
    server_ctx.load_cert_chain(crt, key)
    rows = [r for r in seed_rows() if r.lifecycle_stage == "RUNNING"][:2]
    labels = _cfg().labels

    async def go():
        api = FakeApiServer(bookmark_interval=0.1, token="sa-token")
        url = await api.start(ssl_context=server_ctx)
        assert url.startswith("https://")
        for r in rows:
            api.create(make_job(r.id, labels))
            api.create(make_pod(r.id, labels, status={"phase": "Running"}))
        from nexus_supervisor_amd.store.memory import MemoryStore

        store = MemoryStore(rows)
        kc = KubeClient(KubeConfig(url, token="sa-token", ca_file=crt))
        app = Application(_cfg(**{"cql-store-type": "memory", "rate-limit-elements-per-second": 0}), kube=kc,
                          store=store)
        await app.start()
        assert await app.factory.wait_for_cache_sync(5)
        p = api.get("Pod", "nexus", f"{rows[0].id}-acdey")
        p = dict(p, status={"phase": "Failed", "containerStatuses": [
            {"name": "algorithm", "state": {"terminated": {"reason": "OOMKilled", "exitCode": 137}}}]})
        api.update(p)
        for _ in range(200):
            if store.get(ALGORITHM, rows[0].id).lifecycle_stage == "FAILED" and api.get("Job", "nexus", rows[0].id) is None:
                break
            await asyncio.sleep(0.02)
        assert store.get(ALGORITHM, rows[0].id).lifecycle_stage == "FAILED"
        assert api.get("Job", "nexus", rows[0].id) is None  # the pipelined DELETE, over TLS
        # the fast paths directly: a pipelined DELETE future and a pods/log read
        fut = kc.delete_job_nowait("nexus", rows[1].id)
        assert fut is not None
        kc.check_delete(await fut)
        assert api.get("Job", "nexus", rows[1].id) is None
        api.create(make_pod("tls-log", labels, status={"phase": "Running"}))  # the Jobs' pods were collected
        logged = api.get("Pod", "nexus", "tls-log-acdey")["metadata"]["name"]
        api.set_pod_log("nexus", logged, "algorithm", "hello over tls\n")
        status, body = await kc.pod_log("nexus", logged, "algorithm")
        assert status == 200 and body == b"hello over tls\n"
        # a client without the token is refused on the fast path too
        anon = KubeClient(KubeConfig(url, ca_file=crt))
        status, _ = await anon.pod_log("nexus", logged, "algorithm")
        assert status == 401
        # and one that does not trust the server's certificate never gets an answer
        untrusting = KubeClient(KubeConfig(url, token="sa-token"))
        with pytest.raises(Exception):
            await untrusting.pod_log("nexus", logged, "algorithm", timeout=2.0)
        for c in (anon, untrusting):
            await c.close()
        await app.stop()
        await api.stop()

    arun(go(), timeout=30)
