"""The shard-label admission webhook (``nexus_supervisor_amd/admission.py``): what stamps
``sharding.shard-label`` when the Job's submitter does not.  The reference scales by
adding replicas with no submitter cooperation (``/root/reference/.helm/values.yaml:124-125``);
here unlabelled Jobs from the submitter still reach only their shard's replica."""
import asyncio
import base64
import json
import os
import shutil
import ssl
import subprocess
import sys

import pytest

from nexus_supervisor_amd.admission import WebhookServer, relabel_owned, review, shard_label_patch
from nexus_supervisor_amd.app import Application
from nexus_supervisor_amd.config import load_config
from nexus_supervisor_amd.kube.client import KubeClient, KubeConfig
from nexus_supervisor_amd.models.checkpoint import CheckpointedRequest
from nexus_supervisor_amd.parallel.sharding import shard_of
from nexus_supervisor_amd.store.memory import MemoryStore
from nexus_supervisor_amd.testing.fake_apiserver import FakeApiServer, json_patch
from nexus_supervisor_amd.testing.seed import ALGORITHM, make_job, make_pod

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LABEL = "nexus.amd.com/shard"


def _cfg(index=0, shards=2, **over):
    base = {"cql-store-type": "memory", "rate-limit-elements-per-second": 0, "resync-period": "0s",
            "sharding": {"shards": shards, "shard-index": index, "shard-label": LABEL}}
    base.update(over)
    return load_config(path=None, env={}, overrides=base)


def _review(obj, op="CREATE"):
    return {"apiVersion": "admission.k8s.io/v1", "kind": "AdmissionReview",
            "request": {"uid": "u-1", "operation": op, "object": obj}}


def _job_with_template(name, labels, **extra_labels):
    job = make_job(name, labels)
    job["metadata"]["labels"].update(extra_labels)
    job["spec"] = {"template": {"metadata": {"labels": dict(job["metadata"]["labels"])}, "spec": {}}}
    return job


def test_review_patches_job_and_template_and_pod():
    cfg = _cfg(shards=4)
    job = _job_with_template("run-a", cfg.labels)
    out = review(_review(job), cfg)
    resp = out["response"]
    assert out["kind"] == "AdmissionReview" and resp["uid"] == "u-1" and resp["allowed"] is True
    assert resp["patchType"] == "JSONPatch"
    patched = json_patch(job, json.loads(base64.b64decode(resp["patch"])))
    want = str(shard_of("run-a", 4))
    assert patched["metadata"]["labels"][LABEL] == want
    assert patched["spec"]["template"]["metadata"]["labels"][LABEL] == want
    # "/" in the label key is escaped in the JSON pointer
    assert any(op["path"].endswith("nexus.amd.com~1shard") for op in json.loads(base64.b64decode(resp["patch"])))
    # a pod of the Job: by its job-name label
    pod = make_pod("run-a", cfg.labels)
    pp = json_patch(pod, json.loads(base64.b64decode(review(_review(pod), cfg)["response"]["patch"])))
    assert pp["metadata"]["labels"][LABEL] == want
    # already right: admitted without a patch; wrong (another shard count): replaced
    assert "patch" not in review(_review(patched), cfg)["response"]
    stale = json.loads(json.dumps(patched))
    stale["metadata"]["labels"][LABEL] = "99"
    ops = shard_label_patch(stale, cfg)
    assert {"op": "replace", "path": "/metadata/labels/nexus.amd.com~1shard", "value": want} in ops


def test_review_leaves_others_alone_and_never_vetoes():
    cfg = _cfg(shards=4)
    other = make_job("web-frontend", cfg.labels)
    other["metadata"]["labels"] = {"app": "web"}
    r = review(_review(other), cfg)["response"]
    assert r["allowed"] is True and "patch" not in r
    anon = make_job("", cfg.labels)
    anon["metadata"]["generateName"] = "run-"
    assert shard_label_patch(anon, cfg) is None
    assert "patch" not in review(_review(anon), cfg)["response"]
    assert "patch" not in review(_review(make_job("run-b", cfg.labels), "UPDATE"), cfg)["response"]
    off = _cfg(shards=1)
    assert "patch" not in review(_review(make_job("run-b", off.labels)), off)["response"]


def test_chart_registers_the_webhook():
    sys.path.insert(0, os.path.join(ROOT, "deploy"))
    from render import render_docs

    chart = os.path.join(ROOT, "deploy", "helm", "nexus-supervisor-amd")
    assert not [d for d in render_docs(chart) if d["kind"] == "MutatingWebhookConfiguration"]
    docs = render_docs(chart, values={"supervisor": {"highAvailability": {"sharding": {
        "shards": 4, "shardLabel": LABEL, "webhook": {"enabled": True, "certSecret": "wh-tls", "caBundle": "Q0E="}}}}})
    kinds = {}
    for d in docs:
        kinds.setdefault(d["kind"], []).append(d)
    wh = kinds["MutatingWebhookConfiguration"][0]["webhooks"][0]
    assert wh["failurePolicy"] == "Ignore" and wh["sideEffects"] == "None" and wh["admissionReviewVersions"] == ["v1"]
    assert wh["clientConfig"]["service"]["path"] == "/mutate-shard-label" and wh["clientConfig"]["caBundle"] == "Q0E="
    assert {(tuple(r["apiGroups"]), tuple(r["resources"])) for r in wh["rules"]} == {(("batch",), ("jobs",)),
                                                                                       (("",), ("pods",))}
    assert all(r["operations"] == ["CREATE"] for r in wh["rules"])
    svc = [s for s in kinds["Service"] if s["metadata"]["name"].endswith("-webhook")][0]
    assert svc["spec"]["ports"][0]["targetPort"] == "webhook"
    c = kinds["Deployment"][0]["spec"]["template"]["spec"]["containers"][0]
    env = {e["name"]: e.get("value") for e in c["env"]}
    assert env["NEXUS__SHARDING__SHARD_LABEL"] == LABEL and env["NEXUS__SHARDING__WEBHOOK_PORT"] == "9443"
    assert {"name": "webhook-tls", "mountPath": "/etc/nexus/webhook-tls", "readOnly": True} in c["volumeMounts"]
    sup_role = [r for r in kinds["Role"] if not r["metadata"]["name"].endswith("gpu-agent")][0]
    assert {"apiGroups": ["batch"], "resources": ["jobs"], "verbs": ["patch"]} in sup_role["rules"]


def _self_signed(tmp_path):
    if shutil.which("openssl") is None:
        pytest.skip("openssl not available")
    subprocess.run(["openssl", "req", "-x509", "-newkey", "rsa:2048", "-nodes", "-days", "1", "-subj", "/CN=127.0.0.1",
                    "-addext", "subjectAltName=IP:127.0.0.1", "-keyout", str(tmp_path / "tls.key"),
                    "-out", str(tmp_path / "tls.crt")], check=True, capture_output=True)
    client = ssl.create_default_context(cafile=str(tmp_path / "tls.crt"))
    return str(tmp_path), client


def test_fake_apiserver_calls_the_webhook_over_tls(tmp_path, arun):
    """AdmissionReview round trip as the API server makes it: HTTPS with the CA bundle,
    JSON patch applied to the stored Job; an unreachable webhook admits unchanged."""
    cert_dir, client_ctx = _self_signed(tmp_path)

    async def go():
        cfg = _cfg(shards=4)
        ws = WebhookServer(cfg)
        port = await ws.start("127.0.0.1", 0, cert_dir)
        assert ws.tls
        api = FakeApiServer()
        url = await api.start()
        api.add_mutating_webhook(f"https://127.0.0.1:{port}/mutate-shard-label", ssl_ctx=client_ctx)
        kc = KubeClient(KubeConfig(url))
        await kc.create("Job", "nexus", _job_with_template("run-tls", cfg.labels))
        stored = api.get("Job", "nexus", "run-tls")
        want = str(shard_of("run-tls", 4))
        assert stored["metadata"]["labels"][LABEL] == want
        assert stored["spec"]["template"]["metadata"]["labels"][LABEL] == want
        await ws.stop()
        await kc.create("Job", "nexus", _job_with_template("run-down", cfg.labels))  # failurePolicy: Ignore
        assert LABEL not in api.get("Job", "nexus", "run-down")["metadata"]["labels"] and api.webhook_failures == 1
        await kc.close()
        await api.stop()

    arun(go(), timeout=30)


def test_unlabelled_submissions_reach_only_their_shard(arun):
    """Two static-shard replicas with ``sharding.shard-label``; replica 0 serves the
    webhook.  The "submitter" creates Jobs and Pods through the API without the label: the
    webhook stamps them, each replica's narrowed watches deliver only its shard's runs, and
    every failure is decided by its owner."""
    async def go():
        api = FakeApiServer(bookmark_interval=0.1)
        url = await api.start()
        cfg0 = _cfg(0, **{"sharding": {"shards": 2, "shard-index": 0, "shard-label": LABEL, "webhook-port": 0}})
        ws = WebhookServer(cfg0)
        port = await ws.start("127.0.0.1", 0, "")
        api.add_mutating_webhook(f"http://127.0.0.1:{port}/mutate-shard-label")
        labels = cfg0.labels
        rids = [f"sub-{i:02d}" for i in range(20)]
        submitter = KubeClient(KubeConfig(url))
        for r in rids:
            await submitter.create("Job", "nexus", _job_with_template(r, labels))
            await submitter.create("Pod", "nexus", make_pod(r, labels, status={"phase": "Running"}))
        assert api.webhook_calls == 2 * len(rids)
        store = MemoryStore([CheckpointedRequest(algorithm=ALGORITHM, id=r, lifecycle_stage="RUNNING") for r in rids])
        apps = [Application(_cfg(k), kube=KubeClient(KubeConfig(url)), store=store) for k in (0, 1)]
        for a in apps:
            await a.start()
            await a.factory.wait_for_cache_sync(5)
        for k, a in enumerate(apps):
            mine = {r for r in rids if shard_of(r, 2) == k}
            pods = {p["metadata"]["labels"]["batch.kubernetes.io/job-name"] for p in a.supervisor.pod_informer.indexer.values()}
            jobs = {j["metadata"]["name"] for j in a.supervisor.job_informer.indexer.values()}
            assert pods == mine and jobs == mine, k
        for r in rids:
            p = json.loads(json.dumps(api.get("Pod", "nexus", f"{r}-acdey")))
            p["status"] = {"phase": "Failed", "containerStatuses": [{"name": "algorithm", "restartCount": 0, "state": {
                "terminated": {"reason": "OOMKilled", "exitCode": 137}}}]}
            api.update(p)
        for _ in range(200):
            if all(store.get(ALGORITHM, r).lifecycle_stage == "FAILED" for r in rids):
                break
            await asyncio.sleep(0.02)
        assert all(store.get(ALGORITHM, r).lifecycle_stage == "FAILED" for r in rids)
        per = [a.metrics.counter("decisions_applied", {"stage": "FAILED", "class": "host-oom"}) for a in apps]
        assert per == [sum(1 for r in rids if shard_of(r, 2) == k) for k in (0, 1)]
        for a in apps:
            await a.stop()
        await ws.stop()
        await submitter.close()
        await api.stop()

    arun(go(), timeout=40)


def test_relabel_after_the_shard_count_changed(arun):
    """Runs labelled for 2 shards, replicas now configured for 4: each replica re-stamps
    the runs of its own shards (Jobs and Pods), so together they fix every run."""
    async def go():
        api = FakeApiServer()
        url = await api.start()
        labels = _cfg(0).labels
        rids = [f"old-{i:02d}" for i in range(24)]
        for r in rids:
            job, pod = make_job(r, labels), make_pod(r, labels)
            for o in (job, pod):
                o["metadata"]["labels"][LABEL] = str(shard_of(r, 2))
                api.create(o)
        kc = KubeClient(KubeConfig(url))
        total = 0
        for k in range(4):
            cfg = _cfg(k, shards=4)
            got = await relabel_owned(cfg, kc, {k})
            total += got["relabelled"]
            assert got["errors"] == 0
        for r in rids:
            want = str(shard_of(r, 4))
            assert api.get("Job", "nexus", r)["metadata"]["labels"][LABEL] == want
            assert api.get("Pod", "nexus", f"{r}-acdey")["metadata"]["labels"][LABEL] == want
        wrong_before = sum(2 for r in rids if shard_of(r, 2) != shard_of(r, 4))
        assert total == wrong_before
        again = await relabel_owned(_cfg(0, shards=4), kc, None)
        assert again["relabelled"] == 0 and again["checked"] == 2 * len(rids)
        await kc.close()
        await api.stop()

    arun(go(), timeout=30)


def test_webhook_outage_runs_are_repaired_and_decided(arun):
    """The webhook is down (failurePolicy: Ignore) while 100 Nexus Jobs and their pods are
    submitted unlabelled: invisible to both shard-narrowed replicas — until each replica's
    audit re-stamps the runs of its shards.  Every run is decided within one audit interval
    plus settle (the reference can not lose a run this way: every replica sees everything,
    ``/root/reference/.helm/values.yaml:124-125``)."""
    import time as _time

    async def go():
        api = FakeApiServer(bookmark_interval=0.1)
        url = await api.start()
        api.add_mutating_webhook("http://127.0.0.1:9/mutate-shard-label")  # nothing listens there
        labels = _cfg(0).labels
        rids = [f"outage-{i:03d}" for i in range(100)]
        store = MemoryStore([CheckpointedRequest(algorithm=ALGORITHM, id=r, lifecycle_stage="RUNNING") for r in rids])
        interval = 0.5
        apps = [Application(_cfg(k, **{"sharding": {"shards": 2, "shard-index": k, "shard-label": LABEL,
                                                     "audit-interval": f"{interval}s"}}),
                            kube=KubeClient(KubeConfig(url)), store=store) for k in (0, 1)]
        for a in apps:
            await a.start()
            await a.factory.wait_for_cache_sync(5)
        submitter = KubeClient(KubeConfig(url))
        t0 = _time.monotonic()
        for r in rids:
            await submitter.create("Job", "nexus", _job_with_template(r, labels))
            pod = make_pod(r, labels, status={"phase": "Failed", "containerStatuses": [{
                "name": "algorithm", "restartCount": 0, "state": {"terminated": {"reason": "OOMKilled", "exitCode": 137}}}]})
            await submitter.create("Pod", "nexus", pod)
        assert api.webhook_failures == 2 * len(rids)  # every submission admitted unlabelled
        for _ in range(400):
            if all(store.get(ALGORITHM, r).lifecycle_stage == "FAILED" for r in rids):
                break
            await asyncio.sleep(0.02)
        took = _time.monotonic() - t0
        assert all(store.get(ALGORITHM, r).lifecycle_stage == "FAILED" for r in rids)
        assert took < interval + 3.0, took
        repaired = [a.metrics.counter("shard_label_repaired") for a in apps]
        assert sum(repaired) == 2 * len(rids) and all(repaired)  # each replica fixed its own shard's runs
        per = [a.metrics.counter("decisions_applied", {"stage": "FAILED", "class": "host-oom"}) for a in apps]
        assert per == [sum(1 for r in rids if shard_of(r, 2) == k) for k in (0, 1)]
        for a in apps:
            await a.stop()
        await submitter.close()
        await api.stop()

    arun(go(), timeout=60)


def test_audit_fixes_labels_of_a_stale_shard_count(arun):
    """a Job labelled with an in-range value computed for another shard count
    (an old replica's webhook during a rolling change of ``shards``) matches the wrong
    replica's selector.  The replica whose selector it matches moves it to its owner on the
    periodic full check (``relabel-every``); out-of-range values are caught every pass."""
    async def go():
        api = FakeApiServer()
        url = await api.start()
        labels = _cfg(0).labels
        rids = [f"stale-{i:02d}" for i in range(40)]
        for r in rids:
            job, pod = make_job(r, labels), make_pod(r, labels)
            for o in (job, pod):
                o["metadata"]["labels"][LABEL] = str(shard_of(r, 2))  # stamped for 2 shards
                api.create(o)
        api.create(dict(make_job("stale-x", labels), metadata=dict(make_job("stale-x", labels)["metadata"],
                                                                    labels=dict(labels_with(labels), **{LABEL: "7"}))))
        kc = KubeClient(KubeConfig(url))
        from nexus_supervisor_amd.admission import ShardLabelKeeper

        outs = []
        for k in range(4):
            cfg = _cfg(k, shards=4, **{"sharding": {"shards": 4, "shard-index": k, "shard-label": LABEL,
                                                     "relabel-every": 1}})
            keeper = ShardLabelKeeper(cfg, kc, None, None, lambda k=k: {k}, interval=0)
            outs.append(await keeper.audit_pass())
        assert sum(o["missing"] for o in outs) == 4  # "7" names no shard: every replica counts it
        for r in rids + ["stale-x"]:
            assert api.get("Job", "nexus", r)["metadata"]["labels"][LABEL] == str(shard_of(r, 4)), r
        for r in rids:
            assert api.get("Pod", "nexus", f"{r}-acdey")["metadata"]["labels"][LABEL] == str(shard_of(r, 4)), r
        assert sum(o["wrong"] for o in outs) >= 1
        again = ShardLabelKeeper(_cfg(0, shards=4, **{"sharding": {"shards": 4, "shard-label": LABEL,
                                                                    "relabel-every": 1}}),
                                 kc, None, None, lambda: None, interval=0)
        assert (await again.audit_pass())["repaired"] == 0
        await kc.close()
        await api.stop()

    arun(go(), timeout=30)


def labels_with(labels):
    from nexus_supervisor_amd.testing.seed import run_labels

    return run_labels(labels)


def test_relabel_passes_run_one_at_a_time_and_merge(arun):
    """shard gains while a re-label pass runs are merged into the next pass;
    never two passes at once; stop() cancels the pass."""
    from nexus_supervisor_amd.admission import ShardLabelKeeper

    class SlowKube:
        def __init__(self):
            self.active = 0
            self.max_active = 0
            self.lists = []

        async def request(self, method, path, params=None, body=None):
            self.active += 1
            self.max_active = max(self.max_active, self.active)
            await asyncio.sleep(0.05)
            self.active -= 1
            self.lists.append(path)
            return {"items": []}

        async def patch_merge(self, *a, **k):
            return {}

    async def go():
        kube = SlowKube()
        keeper = ShardLabelKeeper(_cfg(0, shards=8), kube, None, None, lambda: {0}, interval=0)
        keeper.request_relabel({1})
        await asyncio.sleep(0.01)
        keeper.request_relabel({2})
        keeper.request_relabel({3})
        for _ in range(100):
            if keeper._relabel is not None and keeper._relabel.done():
                break
            await asyncio.sleep(0.02)
        assert kube.max_active == 1
        assert len(kube.lists) == 4  # two passes (Jobs + Pods each): {1}, then {2, 3} merged
        keeper.request_relabel({4})
        await keeper.stop()
        assert keeper._relabel is None

    arun(go(), timeout=20)


def test_webhook_reloads_a_renewed_certificate_and_reports_expiry(tmp_path, arun):
    """cert-manager renews the mounted Secret — the webhook serves the new
    certificate without a restart; webhook_cert_expiry_seconds tracks the one served."""
    if shutil.which("openssl") is None:
        pytest.skip("openssl not available")
    from nexus_supervisor_amd.obs.metrics import Metrics

    def mint(days, cn):
        subprocess.run(["openssl", "req", "-x509", "-newkey", "rsa:2048", "-nodes", "-days", str(days), "-subj",
                        f"/CN={cn}", "-addext", "subjectAltName=IP:127.0.0.1", "-keyout", str(tmp_path / "new.key"),
                        "-out", str(tmp_path / "new.crt")], check=True, capture_output=True)
        os.replace(tmp_path / "new.key", tmp_path / "tls.key")
        os.replace(tmp_path / "new.crt", tmp_path / "tls.crt")

    async def peer_cn(port):
        ctx = ssl.create_default_context()
        ctx.check_hostname = False
        ctx.verify_mode = ssl.CERT_NONE
        r, w = await asyncio.open_connection("127.0.0.1", port, ssl=ctx)
        der = w.get_extra_info("ssl_object").getpeercert(binary_form=True)
        w.close()
        return der

    async def go():
        mint(1, "first")
        m = Metrics("t")
        ws = WebhookServer(_cfg(shards=4), m, reload_interval=0)
        port = await ws.start("127.0.0.1", 0, str(tmp_path))
        exp1 = m.gauge("webhook_cert_expiry_seconds")
        assert 0 < exp1 <= 86400 + 60
        der1 = await peer_cn(port)
        assert ws.check_cert() is False  # unchanged files: nothing reloaded
        mint(30, "second")
        assert ws.check_cert() is True and ws.reloads == 1
        der2 = await peer_cn(port)
        assert der2 != der1
        assert m.gauge("webhook_cert_expiry_seconds") > 29 * 86400
        await ws.stop()

    arun(go(), timeout=30)


def test_cert_bootstrap_mints_one_pair_for_all_replicas_and_sets_ca_bundle(tmp_path, arun):
    """sharding.webhook-cert-bootstrap: no cert-manager — two replicas race to mint the
    webhook's certificate; one pair wins the Secret's compare-and-swap and both serve it;
    the MutatingWebhookConfiguration's caBundle is set, and the API server verifies the
    webhook with it.  Near expiry the pair is renewed with the old CA kept in the bundle."""
    from nexus_supervisor_amd.webhook_certs import WebhookCertBootstrap, decode_cert

    async def go():
        api = FakeApiServer()
        url = await api.start()
        api.create({"apiVersion": "admissionregistration.k8s.io/v1", "kind": "MutatingWebhookConfiguration",
                    "metadata": {"name": "nexus-shard-label"},
                    "webhooks": [{"name": "shard-label.nexus.amd.com", "clientConfig": {"service": {
                        "name": "nexus-webhook", "namespace": "nexus", "path": "/mutate-shard-label"}}}]})
        kcs = [KubeClient(KubeConfig(url)) for _ in range(2)]
        boots = [WebhookCertBootstrap(kc, "nexus", "nexus-webhook-tls", "nexus-shard-label", "nexus-webhook",
                                      str(tmp_path / f"r{i}")) for i, kc in enumerate(kcs)]
        pairs = await asyncio.gather(*(b.sync() for b in boots))
        assert pairs[0][1]["tls.crt"] == pairs[1][1]["tls.crt"]  # one pair for every replica
        assert sum(b.minted for b in boots) >= 1
        sec = api.get("Secret", "nexus", "nexus-webhook-tls")
        assert sec["type"] == "kubernetes.io/tls" and set(sec["data"]) == {"tls.crt", "tls.key", "ca.crt"}
        info = decode_cert(pairs[0][1]["tls.crt"])
        assert ("DNS", "nexus-webhook.nexus.svc") in info["subjectAltName"]
        wh = api.get("MutatingWebhookConfiguration", "", "nexus-shard-label")["webhooks"][0]
        ca = base64.b64decode(wh["clientConfig"]["caBundle"]).decode()
        assert ca == pairs[0][1]["ca.crt"]
        # the API server (trusting caBundle) calls the webhook serving the minted pair
        cfg = _cfg(shards=4)
        ws = WebhookServer(cfg, reload_interval=0)
        port = await ws.start("127.0.0.1", 0, str(tmp_path / "r0"))
        client = ssl.create_default_context(cadata=ca)
        client.check_hostname = False  # dialled by IP here; the SAN names the Service
        api.add_mutating_webhook(f"https://127.0.0.1:{port}/mutate-shard-label", ssl_ctx=client)
        await kcs[0].create("Job", "nexus", _job_with_template("boot-1", cfg.labels))
        assert api.get("Job", "nexus", "boot-1")["metadata"]["labels"][LABEL] == str(shard_of("boot-1", 4))
        assert api.webhook_failures == 0
        # a second sync changes nothing; 340 days later the pair is renewed, old CA kept
        assert (await boots[1].sync())[0] is False and boots[1].ca_patches == 0
        later = boots[0]
        later.clock = lambda: __import__("time").time() + 340 * 86400
        changed, fresh = await later.sync()
        assert changed and fresh["tls.crt"] != pairs[0][1]["tls.crt"]
        bundle = base64.b64decode(api.get("MutatingWebhookConfiguration", "", "nexus-shard-label")
                                  ["webhooks"][0]["clientConfig"]["caBundle"]).decode()
        assert bundle.count("BEGIN CERTIFICATE") == 2 and bundle.endswith(ca)
        assert ws.check_cert() is True  # the server picks the renewed pair up
        await ws.stop()
        for kc in kcs:
            await kc.close()
        await api.stop()

    arun(go(), timeout=30)


def test_chart_cert_bootstrap_and_audit_settings():
    sys.path.insert(0, os.path.join(ROOT, "deploy"))
    from render import render_docs

    chart = os.path.join(ROOT, "deploy", "helm", "nexus-supervisor-amd")
    docs = render_docs(chart, values={"supervisor": {"highAvailability": {"sharding": {
        "shards": 4, "shardLabel": LABEL, "auditInterval": "30s", "webhook": {"enabled": True, "certBootstrap": True}}}}})
    kinds = {}
    for d in docs:
        kinds.setdefault(d["kind"], []).append(d)
    wh = kinds["MutatingWebhookConfiguration"][0]
    assert "caBundle" not in wh["webhooks"][0]["clientConfig"]  # the replicas set it
    c = kinds["Deployment"][0]["spec"]["template"]["spec"]["containers"][0]
    env = {e["name"]: e.get("value") for e in c["env"]}
    assert env["NEXUS__SHARDING__WEBHOOK_CERT_BOOTSTRAP"] == "true"
    assert env["NEXUS__SHARDING__WEBHOOK_CONFIG_NAME"] == wh["metadata"]["name"]
    assert env["NEXUS__SHARDING__AUDIT_INTERVAL"] == "30s" and env["NEXUS__SHARDING__REPAIR_LABELS"].lower() == "true"
    svc = [s for s in kinds["Service"] if s["metadata"]["name"].endswith("-webhook")][0]
    assert env["NEXUS__SHARDING__WEBHOOK_SERVICE"] == svc["metadata"]["name"]
    vols = {v["name"]: v for v in kinds["Deployment"][0]["spec"]["template"]["spec"]["volumes"]}
    assert "emptyDir" in vols["webhook-tls"]
    cr = [r for r in kinds["ClusterRole"] if r["metadata"]["name"].endswith("-webhook-ca")][0]
    assert cr["rules"][0]["resourceNames"] == [wh["metadata"]["name"]] and set(cr["rules"][0]["verbs"]) == {"get", "update"}
    sup_role = [r for r in kinds["Role"] if not r["metadata"]["name"].endswith("gpu-agent")][0]
    assert {"apiGroups": [""], "resources": ["secrets"], "resourceNames": [env["NEXUS__SHARDING__WEBHOOK_SECRET"]],
            "verbs": ["get", "update"]} in sup_role["rules"]
    # the config the chart renders loads (every env name is a real key)
    from nexus_supervisor_amd.config import load_config

    cfg = load_config(path=None, env={k: v for k, v in env.items() if k.startswith("NEXUS__") and v is not None})
    assert cfg.sharding.webhook_cert_bootstrap and cfg.sharding.audit_interval == 30.0
