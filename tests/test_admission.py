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
