"""Helm chart render tests (no helm binary offline: ``deploy/render.py`` renders the
Go-template subset the chart uses).  Parity target: the reference chart maps the
same values to the same ``NEXUS__*`` env names
(``/root/reference/.helm/templates/deployment.yaml:48-67``)."""
import os
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deploy"))

from render import render_docs  # noqa: E402

from nexus_supervisor_amd.config import iter_keys, load_config  # noqa: E402

CHART = os.path.join(ROOT, "deploy", "helm", "nexus-supervisor-amd")


def _by_kind(docs):
    out = {}
    for d in docs:
        out.setdefault(d["kind"], []).append(d)
    return out


def _env(container):
    return {e["name"]: e.get("value") for e in container.get("env", [])}


def test_default_render_objects():
    k = _by_kind(render_docs(CHART))
    assert {"Deployment", "DaemonSet", "Role", "RoleBinding", "ServiceAccount", "Service", "PodDisruptionBudget"} <= set(k)
    dep = k["Deployment"][0]
    c = dep["spec"]["template"]["spec"]["containers"][0]
    assert c["args"] == ["supervisor"]
    assert c["livenessProbe"]["httpGet"]["path"] == "/healthz" and c["readinessProbe"]["httpGet"]["path"] == "/readyz"
    assert dep["spec"]["replicas"] == 2


def test_env_names_are_config_keys_and_load_back():
    dep = _by_kind(render_docs(CHART))["Deployment"][0]
    env = _env(dep["spec"]["template"]["spec"]["containers"][0])
    known = {name for _p, name, _d, _f in iter_keys()}
    nexus = {k: v for k, v in env.items() if k.startswith("NEXUS__")}
    assert set(nexus) <= known, set(nexus) - known
    # the reference's env names (deployment.yaml:48-67) are all present
    for name in ("NEXUS__RESOURCE_NAMESPACE", "NEXUS__CQL_STORE_TYPE", "NEXUS__LOG_LEVEL", "NEXUS__FAILURE_RATE_BASE_DELAY",
                 "NEXUS__FAILURE_RATE_MAX_DELAY", "NEXUS__RATE_LIMIT_ELEMENTS_PER_SECOND",
                 "NEXUS__RATE_LIMIT_ELEMENTS_BURST", "NEXUS__WORKERS", "NEXUS__KUBE_CONFIG_PATH"):
        assert name in nexus, name
    cfg = load_config(path=None, env=nexus)
    assert cfg.workers == 2 and cfg.rate_limit_elements_per_second == 10 and cfg.rate_limit_elements_burst == 100
    assert cfg.failure_rate_base_delay == pytest.approx(0.1) and cfg.failure_rate_max_delay == pytest.approx(1.0)
    assert cfg.cql_store_type == "astra" and cfg.resource_namespace == "nexus"
    assert cfg.leader_election.enabled and cfg.leader_election.lease_duration == 15.0
    assert cfg.gpu.evidence_wait == pytest.approx(2.0) and cfg.observability.http_port == 9100


def test_rbac_namespaced_and_cluster_scoped():
    k = _by_kind(render_docs(CHART))
    sup_role = [r for r in k["Role"] if not r["metadata"]["name"].endswith("gpu-agent")][0]
    rules = {(tuple(r["apiGroups"]), tuple(r["resources"])): set(r["verbs"]) for r in sup_role["rules"]}
    assert rules[(("",), ("events", "pods"))] == {"get", "list", "watch"}
    assert "delete" in rules[(("batch",), ("jobs",))]
    assert {"get", "create", "update"} <= rules[(("coordination.k8s.io",), ("leases",))]
    k2 = _by_kind(render_docs(CHART, sets=["rbac.clusterScoped=true"]))
    assert "ClusterRole" in k2 and "ClusterRoleBinding" in k2
    assert k2["ClusterRoleBinding"][0]["roleRef"]["kind"] == "ClusterRole"


def test_agent_daemonset_gpu_access():
    ds = _by_kind(render_docs(CHART))["DaemonSet"][0]
    spec = ds["spec"]["template"]["spec"]
    assert spec["hostPID"] is True
    mounts = {m["mountPath"] for m in spec["containers"][0]["volumeMounts"]}
    assert {"/dev/kfd", "/dev/dri", "/var/lib/kubelet/pod-resources"} <= mounts
    env = {e["name"]: e for e in spec["containers"][0]["env"]}
    assert env["NODE_NAME"]["valueFrom"]["fieldRef"]["fieldPath"] == "spec.nodeName"
    assert spec["nodeSelector"] == {"amd.com/gpu.product-name": "AMD_Instinct_MI355X_OAM"}
    assert "DaemonSet" not in _by_kind(render_docs(CHART, sets=["agent.enabled=false"]))


def test_scylla_and_datadog_values():
    docs = render_docs(CHART, values={"supervisor": {"config": {"cqlStore": {"type": "scylla", "scylla": {
        "hosts": ["scylla-0.scylla", "scylla-1.scylla"], "localDc": "dc1"}}}}, "datadog": {"enabled": True}})
    dep = _by_kind(docs)["Deployment"][0]
    c = dep["spec"]["template"]["spec"]["containers"][0]
    env = _env(c)
    assert env["NEXUS__SCYLLA_CQL_STORE__HOSTS"] == "scylla-0.scylla,scylla-1.scylla"
    cfg = load_config(path=None, env={k: v for k, v in env.items() if k.startswith("NEXUS__") and v is not None})
    assert cfg.scylla_cql_store.hosts == ["scylla-0.scylla", "scylla-1.scylla"] and cfg.scylla_cql_store.local_dc == "dc1"
    assert env["DD_DOGSTATSD_URL"] == "unix:///var/run/datadog/dsd.socket"
    assert any(v["name"] == "dsdsocket" for v in dep["spec"]["template"]["spec"]["volumes"])
    # the secretRef is rendered whenever secretRefEnabled (reference quirk fixed)
    assert c["envFrom"][0]["secretRef"]["name"].endswith("-cql")


def test_local_harness_files():
    """docker-compose (reference docker-compose.yaml), schema/seed file generated from the
    model, and the local config overlay."""
    import yaml

    sys_path_root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(sys_path_root, "tools"))
    import gen_test_resources

    with open(gen_test_resources.OUT) as f:
        assert f.read() == gen_test_resources.render(), "run tools/gen_test_resources.py"
    with open(os.path.join(sys_path_root, "deploy", "docker-compose.yaml")) as f:
        dc = yaml.safe_load(f)
    assert {"scylla", "prepare_scylla", "cqlsrv"} <= set(dc["services"])
    from nexus_supervisor_amd.config import load_config

    c = load_config(path=os.path.join(sys_path_root, "deploy", "appconfig.yaml"), env={"APPLICATION_ENVIRONMENT": "local"})
    assert c.cql_store_type == "scylla" and c.scylla_cql_store.hosts == ["127.0.0.1"] and c.observability.http_port == 8080


def test_kindload_manifests_seed_and_wait(arun):
    """BASELINE config 2 tooling: real failing Job manifests + row seeding + stage wait."""
    from nexus_supervisor_amd.bench import kindload as kl
    from nexus_supervisor_amd.bench.wire import schema_statements
    from nexus_supervisor_amd.testing.cqlsrv import CqlServer

    docs = kl.manifests(10, seed=3)
    assert len(docs) == 10 and len({d["metadata"]["name"] for d in docs}) == 10
    assert [d["metadata"]["name"] for d in docs] == [r for r, _ in kl.runs(10, seed=3)]
    oom = docs[0]["spec"]["template"]["spec"]["containers"][0]
    assert oom["resources"]["limits"]["memory"] == "24Mi" and "tail /dev/zero" in oom["command"][-1]
    assert docs[0]["spec"]["podFailurePolicy"]["rules"][0]["onExitCodes"]["values"] == [137, 255]
    assert ".invalid/" in docs[1]["spec"]["template"]["spec"]["containers"][0]["image"]
    labels = docs[0]["spec"]["template"]["metadata"]["labels"]
    assert labels["science.sneaksanddata.com/nexus-component"] == "algorithm-run"
    assert kl.to_yaml(docs).count("---\n") == 10
    srv = CqlServer(exec_statements=schema_statements()).start()
    try:
        addr = f"127.0.0.1:{srv.port}"

        async def go():
            assert await kl.seed_rows(addr, 10, seed=3) == 10
            st = await kl._store(addr)
            import datetime as dt

            for rid, stage in kl.expected(10, seed=3).items():
                await st.update_status(kl.ALGORITHM, rid, stage, "cause", "details", dt.datetime.now(dt.timezone.utc))
            await st.close()
            return await kl.wait_rows(addr, 10, seed=3, timeout=10, t_apply=time.time() - 1)

        res = arun(go())
        assert res["in_expected_stage"] == 10 and not res["wrong_stage"] and res["missing"] == 0
        assert res["apply_to_checkpoint_p50_ms"] > 0
    finally:
        srv.stop()


def test_reference_rbac_keys_are_honoured():
    """The reference chart's rbac.clusterRole.supervisor.* and
    rbac.clusterRoleBindings.* (/root/reference/.helm/values.yaml:34-53) are not ignored."""
    vals = {"rbac": {"clusterRole": {"supervisor": {"create": True, "additionalLabels": {"team": "ml"},
                                                    "additionalAnnotations": {"note": "x"}}},
                     "clusterRoleBindings": {"create": True}}}
    k = _by_kind(render_docs(CHART, values=vals))
    role = k["ClusterRole"][0]
    assert role["metadata"]["labels"]["team"] == "ml" and role["metadata"]["annotations"]["note"] == "x"
    assert k["ClusterRoleBinding"][0]["roleRef"]["kind"] == "ClusterRole"
    vals["rbac"]["clusterRoleBindings"]["create"] = False
    k = _by_kind(render_docs(CHART, values=vals))
    assert "ClusterRole" in k and "ClusterRoleBinding" not in k
    vals["rbac"]["clusterRole"]["supervisor"]["create"] = False
    k = _by_kind(render_docs(CHART, values=vals))
    assert "ClusterRole" not in k and all(r["metadata"]["name"].endswith("gpu-agent") for r in k.get("Role", []))


def test_sharding_values_render_lease_mode():
    docs = render_docs(CHART, values={"supervisor": {"replicas": 3, "highAvailability": {"sharding": {"shards": 6}}}})
    env = _env(_by_kind(docs)["Deployment"][0]["spec"]["template"]["spec"]["containers"][0])
    cfg = load_config(path=None, env={k: v for k, v in env.items() if k.startswith("NEXUS__") and v is not None})
    assert cfg.sharding.shards == 6 and cfg.sharding.mode == "lease" and cfg.sharding.replicas == 3
    assert "NEXUS__SHARDING__SHARDS" not in _env(_by_kind(render_docs(CHART))["Deployment"][0]["spec"]["template"]["spec"]["containers"][0])


def test_role_name_override_and_log_tail_access():
    """The reference's rbac.clusterRole.supervisor.nameOverride
    (/root/reference/.helm/templates/_helpers.tpl:77-83) names the role and its binding;
    the supervisor may read pods/log and the node agent mounts /var/log/pods read-only
    (the HBM-OOM text of a default pod lives in its container log)."""
    vals = {"rbac": {"clusterRole": {"supervisor": {"create": True, "nameOverride": "nexus-sup-role"}}}}
    k = _by_kind(render_docs(CHART, values=vals))
    assert k["ClusterRole"][0]["metadata"]["name"] == "nexus-sup-role"
    assert k["ClusterRoleBinding"][0]["roleRef"]["name"] == "nexus-sup-role"
    role = [r for r in _by_kind(render_docs(CHART))["Role"] if not r["metadata"]["name"].endswith("gpu-agent")][0]
    assert any(r["resources"] == ["pods/log"] and r["verbs"] == ["get"] for r in role["rules"])
    ds = _by_kind(render_docs(CHART))["DaemonSet"][0]["spec"]["template"]["spec"]
    mounts = {m["mountPath"]: m for m in ds["containers"][0]["volumeMounts"]}
    assert mounts["/var/log/pods"]["readOnly"] is True
    assert {e["name"]: e.get("value") for e in ds["containers"][0]["env"]}["NEXUS_AGENT_LOG_ROOT"] == "/var/log/pods"


def test_dry_run_value_renders_shadow_mode():
    def cfg_of(values=None):
        env = _env(_by_kind(render_docs(CHART, values=values))["Deployment"][0]["spec"]["template"]["spec"]["containers"][0])
        return load_config(path=None, env={k: v for k, v in env.items() if k.startswith("NEXUS__") and v is not None})

    assert cfg_of().dry_run is False
    assert cfg_of({"supervisor": {"config": {"dryRun": True}}}).dry_run is True


def test_monitoring_objects_are_optional_and_name_real_metrics():
    """PodMonitor + PrometheusRule (off by default); every metric an alert names is one the
    supervisor exports (Prometheus exposition of the statsd namespace)."""
    import re

    assert not {"PodMonitor", "PrometheusRule"} & set(_by_kind(render_docs(CHART)))
    k = _by_kind(render_docs(CHART, values={"supervisor": {"observability": {
        "podMonitor": True, "prometheusRule": {"enabled": True, "gpuFaultThreshold": 2}}}}))
    pm = k["PodMonitor"][0]["spec"]
    assert pm["podMetricsEndpoints"][0] == {"port": "http-metrics", "path": "/metrics"}
    rules = {r["alert"]: r for g in k["PrometheusRule"][0]["spec"]["groups"] for r in g["rules"]}
    assert set(rules) == {"NexusGpuFailingRuns", "NexusDecisionsDeadLettered", "NexusNoActiveSupervisor"}
    assert rules["NexusGpuFailingRuns"]["expr"].endswith(">= 2")
    names = {n for r in rules.values() for n in re.findall(r"(nexus_supervisor_[a-z_]+)", r["expr"])}
    assert names == {"nexus_supervisor_gpu_failures_total", "nexus_supervisor_decisions_dead_lettered_total",
                     "nexus_supervisor_active"}


def test_record_events_value_grants_event_create():
    def role(values=None):
        return [r for r in _by_kind(render_docs(CHART, values=values))["Role"]
                if not r["metadata"]["name"].endswith("gpu-agent")][0]

    def creates_events(r):
        return any("events" in x["resources"] and "create" in x["verbs"] for x in r["rules"])

    assert not creates_events(role())
    vals = {"supervisor": {"observability": {"recordEvents": True}}}
    assert creates_events(role(vals))
    env = _env(_by_kind(render_docs(CHART, values=vals))["Deployment"][0]["spec"]["template"]["spec"]["containers"][0])
    cfg = load_config(path=None, env={k: v for k, v in env.items() if k.startswith("NEXUS__") and v is not None})
    assert cfg.observability.record_events is True
