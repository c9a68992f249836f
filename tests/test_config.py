"""Config surface: every reference key, env names, defaults = Helm defaults."""
import os

import pytest

from nexus_supervisor_amd.config import ConfigError, env_name, iter_keys, load_config, redacted
from nexus_supervisor_amd.utils import format_duration, parse_duration

REFERENCE_KEYS = [
    ("astra-cql-store", "secure-connection-bundle-base64"), ("astra-cql-store", "gateway-user"),
    ("astra-cql-store", "gateway-password"), ("scylla-cql-store", "hosts"), ("scylla-cql-store", "port"),
    ("scylla-cql-store", "user"), ("scylla-cql-store", "password"), ("scylla-cql-store", "local-dc"),
    ("cql-store-type",), ("kube-config-path",), ("resource-namespace",), ("log-level",), ("workers",),
    ("failure-rate-base-delay",), ("failure-rate-max-delay",), ("rate-limit-elements-per-second",),
    ("rate-limit-elements-burst",),
]


def test_every_reference_key_exists():
    keys = {k for k, *_ in iter_keys()}
    for k in REFERENCE_KEYS:
        assert k in keys, k


def test_env_names_match_helm():
    # /root/reference/.helm/templates/deployment.yaml:49-66
    assert env_name(("resource-namespace",)) == "NEXUS__RESOURCE_NAMESPACE"
    assert env_name(("cql-store-type",)) == "NEXUS__CQL_STORE_TYPE"
    assert env_name(("rate-limit-elements-per-second",)) == "NEXUS__RATE_LIMIT_ELEMENTS_PER_SECOND"
    assert env_name(("scylla-cql-store", "hosts")) == "NEXUS__SCYLLA_CQL_STORE__HOSTS"


def test_defaults_equal_helm_defaults():
    c = load_config(path=None, env={})
    assert c.resource_namespace == "nexus"
    assert c.cql_store_type == "astra"
    assert c.log_level == "INFO"
    assert c.failure_rate_base_delay == pytest.approx(0.1)
    assert c.failure_rate_max_delay == pytest.approx(1.0)
    assert c.rate_limit_elements_per_second == 10
    assert c.rate_limit_elements_burst == 100
    assert c.workers == 2
    assert c.resync_period == 30.0


def test_reference_appconfig_with_empty_strings(tmp_path):
    # the reference ships every key as "" (appconfig.local.yaml) → defaults, not zeros
    p = tmp_path / "appconfig.yaml"
    p.write_text(
        "astra-cql-store:\n  secure-connection-bundle-base64: \"\"\n  gateway-user: \"\"\n  gateway-password: \"\"\n"
        "scylla-cql-store:\n  hosts: []\n  port: \"\"\n  user: \"\"\n  password: \"\"\n  local-dc: \"\"\n"
        "cql-store-type: scylla\nkube-config-path: \"\"\nresource-namespace: \"\"\nlog-level: \"\"\nworkers: \"\"\n"
        "failure-rate-base-delay: \"\"\nfailure-rate-max-delay: \"\"\nrate-limit-elements-per-second: \"\"\n"
        "rate-limit-elements-burst: \"\"\n")
    c = load_config(str(p), env={})
    assert c.cql_store_type == "scylla"
    assert c.workers == 2 and c.scylla_cql_store.port == 9042 and c.scylla_cql_store.hosts == []


def test_env_overrides_and_env_overlay(tmp_path):
    (tmp_path / "appconfig.yaml").write_text("workers: 3\ncql-store-type: scylla\n")
    (tmp_path / "appconfig.units.yaml").write_text("workers: 5\nscylla-cql-store:\n  hosts: [a, b]\n")
    env = {"APPLICATION_ENVIRONMENT": "units", "NEXUS__FAILURE_RATE_BASE_DELAY": "5ms",
           "NEXUS__SCYLLA_CQL_STORE__PORT": "19042", "NEXUS__RATE_LIMIT_ELEMENTS_PER_SECOND": "0",
           "NEXUS__COMPAT__FULL_ROW_UPSERT": "true"}
    c = load_config(str(tmp_path / "appconfig.yaml"), env=env)
    assert c.workers == 5
    assert c.scylla_cql_store.hosts == ["a", "b"]
    assert c.scylla_cql_store.port == 19042
    assert c.failure_rate_base_delay == pytest.approx(0.005)
    assert c.rate_limit_elements_per_second == 0
    assert c.compat.full_row_upsert is True
    env2 = dict(env, NEXUS__SCYLLA_CQL_STORE__HOSTS="h1, h2,h3")
    assert load_config(str(tmp_path / "appconfig.yaml"), env=env2).scylla_cql_store.hosts == ["h1", "h2", "h3"]


def test_validation():
    with pytest.raises(ConfigError):
        load_config(env={}, overrides={"cql-store-type": "mongo"})
    with pytest.raises(ConfigError):
        load_config(env={"NEXUS__WORKERS": "0"})
    with pytest.raises(ConfigError):
        load_config(env={}, overrides={"failure-rate-base-delay": "2s", "failure-rate-max-delay": "1s"})
    with pytest.raises(ConfigError):
        load_config(env={"NEXUS__WORKERS": "two"})
    with pytest.raises(ConfigError):  # unknown keys: warned by default, fatal in strict mode
        load_config(env={"NEXUS_CONFIG_STRICT": "1"}, overrides={"no-such-key": 1})
    assert load_config(env={}, overrides={"no-such-key": 1}).workers == 2


def test_redacted_masks_secrets():
    c = load_config(env={"NEXUS__SCYLLA_CQL_STORE__PASSWORD": "hunter2"})
    r = redacted(c)
    assert r["scylla-cql-store"]["password"] == "***"


@pytest.mark.parametrize("s,sec", [("100ms", 0.1), ("1s", 1), ("1m30s", 90), ("1h", 3600), ("15m", 900),
                                   ("1.5s", 1.5), ("-2s", -2), ("0", 0), ("250us", 250e-6), ("3ns", 3e-9),
                                   ("2h45m", 9900)])
def test_parse_duration(s, sec):
    assert parse_duration(s) == pytest.approx(sec)


@pytest.mark.parametrize("bad", ["", "10", "1x", "s", "1s2", "abc"])
def test_parse_duration_rejects(bad):
    with pytest.raises(ValueError):
        parse_duration(bad)


def test_format_duration_roundtrip():
    for s in ["100ms", "1s", "1m30s", "1h0m0s", "2.5s", "250µs"]:
        assert parse_duration(format_duration(parse_duration(s))) == pytest.approx(parse_duration(s))
    assert format_duration(90) == "1m30s"
    assert format_duration(0.1) == "100ms"


def test_worker_processes_auto_from_cpu_share(tmp_path, monkeypatch):
    from nexus_supervisor_amd.utils import cpus

    quota = tmp_path / "cpu.max"
    quota.write_text("350000 100000\n")  # a 3.5-CPU Kubernetes limit
    monkeypatch.setattr(os, "sched_getaffinity", lambda _pid: set(range(64)))
    assert cpus.cpu_share(str(quota)) == pytest.approx(3.5)
    quota.write_text("max 100000\n")
    assert cpus.cpu_share(str(quota)) == 64
    assert cpus.cpu_share(str(tmp_path / "missing")) == 64
    assert cpus.auto_worker_processes(share=3.5) == 2 and cpus.auto_worker_processes(share=1.0) == 1
    monkeypatch.setattr(cpus, "CPU_MAX", str(tmp_path / "missing"))
    monkeypatch.setattr(cpus.cpu_share, "__defaults__", (str(tmp_path / "missing"),))
    c = load_config(env={"NEXUS__RUNTIME__WORKER_PROCESSES": "0"})
    assert c.runtime.worker_processes == 6  # 64 CPUs: capped at the efficient point (utils/cpus.py)
    with pytest.raises(ConfigError):
        load_config(env={"NEXUS__RUNTIME__WORKER_PROCESSES": "-1"})
