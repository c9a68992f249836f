"""Parity fixture: the reference's seed rows and its 8 test scenarios.

Seed rows carry the same keys and stages as the reference fixture
(``/root/reference/test-resources/checkpoints.cql:31-101``); scenarios build the
same K8s objects as ``/root/reference/services/supervisor_test.go:46-540`` and
expect the same end stages.  Objects are generated
programmatically from compact tables instead of being transcribed.
"""
from __future__ import annotations

import datetime as _dt
from dataclasses import dataclass
from typing import Any, Dict, List, Optional

from ..config.schema import LabelConfig
from ..models.checkpoint import CheckpointedRequest, LifecycleStage

ALGORITHM = "test-algorithm"
NAMESPACE = "nexus"


def _ts(s: str) -> _dt.datetime:
    return _dt.datetime.fromisoformat(s.replace("Z", "+00:00"))


# (id, stage, content_hash, received_at, api_version, payload_valid_for) per seed row
_SEED = [
    ("f47ac10b-58cc-4372-a567-0e02b2c3d479", "BUFFERED", "new_hash", "2023-10-01T12:00:00.000Z", "v1.0", "1h"),
    ("2c7b6e8d-cc3c-4b5b-a3f6-5d7b9e2c7f2a", "RUNNING", "buffered_hash", "2023-10-02T10:00:00.000Z", "v2.0", "15m"),
    ("3c7b6e8d-cc3c-4b5b-a3f6-5d7b9e2c7f2b", "RUNNING", "buffered_hash", "2023-10-02T10:00:00.000Z", "v2.0", "15m"),
    ("4c7b6e8d-cc3c-fb5b-a3f6-5d7b9e2c7f2b", "BUFFERED", "buffered_hash", "2023-10-02T10:00:00.000Z", "v2.0", "15m"),
    ("1d7b6e8d-cc3c-fb5b-a3f6-5d7b9e2c7f2b", "RUNNING", "buffered_hash", "2023-10-02T10:00:00.000Z", "v2.0", "15m"),
    ("9e7b6e8d-cc3c-fb5b-a3f6-5d7b9e2c7f2b", "BUFFERED", "buffered_hash", "2023-10-02T10:00:00.000Z", "v2.0", "15m"),
    ("6a4b6e8d-cc3c-fb5b-a3f6-5d7b9e2c7f2b", "BUFFERED", "buffered_hash", "2023-10-02T10:00:00.000Z", "v2.0", "15m"),
    ("df1b6e8d-cc3c-fb5b-a3f6-5d7b9e2c7f2b", "CANCELLED", "buffered_hash", "2023-10-02T10:00:00.000Z", "v2.0", "15m"),
]


def seed_rows() -> List[CheckpointedRequest]:
    rows = []
    for rid, stage, chash, received, api, valid_for in _SEED:
        r0 = _ts(received)
        rows.append(CheckpointedRequest(
            algorithm=ALGORITHM, id=rid, lifecycle_stage=stage, payload_uri="http://localhost/payload",
            result_uri=None, algorithm_failure_cause=None, algorithm_failure_details=None,
            received_by_host="host123", received_at=r0, sent_at=r0 + _dt.timedelta(minutes=30),
            applied_configuration="{}", configuration_overrides="{}", content_hash=chash,
            last_modified=r0 + _dt.timedelta(minutes=45), tag="tag_123", api_version=api,
            job_uid="d94c16c8-2c1e-4f3a-85d1-2d9c3b7f0a24" if rid.startswith("f47") else "1f7b6e8d-cc3c-4b5b-a3f6-5d7b9e2c7f2a",
            parent="{}", payload_valid_for=valid_for,
        ))
    return rows


def run_labels(labels: LabelConfig, algorithm: str = ALGORITHM, job_name: Optional[str] = None) -> Dict[str, str]:
    out = {labels.nexus_component_label: labels.algorithm_run_value, labels.job_template_name_key: algorithm}
    if job_name is not None:
        out[labels.job_name_label] = job_name
    return out


def make_job(name: str, labels: LabelConfig, ns: str = NAMESPACE, algorithm: str = ALGORITHM, rv: str = "1", **status) -> Dict[str, Any]:
    job = {"apiVersion": "batch/v1", "kind": "Job",
           "metadata": {"name": name, "namespace": ns, "uid": f"job-uid-{name}", "resourceVersion": rv,
                        "labels": run_labels(labels, algorithm)},
           "spec": {}, "status": dict(status)}
    return job


def make_pod(request_id: str, labels: LabelConfig, ns: str = NAMESPACE, algorithm: str = ALGORITHM, suffix: str = "acdey",
             env: Optional[Dict[str, str]] = None, gpus: int = 0, node: str = "", status: Optional[Dict[str, Any]] = None,
             rv: str = "1", annotations: Optional[Dict[str, str]] = None) -> Dict[str, Any]:
    container: Dict[str, Any] = {"name": "algorithm", "image": "algo:latest"}
    if env:
        container["env"] = [{"name": k, "value": v} for k, v in env.items()]
    if gpus:
        container["resources"] = {"limits": {"amd.com/gpu": str(gpus)}, "requests": {"amd.com/gpu": str(gpus)}}
    meta: Dict[str, Any] = {"name": f"{request_id}-{suffix}", "namespace": ns, "uid": f"pod-uid-{request_id}-{suffix}",
                            "resourceVersion": rv, "labels": run_labels(labels, algorithm, request_id)}
    if annotations:
        meta["annotations"] = dict(annotations)
    spec: Dict[str, Any] = {"containers": [container]}
    if node:
        spec["nodeName"] = node
    return {"apiVersion": "v1", "kind": "Pod", "metadata": meta, "spec": spec, "status": status or {}}


_EV_SEQ = [0]


def make_event(kind: str, involved_name: str, reason: str, message: str = "", ns: str = NAMESPACE,
               name: Optional[str] = None, event_time: Optional[str] = None, uid: str = "", count: int = 1) -> Dict[str, Any]:
    _EV_SEQ[0] += 1
    ev: Dict[str, Any] = {
        "apiVersion": "v1", "kind": "Event",
        "metadata": {"name": name or f"ev-{_EV_SEQ[0]}", "namespace": ns, "uid": f"ev-uid-{_EV_SEQ[0]}",
                     "resourceVersion": str(_EV_SEQ[0])},
        "involvedObject": {"kind": kind, "name": involved_name, "namespace": ns, "uid": uid},
        "reason": reason, "message": message, "type": "Normal" if reason == "Started" else "Warning", "count": count,
    }
    if event_time:
        ev["eventTime"] = event_time
    return ev


@dataclass
class Scenario:
    name: str
    request_ids: List[str]
    objects: List[Dict[str, Any]]
    expected: Dict[str, str]  # request id -> stage


def reference_scenarios(labels: Optional[LabelConfig] = None) -> List[Scenario]:
    """The 8 reference scenarios (``supervisor_test.go:542-550``)."""
    labels = labels or LabelConfig()
    ids = [r[0] for r in _SEED]
    fc, dl, bo, st, oom, pf, pb, cn = ids
    S = LifecycleStage
    return [
        Scenario("failed-create", [fc], [make_event("Job", fc, "FailedCreate", name="test-failed-create-event"),
                                         make_job(fc, labels)], {fc: S.SCHEDULING_FAILED}),
        Scenario("deadline-and-backoff", [dl, bo],
                 [make_job(dl, labels), make_job(bo, labels),
                  make_event("Job", dl, "DeadlineExceeded", name="test-deadlineexceeded"),
                  make_event("Job", bo, "BackoffLimitExceeded", name="test-backoffexceeded")],
                 {dl: S.DEADLINE_EXCEEDED, bo: S.DEADLINE_EXCEEDED}),
        Scenario("pod-started", [st], [make_event("Pod", f"{st}-acdey", "Started", name="test-pod-started"),
                                       make_pod(st, labels)], {st: S.RUNNING}),
        Scenario("pod-failure-policy-oom", [oom], [make_event("Job", oom, "PodFailurePolicy", name="test-pod-out-of-memory"),
                                                   make_job(oom, labels)], {oom: S.FAILED}),
        Scenario("pod-failed", [pf], [make_event("Pod", f"{pf}-acdey", "Failed", name="test-pod-failed"),
                                      make_job(pf, labels), make_pod(pf, labels)], {pf: S.SCHEDULING_FAILED}),
        Scenario("pod-backoff", [pb], [make_event("Pod", f"{pb}-acdey", "BackOff", name="test-pod-backoff"),
                                       make_job(pb, labels), make_pod(pb, labels)], {pb: S.FAILED}),
        Scenario("started-after-cancel", [cn], [make_event("Pod", f"{cn}-acdey", "Started", name="test-pod-started-cancelled"),
                                                make_job(cn, labels), make_pod(cn, labels)], {cn: S.CANCELLED}),
    ]


def seed_cql_statements(keyspace: str = "nexus", table: str = "checkpoints") -> List[str]:
    """CQL to create + seed the table (what ``prepare-scylla.sh`` applies)."""
    from ..models.checkpoint import COLUMN_NAMES, create_index_cql, create_table_cql

    stmts = [f"CREATE KEYSPACE IF NOT EXISTS {keyspace} WITH replication = {{ 'class': 'SimpleStrategy', 'replication_factor': 1 }};",
             create_table_cql(keyspace, table)]
    stmts += list(create_index_cql(keyspace, table))
    for row in seed_rows():
        vals = []
        for v in row.as_row():
            if v is None:
                vals.append("NULL")
            elif isinstance(v, _dt.datetime):
                vals.append("'" + v.strftime("%Y-%m-%dT%H:%M:%S.") + f"{v.microsecond // 1000:03d}Z'")
            else:
                vals.append("'" + str(v).replace("'", "''") + "'")
        stmts.append(f"INSERT INTO {keyspace}.{table} ({', '.join(COLUMN_NAMES)}) VALUES ({', '.join(vals)});")
    return stmts
