"""Kubelet admission rejections (UnexpectedAdmissionError / OutOfamd.com/gpu /
TopologyAffinityError / other admit handlers).

The reference drops them: a pod refused by its node's kubelet has ``phase: Failed``, a
``status.reason`` and no container statuses, and its Event reason is in no rule
(``/root/reference/services/supervisor.go:254-256``); the Job then retries into
BackoffLimitExceeded and is written DEADLINE_EXCEEDED (``:183-193``).  Here the run is
written SCHEDULING_FAILED with class ``gpu-admission`` (or ``admission``), the node,
the requested GPUs and the node agent's GPU-health record in the trace."""
import json

import pytest

from nexus_supervisor_amd.classify.classifier import EVENT_REASONS_READ, Classifier, event_reasons_read
from nexus_supervisor_amd.config import load_config
from nexus_supervisor_amd.gpu.agent import NodeAgent
from nexus_supervisor_amd.gpu.podresources import (allocatable_ids, decode_allocatable_response,
                                                   encode_allocatable_response)
from nexus_supervisor_amd.gpu.telemetry import FakeTelemetry, node_gpu_health, pod_evidence_provider
from nexus_supervisor_amd.models import LifecycleStage as S
from nexus_supervisor_amd.models import kube
from nexus_supervisor_amd.store.memory import MemoryStore
from nexus_supervisor_amd.testing.inproc import InProcCluster
from nexus_supervisor_amd.testing.seed import ALGORITHM, make_event, make_job, make_pod, seed_rows

BUFFERED_ROW = seed_rows()[0]
BID = BUFFERED_ROW.id
ALLOC_MSG = ("Allocate failed due to requested number of devices unavailable for amd.com/gpu. Requested: 1, "
             "Available: 0, which is unexpected")
OUTOF_MSG = "Pod was rejected: Node didn't have enough resource: amd.com/gpu, requested: 8, used: 8, capacity: 8"


def _cfg(**over):
    base = {"cql-store-type": "memory", "workers": 4, "rate-limit-elements-per-second": 0, "resync-period": "0s"}
    base.update(over)
    return load_config(path=None, env={}, overrides=base)


def _rejected(cfg, reason, message, gpus=1, rv="5", annotations=None):
    return make_pod(BID, cfg.labels, gpus=gpus, node="mi355x-007", rv=rv, annotations=annotations,
                    status={"phase": "Failed", "reason": reason, "message": message})


async def _run(cfg, objects, updates, rows=(BUFFERED_ROW,)):
    store = MemoryStore(rows)
    c = InProcCluster(cfg, store, objects)
    await c.start()
    for etype, obj in updates:
        c.push(obj, etype)
        assert await c.settle(5)
    await c.stop()
    return store, c


def _trace(row):
    return json.loads(row.algorithm_failure_details)


def test_admission_rejection_helper():
    cfg = _cfg()
    assert kube.admission_rejection(_rejected(cfg, "UnexpectedAdmissionError", ALLOC_MSG)) == {
        "reason": "UnexpectedAdmissionError", "message": ALLOC_MSG}
    assert kube.admission_rejection(_rejected(cfg, "OutOfamd.com/gpu", OUTOF_MSG))["reason"] == "OutOfamd.com/gpu"
    assert kube.admission_rejection(_rejected(cfg, "NodeAffinity", "Predicate NodeAffinity failed")) is not None
    # not admission: an eviction, a pod whose containers ran, a Pending pod
    assert kube.admission_rejection(_rejected(cfg, "Evicted", "low memory")) is None
    ran = _rejected(cfg, "UnexpectedAdmissionError", ALLOC_MSG)
    ran["status"]["containerStatuses"] = [{"name": "algorithm", "state": {"terminated": {"exitCode": 1}}}]
    assert kube.admission_rejection(ran) is None
    assert kube.admission_rejection(make_pod(BID, cfg.labels, status={"phase": "Pending"})) is None


@pytest.mark.parametrize("reason,message,klass,extra", [
    ("UnexpectedAdmissionError", ALLOC_MSG, "gpu-admission", {"requested": 1, "available": 0}),
    ("OutOfamd.com/gpu", OUTOF_MSG, "gpu-admission", {"requested": 8, "used": 8, "capacity": 8}),
    ("TopologyAffinityError", "Resources cannot be allocated with Topology locality", "gpu-admission", {"requested": 1}),
    ("OutOfcpu", "Pod was rejected: Node didn't have enough resource: cpu, requested: 64000, used: 190000, "
                 "capacity: 192000", "admission", {"capacity": 192000}),
])
def test_pod_rejected_at_admission_is_scheduling_failed(arun, reason, message, klass, extra):
    cfg = _cfg()
    store, c = arun(_run(cfg, [make_pod(BID, cfg.labels, gpus=1), make_job(BID, cfg.labels)],
                         [("MODIFIED", _rejected(cfg, reason, message))]))
    row = store.get(ALGORITHM, BID)
    assert row.lifecycle_stage == S.SCHEDULING_FAILED
    t = _trace(row)
    assert t["class"] == klass and t["reason"] == reason and t["message"] == message
    adm = t["admission"]
    assert adm["node"] == "mi355x-007" and adm["gpu"] is (klass == "gpu-admission")
    for k, v in extra.items():
        assert adm[k] == v, (k, adm)
    if klass == "gpu-admission":
        assert row.algorithm_failure_cause == (
            "Algorithm submission was buffered, but failed to launch on the target cluster: "
            "Algorithm pod was rejected by its node: no healthy AMD Instinct GPU could be allocated to it.")
        assert adm["resource"] == "amd.com/gpu"
    assert "oom" not in t  # an admission message is never scored as an OOM
    assert c.jobs.deleted == [BID]


def test_admission_event_decides_and_is_read_by_the_hub_filter(arun):
    cfg = _cfg(**{"rules": {"pod-status-rules": False}})  # the Event alone (reference-style path)
    pod = make_pod(BID, cfg.labels, gpus=1, node="mi355x-007")
    ev = make_event("Pod", pod["metadata"]["name"], "UnexpectedAdmissionError", ALLOC_MSG)
    store, _ = arun(_run(cfg, [pod, make_job(BID, cfg.labels)], [("ADDED", ev)]))
    row = store.get(ALGORITHM, BID)
    assert row.lifecycle_stage == S.SCHEDULING_FAILED and _trace(row)["class"] == "gpu-admission"
    assert {"UnexpectedAdmissionError", "TopologyAffinityError", "OutOfamd.com/gpu", "OutOfcpu"} <= EVENT_REASONS_READ
    assert "OutOfexample.com/gpu" in event_reasons_read("example.com/gpu")


def test_observe_policy_then_backoff_limit_carries_the_admission_cause(arun):
    """admission-policy: observe — the rejection decides nothing; the Job's
    BackoffLimitExceeded is written SCHEDULING_FAILED with the admission cause (not the
    reference's DEADLINE_EXCEEDED retry-count text), under oom-fails-backoff-job."""
    cfg = _cfg(**{"rules": {"admission-policy": "observe"}})
    rej = _rejected(cfg, "UnexpectedAdmissionError", ALLOC_MSG)
    job_failed = make_job(BID, cfg.labels, rv="7", conditions=[
        {"type": "Failed", "status": "True", "reason": "BackoffLimitExceeded", "message": "limit"}])
    store, _ = arun(_run(cfg, [make_pod(BID, cfg.labels, gpus=1), make_job(BID, cfg.labels)], [("MODIFIED", rej)]))
    assert store.get(ALGORITHM, BID).lifecycle_stage == S.BUFFERED  # the rejection alone decides nothing
    store2, _ = arun(_run(cfg, [make_pod(BID, cfg.labels, gpus=1), make_job(BID, cfg.labels)],
                          [("MODIFIED", rej), ("MODIFIED", job_failed)]))
    row = store2.get(ALGORITHM, BID)
    assert row.lifecycle_stage == S.SCHEDULING_FAILED
    assert row.algorithm_failure_cause.endswith("no healthy AMD Instinct GPU could be allocated to it.")
    t = _trace(row)
    assert t["class"] == "gpu-admission" and t["admission"]["available"] == 0
    assert t["history"][0]["kind"] == "admission"
    # the compat switch off keeps the reference's stage, the cause goes into the trace
    cfg3 = _cfg(**{"rules": {"admission-policy": "observe", "oom-fails-backoff-job": False}})
    store3, _ = arun(_run(cfg3, [make_pod(BID, cfg3.labels, gpus=1), make_job(BID, cfg3.labels)],
                          [("MODIFIED", rej), ("MODIFIED", job_failed)]))
    row3 = store3.get(ALGORITHM, BID)
    assert row3.lifecycle_stage == S.DEADLINE_EXCEEDED and _trace(row3)["class"] == "gpu-admission"


def test_backoff_limit_first_then_rejected_pod_in_cache(arun):
    """The Job's BackoffLimitExceeded arrives while its admission-rejected pod is already in
    the cache (late_enrich reads the pods at actuation)."""
    cfg = _cfg(**{"rules": {"admission-policy": "observe"}})
    rej = _rejected(cfg, "OutOfamd.com/gpu", OUTOF_MSG)
    job_failed = make_job(BID, cfg.labels, rv="7", conditions=[
        {"type": "Failed", "status": "True", "reason": "BackoffLimitExceeded", "message": "limit"}])
    store, _ = arun(_run(cfg, [rej, make_job(BID, cfg.labels)], [("MODIFIED", job_failed)]))
    row = store.get(ALGORITHM, BID)
    assert row.lifecycle_stage == S.SCHEDULING_FAILED and _trace(row)["class"] == "gpu-admission"


def test_node_health_names_the_unhealthy_gpus():
    tel = FakeTelemetry(n_gpus=8)
    tel.set_ecc(3, uncorrectable=4)
    tel.inject_event(5, "GPU_PRE_RESET", "reset")
    tel.set_xgmi(6, total=7, down=2)
    bdfs = [d["bdf"] for d in tel.devices()]
    h = node_gpu_health(tel, allocatable_bdfs=[b for i, b in enumerate(bdfs) if i not in (3, 5)])
    bad = {u["index"]: u["problems"] for u in h["unhealthy"]}
    assert h["gpus_seen"] == 8 and sorted(bad) == [3, 5, 6]
    assert "ecc_uncorrectable=4" in bad[3] and "not in the kubelet's allocatable set" in bad[3]
    assert any(p.startswith("events=GPU_PRE_RESET") for p in bad[5])
    assert "xgmi_links_down=2/7" in bad[6] and "not in the kubelet's allocatable set" not in bad[6]
    assert h["healthy"] == [0, 1, 2, 4, 7] and h["not_allocatable"] == [3, 5] and h["allocatable"] == 6


def test_allocatable_resources_codec():
    devs = [{"resource_name": "amd.com/gpu", "device_ids": ["0000:0a:00.0", "0000:0b:00.0"]},
            {"resource_name": "amd.com/xgmi", "device_ids": ["x"]}]
    back = decode_allocatable_response(encode_allocatable_response(devs))
    assert back == devs and allocatable_ids(back) == ["0000:0a:00.0", "0000:0b:00.0"]


class _PodRes:
    def __init__(self, alloc):
        self.alloc = alloc

    def list(self):
        return []

    def allocatable(self):
        return [{"resource_name": "amd.com/gpu", "device_ids": self.alloc}]

    def close(self):
        pass


def test_agent_publishes_node_health_for_a_rejected_pod_and_trace_carries_it(arun):
    cfg = _cfg()
    tel = FakeTelemetry(n_gpus=8)
    tel.set_ecc(2, uncorrectable=9)
    bdfs = [d["bdf"] for d in tel.devices()]
    agent = NodeAgent(kube_client=None, telemetry=tel, node_name="mi355x-007", namespace="nexus",
                      pod_resources=_PodRes([b for i, b in enumerate(bdfs) if i != 2]), log_root=None,
                      factory=_NoFactory())
    rej = _rejected(cfg, "UnexpectedAdmissionError", ALLOC_MSG)
    ev = agent.evidence(rej)
    assert ev["gpus"] == [] and ev["node"] == "mi355x-007"
    assert ev["node_health"]["not_allocatable"] == [2] and ev["node_health"]["unhealthy"][0]["index"] == 2
    ann = {"nexus.amd.com/gpu-evidence": json.dumps(dict(ev, reason="admission-rejected"))}
    store, c = arun(_run(cfg, [make_pod(BID, cfg.labels, gpus=1), make_job(BID, cfg.labels)],
                         [("MODIFIED", _rejected(cfg, "UnexpectedAdmissionError", ALLOC_MSG, annotations=ann))]))
    t = _trace(store.get(ALGORITHM, BID))
    assert t["class"] == "gpu-admission"
    assert t["gpu"]["node_health"]["unhealthy"][0]["problems"][0] == "ecc_uncorrectable=9"
    # gpu_failures{node,gpu,class}: the node's one unhealthy GPU is the one counted
    got = [dict(k) for k in c.supervisor.metrics.counters["gpu_failures"]]
    assert got == [{"node": "mi355x-007", "gpu": "2", "class": "gpu-admission"}]


def test_evidence_wait_holds_the_rejection_for_the_agent_record(arun):
    """gpu.evidence-wait: a GPU admission rejection without the agent's record is deferred
    (like a failed GPU pod); the record's arrival decides it with the node health."""
    cfg = _cfg(**{"gpu": {"evidence-wait": "3s"}})
    tel = FakeTelemetry(n_gpus=8)
    tel.inject_event(4, "GPU_POST_RESET", "reset done")
    rej = _rejected(cfg, "UnexpectedAdmissionError", ALLOC_MSG)

    async def go():
        store = MemoryStore([BUFFERED_ROW])
        c = InProcCluster(cfg, store, [make_pod(BID, cfg.labels, gpus=1), make_job(BID, cfg.labels)])
        await c.start()
        c.push(rej, "MODIFIED")
        assert await c.settle(0.3) is False or store.get(ALGORITHM, BID).lifecycle_stage == S.BUFFERED
        assert store.get(ALGORITHM, BID).lifecycle_stage == S.BUFFERED
        ev = {"source": "fake", "gpus": [], "node": "mi355x-007", "node_health": node_gpu_health(tel)}
        c.push(_rejected(cfg, "UnexpectedAdmissionError", ALLOC_MSG, rv="6",
                         annotations={"nexus.amd.com/gpu-evidence": json.dumps(ev)}), "MODIFIED")
        assert await c.settle(5)
        await c.stop()
        return store

    row = arun(go()).get(ALGORITHM, BID)
    assert row.lifecycle_stage == S.SCHEDULING_FAILED
    assert _trace(row)["gpu"]["node_health"]["unhealthy"][0]["index"] == 4


def test_local_provider_answers_node_health_for_a_rejected_pod():
    cfg = _cfg()
    tel = FakeTelemetry(n_gpus=8)
    tel.set_xgmi(1, total=7, down=7)
    prov = pod_evidence_provider(tel)
    ev = prov(_rejected(cfg, "OutOfamd.com/gpu", OUTOF_MSG))
    assert ev["node"] == "mi355x-007" and ev["node_health"]["unhealthy"][0]["index"] == 1
    c = Classifier(labels=cfg.labels, rules=cfg.rules, gpu=cfg.gpu)
    c.evidence_provider = prov
    (res,) = c.classify_pod(_rejected(cfg, "OutOfamd.com/gpu", OUTOF_MSG))
    assert res.failure_class == "gpu-admission" and res.evidence["gpu"]["node_health"]["healthy"] == [0, 2, 3, 4, 5, 6, 7]


class _NoFactory:
    def informer(self, kind):
        return None
