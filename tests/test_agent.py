"""Node GPU agent + supervisor evidence flow (BASELINE config 3 analog on the fake
amd-smi backend): per-GPU attribution via pod-resources / env, evidence
annotations, GPU-fault events, and the supervisor waiting for the evidence."""
import asyncio
import json
import time

from nexus_supervisor_amd.app import Application
from nexus_supervisor_amd.config import load_config
from nexus_supervisor_amd.gpu.agent import NodeAgent, pod_failed
from nexus_supervisor_amd.gpu.podresources import decode_list_response, encode_list_response, gpu_allocations
from nexus_supervisor_amd.gpu.telemetry import FakeTelemetry, evidence_for
from nexus_supervisor_amd.kube.client import KubeClient, KubeConfig
from nexus_supervisor_amd.store.memory import MemoryStore
from nexus_supervisor_amd.testing.fake_apiserver import FakeApiServer
from nexus_supervisor_amd.testing.seed import ALGORITHM, make_job, make_pod, seed_rows

ANN = "nexus.amd.com/gpu-evidence"
MB = 1 << 20


def _failed(pod, message="", reason="Error", code=1):
    p = json.loads(json.dumps(pod))
    p["status"] = {"phase": "Failed", "containerStatuses": [{"name": "algorithm", "restartCount": 0, "state": {
        "terminated": {"reason": reason, "exitCode": code, "message": message}}}]}
    return p


def test_pod_resources_protobuf_roundtrip():
    pods = [{"name": "p0", "namespace": "nexus", "containers": [
        {"name": "algorithm", "devices": [{"resource_name": "amd.com/gpu", "device_ids": ["0000:0a:00.0", "0000:1a:00.0"]},
                                          {"resource_name": "rdma/hca", "device_ids": ["mlx5_0"]}]}]},
            {"name": "p1", "namespace": "nexus", "containers": [{"name": "c", "devices": []}]}]
    assert decode_list_response(encode_list_response(pods)) == pods
    assert gpu_allocations(pods) == {("nexus", "p0"): ["0000:0a:00.0", "0000:1a:00.0"]}


def test_evidence_window_excludes_old_peaks():
    clock = [1000.0]
    tel = FakeTelemetry(n_gpus=2, clock=lambda: clock[0])
    tel.set_vram(1, 294_000, t=900.0)        # an old OOM, long before the pod started
    tel.add_process(4242, 1, 10 * MB, env={"RANK": "5", "LOCAL_RANK": "1"}, pod_uid="uid-a")
    clock[0] = 1010.0
    tel.set_vram(1, 20_000, t=1005.0)
    tel.end_process(4242, 1)
    ev = evidence_for(tel, pod_uid="uid-a", now=1011.0)
    g = ev["gpus"][0]
    assert g["index"] == 1 and g["vram_peak_mb"] == 20_000  # not the 294 GB from t=900
    assert g["procs"][0]["rank"] == 5 and g["procs"][0]["local_rank"] == 1
    assert [e["type"] for e in g.get("events", [])] == []  # PROCESS_END is not an attribution event


def test_agent_annotates_failed_pod_with_allocated_gpu(arun):
    async def go():
        api = FakeApiServer(bookmark_interval=0.1)
        url = await api.start()
        labels = load_config(path=None, env={}, overrides={}).labels
        tel = FakeTelemetry(n_gpus=8)
        pod = make_pod("run-7", labels, gpus=1, node="node-a", env={"RANK": "7"}, status={"phase": "Running"})
        other = make_pod("run-8", labels, gpus=1, node="node-b", status={"phase": "Running"})
        api.create(pod)
        api.create(other)

        class FakePodRes:
            def list(self):
                return [{"name": "run-7-acdey", "namespace": "nexus", "containers": [
                    {"name": "algorithm", "devices": [{"resource_name": "amd.com/gpu", "device_ids": ["0000:0f:00.0"]}]}]}]

            def close(self):
                pass

        kc = KubeClient(KubeConfig(url))
        agent = NodeAgent(kc, tel, "node-a", "nexus", pod_resources=FakePodRes())
        await agent.start()
        await agent.factory.wait_for_cache_sync(5)
        assert [p["metadata"]["name"] for p in agent.pods.indexer.values()] == ["run-7-acdey"]  # node-scoped watch
        # GPU 5 (bdf 0000:0f:00.0) fills up, then the pod dies with a HIP OOM
        tel.set_vram(5, 294_500)
        api.update(_failed(api.get("Pod", "nexus", "run-7-acdey"), "hipErrorOutOfMemory"))
        for _ in range(100):
            ann = (api.get("Pod", "nexus", "run-7-acdey")["metadata"].get("annotations") or {}).get(ANN)
            if ann:
                break
            await asyncio.sleep(0.02)
        ev = json.loads(ann)
        assert [g["index"] for g in ev["gpus"]] == [5] and ev["gpus"][0]["vram_peak_mb"] == 294_500
        assert ev["node"] == "node-a" and ev["reason"] == "pod-failed"
        await agent.stop()
        await kc.close()
        await api.stop()

    arun(go())


def test_agent_gpu_fault_event_annotates_running_pod(arun):
    async def go():
        api = FakeApiServer(bookmark_interval=0.1)
        url = await api.start()
        labels = load_config(path=None, env={}, overrides={}).labels
        tel = FakeTelemetry(n_gpus=8)
        pod = make_pod("run-3", labels, gpus=1, node="n", env={"LOCAL_RANK": "3", "HIP_VISIBLE_DEVICES": "0,1,2,3"},
                       status={"phase": "Running"})
        api.create(pod)
        kc = KubeClient(KubeConfig(url))
        agent = NodeAgent(kc, tel, "n", "nexus", event_poll=0.02)
        await agent.start()
        await agent.factory.wait_for_cache_sync(5)
        assert agent.gpus_for(pod) == [3]
        tel.inject_event(3, "VMFAULT", "page fault at 0xdead")
        for _ in range(100):
            ann = (api.get("Pod", "nexus", "run-3-acdey")["metadata"].get("annotations") or {}).get(ANN)
            if ann:
                break
            await asyncio.sleep(0.02)
        ev = json.loads(ann)
        assert ev["reason"] == "gpu-fault:VMFAULT" and ev["gpus"][0]["events"][0]["type"] == "VMFAULT"
        await agent.stop()
        await kc.close()
        await api.stop()

    arun(go())


def test_supervisor_waits_for_agent_evidence_then_attributes(arun):
    """Cluster supervisor + node agent over one apiserver: the supervisor holds the failed
    GPU pod (gpu.evidence-wait) until the agent's annotation lands, then writes an
    HBM-OOM verdict with the *physical* GPU index into the trace column (the rank's torch
    ordinal 2 behind HIP_VISIBLE_DEVICES=4,5,6,7 is physical GPU 6)."""
    async def go():
        api = FakeApiServer(bookmark_interval=0.1)
        url = await api.start()
        row = seed_rows()[1]  # RUNNING
        cfg = load_config(path=None, env={}, overrides={"cql-store-type": "memory", "rate-limit-elements-per-second": 0,
                                                        "resync-period": "0s", "gpu": {"evidence-wait": "3s"}})
        pod = make_pod(row.id, cfg.labels, gpus=1, node="n", env={"LOCAL_RANK": "2", "HIP_VISIBLE_DEVICES": "4,5,6,7",
                                                                   "RANK": "10", "WORLD_SIZE": "16"},
                       status={"phase": "Running"})
        api.create(pod)
        api.create(make_job(row.id, cfg.labels))
        store = MemoryStore([row])
        app = Application(cfg, kube=KubeClient(KubeConfig(url)), store=store)
        await app.start()
        tel = FakeTelemetry(n_gpus=8)
        kc = KubeClient(KubeConfig(url))
        agent = NodeAgent(kc, tel, "n", "nexus")
        await agent.start()
        await asyncio.gather(app.factory.wait_for_cache_sync(5), agent.factory.wait_for_cache_sync(5))
        tel.set_vram(6, 290_000)
        tel.set_vram(2, 290_000)  # a busy GPU the pod never used must not be blamed
        t0 = time.monotonic()
        msg = ("torch.OutOfMemoryError: HIP out of memory. Tried to allocate 4.00 GiB. GPU 2 has a total capacity of "
               "287.98 GiB of which 1.02 GiB is free.")
        api.update(_failed(api.get("Pod", "nexus", f"{row.id}-acdey"), msg, code=1))
        for _ in range(200):
            if store.get(ALGORITHM, row.id).lifecycle_stage == "FAILED":
                break
            await asyncio.sleep(0.02)
        took = time.monotonic() - t0
        out = store.get(ALGORITHM, row.id)
        assert out.lifecycle_stage == "FAILED" and took < 3.0, took
        trace = json.loads(out.algorithm_failure_details)
        assert trace["class"] == "hbm-oom" and trace["oom"]["gpu_index"] == 6 and trace["oom"]["gpu_logical_index"] == 2
        assert trace["topology"]["rank"] == 10 and trace["topology"]["expected_gpu"] == "6"
        assert [g["index"] for g in trace["gpu"]["gpus"]] == [6]
        assert any("VRAM peak" in sig for sig in trace["oom"]["signals"])
        xg = trace["topology"]["xgmi"]
        assert xg["source"] == "fake" and xg["per_gpu"][0]["links_listed"] == 7 and xg["fully_connected"] is None
        assert sorted(xg["per_gpu"][0]["peers"]) == [0, 1, 2, 3, 4, 5, 7]
        assert app.metrics.counter("decisions_deferred_for_gpu_evidence") == 1
        await agent.stop()
        await kc.close()
        await app.stop()
        await api.stop()

    arun(go(), timeout=30)


def test_evidence_wait_expires_without_agent(arun):
    async def go():
        api = FakeApiServer(bookmark_interval=0.1)
        url = await api.start()
        row = seed_rows()[1]
        cfg = load_config(path=None, env={}, overrides={"cql-store-type": "memory", "rate-limit-elements-per-second": 0,
                                                        "resync-period": "0s", "gpu": {"evidence-wait": "300ms"}})
        pod = make_pod(row.id, cfg.labels, gpus=1, status={"phase": "Running"})
        api.create(pod)
        store = MemoryStore([row])
        app = Application(cfg, kube=KubeClient(KubeConfig(url)), store=store)
        await app.start()
        await app.factory.wait_for_cache_sync(5)
        api.update(_failed(api.get("Pod", "nexus", f"{row.id}-acdey"), reason="OOMKilled", code=137))
        for _ in range(100):
            if store.get(ALGORITHM, row.id).lifecycle_stage == "FAILED":
                break
            await asyncio.sleep(0.02)
        out = store.get(ALGORITHM, row.id)
        assert out.lifecycle_stage == "FAILED"
        assert json.loads(out.algorithm_failure_details)["class"] == "host-oom"
        assert app.metrics.counter("gpu_evidence_wait_expired") == 1
        await app.stop()
        await api.stop()

    arun(go(), timeout=30)


def test_pod_failed_predicate():
    assert pod_failed({"status": {"phase": "Failed"}})
    assert pod_failed({"status": {"reason": "Evicted"}})
    assert not pod_failed({"status": {"phase": "Running", "containerStatuses": [{"state": {"running": {}}}]}})


class _FakePodResources:
    def __init__(self, pods):
        self.pods = pods

    def list(self):
        return self.pods

    def close(self):
        return None


def test_agent_maps_device_plugin_allocation_to_physical_gpus():
    """Device-plugin allocation (kubelet pod-resources, by BDF) is the container's HIP
    ordinal space: a pod allocated physical GPUs 4-7 whose rank 3 OOMs on torch 'GPU 3'
    is attributed to physical GPU 7, and the evidence records the allocation."""
    from nexus_supervisor_amd.classify import Classifier
    from nexus_supervisor_amd.config.schema import LabelConfig
    from nexus_supervisor_amd.gpu.podresources import gpu_allocations

    labels = LabelConfig()
    tel = FakeTelemetry(n_gpus=8)
    bdfs = [d["bdf"] for d in tel.devices()]
    pod = make_pod("alloc-run", labels, gpus=4, node="n", env={"LOCAL_RANK": "3", "RANK": "3", "WORLD_SIZE": "4"}, rv="2",
                   status={"phase": "Failed", "containerStatuses": [{"name": "algorithm", "restartCount": 0, "state": {
                       "terminated": {"reason": "Error", "exitCode": 1, "message":
                                      "HIP out of memory. GPU 3 has a total capacity of 287.98 GiB"}}}]})
    podres = _FakePodResources([{"name": pod["metadata"]["name"], "namespace": pod["metadata"]["namespace"], "containers": [
        {"name": "algorithm", "devices": [{"resource_name": "amd.com/gpu", "device_ids": [bdfs[i] for i in (6, 4, 7, 5)]}]}]}])
    assert gpu_allocations(podres.list())
    agent = NodeAgent(None, tel, "n", "nexus", pod_resources=podres, factory=_NullFactory())
    agent._bdf_index = {d["bdf"]: d["index"] for d in tel.devices()}
    tel.set_vram(7, 294_000)
    ev = agent.evidence(pod)
    assert ev["allocated"] == [4, 5, 6, 7] and [g["index"] for g in ev["gpus"]] == [4, 5, 6, 7]
    pod["metadata"]["annotations"] = {ANN: json.dumps(ev)}
    r = Classifier(labels).classify_pod(pod)[0]
    assert r.evidence["oom"]["gpu_index"] == 7 and r.evidence["oom"]["gpu_logical_index"] == 3
    assert r.evidence["topology"]["expected_gpu"] == "7" and r.evidence["topology"]["physical_devices"] == [4, 5, 6, 7]
    assert r.evidence["oom"]["peak_vram_bytes"] == 294_000 << 20


class _NullFactory:
    def informer(self, kind):
        class _I:
            indexer = {}

            def add_event_handler(self, **kw):
                return None
        return _I()
