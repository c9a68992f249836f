"""HBM-OOM on a *default* pod.

A default pod (``terminationMessagePolicy: File``) that dies of a torch HBM-OOM has an
EMPTY ``terminated.message``: torch prints the OOM to stderr and exits 1.  The reference
only ever sees the Job controller's ``PodFailurePolicy`` event text
(``/root/reference/services/supervisor.go:194-204,311-312``).  Here the OOM text is read
from the container log tail — by the node agent from ``/var/log/pods`` or by the
supervisor over ``pods/<pod>/log`` — and the pod's own processes filling the GPU is a
signature of its own; a previous tenant's VRAM peak alone never is.
"""
import asyncio
import json

from conftest import TIME_SCALE
from nexus_supervisor_amd.app import Application
from nexus_supervisor_amd.classify import Classifier
from nexus_supervisor_amd.config import load_config
from nexus_supervisor_amd.config.schema import GpuConfig, LabelConfig
from nexus_supervisor_amd.gpu import logtail
from nexus_supervisor_amd.gpu.agent import NodeAgent
from nexus_supervisor_amd.gpu.telemetry import FakeTelemetry
from nexus_supervisor_amd.kube.client import KubeClient, KubeConfig
from nexus_supervisor_amd.models.decisions import FailureClass
from nexus_supervisor_amd.store.memory import MemoryStore
from nexus_supervisor_amd.testing.fake_apiserver import FakeApiServer
from nexus_supervisor_amd.testing.fakelogs import write_cri_log
from nexus_supervisor_amd.testing.seed import ALGORITHM, make_job, make_pod, seed_rows

ANN = "nexus.amd.com/gpu-evidence"
TORCH_OOM = ("Traceback (most recent call last):\n  File \"train.py\", line 42, in <module>\n"
             "    x = torch.empty(n, device='cuda')\n"
             "torch.OutOfMemoryError: HIP out of memory. Tried to allocate 20.00 GiB. GPU 0 has a total capacity of "
             "287.98 GiB of which 3.12 GiB is free. Of the allocated memory 270.00 GiB is allocated by PyTorch, and "
             "1.50 GiB is reserved by PyTorch but unallocated.")
PLAIN_CRASH = ("Traceback (most recent call last):\n  File \"train.py\", line 7, in <module>\n"
               "ValueError: expected a positive batch size")


def _failed(pod, message="", reason="Error", code=1, restarts=0, last=False):
    p = json.loads(json.dumps(pod))
    t = {"terminated": {"reason": reason, "exitCode": code, "message": message}}
    cs = {"name": "algorithm", "restartCount": restarts}
    if last:
        cs.update(state={"waiting": {"reason": "CrashLoopBackOff", "message": "back-off 10s"}}, lastState=t)
    else:
        cs["state"] = t
    p["status"] = {"phase": "Running" if last else "Failed", "containerStatuses": [cs]}
    p["metadata"]["resourceVersion"] = str(int(p["metadata"].get("resourceVersion") or 1) + 1)
    return p


# ----------------------------------------------------------------------------- parsing

def test_cri_and_docker_log_lines_and_partials(tmp_path):
    text = "hello\n" + "x" * 50 + "\nlast line"
    path = write_cri_log(str(tmp_path), "nexus", "p", "u", "algorithm", 0, [("stderr", text)], split_at=16)
    lines = logtail.read_tail(path)
    assert lines == ["hello", "x" * 50, "last line"]  # P partials re-joined
    docker = b'{"log":"first\\n","stream":"stderr","time":"t"}\n{"log":"HIP out of memory\\n","stream":"stderr"}\n'
    assert logtail.parse_log_lines(docker) == ["first", "HIP out of memory"]
    assert logtail.parse_log_lines(b"plain text\nmore") == ["plain text", "more"]


def test_read_tail_window_drops_the_cut_line(tmp_path):
    body = "".join(f"line {i:05d} " + "y" * 100 + "\n" for i in range(2000))
    path = write_cri_log(str(tmp_path), "nexus", "p", "u", "algorithm", 0, [("stdout", body)])
    lines = logtail.read_tail(path, max_bytes=4096, max_lines=10)
    assert len(lines) == 10 and lines[-1].startswith("line 01999")
    assert all(ln.startswith("line ") for ln in lines)


def test_scan_keeps_only_signature_lines():
    rec = logtail.scan(TORCH_OOM.splitlines() + ["Exception ignored in atexit"])
    assert rec["match"] == "hbm" and len(rec["lines"]) == 1 and "total capacity" in rec["lines"][0]
    assert logtail.scan(PLAIN_CRASH.splitlines()) == {"match": None, "lines": []}
    host = logtail.scan(["RuntimeError: std::bad_alloc"])
    assert host["match"] == "host"


def test_failed_containers_picks_the_right_instance():
    labels = LabelConfig()
    pod = make_pod("r1", labels, gpus=1)
    assert logtail.failed_containers(_failed(pod)) == [
        {"container": "algorithm", "restart": 0, "previous": False, "exitCode": 1}]
    assert logtail.failed_containers(_failed(pod, restarts=3, last=True))[0]["restart"] == 2
    assert logtail.failed_containers(_failed(pod, restarts=3, last=True))[0]["previous"] is True
    assert logtail.failed_containers(_failed(pod, message="has text")) == []
    assert logtail.failed_containers(_failed(pod, reason="OOMKilled", code=137)) == []
    assert logtail.failed_containers(_failed(pod, code=0, reason="Completed")) == []


# ----------------------------------------------------------------------------- verdicts

def _classify(pod, gev=None, gpu=None, logs=None):
    c = Classifier(LabelConfig(), gpu=gpu or GpuConfig())
    if gev is not None:
        pod["metadata"]["annotations"] = {ANN: json.dumps(gev)}
    if logs is not None:
        c.store_logs(pod, logs)
    return c.classify_pod(pod)


def test_log_tail_makes_a_default_pod_an_hbm_oom():
    labels = LabelConfig()
    pod = _failed(make_pod("r2", labels, gpus=1, env={"LOCAL_RANK": "0", "HIP_VISIBLE_DEVICES": "0"}))
    # no text anywhere: not a pod-level decision (recorded as evidence for the Job's failure)
    assert _classify(json.loads(json.dumps(pod))) == []
    recs = [dict(logtail.scan(TORCH_OOM.splitlines()), container="algorithm", source="pods/log")]
    r = _classify(pod, logs=recs)[0]
    assert r.failure_class == FailureClass.HBM_OOM
    oom = r.evidence["oom"]
    assert oom["gpu_logical_index"] == 0 and oom["requested_bytes"] == 20 << 30
    assert any(s.startswith("HIP OOM signature in pods/log tail of container algorithm") for s in oom["signals"]), oom


def test_vram_numbers_alone_never_make_an_oom():
    """Exit 1 and no OOM text anywhere.  Neither a previous tenant's
    device-wide peak nor the pod's OWN processes holding 99 % of the GPU (PyTorch's caching
    allocator does that in healthy runs) makes an HBM-OOM: the Job decides.  With the
    torch text the own-process peak corroborates and attributes; with exit 137 (SIGKILL,
    an OOM signature) it tips the verdict to HBM; a cgroup OOMKill is never overruled."""
    labels = LabelConfig()
    pod = _failed(make_pod("r3", labels, gpus=1, env={"LOCAL_RANK": "0", "HIP_VISIBLE_DEVICES": "0"}))
    uid = pod["metadata"]["uid"]
    base = {"vram_total_mb": 294896, "vram_peak_mb": 292000, "index": 0, "matched": False}
    other_tenant = {"source": "fake", "gpus": [dict(base, procs=[])], "pod_uid": uid}
    assert _classify(json.loads(json.dumps(pod)), gev=other_tenant) == []  # not an OOM: the Job decides
    own = {"source": "fake", "pod_uid": uid, "gpus": [dict(base, matched=True, proc_peak_vram_bytes=291000 << 20,
                                                          procs=[{"pid": 7, "peak_vram_bytes": 291000 << 20}])]}
    assert _classify(json.loads(json.dumps(pod)), gev=own) == []
    # the log tail names an ordinary error: still not an OOM
    crash = [dict(logtail.scan(PLAIN_CRASH.splitlines()), container="algorithm", restart=0, source="pods/log")]
    assert _classify(json.loads(json.dumps(pod)), gev=own, logs=crash) == []
    # the log tail has the torch OOM: HBM, the own-process peak in the signals
    recs = [dict(logtail.scan(TORCH_OOM.splitlines()), container="algorithm", restart=0, source="pods/log")]
    r = _classify(json.loads(json.dumps(pod)), gev=own, logs=recs)[0]
    assert r.failure_class == FailureClass.HBM_OOM
    assert any(s.startswith("own-process VRAM peak") for s in r.evidence["oom"]["signals"])
    assert r.evidence["oom"]["peak_vram_bytes"] == 291000 << 20
    sigkill = _failed(make_pod("r3", labels, gpus=1), reason="Error", code=137)
    assert _classify(sigkill, gev=own)[0].failure_class == FailureClass.HBM_OOM
    # a cgroup OOMKill is never overruled by VRAM numbers
    killed = _failed(make_pod("r3", labels, gpus=1), reason="OOMKilled", code=137)
    assert _classify(killed, gev=own)[0].failure_class == FailureClass.HOST_OOM


def test_log_fetch_is_asked_for_when_only_vram_numbers_speak():
    """A verdict with no text signature defers for the pods/log read
    (``allow_log_fetch``) instead of deciding from VRAM numbers."""
    labels = LabelConfig()
    pod = _failed(make_pod("r4", labels, gpus=1))
    uid = pod["metadata"]["uid"]
    own = {"source": "fake", "pod_uid": uid, "gpus": [{"vram_total_mb": 294896, "vram_peak_mb": 292000, "index": 0,
                                                        "matched": True, "proc_peak_vram_bytes": 291000 << 20}]}
    pod["metadata"]["annotations"] = {ANN: json.dumps(own)}
    c = Classifier(labels, gpu=GpuConfig())
    assert c.classify_pod(pod, allow_log_fetch=True) == [] and c.deferred
    assert c.deferred_log == [{"container": "algorithm", "restart": 0, "previous": False, "exitCode": 1}]


def test_crashloop_log_cache_is_per_container_instance():
    """Restart 0 of a CrashLoopBackOff pod failed with a
    ValueError (its tail was read and cached); restart 1 then fails with a HIP OOM.  The
    cache is keyed by (pod uid, container, restart), so restart 1's tail is fetched and the
    decision is hbm-oom from it — restart 0's tail never speaks for restart 1."""
    labels = LabelConfig()
    c = Classifier(labels, gpu=GpuConfig())
    base = make_pod("r5", labels, gpus=1, env={"LOCAL_RANK": "0", "HIP_VISIBLE_DEVICES": "0"})
    first = _failed(base, restarts=1, last=True)  # lastState = restart 0
    want = c._log_fetch_needed(first)
    assert [(w["container"], w["restart"]) for w in want] == [("algorithm", 0)]
    c.store_logs(first, [dict(logtail.scan(PLAIN_CRASH.splitlines()), container="algorithm", restart=0,
                              source="pods/log")])
    assert c._log_fetch_needed(first) == []  # read once per instance
    r0 = c.classify_pod(first, allow_log_fetch=True)[0]  # an ordinary crash: crash-loop, no OOM
    assert r0.failure_class == FailureClass.CRASH_LOOP and "oom" not in r0.evidence
    second = _failed(base, restarts=2, last=True)  # lastState = restart 1
    second["metadata"]["resourceVersion"] = "9"
    assert c.classify_pod(second, allow_log_fetch=True) == [] and c.deferred
    assert [(w["container"], w["restart"]) for w in c.deferred_log] == [("algorithm", 1)]
    c.store_logs(second, [dict(logtail.scan(TORCH_OOM.splitlines()), container="algorithm", restart=1,
                               source="pods/log")])
    r = c.classify_pod(second, allow_log_fetch=True)[0]
    assert r.failure_class == FailureClass.HBM_OOM
    assert r.evidence["logs"][0]["restart"] == 1  # only the instance that just failed
    assert len(c.log_cache[base["metadata"]["uid"]]) == 2


# ----------------------------------------------------------------------------- end to end

def _job_failed(job):
    j = json.loads(json.dumps(job))
    j["status"] = {"conditions": [{"type": "Failed", "status": "True", "reason": "BackoffLimitExceeded",
                                   "message": "Job has reached the specified backoff limit"}]}
    j["metadata"]["resourceVersion"] = str(int(j["metadata"].get("resourceVersion") or 1) + 1)
    return j


def _app_cfg(**gpu):
    return load_config(path=None, env={}, overrides={"cql-store-type": "memory", "rate-limit-elements-per-second": 0,
                                                     "resync-period": "0s", "gpu": gpu})


async def _wait_stage(store, rid, stage="FAILED", n=200):
    for _ in range(n):
        if store.get(ALGORITHM, rid).lifecycle_stage == stage:
            return True
        await asyncio.sleep(0.02)
    return False


def test_supervisor_fetches_pods_log_for_a_default_pod(arun):
    """No node agent, empty termination message: the supervisor GETs the failed container's
    log tail (tailLines/limitBytes bounded) once and writes FAILED / hbm-oom, the signal
    naming the pods/log source.  A plain crash next to it stays a fatal error."""
    async def go():
        api = FakeApiServer(bookmark_interval=0.1)
        url = await api.start()
        rows = seed_rows()
        oom_row, crash_row = rows[1], rows[2]  # RUNNING rows
        cfg = _app_cfg()
        pods = {}
        for row in (oom_row, crash_row):
            pods[row.id] = make_pod(row.id, cfg.labels, gpus=1, env={"LOCAL_RANK": "0", "HIP_VISIBLE_DEVICES": "0"},
                                    status={"phase": "Running"})
            api.create(pods[row.id])
            api.create(make_job(row.id, cfg.labels))
        api.set_pod_log("nexus", f"{oom_row.id}-acdey", "algorithm", "step 1\nstep 2\n" + TORCH_OOM + "\n")
        api.set_pod_log("nexus", f"{crash_row.id}-acdey", "algorithm", PLAIN_CRASH + "\n")
        store = MemoryStore([oom_row, crash_row])
        app = Application(cfg, kube=KubeClient(KubeConfig(url)), store=store)
        await app.start()
        await app.factory.wait_for_cache_sync(5)
        for row in (oom_row, crash_row):
            api.update(_failed(api.get("Pod", "nexus", f"{row.id}-acdey")))
        # the Job controller gives up on the crashed run (backoffLimit 0): the Job decides it
        api.update(_job_failed(api.get("Job", "nexus", crash_row.id)))
        assert await _wait_stage(store, oom_row.id)
        assert await _wait_stage(store, crash_row.id, "DEADLINE_EXCEEDED")
        t_oom = json.loads(store.get(ALGORITHM, oom_row.id).algorithm_failure_details)
        assert t_oom["class"] == "hbm-oom" and t_oom["oom"]["kind"] == "hbm"
        assert any("pods/log tail" in s for s in t_oom["oom"]["signals"]), t_oom["oom"]
        assert t_oom["logs"][0]["match"] == "hbm" and "Tried to allocate" in t_oom["logs"][0]["lines"][0]
        crash = store.get(ALGORITHM, crash_row.id)
        assert "hbm" not in (crash.algorithm_failure_details or "")
        assert sorted(q["pod"] for q in api.log_requests) == sorted(f"{r.id}-acdey" for r in (oom_row, crash_row))
        assert all(q["container"] == "algorithm" and q["tailLines"] and q["limitBytes"] for q in api.log_requests)
        assert app.metrics.counter("log_tail_fetches") == 2
        # each run's checkpoint read went out beside its log GET; the decisions took them
        assert app.metrics.counter("checkpoint_reads_prefetched") == 2
        assert app.metrics.counter("checkpoint_reads_prefetch_used") == 2
        await asyncio.sleep(0.2)
        assert len(api.log_requests) == 2  # one fetch per pod
        await app.stop()
        await api.stop()

    arun(go(), timeout=30)


def test_job_failure_waits_for_the_pods_log_read(arun):
    """The Job controller's BackoffLimitExceeded arrives right behind the pod's failure while
    the pods/log read is still on the wire (0.3 s): the Job decision waits for it, so the
    row is FAILED / hbm-oom — the same row the pod decision alone writes — not the
    reference's DEADLINE_EXCEEDED for BackoffLimitExceeded."""
    async def go():
        api = FakeApiServer(bookmark_interval=0.1)
        url = await api.start()
        row = seed_rows()[1]
        cfg = _app_cfg()
        api.create(make_pod(row.id, cfg.labels, gpus=1, status={"phase": "Running"}))
        api.create(make_job(row.id, cfg.labels))
        api.set_pod_log("nexus", f"{row.id}-acdey", "algorithm", TORCH_OOM + "\n")
        api.log_latency = 0.3
        store = MemoryStore([row])
        app = Application(cfg, kube=KubeClient(KubeConfig(url)), store=store)
        await app.start()
        await app.factory.wait_for_cache_sync(5)
        api.update(_failed(api.get("Pod", "nexus", f"{row.id}-acdey")))
        await asyncio.sleep(0.05)
        api.update(_job_failed(api.get("Job", "nexus", row.id)))
        assert await _wait_stage(store, row.id, n=150)
        out = store.get(ALGORITHM, row.id)
        trace = json.loads(out.algorithm_failure_details)
        assert trace["class"] == "hbm-oom", trace
        assert out.algorithm_failure_cause.endswith("Algorithm ran out of GPU memory (HBM) on an AMD Instinct GPU.")
        assert app.metrics.counter("decisions_awaited_log_tail") >= 1
        assert app.metrics.counter("checkpoint_reads_prefetch_used") == 1  # by whichever decision came first
        await app.stop()
        await api.stop()

    arun(go(), timeout=30)


def test_crashloop_previous_instance_and_fetch_errors(arun):
    """CrashLoopBackOff: the log of the *previous* instance (``previous=true``) is read.  A
    failed fetch (apiserver 500) still lets the decision through, without the signature."""
    async def go():
        api = FakeApiServer(bookmark_interval=0.1)
        url = await api.start()
        rows = seed_rows()
        a, b = rows[1], rows[2]
        cfg = _app_cfg()
        for row in (a, b):
            api.create(make_pod(row.id, cfg.labels, gpus=1, status={"phase": "Running"}))
            api.create(make_job(row.id, cfg.labels))
        api.set_pod_log("nexus", f"{a.id}-acdey", "algorithm", TORCH_OOM + "\n", previous=True)
        store = MemoryStore([a, b])
        app = Application(cfg, kube=KubeClient(KubeConfig(url)), store=store)
        await app.start()
        await app.factory.wait_for_cache_sync(5)
        api.update(_failed(api.get("Pod", "nexus", f"{a.id}-acdey"), restarts=2, last=True))
        assert await _wait_stage(store, a.id)
        ta = json.loads(store.get(ALGORITHM, a.id).algorithm_failure_details)
        assert ta["class"] == "hbm-oom", ta
        assert api.log_requests[0]["previous"] == "true"
        api.fail_next[("GET", "PodLog")] = 1
        api.update(_failed(api.get("Pod", "nexus", f"{b.id}-acdey")))
        api.update(_job_failed(api.get("Job", "nexus", b.id)))
        assert await _wait_stage(store, b.id, "DEADLINE_EXCEEDED")
        assert "hbm" not in (store.get(ALGORITHM, b.id).algorithm_failure_details or "")
        assert app.metrics.counter("log_tail_errors") == 1
        await app.stop()
        await api.stop()

    arun(go(), timeout=30)


def test_node_agent_reads_var_log_pods_and_supervisor_attributes(arun, tmp_path):
    """Node agent with a /var/log/pods fixture: the failed container's CRI log carries the
    torch OOM (and the termination message is empty).  The agent's annotation holds the
    matched line; the supervisor (gpu.evidence-wait) writes hbm-oom naming the node-log
    source and never calls pods/log."""
    async def go():
        api = FakeApiServer(bookmark_interval=0.1)
        url = await api.start()
        row = seed_rows()[1]
        cfg = _app_cfg(**{"evidence-wait": "3s"})
        pod = make_pod(row.id, cfg.labels, gpus=1, node="n", env={"LOCAL_RANK": "0", "HIP_VISIBLE_DEVICES": "3"},
                       status={"phase": "Running"})
        api.create(pod)
        api.create(make_job(row.id, cfg.labels))
        write_cri_log(str(tmp_path), "nexus", pod["metadata"]["name"], pod["metadata"]["uid"], "algorithm", 0,
                      [("stdout", "epoch 1 loss 0.3\n"), ("stderr", TORCH_OOM)])
        store = MemoryStore([row])
        app = Application(cfg, kube=KubeClient(KubeConfig(url)), store=store)
        await app.start()
        tel = FakeTelemetry(n_gpus=8)
        kc = KubeClient(KubeConfig(url))
        agent = NodeAgent(kc, tel, "n", "nexus", log_root=str(tmp_path))
        await agent.start()
        await asyncio.gather(app.factory.wait_for_cache_sync(5), agent.factory.wait_for_cache_sync(5))
        api.update(_failed(api.get("Pod", "nexus", pod["metadata"]["name"])))
        assert await _wait_stage(store, row.id)
        trace = json.loads(store.get(ALGORITHM, row.id).algorithm_failure_details)
        assert trace["class"] == "hbm-oom" and trace["oom"]["gpu_index"] == 3, trace["oom"]
        assert any("node-log tail of container algorithm" in s for s in trace["oom"]["signals"]), trace["oom"]
        ann = trace["gpu"]  # the agent's annotation (the pod itself is gone with its Job)
        assert ann["logs"][0]["match"] == "hbm" and ann["logs"][0]["source"] == "node-log"
        assert api.log_requests == []  # auto: the agent read it, no API fetch
        await agent.stop()
        await kc.close()
        await app.stop()
        await api.stop()

    arun(go(), timeout=30)


def test_agent_retries_failed_patch_and_prunes_on_delete(arun, tmp_path):
    """The apiserver answers 500 to the first three annotation PATCHes;
    the evidence still lands, and the agent's per-pod bookkeeping is empty once the pods
    are deleted (no leak, no lost evidence)."""
    async def go():
        api = FakeApiServer(bookmark_interval=0.1)
        url = await api.start()
        labels = load_config(path=None, env={}).labels
        tel = FakeTelemetry(n_gpus=8)
        names = []
        for i in range(3):
            p = make_pod(f"run-{i}", labels, gpus=1, node="n", env={"LOCAL_RANK": "0", "HIP_VISIBLE_DEVICES": str(i)},
                         status={"phase": "Running"})
            api.create(p)
            names.append(p["metadata"]["name"])
        kc = KubeClient(KubeConfig(url))
        agent = NodeAgent(kc, tel, "n", "nexus", log_root=str(tmp_path), retry_base=0.02, retry_max=0.1)
        await agent.start()
        await agent.factory.wait_for_cache_sync(5)
        api.fail_next[("PATCH", "Pod")] = 3
        for n in names:
            api.update(_failed(api.get("Pod", "nexus", n)))
        anns = {}
        for _ in range(int(200 * TIME_SCALE)):
            anns = {n: (api.get("Pod", "nexus", n)["metadata"].get("annotations") or {}).get(ANN) for n in names}
            # the agent counts a PATCH when its answer is in: the server applies it first
            if all(anns.values()) and agent.patches == 3:
                break
            await asyncio.sleep(0.02)
        assert all(anns.values()), anns
        assert agent.patch_failures == 3 and agent.patches == 3
        assert not agent._publishing
        for n in names:
            api.delete("Pod", "nexus", n)
        for _ in range(100):
            if not agent.published:
                break
            await asyncio.sleep(0.02)
        assert agent.published == {}
        await agent.stop()
        await kc.close()
        await api.stop()

    arun(go(), timeout=30)


def test_agent_gives_up_when_the_pod_goes_away(arun, tmp_path):
    async def go():
        api = FakeApiServer(bookmark_interval=0.1)
        url = await api.start()
        labels = load_config(path=None, env={}).labels
        p = make_pod("gone", labels, gpus=1, node="n", env={"HIP_VISIBLE_DEVICES": "0", "LOCAL_RANK": "0"},
                     status={"phase": "Running"})
        api.create(p)
        kc = KubeClient(KubeConfig(url))
        agent = NodeAgent(FailingPatch(kc), FakeTelemetry(n_gpus=2), "n", "nexus", log_root=None, retry_base=0.02,
                          retry_max=0.05)
        await agent.start()
        await agent.factory.wait_for_cache_sync(5)
        api.update(_failed(api.get("Pod", "nexus", p["metadata"]["name"])))
        for _ in range(100):
            if agent.patch_failures >= 3:
                break
            await asyncio.sleep(0.02)
        assert agent._publishing
        api.delete("Pod", "nexus", p["metadata"]["name"])
        for _ in range(100):
            if not agent._publishing and not agent.published:
                break
            await asyncio.sleep(0.02)
        assert not agent._publishing and agent.published == {}
        await agent.stop()
        await kc.close()
        await api.stop()

    arun(go(), timeout=30)


class FailingPatch:
    """KubeClient whose PATCHes always fail (list/watch pass through)."""

    def __init__(self, inner):
        self.inner = inner

    def __getattr__(self, name):
        return getattr(self.inner, name)

    async def patch_merge(self, *a, **kw):
        raise RuntimeError("apiserver unavailable")


def test_log_reader_refuses_names_that_leave_the_log_root(tmp_path):
    """The agent reads /var/log/pods as root: a namespace / pod / uid / container name that
    is not a plain path component never reaches the filesystem."""
    from nexus_supervisor_amd.gpu.logtail import container_log_file

    (tmp_path / "secret.log").write_text("x")
    for ns, pod, uid, ctr in (("..", "p", "u", "c"), ("ns", "p/../..", "u", "c"), ("ns", "p", "u", ".."),
                              ("ns", "p", "", "c"), ("ns", "p", "u", "c\x00")):
        assert container_log_file(str(tmp_path / "pods"), ns, pod, uid, ctr, 0) is None


def test_deferred_decision_keeps_the_failure_arrival_stamps(arun):
    """A default pod's decision waits for its pods/log read (here 0.15 s): its stages start
    at the update that carried the failure — the receive time and the watch batch's delivery
    stamps of the first pass, not of whatever batch is in flight when the log arrives — so
    the wait shows up as the bench's ``classify`` stage instead of vanishing."""
    from nexus_supervisor_amd.bench.runner import PART_NAMES, Tracker, decompose
    from nexus_supervisor_amd.obs import delivery
    from nexus_supervisor_amd.testing.inproc import InProcCluster, RecordingJobs

    class SlowLogs(RecordingJobs):
        async def pod_log(self, *a, **kw):
            await asyncio.sleep(0.15)
            return await super().pod_log(*a, **kw)

    async def go():
        cfg = _app_cfg()
        cfg.observability.stage_timestamps = True
        row = seed_rows()[1]
        pod = make_pod(row.id, cfg.labels, gpus=1, status={"phase": "Running"})
        jobs = SlowLogs([row.id])
        jobs.logs[("nexus", pod["metadata"]["name"], "algorithm")] = (TORCH_OOM + "\n").encode()
        cl = InProcCluster(cfg, MemoryStore([row]), [pod, make_job(row.id, cfg.labels)], jobs=jobs)
        await cl.start()
        delivery.CURRENT["Pod"] = (1.0, 2.0, 3.0)
        cl.push(_failed(pod), "MODIFIED")
        for _ in range(20):
            await asyncio.sleep(0.01)
            if cl.supervisor._log_fetches:
                break
        assert cl.supervisor._log_fetches  # deferred, reading the tail
        delivery.CURRENT["Pod"] = (7.0, 8.0, 9.0)  # a later batch is being dispatched
        for _ in range(200):
            if any(x.outcome == "applied" for x in cl.decisions):
                break
            await asyncio.sleep(0.01)
        d = [x for x in cl.decisions if x.outcome == "applied"][0]
        st = d.result.stamps
        assert d.result.failure_class == FailureClass.HBM_OOM
        assert st["delivery"] == (1.0, 2.0, 3.0)
        assert st["enqueue"] - st["receive"] >= 0.14  # the log wait is classification time
        assert not cl.supervisor._deferred_at
        rec = delivery.record(st, st["delivery"])
        assert len(rec) == 6 and rec[3] >= 0.14 and rec[5] >= rec[3] + rec[4]
        # the Tracker's decomposition: the stages of every band sum to its total
        tr = Tracker()
        parts = []
        for i in range(100):
            total = 1.0 + i / 100
            parts.append((total, 0.1, 0.1, 0.05, 0.05, 0.2 + i / 200, 0.1, total - 0.6 - i / 200))
        tr.parts = parts
        out = decompose(parts)
        assert list(out["stages"]) == list(PART_NAMES)
        for band in ("median_band_mean_ms", "tail_p99_mean_ms"):
            b = out[band]
            assert abs(sum(b[n] for n in PART_NAMES) - b["total"]) < 0.01, b
        delivery.CURRENT.pop("Pod", None)
        await cl.supervisor.stop(drain=False)

    arun(go(), timeout=20)


def test_a_log_read_without_a_decision_forgets_the_arrival_stamps(arun):
    """A default pod whose tail shows an ordinary crash yields no pod-level decision (the
    Job decides): its deferral's arrival stamps are dropped, so a later failure of the same
    pod starts its own clock."""
    from nexus_supervisor_amd.testing.inproc import InProcCluster, RecordingJobs

    async def go():
        cfg = _app_cfg()
        row = seed_rows()[1]
        pod = make_pod(row.id, cfg.labels, gpus=1, status={"phase": "Running"})
        jobs = RecordingJobs([row.id])
        jobs.logs[("nexus", pod["metadata"]["name"], "algorithm")] = (PLAIN_CRASH + "\n").encode()
        cl = InProcCluster(cfg, MemoryStore([row]), [pod, make_job(row.id, cfg.labels)], jobs=jobs)
        await cl.start()
        cl.push(_failed(pod), "MODIFIED")
        sup = cl.supervisor
        for _ in range(100):
            await asyncio.sleep(0.01)
            if sup.metrics.counter("log_tail_fetches") >= 1 and not sup._log_fetches:
                break
        assert sup.metrics.counter("log_tail_fetches") == 1
        assert not sup._deferred_at and not cl.decisions
        await sup.stop(drain=False)

    arun(go(), timeout=20)


def test_prefetched_reads_are_dropped_when_fenced(arun):
    """A checkpoint read prefetched for a deferred GPU failure belongs to the current lease:
    losing it (or the run's shard) cancels the read, so a new leader's decision never takes
    a row read under the old one."""
    from nexus_supervisor_amd.testing.inproc import InProcCluster

    async def go():
        cfg = _app_cfg()
        rows = seed_rows()
        store = MemoryStore(rows)
        pods = [make_pod(r.id, cfg.labels, gpus=1) for r in rows[:2]]
        c = InProcCluster(cfg, store, pods)
        await c.start()
        sup = c.supervisor
        sup.set_active(True)
        assert sup._prefetch_reads
        for p in pods:
            sup._prefetch_read(p)
        sup._prefetch_read(pods[0])  # one read per run
        assert len(sup._prefetch) == 2 and sup.metrics.counter("checkpoint_reads_prefetched") == 2
        futs = [f for f, _t in sup._prefetch.values()]
        sup.fence()
        assert not sup._prefetch
        await asyncio.sleep(0)
        assert all(f.cancelled() or f.done() for f in futs)
        await c.stop()

    arun(go(), timeout=30)


def test_a_stale_prefetched_read_is_never_used(arun):
    """A prefetch whose deferral decided nothing is not taken by a later decision of the run
    once it is older than the longest wait it can overlap: that decision reads again."""
    from nexus_supervisor_amd.testing.inproc import InProcCluster

    async def go():
        cfg = _app_cfg()
        rows = seed_rows()
        store = MemoryStore(rows)
        pod = make_pod(rows[1].id, cfg.labels, gpus=1)
        c = InProcCluster(cfg, store, [pod])
        await c.start()
        sup = c.supervisor
        sup.set_active(True)
        sup._prefetch_read(pod)
        key = (rows[1].algorithm, rows[1].id)
        fut, t0 = sup._prefetch[key]
        await fut
        assert sup._take_prefetch(key) is fut  # fresh: taken
        sup._prefetch_read(pod)
        fut2, _ = sup._prefetch[key]
        sup._prefetch[key] = (fut2, t0 - sup._prefetch_ttl - 1.0)  # as if it were old
        assert sup._take_prefetch(key) is None and key not in sup._prefetch
        await c.stop()

    arun(go(), timeout=30)
