"""GPU-box tests (real MI355X via gpurun): native amd-smi monitor, a real HBM-OOM
from the HIP stress workload attributed to its GPU, and host-OOM kept apart.

BASELINE.json config 3 analog ("inject HBM-OOM … verify per-GPU attribution in
checkpoint") on the one GPU a gpurun box provides.
"""
import json
import os
import subprocess
import time

import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def telemetry():
    from nexus_supervisor_amd.gpu.telemetry import AmdSmiTelemetry

    t = AmdSmiTelemetry(interval=0.1)
    t.start()
    yield t
    t.stop()


@pytest.fixture(scope="module")
def stress_exe():
    from nexus_supervisor_amd._build import binary

    return binary("gpu_stress")


def test_native_modules_load():
    from nexus_supervisor_amd import _amdsmi_monitor, _cql_native  # noqa: F401

    assert _cql_native.murmur3_token(b"123") == -7468325962851647638


def test_monitor_sees_mi355x(telemetry):
    devs = telemetry.devices()
    assert devs, "amd-smi reported no GPU"
    d = devs[0]
    assert d["vram_total_mb"] > 250_000, d  # 288 GB HBM3E
    assert "MI355" in d["market_name"] or d["vram_total_mb"] > 280_000
    time.sleep(0.3)
    snap = telemetry.snapshot()
    assert snap[0]["vram_total_mb"] == d["vram_total_mb"]
    assert telemetry.samples >= 2


def test_native_history_mirrors_into_worker_view(telemetry, stress_exe):
    """The replica's one amd-smi monitor forwarded to a shard worker (RemoteTelemetry):
    the mirrored VRAM peak of a real 16 GiB hold equals the native monitor's."""
    from nexus_supervisor_amd.gpu.telemetry import RemoteTelemetry, telemetry_message

    mirror, since = RemoteTelemetry(), {}
    t0 = time.time()
    mirror.update(json.loads(json.dumps(telemetry_message(telemetry, since))))
    p = subprocess.run([stress_exe, "hold", "--gib", "16", "--seconds", "1.0"], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    time.sleep(0.3)
    mirror.update(json.loads(json.dumps(telemetry_message(telemetry, since))))
    t1 = time.time()
    gi = telemetry.devices()[0]["index"]
    native = telemetry.peak_between(gi, t0, t1)
    assert native > 16_000 and mirror.peak_between(gi, t0, t1) == native
    assert len(telemetry.history(gi, t0)) >= 5


def _run_oom(exe, tmp_path, env_extra):
    log = tmp_path / "termination.log"
    env = dict(os.environ, **env_extra)
    t0 = time.time()
    p = subprocess.Popen([exe, "hbm-oom", "--chunk-gib", "4", "--linger", "1.0", "--termination-log", str(log),
                          "--max-gib", "400"], env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    out, err = p.communicate(timeout=180)
    return p.pid, p.returncode, log.read_text() if log.exists() else "", out, err, t0, time.time()


def test_real_hbm_oom_attributed_to_gpu(telemetry, stress_exe, tmp_path):
    """A real HIP OOM on the box's MI355X: the failing process is matched by PID (VERDICT
    r1 weak #2 — amd-smi reports host-namespace PIDs here, so the monitor's DRM-fdinfo
    scan of our own /proc supplies the PID, its rank env and its own VRAM peak), the
    verdict is hbm-oom on that GPU and the trace carries the measured xGMI links."""
    from nexus_supervisor_amd.classify import Classifier, render_trace
    from nexus_supervisor_amd.config.schema import LabelConfig
    from nexus_supervisor_amd.gpu.telemetry import evidence_for
    from nexus_supervisor_amd.models.decisions import FailureClass
    from nexus_supervisor_amd.testing.seed import make_pod

    env = {"RANK": "3", "LOCAL_RANK": "0", "WORLD_SIZE": "8", "LOCAL_WORLD_SIZE": "8", "MASTER_ADDR": "10.0.0.7",
           "MASTER_PORT": "29500"}
    pid, rc, msg, out, err, t0, t1 = _run_oom(stress_exe, tmp_path, env)
    assert rc == 1, (rc, out[-500:], err[-500:])
    assert "hipErrorOutOfMemory" in msg or "out of memory" in msg.lower(), msg
    time.sleep(0.3)
    ev = evidence_for(telemetry, pids=[pid], gpu_indices=[0], lookback=t1 - t0 + 5)
    assert ev is not None
    g = ev["gpus"][0]
    assert g["vram_peak_mb"] >= 0.9 * g["vram_total_mb"], g
    mine = [p for p in g["procs"] if p["pid"] == pid]
    pid_matched = bool(mine)
    assert pid_matched, (telemetry.proc_mode, g)
    assert mine[0]["rank"] == 3 and mine[0]["world_size"] == 8, mine
    assert mine[0]["peak_vram_bytes"] >= 0.8 * g["vram_total_mb"] * (1 << 20), mine
    assert g["window"][0] >= t0 - 1.0  # the window is the process's own lifetime, not the lookback

    labels = LabelConfig()
    pod_env = dict(env, HIP_VISIBLE_DEVICES="0")
    pod = make_pod("gpu-oom-run", labels, env=pod_env, gpus=1, node="mi355x-box", rv="2", status={
        "phase": "Failed", "containerStatuses": [{"name": "algorithm", "restartCount": 0, "state": {
            "terminated": {"reason": "Error", "exitCode": 1, "message": msg}}}]})
    pod["metadata"]["annotations"] = {"nexus.amd.com/gpu-evidence": json.dumps(ev)}
    c = Classifier(labels)
    res = c.classify_pod(pod)
    assert len(res) == 1
    r = res[0]
    assert r.failure_class == FailureClass.HBM_OOM
    assert r.evidence["oom"]["kind"] == "hbm"
    assert r.evidence["oom"]["gpu_index"] == 0
    assert r.evidence["oom"]["peak_vram_bytes"] == mine[0]["peak_vram_bytes"]
    assert r.evidence["topology"]["rank"] == 3 and r.evidence["topology"]["world_size"] == 8
    trace = json.loads(render_trace(r))
    assert trace["class"] == "hbm-oom" and trace["gpu"]["gpus"][0]["index"] == 0
    xg = trace["topology"]["xgmi"]
    if g.get("links"):  # amd-smi link metrics: the GPU's real xGMI ports and peers
        assert xg["source"] == "amdsmi" and all(r.get("max_gbps") for r in xg["per_gpu"]), xg
        r0 = xg["per_gpu"][0]
        assert r0["links_listed"] == len(g["links"]) and xg["fully_connected"] is None  # one GPU: nothing to connect
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/hbm_oom_attribution.json", "w") as f:
        json.dump({"pid_matched": pid_matched, "proc_source": telemetry.proc_mode, "pid": pid,
                   "evidence": ev, "trace": trace, "message": msg}, f, indent=1)


def test_host_oom_not_blamed_on_idle_gpu(telemetry):
    from nexus_supervisor_amd.classify import Classifier
    from nexus_supervisor_amd.config.schema import LabelConfig
    from nexus_supervisor_amd.gpu.telemetry import pod_evidence_provider
    from nexus_supervisor_amd.models.decisions import FailureClass
    from nexus_supervisor_amd.testing.seed import make_pod

    time.sleep(2.5)  # let the OOM test's VRAM peak leave the lookback window
    labels = LabelConfig()
    c = Classifier(labels)
    c.evidence_provider = pod_evidence_provider(telemetry, lookback=1.0)
    pod = make_pod("host-oom-run", labels, env={"LOCAL_RANK": "0", "HIP_VISIBLE_DEVICES": "0"}, gpus=1, rv="2", status={
        "phase": "Failed", "containerStatuses": [{"name": "algorithm", "restartCount": 0, "state": {
            "terminated": {"reason": "OOMKilled", "exitCode": 137}}}]})
    res = c.classify_pod(pod)
    assert res and res[0].failure_class == FailureClass.HOST_OOM
    assert res[0].evidence["oom"]["kind"] == "host"


def test_hold_workload_visible_as_process(telemetry, stress_exe):
    p = subprocess.Popen([stress_exe, "hold", "--gib", "16", "--seconds", "2.0"], stdout=subprocess.PIPE,
                         stderr=subprocess.PIPE, text=True)
    try:
        deadline = time.time() + 20
        seen = None
        while time.time() < deadline and p.poll() is None:
            snap = telemetry.snapshot(False)
            used = snap[0]["vram_used_mb"]
            if used >= 15_000:
                seen = used
                break
            time.sleep(0.1)
        assert seen is not None, "VRAM use of the hold workload never showed up"
    finally:
        out, err = p.communicate(timeout=60)
    assert p.returncode == 0, err


def test_cfg3_stress_pods_with_real_hbm_oom(arun):
    """BASELINE config 3 on the box's one MI355X: 7 pods hold 30 GiB each, an 8th is
    driven to a real HIP OOM; the checkpoint row must say hbm-oom on GPU 0 with the
    VRAM peak near the 288 GB capacity."""
    from nexus_supervisor_amd.bench.scenarios import cfg3_gpu

    r = arun(cfg3_gpu("uncapped", holders=7, hold_gib=30.0), timeout=300)
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/cfg3.json", "w") as f:
        json.dump(r, f, indent=1)
    assert r["oom_rc"] == 1 and r["stage"] == "FAILED", r
    assert r["trace_class"] == "hbm-oom" and r["gpu_index"] == 0, r
    assert r["vram_peak_mb"] >= 0.9 * r["vram_total_mb"], r
    assert r["acked"] == 1 and r["p50_ms"] < 1000, r


def test_node_agent_annotates_real_hbm_oom(stress_exe, tmp_path, arun):
    """The per-node agent on a real MI355X: the pod's GPU comes from the kubelet
    pod-resources allocation (the device's real PCI BDF from amd-smi); after a real HIP
    OOM the failed pod is annotated with that GPU's evidence (VRAM peak ≈ 288 GB)."""
    from nexus_supervisor_amd.config import load_config
    from nexus_supervisor_amd.gpu.agent import NodeAgent
    from nexus_supervisor_amd.kube.client import KubeClient, KubeConfig
    from nexus_supervisor_amd.testing.fake_apiserver import FakeApiServer
    from nexus_supervisor_amd.gpu.telemetry import AmdSmiTelemetry
    from nexus_supervisor_amd.testing.seed import make_pod

    telemetry = AmdSmiTelemetry(interval=0.1)  # the agent owns (and stops) its monitor
    telemetry.start()
    dev0 = telemetry.devices()[0]
    assert dev0.get("bdf"), dev0

    class PodRes:
        def list(self):
            return [{"name": "oom-run-w0", "namespace": "nexus", "containers": [
                {"name": "algorithm", "devices": [{"resource_name": "amd.com/gpu", "device_ids": [dev0["bdf"]]}]}]}]

        def close(self):
            pass

    async def go():
        api = FakeApiServer(bookmark_interval=0.1)
        url = await api.start()
        labels = load_config(path=None, env={}).labels
        api.create(make_pod("oom-run", labels, suffix="w0", gpus=1, node="mi355x-box", status={"phase": "Running"}))
        kc = KubeClient(KubeConfig(url))
        agent = NodeAgent(kc, telemetry, "mi355x-box", "nexus", pod_resources=PodRes())
        await agent.start()
        assert await agent.factory.wait_for_cache_sync(10)
        loop = asyncio.get_running_loop()
        pid, rc, msg, out, err, t0, t1 = await loop.run_in_executor(None, _run_oom, stress_exe, tmp_path,
                                                                     {"HIP_VISIBLE_DEVICES": "0"})
        assert rc == 1, (rc, err[-400:])
        p = api.get("Pod", "nexus", "oom-run-w0")
        p = dict(p, status={"phase": "Failed", "containerStatuses": [{"name": "algorithm", "state": {
            "terminated": {"reason": "Error", "exitCode": 1, "message": msg}}}]})
        api.update(p)
        ann = None
        for _ in range(200):
            ann = (api.get("Pod", "nexus", "oom-run-w0")["metadata"].get("annotations") or {}).get(
                "nexus.amd.com/gpu-evidence")
            if ann:
                break
            await asyncio.sleep(0.05)
        await agent.stop()
        await kc.close()
        await api.stop()
        return ann

    import asyncio

    ann = arun(go(), timeout=240)
    assert ann, "agent never annotated the failed pod"
    ev = json.loads(ann)
    g = ev["gpus"][0]
    assert g["index"] == 0 and g["bdf"].lower().endswith(dev0["bdf"].lower()[-7:])
    assert g["vram_peak_mb"] >= 0.9 * g["vram_total_mb"], g
    assert ev["source"] == "amdsmi" and ev["reason"] == "pod-failed"
    assert ev["allocated"] == [0], ev  # the device-plugin allocation travels with the evidence


# ----------------------------------------------------------------------------- default pods
# A default pod (terminationMessagePolicy: File) that dies of an
# HBM-OOM has an EMPTY termination message; the OOM text is on stderr only, and the
# process's VRAM is freed the moment it exits.  Production sample interval (0.5 s).

def _default_pod(labels, rid, gpus=1):
    from nexus_supervisor_amd.testing.seed import make_pod

    return make_pod(rid, labels, gpus=gpus, node="mi355x-box", env={"LOCAL_RANK": "0", "HIP_VISIBLE_DEVICES": "0",
                                                                   "RANK": "0", "WORLD_SIZE": "1"},
                    status={"phase": "Running"})


def _exit_status(pod, code):
    p = json.loads(json.dumps(pod))
    p["status"] = {"phase": "Failed", "containerStatuses": [{"name": "algorithm", "restartCount": 0, "state": {
        "terminated": {"reason": "Error", "exitCode": code, "message": ""}}}]}
    return p


def _supervise_default_pod(arun, tmp_path, stream_text, rc, *, agent: bool, telemetry=None):
    """One default GPU pod fails with exit ``rc`` and an empty termination message; its
    stderr is ``stream_text``.  ``agent``: the node agent reads it from a /var/log/pods
    fixture (CRI format, what the kubelet holds); else the supervisor GETs pods/log
    (``telemetry``: with the co-located monitor's GPU evidence).  Returns the checkpoint
    row's trace."""
    import asyncio

    from nexus_supervisor_amd.app import Application
    from nexus_supervisor_amd.config import load_config
    from nexus_supervisor_amd.gpu.agent import NodeAgent
    from nexus_supervisor_amd.gpu.telemetry import AmdSmiTelemetry
    from nexus_supervisor_amd.kube.client import KubeClient, KubeConfig
    from nexus_supervisor_amd.store.memory import MemoryStore
    from nexus_supervisor_amd.testing.fake_apiserver import FakeApiServer
    from nexus_supervisor_amd.testing.fakelogs import write_cri_log
    from nexus_supervisor_amd.testing.seed import ALGORITHM, make_job, seed_rows

    row = seed_rows()[1]  # RUNNING
    cfg = load_config(path=None, env={}, overrides={
        "cql-store-type": "memory", "rate-limit-elements-per-second": 0, "resync-period": "0s",
        "gpu": {"sample-interval": "500ms", "evidence-wait": "3s" if agent else "0s"}})
    pod = _default_pod(cfg.labels, row.id)
    name, uid = pod["metadata"]["name"], pod["metadata"]["uid"]
    logroot = tmp_path / "var-log-pods"
    write_cri_log(str(logroot), "nexus", name, uid, "algorithm", 0, [("stderr", stream_text)])

    async def go():
        api = FakeApiServer(bookmark_interval=0.1)
        url = await api.start()
        api.create(pod)
        api.create(make_job(row.id, cfg.labels))
        api.set_pod_log("nexus", name, "algorithm", stream_text)
        store = MemoryStore([row])
        app = Application(cfg, kube=KubeClient(KubeConfig(url)), store=store)
        await app.start()
        if telemetry is not None:
            from nexus_supervisor_amd.gpu.telemetry import pod_evidence_provider

            app.supervisor.classifier.evidence_provider = pod_evidence_provider(telemetry, lookback=120)
        kc = ag = None
        if agent:
            tel = AmdSmiTelemetry(interval=cfg.gpu.sample_interval)  # the agent owns (and stops) it
            kc = KubeClient(KubeConfig(url))
            ag = NodeAgent(kc, tel, "mi355x-box", "nexus", log_root=str(logroot))
            await ag.start()
            assert await ag.factory.wait_for_cache_sync(10)
        assert await app.factory.wait_for_cache_sync(10)
        api.update(_exit_status(api.get("Pod", "nexus", name), rc))
        for _ in range(300):
            if store.get(ALGORITHM, row.id).lifecycle_stage == "FAILED":
                break
            await asyncio.sleep(0.02)
        out = store.get(ALGORITHM, row.id)
        log_requests = list(api.log_requests)
        if ag is not None:
            await ag.stop()
            await kc.close()
        await app.stop()
        await api.stop()
        return out, log_requests

    out, log_requests = arun(go(), timeout=120)
    assert out.lifecycle_stage == "FAILED", (out.lifecycle_stage, out.algorithm_failure_details)
    return json.loads(out.algorithm_failure_details), log_requests


def test_default_pod_hbm_oom_from_log_tail(stress_exe, tmp_path, arun):
    """gpu_stress in the default-pod shape (--no-termination-log --linger 0): a real HIP
    OOM on the MI355X, the torch-worded error on stderr only, exit 1 at once.  Read from
    the node's log by the agent, and over pods/log by the supervisor alone: both rows are
    FAILED / hbm-oom / GPU 0 with a signal naming the log-tail source."""
    p = subprocess.run([stress_exe, "hbm-oom", "--chunk-gib", "4", "--no-termination-log", "--linger", "0",
                        "--max-gib", "400"], capture_output=True, text=True, timeout=180)
    assert p.returncode == 1, (p.returncode, p.stderr[-500:])
    assert "torch.OutOfMemoryError: HIP out of memory" in p.stderr, p.stderr[-500:]
    text = p.stdout[-4000:] + p.stderr
    results = {}
    for agent in (True, False):
        trace, reqs = _supervise_default_pod(arun, tmp_path / ("agent" if agent else "api"), text, p.returncode,
                                             agent=agent)
        src = "node-log tail" if agent else "pods/log tail"
        assert trace["class"] == "hbm-oom" and trace["oom"]["kind"] == "hbm", trace
        assert trace["oom"]["gpu_index"] == 0, trace["oom"]
        assert any(src in s for s in trace["oom"]["signals"]), trace["oom"]["signals"]
        assert (reqs == []) if agent else len(reqs) == 1
        results["agent" if agent else "pods_log"] = trace
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/default_pod_hbm_oom.json", "w") as f:
        json.dump({"sample_interval_s": 0.5, "stress_rc": p.returncode, "stderr_tail": p.stderr[-1200:],
                   "traces": results}, f, indent=1)


def test_default_pod_real_torch_oom(tmp_path, arun):
    """A real PyTorch HBM-OOM (torch.empty larger than the 288 GB HBM3E): torch's own
    exception text on stderr, exit 1, nothing in the termination message — classified
    hbm-oom from the pods/log tail."""
    import sys

    code = ("import torch\n"
            "torch.ones(1, device='cuda')\n"
            "x = torch.empty(int(320 * 2**30), dtype=torch.uint8, device='cuda')\n")
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert p.returncode == 1, (p.returncode, p.stderr[-800:])
    assert "OutOfMemoryError" in p.stderr, p.stderr[-800:]
    trace, reqs = _supervise_default_pod(arun, tmp_path, p.stderr, p.returncode, agent=False)
    assert trace["class"] == "hbm-oom" and trace["oom"]["requested_bytes"] == 320 << 30, trace["oom"]
    assert trace["oom"]["gpu_index"] == 0 and any("pods/log tail" in s for s in trace["oom"]["signals"])
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/default_pod_torch_oom.json", "w") as f:
        json.dump({"stderr_tail": p.stderr[-1500:], "trace": trace}, f, indent=1)


def test_previous_tenants_peak_does_not_make_a_crash_an_oom(stress_exe):
    """Negative: a previous tenant holds 280 GiB (≥ 97 % of the MI355X) and exits; then a
    pod on the same GPU exits 1 with no OOM text.  The device-wide peak is in the window,
    but it is not the pod's own (no process of the pod matched): no OOM verdict."""
    from nexus_supervisor_amd.gpu import oom
    from nexus_supervisor_amd.gpu.telemetry import AmdSmiTelemetry, evidence_for

    tel = AmdSmiTelemetry(interval=0.5)
    tel.start()
    try:
        t0 = time.time()
        p = subprocess.run([stress_exe, "hold", "--gib", "280", "--seconds", "2.0"], capture_output=True, text=True,
                           timeout=180)
        assert p.returncode == 0, p.stderr[-400:]
        time.sleep(0.6)
        ev = evidence_for(tel, pod_uid="pod-uid-crash", gpu_indices=[0], lookback=time.time() - t0 + 2)
    finally:
        tel.stop()
    g = ev["gpus"][0]
    assert g["vram_peak_mb"] >= 0.97 * g["vram_total_mb"], g  # the tenant's peak is in the window
    assert not g["matched"] and "proc_peak_vram_bytes" not in g
    v = oom.analyze(["Traceback (most recent call last):", "ValueError: bad batch"],
                    [{"container": "algorithm", "exitCode": 1, "reason": "Error", "message": ""}], ev)
    assert v.kind is None and not v.signature, v.as_dict()
    assert any("not an OOM verdict" in s for s in v.signals), v.signals


def test_multi_rank_job_root_cause_from_a_real_hbm_oom(telemetry, stress_exe, tmp_path):
    """A 2-rank job (one pod per rank): rank 1 hits a real HIP OOM on this MI355X, rank 0
    dies later of its all-reduce's watchdog timeout.  The Job-level decision
    (BackoffLimitExceeded) names rank 1 as the culprit, is an hbm-oom on GPU 0 from the real
    evidence, and counts rank 0 as collateral (gpu/collective.py)."""
    from nexus_supervisor_amd.classify import Classifier, render_trace
    from nexus_supervisor_amd.config.schema import LabelConfig
    from nexus_supervisor_amd.gpu.telemetry import evidence_for
    from nexus_supervisor_amd.models.decisions import FailureClass
    from nexus_supervisor_amd.testing.seed import make_event, make_job, make_pod

    env = {"RANK": "1", "LOCAL_RANK": "0", "WORLD_SIZE": "2", "MASTER_ADDR": "10.0.0.9", "MASTER_PORT": "29500"}
    pid, rc, msg, out, err, t0, t1 = _run_oom(stress_exe, tmp_path, env)
    assert rc == 1 and ("hipErrorOutOfMemory" in msg or "out of memory" in msg.lower()), (rc, msg, err[-300:])
    time.sleep(0.3)
    ev = evidence_for(telemetry, pids=[pid], gpu_indices=[0], lookback=t1 - t0 + 5)
    labels = LabelConfig()
    run = "ddp-real-oom"

    def rank_pod(r, message, finished, evidence=None):
        p = make_pod(run, labels, suffix=f"r{r}", gpus=1, rv="4", node="mi355x-box",
                     env={"RANK": str(r), "WORLD_SIZE": "2", "LOCAL_RANK": "0", "HIP_VISIBLE_DEVICES": "0"},
                     status={"phase": "Failed", "containerStatuses": [{"name": "algorithm", "restartCount": 0, "state": {
                         "terminated": {"reason": "Error", "exitCode": 1, "message": message, "finishedAt": finished}}}]})
        if evidence:
            p["metadata"]["annotations"] = {"nexus.amd.com/gpu-evidence": json.dumps(evidence)}
        return p

    watchdog = ("[Rank 0] Watchdog caught collective operation timeout: WorkNCCL(SeqNum=77, OpType=ALLREDUCE) ran for "
                "600010 milliseconds before timing out.")
    pods = [rank_pod(0, watchdog, "2026-10-17T10:10:00Z"), rank_pod(1, msg, "2026-10-17T10:00:00Z", ev)]
    job = make_job(run, labels)

    class Lookup:
        def get(self, kind, name):
            return job if kind == "Job" and name == run else None

        def pods_of_job(self, name):
            return pods

    _s, [r] = Classifier(labels).classify_event(make_event("Job", run, "BackoffLimitExceeded", "backoff limit"), Lookup())
    assert r.failure_class == FailureClass.HBM_OOM, r.evidence
    assert r.evidence["oom"]["gpu_index"] == 0
    ranks = r.evidence["ranks"]
    assert ranks["culprit"]["rank"] == 1 and ranks["culprit"]["kind"] == "hbm-oom" and ranks["collateral"] == 1
    trace = json.loads(render_trace(r))
    assert trace["ranks"]["culprit"]["pod"] == f"{run}-r1"
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/multi_rank_root_cause.json", "w") as f:
        json.dump({"trace": trace, "message": msg}, f, indent=1)


def test_real_hip_runtime_oom_wording_on_a_full_gpu(stress_exe, tmp_path, arun, telemetry):
    """The GPU is filled by another tenant (``gpu_stress hbm-oom`` holding every chunk it
    got), then a fresh torch process needs a HIP context, a hipBLAS handle and a 2 GiB
    buffer.  Two fill levels:

    * 0.5 GiB chunks (under 0.5 GiB left): the context comes up and the allocation fails —
      whatever ROCm / torch print (``HIP error: out of memory``, a hipBLAS / rocBLAS status,
      torch's ``OutOfMemoryError``) is the real text of a default pod's log tail and must be
      classified hbm-oom on GPU 0;
    * then 8 MiB chunks into the rest (under 8 MiB left): the process may die while the HIP
      runtime initialises.  If it printed an allocation failure that is hbm-oom as above; if
      it printed none (a crash with nothing in the log) the row must NOT claim an HBM-OOM —
      the other tenant's full GPU is no evidence about this pod."""
    import sys

    from nexus_supervisor_amd.gpu import oom

    code = ("import torch\n"
            "a = torch.randn(256, 256, device='cuda')\n"
            "b = a @ a\n"
            "c = torch.empty(int(2 * 2**30), dtype=torch.uint8, device='cuda')\n"
            "torch.cuda.synchronize()\n")
    holders, fills, runs = [], [], []
    try:
        for i, chunk in enumerate(("0.5", "0.0078125")):
            done = tmp_path / f"filler{i}.termination"
            holders.append(subprocess.Popen([stress_exe, "hbm-oom", "--chunk-gib", chunk, "--linger", "120",
                                             "--termination-log", str(done), "--max-gib", "400"],
                                            stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
            deadline = time.time() + 150
            while not done.exists() and holders[-1].poll() is None and time.time() < deadline:
                time.sleep(0.2)
            assert done.exists() and holders[-1].poll() is None, f"filler {i} did not reach its OOM"
            fills.append(done.read_text()[:300])
            p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240)
            run = {"fill_chunk_gib": float(chunk), "rc": p.returncode, "stderr": p.stderr}
            # decided while the fillers still hold the GPU: the trace names who filled it
            run["decision"] = _decide_on_full_gpu(arun, tmp_path / f"run{i}", p.stderr, p.returncode, telemetry)
            runs.append(run)
    finally:
        for holder in holders:
            holder.terminate()
            try:
                holder.wait(30)
            except subprocess.TimeoutExpired:
                holder.kill()
                holder.wait(30)
    out = []
    for k, r in enumerate(runs):
        assert r["rc"] != 0, (r["rc"], r["stderr"][-800:])
        sig = oom.hbm_signature(r["stderr"])
        if k == 0:
            assert sig, r["stderr"][-1500:]
        trace, verdict = r["decision"]
        if sig:
            assert trace["class"] == "hbm-oom" and trace["oom"].get("gpu_index", 0) == 0, trace
        else:
            # no text, a crash (exit 139 at HIP init was seen here): no HBM-OOM may be read into
            # it; its Job's BackoffLimitExceeded decides
            assert "oom" not in trace and trace["class"] != "hbm-oom", trace
        # either way the GPU is named as someone else's: the filler's ~287 GiB is the holder
        fo = trace["foreign_occupancy"]
        assert fo["gpu"] == 0 and fo["own_peak_bytes"] < 0.1 * fo["total_bytes"], fo
        assert fo["holders"] and fo["holders"][0]["vram_bytes"] >= 250 * (1 << 30), fo["holders"]
        out.append({"fill_chunk_gib": r["fill_chunk_gib"], "rc": r["rc"], "signature": sig,
                    "runtime_check_wording": "error: out of memory" in r["stderr"].lower(),
                    "stderr_tail": r["stderr"][-1500:], "verdict": verdict, "trace": trace})
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/hip_runtime_oom.json", "w") as f:
        json.dump({"fillers": fills, "runs": out}, f, indent=1)


def _decide_on_full_gpu(arun, tmp_path, stderr, rc, telemetry):
    """The decision a failed default pod gets on this box's (filled) GPU with the
    co-located monitor's evidence: the pod-status decision when its log tail holds an
    allocation failure, else (a crash with no text) its Job's BackoffLimitExceeded.
    Returns (trace, verdict)."""
    from nexus_supervisor_amd.classify import Classifier, render_trace
    from nexus_supervisor_amd.config.schema import LabelConfig
    from nexus_supervisor_amd.gpu import oom
    from nexus_supervisor_amd.gpu.telemetry import pod_evidence_provider
    from nexus_supervisor_amd.testing.seed import make_event, make_job

    exit_code = rc if rc > 0 else 128 - rc  # killed by a signal: 128 + signo
    if oom.hbm_signature(stderr):
        trace, _reqs = _supervise_default_pod(arun, tmp_path, stderr, exit_code, agent=False, telemetry=telemetry)
        return trace, trace["class"]
    labels = LabelConfig()
    pod = _exit_status(_default_pod(labels, "crash-at-init"), exit_code)
    job = make_job("crash-at-init", labels)

    class Lookup:
        def get(self, kind, name):
            return job if kind == "Job" else None

        def pods_of_job(self, name):
            return [pod]

    c = Classifier(labels)
    c.evidence_provider = pod_evidence_provider(telemetry, lookback=120)
    _s, [r] = c.classify_event(make_event("Job", "crash-at-init", "BackoffLimitExceeded", "backoff limit"), Lookup())
    trace = json.loads(render_trace(r))
    return trace, f"no OOM verdict (exit {exit_code}, no allocation-failure text), GPU occupied"


def test_node_agent_privileges_reported_on_the_box(stress_exe, tmp_path):
    """gpurun boxes run this suite as an ordinary user — the situation of an agent image's
    default UID.  Its own processes are still attributed (same UID), every refused read of
    another user's /proc entry is counted (agent_proc_scan_denied{source}), an unreadable
    container log is reported as a denial, and the privilege check says the agent lacks
    what the chart gives it (root)."""
    from nexus_supervisor_amd.gpu.agent import NodeAgent, process_privileges
    from nexus_supervisor_amd.gpu.telemetry import AmdSmiTelemetry, evidence_for

    priv = process_privileges()
    tel = AmdSmiTelemetry(interval=0.1, proc_source="drm")
    tel.start()
    try:
        t0 = time.time()
        p = subprocess.Popen([stress_exe, "hold", "--gib", "8", "--seconds", "2.0"], stdout=subprocess.PIPE,
                             stderr=subprocess.PIPE, text=True)
        out, err = p.communicate(timeout=120)
        assert p.returncode == 0, err[-400:]
        time.sleep(0.3)
        ev = evidence_for(tel, pids=[p.pid], gpu_indices=[0], lookback=time.time() - t0 + 2)

        class _NullFactory:
            def informer(self, kind, **kw):
                return None

        logs = tmp_path / "pods"
        d = logs / "nexus_run-w0_uid-1" / "algorithm"
        d.mkdir(parents=True)
        (d / "0.log").write_text("x stderr F RuntimeError: HIP error: out of memory\n")
        os.chmod(d / "0.log", 0)
        agent = NodeAgent(None, tel, "box", "nexus", factory=_NullFactory(), log_root=str(logs))
        pod = {"metadata": {"name": "run-w0", "namespace": "nexus", "uid": "uid-1"},
               "status": {"phase": "Failed", "containerStatuses": [{"name": "algorithm", "restartCount": 0, "state": {
                   "terminated": {"reason": "Error", "exitCode": 1, "message": ""}}}]}}
        recs = agent.log_evidence(pod)
        new = agent.check_denials()
        denials = tel.denials()
    finally:
        tel.stop()
    g = ev["gpus"][0]
    assert any(x["pid"] == p.pid for x in g["procs"]), g  # the same UID's process: attributed
    counters = {k: {tuple(sorted(lab)): v for lab, v in vals.items()} for k, vals in agent.metrics.counters.items()}
    if os.geteuid() != 0:
        assert not priv["sufficient"], priv
        assert denials.get("fd", 0) > 0 and new.get("fd", 0) > 0, denials  # root's processes: refused, counted
        assert counters["agent_proc_scan_denied"][(("source", "fd"),)] > 0
        assert recs[0].get("denied") is True and counters["agent_log_read_denied"][()] == 1
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/agent_privileges.json", "w") as f:
        json.dump({"euid": os.geteuid(), "privileges": priv, "denials": denials, "log_record": recs,
                   "own_process_attributed": True}, f, indent=1)


def test_cfg3a_agent_path_real_hbm_oom(arun):
    """Config 3a on the MI355X: the node agent as its own process (amd-smi at the
    production 0.5 s interval, /var/log/pods reader), the supervisor without local
    telemetry waiting ``gpu.evidence-wait: 2s`` for its annotation.  Each of 10 default
    pods is preceded by a real HIP OOM whose stderr is the pod's log; every row must be
    FAILED / hbm-oom / GPU 0 from the agent's node-log reading, with no pods/log read and
    no expired wait."""
    from nexus_supervisor_amd.bench.scenarios import cfg3_agent

    r = arun(cfg3_agent("uncapped", runs=10, gpu=True), timeout=600)
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/cfg3a.json", "w") as f:
        json.dump(r, f, indent=1)
    assert r["oom_rcs"] == [1] and r["acked"] == 10 and r["wrong"] == 0, r
    assert r["supervisor_pod_log_reads"] == 0 and r["evidence_wait_expired"] == 0, r
    assert r["rows_with_gpu_record"] == 10 and r["vram_total_mb"] > 250_000, r
    assert r["vram_peak_mb"] >= 0.9 * r["vram_total_mb"], r


_REBUILT_CHECK = r"""
import json, os, subprocess, sys, time
tmp = os.environ["NEXUS_NATIVE_DIR"]
from nexus_supervisor_amd import _amdsmi_monitor, _cql_native, _kube_native
mods = {m.__name__: m.__file__ for m in (_amdsmi_monitor, _cql_native, _kube_native)}
assert all(f.startswith(tmp) for f in mods.values()), mods
assert _cql_native.murmur3_token(b"123") == -7468325962851647638
router = _kube_native.ShardRouter(0, 2, 7, "app.kubernetes.io/name", 30.0)
from nexus_supervisor_amd.gpu.telemetry import AmdSmiTelemetry
tel = AmdSmiTelemetry(interval=0.05)
tel.start()
try:
    t0 = time.time()
    p = subprocess.run([os.path.join(tmp, "gpu_stress"), "hold", "--gib", "4", "--seconds", "0.6"],
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    time.sleep(0.2)
    gi = tel.devices()[0]["index"]
    peak = tel.peak_between(gi, t0, time.time())
finally:
    tel.stop()
print(json.dumps({"modules": mods, "peak_mb": peak}))
"""


def test_native_code_rebuilt_from_source_on_the_box(tmp_path):
    """The pushed tree carries container-built ``.so`` files; this rebuilds the native
    extensions and the gfx950 HIP workload from source *on the box* (its own hipcc and
    g++), loads the rebuilt extensions in a fresh interpreter (``NEXUS_NATIVE_DIR``) and
    has the rebuilt amd-smi monitor see the rebuilt HIP workload's 4 GiB on the MI355X."""
    import hashlib
    import sys

    from nexus_supervisor_amd import _build

    only = ["cql_native", "kube_native", "amdsmi_monitor", "gpu_stress"]
    t0 = time.time()
    lines = _build.build(force=True, only=only, out_root=str(tmp_path))
    build_s = time.time() - t0
    assert all(": built " in ln for ln in lines), lines
    ts, intree = _build.targets(out_root=str(tmp_path)), _build.targets()

    def sha(path):
        with open(path, "rb") as f:
            return hashlib.sha256(f.read()).hexdigest()[:16]

    env = dict(os.environ, NEXUS_NATIVE_DIR=str(tmp_path))
    p = subprocess.run([sys.executable, "-c", _REBUILT_CHECK], capture_output=True, text=True, timeout=180, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    res = json.loads(p.stdout.strip().splitlines()[-1])
    assert res["peak_mb"] >= 4000, res
    tools = {}
    for name, cmd in (("hipcc", [os.path.join(_build.ROCM, "bin", "hipcc"), "--version"]), ("cxx", [_build._cxx(), "--version"])):
        out = subprocess.run(cmd, capture_output=True, text=True).stdout.strip().splitlines()
        tools[name] = out[0] if out else ""
    rec = {"build_s": round(build_s, 1), "built": lines, "tools": tools, "loaded": res["modules"],
           "peak_mb": res["peak_mb"],
           "sha16": {n: {"in_tree": sha(intree[n]["out"]) if os.path.exists(intree[n]["out"]) else None,
                         "rebuilt": sha(ts[n]["out"])} for n in only}}
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/box_rebuild.json", "w") as f:
        json.dump(rec, f, indent=1)
