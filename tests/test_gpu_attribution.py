"""HBM-OOM vs host-OOM scoring and RCCL/xGMI topology parsing (CPU-only)."""
import json

from nexus_supervisor_amd.gpu import oom
from nexus_supervisor_amd.gpu.topology import expected_gpu, merge_process_ranks, rank_env_from_environ, topology_from_env

# verbatim message produced by torch on an MI355X box (profiles/box_probe_r1.json)
TORCH_HBM_OOM = ("torch.OutOfMemoryError: HIP out of memory. Tried to allocate 431.98 GiB. GPU 0 has a total capacity "
                 "of 287.98 GiB of which 287.37 GiB is free. Of the allocated memory 0 bytes is allocated by PyTorch")


def test_torch_hip_oom_is_hbm():
    v = oom.analyze([TORCH_HBM_OOM])
    assert v.kind == "hbm"
    assert v.gpu_index == 0
    assert v.capacity_bytes == int(287.98 * (1 << 30))
    assert v.requested_bytes == int(431.98 * (1 << 30))


def test_cgroup_oomkilled_is_host():
    v = oom.analyze([], [{"reason": "OOMKilled", "exitCode": 137, "container": "algo"}])
    assert v.kind == "host" and v.host_score >= 1.0


def test_oomkilled_wins_tie_with_hip_message():
    v = oom.analyze([TORCH_HBM_OOM], [{"reason": "OOMKilled", "exitCode": 137}])
    assert v.kind == "host"


def test_vram_peak_alone_is_not_an_oom_verdict():
    """A full GPU without any OOM signature (exit 1, no allocation failure) is recorded as
    a signal, not a verdict: a GPU left full by a previous tenant must not turn a plain
    crash into an HBM-OOM that bypasses the Job's retry policy."""
    ev = {"gpus": [{"index": 3, "vram_total_mb": 294896, "vram_peak_mb": 294000},
                   {"index": 4, "vram_total_mb": 294896, "vram_peak_mb": 1000}]}
    v = oom.analyze(["RuntimeError: something failed"], [{"exitCode": 1}], ev, expected_gpu="3")
    assert v.kind is None and v.hbm_score >= 0.5
    assert any("no OOM signature" in s for s in v.signals)
    # SIGKILL (exit 137, no cgroup OOMKilled) on a full GPU: the VRAM evidence decides HBM
    v = oom.analyze([], [{"exitCode": 137}], ev, expected_gpu="3")
    assert v.kind == "hbm" and v.gpu_index == 3


def test_torch_logical_gpu_maps_to_physical_through_visible_devices():
    """Torch's 'GPU 3' is the process's logical ordinal.  With
    HIP_VISIBLE_DEVICES=4,5,6,7 and LOCAL_RANK=3 the failing GPU is physical 7; the trace
    records both and reads GPU 7's evidence, never GPU 3's."""
    from nexus_supervisor_amd.classify import Classifier
    from nexus_supervisor_amd.config.schema import LabelConfig
    from nexus_supervisor_amd.testing.seed import make_pod

    msg = ("torch.OutOfMemoryError: HIP out of memory. Tried to allocate 8.00 GiB. GPU 3 has a total capacity of "
           "287.98 GiB of which 2.10 GiB is free.")
    ev = {"source": "agent", "gpus": [
        {"index": 3, "vram_total_mb": 294896, "vram_peak_mb": 294500, "procs": []},  # another pod's full GPU
        {"index": 7, "vram_total_mb": 294896, "vram_peak_mb": 292000, "proc_peak_vram_bytes": 280 << 30,
         "procs": [{"pid": 4242, "rank": 3, "local_rank": 3}]}]}
    topo = topology_from_env({"HIP_VISIBLE_DEVICES": "4,5,6,7", "LOCAL_RANK": "3", "RANK": "3", "WORLD_SIZE": "4"})
    assert topo["visible_devices"] == ["4", "5", "6", "7"] and topo["expected_gpu"] == "7"
    v = oom.analyze([msg], [{"exitCode": 1}], ev, topo["expected_gpu"], topo=topo)
    assert v.kind == "hbm" and v.gpu_index == 7 and v.gpu_logical_index == 3
    assert v.peak_vram_bytes == 280 << 30 and v.device_peak_vram_bytes == 292000 << 20
    assert not any("GPU 3 " in s for s in v.signals)

    labels = LabelConfig()
    pod = make_pod("remapped", labels, gpus=4, rv="2", env={"HIP_VISIBLE_DEVICES": "4,5,6,7", "LOCAL_RANK": "3"}, status={
        "phase": "Failed", "containerStatuses": [{"name": "algorithm", "restartCount": 0, "state": {
            "terminated": {"reason": "Error", "exitCode": 1, "message": msg}}}]})
    pod["metadata"]["annotations"] = {"nexus.amd.com/gpu-evidence": json.dumps(ev)}
    r = Classifier(labels).classify_pod(pod)[0]
    assert r.evidence["oom"]["gpu_index"] == 7 and r.evidence["oom"]["gpu_logical_index"] == 3
    assert r.evidence["topology"]["expected_gpu"] == "7"


def test_layered_device_env_and_uuids():
    from nexus_supervisor_amd.gpu.topology import device_map, physical_gpu, resolve_devices

    # ROCr narrows first, HIP indexes into ROCr's list
    t = topology_from_env({"ROCR_VISIBLE_DEVICES": "2,3,6,7", "HIP_VISIBLE_DEVICES": "1,3", "LOCAL_RANK": "1"})
    assert t["visible_devices"] == ["3", "7"] and t["expected_gpu"] == "7"
    assert physical_gpu(t, 0) == 3 and physical_gpu(t, 5) is None
    # device-plugin allocation: the container's ordinals are the allocated GPUs in node order
    assert device_map(t["device_chain"], list(range(8, 16))) == ["11", "15"]
    # UUID entries resolve against telemetry records
    u = topology_from_env({"HIP_VISIBLE_DEVICES": "GPU-abc,GPU-def", "LOCAL_RANK": "1"})
    gpus = [{"index": 2, "uuid": "GPU-abc"}, {"index": 5, "uuid": "GPU-def"}]
    assert physical_gpu(u, 1, gpus) == 5
    r = resolve_devices(u, {"gpus": gpus})
    assert r["physical_devices"] == [2, 5] and r["expected_gpu"] == "5" and r["expected_gpu_logical"] == 1
    assert u["expected_gpu"] == "GPU-def"  # the memoised per-version record is not mutated


def test_plain_failure_is_not_oom():
    v = oom.analyze(["ValueError: bad input"], [{"exitCode": 1, "reason": "Error"}])
    assert v.kind is None


def test_host_memoryerror():
    v = oom.analyze(["Traceback...\nMemoryError"], [{"exitCode": 1}])
    assert v.kind == "host"


def test_hip_error_variants():
    for msg in ["hipErrorOutOfMemory: out of memory", "RCCL WARN Cuda failure 'out of memory'",
                "hipMalloc failed with error 2", "HSA_STATUS_ERROR_OUT_OF_RESOURCES"]:
        assert oom.analyze([msg]).kind == "hbm", msg


def test_topology_from_torchrun_env():
    env = {"RANK": "5", "WORLD_SIZE": "16", "LOCAL_RANK": "5", "LOCAL_WORLD_SIZE": "8", "MASTER_ADDR": "10.0.0.1",
           "MASTER_PORT": "29500", "HIP_VISIBLE_DEVICES": "0,1,2,3,4,5,6,7", "NCCL_SOCKET_IFNAME": "eth0",
           "RCCL_MSCCL_ENABLE": "0", "UNRELATED": "x"}
    t = topology_from_env(env, gpus_requested=8, node="mi355x-07")
    assert t["rank"] == 5 and t["world_size"] == 16 and t["local_rank"] == 5
    assert t["master_addr"] == "10.0.0.1" and t["master_port"] == 29500
    assert t["expected_gpu"] == "5"
    assert t["xgmi"] == {"source": "platform-default", "local_gpus": 8, "links_per_gpu": 7, "fully_connected": True}
    assert t["collective_env"] == {"NCCL_SOCKET_IFNAME": "eth0", "RCCL_MSCCL_ENABLE": "0"}
    assert t["backend"] == "rccl" and t["node"] == "mi355x-07"
    json.dumps(t)


def test_topology_indexed_job_and_single_gpu():
    t = topology_from_env({"JOB_COMPLETION_INDEX": "3", "ROCR_VISIBLE_DEVICES": "6"}, gpus_requested=1)
    assert t["rank"] == 3 and t["expected_gpu"] == "6" and t["visible_devices_var"] == "ROCR_VISIBLE_DEVICES"
    assert expected_gpu({"visible_devices": ["0", "1"], "local_rank": 9}) is None
    assert topology_from_env({}) == {}


def test_merge_process_ranks_and_environ():
    ev = {"gpus": [{"index": 2, "procs": [{"pid": 11, "rank": 1, "local_rank": 1}]},
                   {"index": 1, "procs": [{"pid": 10, "rank": 0, "local_rank": 0}]}]}
    t = merge_process_ranks({"rank": 0}, ev)
    assert [e["gpu"] for e in t["rank_map"]] == [1, 2]
    env = rank_env_from_environ(["RANK=3", "PATH=/bin", "LOCAL_RANK=1", "HIP_VISIBLE_DEVICES=1"])
    assert env == {"RANK": "3", "LOCAL_RANK": "1", "HIP_VISIBLE_DEVICES": "1"}


def test_xgmi_link_down_and_ecc_are_gpu_faults():
    """A rank whose GPU lost xGMI links (RCCL transport) or took an uncorrectable ECC error
    fails as a GPU fault, not a plain error; the trace carries the link state."""
    from nexus_supervisor_amd.classify import Classifier, render_trace
    from nexus_supervisor_amd.config.schema import LabelConfig
    from nexus_supervisor_amd.gpu.telemetry import FakeTelemetry, pod_evidence_provider
    from nexus_supervisor_amd.models.decisions import FailureClass
    from nexus_supervisor_amd.testing.seed import make_pod

    labels = LabelConfig()
    for gpu, inject, expect in ((5, lambda t: t.set_xgmi(5, total=7, down=2), "XGMI_LINK_DOWN"),
                                (2, lambda t: t.set_ecc(2, uncorrectable=3), "ECC_UNCORRECTABLE")):
        tel = FakeTelemetry(n_gpus=8)
        inject(tel)
        tel.set_xgmi(0, total=7, down=0)  # healthy GPU: no event
        c = Classifier(labels)
        c.evidence_provider = pod_evidence_provider(tel)
        env = {"LOCAL_RANK": str(gpu), "RANK": str(gpu), "WORLD_SIZE": "8", "HIP_VISIBLE_DEVICES": "0,1,2,3,4,5,6,7"}
        pod = make_pod(f"run-{gpu}", labels, env=env, gpus=1, rv="2", status={
            "phase": "Failed", "containerStatuses": [{"name": "algorithm", "restartCount": 0, "state": {"terminated": {
                "reason": "Error", "exitCode": 1,
                "message": "RuntimeError: NCCL Error 6: remote process exited or there was a network error"}}}]})
        res = c.classify_pod(pod)
        assert len(res) == 1 and res[0].failure_class == FailureClass.GPU_FAULT, res
        assert expect in res[0].run_status_trace or expect in (res[0].reason or "")
        trace = json.loads(render_trace(res[0]))
        g = trace["gpu"]["gpus"][0]
        assert g["index"] == gpu and any(e["type"] == expect for e in g["events"])
        if expect == "XGMI_LINK_DOWN":  # the link state is stated once, in the fabric summary
            xg = trace["topology"]["xgmi"]["per_gpu"][0]
            assert xg["gpu"] == 5 and xg["ports_down"] == 2 and xg["ports_total"] == 7 and xg["ports_up"] == 5
        assert not [e for e in tel.snapshot()[0]["events"]]


def test_oom_keyword_prefilter_matches_full_pattern_scan():
    """The literal-keyword prefilter never hides a signature the regex lists would find."""
    from hypothesis import given, settings, strategies as st

    from nexus_supervisor_amd.gpu import oom as O

    def full(patterns, text):
        for p in patterns:
            m = p.search(text)
            if m:
                return m.group(0)
        return None

    fragments = ["hipErrorOutOfMemory", "HIP out of memory", "CUDA OUT OF MEMORY", "OutOfMemoryError", "hipMallocManaged",
                 " failed", "RCCL", "NCCL", " out of memory", "HSA_STATUS_ERROR_OUT_OF_RESOURCES", "GPU", "MemoryError",
                 "std::bad_alloc", "Cannot allocate memory", "Memory cgroup", "OOMKilled", "RESOURCE_EXHAUSTED: ",
                 "Out of memory while trying to allocate", "Back-off pulling image", " ", "\n", "x"]

    @settings(max_examples=400, deadline=None)
    @given(st.lists(st.sampled_from(fragments), max_size=8).map("".join))
    def check(text):
        assert O.hbm_signature(text) == full(O.HBM_PATTERNS, text)
        assert O.host_signature(text) == full(O.HOST_PATTERNS, text)

    check()


def test_peak_series_matches_a_scan():
    """The mirrored telemetry's window peak (block maxima + bisect) equals a full scan."""
    import random

    from nexus_supervisor_amd.gpu.telemetry import _PeakSeries

    rng = random.Random(0)
    s, data, t = _PeakSeries(), [], 0.0
    for _ in range(2000):
        t += rng.random()
        data.append((t, rng.randrange(1000)))
    s.extend(data[:1000])
    s.extend(data[1000:])
    s.extend([(1.0, 5000)])  # out of order: ignored
    for _ in range(500):
        a = rng.uniform(-5, t + 5)
        b = rng.uniform(a, t + 5)
        assert s.peak(a, b) == max((v for ts, v in data if a <= ts <= b), default=0)
    s.trim(t / 2)
    assert s.t[0] <= t / 2 and len(s) < len(data)
    assert s.peak(t / 2, t) == max(v for ts, v in data if t / 2 <= ts <= t)


def test_unmatched_pods_share_one_snapshot_evidence_matched_pods_get_their_own():
    """Pods with no process on any GPU get the expected devices' records of the current
    snapshot — built once per snapshot and shared (each with its own pod UID); a pod whose
    processes the monitor matched by cgroup UID gets its own records with them."""
    from nexus_supervisor_amd.config.schema import LabelConfig
    from nexus_supervisor_amd.gpu.telemetry import FakeTelemetry, pod_evidence_provider
    from nexus_supervisor_amd.testing.seed import make_pod

    labels = LabelConfig()
    tel = FakeTelemetry(n_gpus=8)
    tel.set_vram(3, 200_000)
    env = {"LOCAL_RANK": "3", "RANK": "3", "WORLD_SIZE": "8", "HIP_VISIBLE_DEVICES": "0,1,2,3,4,5,6,7"}
    a, b, c = (make_pod(f"run-{x}", labels, env=env, gpus=1, node="n1") for x in "abc")
    tel.add_process(4242, 3, vram_bytes=1 << 30, pod_uid=c["metadata"]["uid"])
    prov = pod_evidence_provider(tel)
    ea, eb, ec = prov(a), prov(b), prov(c)
    assert ea["pod_uid"] == a["metadata"]["uid"] and eb["pod_uid"] == b["metadata"]["uid"]
    assert ea["gpus"] is eb["gpus"] and ea["gpus"][0]["index"] == 3 and not ea["gpus"][0]["matched"]
    assert ec["gpus"] is not ea["gpus"] and ec["gpus"][0]["matched"] and ec["gpus"][0]["procs"][0]["pid"] == 4242
