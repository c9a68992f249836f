"""HBM-OOM needs a GPU.

A CPU-only pod (no ``amd.com/gpu`` request, no GPU process of its own) whose JVM runs out
of heap must never be written as "ran out of GPU memory (HBM)": the HBM pattern is
anchored to torch / HIP words, the JVM / numpy / C++ / Go allocation failures are host
OOMs, and every HBM verdict is gated on GPU involvement.  The reference writes a plain
fatal error for these and never claims a device
(``/root/reference/services/supervisor.go:194-204,310-335``).
"""
import asyncio
import json

import pytest

from nexus_supervisor_amd.app import Application
from nexus_supervisor_amd.classify import Classifier
from nexus_supervisor_amd.config import load_config
from nexus_supervisor_amd.config.schema import GpuConfig, LabelConfig
from nexus_supervisor_amd.gpu import oom
from nexus_supervisor_amd.kube.client import KubeClient, KubeConfig
from nexus_supervisor_amd.models.decisions import FailureClass
from nexus_supervisor_amd.store.memory import MemoryStore
from nexus_supervisor_amd.testing.fake_apiserver import FakeApiServer
from nexus_supervisor_amd.testing.seed import ALGORITHM, make_job, make_pod, seed_rows

JAVA = 'Exception in thread "main" java.lang.OutOfMemoryError: Java heap space'
NUMPY = ("numpy.core._exceptions._ArrayMemoryError: Unable to allocate 3.00 GiB for an array with shape "
         "(402653184,) and data type float64")
NUMPY_MSG_ONLY = "MemoryError: Unable to allocate 3.00 GiB for an array with shape (402653184,) and data type float64"
BAD_ALLOC = "terminate called after throwing an instance of 'std::bad_alloc'\n  what():  std::bad_alloc"
GO = "fatal error: runtime: out of memory"
NODE = "FATAL ERROR: Reached heap limit Allocation failed - JavaScript heap out of memory"
TORCH = ("torch.OutOfMemoryError: HIP out of memory. Tried to allocate 20.00 GiB. GPU 0 has a total capacity of "
         "287.98 GiB of which 3.12 GiB is free.")
HIP_RT = "hipMalloc failed: hipErrorOutOfMemory (out of memory)"

HOST_TEXTS = [JAVA, NUMPY, NUMPY_MSG_ONLY, BAD_ALLOC, GO, NODE]


@pytest.mark.parametrize("text", HOST_TEXTS, ids=["java", "numpy", "numpy-msg", "bad_alloc", "go", "node"])
def test_host_allocation_texts_are_host_oom(text):
    assert oom.host_signature(text)
    assert not oom.hbm_signature(text), text
    for involved in (True, False, None):
        v = oom.analyze([text], [{"container": "c", "exitCode": 1, "reason": "Error"}], gpu_involved=involved)
        assert v.kind == "host", (text, involved, v.signals)


@pytest.mark.parametrize("text", [TORCH, HIP_RT])
def test_hip_texts_need_a_gpu(text):
    term = [{"container": "c", "exitCode": 1, "reason": "Error"}]
    assert oom.analyze([text], term, gpu_involved=True).kind == "hbm"
    assert oom.analyze([text], term, gpu_involved=None).kind == "hbm"  # pod unknown: anchored words count
    v = oom.analyze([text], term, gpu_involved=False)
    assert v.kind is None and v.gpu_index is None
    assert any("on a pod with no GPU" in s for s in v.signals), v.signals


def test_bare_outofmemoryerror_is_not_hbm():
    assert oom.hbm_signature("java.lang.OutOfMemoryError: GC overhead limit exceeded") is None
    assert oom.hbm_signature("OutOfMemoryError") is None
    assert oom.hbm_signature("torch.cuda.OutOfMemoryError: HIP out of memory")
    assert oom.hbm_signature("torch.OutOfMemoryError: CUDA out of memory")


def test_gpu_involved_rule():
    assert oom.gpu_involved(1, None)
    assert not oom.gpu_involved(0, None)
    assert not oom.gpu_involved(0, {"gpus": [{"index": 0, "vram_peak_mb": 290000, "procs": []}]})
    assert oom.gpu_involved(0, {"gpus": [{"index": 0, "matched": True}]})  # reached /dev/kfd without a request


def _failed(pod, message, reason="Error", code=1):
    p = json.loads(json.dumps(pod))
    p["status"] = {"phase": "Failed", "containerStatuses": [
        {"name": "algorithm", "restartCount": 0,
         "state": {"terminated": {"reason": reason, "exitCode": code, "message": message}}}]}
    p["metadata"]["resourceVersion"] = "2"
    return p


@pytest.mark.parametrize("text", HOST_TEXTS + [TORCH, HIP_RT])
def test_cpu_only_pod_is_never_hbm_oom(text):
    """Table: a pod with no GPU request, each text in its termination message."""
    labels = LabelConfig()
    pod = _failed(make_pod("cpu", labels, gpus=0), text)
    out = Classifier(labels, gpu=GpuConfig()).classify_pod(pod, allow_log_fetch=True)
    for r in out:
        assert r.failure_class != FailureClass.HBM_OOM, (text, r.evidence)
        assert "GPU memory" not in r.run_status_message
    if text in HOST_TEXTS:
        assert out and out[0].failure_class == FailureClass.HOST_OOM


def test_cpu_only_pod_with_full_gpu_evidence_is_not_hbm():
    """A previous tenant's full GPU in the evidence of a CPU-only pod on a GPU node."""
    labels = LabelConfig()
    pod = _failed(make_pod("cpu2", labels, gpus=0), TORCH)
    gev = {"source": "fake", "gpus": [{"index": 0, "vram_total_mb": 294896, "vram_peak_mb": 294000, "procs": [],
                                       "events": [{"type": "VMFAULT"}]}]}
    pod["metadata"]["annotations"] = {"nexus.amd.com/gpu-evidence": json.dumps(gev)}
    out = Classifier(labels, gpu=GpuConfig()).classify_pod(pod)
    assert all(r.failure_class not in (FailureClass.HBM_OOM, FailureClass.GPU_FAULT) for r in out), out


def test_gpu_pod_with_torch_text_is_hbm():
    labels = LabelConfig()
    pod = _failed(make_pod("gpu", labels, gpus=1, env={"LOCAL_RANK": "0", "HIP_VISIBLE_DEVICES": "0"}), TORCH)
    r = Classifier(labels, gpu=GpuConfig()).classify_pod(pod)[0]
    assert r.failure_class == FailureClass.HBM_OOM and r.evidence["oom"]["gpu_logical_index"] == 0
    pod = _failed(make_pod("gpu2", labels, gpus=1), JAVA)
    assert Classifier(labels, gpu=GpuConfig()).classify_pod(pod)[0].failure_class == FailureClass.HOST_OOM


def _app_cfg(**rules):
    return load_config(path=None, env={}, overrides={"cql-store-type": "memory", "rate-limit-elements-per-second": 0,
                                                     "resync-period": "0s", "rules": rules})


def test_cpu_pod_oom_end_to_end_counts_no_gpu_failure(arun):
    """A CPU-only pod dies of a JVM heap OOM, a GPU pod of a torch HBM-OOM: the CPU row is
    host-oom with the host message, and ``gpu_failures`` counts only the GPU pod."""
    async def go():
        api = FakeApiServer(bookmark_interval=0.1)
        url = await api.start()
        rows = seed_rows()
        cpu_row, gpu_row = rows[1], rows[2]
        cfg = _app_cfg()
        api.create(make_pod(cpu_row.id, cfg.labels, gpus=0, status={"phase": "Running"}))
        api.create(make_pod(gpu_row.id, cfg.labels, gpus=1, env={"LOCAL_RANK": "0", "HIP_VISIBLE_DEVICES": "0"},
                            status={"phase": "Running"}))
        for row in (cpu_row, gpu_row):
            api.create(make_job(row.id, cfg.labels))
        store = MemoryStore([cpu_row, gpu_row])
        app = Application(cfg, kube=KubeClient(KubeConfig(url)), store=store)
        await app.start()
        await app.factory.wait_for_cache_sync(5)
        api.update(_failed(api.get("Pod", "nexus", f"{cpu_row.id}-acdey"), JAVA))
        api.update(_failed(api.get("Pod", "nexus", f"{gpu_row.id}-acdey"), TORCH))
        for _ in range(200):
            if all(store.get(ALGORITHM, r.id).lifecycle_stage == "FAILED" for r in (cpu_row, gpu_row)):
                break
            await asyncio.sleep(0.02)
        cpu = store.get(ALGORITHM, cpu_row.id)
        assert cpu.lifecycle_stage == "FAILED"
        assert "GPU" not in cpu.algorithm_failure_cause, cpu.algorithm_failure_cause
        t_cpu = json.loads(cpu.algorithm_failure_details)
        assert t_cpu["class"] == "host-oom" and t_cpu["oom"]["kind"] == "host", t_cpu
        gpu = store.get(ALGORITHM, gpu_row.id)
        assert json.loads(gpu.algorithm_failure_details)["class"] == "hbm-oom"
        counted = app.metrics.counters.get("gpu_failures", {})
        assert sum(counted.values()) == 1, counted
        assert all(dict(k)["class"] == "hbm-oom" for k in counted), counted
        await app.stop()
        await api.stop()

    arun(go(), timeout=30)


# Runtime-check and math-library wordings a ROCm job prints when the GPU is full: torch's
# C10_HIP_CHECK (HIP context / hipBLAS handle / RCCL cannot allocate), the HIP enum, and
# the hipBLAS / cuBLAS / rocBLAS / MIOpen allocation-failure statuses.
LIB_TEXTS = {
    "hip-check": "RuntimeError: HIP error: out of memory\nHIP kernel errors might be asynchronously reported",
    "cuda-check": "RuntimeError: CUDA error: out of memory\nCompile with `TORCH_USE_CUDA_DSA` to enable",
    "hip-enum": "hipMemcpy returned hipErrorMemoryAllocation",
    "hipblas": "RuntimeError: HIPBLAS_STATUS_ALLOC_FAILED when calling `hipblasCreate(handle)`",
    "cublas": "RuntimeError: CUDA error: CUBLAS_STATUS_ALLOC_FAILED when calling `cublasCreate(handle)`",
    "hipblaslt": "hipBLASLt error: HIPBLASLT_STATUS_ALLOC_FAILED",
    "rocblas": "rocBLAS error: rocblas_status_memory_error from rocblas_gemm_ex",
    "miopen": "MIOpen Error: miopenStatusAllocFailed in convolution workspace",
}


@pytest.mark.parametrize("name", sorted(LIB_TEXTS))
def test_hip_runtime_and_library_oom_texts(name):
    text = LIB_TEXTS[name]
    assert oom.hbm_signature(text), name
    assert not oom.host_signature(text) or name in ("hip-check", "cuda-check"), name
    term = [{"container": "c", "exitCode": 1, "reason": "Error"}]
    assert oom.analyze([text], term, gpu_involved=True).kind == "hbm", name
    # a CPU-only pod with the same words stays non-HBM
    v = oom.analyze([text], term, gpu_involved=False)
    assert v.kind != "hbm", (name, v.signals)


def test_torch_default_cpu_allocator_is_host_oom():
    text = ("RuntimeError: [enforce fail at alloc_cpu.cpp:117] data. DefaultCPUAllocator: not enough memory: "
            "you tried to allocate 68719476736 bytes.")
    assert oom.host_signature(text)
    assert not oom.hbm_signature(text)
    for involved in (True, False, None):
        v = oom.analyze([text], [{"container": "c", "exitCode": 1, "reason": "Error"}], gpu_involved=involved)
        assert v.kind == "host", (involved, v.signals)
