"""A GPU filled by someone else (VERDICT r5 missing #3).

Zombie or leaked HBM from a previous tenant is a common MI355X failure: the pod's own
allocator holds a few MiB while another process holds the 288 GB.  The trace must name
the holder (pid, pod or ``host``, VRAM) and keep the stage the evidence gives; a crash at
HIP init on such a GPU (exit 139, no text) records the GPU as occupied instead of no GPU.
The reference writes a plain fatal error and never looks at the GPU
(``/root/reference/services/supervisor.go:194-204``)."""
import json

from nexus_supervisor_amd.config import load_config
from nexus_supervisor_amd.gpu import oom
from nexus_supervisor_amd.gpu.telemetry import FakeTelemetry, evidence_for, pod_evidence_provider
from nexus_supervisor_amd.models import LifecycleStage as S
from nexus_supervisor_amd.store.memory import MemoryStore
from nexus_supervisor_amd.testing.inproc import InProcCluster
from nexus_supervisor_amd.testing.seed import ALGORITHM, make_job, make_pod, seed_rows

GIB = 1 << 30
RUNNING_ROW = seed_rows()[1]
RID = RUNNING_ROW.id
ENV = {"RANK": "0", "WORLD_SIZE": "1", "LOCAL_RANK": "0", "HIP_VISIBLE_DEVICES": "0"}
TORCH_OOM = ("torch.OutOfMemoryError: HIP out of memory. Tried to allocate 2.00 GiB. GPU 0 has a total capacity of "
             "287.98 GiB of which 78.00 MiB is free. Of the allocated memory 76.50 MiB is allocated by PyTorch")


def _cfg():
    return load_config(path=None, env={}, overrides={"cql-store-type": "memory", "rate-limit-elements-per-second": 0,
                                                     "resync-period": "0s", "rules": {"job-pod-settle": "0s"}})


def _filled_gpu():
    tel = FakeTelemetry(n_gpus=8)
    total_mb = tel.devices()[0]["vram_total_mb"]
    tel.add_process(4242, 0, vram_bytes=287 * GIB, name="python3")            # the leaked tenant (no pod)
    tel.add_process(5151, 0, vram_bytes=1 * GIB, pod_uid="other-pod-uid")     # a small neighbour pod
    tel.set_vram(0, int(total_mb * 0.995))
    return tel


def test_evidence_lists_the_holders_and_the_verdict_flags_foreign_occupancy():
    tel = _filled_gpu()
    tel.add_process(777, 0, vram_bytes=76 << 20, pod_uid="pod-uid-mine")
    ev = evidence_for(tel, pod_uid="pod-uid-mine", gpu_indices=[0], lookback=60)
    g = ev["gpus"][0]
    assert [h["pid"] for h in g["holders"]] == [4242, 5151]
    assert g["holders"][0] == {"pid": 4242, "vram_bytes": 287 * GIB, "owner": "host", "name": "python3", "alive": True}
    assert g["holders"][1]["owner"] == "other-pod-uid"
    v = oom.analyze([TORCH_OOM], [{"container": "algorithm", "exitCode": 1, "reason": "Error"}], ev, "0")
    assert v.kind == "hbm"  # the stage is what the evidence says
    assert v.foreign["gpu"] == 0 and v.foreign["holders"][0]["pid"] == 4242
    assert v.as_dict()["foreign_occupancy"] is True
    assert any(s.startswith("foreign occupancy: GPU 0 was 99% full") and "pid 4242 (host) 287.0 GiB" in s
               for s in v.signals), v.signals
    # the pod's own processes filled it: no foreign occupancy
    tel2 = FakeTelemetry(n_gpus=8)
    tel2.add_process(777, 0, vram_bytes=286 * GIB, pod_uid="pod-uid-mine")
    tel2.set_vram(0, int(tel2.devices()[0]["vram_total_mb"] * 0.99))
    ev2 = evidence_for(tel2, pod_uid="pod-uid-mine", gpu_indices=[0], lookback=60)
    assert oom.analyze([TORCH_OOM], [{"container": "algorithm", "exitCode": 1}], ev2, "0").foreign is None


def _run(tel, updates, objects):
    import asyncio

    cfg = _cfg()
    store = MemoryStore([RUNNING_ROW])

    async def go():
        c = InProcCluster(cfg, store, objects)
        c.supervisor.classifier.evidence_provider = pod_evidence_provider(tel, lookback=60)
        await c.start()
        for etype, obj in updates:
            c.push(obj, etype)
            assert await c.settle(5)
        await c.stop()

    asyncio.run(go())
    return store.get(ALGORITHM, RID)


def test_hbm_oom_on_a_gpu_someone_else_filled_names_the_holder():
    cfg = _cfg()
    tel = _filled_gpu()
    pod = make_pod(RID, cfg.labels, env=ENV, gpus=1, node="mi355x-009")
    failed = make_pod(RID, cfg.labels, env=ENV, gpus=1, node="mi355x-009", rv="5", status={
        "phase": "Failed", "containerStatuses": [{"name": "algorithm", "restartCount": 0, "state": {
            "terminated": {"reason": "Error", "exitCode": 1, "message": TORCH_OOM}}}]})
    row = _run(tel, [("MODIFIED", failed)], [pod, make_job(RID, cfg.labels)])
    assert row.lifecycle_stage == S.FAILED
    t = json.loads(row.algorithm_failure_details)
    assert t["class"] == "hbm-oom"
    fo = t["foreign_occupancy"]
    assert fo["gpu"] == 0 and fo["holders"][0]["pid"] == 4242 and fo["holders"][0]["vram_bytes"] == 287 * GIB
    assert fo["holders"][0]["owner"] == "host" and fo["own_peak_bytes"] == 0
    assert t["gpu"]["gpus"][0]["holders"][0]["pid"] == 4242


def test_crash_at_hip_init_on_a_full_gpu_records_it_occupied():
    """Exit 139 with no text on a GPU someone else filled: no OOM is claimed and the stage
    stays the Job's (DEADLINE_EXCEEDED for BackoffLimitExceeded, as the reference), but the
    trace names GPU 0 as occupied and its holder."""
    cfg = _cfg()
    tel = _filled_gpu()
    pod = make_pod(RID, cfg.labels, env=ENV, gpus=1, node="mi355x-009")
    crashed = make_pod(RID, cfg.labels, env=ENV, gpus=1, node="mi355x-009", rv="5", status={
        "phase": "Failed", "containerStatuses": [{"name": "algorithm", "restartCount": 0, "state": {
            "terminated": {"reason": "Error", "exitCode": 139, "message": ""}}}]})
    job_failed = make_job(RID, cfg.labels, rv="7", conditions=[
        {"type": "Failed", "status": "True", "reason": "BackoffLimitExceeded", "message": "backoff limit"}])
    row = _run(tel, [("MODIFIED", crashed), ("MODIFIED", job_failed)], [pod, make_job(RID, cfg.labels)])
    assert row.lifecycle_stage == S.DEADLINE_EXCEEDED
    t = json.loads(row.algorithm_failure_details)
    assert "oom" not in t
    assert t["foreign_occupancy"]["gpu"] == 0 and t["foreign_occupancy"]["holders"][0]["owner"] == "host"
    assert t["gpu"]["gpus"][0]["index"] == 0
