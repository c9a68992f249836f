"""Multi-rank root cause (gpu/collective.py): the rank that ran out of HBM is the culprit,
the ranks that died in their next all-reduce are its collateral, and the OOM's GPU is
mapped through the culprit's own device env — not the last pod's."""
import json

from nexus_supervisor_amd.classify import Classifier
from nexus_supervisor_amd.classify.classifier import render_trace
from nexus_supervisor_amd.config.schema import LabelConfig
from nexus_supervisor_amd.gpu.collective import collective_signature
from nexus_supervisor_amd.models.decisions import FailureClass as F
from nexus_supervisor_amd.testing.seed import make_event, make_job, make_pod

LABELS = LabelConfig()
RUN = "ddp-run"
WATCHDOG = ("[rank{r}]:[E ProcessGroupNCCL.cpp:616] [Rank {r}] Watchdog caught collective operation timeout: "
            "WorkNCCL(SeqNum=1822, OpType=ALLREDUCE, NumelIn=2048, NumelOut=2048, Timeout(ms)=600000) ran for "
            "600012 milliseconds before timing out.")
HIP_OOM = ("torch.OutOfMemoryError: HIP out of memory. Tried to allocate 16.00 GiB. GPU 0 has a total capacity of "
           "287.98 GiB of which 1.02 GiB is free.")


class _Lookup:
    def __init__(self, job, pods):
        self.job, self.pods = job, pods

    def get(self, kind, name):
        return self.job if kind == "Job" and name == RUN else None

    def pods_of_job(self, name):
        return list(self.pods) if name == RUN else []


def _rank_pod(r, message, exit_code=1, finished="2026-10-17T10:00:00Z", reason="Error"):
    """One pod per rank (indexed Job), rank r pinned to physical GPU r via HIP_VISIBLE_DEVICES."""
    return make_pod(RUN, LABELS, suffix=f"r{r}", gpus=1, rv="5",
                    env={"RANK": str(r), "WORLD_SIZE": "4", "LOCAL_RANK": "0", "HIP_VISIBLE_DEVICES": str(r)},
                    status={"phase": "Failed", "containerStatuses": [{"name": "algorithm", "restartCount": 0, "state": {
                        "terminated": {"reason": reason, "exitCode": exit_code, "message": message,
                                       "finishedAt": finished}}}]})


def test_collective_signatures():
    assert "Watchdog caught collective operation timeout" in collective_signature(WATCHDOG.format(r=1))
    assert collective_signature("RuntimeError: NCCL communicator was aborted on rank 2.")
    assert collective_signature("torch.distributed.DistBackendError: NCCL error in: ... ncclRemoteError: "
                                "A call failed possibly due to a network error or a remote process exiting prematurely.")
    assert collective_signature("plain ValueError: bad shape") is None
    assert collective_signature(HIP_OOM) is None


def test_hbm_oom_rank_is_the_culprit_and_maps_its_own_gpu():
    pods = [_rank_pod(0, WATCHDOG.format(r=0), finished="2026-10-17T10:10:01Z"),
            _rank_pod(1, WATCHDOG.format(r=1), finished="2026-10-17T10:10:02Z"),
            _rank_pod(2, HIP_OOM, finished="2026-10-17T10:00:00Z"),
            _rank_pod(3, WATCHDOG.format(r=3), finished="2026-10-17T10:10:00Z")]
    job = make_job(RUN, LABELS)
    ev = make_event("Job", RUN, "BackoffLimitExceeded", "Job has reached the specified backoff limit")
    status, [r] = Classifier(LABELS).classify_event(ev, _Lookup(job, pods))
    assert r.failure_class == F.HBM_OOM
    # torch's "GPU 0" is rank 2's only visible device: physical GPU 2 (the last pod would say 3)
    assert r.evidence["oom"]["gpu_index"] == 2 and r.evidence["oom"]["gpu_logical_index"] == 0
    ranks = r.evidence["ranks"]
    assert ranks["culprit"]["pod"] == f"{RUN}-r2" and ranks["culprit"]["kind"] == "hbm-oom" and ranks["culprit"]["rank"] == 2
    assert ranks["failed"] == 4 and ranks["collateral"] == 3 and not ranks["all_collective"]
    assert [p["rank"] for p in ranks["pods"]] == [3, 0, 1]  # collateral in the order it failed
    doc = json.loads(render_trace(r))
    assert doc["class"] == "hbm-oom" and doc["ranks"]["culprit"]["rank"] == 2


def test_all_ranks_collective_is_a_collective_failure():
    pods = [_rank_pod(r, WATCHDOG.format(r=r), finished=f"2026-10-17T10:10:0{r}Z") for r in range(4)]
    job = make_job(RUN, LABELS)
    ev = make_event("Job", RUN, "BackoffLimitExceeded", "Job has reached the specified backoff limit")
    _status, [r] = Classifier(LABELS).classify_event(ev, _Lookup(job, pods))
    assert r.failure_class == F.COLLECTIVE and "oom" not in r.evidence
    assert r.evidence["ranks"]["all_collective"] and r.evidence["ranks"]["culprit"]["rank"] == 0


def test_own_error_beats_collateral_and_single_pod_jobs_have_no_rank_block():
    pods = [_rank_pod(0, WATCHDOG.format(r=0), finished="2026-10-17T10:00:00Z"),
            _rank_pod(1, "Traceback ... ValueError: NaN loss", finished="2026-10-17T10:05:00Z")]
    _s, [r] = Classifier(LABELS).classify_event(make_event("Job", RUN, "BackoffLimitExceeded", "limit"),
                                                _Lookup(make_job(RUN, LABELS), pods))
    assert r.evidence["ranks"]["culprit"]["rank"] == 1 and r.evidence["ranks"]["culprit"]["kind"] == "error"
    _s, [r1] = Classifier(LABELS).classify_event(make_event("Job", RUN, "BackoffLimitExceeded", "limit"),
                                                 _Lookup(make_job(RUN, LABELS), pods[:1]))
    assert "ranks" not in r1.evidence


def test_trace_with_many_ranks_stays_bounded():
    pods = [_rank_pod(r, WATCHDOG.format(r=r) * 3, finished=f"2026-10-17T10:{r:02d}:00Z") for r in range(64)]
    _s, [r] = Classifier(LABELS).classify_event(make_event("Job", RUN, "BackoffLimitExceeded", "limit"),
                                                _Lookup(make_job(RUN, LABELS), pods))
    assert r.evidence["ranks"]["pods_total"] == 64 and len(r.evidence["ranks"]["pods"]) == 7
    out = render_trace(r, max_bytes=2048)
    assert len(out.encode()) <= 2048 and json.loads(out)["class"] == "collective"


def test_xgmi_link_down_rank_makes_a_gpu_fault():
    """A rank whose node agent saw its xGMI link go down is the culprit of the others'
    collective timeouts: the Job-level decision is a GPU fault, not a generic one."""
    ev = {"source": "agent", "gpus": [{"index": 1, "vram_total_mb": 294896, "vram_peak_mb": 1000, "procs": [],
                                       "events": [{"type": "XGMI_LINK_DOWN", "t": 1.0, "message": "1/7 xGMI links down"}]}]}
    bad = _rank_pod(1, "RuntimeError: NCCL communicator was aborted", finished="2026-10-17T10:00:05Z")
    bad["metadata"]["annotations"] = {"nexus.amd.com/gpu-evidence": json.dumps(ev)}
    pods = [_rank_pod(0, WATCHDOG.format(r=0), finished="2026-10-17T10:00:01Z"), bad]
    _s, [r] = Classifier(LABELS).classify_event(make_event("Job", RUN, "BackoffLimitExceeded", "limit"),
                                                _Lookup(make_job(RUN, LABELS), pods))
    assert r.failure_class == F.GPU_FAULT
    assert r.evidence["ranks"]["culprit"]["rank"] == 1 and r.evidence["ranks"]["culprit"]["kind"] == "gpu-fault"
    assert r.evidence["ranks"]["culprit"]["collective"].startswith("NCCL communicator was aborted")
