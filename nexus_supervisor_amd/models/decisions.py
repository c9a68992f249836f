"""Classifier output types.

``DecisionAction`` and ``RunStatusAnalysisResult`` mirror
``/root/reference/services/supervisor.go:49-66``.  This build adds evidence
fields (failure class, GPU attribution, rank topology, stage timestamps) that
end up in the trace column (``algorithm_failure_details``).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Dict, Optional


class DecisionAction:
    TO_FAIL_STUCK_IN_PENDING = "ToFailStuckInPending"
    TO_FAIL_FATAL_ERROR = "ToFailFatalError"
    TO_FAIL_DEADLINE_EXCEEDED = "ToFailDeadlineExceeded"
    TO_RUNNING = "ToRunning"

    ALL = (TO_FAIL_STUCK_IN_PENDING, TO_FAIL_FATAL_ERROR, TO_FAIL_DEADLINE_EXCEEDED, TO_RUNNING)
    FAILING = (TO_FAIL_STUCK_IN_PENDING, TO_FAIL_FATAL_ERROR, TO_FAIL_DEADLINE_EXCEEDED)


class FailureClass:
    """Finer-grained failure taxonomy recorded in the trace (north star)."""

    NONE = ""
    SCHEDULING = "scheduling"            # FailedCreate / pod Failed / unschedulable
    IMAGE_PULL = "image-pull"            # ErrImagePull / ImagePullBackOff
    CRASH_LOOP = "crash-loop"            # CrashLoopBackOff
    HOST_OOM = "host-oom"                # cgroup OOMKilled, exit 137
    HBM_OOM = "hbm-oom"                  # HIP out-of-memory on an MI355X (288 GB HBM3E)
    GPU_FAULT = "gpu-fault"              # VM fault / GPU reset / xGMI / ECC
    EVICTED = "evicted"                  # kubelet eviction / preemption
    DEADLINE = "deadline"                # activeDeadlineSeconds
    BACKOFF_LIMIT = "backoff-limit"      # BackoffLimitExceeded
    FATAL = "fatal"                      # PodFailurePolicy / other fatal exit
    CONFIG = "config"                    # CreateContainerConfigError
    COLLECTIVE = "collective"            # every failed rank shows only RCCL / collective errors
    # the node's kubelet refused the pod at admission because of its GPUs: the device
    # plugin could not allocate (UnexpectedAdmissionError), OutOf<gpu-resource>, or the
    # topology manager could not align the GPUs (TopologyAffinityError)
    GPU_ADMISSION = "gpu-admission"
    ADMISSION = "admission"              # any other kubelet admission rejection (OutOfcpu, NodeAffinity, ...)


@dataclass
class RunStatusAnalysisResult:
    action: str
    run_status_message: str
    run_status_trace: str
    object_uid: str = ""
    object_kind: str = ""
    request_id: str = ""
    algorithm: str = ""
    # ---- extensions ----
    reason: str = ""
    failure_class: str = FailureClass.NONE
    evidence: Dict[str, Any] = field(default_factory=dict)
    # monotonic timestamps per pipeline stage (watch-receive → classify → ... → cql-ack)
    stamps: Dict[str, float] = field(default_factory=dict)
    event_uid: str = ""
    attempts: int = 0
    pending_delete: bool = False  # a concurrent Job DELETE failed; retry must still delete
    answered: int = 0  # the attempt (``attempts``) in which the checkpoint store last answered
    # deferred enrichment (Classifier.lazy_enrich): (pods, texts, verdict) until the decision
    # is actually written — duplicates of a decided run are never enriched
    pending_enrich: Any = None

    @property
    def key(self):
        return (self.algorithm, self.request_id)

    def has_evidence(self) -> bool:
        return bool(self.evidence) or bool(self.failure_class)


@dataclass
class Decision:
    """What :func:`superviseAction`-equivalent actuation did (returned for tests/metrics)."""

    result: RunStatusAnalysisResult
    outcome: str  # applied | skipped-finished | skipped-missing | deleted-only | dead-letter
    new_stage: Optional[str] = None
    job_deleted: bool = False
