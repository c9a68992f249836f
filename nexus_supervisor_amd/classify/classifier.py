"""Failure-reason classifier: K8s Events / Pod status / Job status → decisions.

Three rule sets:

* **R-EVT** — the reference event table, byte-exact
  (``/root/reference/services/supervisor.go:137-259``; :mod:`.reference_rules`).
* **R-POD / R-JOB** — status-based rules the reference lacks (it registers no
  Pod/Job handlers, ``supervisor.go:124-128``): OOMKilled, HBM-OOM, Evicted,
  ImagePullBackOff/ErrImagePull, CreateContainerConfigError, CrashLoopBackOff,
  Unschedulable, and Job ``Failed`` conditions (so a lost Event — K8s events
  are best-effort — no longer loses the decision).
* **R-GPU** — every failing decision is enriched with the rank topology
  (:mod:`..gpu.topology`), node-agent GPU evidence (pod annotation) and the
  HBM-vs-host OOM verdict (:mod:`..gpu.oom`).

Everything here is pure and synchronous: it runs on the informer dispatch path
and never does I/O.
"""
from __future__ import annotations

import json
import re
import time
from collections import OrderedDict
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional, Tuple

from ..config.schema import GpuConfig, LabelConfig, RulesConfig
from ..gpu import collective, logtail
from ..gpu import oom as oom_mod
from ..gpu.telemetry import FAULT_EVENTS
from ..gpu.topology import merge_process_ranks, resolve_devices, topology_from_pod, xgmi_from_evidence
from ..models import kube
from ..models.decisions import DecisionAction as A
from ..models.decisions import FailureClass as F
from ..models.decisions import RunStatusAnalysisResult
from . import reference_rules as R

IGNORED = "ignored"        # not a Nexus run object / uninteresting kind
STALE = "stale"            # involved object not in cache (yet)
NOOP = "noop"              # Nexus event with a reason we do not act on
DECIDED = "decided"
EVIDENCE = "evidence"      # recorded for later enrichment, no decision

MSG_HOST_OOM = "Algorithm container was OOMKilled: host memory limit exceeded."
MSG_HBM_OOM = "Algorithm ran out of GPU memory (HBM) on an AMD Instinct GPU."
MSG_EVICTED = "Algorithm pod was evicted from its node."
MSG_IMAGE_PULL = "Unable to pull the algorithm container image."
MSG_CONFIG = "Unable to create the algorithm container - please review configuration and try again."
MSG_CRASH_LOOP = "Algorithm container is crash-looping."
MSG_UNSCHEDULABLE = "Algorithm pod could not be scheduled on the target cluster."
MSG_GPU_FAULT = "Algorithm hit a GPU fault."
MSG_GPU_ADMISSION = "Algorithm pod was rejected by its node: no healthy AMD Instinct GPU could be allocated to it."
MSG_ADMISSION = "Algorithm pod was rejected by its node at admission."

IMAGE_PULL_WAITING = ("ErrImagePull", "ImagePullBackOff", "InvalidImageName", "ErrImageNeverPull")
CONFIG_WAITING = ("CreateContainerConfigError", "CreateContainerError", "RunContainerError")
EVICTION_EVENT_REASONS = ("Evicted", "Preempted", "Preempting", "TaintManagerEviction")
NO_GPU_CLASSES = (F.IMAGE_PULL, F.CONFIG, F.SCHEDULING)
ADMISSION_CLASSES = (F.GPU_ADMISSION, F.ADMISSION)
# kubelet admission rejections recorded as pod Events (the OutOf<resource> ones are matched
# by prefix; event_reasons_read() lists the common resources for the watch hub's filter)
ADMISSION_EVENT_REASONS = ("UnexpectedAdmissionError", "TopologyAffinityError")
# the device manager's / resource fit's numbers in an admission message
_ALLOC_NUMS = re.compile(r"Requested:\s*(\d+),\s*Available:\s*(\d+)", re.I)
_FIT_NUMS = re.compile(r"requested:\s*(\d+),\s*used:\s*(\d+),\s*capacity:\s*(\d+)", re.I)
JOB_FAILED_CONDITION_REASONS = ("DeadlineExceeded", "BackoffLimitExceeded", "PodFailurePolicy",
                                "MaxFailedIndexesExceeded", "FailedIndexes")


class ObjectLookup:
    """What the classifier needs from the informer caches (namespace already bound)."""

    def get(self, kind: str, name: str) -> Optional[Dict[str, Any]]:  # pragma: no cover - interface
        raise NotImplementedError

    def pods_of_job(self, job_name: str) -> List[Dict[str, Any]]:  # pragma: no cover - interface
        return []


@dataclass
class EvidenceBook:
    """Bounded per-run memory of non-decisive observations (evictions, exit codes,
    unschedulable periods) used to enrich the eventual terminal decision."""

    capacity: int = 50_000
    _data: "OrderedDict[Tuple[str, str], List[Dict[str, Any]]]" = field(default_factory=OrderedDict)

    def add(self, key: Tuple[str, str], item: Dict[str, Any]) -> None:
        lst = self._data.get(key)
        if lst is None:
            lst = self._data[key] = []
            if len(self._data) > self.capacity:
                self._data.popitem(last=False)
        else:
            self._data.move_to_end(key)
        if item not in lst:
            lst.append(item)
            del lst[:-16]

    def get(self, key) -> List[Dict[str, Any]]:
        return list(self._data.get(key, ()))

    def pop(self, key) -> List[Dict[str, Any]]:
        return self._data.pop(key, [])

    def __len__(self):
        return len(self._data)


class Classifier:
    def __init__(self, labels: Optional[LabelConfig] = None, rules: Optional[RulesConfig] = None,
                 gpu: Optional[GpuConfig] = None, clock: Callable[[], float] = time.monotonic):
        self.labels = labels or LabelConfig()
        self.rules = rules or RulesConfig()
        self.gpu = gpu or GpuConfig()
        self.evidence = EvidenceBook()
        self.clock = clock
        # Live GPU evidence for pods without an agent annotation (supervisor co-located
        # with the GPUs, or a node agent in-process): pod -> evidence record or None.
        self.evidence_provider: Optional[Callable[[Dict[str, Any]], Optional[Dict[str, Any]]]] = None
        self.deferred = False
        # defer _enrich of failing decisions to finish() (the Supervisor turns it on)
        self.lazy_enrich = False
        # failed GPU pod whose OOM signature may only be in its container log: the
        # (container, previous) instances to fetch (set by classify_pod, see log_cache)
        self.deferred_log: List[Dict[str, Any]] = []
        # pod uid -> {(container, restart): log-tail record} fetched by the supervisor
        # (pods/log API; logtail.py) — one read per container instance
        self.log_cache: "OrderedDict[str, Dict[Tuple[str, Optional[int]], Dict[str, Any]]]" = OrderedDict()
        self._ctx_cache: Dict[Tuple[str, str, bool], Tuple[Dict[str, Any], Optional[Dict[str, Any]]]] = {}

    # ------------------------------------------------------------ helpers
    def is_nexus(self, obj: Optional[Dict[str, Any]]) -> bool:
        """nexus-core ``resolvers.IsNexusRunEvent`` label check."""
        if not obj:
            return False
        return kube.labels_of(obj).get(self.labels.nexus_component_label) == self.labels.algorithm_run_value

    def _algorithm(self, obj) -> str:
        return kube.labels_of(obj).get(self.labels.job_template_name_key, "")

    def _pod_request_id(self, pod) -> str:
        return kube.labels_of(pod).get(self.labels.job_name_label, "")

    def _result(self, action, message, trace, involved, request_id, algorithm, reason, fclass, source, event_uid="") -> RunStatusAnalysisResult:
        r = RunStatusAnalysisResult(
            action=action, run_status_message=message, run_status_trace=trace or "",
            object_uid=(involved or {}).get("uid", "") or "", object_kind=(involved or {}).get("kind", "") or "",
            request_id=request_id, algorithm=algorithm, reason=reason, failure_class=fclass, event_uid=event_uid,
        )
        r.evidence["source"] = source
        return r

    # ------------------------------------------------------------ R-EVT
    def classify_event(self, event: Dict[str, Any], lookup: ObjectLookup) -> Tuple[str, List[RunStatusAnalysisResult]]:
        inv = event.get("involvedObject") or {}
        kind = inv.get("kind", "")
        if kind not in ("Job", "Pod"):
            return IGNORED, []
        if event.get("reason", "") not in _EVENT_REASONS and not event.get("reason", "").startswith("OutOf"):
            # most of a namespace's Events (Scheduled, Pulling, Pulled, Created, Killing,
            # SuccessfulCreate, ...) decide nothing: no cache lookup, no stale-event parking
            return NOOP, []
        obj = lookup.get(kind, inv.get("name", ""))
        if obj is None:
            return STALE, []
        if not self.is_nexus(obj):
            return IGNORED, []
        reason = event.get("reason", "")
        message = event.get("message", "") or ""
        ev_uid = kube.uid_of(event)
        if kind == "Job":
            rule = R.JOB_EVENT_RULES.get(reason)
            if rule is None:
                return NOOP, []
            action, msg, fclass = rule
            res = self._result(action, msg, message, inv, inv.get("name", ""), self._algorithm(obj), reason, fclass, "event", ev_uid)
            self._enrich(res, pods=lookup.pods_of_job(inv.get("name", "")), texts=[message])
            return DECIDED, [res]
        # Pod
        request_id = self._pod_request_id(obj)
        algorithm = self._algorithm(obj)
        rule = R.POD_EVENT_RULES.get(reason)
        if rule is not None:
            action, fclass = rule
            if reason == "BackOff" and "pulling image" in message.lower():
                fclass = F.IMAGE_PULL
            elif reason == "BackOff" and "restarting failed container" in message.lower():
                fclass = F.CRASH_LOOP
            elif reason == "Failed" and ("image" in message.lower()):
                fclass = F.IMAGE_PULL
            res = self._result(action, reason, message, inv, request_id, algorithm, reason, fclass, "event", ev_uid)
            if action != A.TO_RUNNING:
                self._enrich(res, pods=[obj], texts=[message])
            return DECIDED, [res]
        if reason in EVICTION_EVENT_REASONS:
            item = {"kind": "evicted", "reason": reason, "message": message, "pod": kube.name_of(obj)}
            if self.rules.evicted_policy == "fail":
                res = self._result(A.TO_FAIL_FATAL_ERROR, MSG_EVICTED, message, inv, request_id, algorithm, reason, F.EVICTED, "event", ev_uid)
                self._enrich(res, pods=[obj], texts=[message])
                return DECIDED, [res]
            self.evidence.add((algorithm, request_id), item)
            return EVIDENCE, []
        if reason == "FailedScheduling":
            self.evidence.add((algorithm, request_id), {"kind": "unschedulable", "message": message})
            return EVIDENCE, []
        if reason in ADMISSION_EVENT_REASONS or reason.startswith("OutOf"):
            # the kubelet's rejection Event: the pod-status rule decides from the pod's own
            # Failed status when it can wait for the node agent's GPU evidence (the kubelet
            # always writes that status); otherwise the Event decides
            det = self._admission_detail(reason, message, obj)
            wait_for_status = (self.rules.pod_status_rules and det["gpu"] and self.gpu.evidence_wait > 0
                               and not self.has_gpu_evidence(obj))
            if self.rules.admission_policy == "observe" or wait_for_status:
                self.evidence.add((algorithm, request_id), dict(det, kind="admission", message=message[-512:]))
                return EVIDENCE, []
            return DECIDED, [self._admission_result(obj, det, message, inv, request_id, algorithm, "event", ev_uid)]
        return NOOP, []

    # ------------------------------------------------------------ kubelet admission
    def _admission_detail(self, reason: str, message: str, pod: Optional[Dict[str, Any]]) -> Dict[str, Any]:
        """What a kubelet admission rejection says: whether it is about the pod's GPUs (the
        device plugin could not allocate — an unhealthy GPU after a reset or ECC storm, a
        restarting device plugin —, OutOf<gpu resource>, or the topology manager could not
        align the GPUs), the node, and the counts the message carries."""
        res = self.gpu.gpu_resource_name
        req = kube.gpu_request(pod, res) if pod else 0
        gpu = (reason == "OutOf" + res or (bool(res) and res in message)
               or (req > 0 and reason in ADMISSION_EVENT_REASONS))
        d: Dict[str, Any] = {"reason": reason, "gpu": gpu, "node": ((pod or {}).get("spec") or {}).get("nodeName", "")}
        if gpu:
            d["resource"] = res
            d["requested"] = req
        m = _ALLOC_NUMS.search(message)
        if m:
            d["requested"], d["available"] = int(m.group(1)), int(m.group(2))
        else:
            m = _FIT_NUMS.search(message)
            if m:
                d["requested"], d["used"], d["capacity"] = int(m.group(1)), int(m.group(2)), int(m.group(3))
        return d

    def _admission_result(self, pod, det, message, inv, request_id, algorithm, source, ev_uid="") -> RunStatusAnalysisResult:
        gpu = det["gpu"]
        res = self._result(A.TO_FAIL_STUCK_IN_PENDING, MSG_GPU_ADMISSION if gpu else MSG_ADMISSION, message, inv,
                           request_id, algorithm, det["reason"], F.GPU_ADMISSION if gpu else F.ADMISSION, source, ev_uid)
        res.evidence["admission"] = det
        self._enrich(res, pods=[pod])
        return res

    # ------------------------------------------------------------ R-POD
    def has_gpu_evidence(self, pod: Dict[str, Any]) -> bool:
        return self.evidence_provider is not None or bool(kube.annotations_of(pod).get(self.gpu.evidence_annotation))

    def classify_pod(self, pod: Dict[str, Any], old: Optional[Dict[str, Any]] = None,
                     allow_wait: bool = False, allow_log_fetch: bool = False) -> List[RunStatusAnalysisResult]:
        """Pod-status rules.  With ``allow_wait`` a failed GPU pod whose node agent has not
        annotated it yet is *deferred* (``self.deferred`` set, no result) so the caller can
        give the evidence ``gpu.evidence-wait`` to arrive.  With ``allow_log_fetch`` a failed
        GPU container with an empty termination message and no OOM verdict yet is deferred
        too (``self.deferred_log`` names the container instances) until the caller stored
        its log tail in :attr:`log_cache` (``gpu.log-tail``; a default pod's termination
        message is empty, its OOM text is in the log)."""
        self.deferred = False
        if self.deferred_log:
            self.deferred_log = []
        if not self.rules.pod_status_rules or not self.is_nexus(pod):
            return []
        if old is not None and kube.resource_version(old) == kube.resource_version(pod) and kube.resource_version(pod):
            return []  # resync replay of an unchanged object
        status = pod.get("status") or {}
        if (not status.get("containerStatuses") and not status.get("initContainerStatuses")
                and not status.get("conditions") and status.get("reason") != "Evicted"
                and status.get("phase") != "Failed"):
            return []  # freshly created / not yet scheduled: nothing any rule can match
        request_id = self._pod_request_id(pod)
        if not request_id:
            return []
        algorithm = self._algorithm(pod)
        key = (algorithm, request_id)
        inv = {"kind": "Pod", "name": kube.name_of(pod), "uid": kube.uid_of(pod)}
        # 0. refused by the node's kubelet at admission (Failed, no container ever created)
        rej = kube.admission_rejection(pod)
        if rej is not None:
            det = self._admission_detail(rej["reason"], rej["message"], pod)
            if self.rules.admission_policy == "observe":
                self.evidence.add(key, dict(det, kind="admission", message=rej["message"][-512:]))
                return []
            if det["gpu"] and allow_wait and not self.has_gpu_evidence(pod):
                self.deferred = True  # the node agent's GPU-health record is on its way
                return []
            return [self._admission_result(pod, det, rej["message"], inv, request_id, algorithm, "pod-status")]
        current_terms = [t for t in kube.terminated_states(pod) if t["which"] == "state"]
        # 1. OOM (host cgroup OOMKilled or HIP OOM signature on a terminated container)
        failed_terms = [t for t in current_terms if t.get("exitCode", 0) != 0 or t.get("reason") == "OOMKilled"]
        if failed_terms:
            if allow_wait and not self.has_gpu_evidence(pod) and kube.gpu_request(pod, self.gpu.gpu_resource_name) > 0:
                self.deferred = True
                return []
            if allow_log_fetch and not any(t.get("message") or t.get("reason") == "OOMKilled" for t in failed_terms):
                # nothing here can be a text signature: ask for the tail of every instance not
                # read yet before scoring (the second pass scores once, with the tail)
                want = self._log_fetch_needed(pod)
                if want:
                    self.deferred_log = want
                    self.deferred = True
                    return []
            verdict = self._oom(pod, [], failed_terms)
            if allow_log_fetch and not verdict.text_signature:
                # no verdict, or one resting only on exit codes / VRAM numbers: the log tail
                # (a traceback, a collective timeout, the HIP OOM line) decides first
                want = self._log_fetch_needed(pod)
                if want:
                    self.deferred_log = want
                    self.deferred = True
                    return []
            if verdict.kind:
                hbm = verdict.kind == "hbm"
                t0 = failed_terms[0]
                res = self._result(A.TO_FAIL_FATAL_ERROR, MSG_HBM_OOM if hbm else MSG_HOST_OOM,
                                   t0.get("message") or t0.get("reason") or "", inv, request_id, algorithm,
                                   t0.get("reason") or "Error", F.HBM_OOM if hbm else F.HOST_OOM, "pod-status")
                self._enrich(res, pods=[pod], verdict=verdict)
                return [res]
            faults = self._gpu_faults(pod)
            if faults:
                t0 = failed_terms[0]
                res = self._result(A.TO_FAIL_FATAL_ERROR, MSG_GPU_FAULT, t0.get("message") or t0.get("reason") or "", inv,
                                   request_id, algorithm, "GpuFault:" + ",".join(faults), F.GPU_FAULT, "pod-status")
                self._enrich(res, pods=[pod], verdict=verdict)
                return [res]
            for t in failed_terms:
                self.evidence.add(key, {"kind": "exit", "container": t.get("container"), "exitCode": t.get("exitCode"),
                                        "reason": t.get("reason"), "message": (t.get("message") or "")[-512:]})
        # 2. eviction
        if status.get("reason") == "Evicted" or self._disruption(pod):
            msg = status.get("message", "") or (self._disruption(pod) or {}).get("message", "")
            if self.rules.evicted_policy == "fail":
                res = self._result(A.TO_FAIL_FATAL_ERROR, MSG_EVICTED, msg, inv, request_id, algorithm,
                                   status.get("reason") or "DisruptionTarget", F.EVICTED, "pod-status")
                self._enrich(res, pods=[pod], texts=[msg])
                return [res]
            self.evidence.add(key, {"kind": "evicted", "message": msg, "pod": kube.name_of(pod)})
            return []
        # 3./4./5. waiting states
        for w in kube.waiting_states(pod):
            wr = w.get("reason", "")
            if wr in IMAGE_PULL_WAITING:
                res = self._result(A.TO_FAIL_STUCK_IN_PENDING, MSG_IMAGE_PULL, w.get("message", ""), inv, request_id, algorithm, wr, F.IMAGE_PULL, "pod-status")
                self._enrich(res, pods=[pod])
                return [res]
            if wr in CONFIG_WAITING:
                res = self._result(A.TO_FAIL_STUCK_IN_PENDING, MSG_CONFIG, w.get("message", ""), inv, request_id, algorithm, wr, F.CONFIG, "pod-status")
                self._enrich(res, pods=[pod])
                return [res]
            if wr == "CrashLoopBackOff":
                if allow_log_fetch:
                    want = self._log_fetch_needed(pod)
                    if want:  # the last instance's OOM text may be in its log only
                        self.deferred_log = want
                        self.deferred = True
                        return []
                texts = [t.get("message", "") for t in kube.terminated_states(pod)]
                res = self._result(A.TO_FAIL_FATAL_ERROR, MSG_CRASH_LOOP, w.get("message", ""), inv, request_id, algorithm, wr, F.CRASH_LOOP, "pod-status")
                self._enrich(res, pods=[pod], texts=texts)
                return [res]
        # 6. unschedulable
        sched = kube.condition(pod, "PodScheduled")
        if sched and sched.get("status") == "False" and sched.get("reason") == "Unschedulable":
            self.evidence.add(key, {"kind": "unschedulable", "message": sched.get("message", "")})
            if self.rules.unschedulable_timeout > 0 and self._pending_for(pod) >= self.rules.unschedulable_timeout:
                res = self._result(A.TO_FAIL_STUCK_IN_PENDING, MSG_UNSCHEDULABLE, sched.get("message", ""), inv, request_id, algorithm,
                                   "Unschedulable", F.SCHEDULING, "pod-status")
                self._enrich(res, pods=[pod])
                return [res]
            return []
        # 7. running (backup for a lost "Started" event): only the pod's transition to Running
        # is a start — a pod already running when it is first listed (a restart's initial LIST
        # of 10k live runs) is not, and its Started Event is replayed from the Event list; a
        # pod being deleted is not starting either.  A run whose Started Event expired while
        # the supervisor was down is caught by the supervisor's running sweep
        # (rules.running-sweep-rate, :meth:`running_result`)
        if (old is not None and status.get("phase") == "Running" and not _running(old)
                and not kube.meta(pod).get("deletionTimestamp") and _running(pod)):
            res = self._result(A.TO_RUNNING, "Started", "", inv, request_id, algorithm, "Running", F.NONE, "pod-status")
            return [res]
        return []

    def running_result(self, pod: Dict[str, Any]) -> Optional[RunStatusAnalysisResult]:
        """``ToRunning`` for a Nexus pod that is running now (not being deleted), else None:
        the running sweep's decision for a run whose Started Event is gone (event TTL)."""
        if not self.is_nexus(pod) or kube.meta(pod).get("deletionTimestamp"):
            return None
        if (pod.get("status") or {}).get("phase") != "Running" or not _running(pod):
            return None
        request_id = self._pod_request_id(pod)
        if not request_id:
            return None
        inv = {"kind": "Pod", "name": kube.name_of(pod), "uid": kube.uid_of(pod)}
        return self._result(A.TO_RUNNING, "Started", "", inv, request_id, self._algorithm(pod), "Running", F.NONE,
                            "running-sweep")

    def _disruption(self, pod) -> Optional[Dict[str, Any]]:
        c = kube.condition(pod, "DisruptionTarget")
        if c and c.get("status") == "True":
            return c
        return None

    def _pending_for(self, pod) -> float:
        import datetime as dt
        ts = kube.meta(pod).get("creationTimestamp")
        if not ts:
            return 0.0
        try:
            t = dt.datetime.fromisoformat(ts.replace("Z", "+00:00"))
        except ValueError:
            return 0.0
        return (dt.datetime.now(dt.timezone.utc) - t).total_seconds()

    # ------------------------------------------------------------ R-JOB
    def classify_job(self, job: Dict[str, Any], old: Optional[Dict[str, Any]], lookup: ObjectLookup) -> List[RunStatusAnalysisResult]:
        if not self.rules.pod_status_rules or not self.is_nexus(job):
            return []
        if old is not None and kube.resource_version(old) == kube.resource_version(job) and kube.resource_version(job):
            return []
        cond = kube.condition(job, "Failed")
        if not cond or cond.get("status") != "True":
            return []
        if old is not None:
            oc = kube.condition(old, "Failed")
            if oc and oc.get("status") == "True":
                return []  # already failed before this update
        reason = cond.get("reason", "")
        rule = R.JOB_EVENT_RULES.get(reason)
        if rule is None:
            if reason not in JOB_FAILED_CONDITION_REASONS:
                return []
            rule = (A.TO_FAIL_FATAL_ERROR, R.MSG_FATAL, F.FATAL)
        action, msg, fclass = rule
        name = kube.name_of(job)
        inv = {"kind": "Job", "name": name, "uid": kube.uid_of(job)}
        res = self._result(action, msg, cond.get("message", ""), inv, name, self._algorithm(job), reason, fclass, "job-status")
        self._enrich(res, pods=lookup.pods_of_job(name), texts=[cond.get("message", "")])
        return [res]

    # ------------------------------------------------------------ R-GPU enrichment
    def _gpu_evidence(self, pod) -> Optional[Dict[str, Any]]:
        raw = kube.annotations_of(pod).get(self.gpu.evidence_annotation)
        if not raw:
            if self.evidence_provider is not None:
                try:
                    return self.evidence_provider(pod)
                except Exception:  # evidence is advisory; never fail a decision on it
                    return None
            return None
        try:
            ev = json.loads(raw)
        except (TypeError, ValueError):
            return None
        return ev if isinstance(ev, dict) else None

    def _pod_ctx(self, pod, want_gpu: bool = True):
        """(topology, gpu evidence) for a pod version, memoised: the OOM verdict and the
        enrichment of one decision read the same pod, and evidence snapshots are not free."""
        key = (kube.uid_of(pod) or kube.name_of(pod), kube.resource_version(pod), want_gpu)
        hit = self._ctx_cache.get(key)
        if hit is not None:
            return hit
        topo = topology_from_pod(pod, self.gpu.gpu_resource_name)
        gev = self._gpu_evidence(pod) if want_gpu else None
        if gev:
            # physical view: device-plugin allocation / UUIDs → physical GPUs, measured xGMI
            topo = xgmi_from_evidence(resolve_devices(topo, gev), gev)
        if len(self._ctx_cache) > 4096:
            self._ctx_cache.clear()
        self._ctx_cache[key] = (topo, gev)
        return topo, gev

    def _gpu_faults(self, pod) -> List[str]:
        """GPU fault events (VM fault, reset) inside the pod's evidence window."""
        _topo, gev = self._pod_ctx(pod)
        if not gev or not self._uses_gpu(pod, gev):
            return []
        kinds = set()
        for g in gev.get("gpus", []):
            for e in g.get("events", []):
                if e.get("type") in FAULT_EVENTS:
                    kinds.add(e["type"])
        return sorted(kinds)

    def _uses_gpu(self, pod, gev) -> bool:
        """HBM verdicts and GPU faults need a GPU: the pod requests ``gpu-resource-name``
        or the evidence matched its own processes on one."""
        return oom_mod.gpu_involved(kube.gpu_request(pod, self.gpu.gpu_resource_name), gev)

    def _oom(self, pod, texts, terms) -> oom_mod.OomVerdict:
        topo, gev = self._pod_ctx(pod)
        return oom_mod.analyze(list(texts) + self._log_texts(pod, gev), terms, gev, topo.get("expected_gpu"),
                               self.gpu.hbm_capacity_gb, self.gpu.hbm_oom_fraction, topo=topo,
                               gpu_involved=self._uses_gpu(pod, gev))

    # ------------------------------------------------------------ container log tails
    def _cached_logs(self, pod) -> List[Dict[str, Any]]:
        """Fetched log records of the pod's *current* failed container instances: a
        CrashLoopBackOff pod's earlier instance (read for an earlier failure) never speaks
        for the instance that just failed."""
        if not self.log_cache:
            return []
        got = self.log_cache.get(kube.uid_of(pod) or kube.name_of(pod))
        if not got:
            return []
        out = []
        for fc in logtail.failed_containers(pod):
            r = got.get((fc["container"], fc["restart"]))
            if r is None:
                r = got.get((fc["container"], None))  # a record that named no instance
            if r is not None:
                out.append(r)
        return out

    def _log_records(self, pod, gev) -> List[Dict[str, Any]]:
        if self.gpu.log_tail == "off":
            return []
        agent = (gev or _NO_EV).get("logs")
        got = self._cached_logs(pod)
        if not agent:
            return got
        recs = list(agent)
        if got:
            recs.extend(got)
        return recs

    def _log_texts(self, pod, gev) -> List[Tuple[str, str]]:
        recs = self._log_records(pod, gev)
        return logtail.log_texts(recs) if recs else []

    def _log_fetch_needed(self, pod) -> List[Dict[str, Any]]:
        """Container instances whose log tail the supervisor should fetch (``pods/log``):
        a GPU pod's failed containers with an empty termination message that neither the
        node agent (``auto``) nor an earlier fetch has read."""
        mode = self.gpu.log_tail
        if mode not in ("auto", "api") or kube.gpu_request(pod, self.gpu.gpu_resource_name) <= 0:
            return []
        want = logtail.failed_containers(pod)
        got = self.log_cache.get(kube.uid_of(pod) or kube.name_of(pod)) if self.log_cache else None
        if want and got:
            # one fetch per container *instance* (pod uid, container, restart)
            want = [w for w in want if (w["container"], w["restart"]) not in got and (w["container"], None) not in got]
        if want and mode == "auto":
            _topo, gev = self._pod_ctx(pod)
            read = {(r.get("container"), r.get("restart")) for r in (gev or {}).get("logs") or () if not r.get("error")}
            want = [w for w in want if (w["container"], w["restart"]) not in read and (w["container"], None) not in read]
        return want

    def store_logs(self, pod, records: List[Dict[str, Any]]) -> None:
        """Log-tail records fetched for ``pod``, keyed by container instance
        ``(container, restart)`` (kept even when empty or failed: one fetch per instance);
        bounded LRU over pods, at most 16 instances per pod."""
        key = kube.uid_of(pod) or kube.name_of(pod)
        inst = self.log_cache.get(key)
        if inst is None:
            inst = self.log_cache[key] = {}
        else:
            self.log_cache.move_to_end(key)
        for r in records:
            ik = (r.get("container", ""), r.get("restart"))
            inst.pop(ik, None)
            inst[ik] = r
        while len(inst) > 16:
            del inst[next(iter(inst))]
        while len(self.log_cache) > 4096:
            self.log_cache.popitem(last=False)

    def _root_cause(self, pods: List[Dict[str, Any]]) -> Tuple[Optional[Dict[str, Any]], Dict[str, Any]]:
        """Culprit pod and the ``ranks`` trace block of a multi-pod job (:mod:`..gpu.collective`):
        the rank that ran out of memory or failed on its own, not one that died of its
        collective's collateral."""
        recs = []
        by_name: Dict[str, Dict[str, Any]] = {}
        for p in pods:
            terms = list(kube.terminated_states(p))
            if not terms:
                continue
            topo, gev = self._pod_ctx(p)
            texts = [(f"termination message of container {t.get('container', '')}", t["message"])
                     for t in terms if t.get("message")] + self._log_texts(p, gev)
            if self._uses_gpu(p, gev) and any(oom_mod.hbm_signature(x) for _s, x in texts):
                kind = "hbm"
            elif any(t.get("reason") == "OOMKilled" for t in terms) or any(oom_mod.host_signature(x) for _s, x in texts):
                kind = "host"
            else:
                kind = None
            name = kube.name_of(p)
            rec = collective.pod_failure(name, terms, texts, kind, bool(self._gpu_faults(p)), topo.get("rank"))
            if rec is not None:
                recs.append(rec)
                by_name[name] = p
        culprit, block = collective.rank_summary(recs)
        return (by_name[culprit["pod"]] if culprit else None), block

    def _apply_ranks(self, res: RunStatusAnalysisResult, pods: List[Dict[str, Any]]) -> Optional[Dict[str, Any]]:
        """Record the ``ranks`` block of a multi-pod decision and refine a generic failure
        class from it (every rank collective-only → ``collective``; a culprit with GPU fault
        evidence, e.g. an xGMI link down → ``gpu-fault``); returns the culprit pod."""
        culprit, block = self._root_cause(pods)
        if culprit is None:
            return None
        res.evidence["ranks"] = block
        if res.failure_class in (F.FATAL, F.BACKOFF_LIMIT, F.NONE, F.COLLECTIVE):
            if block["all_collective"]:
                res.failure_class = F.COLLECTIVE
            elif block["culprit"]["kind"] == "gpu-fault":
                res.failure_class = F.GPU_FAULT
        return culprit

    def _enrich(self, res: RunStatusAnalysisResult, pods=(), texts=(), verdict: Optional[oom_mod.OomVerdict] = None) -> None:
        if not self.gpu.attribution_enabled:
            return
        if self.lazy_enrich:
            # a run's failure usually arrives as two or three decisions (the pod's status, the
            # Job's event and condition) of which one is written: enrich that one, at
            # actuation (:meth:`finish`)
            res.pending_enrich = (pods, texts, verdict)
            return
        self._enrich_now(res, pods, texts, verdict)

    def finish(self, res: RunStatusAnalysisResult, lookup: ObjectLookup) -> None:
        """Complete a decision about to be written: the deferred enrichment (with the pod
        versions seen at classification), then :meth:`late_enrich`."""
        p = res.pending_enrich
        if p is not None:
            res.pending_enrich = None
            pods, texts, verdict = p
            if res.object_kind == "Job":
                # a Job-level decision speaks for its pods as they are now: the node agent's
                # evidence annotation (or the OOM termination) may have landed since the Job's
                # update was classified
                pods = lookup.pods_of_job(res.request_id) or pods
            self._enrich_now(res, pods, texts, verdict)
        self.late_enrich(res, lookup)

    def _enrich_now(self, res: RunStatusAnalysisResult, pods=(), texts=(),
                    verdict: Optional[oom_mod.OomVerdict] = None) -> None:
        pods = [p for p in pods if p]
        key = res.key
        if pods:
            pod = pods[-1]
            if len(pods) > 1:
                # the culprit's topology maps the failing GPU, its evidence attributes it
                pod = self._apply_ranks(res, pods) or pod
            # a container that never started (image pull / config / scheduling) never touched a GPU
            want_gpu = res.failure_class not in NO_GPU_CLASSES
            topo, gev = self._pod_ctx(pod, want_gpu)
            topo = merge_process_ranks(topo, gev)
            if topo:
                res.evidence["topology"] = topo
            if gev:
                res.evidence["gpu"] = gev
            logs = [r for p in pods for r in self._cached_logs(p)] if self.log_cache else None
            if logs and want_gpu:
                res.evidence["logs"] = logs
            if verdict is None and res.action != A.TO_RUNNING and res.failure_class not in ADMISSION_CLASSES:
                terms = [t for p in pods for t in kube.terminated_states(p)]
                ltexts = [x for p in pods for x in self._log_texts(p, gev if p is pod else self._pod_ctx(p)[1])]
                verdict = oom_mod.analyze(list(texts) + ltexts, terms, gev,
                                          topo.get("expected_gpu"), self.gpu.hbm_capacity_gb, self.gpu.hbm_oom_fraction,
                                          topo=topo, gpu_involved=self._any_gpu(pods, pod, gev))
        elif verdict is None and res.action != A.TO_RUNNING and any(texts):
            verdict = oom_mod.analyze(texts, (), None, None, self.gpu.hbm_capacity_gb, self.gpu.hbm_oom_fraction)
        if verdict is not None:
            if verdict.kind:
                res.evidence["oom"] = verdict.as_dict()
                if res.failure_class in (F.FATAL, F.BACKOFF_LIMIT, F.NONE, F.CRASH_LOOP, F.COLLECTIVE):
                    res.failure_class = F.HBM_OOM if verdict.kind == "hbm" else F.HOST_OOM
            if verdict.foreign is not None:
                # someone else filled the GPU: recorded with its holders whatever the verdict (a
                # crash at HIP init on a full GPU has no OOM text, but is "gpu-occupied")
                res.evidence["foreign_occupancy"] = verdict.foreign
        if res.action != A.TO_RUNNING:
            self._apply_history(res)

    def _any_gpu(self, pods, pod, gev) -> bool:
        return any(self._uses_gpu(p, gev if p is pod else self._pod_ctx(p)[1]) for p in pods)

    def _apply_history(self, res: RunStatusAnalysisResult) -> None:
        """Attach the run's non-decisive history and settle the cause of a Job's
        BackoffLimitExceeded.  Called at the end of classification and again at actuation
        (:meth:`late_enrich`), so the outcome is the same whichever watch stream — Pod or
        Job / Event — delivered first."""
        prior = self.evidence.get(res.key)
        if prior:
            res.evidence["history"] = prior
            if res.failure_class == F.BACKOFF_LIMIT:
                adm = [p for p in prior if p.get("kind") == "admission"]
                if adm:
                    # its pods were refused by their nodes' kubelets: never ran, never retried
                    # of their own doing (a GPU admission outranks any other rejection)
                    a = next((p for p in adm if p.get("gpu")), adm[-1])
                    res.failure_class = F.GPU_ADMISSION if a.get("gpu") else F.ADMISSION
                    res.evidence.setdefault("admission", {k: v for k, v in a.items() if k not in ("kind", "message")})
                elif any(p.get("kind") == "evicted" for p in prior):
                    res.failure_class = F.EVICTED
        if (res.action == A.TO_FAIL_DEADLINE_EXCEEDED and res.reason == "BackoffLimitExceeded"
                and self.rules.oom_fails_backoff_job):
            # BackoffLimitExceeded of a run whose pods died of an OOM, were evicted or were
            # refused at kubelet admission: the run neither timed out nor ran out of retries of
            # its own doing — write the row the pod-status rule / ``evicted-policy: fail``
            # writes (FAILED, or SCHEDULING_FAILED for an admission rejection, with that cause).
            # On by default; false keeps the reference's DEADLINE_EXCEEDED for
            # BackoffLimitExceeded (supervisor.go:183-193), the class and evidence then go into
            # the trace only (docs/PARITY.md)
            cause = _BACKOFF_CAUSE.get(res.failure_class)
            if cause is not None:
                res.action, res.run_status_message = cause

    def late_enrich(self, res: RunStatusAnalysisResult, lookup: ObjectLookup) -> None:
        """Re-enrich a Job-level decision just before it is written.

        Pods and Jobs arrive on separate watch streams, so a Job's failure can be
        classified before its pods' last updates (eviction, OOM termination) are seen.
        By actuation time (after queueing and the checkpoint read) they usually have
        been; this costs no extra latency."""
        if not self.gpu.attribution_enabled or res.action == A.TO_RUNNING or res.object_kind != "Job":
            return
        if res.failure_class in (F.BACKOFF_LIMIT, F.FATAL, F.NONE, F.COLLECTIVE):
            pods = lookup.pods_of_job(res.request_id)
            for pod in pods:
                st = pod.get("status") or {}
                if st.get("reason") == "Evicted" or self._disruption(pod):
                    self.evidence.add(res.key, {"kind": "evicted", "message": st.get("message", ""), "pod": kube.name_of(pod)})
                else:
                    rej = kube.admission_rejection(pod)
                    if rej is not None:
                        det = self._admission_detail(rej["reason"], rej["message"], pod)
                        self.evidence.add(res.key, dict(det, kind="admission", message=rej["message"][-512:]))
            culprit = pods[-1] if pods else None
            if len(pods) > 1:
                # the pods' last updates may have landed after the Job's: rank them again
                culprit = self._apply_ranks(res, pods) or culprit
            if pods and "oom" not in res.evidence:
                terms = [t for p in pods for t in kube.terminated_states(p)]
                if terms:
                    topo, gev = self._pod_ctx(culprit)
                    ltexts = [x for p in pods for x in self._log_texts(p, self._pod_ctx(p)[1])]
                    v = oom_mod.analyze(ltexts, terms, gev, topo.get("expected_gpu"),
                                        self.gpu.hbm_capacity_gb, self.gpu.hbm_oom_fraction, topo=topo,
                                        gpu_involved=self._any_gpu(pods, culprit, gev))
                    if v.kind:
                        res.evidence["oom"] = v.as_dict()
                        res.failure_class = F.HBM_OOM if v.kind == "hbm" else F.HOST_OOM
                        if gev and "gpu" not in res.evidence:
                            res.evidence["gpu"] = gev
                    if v.foreign is not None and "foreign_occupancy" not in res.evidence:
                        res.evidence["foreign_occupancy"] = v.foreign
                        if gev and "gpu" not in res.evidence:
                            res.evidence["gpu"] = gev
        self._apply_history(res)


_NO_EV: Dict[str, Any] = {}
# Event reasons any rule reads (decisions and evidence); OutOf<resource> is matched by prefix
_EVENT_REASONS = frozenset(R.JOB_EVENT_RULES) | frozenset(R.POD_EVENT_RULES) | frozenset(EVICTION_EVENT_REASONS) | {
    "FailedScheduling"} | frozenset(ADMISSION_EVENT_REASONS)
# the kubelet's resource-fit rejections (OutOf<resource>) the watch hub lets through
_OUT_OF = ("OutOfcpu", "OutOfmemory", "OutOfpods", "OutOfephemeral-storage")


def event_reasons_read(gpu_resource: str = "amd.com/gpu") -> frozenset:
    """Every Event reason a rule reads, for the watch hub's exact-match filter (the
    OutOf<resource> rejections of the GPU resource and the common host resources)."""
    return _EVENT_REASONS | frozenset(_OUT_OF) | frozenset(("OutOf" + gpu_resource,) if gpu_resource else ())


# every Event reason a rule reads; the watch hub drops the others before decode
EVENT_REASONS_READ = event_reasons_read()
# the Normal Events every run start and end emits (scheduler, kubelet, job controller): about
# a third of a busy namespace's watch objects, none of them read by a rule
EVENT_NOISE_REASONS = ("Scheduled", "Pulling", "Pulled", "Created", "Killing", "SuccessfulCreate",
                       "SuccessfulDelete", "Completed")


def event_field_selector(gpu_resource: str = "amd.com/gpu") -> str:
    """Server-side field selector of the Event watch: ``reason!=X`` for each noise reason
    no rule reads (Kubernetes ANDs the terms; Events support ``reason`` as a selectable
    field), so the API server never sends them.  A reason a rule reads is never excluded."""
    read = event_reasons_read(gpu_resource)
    return ",".join(f"reason!={r}" for r in EVENT_NOISE_REASONS if r not in read)
# BackoffLimitExceeded whose cause was found: the run's (action, failure message) per class
_BACKOFF_CAUSE = {F.HBM_OOM: (A.TO_FAIL_FATAL_ERROR, MSG_HBM_OOM), F.HOST_OOM: (A.TO_FAIL_FATAL_ERROR, MSG_HOST_OOM),
                  F.EVICTED: (A.TO_FAIL_FATAL_ERROR, MSG_EVICTED),
                  F.GPU_ADMISSION: (A.TO_FAIL_STUCK_IN_PENDING, MSG_GPU_ADMISSION),
                  F.ADMISSION: (A.TO_FAIL_STUCK_IN_PENDING, MSG_ADMISSION)}


def _running(pod) -> bool:
    """A container of the pod is running."""
    st = pod.get("status") or {}
    return any((cs.get("state") or {}).get("running") for cs in (st.get("containerStatuses") or []))
_PLAIN_CLASSES = frozenset((F.NONE, F.SCHEDULING, F.DEADLINE, F.FATAL, F.BACKOFF_LIMIT))


TRACE_TOP_PROCS = 4   # per GPU, by VRAM peak
TRACE_MAX_EVENTS = 8  # per GPU, newest


def render_trace(res: RunStatusAnalysisResult, fmt: str = "auto", max_bytes: int = 8192) -> str:
    """Trace column (``algorithm_failure_details``) for a decision.

    ``raw`` — the event/status message, as the reference (``supervisor.go:299``);
    ``json`` — message + reason + failure class + evidence; ``auto`` — json only
    when there is evidence beyond the message.

    Bounded (``rules.trace-max-bytes``, the row is a text column): per GPU the top
    ``TRACE_TOP_PROCS`` processes by VRAM peak and the newest ``TRACE_MAX_EVENTS`` events,
    the xGMI fabric as a per-GPU summary (:func:`..gpu.topology.xgmi_from_evidence`), and a
    deterministic trimming ladder (:func:`_trim_trace`) when the document still exceeds
    the cap — a real 8-GPU job's row stays small and the most telling facts survive."""
    ev = res.evidence
    if fmt == "raw" or (fmt == "auto" and res.failure_class in _PLAIN_CLASSES
                        and (not ev or (len(ev) == 1 and "source" in ev))):
        return res.run_status_trace
    doc = {"message": res.run_status_trace, "reason": res.reason, "class": res.failure_class,
           "source": ev.get("source", "")}
    for k, v in ev.items():
        if k != "source":
            doc[k] = v
    gpu, topo = doc.get("gpu"), doc.get("topology")
    xgmi = (topo or {}).get("xgmi")
    if gpu and gpu.get("gpus"):
        # the per-GPU records are shared by every decision of one telemetry snapshot
        # (telemetry.pod_evidence_provider): bound + encode them once per record list
        doc["gpu"] = dict(gpu, gpus=_trace_gpus(gpu.get("gpus") or []))
    if xgmi and _native_dumps is not None:
        # the xGMI block is shared by every decision of one telemetry snapshot
        # (topology.xgmi_from_evidence): encode it once, splice it into each trace
        doc["topology"] = dict(topo, xgmi=_raw_json(xgmi))
    # key order is the (deterministic) construction order: sorting every object doubled the
    # cost of the largest per-decision serialisation (profiles/r2_*_pprof_*)
    if _native_dumps is not None:
        raw = _native_dumps(doc, default=str)  # UTF-8 bytes: the cap is measured without re-encoding
        if max_bytes and len(raw) > max_bytes:
            return _trim_trace(doc, max_bytes)
        return raw.decode()
    out = _dumps(doc)
    if max_bytes and len(out.encode()) > max_bytes:
        out = _trim_trace(doc, max_bytes)
    return out


def _dumps(doc) -> str:
    if _native_dumps is not None:
        return _native_dumps(doc, default=str).decode()
    return json.dumps(doc, separators=(",", ":"), default=_json_default, ensure_ascii=False)


def _plain(obj):
    """A document with every spliced RawJSON decoded (for trimming)."""
    return json.loads(json.dumps(obj, separators=(",", ":"), default=_json_default, ensure_ascii=False))


def _trim_trace(doc: Dict[str, Any], max_bytes: int) -> str:
    """Deterministic trimming ladder: each step drops less telling detail than the next,
    and the document is re-measured after each; ``trimmed`` lists the steps applied."""
    d = _plain(doc)
    steps: List[str] = []

    def size() -> int:
        return len(json.dumps(dict(d, trimmed=steps), separators=(",", ":"), ensure_ascii=False).encode())

    def gpus():
        return ((d.get("gpu") or {}).get("gpus")) or []

    def slim(g):
        for k in [k for k in g if k not in ("index", "vram_total_mb", "vram_peak_mb", "matched", "proc_peak_vram_bytes")]:
            del g[k]

    topo = d.get("topology") or {}
    xg = topo.get("xgmi") or {}
    ladder = [
        # (a step returning False had nothing to trim and is not listed)
        ("gpu.holders:1", lambda: [g.__setitem__("holders", g["holders"][:1]) for g in gpus()
                                   if len(g.get("holders") or ()) > 1] or False),
        ("foreign_occupancy.holders:1", lambda: d["foreign_occupancy"].__setitem__(
            "holders", d["foreign_occupancy"]["holders"][:1])
         if len((d.get("foreign_occupancy") or {}).get("holders") or ()) > 1 else False),
        ("gpu.procs:1", lambda: [g.__setitem__("procs", (g.get("procs") or [])[:1]) for g in gpus()]),
        ("gpu.events:2", lambda: [g.__setitem__("events", (g.get("events") or [])[-2:]) for g in gpus() if "events" in g]),
        ("history:4", lambda: d.__setitem__("history", (d.get("history") or [])[-4:]) if "history" in d else None),
        ("ranks.pods:2", lambda: (d.get("ranks") or {}).__setitem__("pods", (d.get("ranks") or {}).get("pods", [])[:2])
         if (d.get("ranks") or {}).get("pods") else None),
        ("topology.collective_env", lambda: topo.pop("collective_env", None)),
        ("logs.lines:1", lambda: [r.__setitem__("lines", [x[-300:] for x in (r.get("lines") or [])[-1:]])
                                  for r in (d.get("logs") or []) + ((d.get("gpu") or {}).get("logs") or [])]),
        ("oom.signals:4", lambda: (d.get("oom") or {}).__setitem__("signals", (d.get("oom") or {}).get("signals", [])[:4])
         if d.get("oom") else None),
        ("topology.rank_map", lambda: topo.pop("rank_map", None)),
        ("ranks.pods", lambda: (d.get("ranks") or {}).pop("pods", None)),
        ("gpu.procs", lambda: [g.pop("procs", None) for g in gpus()]),
        ("gpu.holders", lambda: [g.pop("holders") for g in gpus() if "holders" in g] or False),
        ("gpu.events", lambda: [g.pop("events", None) for g in gpus()]),
        ("gpu.gpus:slim", lambda: [slim(g) for g in gpus()]),
        ("topology.xgmi.peers", lambda: [r.pop("peers", None) for r in xg.get("per_gpu", [])]),
        ("topology.xgmi.per_gpu", lambda: xg.pop("per_gpu", None)),
        ("message:1024", lambda: d.__setitem__("message", (d.get("message") or "")[-1024:])),
        ("topology.xgmi", lambda: topo.pop("xgmi", None)),
    ]
    for name, step in ladder:
        if size() <= max_bytes:
            break
        if step() is False:
            continue
        steps.append(name)
    if size() > max_bytes:
        # last resort: the decision's essentials only
        keep = {k: d[k] for k in ("message", "reason", "class", "source") if k in d}
        if d.get("oom"):
            keep["oom"] = {k: v for k, v in d["oom"].items() if k != "signals"}
        keep["message"] = (keep.get("message") or "")[-min(1024, max_bytes // 4):]
        d = keep
        steps.append("essentials")
    d["trimmed"] = steps
    return json.dumps(d, separators=(",", ":"), ensure_ascii=False)


class RawJSON(bytes):
    """Pre-encoded JSON spliced verbatim by the native encoder."""


_RAW_MEMO: Dict[int, Tuple[Any, RawJSON]] = {}


def _raw_json(obj) -> RawJSON:
    hit = _RAW_MEMO.get(id(obj))
    if hit is not None and hit[0] is obj:
        return hit[1]
    raw = RawJSON(_native_dumps(obj, default=str))
    if len(_RAW_MEMO) > 512:
        _RAW_MEMO.clear()
    _RAW_MEMO[id(obj)] = (obj, raw)  # holds obj: its id cannot be reused while cached
    return raw


_GPUS_MEMO: Dict[int, Tuple[Any, Any]] = {}
# fields a trace states once elsewhere: the link list and port counts (topology.xgmi), and
# each process's world sizes / visible devices (topology)
_GPU_DUP = frozenset(("links", "xgmi_links_up", "xgmi_links_down", "xgmi_links_total", "xgmi_hive_id"))
_PROC_DUP = frozenset(("world_size", "local_world_size", "visible_devices"))


def _trace_gpus(gpus: List[Dict[str, Any]]):
    """Per-GPU records as they go into a trace: without the link list (the fabric is in
    topology.xgmi), the top processes by VRAM peak (``procs_total`` says how many there
    were) and the newest events; memoised per (shared, immutable) record list."""
    hit = _GPUS_MEMO.get(id(gpus))
    if hit is not None and hit[0] is gpus:
        return hit[1]
    out_l = []
    for g in gpus:
        r = {k: v for k, v in g.items() if k not in _GPU_DUP}
        procs = g.get("procs")
        if procs:
            top = sorted(procs, key=lambda p: (-(p.get("peak_vram_bytes") or 0), p.get("pid") or 0))[:TRACE_TOP_PROCS]
            r["procs"] = [{k: v for k, v in p.items() if k not in _PROC_DUP} for p in top]
            if len(procs) > TRACE_TOP_PROCS:
                r["procs_total"] = len(procs)
        evs = g.get("events")
        if evs and len(evs) > TRACE_MAX_EVENTS:
            r["events"] = evs[-TRACE_MAX_EVENTS:]
            r["events_total"] = len(evs)
        out_l.append(r)
    out = RawJSON(_native_dumps(out_l, default=str)) if _native_dumps is not None else out_l
    if len(_GPUS_MEMO) > 512:
        _GPUS_MEMO.clear()
    _GPUS_MEMO[id(gpus)] = (gpus, out)  # holds the list: its id cannot be reused while cached
    return out


def _json_default(o):
    if isinstance(o, RawJSON):
        return json.loads(o)
    return str(o)


try:  # compact UTF-8 JSON (csrc/kube/json_encode.cpp); same document as the json fallback
    from .._kube_native import dumps as _native_dumps
except ImportError:  # pragma: no cover - CPU hosts without the native build
    _native_dumps = None
