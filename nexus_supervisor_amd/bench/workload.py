"""Synthetic Nexus cluster traffic for the north-star benchmark (BASELINE.json:
"pod-fail→checkpoint p50/p99 latency + events/sec at 10k concurrent jobs",
synthetic pod-failure events with random job IDs).

A :class:`Workload` owns a pool of ``concurrent_jobs`` Nexus runs (Job + Pod objects with
torchrun/RCCL env for one MI355X GPU-job slot) and produces the watch stream a real
namespace carries while runs start and fail at a steady rate — not only the failures.

Life of a run (what the reference sees on its three watches,
``/root/reference/services/supervisor.go:73-75,124-128``):

1. **created** (step k): the receiver has written the run's row ``BUFFERED``; the Job
   controller creates the Job (Job ADDED, Event ``SuccessfulCreate``) and its Pod (Pod ADDED,
   ``Pending``, unscheduled).
2. **started** (step k+1): Event ``Scheduled``, Pod MODIFIED (bound to its node), Events
   ``Pulling`` / ``Pulled`` / ``Created`` / ``Started``, Pod MODIFIED (``Running``), Job
   MODIFIED (``active``/``ready``).  The ``Started`` Event is the reference's most frequent
   decision: ``ToRunning`` → checkpoint read + upsert ``RUNNING``
   (``supervisor.go:224-233,361-370``).  A fifth of the failures (``image-pull``) are runs
   whose start fails instead.
3. **failed** (any later step): the pod / Job / Event traffic of its failure kind (below),
   then the supervisor's Job DELETE (the apiserver answers with Job and Pod DELETED lines),
   and a step later the run's Events expire (Event DELETED lines: the apiserver's event TTL,
   compressed — at steady state events expire as fast as they are created).

Each step fails ``events`` runs and creates as many, so the concurrency stays constant;
every failure brings its replacement run's whole start, about 20 watch objects in all.

Failure mix (Nexus Jobs carry a ``podFailurePolicy`` that fails the Job on exit 137 / 255 —
the reference's OOM path, ``supervisor_test.go:274-329`` — and ``backoffLimit: 0``):

==================  ==========================================================  ==================
kind                watch traffic                                               expected stage
==================  ==========================================================  ==================
host-oom            Pod MODIFIED terminated OOMKilled 137; Job MODIFIED Failed  FAILED
                    (PodFailurePolicy); Event (Job) PodFailurePolicy
hbm-oom             Pod MODIFIED exit 1 + HIP OOM (termination message, or the  FAILED
                    container log of a default pod — LOG, written before the
                    termination: pods/log, and with the simulator's --log-root a
                    kubelet-style /var/log/pods the node agent reads); Job
                    MODIFIED Failed (BackoffLimitExceeded); Event (Job)
                    BackoffLimitExceeded
image-pull          (a starting run) Event Scheduled, Pod bound, Event Pulling,  SCHEDULING_FAILED
                    Event Failed (ErrImagePull), Pod waiting ErrImagePull,
                    Event BackOff (pulling image), Pod waiting ImagePullBackOff
gpu-admission       (a starting run) Event Scheduled; Pod MODIFIED bound,        SCHEDULING_FAILED
                    Failed/UnexpectedAdmissionError (device plugin "Allocate
                    failed … amd.com/gpu"), no containers; Event (Pod)
                    UnexpectedAdmissionError; Job MODIFIED Failed
                    (BackoffLimitExceeded); Event (Job) BackoffLimitExceeded
pod-failure-policy  Pod MODIFIED exit 255 (a default pod: its log holds a plain     FAILED
                    traceback); Event (Job) PodFailurePolicy; Job MODIFIED Failed
                    (PodFailurePolicy) — reference R-EVT path
deadline            Event (Job) DeadlineExceeded; Job MODIFIED Failed           DEADLINE_EXCEEDED
                    (DeadlineExceeded); Event (Pod) Killing; Pod MODIFIED
                    (deletionTimestamp) — reference R-EVT path
evicted             Pod MODIFIED Failed/Evicted (DisruptionTarget); Event (Pod)  FAILED (eviction
                    Evicted; Job MODIFIED Failed (BackoffLimitExceeded); Event    cause,
                    (Job) BackoffLimitExceeded                                   rules.oom-fails-
                                                                                 backoff-job)
==================  ==========================================================  ==================
"""
from __future__ import annotations

import collections
import datetime as _dt
import random
from typing import Any, Deque, Dict, List, Optional, Tuple

from ..config.schema import LabelConfig
from ..models.checkpoint import CheckpointedRequest, LifecycleStage
from ..parallel.sharding import shard_of as _shard_of
from ..testing.seed import run_labels

DEFAULT_HIP_OOM = ("hipErrorOutOfMemory: HIP out of memory. Tried to allocate 4.00 GiB. GPU 0 has a total capacity of "
                   "287.98 GiB; 284.00 GiB already allocated by this process")

MIX: Tuple[Tuple[str, float, str], ...] = (
    ("host-oom", 0.30, LifecycleStage.FAILED),
    ("hbm-oom", 0.20, LifecycleStage.FAILED),
    ("image-pull", 0.17, LifecycleStage.SCHEDULING_FAILED),
    ("gpu-admission", 0.03, LifecycleStage.SCHEDULING_FAILED),
    ("pod-failure-policy", 0.10, LifecycleStage.FAILED),
    ("deadline", 0.10, LifecycleStage.DEADLINE_EXCEEDED),
    ("evicted", 0.10, LifecycleStage.FAILED),
)
START_KINDS = ("image-pull", "gpu-admission")  # failures of a starting run (the pod never ran)
# the AMD device plugin's allocation failure on a node whose GPU went unhealthy (kubelet
# device manager wording)
GPU_ADMISSION_MESSAGE = ("Allocate failed due to requested number of devices unavailable for amd.com/gpu. "
                         "Requested: 1, Available: 0, which is unexpected")

# what a running GPU pod's status / a started Job's status look like
_T0 = "2026-01-01T00:00:00Z"


def shard_of(algorithm: str, request_id: str, shards: int) -> int:
    """Replica shard of a run, as ``Supervisor.owns`` computes it (``parallel/sharding.py``)."""
    return _shard_of(request_id, shards)


class StepTraffic:
    """One step's generated input: the failed and the started runs, the watch traffic, the
    rows the receiver inserts first, and the stage each decision must write (fixed at
    generation: a run started here may fail in a later step)."""

    __slots__ = ("failed", "started", "traffic", "rows", "expected", "start_expected", "kinds")

    def __init__(self):
        self.failed: List[str] = []
        self.started: List[str] = []
        self.traffic: List[Tuple[str, Dict[str, Any]]] = []
        self.rows: List[CheckpointedRequest] = []
        self.expected: Dict[str, str] = {}
        self.start_expected: Dict[str, str] = {}
        self.kinds: Dict[str, str] = {}  # failed run -> failure kind (MIX)

    def __iter__(self):
        """``failed, traffic, rows = workload.step(n)``."""
        return iter((self.failed, self.traffic, self.rows))

    def doc(self, t_push: float) -> Dict[str, Any]:
        """The cluster's answer to a step (``/bench/step``)."""
        doc = {"rids": self.failed, "t_push": t_push, "expected": self.expected, "started": self.started,
               "start_expected": self.start_expected}
        if len(self.kinds) <= 8:  # a probe arrival: its failure's kind (the probe's tail report)
            doc["kinds"] = self.kinds
        return doc


class Workload:
    def __init__(self, concurrent_jobs: int = 10_000, rank: int = 0, world: int = 1, seed: int = 0,
                 labels: Optional[LabelConfig] = None, namespace: str = "nexus", algorithm: str = "bench-algorithm",
                 hip_oom_message: str = DEFAULT_HIP_OOM, gpus_per_node: int = 8, shards: int = 1, shard_index: int = 0,
                 shard_label: str = "", hbm_shape: str = "termination-message", run_starts: bool = True,
                 visible_devices: Optional[str] = None):
        self.rng = random.Random(seed * 7919 + rank)
        self.labels = labels or LabelConfig()
        self.ns = namespace
        self.algorithm = algorithm
        self.rank = rank
        self.world = world
        self.hip_oom_message = hip_oom_message
        self.gpus_per_node = gpus_per_node
        self.shards = shards
        self.shard_index = shard_index
        # hbm-oom failures: "termination-message" (the HIP text in terminated.message) or
        # "default-pod" (terminationMessagePolicy: File — an empty message, the text in the
        # container log: a ("LOG", …) traffic line the apiserver serves from pods/log)
        self.hbm_shape = hbm_shape
        # False: the round-4 shape — new runs are ADDED and never start (rows seeded RUNNING)
        self.run_starts = run_starts
        # the pods' HIP_VISIBLE_DEVICES: None = every GPU of the node (an 8-way torchrun job's
        # rank on this slot), or one GPU ("3": a node-mode slot whose pods the device plugin
        # gave GPU 3 — a process there calls it "GPU 0")
        self.visible_devices = visible_devices
        # sharding.shard-label: the submitter stamps each run's shard on its Job and pod template
        self.shard_label = shard_label if shards > 1 else ""
        self.live: List[str] = []      # running runs (may fail)
        self.pending: List[str] = []   # created, starting next step
        self.pods: Dict[str, Dict[str, Any]] = {}
        self.jobs: Dict[str, Dict[str, Any]] = {}
        self.events: Dict[str, List[Dict[str, Any]]] = {}  # run → its live Events (expire after it fails)
        self._expiring: Deque[List[Dict[str, Any]]] = collections.deque()
        self.expected: Dict[str, str] = {}
        self.kind_of: Dict[str, str] = {}  # failed run → failure kind (diagnostics)
        self._rv = 1000
        self._seq = 0
        self._ev = 0
        self.concurrent_jobs = concurrent_jobs
        self._kinds = [k for k, _, _ in MIX]
        self._weights = [w for _, w, _ in MIX]
        self._run_kinds = [k for k in self._kinds if k not in START_KINDS]
        self._run_weights = [w for k, w, _ in MIX if k not in START_KINDS]
        self._stage = {k: s for k, _, s in MIX}

    # ------------------------------------------------------------ ids / objects
    def _new_id(self) -> str:
        bits = self.rng.getrandbits
        while True:
            self._seq += 1
            # RFC 4122 v4 layout from 128 random bits (same ids as uuid.UUID(int=..., version=4))
            n = (bits(128) & ~(0xF000 << 64) | (0x4000 << 64)) & ~(0xC000 << 48) | (0x8000 << 48)
            h = "%032x" % n
            rid = f"{h[:8]}-{h[8:12]}-{h[12:16]}-{h[16:20]}-{h[20:]}"
            if self.shards <= 1 or shard_of(self.algorithm, rid, self.shards) == self.shard_index:
                return rid

    def _next_rv(self) -> str:
        self._rv += 1
        return str(self._rv)

    def _run_env(self, rid: str) -> Dict[str, str]:
        # one GPU-job slot per rank: an 8-way torchrun job whose local rank sits on this slot's GPU
        local = self.rank % self.gpus_per_node
        return {"RANK": str(local), "WORLD_SIZE": str(self.gpus_per_node), "LOCAL_RANK": str(local),
                "LOCAL_WORLD_SIZE": str(self.gpus_per_node), "MASTER_ADDR": f"{rid[:8]}-0.nexus-headless",
                "MASTER_PORT": "29500", "HIP_VISIBLE_DEVICES": self.visible_devices if self.visible_devices is not None
                else ",".join(str(i) for i in range(self.gpus_per_node)),
                "NCCL_IB_DISABLE": "1", "RCCL_MSCCLPP_ENABLE": "1"}

    def _templates(self):
        """Per-workload constant parts of the Job/Pod objects (built once)."""
        t = getattr(self, "_tmpl", None)
        if t is None:
            env = [{"name": k, "value": v} for k, v in self._run_env("x" * 8).items()]
            mi = next(i for i, e in enumerate(env) if e["name"] == "MASTER_ADDR")
            gpu = {"amd.com/gpu": "1"}
            job_labels = run_labels(self.labels, self.algorithm)
            t = self._tmpl = (env, mi, gpu, job_labels, f"mi355x-{self.rank // self.gpus_per_node:03d}")
        return t

    def _event(self, rid: str, kind: str, name: str, uid: str, reason: str, message: str,
               etype: str = "Normal", component: str = "kubelet") -> Dict[str, Any]:
        """A core/v1 Event about ``kind``/``name`` (kept per run so it can expire)."""
        self._ev += 1
        ev = {"apiVersion": "v1", "kind": "Event",
              "metadata": {"name": f"{name}.{self._ev:x}", "namespace": self.ns, "uid": f"ev-{self.rank}-{self._ev}",
                           "resourceVersion": self._next_rv(), "creationTimestamp": _T0},
              "involvedObject": {"kind": kind, "name": name, "namespace": self.ns, "uid": uid,
                                 "apiVersion": "batch/v1" if kind == "Job" else "v1"},
              "reason": reason, "message": message, "type": etype, "count": 1,
              "source": {"component": component}, "firstTimestamp": _T0, "lastTimestamp": _T0}
        self.events.setdefault(rid, []).append(ev)
        return ev

    def _pod_event(self, rid: str, reason: str, message: str, etype: str = "Normal", component: str = "kubelet"):
        pod = self.pods[rid]
        m = pod["metadata"]
        return self._event(rid, "Pod", m["name"], m["uid"], reason, message, etype, component)

    def _job_event(self, rid: str, reason: str, message: str, etype: str = "Warning"):
        return self._event(rid, "Job", rid, f"job-uid-{rid}", reason, message, etype, "job-controller")

    def _mod(self, obj: Dict[str, Any], status: Dict[str, Any], spec: Optional[Dict[str, Any]] = None,
             meta: Optional[Dict[str, Any]] = None) -> Dict[str, Any]:
        """A new version of ``obj`` (shallow: the unchanged parts are shared)."""
        o = dict(obj)
        o["metadata"] = dict(obj["metadata"], resourceVersion=self._next_rv(), **(meta or {}))
        if spec is not None:
            o["spec"] = dict(obj["spec"], **spec)
        o["status"] = status
        return o

    def new_run(self, stage: str = LifecycleStage.BUFFERED, running: bool = False
                ) -> Tuple[str, Dict[str, Any], Dict[str, Any], CheckpointedRequest]:
        """A run's Job, Pod and checkpoint row: ``running`` = an existing running run (the
        initial pool), else a new one whose pod is Pending and unscheduled."""
        rid = self._new_id()
        env_t, mi, gpu, job_labels, node = self._templates()
        ns, lab = self.ns, self.labels
        if self.shard_label:
            job_labels = dict(job_labels, **{self.shard_label: str(self.shard_index)})
        job = {"apiVersion": "batch/v1", "kind": "Job",
               "metadata": {"name": rid, "namespace": ns, "uid": f"job-uid-{rid}", "resourceVersion": self._next_rv(),
                            "creationTimestamp": _T0, "labels": dict(job_labels)},
               "spec": {"backoffLimit": 0, "podFailurePolicy": {"rules": [
                   {"action": "FailJob", "onExitCodes": {"operator": "In", "values": [137, 255]}}]}},
               "status": {"active": 1, "ready": 1, "startTime": _T0} if running else {"active": 1}}
        env = list(env_t)
        env[mi] = {"name": "MASTER_ADDR", "value": f"{rid[:8]}-0.nexus-headless"}
        pod_labels = dict(job_labels)
        pod_labels[lab.job_name_label] = rid
        spec = {"containers": [{"name": "algorithm", "image": "algo:latest", "env": env,
                                "resources": {"limits": gpu, "requests": gpu}}], "restartPolicy": "Never"}
        if running:
            spec["nodeName"] = node
            status = {"phase": "Running", "conditions": [{"type": "Ready", "status": "True"}],
                      "containerStatuses": [{"name": "algorithm", "ready": True, "restartCount": 0,
                                             "state": {"running": {"startedAt": _T0}}}]}
        else:
            status = {"phase": "Pending"}
        pod = {"apiVersion": "v1", "kind": "Pod",
               "metadata": {"name": f"{rid}-w0", "namespace": ns, "uid": f"pod-uid-{rid}-w0",
                            "resourceVersion": self._next_rv(), "creationTimestamp": _T0, "labels": pod_labels},
               "spec": spec, "status": status}
        now = _dt.datetime.now(_dt.timezone.utc)
        row = CheckpointedRequest(algorithm=self.algorithm, id=rid, lifecycle_stage=stage,
                                  payload_uri=f"s3://nexus/payloads/{rid}", received_by_host="receiver-0", received_at=now,
                                  sent_at=now, applied_configuration="{}", configuration_overrides="{}",
                                  content_hash=rid[:16], last_modified=now, tag="bench", api_version="1.3",
                                  job_uid=f"job-uid-{rid}", parent="{}", payload_valid_for="1h")
        self.pods[rid] = pod
        self.jobs[rid] = job
        return rid, job, pod, row

    def initial(self) -> Tuple[List[Dict[str, Any]], List[CheckpointedRequest]]:
        """The namespace at the start: ``concurrent_jobs`` running runs (rows RUNNING)."""
        objs, rows = [], []
        for _ in range(self.concurrent_jobs):
            rid, job, pod, row = self.new_run(LifecycleStage.RUNNING, running=True)
            self.live.append(rid)
            objs += [job, pod]
            rows.append(row)
        return objs, rows

    # ------------------------------------------------------------ run start
    def _create(self, st: StepTraffic) -> None:
        if self.run_starts:
            rid, job, pod, row = self.new_run()
            st.traffic.append(("ADDED", job))
            st.traffic.append(("ADDED", self._job_event(rid, "SuccessfulCreate", f"Created pod: {rid}-w0", "Normal")))
            st.traffic.append(("ADDED", pod))
            self.pending.append(rid)
        else:
            rid, job, pod, row = self.new_run(LifecycleStage.RUNNING)
            st.traffic += [("ADDED", job), ("ADDED", pod)]
            self.live.append(rid)
        st.rows.append(row)

    def _schedule(self, rid: str, out: List[Tuple[str, Dict[str, Any]]]) -> None:
        pod = self.pods[rid]
        node = self._templates()[4]
        out.append(("ADDED", self._pod_event(rid, "Scheduled",
                                             f"Successfully assigned {self.ns}/{pod['metadata']['name']} to {node}",
                                             component="default-scheduler")))
        pod = self.pods[rid] = self._mod(pod, {"phase": "Pending", "conditions": [
            {"type": "PodScheduled", "status": "True"}]}, spec={"nodeName": node})
        out.append(("MODIFIED", pod))
        out.append(("ADDED", self._pod_event(rid, "Pulling", 'Pulling image "algo:latest"')))

    def _start(self, rid: str, st: StepTraffic) -> None:
        out = st.traffic
        self._schedule(rid, out)
        out.append(("ADDED", self._pod_event(rid, "Pulled", 'Successfully pulled image "algo:latest" in 1.204s '
                                                            '(1.204s including waiting). Image size: 7340032000 bytes.')))
        out.append(("ADDED", self._pod_event(rid, "Created", "Created container algorithm")))
        out.append(("ADDED", self._pod_event(rid, "Started", "Started container algorithm")))
        pod = self.pods[rid] = self._mod(self.pods[rid], {
            "phase": "Running", "startTime": _T0,
            "conditions": [{"type": "PodScheduled", "status": "True"}, {"type": "Ready", "status": "True"}],
            "containerStatuses": [{"name": "algorithm", "ready": True, "restartCount": 0,
                                   "state": {"running": {"startedAt": _T0}}}]})
        out.append(("MODIFIED", pod))
        job = self.jobs[rid] = self._mod(self.jobs[rid], {"active": 1, "ready": 1, "startTime": _T0})
        out.append(("MODIFIED", job))
        st.started.append(rid)
        st.start_expected[rid] = LifecycleStage.RUNNING
        self.expected[rid] = LifecycleStage.RUNNING
        self.live.append(rid)

    # ------------------------------------------------------------ failures
    def _job_failed(self, rid: str, reason: str, message: str) -> Dict[str, Any]:
        job = self.jobs[rid] = self._mod(self.jobs[rid], {
            "failed": 1, "startTime": _T0,
            "conditions": [{"type": "FailureTarget", "status": "True", "reason": reason, "message": message},
                           {"type": "Failed", "status": "True", "reason": reason, "message": message}]})
        return job

    def _terminated(self, rid: str, state: Dict[str, Any], phase: str = "Failed") -> Dict[str, Any]:
        pod = self.pods[rid] = self._mod(self.pods[rid], {
            "phase": phase, "startTime": _T0,
            "conditions": [{"type": "PodScheduled", "status": "True"}, {"type": "Ready", "status": "False"}],
            "containerStatuses": [{"name": "algorithm", "ready": False, "restartCount": 0, "state": state}]})
        return pod

    def _fail(self, rid: str, kind: str, st: StepTraffic) -> None:
        out = st.traffic
        pod_name = self.pods[rid]["metadata"]["name"]
        if kind == "host-oom":
            out.append(("MODIFIED", self._terminated(rid, {"terminated": {"reason": "OOMKilled", "exitCode": 137,
                                                                          "message": ""}})))
            msg = (f"Container algorithm for pod {self.ns}/{pod_name} failed with exit code 137 matching FailJob rule "
                   "at index 0")
            out.append(("MODIFIED", self._job_failed(rid, "PodFailurePolicy", msg)))
            out.append(("ADDED", self._job_event(rid, "PodFailurePolicy", msg)))
        elif kind == "hbm-oom":
            default_pod = self.hbm_shape == "default-pod"
            if default_pod:
                # the container runtime has the process's stderr in the log before the kubelet
                # reports the container terminated
                out.append(("LOG", {"namespace": self.ns, "pod": pod_name, "container": "algorithm",
                                    "uid": self.pods[rid]["metadata"]["uid"],
                                    "text": f"epoch 3 step 1200 loss 0.412\n{self.hip_oom_message}\n"}))
            out.append(("MODIFIED", self._terminated(rid, {"terminated": {
                "reason": "Error", "exitCode": 1, "message": "" if default_pod else self.hip_oom_message}})))
            msg = "Job has reached the specified backoff limit"
            out.append(("MODIFIED", self._job_failed(rid, "BackoffLimitExceeded", msg)))
            out.append(("ADDED", self._job_event(rid, "BackoffLimitExceeded", msg)))
        elif kind == "image-pull":
            self._schedule(rid, out)
            img = f"registry.local/algo:{rid[:8]}"
            out.append(("ADDED", self._pod_event(rid, "Failed", f'Failed to pull image "{img}": rpc error: code = '
                                                                f'NotFound desc = manifest unknown', "Warning")))
            for reason, msg in (("ErrImagePull", f'rpc error: code = NotFound desc = failed to pull "{img}"'),
                                ("ImagePullBackOff", f'Back-off pulling image "{img}"')):
                pod = self.pods[rid] = self._mod(self.pods[rid], {
                    "phase": "Pending", "conditions": [{"type": "PodScheduled", "status": "True"}],
                    "containerStatuses": [{"name": "algorithm", "ready": False, "restartCount": 0,
                                           "state": {"waiting": {"reason": reason, "message": msg}}}]})
                out.append(("MODIFIED", pod))
                if reason == "ErrImagePull":
                    out.append(("ADDED", self._pod_event(rid, "BackOff", f'Back-off pulling image "{img}"', "Warning")))
        elif kind == "gpu-admission":
            # bound to a node whose GPU the device plugin marked unhealthy: the kubelet refuses
            # the pod at admission (Failed, no container ever created), the Job controller
            # counts the failure against backoffLimit 0
            node = self._templates()[4]
            out.append(("ADDED", self._pod_event(rid, "Scheduled", f"Successfully assigned {self.ns}/{pod_name} to {node}",
                                                 component="default-scheduler")))
            out.append(("MODIFIED", self._mod(self.pods[rid], {"phase": "Failed", "reason": "UnexpectedAdmissionError",
                                                                "message": GPU_ADMISSION_MESSAGE},
                                              spec={"nodeName": node})))
            out.append(("ADDED", self._pod_event(rid, "UnexpectedAdmissionError", GPU_ADMISSION_MESSAGE, "Warning")))
            msg = "Job has reached the specified backoff limit"
            out.append(("MODIFIED", self._job_failed(rid, "BackoffLimitExceeded", msg)))
            out.append(("ADDED", self._job_event(rid, "BackoffLimitExceeded", msg)))
        elif kind == "pod-failure-policy":
            if self.hbm_shape == "default-pod":
                # a default pod's log always exists: here a plain crash, nothing an OOM rule reads
                out.append(("LOG", {"namespace": self.ns, "pod": pod_name, "container": "algorithm",
                                    "uid": self.pods[rid]["metadata"]["uid"],
                                    "text": "Traceback (most recent call last):\n  File \"train.py\", line 212, in <module>\n"
                                            "RuntimeError: invalid dataset shard index\n"}))
            out.append(("MODIFIED", self._terminated(rid, {"terminated": {"reason": "Error", "exitCode": 255,
                                                                          "message": ""}})))
            msg = (f"Container algorithm for pod {self.ns}/{pod_name} failed with exit code 255 matching FailJob rule "
                   "at index 0")
            out.append(("ADDED", self._job_event(rid, "PodFailurePolicy", msg)))
            out.append(("MODIFIED", self._job_failed(rid, "PodFailurePolicy", msg)))
        elif kind == "deadline":
            msg = "Job was active longer than specified deadline"
            out.append(("ADDED", self._job_event(rid, "DeadlineExceeded", msg)))
            out.append(("MODIFIED", self._job_failed(rid, "DeadlineExceeded", msg)))
            out.append(("ADDED", self._pod_event(rid, "Killing", "Stopping container algorithm")))
            pod = self.pods[rid] = self._mod(self.pods[rid], self.pods[rid]["status"],
                                             meta={"deletionTimestamp": _T0, "deletionGracePeriodSeconds": 30})
            out.append(("MODIFIED", pod))
        else:  # evicted
            msg = "The node was low on resource: memory. Threshold quantity: 100Mi, available: 60Mi."
            pod = self.pods[rid] = self._mod(self.pods[rid], {
                "phase": "Failed", "reason": "Evicted", "message": msg,
                "conditions": [{"type": "DisruptionTarget", "status": "True", "reason": "TerminationByKubelet",
                                "message": msg}]})
            out.append(("MODIFIED", pod))
            out.append(("ADDED", self._pod_event(rid, "Evicted", msg, "Warning")))
            jmsg = "Job has reached the specified backoff limit"
            out.append(("MODIFIED", self._job_failed(rid, "BackoffLimitExceeded", jmsg)))
            out.append(("ADDED", self._job_event(rid, "BackoffLimitExceeded", jmsg)))
        st.failed.append(rid)
        st.expected[rid] = self.expected[rid] = self._stage[kind]
        self.kind_of[rid] = kind
        st.kinds[rid] = kind
        # the supervisor's Job DELETE removes the Job and (GC) its pod; its Events expire later
        self.pods.pop(rid, None)
        self.jobs.pop(rid, None)
        evs = self.events.pop(rid, None)
        if evs:
            self._expiring[-1].extend(evs)

    def expire_all(self) -> List[Tuple[str, Dict[str, Any]]]:
        """Every Event still waiting for its TTL, as DELETED lines, now (the latency probe
        lets the saturated steps' Events expire before its first arrival instead of in it)."""
        out: List[Tuple[str, Dict[str, Any]]] = []
        while self._expiring:
            out.extend(("DELETED", ev) for ev in self._expiring.popleft())
        return out

    def fail_with(self, kind: str, message: Optional[str] = None, rid: Optional[str] = None) -> StepTraffic:
        """One running run (``rid``, else a random one) fails as ``kind`` (``message``: the
        HIP text of an hbm-oom, e.g. a real OOM's); its replacement is created."""
        st = StepTraffic()
        if rid is None:
            rid = self.live.pop(self.rng.randrange(len(self.live)))
        else:
            self.live.remove(rid)
        if not self._expiring:
            self._expiring.append([])
        saved = self.hip_oom_message
        if message:
            self.hip_oom_message = message
        try:
            self._fail(rid, kind, st)
        finally:
            self.hip_oom_message = saved
        self._create(st)
        return st

    def create(self, n: int) -> StepTraffic:
        """``n`` new runs (Job + Pending Pod ADDED, rows BUFFERED) that start — or fail to
        start (image-pull, gpu-admission) — in the next :meth:`step`."""
        st = StepTraffic()
        for _ in range(n):
            self._create(st)
        return st

    def step(self, events: int, kinds: Optional[List[str]] = None) -> StepTraffic:
        """Fail ``events`` runs, start last step's new runs, create ``events`` new ones.
        ``kinds`` restricts the failure mix (uniform over the given kinds)."""
        st = StepTraffic()
        # the Events of runs that failed two steps ago expire (TTL)
        while len(self._expiring) >= 2:
            for ev in self._expiring.popleft():
                st.traffic.append(("DELETED", ev))
        self._expiring.append([])
        rng = self.rng
        if kinds:
            chosen = rng.choices(list(kinds), k=events)
        else:
            chosen = rng.choices(self._kinds, self._weights, k=events)
        # start failures need a starting run: at most one per pending run, the rest fail running runs
        start_fail = [k for k in chosen if k in START_KINDS][:len(self.pending)]
        run_fail = [k for k in chosen if k not in START_KINDS]
        missing = events - len(start_fail) - len(run_fail)
        if missing > 0:
            allowed = [k for k in (kinds or ()) if k not in START_KINDS]
            run_fail += (rng.choices(allowed, k=missing) if allowed
                         else rng.choices(self._run_kinds, self._run_weights, k=missing))
        n = min(len(run_fail), len(self.live))
        idx = rng.sample(range(len(self.live)), n)
        picked = [self.live[i] for i in idx]
        dead = set(picked)
        self.live = [r for r in self.live if r not in dead]
        for rid, kind in zip(picked, run_fail):
            self._fail(rid, kind, st)
        # last step's new runs: some fail to start, the others start
        starting, self.pending = self.pending, []
        bad = set(rng.sample(range(len(starting)), len(start_fail))) if start_fail else set()
        ki = iter(start_fail)
        for i, rid in enumerate(starting):
            if i in bad:
                self._fail(rid, next(ki), st)
            else:
                self._start(rid, st)
        for _ in range(len(st.failed)):
            self._create(st)
        return st
