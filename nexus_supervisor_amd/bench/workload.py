"""Synthetic pod-failure workload for the north-star benchmark (BASELINE.json:
"pod-fail→checkpoint p50/p99 latency + events/sec at 10k concurrent jobs",
synthetic pod-failure events with random job IDs).

A :class:`Workload` owns a pool of ``concurrent_jobs`` live Nexus runs (Job + Pod
objects with torchrun/RCCL env for one MI355X GPU-job slot, plus a RUNNING
checkpoint row each).  :meth:`Workload.step` picks ``events`` random live runs,
produces the watch traffic of their failure, and replaces each failed run with a
fresh one (ADDED Job + Pod, new checkpoint row) so the concurrency stays
constant — the churn is part of what the supervisor's informers must absorb.

Failure mix (one decisive signal per run; every one must end in a checkpoint write):

=================  ==========================================================  ==================
kind               watch traffic                                               expected stage
=================  ==========================================================  ==================
host-oom           Pod MODIFIED: terminated OOMKilled, exit 137                FAILED
hbm-oom            Pod MODIFIED: exit 1 + HIP OOM message (real one from the    FAILED
                   rank's GPU when available)
image-pull         Pod MODIFIED: waiting ImagePullBackOff                      SCHEDULING_FAILED
pod-failure-policy Event ADDED (Job, PodFailurePolicy) — reference R-EVT path  FAILED
deadline           Event ADDED (Job, DeadlineExceeded) — reference R-EVT path  DEADLINE_EXCEEDED
evicted            Pod MODIFIED (Evicted) then Job MODIFIED (Failed condition,  DEADLINE_EXCEEDED
                   BackoffLimitExceeded)
=================  ==========================================================  ==================
"""
from __future__ import annotations

import datetime as _dt
import random
import uuid
from typing import Any, Dict, List, Optional, Tuple

from ..config.schema import LabelConfig
from ..models.checkpoint import CheckpointedRequest, LifecycleStage
from ..parallel.sharding import shard_of as _shard_of
from ..testing.seed import make_event, make_job, make_pod, run_labels

DEFAULT_HIP_OOM = ("hipErrorOutOfMemory: HIP out of memory. Tried to allocate 4.00 GiB. GPU 0 has a total capacity of "
                   "287.98 GiB; 284.00 GiB already allocated by this process")

MIX: Tuple[Tuple[str, float, str], ...] = (
    ("host-oom", 0.30, LifecycleStage.FAILED),
    ("hbm-oom", 0.20, LifecycleStage.FAILED),
    ("image-pull", 0.20, LifecycleStage.SCHEDULING_FAILED),
    ("pod-failure-policy", 0.10, LifecycleStage.FAILED),
    ("deadline", 0.10, LifecycleStage.DEADLINE_EXCEEDED),
    ("evicted", 0.10, LifecycleStage.DEADLINE_EXCEEDED),
)


def shard_of(algorithm: str, request_id: str, shards: int) -> int:
    """Replica shard of a run, as ``Supervisor.owns`` computes it (``parallel/sharding.py``)."""
    return _shard_of(request_id, shards)


class Workload:
    def __init__(self, concurrent_jobs: int = 10_000, rank: int = 0, world: int = 1, seed: int = 0,
                 labels: Optional[LabelConfig] = None, namespace: str = "nexus", algorithm: str = "bench-algorithm",
                 hip_oom_message: str = DEFAULT_HIP_OOM, gpus_per_node: int = 8, shards: int = 1, shard_index: int = 0,
                 shard_label: str = "", hbm_shape: str = "termination-message"):
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
        # sharding.shard-label: the submitter stamps each run's shard on its Job and pod template
        self.shard_label = shard_label if shards > 1 else ""
        self.live: List[str] = []
        self.pods: Dict[str, Dict[str, Any]] = {}
        self.jobs: Dict[str, Dict[str, Any]] = {}
        self.expected: Dict[str, str] = {}
        self.kind_of: Dict[str, str] = {}  # failed run → failure kind (diagnostics)
        self._rv = 1000
        self._seq = 0
        self.concurrent_jobs = concurrent_jobs
        self._kinds = [k for k, _, _ in MIX]
        self._weights = [w for _, w, _ in MIX]
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
                "MASTER_PORT": "29500", "HIP_VISIBLE_DEVICES": ",".join(str(i) for i in range(self.gpus_per_node)),
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

    def new_run(self) -> Tuple[str, Dict[str, Any], Dict[str, Any], CheckpointedRequest]:
        rid = self._new_id()
        env_t, mi, gpu, job_labels, node = self._templates()
        ns, lab = self.ns, self.labels
        if self.shard_label:
            job_labels = dict(job_labels, **{self.shard_label: str(self.shard_index)})
        job = {"apiVersion": "batch/v1", "kind": "Job",
               "metadata": {"name": rid, "namespace": ns, "uid": f"job-uid-{rid}", "resourceVersion": self._next_rv(),
                            "labels": dict(job_labels)},
               "spec": {}, "status": {"active": 1}}
        env = list(env_t)
        env[mi] = {"name": "MASTER_ADDR", "value": f"{rid[:8]}-0.nexus-headless"}
        pod_labels = dict(job_labels)
        pod_labels[lab.job_name_label] = rid
        pod = {"apiVersion": "v1", "kind": "Pod",
               "metadata": {"name": f"{rid}-w0", "namespace": ns, "uid": f"pod-uid-{rid}-w0",
                            "resourceVersion": self._next_rv(), "labels": pod_labels},
               "spec": {"containers": [{"name": "algorithm", "image": "algo:latest", "env": env,
                                        "resources": {"limits": gpu, "requests": gpu}}], "nodeName": node},
               "status": {"phase": "Pending"}}
        now = _dt.datetime.now(_dt.timezone.utc)
        row = CheckpointedRequest(algorithm=self.algorithm, id=rid, lifecycle_stage=LifecycleStage.RUNNING,
                                  payload_uri=f"s3://nexus/payloads/{rid}", received_by_host="receiver-0", received_at=now,
                                  sent_at=now, applied_configuration="{}", configuration_overrides="{}",
                                  content_hash=rid[:16], last_modified=now, tag="bench", api_version="1.3",
                                  job_uid=f"job-uid-{rid}", parent="{}", payload_valid_for="1h")
        self.live.append(rid)
        self.pods[rid] = pod
        self.jobs[rid] = job
        return rid, job, pod, row

    def initial(self) -> Tuple[List[Dict[str, Any]], List[CheckpointedRequest]]:
        objs, rows = [], []
        for _ in range(self.concurrent_jobs):
            _, job, pod, row = self.new_run()
            objs += [job, pod]
            rows.append(row)
        return objs, rows

    # ------------------------------------------------------------ failures
    def _fail(self, rid: str, kind: str) -> List[Tuple[str, Dict[str, Any]]]:
        pod = self.pods.pop(rid)
        job = self.jobs.pop(rid)
        out: List[Tuple[str, Dict[str, Any]]] = []
        if kind in ("host-oom", "hbm-oom", "image-pull", "evicted"):
            p = dict(pod)
            p["metadata"] = dict(pod["metadata"], resourceVersion=self._next_rv())
            if kind == "host-oom":
                st = {"terminated": {"reason": "OOMKilled", "exitCode": 137, "message": ""}}
                status = {"phase": "Failed", "containerStatuses": [{"name": "algorithm", "state": st, "restartCount": 0}]}
            elif kind == "hbm-oom":
                default_pod = self.hbm_shape == "default-pod"
                st = {"terminated": {"reason": "Error", "exitCode": 1,
                                     "message": "" if default_pod else self.hip_oom_message}}
                status = {"phase": "Failed", "containerStatuses": [{"name": "algorithm", "state": st, "restartCount": 0}]}
                if default_pod:
                    out.append(("LOG", {"namespace": self.ns, "pod": pod["metadata"]["name"], "container": "algorithm",
                                        "text": f"epoch 3 step 1200 loss 0.412\n{self.hip_oom_message}\n"}))
            elif kind == "image-pull":
                st = {"waiting": {"reason": "ImagePullBackOff",
                                  "message": f'Back-off pulling image "registry.local/algo:{rid[:8]}"'}}
                status = {"phase": "Pending", "containerStatuses": [{"name": "algorithm", "state": st, "restartCount": 0}]}
            else:
                status = {"phase": "Failed", "reason": "Evicted",
                          "message": "The node was low on resource: memory. Threshold quantity: 100Mi, available: 60Mi."}
            p["status"] = status
            out.append(("MODIFIED", p))
            if kind == "evicted":
                j = dict(job)
                j["metadata"] = dict(job["metadata"], resourceVersion=self._next_rv())
                j["status"] = {"failed": 1, "conditions": [{"type": "Failed", "status": "True", "reason": "BackoffLimitExceeded",
                                                            "message": "Job has reached the specified backoff limit"}]}
                out.append(("MODIFIED", j))
        elif kind == "pod-failure-policy":
            out.append(("ADDED", make_event("Job", rid, "PodFailurePolicy", ns=self.ns,
                                            message="Container algorithm for pod nexus/" + rid + "-w0 failed with exit code 137 matching FailJob rule at index 0")))
        elif kind == "deadline":
            out.append(("ADDED", make_event("Job", rid, "DeadlineExceeded", ns=self.ns,
                                            message="Job was active longer than specified deadline")))
        self.expected[rid] = self._stage[kind]
        self.kind_of[rid] = kind
        return out

    def step(self, events: int, kinds: Optional[List[str]] = None
             ) -> Tuple[List[str], List[Tuple[str, Dict[str, Any]]], List[CheckpointedRequest]]:
        """Fail ``events`` random live runs; returns (failed ids, watch traffic, new rows).
        ``kinds`` restricts the failure mix (uniform over the given kinds)."""
        traffic: List[Tuple[str, Dict[str, Any]]] = []
        failed: List[str] = []
        rows: List[CheckpointedRequest] = []
        n = min(events, len(self.live))
        idx = self.rng.sample(range(len(self.live)), n)
        picked = [self.live[i] for i in idx]
        dead = set(picked)
        self.live = [r for r in self.live if r not in dead]
        if kinds:
            chosen = self.rng.choices(list(kinds), k=n)
        else:
            chosen = self.rng.choices(self._kinds, self._weights, k=n)
        for rid, kind in zip(picked, chosen):
            traffic += self._fail(rid, kind)
            failed.append(rid)
            _, job, pod, row = self.new_run()
            traffic += [("ADDED", job), ("ADDED", pod)]
            rows.append(row)
        return failed, traffic, rows
