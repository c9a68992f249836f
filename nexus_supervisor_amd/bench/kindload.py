"""BASELINE.json config 2 on a real cluster: "kind cluster, 100 synthetic failing pods
(OOMKilled/ImagePullBackOff mix), 1 supervisor replica, local Scylla".

Generates Nexus-labelled ``batch/v1`` Jobs whose pods really fail, seeds their
BUFFERED checkpoint rows, and then polls the rows until the supervisor has moved
every one to its failed stage, reporting apply → checkpoint latency:

=============  ==========================================================  ==================
kind           how it fails on a real kubelet                              expected stage
=============  ==========================================================  ==================
host-oom       busybox ``tail /dev/zero`` under a 24 Mi memory limit:       FAILED
               OOMKilled, exit 137 → Job ``podFailurePolicy`` FailJob
image-pull     image from a non-resolvable registry: ErrImagePull /         SCHEDULING_FAILED
               ImagePullBackOff
=============  ==========================================================  ==================

    python -m nexus_supervisor_amd.bench.kindload manifests --pods 100 > jobs.yaml
    python -m nexus_supervisor_amd.bench.kindload seed --cql 127.0.0.1:9042 --pods 100
    kubectl apply -f jobs.yaml && python -m nexus_supervisor_amd.bench.kindload wait --cql 127.0.0.1:9042 --pods 100

Ids are derived from ``--seed`` so the three steps agree without shared state.
``deploy/kind/run-config2.sh`` strings them together.
"""
from __future__ import annotations

import argparse
import asyncio
import datetime as _dt
import json
import random
import sys
import time
import uuid
from typing import Any, Dict, List, Tuple

from ..config.schema import LabelConfig
from ..models.checkpoint import CheckpointedRequest, LifecycleStage
from ..testing.seed import run_labels

KINDS = (("host-oom", LifecycleStage.FAILED), ("image-pull", LifecycleStage.SCHEDULING_FAILED))
ALGORITHM = "kind-load"


def runs(n: int, seed: int = 0) -> List[Tuple[str, str]]:
    """``n`` (request id, kind) pairs, alternating kinds, random v4 ids."""
    rng = random.Random(seed)
    return [(str(uuid.UUID(int=rng.getrandbits(128), version=4)), KINDS[i % len(KINDS)][0]) for i in range(n)]


def job_manifest(rid: str, kind: str, labels: LabelConfig, namespace: str = "nexus") -> Dict[str, Any]:
    container: Dict[str, Any] = {"name": "algorithm", "imagePullPolicy": "IfNotPresent"}
    if kind == "host-oom":
        container.update(image="busybox:1.36", command=["sh", "-c", "tail /dev/zero"],
                         resources={"limits": {"memory": "24Mi"}, "requests": {"memory": "24Mi"}})
    else:
        container.update(image=f"registry.nexus.invalid/algorithms/{rid[:8]}:0", imagePullPolicy="Always")
    pod_labels = run_labels(labels, ALGORITHM)
    return {
        "apiVersion": "batch/v1", "kind": "Job",
        "metadata": {"name": rid, "namespace": namespace, "labels": run_labels(labels, ALGORITHM)},
        "spec": {
            "backoffLimit": 0,
            "activeDeadlineSeconds": 600,
            "ttlSecondsAfterFinished": 600,
            # how nexus turns OOM exit codes into a Job failure (PodFailurePolicy)
            "podFailurePolicy": {"rules": [{"action": "FailJob", "onExitCodes": {
                "containerName": "algorithm", "operator": "In", "values": [137, 255]}}]},
            "template": {
                "metadata": {"labels": pod_labels},
                "spec": {"restartPolicy": "Never", "containers": [container]},
            },
        },
    }


def manifests(n: int, seed: int = 0, namespace: str = "nexus", labels: LabelConfig = None) -> List[Dict[str, Any]]:
    labels = labels or LabelConfig()
    return [job_manifest(rid, kind, labels, namespace) for rid, kind in runs(n, seed)]


def to_yaml(docs: List[Dict[str, Any]]) -> str:
    # JSON is valid YAML; one document per object keeps kubectl happy
    return "".join("---\n" + json.dumps(d, indent=1) + "\n" for d in docs)


def rows(n: int, seed: int = 0) -> List[CheckpointedRequest]:
    now = _dt.datetime.now(_dt.timezone.utc)
    return [CheckpointedRequest(algorithm=ALGORITHM, id=rid, lifecycle_stage=LifecycleStage.BUFFERED,
                                payload_uri=f"s3://nexus/payloads/{rid}", received_by_host="kindload", received_at=now,
                                sent_at=now, applied_configuration="{}", configuration_overrides="{}",
                                content_hash=rid[:16], last_modified=now, tag="kindload", api_version="1.3",
                                job_uid="", parent="{}", payload_valid_for="1h")
            for rid, _ in runs(n, seed)]


def expected(n: int, seed: int = 0) -> Dict[str, str]:
    stage = dict(KINDS)
    return {rid: stage[kind] for rid, kind in runs(n, seed)}


async def _store(cql: str):
    from ..store.cql import CqlCheckpointStore, CqlSession

    host, _, port = cql.partition(":")
    st = CqlCheckpointStore(CqlSession([(host, int(port or 9042))]))
    await st.connect()
    return st


async def seed_rows(cql: str, n: int, seed: int = 0) -> int:
    st = await _store(cql)
    try:
        rs = rows(n, seed)
        await asyncio.gather(*(st.upsert_checkpoint(r) for r in rs))
        return len(rs)
    finally:
        await st.close()


async def wait_rows(cql: str, n: int, seed: int = 0, timeout: float = 600.0, t_apply: float = 0.0) -> Dict[str, Any]:
    """Poll until every run is in its expected stage; latency = row ``last_modified`` −
    ``t_apply`` (wall clock of the ``kubectl apply``)."""
    st = await _store(cql)
    exp = expected(n, seed)
    done: Dict[str, float] = {}
    wrong: Dict[str, str] = {}
    deadline = time.monotonic() + timeout
    try:
        while len(done) + len(wrong) < len(exp) and time.monotonic() < deadline:
            for rid, stage in exp.items():
                if rid in done or rid in wrong:
                    continue
                r = await st.read_checkpoint(ALGORITHM, rid)
                if r is None or r.lifecycle_stage == LifecycleStage.BUFFERED:
                    continue
                if r.lifecycle_stage == stage:
                    done[rid] = r.last_modified.timestamp() if r.last_modified else time.time()
                else:
                    wrong[rid] = r.lifecycle_stage
            await asyncio.sleep(0.5)
    finally:
        await st.close()
    lat = sorted((t - t_apply) * 1000.0 for t in done.values()) if t_apply else []
    q = (lambda p: round(lat[min(len(lat) - 1, int(round(p * (len(lat) - 1))))], 1)) if lat else (lambda p: None)
    return {"runs": len(exp), "in_expected_stage": len(done), "wrong_stage": wrong, "missing": len(exp) - len(done) - len(wrong),
            "apply_to_checkpoint_p50_ms": q(0.5), "apply_to_checkpoint_p99_ms": q(0.99)}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("command", choices=("manifests", "seed", "wait"))
    ap.add_argument("--pods", type=int, default=100)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--namespace", default="nexus")
    ap.add_argument("--cql", default="127.0.0.1:9042")
    ap.add_argument("--timeout", type=float, default=600.0)
    ap.add_argument("--t-apply", type=float, default=0.0, help="epoch seconds of the kubectl apply (latency origin)")
    args = ap.parse_args(argv)
    if args.command == "manifests":
        sys.stdout.write(to_yaml(manifests(args.pods, args.seed, args.namespace)))
        return 0
    if args.command == "seed":
        print(json.dumps({"seeded": asyncio.run(seed_rows(args.cql, args.pods, args.seed))}))
        return 0
    res = asyncio.run(wait_rows(args.cql, args.pods, args.seed, args.timeout, args.t_apply))
    print(json.dumps(res))
    return 0 if not res["wrong_stage"] and not res["missing"] else 1


if __name__ == "__main__":
    sys.exit(main())
