"""``python -m nexus_supervisor_amd explain FILE|-``: what the supervisor would decide for
a set of Kubernetes objects, and why — offline, with the effective configuration.

Input is what ``kubectl get … -o json`` prints: one object, a ``List``, or several JSON
documents one after another (e.g. ``kubectl get pod,job,events -l <run> -o json``).
Every Event, Pod and Job is run through the same classifier the supervisor uses
(reference event table, pod/job status rules, GPU enrichment from the node agent's
``nexus.amd.com/gpu-evidence`` annotation when the pod carries it); Events resolve
their involved object among the objects given, as the informer caches would.  For each
decision it prints the action, the lifecycle stage, the failure class, the exact
``algorithm_failure_cause`` and ``algorithm_failure_details`` the checkpoint write would
carry, and the OOM verdict's signals — the question an operator asks about a run the
supervisor marked FAILED ("why HBM-OOM, on which GPU?").

The reference has no such tool; its decision logic (``/root/reference/services/
supervisor.go:137-259``) is only observable by running it against a cluster.
"""
from __future__ import annotations

import json
import sys
from typing import Any, Dict, Iterable, List, Optional

from .classify import reference_rules as R
from .classify.classifier import STALE, Classifier, ObjectLookup, render_trace
from .config.schema import SupervisorConfig
from .models import kube
from .models.decisions import DecisionAction as A


class _Objects(ObjectLookup):
    def __init__(self, objs: Iterable[Dict[str, Any]], job_label: str):
        self.by = {(o.get("kind"), kube.name_of(o)): o for o in objs}
        self.job_label = job_label

    def get(self, kind: str, name: str) -> Optional[Dict[str, Any]]:
        return self.by.get((kind, name))

    def pods_of_job(self, job_name: str) -> List[Dict[str, Any]]:
        return [o for (k, _n), o in self.by.items() if k == "Pod" and kube.labels_of(o).get(self.job_label) == job_name]


def parse_objects(text: str) -> List[Dict[str, Any]]:
    """Kubernetes objects from ``kubectl -o json`` output (object, List, or a stream of
    documents); a List's items get their kind from ``<Kind>List`` when they lack one."""
    dec = json.JSONDecoder()
    out: List[Dict[str, Any]] = []
    i, n = 0, len(text)
    while i < n:
        while i < n and text[i].isspace():
            i += 1
        if i >= n:
            break
        doc, i = dec.raw_decode(text, i)
        stack = [doc]
        while stack:
            d = stack.pop(0)
            if not isinstance(d, dict):
                continue
            if isinstance(d.get("items"), list):
                kind = d.get("kind", "")
                item_kind = kind[:-4] if kind.endswith("List") and kind != "List" else ""
                for it in d["items"]:
                    if isinstance(it, dict) and item_kind and not it.get("kind"):
                        it = dict(it, kind=item_kind)
                    stack.append(it)
            elif d.get("kind") in ("Event", "Pod", "Job"):
                out.append(d)
    return out


def explain(objs: List[Dict[str, Any]], cfg: SupervisorConfig) -> List[Dict[str, Any]]:
    """One record per classified object: ``status`` (decided / stale / noop / ignored /
    deferred / evidence) and, for decisions, what the checkpoint write would carry."""
    from .supervisor import STAGE_FOR_ACTION

    cfg.stages.apply()
    c = Classifier(cfg.labels, cfg.rules, cfg.gpu)
    look = _Objects(objs, cfg.labels.job_name_label)
    # Pods and Jobs first (their status is evidence for what follows), then Events in time order
    order = sorted(objs, key=lambda o: (o.get("kind") == "Event", str(o.get("lastTimestamp") or o.get("eventTime") or "")))
    out: List[Dict[str, Any]] = []
    for o in order:
        kind = o.get("kind")
        rec: Dict[str, Any] = {"object": f"{kind}/{kube.name_of(o)}"}
        if kind == "Event":
            rec["reason"] = o.get("reason", "")
            status, results = c.classify_event(o, look)
            if status == STALE:
                rec["note"] = "involved object not among the inputs (the supervisor would park the event)"
        elif kind == "Pod":
            results = c.classify_pod(o, None)
            status = "decided" if results else ("deferred" if c.deferred else "noop")
        else:
            results = c.classify_job(o, None, look)
            status = "decided" if results else "noop"
        rec["status"] = status
        decisions = []
        for r in results:
            if r.action != A.TO_RUNNING:
                c.late_enrich(r, look)
            d: Dict[str, Any] = {"request_id": r.request_id, "algorithm": r.algorithm, "action": r.action,
                                 "lifecycle_stage": STAGE_FOR_ACTION[r.action](), "failure_class": r.failure_class,
                                 "reason": r.reason, "delete_job": r.action != A.TO_RUNNING}
            if r.action != A.TO_RUNNING:
                d["algorithm_failure_cause"] = R.failure_cause(r.action, r.run_status_message,
                                                               cfg.compat.doubled_fatal_cause)
                d["algorithm_failure_details"] = render_trace(r, cfg.rules.trace_format, cfg.rules.trace_max_bytes)
            for k in ("oom", "ranks"):  # the OOM verdict's signals; a multi-rank job's culprit
                if r.evidence.get(k):
                    d[k] = r.evidence[k]
            decisions.append(d)
        if decisions:
            rec["decisions"] = decisions
        out.append(rec)
    return out


def main(argv: List[str]) -> int:
    from .config import load_config

    if len(argv) != 1:
        print("usage: python -m nexus_supervisor_amd explain FILE|-   (kubectl get … -o json output)", file=sys.stderr)
        return 2
    text = sys.stdin.read() if argv[0] == "-" else open(argv[0]).read()
    cfg = load_config()
    print(json.dumps(explain(parse_objects(text), cfg), indent=2, default=str))
    return 0
