"""Mutating admission webhook that stamps ``sharding.shard-label`` on Nexus runs.

With ``sharding.shard-label`` each replica watches only its shards' Pods and Jobs
(``<label> in (owned…)``, filtered by the API server's watch cache), so N replicas on one
namespace do not each decode the whole stream.  That needs the label on every Nexus Job and
its pods — and no Nexus component stamps it: the reference scales by adding replicas with
no cooperation from the submitter at all (``/root/reference/.helm/values.yaml:124-125``).
This webhook, served by the supervisor itself (``sharding.webhook-port``), adds it at
admission:

* **Job CREATE** — ``metadata.labels[<label>]`` and ``spec.template.metadata.labels[<label>]``
  = ``shard_of(job name, shards)`` (the pod template is immutable afterwards, so this is
  the moment);
* **Pod CREATE** — ``metadata.labels[<label>]`` from the pod's
  ``batch.kubernetes.io/job-name`` label (pods of Jobs created before the webhook existed,
  or by a controller that copies labels selectively).

A Job created with ``generateName`` and no name has no shard yet: it is admitted
unchanged (``nexus_webhook_admissions{result="no-name"}``) and the replicas' audit
(``shard_label_missing``) reports it.  The chart registers the webhook with
``failurePolicy: Ignore``: an unreachable webhook never blocks a submission.

**When ``sharding.shards`` changes** every existing label is computed for the old count.
Each replica therefore runs :func:`relabel_owned` at startup: one LIST of the namespace's
Nexus Jobs and Pods, a merge PATCH of the label on every run of *its own* shards whose
label differs — replicas fix disjoint sets, together all of them.  Until it finishes a
run may be invisible to its new owner (the audit counts it); a run mid-flight keeps its
pods, so nothing is lost, only decided after the re-label.

Served over TLS from a Secret's ``tls.crt`` / ``tls.key`` (``sharding.webhook-cert-dir``);
without them (tests, dev) plain HTTP with a warning.
"""
from __future__ import annotations

import base64
import json
import logging
import os
import ssl
from typing import Any, Dict, List, Optional

from .parallel.sharding import shard_of

log = logging.getLogger("nexus_supervisor_amd.admission")
PATH = "/mutate-shard-label"


def _pointer(key: str) -> str:
    """RFC 6901 escaping of one path segment (label keys contain '/')."""
    return key.replace("~", "~0").replace("/", "~1")


def _label_ops(base: str, labels: Optional[Dict[str, str]], key: str, value: str) -> List[Dict[str, Any]]:
    if labels is None:
        return [{"op": "add", "path": base, "value": {key: value}}]
    if labels.get(key) == value:
        return []
    return [{"op": "replace" if key in labels else "add", "path": f"{base}/{_pointer(key)}", "value": value}]


def shard_label_patch(obj: Dict[str, Any], cfg) -> Optional[List[Dict[str, Any]]]:
    """JSON Patch that stamps the shard label on a Nexus Job (and its pod template) or
    Pod; ``[]`` when nothing is to change, None when the object has no shard yet."""
    s = cfg.sharding
    kind = obj.get("kind")
    meta = obj.get("metadata") or {}
    labels = meta.get("labels")
    if kind == "Job":
        name = meta.get("name") or ""
    elif kind == "Pod":
        name = (labels or {}).get(cfg.labels.job_name_label) or ""
    else:
        return []
    if not name:
        return None
    value = str(shard_of(name, max(1, s.shards)))
    ops = _label_ops("/metadata/labels", labels, s.shard_label, value)
    if kind == "Job":
        tmpl = (obj.get("spec") or {}).get("template")
        if isinstance(tmpl, dict):
            tmeta = tmpl.get("metadata")
            if tmeta is None:
                ops.append({"op": "add", "path": "/spec/template/metadata", "value": {"labels": {s.shard_label: value}}})
            else:
                ops += _label_ops("/spec/template/metadata/labels", tmeta.get("labels"), s.shard_label, value)
    return ops


def review(doc: Dict[str, Any], cfg, metrics=None) -> Dict[str, Any]:
    """AdmissionReview (admission.k8s.io/v1) in, AdmissionReview with the response out.
    Always allows: the webhook only adds a label, it never vetoes a submission."""
    req = doc.get("request") or {}
    resp: Dict[str, Any] = {"uid": req.get("uid", ""), "allowed": True}
    result = "unchanged"
    obj = req.get("object") or {}
    if req.get("operation", "CREATE") == "CREATE" and cfg.sharding.shard_label and cfg.sharding.shards > 1:
        if "kind" not in obj and req.get("kind"):
            obj = dict(obj, kind=(req.get("kind") or {}).get("kind"))
        lab = (obj.get("metadata") or {}).get("labels") or {}
        nexus = lab.get(cfg.labels.nexus_component_label) == cfg.labels.algorithm_run_value
        ops = shard_label_patch(obj, cfg) if nexus else []
        if ops is None:
            result = "no-name"
        elif ops:
            resp["patchType"] = "JSONPatch"
            resp["patch"] = base64.b64encode(json.dumps(ops, separators=(",", ":")).encode()).decode()
            result = "patched"
        elif not nexus:
            result = "not-nexus"
    if metrics is not None:
        metrics.inc("webhook_admissions", labels={"result": result, "kind": str(obj.get("kind") or "")})
    return {"apiVersion": doc.get("apiVersion", "admission.k8s.io/v1"), "kind": "AdmissionReview", "response": resp}


def server_ssl_context(cert_dir: str) -> Optional[ssl.SSLContext]:
    crt, key = os.path.join(cert_dir, "tls.crt"), os.path.join(cert_dir, "tls.key")
    if not (cert_dir and os.path.exists(crt) and os.path.exists(key)):
        return None
    ctx = ssl.create_default_context(ssl.Purpose.CLIENT_AUTH)
    ctx.minimum_version = ssl.TLSVersion.TLSv1_2
    ctx.load_cert_chain(crt, key)
    return ctx


class WebhookServer:
    """``POST /mutate-shard-label`` (AdmissionReview v1) and ``GET /healthz``."""

    def __init__(self, cfg, metrics=None):
        self.cfg = cfg
        self.metrics = metrics
        self.runner = None
        self.port = 0
        self.tls = False

    async def start(self, host: str, port: int, cert_dir: str = "") -> int:
        from aiohttp import web

        async def h_review(request):
            try:
                doc = await request.json()
            except ValueError:
                return web.json_response({"error": "bad AdmissionReview"}, status=400)
            return web.json_response(review(doc, self.cfg, self.metrics))

        async def h_healthz(_request):
            return web.Response(text="ok")

        app = web.Application(client_max_size=4 << 20)
        app.router.add_post(PATH, h_review)
        app.router.add_get("/healthz", h_healthz)
        self.runner = web.AppRunner(app, access_log=None)
        await self.runner.setup()
        ctx = server_ssl_context(cert_dir)
        self.tls = ctx is not None
        if not self.tls:
            log.warning("shard-label webhook serving plain HTTP (no tls.crt / tls.key in %r): the API server "
                        "only calls HTTPS webhooks", cert_dir)
        site = web.TCPSite(self.runner, host, port, ssl_context=ctx)
        await site.start()
        self.port = site._server.sockets[0].getsockname()[1]  # noqa: SLF001
        return self.port

    async def stop(self) -> None:
        if self.runner is not None:
            await self.runner.cleanup()
            self.runner = None


async def relabel_owned(cfg, kube, owned, metrics=None, log_=None, page: int = 500) -> Dict[str, int]:
    """Re-label this replica's runs whose shard label differs from ``shard_of(job name,
    shards)`` (after ``sharding.shards`` changed): Jobs by name, Pods by their job-name
    label.  ``owned``: this replica's shard set (None = every shard).  Returns counts."""
    from .kube.client import resource_path

    s = cfg.sharding
    out = {"checked": 0, "relabelled": 0, "errors": 0}
    if not s.shard_label or s.shards <= 1:
        return out
    sel = f"{cfg.labels.nexus_component_label}={cfg.labels.algorithm_run_value}"
    for kind in ("Job", "Pod"):
        cont = ""
        while True:
            params = {"labelSelector": sel, "limit": str(page)}
            if cont:
                params["continue"] = cont
            doc = await kube.request("GET", resource_path(kind, cfg.resource_namespace), params=params)
            for item in doc.get("items") or ():
                meta = item.get("metadata") or {}
                lab = meta.get("labels") or {}
                name = meta.get("name", "") if kind == "Job" else lab.get(cfg.labels.job_name_label, "")
                if not name:
                    continue
                want = shard_of(name, s.shards)
                if owned is not None and want not in owned:
                    continue
                out["checked"] += 1
                if lab.get(s.shard_label) == str(want):
                    continue
                try:
                    await kube.patch_merge(kind, cfg.resource_namespace, meta["name"],
                                           {"metadata": {"labels": {s.shard_label: str(want)}}})
                    out["relabelled"] += 1
                except Exception as exc:  # noqa: BLE001 - the audit keeps reporting what is left
                    out["errors"] += 1
                    if log_ is not None:
                        log_.error(exc, "shard re-label failed", kind=kind, name=meta.get("name"))
            cont = (doc.get("metadata") or {}).get("continue") or ""
            if not cont:
                break
    if metrics is not None:
        metrics.inc("shard_relabelled", out["relabelled"])
    if log_ is not None and (out["relabelled"] or out["errors"]):
        log_.info("shard labels re-stamped for the current shard count", shards=s.shards, **out)
    return out
