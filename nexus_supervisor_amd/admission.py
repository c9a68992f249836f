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

**Self-healing** (:class:`ShardLabelKeeper`).  The webhook is ``failurePolicy: Ignore``,
so while it is unreachable (an expired certificate, a rollout with no ready endpoint, a
``caBundle`` mismatch) Jobs are admitted unlabelled — seen by no replica.  The reference
cannot lose a run this way: every replica sees everything (``values.yaml:124-125``).  So
every ``sharding.audit-interval`` each replica LISTs the Nexus Jobs and Pods whose label is
missing or names no shard (``<label> notin (0..shards-1)`` — ``notin`` also matches a
missing key) and PATCHes the ones of its own shards; every ``sharding.relabel-every``
passes it also re-checks the runs labelled with its shards (``<label> in (owned)``) and
fixes any whose label disagrees with ``shard_of(name, shards)`` (an old replica's webhook
during a rolling change of ``shards``, a submitter with a stale count).  A run submitted
during an outage is thus decided within one audit interval.  Re-label passes (startup,
shard gains) run one at a time; shards gained meanwhile are merged into the next pass.

Served over TLS from a Secret's ``tls.crt`` / ``tls.key`` (``sharding.webhook-cert-dir``);
without them (tests, dev) plain HTTP with a warning.
"""
from __future__ import annotations

import base64
import json
import logging
import os
import ssl
from typing import Any, Callable, Dict, Iterable, List, Optional, Set

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


def cert_not_after(path: str) -> Optional[float]:
    """Expiry (epoch seconds) of the first certificate of a PEM file, None if unreadable."""
    try:
        info = ssl._ssl._test_decode_cert(path)  # noqa: SLF001 - the stdlib's own PEM → dict
        return float(ssl.cert_time_to_seconds(info["notAfter"]))
    except (OSError, KeyError, ValueError, ssl.SSLError):
        return None


def _cert_mtimes(cert_dir: str):
    out = []
    for f in ("tls.crt", "tls.key"):
        try:
            out.append(os.stat(os.path.join(cert_dir, f)).st_mtime_ns)
        except OSError:
            out.append(None)
    return tuple(out)


class WebhookServer:
    """``POST /mutate-shard-label`` (AdmissionReview v1) and ``GET /healthz``.

    The serving certificate is re-read when ``tls.crt`` / ``tls.key`` change on disk
    (cert-manager renewing the mounted Secret; :meth:`check_cert` every ``reload_interval``),
    so a renewal takes effect without a restart; ``webhook_cert_expiry_seconds`` says how
    long the one being served has left (alert well before 0: an expired certificate makes
    the API server skip the webhook — ``failurePolicy: Ignore`` — and the audit's repairs
    become the only labelling)."""

    def __init__(self, cfg, metrics=None, reload_interval: float = 30.0):
        self.cfg = cfg
        self.metrics = metrics
        self.runner = None
        self.port = 0
        self.tls = False
        self.ctx: Optional[ssl.SSLContext] = None
        self.cert_dir = ""
        self.reload_interval = reload_interval
        self.reloads = 0
        self.not_after: Optional[float] = None
        self._mtimes = None
        self._watch = None
        self.bootstrap = None  # webhook_certs.WebhookCertBootstrap (sharding.webhook-cert-bootstrap)

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
        self.ctx, self.cert_dir = ctx, cert_dir
        if not self.tls:
            log.warning("shard-label webhook serving plain HTTP (no tls.crt / tls.key in %r): the API server "
                        "only calls HTTPS webhooks", cert_dir)
        else:
            self._mtimes = _cert_mtimes(cert_dir)
            self._note_expiry()
            if self.reload_interval > 0:
                import asyncio

                self._watch = asyncio.ensure_future(self._watch_cert())
        site = web.TCPSite(self.runner, host, port, ssl_context=ctx)
        await site.start()
        self.port = site._server.sockets[0].getsockname()[1]  # noqa: SLF001
        return self.port

    def _note_expiry(self) -> None:
        import time

        self.not_after = cert_not_after(os.path.join(self.cert_dir, "tls.crt"))
        if self.metrics is not None and self.not_after is not None:
            self.metrics.set("webhook_cert_expiry_seconds", round(self.not_after - time.time(), 1))

    def check_cert(self) -> bool:
        """Reload the serving certificate into the live context when its files changed
        (``SSLContext.load_cert_chain`` on the same context: new handshakes use it, open
        connections keep theirs); refresh the expiry gauge.  True when reloaded."""
        if self.ctx is None:
            return False
        cur = _cert_mtimes(self.cert_dir)
        changed = cur != self._mtimes and None not in cur
        if changed:
            try:
                self.ctx.load_cert_chain(os.path.join(self.cert_dir, "tls.crt"), os.path.join(self.cert_dir, "tls.key"))
            except (OSError, ssl.SSLError) as exc:  # a half-written pair: the next check retries
                log.warning("webhook certificate reload failed (keeping the one in use): %s", exc)
                return False
            self._mtimes = cur
            self.reloads += 1
            if self.metrics is not None:
                self.metrics.inc("webhook_cert_reloads")
            log.info("webhook serving certificate reloaded from %s", self.cert_dir)
        self._note_expiry()
        return changed

    async def _watch_cert(self) -> None:
        import asyncio

        while True:
            await asyncio.sleep(self.reload_interval)
            try:
                self.check_cert()
            except Exception as exc:  # noqa: BLE001 - never take the webhook down over a reload
                log.warning("webhook certificate check failed: %s", exc)

    async def stop(self) -> None:
        if self.bootstrap is not None:
            await self.bootstrap.stop()
        if self._watch is not None:
            self._watch.cancel()
            self._watch = None
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


async def _list_pages(kube, kind: str, namespace: str, selector: str, page: int, max_items: int):
    """Items of a paged LIST (at most ``max_items``), yielded page by page."""
    from .kube.client import resource_path

    cont, seen = "", 0
    while True:
        params = {"labelSelector": selector, "limit": str(page)}
        if cont:
            params["continue"] = cont
        doc = await kube.request("GET", resource_path(kind, namespace), params=params)
        items = doc.get("items") or []
        seen += len(items)
        yield items
        cont = (doc.get("metadata") or {}).get("continue") or ""
        if not cont or seen >= max_items:
            return


class ShardLabelKeeper:
    """``sharding.shard-label`` upkeep of one replica (in the process that holds its API
    client): the periodic audit that finds — and repairs — runs no replica can see, and
    the re-label passes after a change of ``shards`` (startup, shard gains), one at a time.

    ``owned()`` returns the replica's current shard set (None = every shard)."""

    def __init__(self, cfg, kube, metrics, log_, owned: Callable[[], Optional[Iterable[int]]],
                 interval: Optional[float] = None, page: int = 500, max_items: int = 20_000):
        s = cfg.sharding
        self.cfg = cfg
        self.kube = kube
        self.metrics = metrics
        self.log = log_
        self.owned = owned
        self.interval = s.audit_interval if interval is None else interval
        self.repair = s.repair_labels
        self.relabel_every = max(1, int(s.relabel_every))
        self.page = page
        self.max_items = max_items
        self._base = f"{cfg.labels.nexus_component_label}={cfg.labels.algorithm_run_value}"
        self._audit: Optional["asyncio.Task"] = None
        self._relabel: Optional["asyncio.Task"] = None
        self._pending: Set[int] = set()
        self._pending_all = False
        self.passes = 0
        self.last: Dict[str, int] = {}
        self._warned = False

    # ---------------------------------------------------------------- lifecycle
    def start(self) -> None:
        import asyncio

        if self._audit is None and self.interval > 0:
            self._audit = asyncio.ensure_future(self._audit_loop())

    async def stop(self) -> None:
        import asyncio

        tasks = [t for t in (self._audit, self._relabel) if t is not None]
        for t in tasks:
            t.cancel()
        await asyncio.gather(*tasks, return_exceptions=True)
        self._audit = self._relabel = None

    # ---------------------------------------------------------------- re-label passes
    def request_relabel(self, shards: Optional[Iterable[int]]) -> None:
        """Re-stamp the runs of ``shards`` (None = every shard) whose label was computed for
        another shard count.  One pass runs at a time; shards requested while it runs are
        merged into the next one (a lease rebalance gains several in a row)."""
        import asyncio

        if not self.cfg.sharding.relabel:
            return
        if shards is None:
            self._pending_all = True
        else:
            self._pending.update(int(k) for k in shards)
        if not (self._pending or self._pending_all):
            return
        if self._relabel is None or self._relabel.done():
            self._relabel = asyncio.ensure_future(self._relabel_runner())

    async def _relabel_runner(self) -> None:
        import asyncio

        while self._pending or self._pending_all:
            want = None if self._pending_all else frozenset(self._pending)
            self._pending, self._pending_all = set(), False
            try:
                await relabel_owned(self.cfg, self.kube, want, self.metrics, self.log, page=self.page)
            except asyncio.CancelledError:
                raise
            except Exception as exc:  # noqa: BLE001 - the audit keeps repairing what is left
                if self.log is not None:
                    self.log.error(exc, "shard re-label pass failed")

    # ---------------------------------------------------------------- the audit
    async def _audit_loop(self) -> None:
        import asyncio

        while True:
            try:
                await self.audit_pass()
            except asyncio.CancelledError:
                raise
            except Exception as exc:  # noqa: BLE001 - an audit, never a reason to stop
                if self.log is not None:
                    self.log.v(1).info("shard label audit failed", error=str(exc))
            await asyncio.sleep(self.interval)

    def _name(self, kind: str, item) -> str:
        meta = item.get("metadata") or {}
        if kind == "Job":
            return meta.get("name", "")
        return (meta.get("labels") or {}).get(self.cfg.labels.job_name_label, "")

    async def _patch(self, kind: str, item, value: str) -> bool:
        meta = item.get("metadata") or {}
        try:
            await self.kube.patch_merge(kind, self.cfg.resource_namespace, meta.get("name", ""),
                                        {"metadata": {"labels": {self.cfg.sharding.shard_label: value}}})
            return True
        except Exception as exc:  # noqa: BLE001 - counted; the next pass retries
            if self.log is not None:
                self.log.v(1).info("shard label repair failed", kind=kind, name=meta.get("name"), error=str(exc))
            return False

    async def audit_pass(self) -> Dict[str, int]:
        """One audit: Nexus Jobs / Pods whose label is missing or names no shard — every
        replica counts them (``shard_label_missing``: Jobs), each repairs those of its own
        shards; every ``relabel-every`` passes also the runs labelled with its own shards
        whose label disagrees with their name (``shard_label_wrong``).  Returns counts."""
        s = self.cfg.sharding
        ns = self.cfg.resource_namespace
        label = s.shard_label
        owned = self.owned()
        owned = None if owned is None else frozenset(int(k) for k in owned)
        out = {"missing": 0, "missing_pods": 0, "wrong": 0, "repaired": 0, "errors": 0}
        examples: List[str] = []
        every = ",".join(str(k) for k in range(s.shards))
        sel = f"{self._base},{label} notin ({every})"
        for kind in ("Job", "Pod"):
            async for items in _list_pages(self.kube, kind, ns, sel, self.page, self.max_items):
                for item in items:
                    name = self._name(kind, item)
                    if not name:
                        continue
                    out["missing" if kind == "Job" else "missing_pods"] += 1
                    if kind == "Job" and len(examples) < 5:
                        examples.append(name)
                    want = shard_of(name, s.shards)
                    if self.repair and (owned is None or want in owned):
                        if await self._patch(kind, item, str(want)):
                            out["repaired"] += 1
                        else:
                            out["errors"] += 1
        self.passes += 1
        if self.passes % self.relabel_every == 0 and (owned is None or owned):
            mine = sorted(owned) if owned is not None else list(range(s.shards))
            sel_in = f"{self._base},{label} in ({','.join(str(k) for k in mine)})"
            for kind in ("Job", "Pod"):
                async for items in _list_pages(self.kube, kind, ns, sel_in, self.page, self.max_items):
                    for item in items:
                        name = self._name(kind, item)
                        if not name:
                            continue
                        want = str(shard_of(name, s.shards))
                        if ((item.get("metadata") or {}).get("labels") or {}).get(label) == want:
                            continue
                        out["wrong"] += 1
                        # labelled for one of our shards, but its name hashes elsewhere: we are
                        # the replica that sees it, so we move it to its owner
                        if self.repair:
                            if await self._patch(kind, item, want):
                                out["repaired"] += 1
                            else:
                                out["errors"] += 1
            if self.metrics is not None:
                self.metrics.set("shard_label_wrong", float(out["wrong"]))
        if self.metrics is not None:
            self.metrics.set("shard_label_missing", float(out["missing"]))
            if out["repaired"]:
                self.metrics.inc("shard_label_repaired", out["repaired"])
            if out["errors"]:
                self.metrics.inc("shard_label_repair_errors", out["errors"])
        if self.log is not None:
            if out["missing"] and not self._warned:
                self.log.warning("Nexus Jobs without a valid shard label (invisible to every replica until repaired; "
                                 "is the shard-label webhook reachable?)", label=label, jobs=out["missing"],
                                 examples=examples, repaired=out["repaired"])
            elif out["repaired"] or out["wrong"]:
                self.log.info("shard labels repaired", **out)
        self._warned = bool(out["missing"])
        self.last = out
        return out
