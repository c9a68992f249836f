"""In-memory kube-apiserver speaking the real REST + watch wire protocol (aiohttp).

The reference tests against client-go's tracker-backed ``fake.NewClientset``
(``/root/reference/services/supervisor_test.go:13,40``), which bypasses HTTP.
This fake sits behind a real socket so the supervisor's own REST/watch client
(:mod:`nexus_supervisor_amd.kube.client`) is exercised end to end:

* LIST (``limit``/``continue``, equality label selectors), GET, POST, PUT (409 on
  a stale ``resourceVersion``), merge-PATCH, DELETE (``propagationPolicy``
  Background/Foreground garbage-collects a Job's pods like the GC controller);
* WATCH from a ``resourceVersion`` with bookmarks and ``timeoutSeconds``; events
  are serialised once and fanned out to every watcher as chunked JSON lines;
* fault injection: :meth:`expire` (history compaction → ``410 Gone`` for
  resuming watches), :meth:`close_watches` (dropped streams), per-path error
  injection, request latency; Leases (``coordination.k8s.io/v1``) for leader
  election tests.
"""
from __future__ import annotations

import asyncio
import collections
import copy
import datetime as _dt
import json
import re
import time
import uuid
from typing import Any, Deque, Dict, List, Optional, Set, Tuple

from . import miniweb as web

from ..kube.client import RESOURCES

_PLURAL_TO_KIND = {plural: kind for kind, (_prefix, plural) in RESOURCES.items()}
_API_VERSION = {"Event": "v1", "Pod": "v1", "Node": "v1", "Job": "batch/v1", "Lease": "coordination.k8s.io/v1",
                "Secret": "v1", "MutatingWebhookConfiguration": "admissionregistration.k8s.io/v1"}


_ISO_CACHE = [0, ""]


def _now_iso() -> str:
    """RFC 3339 seconds (memoised per second: creation bursts reuse the string)."""
    t = int(time.time())
    if _ISO_CACHE[0] != t:
        _ISO_CACHE[0] = t
        _ISO_CACHE[1] = _dt.datetime.fromtimestamp(t, _dt.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")
    return _ISO_CACHE[1]


try:  # native compact encoder (csrc/kube/json_encode.cpp): ~4x the json module on pod objects
    from .._kube_native import dumps as _native_dumps

    def _watch_line(etype: str, obj: Dict[str, Any]) -> bytes:
        return _native_dumps({"type": etype, "object": obj}, newline=True)
except ImportError:  # pragma: no cover
    _ENCODE = json.JSONEncoder(separators=(",", ":")).encode

    def _watch_line(etype: str, obj: Dict[str, Any]) -> bytes:
        return _ENCODE({"type": etype, "object": obj}).encode() + b"\n"


_SET_REQ = re.compile(r"^\s*(\S+)\s+(in|notin)\s*\(([^)]*)\)\s*$")


def _split_selector(sel: str) -> List[str]:
    """Comma-split a selector, keeping the commas inside a set's parentheses."""
    parts, depth, cur = [], 0, []
    for ch in sel or "":
        if ch == "(":
            depth += 1
        elif ch == ")":
            depth -= 1
        if ch == "," and depth == 0:
            parts.append("".join(cur))
            cur = []
        else:
            cur.append(ch)
    parts.append("".join(cur))
    return [p.strip() for p in parts if p.strip()]


def _parse_selector(sel: str) -> List[Tuple[str, str, Any]]:
    out: List[Tuple[str, str, Any]] = []
    for part in _split_selector(sel):
        m = _SET_REQ.match(part)
        if m:
            out.append((m.group(1), m.group(2), frozenset(v.strip() for v in m.group(3).split(",") if v.strip())))
        elif "!=" in part:
            k, v = part.split("!=", 1)
            out.append((k.strip(), "!=", v.strip()))
        elif "==" in part:
            k, v = part.split("==", 1)
            out.append((k.strip(), "=", v.strip()))
        elif "=" in part:
            k, v = part.split("=", 1)
            out.append((k.strip(), "=", v.strip()))
        elif part.startswith("!"):
            out.append((part[1:], "!", None))
        else:
            out.append((part, "exists", None))
    return out


def _matches(labels: Dict[str, str], sel) -> bool:
    for k, op, v in sel:
        if op == "=" and labels.get(k) != v:
            return False
        if op == "!=" and labels.get(k) == v:
            return False
        if op == "exists" and k not in labels:
            return False
        if op == "!" and k in labels:
            return False
        if op == "in" and labels.get(k) not in v:
            return False
        if op == "notin" and k in labels and labels[k] in v:
            return False
    return True


_FIELD_PATHS = ("metadata.name", "metadata.namespace", "spec.nodeName", "status.phase", "involvedObject.kind",
                "involvedObject.name", "reason", "type")


_FIELD_KEYS = tuple(("\0f:" + p, tuple(p.split("."))) for p in _FIELD_PATHS)


def _selectable(obj: Dict[str, Any]) -> Dict[str, str]:
    """Labels plus the supported field-selector paths (prefixed ``\0f:``) of an object."""
    out = dict((obj.get("metadata") or {}).get("labels") or {})
    for key, parts in _FIELD_KEYS:
        cur: Any = obj
        for part in parts:
            cur = cur.get(part) if type(cur) is dict else None
            if cur is None:
                break
        if type(cur) is str:
            out[key] = cur
    return out


def _parse_fields(sel: str):
    return [("\0f:" + k, op, v) for k, op, v in _parse_selector(sel)]


def _merge(dst: Dict[str, Any], patch: Dict[str, Any]) -> Dict[str, Any]:
    for k, v in patch.items():
        if v is None:
            dst.pop(k, None)
        elif isinstance(v, dict) and isinstance(dst.get(k), dict):
            _merge(dst[k], v)
        else:
            dst[k] = copy.deepcopy(v)
    return dst


class _Watcher:
    """One watch stream: committed lines buffer here until the stream's writer drains
    them (a list + one wakeup future: no per-event queue/task machinery)."""

    __slots__ = ("ns", "sel", "buf", "closed", "wake")

    def __init__(self, ns, sel):
        self.ns = ns
        self.sel = sel
        self.buf: List[bytes] = []
        self.closed = False
        self.wake: Optional[asyncio.Future] = None

    def push(self, line: bytes) -> None:
        if self.closed:
            return  # committed after the stream was cut: the client resumes (or gets 410)
        self.buf.append(line)
        w = self.wake
        if w is not None and not w.done():
            w.set_result(None)

    def close(self) -> None:
        self.closed = True
        w = self.wake
        if w is not None and not w.done():
            w.set_result(None)

    async def wait(self, timeout: float) -> None:
        if self.buf or self.closed:
            return
        loop = asyncio.get_running_loop()
        fut = self.wake = loop.create_future()
        h = loop.call_later(timeout, lambda: fut.done() or fut.set_result(None))
        try:
            await fut
        finally:
            h.cancel()
            self.wake = None


def json_patch(obj: Dict[str, Any], ops) -> Dict[str, Any]:
    """RFC 6902 ``add`` / ``replace`` / ``remove`` over JSON-pointer paths (what mutating
    webhooks send); returns a patched deep copy."""
    out = copy.deepcopy(obj)
    for op in ops:
        parts = [p.replace("~1", "/").replace("~0", "~") for p in op["path"].split("/")[1:]]
        cur = out
        for p in parts[:-1]:
            cur = cur[int(p)] if isinstance(cur, list) else cur[p]
        last = parts[-1]
        if op["op"] in ("add", "replace"):
            if isinstance(cur, list):
                idx = len(cur) if last == "-" else int(last)
                if op["op"] == "add":
                    cur.insert(idx, op["value"])
                else:
                    cur[idx] = op["value"]
            else:
                if op["op"] == "replace" and last not in cur:
                    raise KeyError(op["path"])
                cur[last] = op["value"]
        elif op["op"] == "remove":
            del cur[int(last) if isinstance(cur, list) else last]
        else:
            raise ValueError(f"unsupported patch op {op['op']}")
    return out


class FakeApiServer:
    def __init__(self, *, token: str = "", history: int = 200_000, bookmark_interval: float = 1.0,
                 gc_pods_on_job_delete: bool = True):
        self.token = token
        self.history_cap = history
        self.bookmark_interval = bookmark_interval
        self.gc_pods = gc_pods_on_job_delete
        self.objects: Dict[str, Dict[Tuple[str, str], Dict[str, Any]]] = {k: {} for k in RESOURCES}
        self.history: Dict[str, Deque[Tuple[int, str, bytes, Dict[str, str]]]] = {k: collections.deque() for k in RESOURCES}
        self.compacted: Dict[str, int] = {k: 0 for k in RESOURCES}
        self.watchers: Dict[str, Set[_Watcher]] = {k: set() for k in RESOURCES}
        self.rv = 1000
        self.deleted: List[Tuple[str, str, str, str]] = []  # (kind, ns, name, propagation)
        self.mutating_webhooks: List[Tuple[str, frozenset, Any]] = []  # (url, kinds, ssl context)
        self.webhook_calls = 0
        self.webhook_failures = 0
        self._pods_by_job: Dict[Tuple[str, str], Set[str]] = {}  # (ns, job-name label) -> pod names (GC index)
        self.fail_next: Dict[Tuple[str, str], int] = {}  # (method, kind) -> count of 500s to inject
        # (method, kind) -> count of 429s to inject, each with ``Retry-After: retry_after``
        # (API Priority and Fairness rejecting the request); kind "PodLog" for pods/log
        self.throttle_next: Dict[Tuple[str, str], int] = {}
        self.retry_after = "1"
        # (monotonic t, method, kind, name, status) of every throttled request and of every
        # request to a name that was throttled before (to check retries honour the hint)
        self.throttle_log: List[Tuple[float, str, str, str, int]] = []
        self._throttled_names: Set[Tuple[str, str]] = set()
        self.log_inflight = 0
        self.log_inflight_max = 0
        self._snapshots: Dict[str, Tuple[int, List[Dict[str, Any]]]] = {}  # paginated LIST snapshots
        self.latency = 0.0
        # container logs served by GET …/pods/{name}/log: (ns, pod, container, previous) -> text
        self.pod_logs: Dict[Tuple[str, str, str, bool], str] = {}
        self.log_requests: List[Dict[str, str]] = []
        self.log_latency = 0.0  # extra delay of pods/log answers only
        self.coalesce = 0.0005  # watch write coalescing window (seconds)
        self.requests = 0
        self.watch_requests = 0
        self._server: Optional[web.Server] = None
        self.url = ""

    # ------------------------------------------------------------------ lifecycle
    async def start(self, host: str = "127.0.0.1", port: int = 0, ssl_context=None) -> str:
        """Serve on ``host:port`` (0 = any free port); with ``ssl_context`` over TLS, the
        way a real kube-apiserver always answers."""
        srv = web.Server()
        for kind, (prefix, plural) in RESOURCES.items():
            base = f"{prefix}/namespaces/{{ns}}/{plural}"
            srv.add_route("GET", base, self._h_collection)
            srv.add_route("POST", base, self._h_create)
            srv.add_route("GET", base + "/{name}", self._h_get)
            srv.add_route("PUT", base + "/{name}", self._h_replace)
            srv.add_route("PATCH", base + "/{name}", self._h_patch)
            srv.add_route("DELETE", base + "/{name}", self._h_delete)
            srv.add_route("GET", f"{prefix}/{plural}", self._h_collection)
            # cluster-scoped objects (namespace ""): Nodes, MutatingWebhookConfigurations
            srv.add_route("POST", f"{prefix}/{plural}", self._h_create)
            srv.add_route("GET", f"{prefix}/{plural}/{{name}}", self._h_get)
            srv.add_route("PUT", f"{prefix}/{plural}/{{name}}", self._h_replace)
            srv.add_route("PATCH", f"{prefix}/{plural}/{{name}}", self._h_patch)
        srv.add_route("GET", "/api/v1/namespaces/{ns}/pods/{name}/log", self._h_pod_log)
        port = await srv.start(host, port, ssl_context=ssl_context)
        self._server = srv
        self.url = f"{'https' if ssl_context is not None else 'http'}://{host}:{port}"
        return self.url

    async def stop(self) -> None:
        self.close_watches()
        await asyncio.sleep(0)
        if self._server is not None:
            await self._server.stop()
            self._server = None

    # ------------------------------------------------------------------ programmatic API (loop thread)
    def _next_rv(self) -> str:
        self.rv += 1
        return str(self.rv)

    def _record(self, kind: str, etype: str, obj: Dict[str, Any]) -> None:
        rv = int(obj["metadata"]["resourceVersion"])
        line = _watch_line(etype, obj)
        labels = _selectable(obj)
        ns = obj["metadata"].get("namespace", "")
        h = self.history[kind]
        h.append((rv, ns, line, labels))
        if len(h) > self.history_cap:
            old = h.popleft()
            self.compacted[kind] = old[0]
        for w in list(self.watchers[kind]):
            if (not w.ns or w.ns == ns) and _matches(labels, w.sel):
                w.push(line)

    def create(self, obj: Dict[str, Any], copy_obj: bool = True) -> Dict[str, Any]:
        obj = copy.deepcopy(obj) if copy_obj else obj
        kind = obj["kind"]
        obj.setdefault("apiVersion", _API_VERSION.get(kind, "v1"))
        meta = obj.setdefault("metadata", {})
        if not meta.get("name") and meta.get("generateName"):
            meta["name"] = meta["generateName"] + uuid.uuid4().hex[:5]
        key = (meta.get("namespace", ""), meta["name"])
        if key in self.objects[kind]:
            raise KeyError("AlreadyExists")
        meta.setdefault("uid", str(uuid.uuid4()))
        meta.setdefault("creationTimestamp", _now_iso())
        meta["resourceVersion"] = self._next_rv()
        self.objects[kind][key] = obj
        self._index(kind, obj, True)
        self._record(kind, "ADDED", obj)
        return obj

    def _index(self, kind: str, obj: Dict[str, Any], add: bool) -> None:
        if kind != "Pod":
            return
        meta = obj["metadata"]
        job = (meta.get("labels") or {}).get("batch.kubernetes.io/job-name")
        if not job:
            return
        k = (meta.get("namespace", ""), job)
        if add:
            self._pods_by_job.setdefault(k, set()).add(meta["name"])
        else:
            s = self._pods_by_job.get(k)
            if s is not None:
                s.discard(meta["name"])
                if not s:
                    del self._pods_by_job[k]

    def update(self, obj: Dict[str, Any], check_rv: bool = False, copy_obj: bool = True) -> Dict[str, Any]:
        obj = copy.deepcopy(obj) if copy_obj else obj
        kind = obj["kind"]
        meta = obj["metadata"]
        key = (meta.get("namespace", ""), meta["name"])
        cur = self.objects[kind].get(key)
        if cur is None:
            raise KeyError("NotFound")
        if check_rv and meta.get("resourceVersion") and meta["resourceVersion"] != cur["metadata"]["resourceVersion"]:
            raise ValueError("Conflict")
        meta.setdefault("uid", cur["metadata"].get("uid"))
        meta.setdefault("creationTimestamp", cur["metadata"].get("creationTimestamp"))
        obj.setdefault("apiVersion", cur.get("apiVersion"))
        meta["resourceVersion"] = self._next_rv()
        self._index(kind, cur, False)
        self.objects[kind][key] = obj
        self._index(kind, obj, True)
        self._record(kind, "MODIFIED", obj)
        return obj

    def apply(self, etype: str, obj: Dict[str, Any], copy_obj: bool = True) -> None:
        """One line of synthetic cluster traffic (``bench/workload.py``): ADDED / MODIFIED
        (either creates or updates, as the native simulator's ``/sim/apply``), DELETED, or
        LOG (a container log served from ``pods/log``)."""
        if etype == "LOG":
            self.set_pod_log(obj["namespace"], obj["pod"], obj["container"], obj["text"])
        elif etype == "DELETED":
            m = obj["metadata"]
            self.delete(obj["kind"], m.get("namespace", ""), m["name"])
        else:
            key = (obj["metadata"].get("namespace", ""), obj["metadata"]["name"])
            if key in self.objects[obj["kind"]]:
                self.update(obj, copy_obj=copy_obj)
            else:
                self.create(obj, copy_obj=copy_obj)

    def upsert(self, obj: Dict[str, Any]) -> Dict[str, Any]:
        key = (obj["metadata"].get("namespace", ""), obj["metadata"]["name"])
        return self.update(obj) if key in self.objects[obj["kind"]] else self.create(obj)

    def delete(self, kind: str, ns: str, name: str, propagation: str = "Background") -> Optional[Dict[str, Any]]:
        obj = self.objects[kind].pop((ns, name), None)
        if obj is None:
            return None
        self._index(kind, obj, False)
        obj = dict(obj)
        obj["metadata"] = dict(obj["metadata"], resourceVersion=self._next_rv())
        self._record(kind, "DELETED", obj)
        self.deleted.append((kind, ns, name, propagation))
        if kind == "Job" and self.gc_pods and propagation in ("Background", "Foreground"):
            for pname in sorted(self._pods_by_job.get((ns, name), ())):
                self.delete("Pod", ns, pname, propagation)
        return obj

    def get(self, kind: str, ns: str, name: str) -> Optional[Dict[str, Any]]:
        return self.objects[kind].get((ns, name))

    def expire(self, kind: Optional[str] = None) -> None:
        """Compact history (resuming watches get 410 Gone) and drop live watch streams."""
        for k in ([kind] if kind else list(RESOURCES)):
            if self.history[k]:
                self.compacted[k] = self.history[k][-1][0]
            self.history[k].clear()
        self.close_watches(kind)

    def close_watches(self, kind: Optional[str] = None) -> None:
        for k in ([kind] if kind else list(RESOURCES)):
            for w in list(self.watchers[k]):
                w.close()

    # ------------------------------------------------------------------ HTTP
    def _auth(self, req: web.Request) -> Optional[web.Response]:
        if self.token and req.headers.get("Authorization") != f"Bearer {self.token}":
            return self._status(401, "Unauthorized", "Unauthorized")
        return None

    @staticmethod
    def _status(code: int, reason: str, message: str) -> web.Response:
        body = {"kind": "Status", "apiVersion": "v1", "status": "Failure", "message": message, "reason": reason, "code": code}
        return web.json_response(body, status=code)

    def _kind(self, req: web.Request) -> str:
        plural = req.path.rstrip("/").split("/")
        # .../{plural} or .../{plural}/{name}
        for p in reversed(plural):
            if p in _PLURAL_TO_KIND:
                return _PLURAL_TO_KIND[p]
        raise web.HTTPNotFound()

    async def _pre(self, req: web.Request, method: str) -> Optional[web.Response]:
        self.requests += 1
        bad = self._auth(req)
        if bad is not None:
            return bad
        if self.latency:
            await asyncio.sleep(self.latency)
        kind = self._kind(req)
        n = self.fail_next.get((method, kind), 0)
        if n:
            self.fail_next[(method, kind)] = n - 1
            return self._status(500, "InternalError", "injected failure")
        return self._throttle(req, method, kind)

    def _throttle(self, req: web.Request, method: str, kind: str) -> Optional[web.Response]:
        name = req.match_info.get("name", "")
        n = self.throttle_next.get((method, kind), 0)
        if n:
            self.throttle_next[(method, kind)] = n - 1
            self._throttled_names.add((method, name))
            self.throttle_log.append((time.monotonic(), method, kind, name, 429))
            body = {"kind": "Status", "apiVersion": "v1", "status": "Failure", "code": 429, "reason": "TooManyRequests",
                    "message": "too many requests, please try again later", "details": {"retryAfterSeconds": 1}}
            return web.json_response(body, status=429, headers={"Retry-After": self.retry_after})
        if (method, name) in self._throttled_names:
            self.throttle_log.append((time.monotonic(), method, kind, name, 200))
        return None

    async def _h_collection(self, req: web.Request):
        if req.query.get("watch") in ("1", "true"):
            return await self._watch(req)
        bad = await self._pre(req, "LIST")
        if bad is not None:
            return bad
        kind = self._kind(req)
        ns = req.match_info.get("ns", "")
        limit = int(req.query.get("limit", "0") or 0)
        token = req.query.get("continue", "")
        if token:
            # every page of a paginated LIST comes from the snapshot taken by the first
            # page, at that page's resourceVersion (apiserver semantics)
            snap = self._snapshots.get(token.split(":", 1)[0])
            if snap is None:
                return self._status(410, "Expired", "the provided continue parameter is too old")
            snap_rv, items = snap
            start = int(token.split(":", 1)[1])
        else:
            sel = _parse_selector(req.query.get("labelSelector", "")) + _parse_fields(req.query.get("fieldSelector", ""))
            items = [o for (ons, _), o in self.objects[kind].items()
                     if (not ns or ons == ns) and _matches(_selectable(o), sel)]
            items.sort(key=lambda o: (o["metadata"].get("namespace", ""), o["metadata"]["name"]))
            snap_rv, start = self.rv, 0
        meta: Dict[str, Any] = {"resourceVersion": str(snap_rv)}
        if limit and start + limit < len(items):
            if not token:
                sid = uuid.uuid4().hex[:12]
                self._snapshots[sid] = (snap_rv, items)
                while len(self._snapshots) > 64:
                    self._snapshots.pop(next(iter(self._snapshots)))
            else:
                sid = token.split(":", 1)[0]
            meta["continue"] = f"{sid}:{start + limit}"
            page = items[start:start + limit]
        else:
            page = items[start:]
        body = {"kind": f"{kind}List", "apiVersion": _API_VERSION.get(kind, "v1"), "metadata": meta, "items": page}
        return web.Response(body=json.dumps(body, separators=(",", ":")).encode())

    async def _watch(self, req: web.Request):
        bad = self._auth(req)
        if bad is not None:
            return bad
        self.watch_requests += 1
        kind = self._kind(req)
        ns = req.match_info.get("ns", "")
        sel = _parse_selector(req.query.get("labelSelector", "")) + _parse_fields(req.query.get("fieldSelector", ""))
        rv_s = req.query.get("resourceVersion", "")
        timeout = float(req.query.get("timeoutSeconds", "0") or 0) or 1800.0
        bookmarks = req.query.get("allowWatchBookmarks") in ("true", "1")
        resp = web.StreamResponse(status=200, headers={"Content-Type": "application/json"})
        resp.enable_chunked_encoding()
        await resp.prepare(req)
        w = _Watcher(ns, sel)
        # register before replaying history so nothing committed meanwhile is lost
        self.watchers[kind].add(w)
        try:
            if rv_s and rv_s != "0":
                rv = int(rv_s)
                if rv < self.compacted[kind]:
                    gone = {"type": "ERROR", "object": {"kind": "Status", "apiVersion": "v1", "status": "Failure",
                                                        "message": f"too old resource version: {rv} ({self.compacted[kind]})",
                                                        "reason": "Expired", "code": 410}}
                    await resp.write(json.dumps(gone).encode() + b"\n")
                    return resp
                backlog = [line for (hrv, hns, line, labels) in self.history[kind]
                           if hrv > rv and (not ns or hns == ns) and _matches(labels, sel)]
                # live events queued after registration may duplicate the backlog tail: skip by rv
                last_rv = self.history[kind][-1][0] if self.history[kind] else rv
                if backlog:
                    await resp.write(b"".join(backlog))
                skip_upto = last_rv
            else:
                skip_upto = self.rv
            deadline = time.monotonic() + timeout
            while True:
                remaining = deadline - time.monotonic()
                if remaining <= 0:
                    break
                await w.wait(min(remaining, self.bookmark_interval))
                if not w.buf:
                    if w.closed:
                        break
                    if bookmarks:
                        bm = {"type": "BOOKMARK", "object": {"kind": kind, "apiVersion": _API_VERSION.get(kind, "v1"),
                                                             "metadata": {"resourceVersion": str(self.rv)}}}
                        await resp.write(json.dumps(bm).encode() + b"\n")
                    continue
                if len(w.buf) == 1 and self.coalesce > 0 and not w.closed:
                    # like the apiserver's buffered watch writer: let a burst accumulate
                    # briefly and send it as one chunk instead of one write per event
                    await asyncio.sleep(self.coalesce)
                chunk, w.buf = w.buf, []
                if skip_upto:
                    chunk = [c for c in chunk if _line_rv(c) > skip_upto]
                    if chunk:
                        skip_upto = 0
                if chunk:
                    await resp.write(b"".join(chunk))
                if w.closed:
                    break
        except (ConnectionResetError, asyncio.CancelledError):
            pass
        finally:
            self.watchers[kind].discard(w)
        return resp

    def set_pod_log(self, ns: str, pod: str, container: str, text: str, previous: bool = False) -> None:
        self.pod_logs[(ns, pod, container, previous)] = text

    async def _h_pod_log(self, req: web.Request):
        """``pods/{name}/log`` (text/plain): ``container``, ``previous``, ``tailLines`` and
        ``limitBytes`` as the apiserver applies them (limitBytes cuts the tail's end)."""
        self.requests += 1
        bad = self._auth(req)
        if bad is not None:
            return bad
        self.log_inflight += 1
        self.log_inflight_max = max(self.log_inflight_max, self.log_inflight)
        try:
            if self.latency or self.log_latency:
                await asyncio.sleep(self.latency + self.log_latency)
        finally:
            self.log_inflight -= 1
        q = req.query
        self.log_requests.append(dict(q, pod=req.match_info["name"]))
        n = self.fail_next.get(("GET", "PodLog"), 0)
        if n:
            self.fail_next[("GET", "PodLog")] = n - 1
            return self._status(500, "InternalError", "injected failure")
        hot = self._throttle(req, "GET", "PodLog")
        if hot is not None:
            return hot
        ns, name = req.match_info["ns"], req.match_info["name"]
        if (ns, name) not in self.objects["Pod"]:
            return self._status(404, "NotFound", f'pods "{name}" not found')
        prev = q.get("previous") in ("true", "1")
        text = self.pod_logs.get((ns, name, q.get("container", ""), prev))
        if text is None:
            return self._status(400, "BadRequest", f'previous terminated container "{q.get("container")}" not found'
                                if prev else f'container "{q.get("container")}" has no log')
        lines = text.splitlines(keepends=True)
        if q.get("tailLines"):
            lines = lines[-int(q["tailLines"]):]
        body = "".join(lines).encode()
        if q.get("limitBytes"):
            body = body[:int(q["limitBytes"])]
        return web.Response(body=body, content_type="text/plain")

    async def _h_get(self, req: web.Request):
        bad = await self._pre(req, "GET")
        if bad is not None:
            return bad
        kind = self._kind(req)
        obj = self.objects[kind].get((req.match_info.get("ns", ""), req.match_info["name"]))
        if obj is None:
            return self._status(404, "NotFound", f'{kind.lower()}s "{req.match_info["name"]}" not found')
        return web.json_response(obj)

    def add_mutating_webhook(self, url: str, kinds=("Job", "Pod"), ssl_ctx=None) -> None:
        """Call ``url`` (an AdmissionReview v1 endpoint) on every API CREATE of ``kinds``
        and apply its JSON patch, as the API server's mutating admission does;
        ``failurePolicy: Ignore`` — an unreachable or failing webhook admits unchanged."""
        self.mutating_webhooks.append((url, frozenset(kinds), ssl_ctx))

    async def _mutate(self, obj: Dict[str, Any]) -> Dict[str, Any]:
        import aiohttp

        for url, kinds, ctx in self.mutating_webhooks:
            if obj.get("kind") not in kinds:
                continue
            review = {"apiVersion": "admission.k8s.io/v1", "kind": "AdmissionReview", "request": {
                "uid": uuid.uuid4().hex, "kind": {"group": "batch" if obj["kind"] == "Job" else "",
                                                  "version": "v1", "kind": obj["kind"]},
                "operation": "CREATE", "namespace": obj["metadata"].get("namespace", ""), "object": obj}}
            try:
                async with aiohttp.ClientSession() as s:
                    async with s.post(url, json=review, ssl=ctx, timeout=aiohttp.ClientTimeout(total=5)) as r:
                        resp = (await r.json()).get("response") or {}
            except Exception:  # noqa: BLE001 - failurePolicy: Ignore
                self.webhook_failures += 1
                continue
            self.webhook_calls += 1
            if resp.get("patchType") == "JSONPatch" and resp.get("patch"):
                import base64

                obj = json_patch(obj, json.loads(base64.b64decode(resp["patch"])))
        return obj

    async def _h_create(self, req: web.Request):
        bad = await self._pre(req, "POST")
        if bad is not None:
            return bad
        kind = self._kind(req)
        obj = await req.json()
        obj["kind"] = kind
        if req.match_info.get("ns"):
            obj.setdefault("metadata", {})["namespace"] = req.match_info["ns"]
        if self.mutating_webhooks:
            obj = await self._mutate(obj)
        try:
            return web.json_response(self.create(obj), status=201)
        except KeyError:
            return self._status(409, "AlreadyExists", f'{kind.lower()}s "{obj["metadata"].get("name")}" already exists')

    async def _h_replace(self, req: web.Request):
        bad = await self._pre(req, "PUT")
        if bad is not None:
            return bad
        kind = self._kind(req)
        obj = await req.json()
        obj["kind"] = kind
        obj.setdefault("metadata", {}).update(name=req.match_info["name"])
        if req.match_info.get("ns"):
            obj["metadata"]["namespace"] = req.match_info["ns"]
        try:
            return web.json_response(self.update(obj, check_rv=True))
        except KeyError:
            return self._status(404, "NotFound", "not found")
        except ValueError:
            return self._status(409, "Conflict", "the object has been modified; please apply your changes to the latest version")

    async def _h_patch(self, req: web.Request):
        bad = await self._pre(req, "PATCH")
        if bad is not None:
            return bad
        kind = self._kind(req)
        key = (req.match_info.get("ns", ""), req.match_info["name"])
        cur = self.objects[kind].get(key)
        if cur is None:
            return self._status(404, "NotFound", "not found")
        patch = await req.json()
        if req.headers.get("Content-Type", "").startswith("application/json-patch+json"):
            new = json_patch(copy.deepcopy(cur), patch)
        else:
            new = _merge(copy.deepcopy(cur), patch)
        return web.json_response(self.update(new))

    async def _h_delete(self, req: web.Request):
        bad = await self._pre(req, "DELETE")
        if bad is not None:
            return bad
        kind = self._kind(req)
        prop = "Background"
        if req.can_read_body:
            try:
                prop = (await req.json()).get("propagationPolicy", prop)
            except ValueError:
                pass
        prop = req.query.get("propagationPolicy", prop)
        obj = self.delete(kind, req.match_info["ns"], req.match_info["name"], prop)
        if obj is None:
            return self._status(404, "NotFound", f'{kind.lower()}s.{"batch" if kind == "Job" else ""} "{req.match_info["name"]}" not found')
        return web.json_response({"kind": "Status", "apiVersion": "v1", "status": "Success",
                                  "details": {"name": req.match_info["name"], "kind": kind.lower() + "s"}})


def _line_rv(line: bytes) -> int:
    i = line.find(b'"resourceVersion":"')
    if i < 0:
        return 0
    j = line.find(b'"', i + 19)
    try:
        return int(line[i + 19:j])
    except ValueError:
        return 0
