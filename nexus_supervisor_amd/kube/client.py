"""Minimal asyncio Kubernetes REST client: LIST + WATCH, DELETE, PATCH, Leases.

Replaces client-go's clientset + reflectors in the reference
(``/root/reference/app/app_dependencies.go:36-53`` builds the clientset from
``kube-config-path`` — empty means in-cluster; ``services/supervisor.go:70-75``
builds namespaced Event/Pod/Job informers; ``:262-291`` deletes Jobs with
``PropagationPolicy=Background``).  The Python ``kubernetes`` package is not
available offline, so the REST + watch protocol is spoken directly:

* auth: in-cluster service-account token (re-read periodically — projected
  tokens rotate) + CA, or a kubeconfig (token, client cert/key, basic auth,
  CA data or file, ``insecure-skip-tls-verify``);
* LIST with ``limit``/``continue`` pagination; WATCH from the list's
  ``resourceVersion`` with ``allowWatchBookmarks`` and a server timeout, decoded
  line-by-line from the chunked stream; ``410 Gone`` surfaces as an ERROR event
  (the informer re-lists);
* ``ListWatch`` adapter for :mod:`..informer`;
* client-side flow control as client-go has it (:mod:`.flowcontrol`): a ``kube-qps`` /
  ``kube-burst`` token bucket in front of every request (Lease calls exempt: leader
  election must not starve behind a DELETE burst — APF gives it its own priority level
  too), and ``429`` / ``5xx`` answers retried after the server's ``Retry-After``.
"""
from __future__ import annotations

import asyncio
import base64
import contextlib
import json
import logging
import os
import re
import ssl
import tempfile
import time
import urllib.parse
from typing import Any, AsyncIterator, Dict, List, Optional, Tuple

import aiohttp

from ..informer.informer import ListWatch
from ..models.kube import FINISHERS, PROJECTIONS, list_projection, watch_projection
from ..obs import delivery as _delivery
from .errors import ApiError, from_status
from .flowcontrol import EVENT, MUTATE, READ, RetryPolicy, TokenBucket, retry_after


def _native_decoder_available() -> bool:
    """The projected watch decoder is native (``csrc/kube/watch_decoder.cpp``).  A missing
    build is an error — ``python -m nexus_supervisor_amd build`` — unless the plain
    ``json`` path is asked for explicitly with ``NEXUS_PY_WATCH_DECODER=1``."""
    try:
        from .. import _kube_native  # noqa: F401

        return True
    except ImportError as exc:
        if os.environ.get("NEXUS_PY_WATCH_DECODER") == "1":
            log.warning("native watch decoder (_kube_native) not built; using json (NEXUS_PY_WATCH_DECODER=1)")
            return False
        raise ImportError("native watch decoder _kube_native is not built: run `python -m nexus_supervisor_amd build` "
                          "(or set NEXUS_PY_WATCH_DECODER=1 to use the slower json path)") from exc


def _decoder(projection):
    from .. import _kube_native

    return _kube_native.ProjectedDecoder(projection)

log = logging.getLogger("nexus_supervisor_amd.kube")

SA_DIR = "/var/run/secrets/kubernetes.io/serviceaccount"

# kind -> (api prefix, plural)
RESOURCES: Dict[str, Tuple[str, str]] = {
    "Event": ("/api/v1", "events"),
    "Pod": ("/api/v1", "pods"),
    "Job": ("/apis/batch/v1", "jobs"),
    "Lease": ("/apis/coordination.k8s.io/v1", "leases"),
    "Node": ("/api/v1", "nodes"),
    "Secret": ("/api/v1", "secrets"),
    # cluster-scoped (namespace None): the shard-label webhook's registration, whose caBundle
    # sharding.webhook-cert-bootstrap keeps in step with the certificate it minted
    "MutatingWebhookConfiguration": ("/apis/admissionregistration.k8s.io/v1", "mutatingwebhookconfigurations"),
}


_DNS_LABEL = re.compile(r"[a-z0-9]([-a-z0-9]*[a-z0-9])?")


def resource_path(kind: str, namespace: Optional[str], name: Optional[str] = None) -> str:
    prefix, plural = RESOURCES[kind]
    p = f"{prefix}/namespaces/{namespace}/{plural}" if namespace else f"{prefix}/{plural}"
    return f"{p}/{name}" if name else p


_DELETE_BODIES: Dict[str, bytes] = {}


def _delete_body(policy: str) -> bytes:
    b = _DELETE_BODIES.get(policy)
    if b is None:
        b = _DELETE_BODIES[policy] = json.dumps(
            {"kind": "DeleteOptions", "apiVersion": "v1", "propagationPolicy": policy}).encode()
    return b


class KubeConfig:
    def __init__(self, server: str, token: str = "", token_file: str = "", ca_data: Optional[bytes] = None,
                 ca_file: str = "", cert_data: Optional[bytes] = None, key_data: Optional[bytes] = None,
                 insecure: bool = False, username: str = "", password: str = "", namespace: str = "",
                 exec_config: Optional[Dict[str, Any]] = None):
        self.server = server.rstrip("/")
        self.token = token
        self.token_file = token_file
        self.ca_data, self.ca_file = ca_data, ca_file
        self.cert_data, self.key_data = cert_data, key_data
        self.insecure = insecure
        self.username, self.password = username, password
        self.namespace = namespace
        self._token_read = 0.0
        # client.authentication.k8s.io exec credential plugin (kubeconfig users[].user.exec)
        self.exec_config = exec_config
        self._exec_expiry = 0.0

    @classmethod
    def in_cluster(cls) -> "KubeConfig":
        host, port = os.environ.get("KUBERNETES_SERVICE_HOST"), os.environ.get("KUBERNETES_SERVICE_PORT", "443")
        if not host:
            raise ApiError(0, "ConfigError", "not running in a cluster (KUBERNETES_SERVICE_HOST unset) and no kube-config-path")
        if ":" in host and not host.startswith("["):
            host = f"[{host}]"
        ns = ""
        try:
            with open(os.path.join(SA_DIR, "namespace")) as f:
                ns = f.read().strip()
        except OSError:
            pass
        return cls(f"https://{host}:{port}", token_file=os.path.join(SA_DIR, "token"),
                   ca_file=os.path.join(SA_DIR, "ca.crt"), namespace=ns)

    @classmethod
    def from_file(cls, path: str, context: Optional[str] = None) -> "KubeConfig":
        import yaml

        path = os.path.expanduser(path)
        with open(path) as f:
            doc = yaml.safe_load(f) or {}
        base = os.path.dirname(os.path.abspath(path))
        ctx_name = context or doc.get("current-context")
        ctxs = {c["name"]: c.get("context", {}) for c in doc.get("contexts", [])}
        ctx = ctxs.get(ctx_name) or (next(iter(ctxs.values())) if ctxs else {})
        clusters = {c["name"]: c.get("cluster", {}) for c in doc.get("clusters", [])}
        users = {u["name"]: u.get("user", {}) for u in doc.get("users", [])}
        cl = clusters.get(ctx.get("cluster"), next(iter(clusters.values()), {}))
        us = users.get(ctx.get("user"), {})

        def data(d, key):
            if d.get(f"{key}-data"):
                return base64.b64decode(d[f"{key}-data"])
            p = d.get(key)
            if p:
                p = p if os.path.isabs(p) else os.path.join(base, p)
                with open(p, "rb") as fh:
                    return fh.read()
            return None

        token = us.get("token", "")
        token_file = us.get("tokenFile", "")
        return cls(cl.get("server", ""), token=token, token_file=token_file, ca_data=data(cl, "certificate-authority"),
                   cert_data=data(us, "client-certificate"), key_data=data(us, "client-key"),
                   insecure=bool(cl.get("insecure-skip-tls-verify")), username=us.get("username", ""),
                   password=us.get("password", ""), namespace=ctx.get("namespace", ""),
                   exec_config=us.get("exec") or None)

    @classmethod
    def load(cls, kube_config_path: str = "") -> "KubeConfig":
        """``kube-config-path`` semantics of the reference: empty → in-cluster
        (``/root/reference/app/app_dependencies.go:39``)."""
        return cls.from_file(kube_config_path) if kube_config_path else cls.in_cluster()

    def _run_exec_plugin(self) -> None:
        """Run the kubeconfig ``exec`` credential plugin (client-go semantics: ExecCredential
        JSON on stdout, ``status.token`` + optional ``expirationTimestamp``; cached until
        shortly before expiry)."""
        import subprocess

        ex = self.exec_config or {}
        cmd = [ex.get("command", "")] + list(ex.get("args") or [])
        env = dict(os.environ)
        for e in ex.get("env") or []:
            env[e["name"]] = e.get("value", "")
        api = ex.get("apiVersion", "client.authentication.k8s.io/v1")
        env["KUBERNETES_EXEC_INFO"] = json.dumps({"apiVersion": api, "kind": "ExecCredential",
                                                  "spec": {"interactive": False}})
        p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=60)
        if p.returncode != 0:
            raise ApiError(401, "Unauthorized", f"exec credential plugin {cmd[0]!r} failed: {p.stderr.strip()[-300:]}")
        status = (json.loads(p.stdout or "{}").get("status") or {})
        if not status.get("token"):
            raise ApiError(401, "Unauthorized", f"exec credential plugin {cmd[0]!r} returned no token")
        self.token = status["token"]
        exp = status.get("expirationTimestamp")
        if exp:
            import datetime as _dt

            t = _dt.datetime.fromisoformat(exp.replace("Z", "+00:00")).timestamp()
            self._exec_expiry = time.monotonic() + max(0.0, t - time.time() - 30.0)
        else:
            self._exec_expiry = float("inf")

    def bearer(self) -> str:
        if self.exec_config and (not self.token or time.monotonic() >= self._exec_expiry):
            self._run_exec_plugin()
            return self.token
        if self.token_file and (not self.token or time.monotonic() - self._token_read > 60):
            try:
                with open(self.token_file) as f:
                    self.token = f.read().strip()
                self._token_read = time.monotonic()
            except OSError as exc:
                log.warning("cannot read service account token %s: %s", self.token_file, exc)
        return self.token

    def ssl_context(self) -> Optional[ssl.SSLContext]:
        if not self.server.startswith("https"):
            return None
        ctx = ssl.create_default_context()
        if self.insecure:
            ctx.check_hostname = False
            ctx.verify_mode = ssl.CERT_NONE
        elif self.ca_data:
            ctx = ssl.create_default_context(cadata=self.ca_data.decode())
        elif self.ca_file and os.path.exists(self.ca_file):
            ctx = ssl.create_default_context(cafile=self.ca_file)
        if self.cert_data and self.key_data:
            with tempfile.TemporaryDirectory() as d:
                cp, kp = os.path.join(d, "c"), os.path.join(d, "k")
                with open(cp, "wb") as f:
                    f.write(self.cert_data)
                with open(kp, "wb") as f:
                    f.write(self.key_data)
                ctx.load_cert_chain(cp, kp)
        return ctx


def _exempt(path: str) -> bool:
    """Lease calls bypass the client-side bucket (leader election / shard leases)."""
    return "/coordination.k8s.io/" in path


class KubeClient:
    def __init__(self, config: KubeConfig, *, request_timeout: float = 30.0, max_connections: int = 32,
                 user_agent: str = "nexus-supervisor-amd/0.1", pipelined_writes: bool = True, write_connections: int = 4,
                 qps: Optional[float] = None, burst: int = 1, max_retries: int = 10, metrics=None,
                 read_connections: int = 8):
        self.config = config
        self.read_connections = read_connections
        # client-go rest.Config QPS / Burst (kube-qps / kube-burst; 0 = no client-side limit).
        # Given here, they stay: an Application only applies its config's to a client built
        # without them
        self.flow_configured = qps is not None
        self.limiter = TokenBucket(qps or 0.0, burst)
        self.retry = RetryPolicy(max_retries)
        self.metrics = metrics  # obs.metrics.Metrics: kube_throttled / kube_retries / kube_ratelimit_waits
        self.throttled = 0      # 429 / hinted 5xx answers seen
        self.retried = 0        # requests re-sent after a Retry-After
        self.pipelined_writes = pipelined_writes
        self.write_connections = write_connections
        self._fast = None
        self._reads = None  # one-request-per-connection pool for pods/log tails (_read_client)
        self.request_timeout = request_timeout
        self.max_connections = max_connections
        self.user_agent = user_agent
        self._session: Optional[aiohttp.ClientSession] = None
        self.requests = 0

    async def _s(self) -> aiohttp.ClientSession:
        if self._session is None or self._session.closed:
            conn = aiohttp.TCPConnector(limit=self.max_connections, ssl=self.config.ssl_context() or False,
                                        enable_cleanup_closed=True)
            self._session = aiohttp.ClientSession(connector=conn, timeout=aiohttp.ClientTimeout(total=None, sock_connect=10),
                                                  headers={"User-Agent": self.user_agent, "Accept": "application/json"},
                                                  json_serialize=json.dumps)
        return self._session

    def _headers(self, extra: Optional[Dict[str, str]] = None) -> Dict[str, str]:
        h: Dict[str, str] = {}
        tok = self.config.bearer()
        if tok:
            h["Authorization"] = f"Bearer {tok}"
        elif self.config.username:
            raw = f"{self.config.username}:{self.config.password}".encode()
            h["Authorization"] = "Basic " + base64.b64encode(raw).decode()
        if extra:
            h.update(extra)
        return h

    async def close(self) -> None:
        if self._session is not None:
            await self._session.close()
            self._session = None
        if self._fast is not None:
            await self._fast.close()
            self._fast = None
        if self._reads is not None:
            await self._reads.close()
            self._reads = None

    def _read_client(self):
        """Keep-alive connections for the ``pods/log`` reads a GPU failure waits on.  Not
        pipelined (``max_depth`` 1): a tail is proxied through the node's kubelet and may be
        slow, and must not hold up the reads queued behind it.  Through aiohttp one read cost
        ~190 µs of CPU, here ~40 µs (the default-pod HBM-OOM shape reads one per GPU failure)."""
        if self._reads is None:
            from .fasthttp import PipelinedHttp

            self._reads = PipelinedHttp(self.config.server, connections=self.read_connections, max_depth=1,
                                        ssl_ctx=self.config.ssl_context(), timeout=self.request_timeout,
                                        default_headers={"User-Agent": self.user_agent, "Accept": "*/*"})
        return self._reads

    def _fast_client(self):
        if self._fast is None:
            from .fasthttp import PipelinedHttp

            self._fast = PipelinedHttp(self.config.server, connections=self.write_connections,
                                       ssl_ctx=self.config.ssl_context(), timeout=self.request_timeout,
                                       default_headers={"User-Agent": self.user_agent, "Accept": "application/json"})
        return self._fast

    # ------------------------------------------------------------------ flow control
    def set_flow_control(self, qps: float, burst: int, max_retries: int = 10, metrics=None, shared=None) -> None:
        """``kube-qps`` / ``kube-burst`` / ``kube-max-retries`` of this process's share
        (``shared``: the replica's :class:`..flowcontrol.SharedSchedule` instead)."""
        self.limiter = TokenBucket(qps, burst, shared=shared)
        self.retry = RetryPolicy(max_retries)
        if metrics is not None:
            self.metrics = metrics

    @classmethod
    def for_config(cls, cfg, metrics=None, schedule=None, **kw) -> "KubeClient":
        """A client for ``cfg.kube-config-path`` with this process's share of the flow
        control: the replica's shared budget when it has one (``schedule``, or the one a
        shard worker inherited), else 1/K of it for each of K processes."""
        c = cls(KubeConfig.load(cfg.kube_config_path), **kw)
        c.apply_config(cfg, metrics, schedule)
        return c

    def apply_config(self, cfg, metrics=None, schedule=None) -> None:
        from .flowcontrol import replica_schedule, split

        if schedule is None:
            schedule = replica_schedule(cfg)
        if schedule is not None:
            self.set_flow_control(cfg.kube_qps, cfg.kube_burst, cfg.kube_max_retries, metrics, shared=schedule)
        else:
            # K processes and no shared mapping: 1/K each, the hub parent counted as one more
            parts = max(1, int(getattr(cfg.runtime, "worker_processes", 1) or 1))
            if parts > 1:
                parts += 1
            qps, burst = split(cfg.kube_qps, cfg.kube_burst, parts)
            self.set_flow_control(qps, burst, cfg.kube_max_retries, metrics)
        if self._reads is None:  # one connection per concurrent pods/log read
            self.read_connections = max(1, int(getattr(cfg.gpu, "log_tail_concurrency", self.read_connections)))

    async def _admit(self, path: str, method: str = "GET", timeout: Optional[float] = None) -> None:
        lim = self.limiter
        if lim.qps > 0 and not _exempt(path):
            # request classes (flowcontrol.CLASS_WEIGHTS): reads (pods/log tails a decision
            # waits for, LIST / WATCH), mutations (background Job DELETEs, agent PATCHes),
            # decision Events — each with a guaranteed share of the tokens
            prio = READ if method == "GET" else EVENT if method == "POST" and path.endswith("/events") else MUTATE
            d = await lim.wait(prio, timeout)
            if d > 0 and self.metrics is not None:
                self.metrics.inc("kube_ratelimit_waits")
                self.metrics.observe_seconds("kube_ratelimit_wait", d)

    def _backoff(self, method: str, status: int, hint: Optional[float], attempt: int,
                 deadline: Optional[float] = None) -> Optional[float]:
        """Seconds to wait before re-sending an answer ``status`` (None: raise it)."""
        if status < 429:
            return None
        self.throttled += 1
        if self.metrics is not None:
            self.metrics.inc("kube_throttled", labels={"verb": method, "code": str(status)})
        d = self.retry.delay(status, hint)
        if d is None or attempt >= self.retry.max_retries:
            return None
        if deadline is not None and time.monotonic() + d > deadline:
            return None  # the caller's budget ends before the hint: give up now
        self.retried += 1
        if self.metrics is not None:
            self.metrics.inc("kube_retries", labels={"verb": method})
        return d

    async def request(self, method: str, path: str, *, params: Optional[Dict[str, Any]] = None, body: Any = None,
                      content_type: str = "application/json", timeout: Optional[float] = None,
                      decoder=None) -> Dict[str, Any]:
        s = await self._s()
        data = json.dumps(body) if body is not None else None
        attempt = 0
        while True:
            await self._admit(path, method)
            self.requests += 1
            async with s.request(method, self.config.server + path, params=params, data=data,
                                 headers=self._headers({"Content-Type": content_type} if data is not None else None),
                                 timeout=aiohttp.ClientTimeout(total=timeout or self.request_timeout)) as r:
                raw = await r.read()
                status = r.status
                hint = retry_after(r.headers.get("Retry-After")) if status >= 429 else None
            if status >= 400:
                d = self._backoff(method, status, hint, attempt)
                if d is not None:
                    attempt += 1
                    await asyncio.sleep(d)
                    continue
            try:
                if decoder is not None and status < 400 and raw:
                    doc = decoder.decode(raw)
                else:
                    doc = json.loads(raw) if raw else {}
            except ValueError:
                doc = {"message": raw[:500].decode("utf-8", "replace")}
            if status >= 400:
                raise from_status(status, doc, hint)
            return doc

    async def get_raw(self, path: str, params: Optional[Dict[str, str]] = None,
                      timeout: Optional[float] = None) -> Tuple[int, bytes]:
        """GET returning ``(status, raw body)`` (the watch hub splits LIST bodies natively).
        A 429 / hinted 5xx is re-sent after its ``Retry-After`` while that fits in
        ``timeout`` (the whole call's budget)."""
        s = await self._s()
        total = timeout or max(60.0, self.request_timeout)
        deadline = time.monotonic() + total
        attempt = 0
        while True:
            await self._admit(path)
            self.requests += 1
            left = max(0.05, deadline - time.monotonic())
            async with s.get(self.config.server + path, params=params, headers=self._headers(),
                             timeout=aiohttp.ClientTimeout(total=left)) as r:
                status, raw = r.status, await r.read()
                hint = retry_after(r.headers.get("Retry-After")) if status >= 429 else None
            if status >= 429:
                d = self._backoff("GET", status, hint, attempt, deadline)
                if d is not None:
                    attempt += 1
                    await asyncio.sleep(d)
                    continue
            return status, raw

    @contextlib.asynccontextmanager
    async def stream(self, path: str, params: Optional[Dict[str, str]] = None, timeout: float = 330.0):
        """Streaming GET (a watch); yields the response, its ``content`` read raw."""
        s = await self._s()
        await self._admit(path)
        self.requests += 1
        async with s.get(self.config.server + path, params=params, headers=self._headers(),
                         timeout=aiohttp.ClientTimeout(total=timeout, sock_read=timeout)) as r:
            yield r

    # ------------------------------------------------------------------ typed helpers
    async def list(self, kind: str, namespace: Optional[str], *, label_selector: str = "", field_selector: str = "",
                   limit: int = 500, projected: bool = False) -> Tuple[List[Dict[str, Any]], str]:
        decoder = _decoder(list_projection(kind)) if projected else None
        items: List[Dict[str, Any]] = []
        cont = ""
        rv = ""
        while True:
            params: Dict[str, Any] = {"limit": str(limit)}
            if label_selector:
                params["labelSelector"] = label_selector
            if field_selector:
                params["fieldSelector"] = field_selector
            if cont:
                params["continue"] = cont
            doc = await self.request("GET", resource_path(kind, namespace), params=params, decoder=decoder)
            api_version, k = doc.get("apiVersion", ""), kind
            for it in doc.get("items") or []:
                it.setdefault("kind", k)
                if api_version:
                    it.setdefault("apiVersion", api_version)
                items.append(it)
            meta = doc.get("metadata") or {}
            rv = meta.get("resourceVersion", rv)
            cont = meta.get("continue", "")
            if not cont:
                return items, rv

    async def watch(self, kind: str, namespace: Optional[str], resource_version: str, *, label_selector: str = "",
                    field_selector: str = "", timeout_seconds: int = 300, projected: bool = False,
                    router=None) -> AsyncIterator[Tuple[str, Dict[str, Any]]]:
        """Watch stream as ``(type, object)``.  ``router`` = ``(ShardRouter, role)`` drops
        lines another shard worker owns before they are decoded (native decoder only)."""
        s = await self._s()
        params = {"watch": "1", "resourceVersion": resource_version, "allowWatchBookmarks": "true",
                  "timeoutSeconds": str(timeout_seconds)}
        if label_selector:
            params["labelSelector"] = label_selector
        if field_selector:
            params["fieldSelector"] = field_selector
        await self._admit(resource_path(kind, namespace))
        self.requests += 1
        async with s.get(self.config.server + resource_path(kind, namespace), params=params, headers=self._headers(),
                         timeout=aiohttp.ClientTimeout(total=timeout_seconds + 30, sock_read=timeout_seconds + 30)) as r:
            if r.status >= 400:
                doc = {}
                try:
                    doc = json.loads(await r.read())
                except ValueError:
                    pass
                if r.status == 410:
                    yield "ERROR", {"kind": "Status", "code": 410, "reason": "Expired", "message": doc.get("message", "")}
                    return
                hint = retry_after(r.headers.get("Retry-After")) if r.status >= 429 else None
                if r.status >= 429:
                    self._backoff("WATCH", r.status, hint, self.retry.max_retries)  # counted; the informer waits
                raise from_status(r.status, doc, hint)
            decoder = _decoder(watch_projection(kind)) if projected else None
            if decoder is not None and router is not None:
                decoder.set_router(*router)
            if decoder is not None:
                n = 0
                current = _delivery.CURRENT
                async for chunk in r.content.iter_any():
                    t_read = time.monotonic()
                    evs = decoder.feed(chunk)
                    if not evs:
                        continue
                    # hub-less replica: the chunk's read is both the "hub" and "feed" stamp
                    current[kind] = (t_read, t_read, time.monotonic())
                    try:
                        for ev in evs:
                            obj = ev.get("object") or {}
                            if obj.get("kind") is None:
                                obj["kind"] = kind
                            yield ev.get("type", ""), obj
                            n += 1
                            if n % 64 == 0:
                                await asyncio.sleep(0)  # let workers interleave with a large chunk
                    finally:
                        # stamps belong to this chunk only: a later resync / timer / log-fetch
                        # submit must not pick them up
                        current.pop(kind, None)
                return
            loads = json.loads
            buf = b""
            async for chunk in r.content.iter_any():
                buf += chunk
                if b"\n" not in buf:
                    continue
                lines = buf.split(b"\n")
                buf = lines.pop()
                for line in lines:
                    if not line.strip():
                        continue
                    ev = loads(line)
                    obj = ev.get("object") or {}
                    if kind != "Status" and obj.get("kind") is None:
                        obj["kind"] = kind
                    yield ev.get("type", ""), obj
            if buf.strip():
                ev = loads(buf)
                yield ev.get("type", ""), ev.get("object") or {}

    async def get(self, kind: str, namespace: Optional[str], name: str) -> Dict[str, Any]:
        return await self.request("GET", resource_path(kind, namespace, name))

    async def create(self, kind: str, namespace: Optional[str], obj: Dict[str, Any]) -> Dict[str, Any]:
        return await self.request("POST", resource_path(kind, namespace), body=obj)

    async def replace(self, kind: str, namespace: Optional[str], name: str, obj: Dict[str, Any]) -> Dict[str, Any]:
        return await self.request("PUT", resource_path(kind, namespace, name), body=obj)

    async def patch_merge(self, kind: str, namespace: Optional[str], name: str, patch: Dict[str, Any],
                          want_body: bool = True) -> Dict[str, Any]:
        path = resource_path(kind, namespace, name)
        if not self.pipelined_writes:
            return await self.request("PATCH", path, body=patch, content_type="application/merge-patch+json")
        body = json.dumps(patch, separators=(",", ":")).encode()
        return await self._write("PATCH", path, body, "application/merge-patch+json", want_body)

    async def delete(self, kind: str, namespace: Optional[str], name: str, propagation_policy: str = "Background",
                     want_body: bool = True) -> Dict[str, Any]:
        path = resource_path(kind, namespace, name)
        if not self.pipelined_writes:
            body = {"kind": "DeleteOptions", "apiVersion": "v1", "propagationPolicy": propagation_policy}
            return await self.request("DELETE", path, body=body)
        return await self._write("DELETE", path, _delete_body(propagation_policy), "application/json", want_body)

    async def _write(self, method: str, path: str, body: bytes, content_type: str, want_body: bool) -> Dict[str, Any]:
        """A mutation over the pipelined keep-alive connections (an aiohttp request costs
        several times the CPU): flow control, 429 / Retry-After backoff, API errors raised."""
        attempt = 0
        while True:
            await self._admit(path, method)
            self.requests += 1
            status, raw = await self._fast_client().request(method, path, body, self._headers({"Content-Type": content_type}))
            if status < 400 and not want_body:
                return {}  # the object is not needed: skip decoding it
            hint = retry_after(getattr(raw, "retry_after", None)) if status >= 429 else None
            if status >= 429:
                d = self._backoff(method, status, hint, attempt)
                if d is not None:
                    attempt += 1
                    await asyncio.sleep(d)
                    continue
            try:
                doc = json.loads(raw) if raw else {}
            except ValueError:
                doc = {"message": raw[:500].decode("utf-8", "replace")}
            if status >= 400:
                raise from_status(status, doc, hint)
            return doc

    async def pod_log(self, namespace: str, name: str, container: str, *, previous: bool = False,
                      tail_lines: int = 200, limit_bytes: int = 65536, timeout: float = 2.0) -> Tuple[int, bytes]:
        """``GET …/pods/<name>/log`` tail of one container instance: ``(status, raw text)``
        (``previous``: the instance before the last restart)."""
        path = resource_path("Pod", namespace, name) + "/log"
        if not self.pipelined_writes:
            params = {"container": container, "tailLines": str(int(tail_lines)), "limitBytes": str(int(limit_bytes))}
            if previous:
                params["previous"] = "true"
            return await self.get_raw(path, params, timeout=timeout)
        # container names are DNS labels: quoting (urlencode was ~10 % of a read) only when
        # one is not
        c = container if _DNS_LABEL.fullmatch(container) else urllib.parse.quote(container, safe="")
        url = f"{path}?container={c}&tailLines={int(tail_lines)}&limitBytes={int(limit_bytes)}"
        if previous:
            url += "&previous=true"
        deadline = time.monotonic() + timeout
        attempt = 0
        reads = self._read_client()
        while True:
            if self.limiter.qps > 0:
                try:
                    # the token wait counts against the read's own budget: a tail that cannot
                    # be read in time is no evidence, and the decision must not wait longer
                    await self._admit(path, "GET", max(0.0, deadline - time.monotonic()))
                except asyncio.TimeoutError:
                    if self.metrics is not None:
                        self.metrics.inc("kube_ratelimit_gaveup", labels={"verb": "GET"})
                    raise
            self.requests += 1
            left = max(0.05, deadline - time.monotonic())
            # an idle keep-alive connection takes it without a coroutine or a timer per read
            fut = reads.request_nowait("GET", url, None, self._headers(), timeout=left)
            status, raw = await (fut if fut is not None else reads.request("GET", url, None, self._headers(), timeout=left))
            if status >= 429:
                d = self._backoff("GET", status, retry_after(getattr(raw, "retry_after", None)), attempt, deadline)
                if d is not None:
                    attempt += 1
                    await asyncio.sleep(d)
                    continue
            return status, raw

    # JobClient protocol (Supervisor actuator)
    async def delete_job(self, namespace: str, name: str, propagation_policy: str = "Background") -> None:
        await self.delete("Job", namespace, name, propagation_policy, want_body=False)

    def delete_job_nowait(self, namespace: str, name: str, propagation_policy: str = "Background"):
        """Fire the Job DELETE on an already-open pipelined connection; returns a future of
        ``(status, body)`` for :meth:`check_delete`, or ``None`` (use :meth:`delete_job`)."""
        if not self.pipelined_writes or self._fast is None:
            return None
        if not self.limiter.try_accept():
            return None  # no banked token: the retrying coroutine waits for one
        fut = self._fast.request_nowait("DELETE", resource_path("Job", namespace, name), _delete_body(propagation_policy),
                                        self._headers({"Content-Type": "application/json"}))
        if fut is None:
            # no pipelined connection had room: the fallback DELETE takes its own token
            self.limiter.give_back()
        else:
            self.requests += 1
        return fut

    def check_delete(self, result) -> None:
        """Raise the API error of a :meth:`delete_job_nowait` response (2xx: nothing); a
        429's ``Retry-After`` rides on the error (the caller's retry waits for it)."""
        status, raw = result
        if status < 400:
            return
        hint = None
        if status >= 429:
            hint = retry_after(getattr(raw, "retry_after", None))
            self.throttled += 1
            if self.metrics is not None:
                self.metrics.inc("kube_throttled", labels={"verb": "DELETE", "code": str(status)})
            if hint is None and status == 429:
                hint = self.retry.default_429
        try:
            doc = json.loads(raw) if raw else {}
        except ValueError:
            doc = {"message": raw[:500].decode("utf-8", "replace")}
        raise from_status(status, doc, hint)


class KubeListWatch(ListWatch):
    """Informer transport over :class:`KubeClient` (one kind, one namespace)."""

    def __init__(self, client: KubeClient, kind: str, namespace: Optional[str], *, label_selector: str = "",
                 field_selector: str = "", watch_timeout: int = 300, page_size: int = 500, projected: bool = True):
        self.client = client
        self.kind = kind
        self.namespace = namespace
        self.label_selector = label_selector
        self.field_selector = field_selector
        self.watch_timeout = watch_timeout
        self.page_size = page_size
        # native projected decoding when available: objects arrive already slimmed, the
        # informer then only runs the cheap finisher instead of the Python slimmer
        self.projected = projected and _native_decoder_available() and kind in PROJECTIONS
        if self.projected:
            self.transform = FINISHERS.get(kind)
        self.shard_router = None  # (native ShardRouter, role) when this replica is split into workers

    async def list(self):
        return await self.client.list(self.kind, self.namespace, label_selector=self.label_selector,
                                      field_selector=self.field_selector, limit=self.page_size, projected=self.projected)

    def watch(self, resource_version: str):
        return self.client.watch(self.kind, self.namespace, resource_version, label_selector=self.label_selector,
                                 field_selector=self.field_selector, timeout_seconds=self.watch_timeout,
                                 projected=self.projected, router=self.shard_router if self.projected else None)
