"""Process wrapper for the native kube-apiserver simulator (``csrc/kubesim`` →
``bin/nexus-kubesim``).

The simulator speaks the same REST + watch protocol as
:mod:`.fake_apiserver` (the supervisor's :class:`~..kube.client.KubeClient` and
informers run unchanged against it) but on a native epoll loop, so a benchmark's
cluster side is never the bottleneck.  State is driven over HTTP: ordinary REST
calls, or ``POST /sim/apply`` with NDJSON watch events for bulk traffic.
"""
from __future__ import annotations

import json
import os
import subprocess
import tempfile
import time
from typing import Any, Dict, Iterable, List, Optional, Tuple

from ..utils.proc import die_with_parent

try:
    from .._kube_native import dumps as _dumps

    def _line(etype: str, obj: Dict[str, Any]) -> bytes:
        return _dumps({"type": etype, "object": obj}, newline=True)
except ImportError:  # pragma: no cover
    def _line(etype: str, obj: Dict[str, Any]) -> bytes:
        return json.dumps({"type": etype, "object": obj}, separators=(",", ":")).encode() + b"\n"


def encode_events(events: Iterable[Tuple[str, Dict[str, Any]]]) -> bytes:
    """NDJSON body for ``/sim/apply``."""
    return b"".join(_line(t, o) for t, o in events)


class KubeSim:
    def __init__(self, *, host: str = "127.0.0.1", port: int = 0, history: int = 400_000, bookmark_ms: int = 1000,
                 token: str = "", flush_threads: int = 1, api_latency_us: int = 0, write_qps: float = 0.0,
                 write_burst: int = 0, throttle_deletes: int = 0, retry_after: int = 1, prefault_mb: int = 0,
                 apply_threads: int = 1, log_root: str = "", async_gc: bool = False):
        from .._build import binary

        self.exe = os.environ.get("NEXUS_KUBESIM_BINARY") or binary("nexus-kubesim")
        self.dir = tempfile.mkdtemp(prefix="nexus-kubesim-")
        self.host, self.port = host, port
        self.history, self.bookmark_ms, self.token = history, bookmark_ms, token
        self.flush_threads = flush_threads  # parallel watch fan-out (many watching replicas)
        # pricing the API server: answer latency, APF-like write cap (429 + Retry-After) and
        # injected 429s on the first Job DELETEs
        self.api_latency_us, self.write_qps, self.write_burst = api_latency_us, write_qps, write_burst
        self.throttle_deletes, self.retry_after = throttle_deletes, retry_after
        self.prefault_mb = prefault_mb  # heap grown and touched at startup (benchmarks)
        self.apply_threads = apply_threads  # threads preparing a /sim/apply chunk's lines
        self.log_root = log_root  # a kubelet's /var/log/pods the LOG lines are also written to
        # a Background Job DELETE is answered before its pods go (the GC deletes them after)
        self.async_gc = async_gc
        self.proc: Optional[subprocess.Popen] = None
        self.log_path = os.path.join(self.dir, "server.log")
        self.url = ""
        self.apply_url = ""  # the bulk-apply port (its own threads beside the event loop)

    def start(self, timeout: float = 10.0) -> "KubeSim":
        ready = os.path.join(self.dir, "ready")
        if os.path.exists(ready):
            os.unlink(ready)
        argv = [self.exe, "--host", self.host, "--port", str(self.port), "--ready-file", ready,
                "--history", str(self.history), "--bookmark-ms", str(self.bookmark_ms)]
        if self.token:
            argv += ["--token", self.token]
        if self.flush_threads > 1:
            argv += ["--flush-threads", str(self.flush_threads)]
        if self.prefault_mb:
            argv += ["--prefault-mb", str(int(self.prefault_mb))]
        if self.apply_threads > 1:
            argv += ["--apply-threads", str(int(self.apply_threads))]
        if self.api_latency_us:
            argv += ["--api-latency-us", str(int(self.api_latency_us))]
        if self.log_root:
            argv += ["--log-root", self.log_root]
        if self.async_gc:
            argv += ["--async-gc"]
        if self.write_qps:
            argv += ["--write-qps", str(self.write_qps), "--write-burst", str(int(self.write_burst))]
        if self.throttle_deletes:
            argv += ["--throttle-deletes", str(int(self.throttle_deletes))]
        if self.throttle_deletes or self.write_qps:
            argv += ["--retry-after", str(int(self.retry_after))]
        logf = open(self.log_path, "ab")
        # glibc's per-thread cache for every object-sized chunk (up to 4 KiB, no count limit):
        # the simulator allocates and frees a dozen strings per watch line
        env = dict(os.environ)
        env.setdefault("GLIBC_TUNABLES", "glibc.malloc.tcache_count=65535:glibc.malloc.tcache_max=4096")
        self.proc = subprocess.Popen(argv, stdout=logf, stderr=logf, start_new_session=True, env=env,
                                     preexec_fn=die_with_parent())
        logf.close()
        deadline = time.monotonic() + timeout
        while time.monotonic() < deadline:
            if os.path.exists(ready):
                with open(ready) as f:
                    info = json.load(f)
                self.port = info["port"]
                self.url = info["url"]
                self.apply_url = info.get("apply_url", "")
                return self
            if self.proc.poll() is not None:
                raise RuntimeError(f"nexus-kubesim exited rc={self.proc.returncode}: {self.log()}")
            time.sleep(0.01)
        self.stop()
        raise RuntimeError("nexus-kubesim did not become ready")

    def log(self) -> str:
        try:
            with open(self.log_path) as f:
                return f.read()[-4000:]
        except OSError:
            return ""

    def stop(self) -> None:
        if self.proc is not None and self.proc.poll() is None:
            self.proc.terminate()
            try:
                self.proc.wait(5)
            except subprocess.TimeoutExpired:
                self.proc.kill()
                self.proc.wait(5)

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()


class SimControl:
    """Async client for the ``/sim/*`` control endpoints (one pooled aiohttp session).
    ``apply_url``: the simulator's apply port — bulk applies are read and prepared there
    beside the event loop (``expire`` ones still go to the loop)."""

    def __init__(self, url: str, apply_url: str = ""):
        self.url = url.rstrip("/")
        self.apply_url = (apply_url or url).rstrip("/")
        self._s = None
        self._streams: List[Any] = []  # idle pipelined apply connections: (reader, writer)

    async def _session(self):
        if self._s is None:
            import aiohttp

            self._s = aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=600))
        return self._s

    async def apply(self, events: List[Tuple[str, Dict[str, Any]]], expire: bool = False) -> Dict[str, Any]:
        """Commit watch events; ``expire`` compacts history past them before any watcher
        reads them (resuming watches get 410 Gone)."""
        s = await self._session()
        base = self.url if expire else self.apply_url
        async with s.post(base + "/sim/apply", data=encode_events(events), params={"expire": "1"} if expire else None,
                          headers={"Content-Type": "application/x-ndjson"}) as r:
            doc = await r.json(content_type=None)
            if r.status != 200:
                raise RuntimeError(f"/sim/apply: {r.status} {doc}")
            return doc

    async def apply_raw(self, body: bytes) -> Dict[str, Any]:
        """``apply`` with a pre-encoded NDJSON body (:func:`encode_events`)."""
        s = await self._session()
        async with s.post(self.apply_url + "/sim/apply", data=body, headers={"Content-Type": "application/x-ndjson"}) as r:
            doc = await r.json(content_type=None)
            if r.status != 200:
                raise RuntimeError(f"/sim/apply: {r.status} {doc}")
            return doc

    async def apply_pipelined(self, bodies: List[bytes], depth: int = 3) -> List[Dict[str, Any]]:
        """``apply_raw`` for every body, in order, over one keep-alive connection with up to
        ``depth`` requests sent ahead of their answers (HTTP/1.1 pipelining).  The apply port
        reads a connection's requests one after another, so the order of commits is the
        order of ``bodies``; what pipelining removes is the port idling on the generator's
        round trip between two chunks of a step.  Returns each body's answer."""
        import asyncio

        if not bodies:
            return []
        if self._streams:  # one call owns a connection: concurrent callers (slots) never share one
            reader, writer = self._streams.pop()
        else:
            host, port = self.apply_url.split("//", 1)[1].rsplit(":", 1)
            reader, writer = await asyncio.open_connection(host, int(port))
        head = b"POST /sim/apply HTTP/1.1\r\nHost: sim\r\nContent-Type: application/x-ndjson\r\nContent-Length: %d\r\n\r\n"
        out: List[Dict[str, Any]] = []
        sent = 0
        try:
            while sent < min(depth, len(bodies)):
                writer.write(head % len(bodies[sent]))
                writer.write(bodies[sent])
                sent += 1
            await writer.drain()
            for _ in range(len(bodies)):
                hdr = await reader.readuntil(b"\r\n\r\n")
                status = int(hdr.split(b" ", 2)[1])
                clen = 0
                for ln in hdr.split(b"\r\n")[1:]:
                    k, _, v = ln.partition(b":")
                    if k.strip().lower() == b"content-length":
                        clen = int(v)
                doc = json.loads(await reader.readexactly(clen)) if clen else {}
                if status != 200:
                    raise RuntimeError(f"/sim/apply: {status} {doc}")
                out.append(doc)
                if sent < len(bodies):
                    writer.write(head % len(bodies[sent]))
                    writer.write(bodies[sent])
                    sent += 1
                    await writer.drain()
        except BaseException:
            # a broken or abandoned exchange: answers still owed on this connection would
            # be read as the next call's
            writer.close()
            raise
        self._streams.append((reader, writer))
        return out

    async def _post(self, path: str, kind: str = "") -> None:
        s = await self._session()
        async with s.post(self.url + path, params={"kind": kind} if kind else None) as r:
            r.raise_for_status()

    async def expire(self, kind: str = "") -> None:
        await self._post("/sim/expire", kind)

    async def close_watches(self, kind: str = "") -> None:
        await self._post("/sim/close-watches", kind)

    async def stats(self) -> Dict[str, Any]:
        s = await self._session()
        async with s.get(self.url + "/sim/stats") as r:
            return await r.json(content_type=None)

    async def close(self) -> None:
        if self._s is not None:
            await self._s.close()
            self._s = None
        for _, writer in self._streams:
            writer.close()
        self._streams.clear()
