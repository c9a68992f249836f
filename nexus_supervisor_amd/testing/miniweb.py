"""A small HTTP/1.1 server with the subset of the ``aiohttp.web`` API the fake
apiserver uses (routes with ``{placeholders}``, ``Request.json()``,
``Response``/``json_response``, chunked ``StreamResponse``).

Why not aiohttp's server: the benchmark's fake apiserver answers thousands of
pipelined ``DELETE``s per second and streams every watch event; aiohttp's
per-request machinery made the *fake* the bottleneck of the supervisor
benchmark.  This server parses pipelined requests straight from the protocol
buffer, runs each connection's requests in order, and coalesces every response
produced in one loop tick into a single ``send``.
"""
from __future__ import annotations

import asyncio
import collections
import json
import re
from typing import Any, Callable, Deque, Dict, List, Optional, Tuple
from urllib.parse import parse_qsl, unquote, urlsplit

_REASONS = {200: "OK", 201: "Created", 204: "No Content", 400: "Bad Request", 401: "Unauthorized", 404: "Not Found",
            405: "Method Not Allowed", 409: "Conflict", 410: "Gone", 500: "Internal Server Error"}


class HTTPNotFound(Exception):
    status = 404


class _Headers(dict):
    def get(self, k, d=None):  # case-insensitive
        return super().get(k.lower(), d)

    def __getitem__(self, k):
        return super().__getitem__(k.lower())

    def __contains__(self, k):
        return super().__contains__(k.lower())


class Request:
    __slots__ = ("method", "path", "query", "headers", "body", "match_info", "_conn")

    def __init__(self, method, path, query, headers, body, conn):
        self.method = method
        self.path = path
        self.query = query
        self.headers = headers
        self.body = body
        self.match_info: Dict[str, str] = {}
        self._conn = conn

    @property
    def can_read_body(self) -> bool:
        return bool(self.body)

    async def json(self):
        return json.loads(self.body) if self.body else None

    async def read(self) -> bytes:
        return self.body


class Response:
    def __init__(self, *, body: bytes = b"", status: int = 200, content_type: str = "application/json", text: str = None,
                 headers: Optional[Dict[str, str]] = None, charset: str = None):
        self.status = status
        self.body = text.encode() if text is not None else body
        self.content_type = content_type if text is None or content_type != "application/json" else "text/plain"
        self.headers = headers or {}

    def encode(self) -> bytes:
        h = [f"HTTP/1.1 {self.status} {_REASONS.get(self.status, 'OK')}", f"Content-Type: {self.content_type}",
             f"Content-Length: {len(self.body)}"]
        h += [f"{k}: {v}" for k, v in self.headers.items()]
        return ("\r\n".join(h) + "\r\n\r\n").encode("latin-1") + self.body


def json_response(obj: Any, status: int = 200, dumps: Callable = None,
                  headers: Optional[Dict[str, str]] = None) -> Response:
    data = (dumps or (lambda o: json.dumps(o, separators=(",", ":"))))(obj)
    return Response(body=data.encode() if isinstance(data, str) else data, status=status, headers=headers)


class StreamResponse:
    """Chunked streaming response (watch streams)."""

    def __init__(self, status: int = 200, headers: Optional[Dict[str, str]] = None):
        self.status = status
        self.headers = headers or {}
        self._conn: Optional["_Conn"] = None

    def enable_chunked_encoding(self) -> None:
        return None

    async def prepare(self, req: Request) -> None:
        self._conn = req._conn
        h = [f"HTTP/1.1 {self.status} {_REASONS.get(self.status, 'OK')}", "Transfer-Encoding: chunked"]
        h += [f"{k}: {v}" for k, v in self.headers.items()]
        self._conn.send(("\r\n".join(h) + "\r\n\r\n").encode("latin-1"))
        self._conn.streaming = True

    async def write(self, data: bytes) -> None:
        c = self._conn
        if c is None or c.closed:
            raise ConnectionResetError("client went away")
        if data:
            c.send(b"%x\r\n" % len(data) + data + b"\r\n")
        await c.drain()

    def finish(self) -> None:
        if self._conn is not None and not self._conn.closed:
            self._conn.send(b"0\r\n\r\n")
            self._conn.streaming = False


class _Conn(asyncio.Protocol):
    def __init__(self, server: "Server"):
        self.server = server
        self.transport: Optional[asyncio.Transport] = None
        self.buf = bytearray()
        self.queue: Deque[Request] = collections.deque()
        self.worker: Optional[asyncio.Task] = None
        self.out: List[bytes] = []
        self.flush_scheduled = False
        self.closed = False
        self.streaming = False
        self._paused = False
        self._drain_waiter: Optional[asyncio.Future] = None
        self.close_after = False

    def connection_made(self, transport):
        self.transport = transport
        self.server.conns.add(self)

    def connection_lost(self, exc):
        self.closed = True
        self.server.conns.discard(self)
        if self.worker is not None and self.streaming:
            self.worker.cancel()
        if self._drain_waiter is not None and not self._drain_waiter.done():
            self._drain_waiter.set_exception(ConnectionResetError("closed"))

    def pause_writing(self):
        self._paused = True

    def resume_writing(self):
        self._paused = False
        if self._drain_waiter is not None and not self._drain_waiter.done():
            self._drain_waiter.set_result(None)

    async def drain(self) -> None:
        if self._paused and not self.closed:
            self._drain_waiter = asyncio.get_running_loop().create_future()
            await self._drain_waiter

    def send(self, data: bytes) -> None:
        if self.closed:
            return
        self.out.append(data)
        if not self.flush_scheduled:
            self.flush_scheduled = True
            asyncio.get_running_loop().call_soon(self._flush)

    def _flush(self) -> None:
        self.flush_scheduled = False
        if self.out and not self.closed:
            self.transport.write(b"".join(self.out))
        self.out = []
        if self.close_after and not self.queue and not self.streaming and not self.closed:
            self.transport.close()

    def data_received(self, data: bytes) -> None:
        self.buf += data
        while True:
            end = self.buf.find(b"\r\n\r\n")
            if end < 0:
                return
            head = bytes(self.buf[:end]).decode("latin-1").split("\r\n")
            hdrs = _Headers()
            for line in head[1:]:
                k, _, v = line.partition(":")
                hdrs[k.strip().lower()] = v.strip()
            n = int(hdrs.get("content-length", "0") or 0)
            if len(self.buf) < end + 4 + n:
                return
            body = bytes(self.buf[end + 4:end + 4 + n])
            del self.buf[:end + 4 + n]
            try:
                method, target, _ver = head[0].split(" ", 2)
            except ValueError:
                self.transport.close()
                return
            u = urlsplit(target)
            req = Request(method, unquote(u.path), dict(parse_qsl(u.query, keep_blank_values=True)), hdrs, body, self)
            if hdrs.get("connection", "").lower() == "close":
                self.close_after = True
            self.queue.append(req)
            if self.worker is None or self.worker.done():
                self.worker = asyncio.ensure_future(self._work())

    async def _work(self) -> None:
        while self.queue and not self.closed:
            req = self.queue.popleft()
            try:
                resp = await self.server.dispatch(req)
            except HTTPNotFound:
                resp = Response(status=404, body=b'{"kind":"Status","code":404,"reason":"NotFound"}')
            except asyncio.CancelledError:
                return
            except Exception as exc:  # noqa: BLE001
                resp = Response(status=500, body=json.dumps({"kind": "Status", "code": 500, "message": str(exc)}).encode())
            if isinstance(resp, StreamResponse):
                resp.finish()
            elif resp is not None:
                self.send(resp.encode())


class Server:
    def __init__(self):
        self.routes: List[Tuple[str, re.Pattern, Callable]] = []
        self.conns: set = set()
        self._srv: Optional[asyncio.AbstractServer] = None

    def add_route(self, method: str, pattern: str, handler: Callable) -> None:
        rx = "^" + re.sub(r"\{(\w+)\}", r"(?P<\1>[^/]+)", pattern) + "$"
        self.routes.append((method, re.compile(rx), handler))

    async def dispatch(self, req: Request):
        for method, rx, handler in self.routes:
            if method != req.method:
                continue
            m = rx.match(req.path)
            if m:
                req.match_info = m.groupdict()
                return await handler(req)
        raise HTTPNotFound()

    async def start(self, host: str, port: int, backlog: int = 4096, ssl_context=None) -> int:
        loop = asyncio.get_running_loop()
        self._srv = await loop.create_server(lambda: _Conn(self), host, port, backlog=backlog, ssl=ssl_context)
        return self._srv.sockets[0].getsockname()[1]

    async def stop(self) -> None:
        if self._srv is not None:
            self._srv.close()
            for c in list(self.conns):
                if c.transport is not None:
                    c.transport.close()
            await self._srv.wait_closed()
            self._srv = None
