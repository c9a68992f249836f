"""Pipelined HTTP/1.1 client for the supervisor's Kubernetes write path.

Every failing decision issues one ``DELETE …/jobs/{name}`` (the reference:
``/root/reference/services/supervisor.go:262-291``).  Through a general-purpose
client each request costs a connection checkout, header objects and at least
one ``send``/``recv`` pair; at thousands of decisions per second that overhead
dominates the actuator.  This client keeps a few persistent connections,
*pipelines* requests on them (HTTP/1.1 §6.3.2 — Go's ``net/http`` and aiohttp
servers both process pipelined requests in order), coalesces every request
issued in one loop tick into a single ``send``, and parses responses
incrementally in arrival order.

Only idempotent methods should be pipelined (a connection dropped mid-flight
fails every request queued on it; DELETE retried after a lost response sees
``404``, which the actuator treats as success).
"""
from __future__ import annotations

import asyncio
import collections
import ssl as _ssl
from typing import Deque, Dict, List, Optional, Tuple
from urllib.parse import urlsplit


class _Expired(Exception):
    pass


def _expire(fut: asyncio.Future) -> None:
    if not fut.done():
        fut.set_exception(_Expired())


class HttpError(Exception):
    pass


def _header(head: bytes, name: bytes) -> bytes:
    """Value of header ``name`` (``b"\\r\\nname:"``, lower case) in a lower-cased response
    head that ends with CRLF; empty when absent."""
    i = head.find(name)
    if i < 0:
        return b""
    i += len(name)
    return head[i: head.index(b"\r\n", i)].strip()


class HintedBody(bytes):
    """Body of an error answer that carried a ``Retry-After`` header (raw header value in
    :attr:`retry_after`): the result stays ``(status, body)``."""

    retry_after: bytes = b""


def _expire_and_reset(fut: asyncio.Future, conn: "_Conn", what: str) -> None:
    if not fut.done():
        fut.set_exception(HttpError(f"{what} timed out"))
        conn._fail(HttpError("request timed out"))  # response order on this connection unknown


class _Conn(asyncio.Protocol):
    def __init__(self, pool: "PipelinedHttp"):
        self.pool = pool
        self.transport: Optional[asyncio.Transport] = None
        self.waiting: Deque[asyncio.Future] = collections.deque()
        # (deadline, method, path) of each request_nowait in ``waiting`` order (None for a
        # request() with its own timer): FIFO on one connection, so the head expires first
        self.deadlines: Deque[Optional[Tuple[float, str, str]]] = collections.deque()
        self.buf = bytearray()
        self.out: List[bytes] = []
        self.flush_scheduled = False
        self.closed = False
        # parser state for the response at the head of the queue
        self._status = 0
        self._close = False
        self._need = -1       # body bytes still needed (content-length mode)
        self._chunked = False
        self._body = bytearray()
        self._in_body = False
        self._hint = b""

    # ----------------------------------------------------------- asyncio.Protocol
    def connection_made(self, transport):
        self.transport = transport

    def connection_lost(self, exc):
        self.closed = True
        err = HttpError(f"connection lost: {exc}")
        self.deadlines.clear()
        while self.waiting:
            f = self.waiting.popleft()
            if not f.done():
                f.set_exception(err)
        self.pool._drop(self)

    def data_received(self, data: bytes):
        self.buf += data
        try:
            while self.waiting and self._parse():
                pass
        except HttpError as exc:
            self._fail(exc)

    # ----------------------------------------------------------- parsing
    def _parse(self) -> bool:
        buf = self.buf
        if not self._in_body:
            end = buf.find(b"\r\n\r\n")
            if end < 0:
                return False
            # only the status and the three framing headers matter: find them in the
            # lower-cased head instead of building a header dict per response
            head = bytes(buf[:end + 2]).lower()
            del buf[: end + 4]
            sp = head.find(b" ")
            if not head.startswith(b"http/1.") or sp < 0:
                raise HttpError(f"bad status line {head[:80]!r}")
            try:
                self._status = int(head[sp + 1: sp + 4])
            except ValueError:
                raise HttpError(f"bad status line {head[:80]!r}") from None
            self._chunked = b"chunked" in _header(head, b"\r\ntransfer-encoding:")
            self._need = -1 if self._chunked else int(_header(head, b"\r\ncontent-length:") or b"0")
            self._close = _header(head, b"\r\nconnection:") == b"close"
            # 429 / 5xx: keep the server's Retry-After hint (API Priority and Fairness)
            self._hint = _header(head, b"\r\nretry-after:") if self._status >= 429 else b""
            self._body = bytearray()
            self._in_body = True
        if self._chunked:
            while True:
                end = buf.find(b"\r\n")
                if end < 0:
                    return False
                size = int(bytes(buf[:end]).split(b";", 1)[0], 16)
                if len(buf) < end + 2 + size + 2:
                    return False
                if size == 0:
                    # no trailers expected from the apiserver
                    del buf[: end + 4]
                    break
                self._body += buf[end + 2: end + 2 + size]
                del buf[: end + 2 + size + 2]
        else:
            if len(buf) < self._need:
                return False
            self._body = bytearray(buf[: self._need])
            del buf[: self._need]
        self._in_body = False
        fut = self.waiting.popleft()
        self.deadlines.popleft()
        if not fut.done():
            if self._hint:
                body = HintedBody(self._body)
                body.retry_after = self._hint
                fut.set_result((self._status, body))
            else:
                fut.set_result((self._status, bytes(self._body)))
        if self._close:
            self.transport.close()
        return True

    def _fail(self, exc: Exception) -> None:
        self.deadlines.clear()
        while self.waiting:
            f = self.waiting.popleft()
            if not f.done():
                f.set_exception(exc)
        if self.transport is not None:
            self.transport.close()

    # ----------------------------------------------------------- sending
    def send(self, data: bytes, fut: asyncio.Future, deadline: Optional[Tuple[float, str, str]] = None) -> None:
        self.waiting.append(fut)
        self.deadlines.append(deadline)
        self.out.append(data)
        if not self.flush_scheduled:
            self.flush_scheduled = True
            asyncio.get_running_loop().call_soon(self._flush)

    def _flush(self) -> None:
        self.flush_scheduled = False
        if self.out and not self.closed and self.transport is not None:
            self.transport.write(b"".join(self.out))
        self.out = []


class PipelinedHttp:
    def __init__(self, base_url: str, *, connections: int = 4, max_depth: int = 128,
                 ssl_ctx: Optional[_ssl.SSLContext] = None, default_headers: Optional[Dict[str, str]] = None,
                 timeout: float = 30.0):
        u = urlsplit(base_url)
        self.host = u.hostname or "127.0.0.1"
        self.port = u.port or (443 if u.scheme == "https" else 80)
        self.https = u.scheme == "https"
        self.ssl_ctx = ssl_ctx if self.https else None
        self.hostport = f"{self.host}:{self.port}" if u.port else self.host
        self.n = max(1, connections)
        self.max_depth = max_depth
        self.default_headers = dict(default_headers or {})
        self.timeout = timeout
        self._conns: List[_Conn] = []
        self._connecting: Optional[asyncio.Future] = None
        self.requests = 0
        self._head_cache: Dict[Tuple, bytes] = {}
        self._sweeper: Optional[asyncio.TimerHandle] = None

    def _drop(self, c: _Conn) -> None:
        if c in self._conns:
            self._conns.remove(c)

    async def _open(self) -> _Conn:
        loop = asyncio.get_running_loop()
        kw = {"ssl": self.ssl_ctx, "server_hostname": self.host} if self.https else {}
        _, proto = await loop.create_connection(lambda: _Conn(self), self.host, self.port, **kw)
        sock = proto.transport.get_extra_info("socket")
        if sock is not None:
            import socket

            try:
                sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            except OSError:
                pass
        self._conns.append(proto)
        return proto

    async def _fill(self) -> None:
        missing = self.n - len([c for c in self._conns if not c.closed])
        if missing > 0:
            await asyncio.gather(*(self._open() for _ in range(missing)))

    async def _pick(self) -> _Conn:
        live = [c for c in self._conns if not c.closed]
        if len(live) < self.n:
            # (re)open the pool once; concurrent callers wait on the same attempt
            if self._connecting is None or self._connecting.done():
                self._connecting = asyncio.ensure_future(self._fill())
            if not live:
                await asyncio.shield(self._connecting)
                live = [c for c in self._conns if not c.closed]
                if not live:
                    raise HttpError(f"cannot connect to {self.hostport}")
        best = min(live, key=lambda c: len(c.waiting))
        if len(best.waiting) >= self.max_depth:
            # all connections saturated: wait for the shortest queue to drain a bit
            while len(best.waiting) >= self.max_depth and not best.closed:
                await asyncio.sleep(0.001)
        return best

    def request_nowait(self, method: str, path: str, body: Optional[bytes] = None,
                       headers: Optional[Dict[str, str]] = None,
                       timeout: Optional[float] = None) -> Optional[asyncio.Future]:
        """Send on an open connection with room in its pipeline and return the response
        future (``(status, body)``; fails with :class:`HttpError` on timeout / connection
        loss) — no coroutine, no Task.  ``None`` when no connection can take it right now
        (the caller falls back to :meth:`request`)."""
        best = None
        for c in self._conns:
            if not c.closed and len(c.waiting) < self.max_depth and (best is None or len(c.waiting) < len(best.waiting)):
                best = c
        if best is None or len(self._conns) < self.n:
            return None
        loop = asyncio.get_running_loop()
        fut = loop.create_future()
        # no timer per request: the deadline rides with the request and one sweep per pool
        # fails an expired head of line (a TimerHandle + done-callback per DELETE was ~1 %
        # of a shard worker's CPU)
        limit = self.timeout if timeout is None else timeout
        best.send(self._encode(method, path, body, headers), fut, (loop.time() + limit, method, path))
        self.requests += 1
        if self._sweeper is None:
            self._arm_sweep(loop, limit)
        return fut

    def _arm_sweep(self, loop, limit: Optional[float] = None) -> None:
        t = min(self.timeout, limit) if limit is not None else self.timeout
        self._sweeper = loop.call_later(min(1.0, max(t / 4, 0.005)), self._sweep)

    def _sweep(self) -> None:
        """Fail the connections whose oldest pipelined request is past its deadline (the
        response order on them is unknown from then on), re-arm while any is pending."""
        self._sweeper = None
        loop = asyncio.get_running_loop()
        now = loop.time()
        pending = False
        for c in list(self._conns):
            dl = c.deadlines
            if dl and dl[0] is not None and dl[0][0] <= now:  # None: a request() with its own timer
                _, method, path = dl[0]
                _expire_and_reset(c.waiting[0], c, f"{method} {path}")
            if c.waiting:
                pending = True
        if pending:
            self._arm_sweep(loop)

    def _encode(self, method: str, path: str, body: Optional[bytes], headers: Optional[Dict[str, str]]) -> bytes:
        """Request bytes; the header block (Host, default and per-call headers) is encoded
        once per distinct header set."""
        key = tuple(headers.items()) if headers else ()
        head = self._head_cache.get(key)
        if head is None:
            h = dict(self.default_headers)
            if headers:
                h.update(headers)
            lines = [f"Host: {self.hostport}"] + [f"{k}: {v}" for k, v in h.items()]
            head = ("\r\n".join(lines) + "\r\nContent-Length: ").encode("latin-1")
            if len(self._head_cache) > 64:
                self._head_cache.clear()
            self._head_cache[key] = head
        return b"%s %s HTTP/1.1\r\n%s%d\r\n\r\n%s" % (method.encode(), path.encode("latin-1"), head,
                                                              len(body) if body else 0, body or b"")

    async def request(self, method: str, path: str, body: Optional[bytes] = None,
                      headers: Optional[Dict[str, str]] = None, timeout: Optional[float] = None) -> Tuple[int, bytes]:
        conn = await self._pick()
        loop = asyncio.get_running_loop()
        fut = loop.create_future()
        conn.send(self._encode(method, path, body, headers), fut)
        self.requests += 1
        # deadline as a timer on the future (asyncio.wait_for would cost a Task per request)
        timer = loop.call_later(self.timeout if timeout is None else timeout, _expire, fut)
        try:
            return await fut
        except _Expired:
            # the response order on this connection is now unknown: reset it
            conn._fail(HttpError("request timed out"))
            raise HttpError(f"{method} {path} timed out") from None
        finally:
            timer.cancel()

    async def close(self) -> None:
        if self._sweeper is not None:
            self._sweeper.cancel()
            self._sweeper = None
        for c in list(self._conns):
            if c.transport is not None:
                c.transport.close()
        self._conns.clear()
        await asyncio.sleep(0)
