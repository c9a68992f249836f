"""``kube/fasthttp.py``: pipelined requests answer in order, chunked and content-length
bodies parse, a stalled connection's requests expire by the pool's deadline sweep (no
timer per request) and the connection is reset, and the header block is encoded once."""
import asyncio

import pytest

from nexus_supervisor_amd.kube.fasthttp import HttpError, PipelinedHttp


async def _server(handler):
    srv = await asyncio.start_server(handler, "127.0.0.1", 0)
    return srv, f"http://127.0.0.1:{srv.sockets[0].getsockname()[1]}"


async def _read_request(r):
    head = await r.readuntil(b"\r\n\r\n")
    lines = head.decode().split("\r\n")
    n = 0
    for ln in lines[1:]:
        if ln.lower().startswith("content-length:"):
            n = int(ln.split(":", 1)[1])
    body = await r.readexactly(n) if n else b""
    return lines, body


def test_pipelined_order_and_bodies(arun):
    seen = []

    async def handler(r, w):
        i = 0
        try:
            while True:
                lines, body = await _read_request(r)
                seen.append((lines[0], body, [x for x in lines if x.startswith("X-")]))
                if i % 2:
                    payload = lines[0].encode()
                    w.write(b"HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\n"
                            + b"%x\r\n%s\r\n0\r\n\r\n" % (len(payload), payload))
                else:
                    w.write(b"HTTP/1.1 404 Not Found\r\nContent-Length: %d\r\n\r\n%s" % (len(lines[0]), lines[0].encode()))
                i += 1
                await w.drain()
        except (asyncio.IncompleteReadError, ConnectionError):
            pass

    async def main():
        srv, url = await _server(handler)
        c = PipelinedHttp(url, connections=1, default_headers={"X-Default": "1"})
        await c.request("GET", "/warm")  # opens the pool
        futs = [c.request_nowait("DELETE", f"/jobs/j{i}", b'{"a":1}', {"X-Call": "z"}) for i in range(20)]
        assert all(f is not None for f in futs)
        out = await asyncio.gather(*futs)
        assert [b.decode() for _, b in out] == [f"DELETE /jobs/j{i} HTTP/1.1" for i in range(20)]
        assert {s for s, _ in out} == {200, 404}
        assert all(body == b'{"a":1}' and hdrs == ["X-Default: 1", "X-Call: z"] for _l, body, hdrs in seen[1:])
        assert len(c._head_cache) == 2  # one block per distinct header set (request + request_nowait)
        await c.close()
        srv.close()
        await srv.wait_closed()

    arun(main(), timeout=20)


def test_request_nowait_expires_by_sweep_and_resets_connection(arun):
    async def handler(r, w):
        try:
            lines, _ = await _read_request(r)
            if lines[0].startswith("GET /warm"):
                w.write(b"HTTP/1.1 200 OK\r\nContent-Length: 0\r\n\r\n")
                await w.drain()
            await asyncio.sleep(30)  # never answers the DELETEs
        except (asyncio.IncompleteReadError, ConnectionError, asyncio.CancelledError):
            pass

    async def main():
        srv, url = await _server(handler)
        c = PipelinedHttp(url, connections=1, timeout=0.2)
        await c.request("GET", "/warm")
        f1 = c.request_nowait("DELETE", "/jobs/a")
        f2 = c.request_nowait("DELETE", "/jobs/b")
        t0 = asyncio.get_running_loop().time()
        with pytest.raises(HttpError, match="DELETE /jobs/a timed out"):
            await f1
        with pytest.raises(HttpError):
            await f2  # same connection: its response order is unknown after a timeout
        assert asyncio.get_running_loop().time() - t0 < 3.0  # 0.2 s deadline + sweep period, with CI load slack
        await asyncio.sleep(0.4)
        assert c._sweeper is None  # nothing pending: the sweep is not re-armed
        await c.close()
        srv.close()
        await srv.wait_closed()

    arun(main(), timeout=20)


def test_connection_close_and_mixed_case_headers(arun):
    async def handler(r, w):
        try:
            lines, _ = await _read_request(r)
            w.write(b"HTTP/1.1 201 Created\r\nCONTENT-LENGTH: 2\r\nConnection: Close\r\nX-A: b\r\n\r\nok")
            await w.drain()
            await asyncio.sleep(0.5)
        except (asyncio.IncompleteReadError, ConnectionError):
            pass

    async def main():
        srv, url = await _server(handler)
        c = PipelinedHttp(url, connections=1)
        status, body = await c.request("GET", "/x")
        assert (status, body) == (201, b"ok")
        await asyncio.sleep(0.05)
        assert all(conn.closed or conn.transport.is_closing() for conn in c._conns) or not c._conns
        await c.close()
        srv.close()
        await srv.wait_closed()

    arun(main(), timeout=20)
