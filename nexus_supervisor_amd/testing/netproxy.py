"""A TCP proxy that can partition its clients from the upstream (chaos tests).

``pause()`` stops moving bytes in both directions — requests already written and new
connections alike hang, exactly like an apiserver stalled behind a broken network path
(the client's own timeouts are what end them); ``resume()`` lets the held bytes through.
One proxy per replica gives a partition of *that* replica only, which a fake apiserver's
global latency cannot express.
"""
from __future__ import annotations

import asyncio
from typing import Optional, Set


class PausableProxy:
    def __init__(self, upstream_host: str, upstream_port: int):
        self.upstream = (upstream_host, upstream_port)
        self._open = asyncio.Event()
        self._open.set()
        self._server: Optional[asyncio.AbstractServer] = None
        self._tasks: Set[asyncio.Task] = set()
        self.port = 0
        self.connections = 0

    async def start(self, host: str = "127.0.0.1") -> str:
        self._server = await asyncio.start_server(self._client, host, 0)
        self.port = self._server.sockets[0].getsockname()[1]
        return f"http://{host}:{self.port}"

    def pause(self) -> None:
        self._open.clear()

    def resume(self) -> None:
        self._open.set()

    @property
    def paused(self) -> bool:
        return not self._open.is_set()

    async def _pipe(self, r: asyncio.StreamReader, w: asyncio.StreamWriter) -> None:
        try:
            while True:
                data = await r.read(65536)
                if not data:
                    break
                await self._open.wait()
                w.write(data)
                await w.drain()
        except (ConnectionError, asyncio.CancelledError):
            pass
        finally:
            try:
                w.close()
            except Exception:  # noqa: BLE001
                pass

    async def _client(self, cr: asyncio.StreamReader, cw: asyncio.StreamWriter) -> None:
        self.connections += 1
        await self._open.wait()
        try:
            ur, uw = await asyncio.open_connection(*self.upstream)
        except OSError:
            cw.close()
            return
        for t in (asyncio.ensure_future(self._pipe(cr, uw)), asyncio.ensure_future(self._pipe(ur, cw))):
            self._tasks.add(t)
            t.add_done_callback(self._tasks.discard)

    async def stop(self) -> None:
        self.resume()
        if self._server is not None:
            self._server.close()
            await self._server.wait_closed()
        for t in list(self._tasks):
            t.cancel()
        await asyncio.gather(*self._tasks, return_exceptions=True)
