"""Asyncio CQL v4 client and the Scylla / Astra checkpoint store.

Replaces nexus-core's gocqlx-based ``request.CqlStore`` (constructed at
``/root/reference/app/app_dependencies.go:18-34``; used for ``ReadCheckpoint`` /
``UpsertCheckpoint`` at ``/root/reference/services/supervisor.go:264,301,328,353,364``).

Design:

* **native codec** — frames are built and responses split + decoded by the C++
  extension ``_cql_native`` (``csrc/cql``); Python only matches stream ids.
* **multiplexed connections** — up to 32k in-flight requests per connection on
  stream ids; writes issued in the same loop tick are coalesced into one
  ``send`` (the supervisor's workers issue hundreds of requests concurrently).
* **prepared statements** — prepared once per query, re-prepared transparently
  on ``UNPREPARED`` (server restart), result metadata cached so responses are
  requested with ``skip_metadata``.
* **token-aware, DC-aware routing** — the ring comes from ``system.local`` /
  ``system.peers``; the partition key ``((algorithm, id))`` is hashed with
  Cassandra's Murmur3 (native) and the request goes straight to the owner in
  ``local-dc`` (one network hop, no coordinator forwarding).
* **Scylla shard-aware routing** — what the reference gets from the scylladb/gocql
  fork it pins (``/root/reference/go.mod:93``): ``OPTIONS`` before ``STARTUP`` reads
  ``SCYLLA_SHARD`` / ``SCYLLA_NR_SHARDS`` / ``SCYLLA_SHARDING_IGNORE_MSB`` /
  ``SCYLLA_SHARD_AWARE_PORT``; one connection per shard is opened on the shard-aware
  port from a local port ``≡ shard (mod nr_shards)`` (or, without that port, by
  reconnecting until every shard is covered), and each request goes to the
  connection of the shard owning its token (``biased-token-round-robin``), so the
  node never forwards it across cores.
* **retries** — idempotent requests are retried on another host after
  connection loss, ``Overloaded``, ``Unavailable`` or timeouts; hosts that fail
  are reconnected in the background with exponential backoff.
* **Astra** — the Secure Connect Bundle (base64 zip: ``config.json``,
  ``ca.crt``, ``cert``, ``key``) gives a mutual-TLS context and the SNI proxy;
  node connections go through the proxy with the host id as SNI.
"""
from __future__ import annotations

import asyncio
import base64
import bisect
import datetime as _dt
import io
import json
import logging
import operator
import random
import re
import ssl
import time
import zipfile
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, Iterable, List, Optional, Sequence, Tuple

from ..models.checkpoint import COLUMN_NAMES, COLUMNS, KEYSPACE, TABLE, CheckpointedRequest, StageRow
from .base import CheckpointStore, NotSent, StoreError

log = logging.getLogger("nexus_supervisor_amd.cql")

try:
    from .. import _cql_native as N  # type: ignore
except ImportError as _exc:  # pragma: no cover - build hint
    N = None
    _IMPORT_ERROR = _exc

EPOCH = _dt.datetime(1970, 1, 1, tzinfo=_dt.timezone.utc)


def _ms_to_dt(ms: int) -> _dt.datetime:
    return EPOCH + _dt.timedelta(milliseconds=ms)


def _build_execute_fast(stream, qid, vals, codes, types, cl, skip, serial):
    """EXECUTE frame through the scalar fast encoder (one per decision read and write)."""
    out = N.encode_execute_fast(stream, qid, vals, codes, cl, skip, serial)
    if out is NotImplemented:  # a value of an unexpected Python type
        out = N.encode_execute(stream, qid, vals, types, cl, skip, -1, None, serial, None)
    return out


def _build_execute(stream, qid, vals, codes, types, cl, skip, serial):
    return N.encode_execute(stream, qid, vals, types, cl, skip, -1, None, serial, None)


def _native():
    if N is None:
        raise StoreError("native CQL codec not built: run `python -m nexus_supervisor_amd._build`") from _IMPORT_ERROR
    return N


if N is not None:
    N.set_timestamp_factory(_ms_to_dt)

OP_ERROR, OP_READY, OP_AUTHENTICATE, OP_SUPPORTED, OP_RESULT, OP_AUTH_SUCCESS = 0x00, 0x02, 0x03, 0x06, 0x08, 0x10
OP_EVENT, OP_AUTH_CHALLENGE = 0x0C, 0x0E

CONSISTENCY = {"ANY": 0, "ONE": 1, "TWO": 2, "THREE": 3, "QUORUM": 4, "ALL": 5, "LOCAL_QUORUM": 6, "EACH_QUORUM": 7,
               "SERIAL": 8, "LOCAL_SERIAL": 9, "LOCAL_ONE": 10}
T_VARCHAR, T_TIMESTAMP, T_BOOLEAN = 0x0D, 0x0B, 0x04
_TYPE_IDS = {"text": T_VARCHAR, "timestamp": T_TIMESTAMP}

ERR_OVERLOADED, ERR_UNAVAILABLE, ERR_IS_BOOTSTRAPPING = 0x1001, 0x1000, 0x1002
ERR_WRITE_TIMEOUT, ERR_READ_TIMEOUT, ERR_UNPREPARED, ERR_SERVER = 0x1100, 0x1200, 0x2500, 0x0000
_AVAILABILITY = frozenset((ERR_OVERLOADED, ERR_UNAVAILABLE, ERR_IS_BOOTSTRAPPING))
RETRYABLE = {ERR_OVERLOADED, ERR_UNAVAILABLE, ERR_IS_BOOTSTRAPPING, ERR_WRITE_TIMEOUT, ERR_READ_TIMEOUT, ERR_SERVER}


class CqlError(StoreError):
    def __init__(self, code: int, message: str, extra: Optional[Dict[str, Any]] = None):
        super().__init__(f"CQL error 0x{code:04x}: {message}")
        self.code = code
        self.message = message
        self.extra = extra or {}
        # the coordinator (or the whole cluster) cannot serve: Unavailable / Overloaded /
        # IsBootstrapping.  A server-side Read/WriteTimeout is one partition's replicas
        # being slow (or LWT contention), Invalid / Syntax a bad request: not the store
        self.availability = code in _AVAILABILITY


class ConnectionClosed(StoreError):
    pass


class RequestTimeout(StoreError):
    pass


# ---------------------------------------------------------------------------- connection
class _Protocol(asyncio.Protocol):
    def __init__(self, conn: "CqlConnection"):
        self.conn = conn

    def connection_made(self, transport):
        self.conn._transport = transport

    def data_received(self, data: bytes):
        self.conn._on_data(data)

    def connection_lost(self, exc):
        self.conn._on_lost(exc)


_MASK64 = (1 << 64) - 1


def scylla_shard_of(token: int, nr_shards: int, ignore_msb: int) -> int:
    """Scylla's ``biased-token-round-robin`` sharding: shard of a Murmur3 token."""
    z = ((token + (1 << 63)) << ignore_msb) & _MASK64
    return (z * nr_shards) >> 64


class CqlConnection:
    """One multiplexed CQL connection."""

    MAX_STREAMS = 32768

    def __init__(self, host: str, port: int, *, user: str = "", password: str = "", ssl_ctx: Optional[ssl.SSLContext] = None,
                 server_hostname: Optional[str] = None, request_timeout: float = 5.0, connect_timeout: float = 5.0,
                 local_port: int = 0):
        self.host, self.port = host, port
        self.local_port = local_port  # shard-aware port: the source port selects the shard
        self.supported: Dict[str, List[str]] = {}
        self.user, self.password = user, password
        self.ssl_ctx, self.server_hostname = ssl_ctx, server_hostname
        self.request_timeout, self.connect_timeout = request_timeout, connect_timeout
        self._transport: Optional[asyncio.Transport] = None
        self._reader = _native().FrameReader()
        self._pending: Dict[int, asyncio.Future] = {}
        self._free: List[int] = list(range(self.MAX_STREAMS - 1, 0, -1))  # stream 0 unused, -1.. events
        # request deadlines, checked by one sweeper per connection instead of a timer per
        # request; a timed-out stream id stays reserved ("orphaned") until its late
        # response arrives, so it can never resolve a newer request
        self._deadline: Dict[int, float] = {}
        self._orphans: set = set()
        self._sweeper: Optional[asyncio.Task] = None
        self._out: List[bytes] = []
        self._flush_scheduled = False
        self._loop: Optional[asyncio.AbstractEventLoop] = None
        self.closed = True
        self.keyspace: Optional[str] = None
        self.prepared_here: set = set()
        self.requests = 0

    @property
    def address(self) -> Tuple[str, int]:
        return (self.host, self.port)

    async def connect(self, keyspace: Optional[str] = None) -> None:
        self._loop = asyncio.get_running_loop()
        kw: Dict[str, Any] = {}
        if self.ssl_ctx is not None:
            kw["ssl"] = self.ssl_ctx
            kw["server_hostname"] = self.server_hostname or self.host
        if self.local_port:
            kw["local_addr"] = ("0.0.0.0", self.local_port)
        await asyncio.wait_for(self._loop.create_connection(lambda: _Protocol(self), self.host, self.port, **kw),
                               self.connect_timeout)
        self.closed = False
        self._sweeper = self._loop.create_task(self._sweep_deadlines())
        sock = self._transport.get_extra_info("socket")
        if sock is not None:
            import socket as _s

            try:
                sock.setsockopt(_s.IPPROTO_TCP, _s.TCP_NODELAY, 1)
            except OSError:
                pass
        opts = await self.request(lambda s: N.encode_options(s))
        if opts[0] == "supported":
            self.supported = dict(opts[1])
        resp = await self.request(lambda s: N.encode_startup(s, {"CQL_VERSION": "3.0.0"}))
        if resp[0] == "authenticate":
            token = b"\x00" + self.user.encode() + b"\x00" + self.password.encode()
            resp = await self.request(lambda s: N.encode_auth_response(s, token))
            if resp[0] == "error":
                raise CqlError(resp[1], resp[2], resp[3])
        elif resp[0] != "ready":
            raise StoreError(f"unexpected STARTUP response {resp!r}")
        if keyspace:
            await self.use(keyspace)

    async def use(self, keyspace: str) -> None:
        r = await self.request(lambda s: N.encode_query(s, f'USE "{keyspace}"', None, None, CONSISTENCY["ONE"]))
        if r[0] == "error":
            raise CqlError(r[1], r[2], r[3])
        self.keyspace = keyspace

    # -------------------------------------------------------------- I/O
    def _on_data(self, data: bytes) -> None:
        try:
            frames = self._reader.feed(data)
        except ValueError as exc:
            log.error("protocol error from %s:%s: %s", self.host, self.port, exc)
            self.close()
            return
        pending = self._pending
        deadline = self._deadline
        for stream, _op, dec in frames:
            fut = pending.pop(stream, None)
            if fut is None:
                if stream in self._orphans:  # late answer to a timed-out request
                    self._orphans.discard(stream)
                    self._free.append(stream)
                continue  # or a server push (EVENT)
            deadline.pop(stream, None)
            self._free.append(stream)
            if not fut.done():
                fut.set_result(dec)

    def _on_lost(self, exc) -> None:
        self.closed = True
        err = ConnectionClosed(f"connection to {self.host}:{self.port} lost: {exc}")
        pending, self._pending = self._pending, {}
        for fut in pending.values():
            if not fut.done():
                fut.set_exception(err)
        self._free = list(range(self.MAX_STREAMS - 1, 0, -1))
        self._deadline.clear()
        self._orphans.clear()
        if self._sweeper is not None:
            self._sweeper.cancel()

    def _flush(self) -> None:
        self._flush_scheduled = False
        if self._out and self._transport is not None and not self.closed:
            data = b"".join(self._out) if len(self._out) > 1 else self._out[0]
            self._out = []
            self._transport.write(data)
        else:
            self._out = []

    def request_nowait(self, build, hint=None, timeout: Optional[float] = None, args: Optional[tuple] = None) -> asyncio.Future:
        """Send one request frame built by ``build(stream, *args)``; returns the response future."""
        if self.closed:
            raise ConnectionClosed(f"connection to {self.host}:{self.port} is closed")
        if not self._free:
            raise StoreError("no free stream ids")
        stream = self._free.pop()
        fut = self._loop.create_future()
        self._pending[stream] = fut
        self._deadline[stream] = self._loop.time() + (timeout or self.request_timeout)
        if hint is not None:
            self._reader.expect(stream, hint)
        self._out.append(build(stream) if args is None else build(stream, *args))
        self.requests += 1
        if not self._flush_scheduled:
            self._flush_scheduled = True
            self._loop.call_soon(self._flush)
        return fut

    async def request(self, build, hint=None, timeout: Optional[float] = None):
        return await self.request_nowait(build, hint, timeout)

    async def _sweep_deadlines(self) -> None:
        while not self.closed:
            await asyncio.sleep(min(0.1, self.request_timeout / 4))
            now = self._loop.time()
            expired = [s for s, d in self._deadline.items() if d <= now]
            for stream in expired:
                del self._deadline[stream]
                fut = self._pending.pop(stream, None)
                self._reader.forget(stream)
                self._orphans.add(stream)
                if fut is not None and not fut.done():
                    fut.set_exception(RequestTimeout(f"request to {self.host}:{self.port} timed out"))
            if len(self._orphans) > 1024:  # the server stopped answering: start over
                self.close()

    @property
    def in_flight(self) -> int:
        return len(self._pending)

    def scylla(self, key: str) -> Optional[str]:
        v = self.supported.get(key)
        return v[0] if v else None

    def close(self) -> None:
        if self._transport is not None:
            self._transport.close()
        self.closed = True
        if self._sweeper is not None:
            self._sweeper.cancel()


# ---------------------------------------------------------------------------- session
@dataclass
class PreparedStatement:
    query: str
    query_id: bytes
    bind_types: List[Any]
    pk_indexes: List[int]
    result_names: Optional[Tuple[str, ...]]
    result_types: Optional[List[Any]]
    keyspace: str = ""
    _pk_get: Optional[Callable[[Sequence[Any]], Tuple]] = field(default=None, repr=False, compare=False)
    # a conditional (LWT) statement: never executed with skip_metadata — its not-applied
    # answer carries the condition's columns, a different shape from the prepared one
    conditional: bool = False

    @property
    def codes(self) -> Optional[bytes]:
        """One type-id byte per bind marker when every bind type is a scalar the native fast
        encoder writes (``encode_execute_fast``), else None (computed once)."""
        c = self.__dict__.get("_codes", False)
        if c is False:
            ok = all(isinstance(t, int) and t in _FAST_CODES for t in self.bind_types)
            c = self.__dict__["_codes"] = bytes(self.bind_types) if ok else None
        return c


# ascii bigint blob boolean counter double int timestamp varchar time
_FAST_CODES = frozenset((0x01, 0x02, 0x03, 0x04, 0x05, 0x07, 0x09, 0x0B, 0x0D, 0x12))

_CONDITIONAL = re.compile(r"^\s*(?:UPDATE|INSERT|DELETE)\b.*\bIF\b", re.I | re.S)


def is_conditional(query: str) -> bool:
    """An LWT write (``UPDATE … IF …``, ``INSERT … IF NOT EXISTS``, ``DELETE … IF EXISTS``)."""
    return bool(_CONDITIONAL.match(query))


def _pk_getter(indexes: Sequence[int]) -> Callable[[Sequence[Any]], Tuple]:
    """values → partition-key tuple (a C-level itemgetter; always a tuple)."""
    if len(indexes) == 1:
        i = indexes[0]
        return lambda values: (values[i],)
    return operator.itemgetter(*indexes)


_HOST_EPOCH = [0]  # bumped on every host up/down flip: invalidates routing caches
_NO_HOSTS: frozenset = frozenset()


@dataclass
class Host:
    address: Tuple[str, int]
    dc: str = ""
    rack: str = ""
    host_id: str = ""
    tokens: List[int] = field(default_factory=list)
    conns: List[CqlConnection] = field(default_factory=list)
    _up: bool = False
    failures: int = 0
    next_retry: float = 0.0
    rr: int = 0
    # Scylla sharding of this node (0 = not sharded / unknown) and its connections by shard
    nr_shards: int = 0
    ignore_msb: int = 0
    shard_conns: List[List[CqlConnection]] = field(default_factory=list)

    def shard_of(self, token: Optional[int]) -> Optional[int]:
        if token is None or self.nr_shards <= 1:
            return None
        return scylla_shard_of(token, self.nr_shards, self.ignore_msb)

    @property
    def up(self) -> bool:
        return self._up

    @up.setter
    def up(self, v: bool) -> None:
        if v != self._up:
            self._up = v
            _HOST_EPOCH[0] += 1

    def pick(self, shard: Optional[int] = None) -> Optional[CqlConnection]:
        """Least in-flight live connection (of ``shard`` when the node is sharded and has
        one), scanning from a rotating start (ties spread)."""
        conns = self.conns
        if shard is not None and shard < len(self.shard_conns):
            own = self.shard_conns[shard]
            if len(own) == 1:  # the usual case: one connection per shard
                if not own[0].closed:
                    return own[0]
            else:
                own = [c for c in own if not c.closed]
                if own:
                    conns = own
        n = len(conns)
        if n == 1:
            c = conns[0]
            return None if c.closed else c
        self.rr += 1
        best = None
        for k in range(n):
            c = conns[(self.rr + k) % n]
            if not c.closed and (best is None or c.in_flight < best.in_flight):
                best = c
        return best


@dataclass
class Rows:
    names: Tuple[str, ...]
    rows: List[tuple]
    paging_state: Optional[bytes] = None

    def dicts(self) -> List[Dict[str, Any]]:
        return [dict(zip(self.names, r)) for r in self.rows]

    def __iter__(self):
        return iter(self.rows)

    def __len__(self):
        return len(self.rows)


class CqlSession:
    def __init__(self, contact_points: Sequence[Tuple[str, int]], *, keyspace: Optional[str] = None, user: str = "",
                 password: str = "", local_dc: str = "", connections_per_host: int = 2, request_timeout: float = 5.0,
                 connect_timeout: float = 5.0, token_aware: bool = True, consistency: str = "LOCAL_QUORUM",
                 ssl_ctx: Optional[ssl.SSLContext] = None, sni_proxy: Optional[Tuple[str, int]] = None,
                 max_retries: int = 3, discover: bool = True, shard_aware: bool = True, connections_per_shard: int = 1):
        if not contact_points:
            raise StoreError("no CQL contact points configured")
        self.contact_points = list(contact_points)
        self.keyspace = keyspace
        self.user, self.password = user, password
        self.local_dc = local_dc
        self.per_host = max(1, connections_per_host)
        self.request_timeout, self.connect_timeout = request_timeout, connect_timeout
        self.token_aware = token_aware
        self.consistency = CONSISTENCY[consistency.upper()]
        self.ssl_ctx = ssl_ctx
        self.sni_proxy = sni_proxy
        self.max_retries = max_retries
        self.discover = discover
        self.shard_aware = shard_aware and sni_proxy is None
        self.shard_aware_port = True  # use SCYLLA_SHARD_AWARE_PORT when advertised (falls back per host)
        self._sharded = False  # some node advertised Scylla shards
        self._tokens: Dict[tuple, int] = {}  # partition key values → token (recent)
        # partition key values → (routing epoch, token, owner host, shard): a decision reads
        # then writes one partition; the second statement skips ring lookup and shard math
        self._routes: Dict[tuple, Tuple[Any, int, Host, Optional[int], bool]] = {}
        self.per_shard = max(1, connections_per_shard)
        self.hosts: Dict[Tuple[str, int], Host] = {}
        self._ring: List[int] = []
        self._ring_hosts: List[Host] = []
        self._prepared: Dict[str, PreparedStatement] = {}
        self._preparing: Dict[str, asyncio.Future] = {}
        self._reconnector: Optional[asyncio.Task] = None
        self._rr = 0
        self._plan_key: Optional[Tuple[int, int]] = None
        self._plan_up: List[Host] = []
        self._plan_owner: Dict[int, List[Host]] = {}
        self.stats = {"requests": 0, "retries": 0, "reprepares": 0, "token_routed": 0, "shard_routed": 0}

    # -------------------------------------------------------------- lifecycle
    def _new_conn(self, h: Host, port: Optional[int] = None, local_port: int = 0) -> CqlConnection:
        host, hport = h.address
        server_hostname = None
        if self.sni_proxy is not None:
            server_hostname = h.host_id or host
            host, hport = self.sni_proxy
        return CqlConnection(host, port or hport, user=self.user, password=self.password, ssl_ctx=self.ssl_ctx,
                             server_hostname=server_hostname, request_timeout=self.request_timeout,
                             connect_timeout=self.connect_timeout, local_port=local_port)

    async def _open_host(self, h: Host) -> None:
        first = self._new_conn(h)
        opened: List[CqlConnection] = [first]
        try:
            await first.connect(self.keyspace)
            nr = int(first.scylla("SCYLLA_NR_SHARDS") or 0) if self.shard_aware else 0
            if nr > 1 and first.scylla("SCYLLA_SHARDING_ALGORITHM") in (None, "biased-token-round-robin"):
                conns, by_shard = await self._open_shards(h, first, nr, opened)
                h.nr_shards, h.ignore_msb = nr, int(first.scylla("SCYLLA_SHARDING_IGNORE_MSB") or 0)
                self._sharded = True
            else:
                rest = [self._new_conn(h) for _ in range(self.per_host - 1)]
                opened.extend(rest)
                await asyncio.gather(*(c.connect(self.keyspace) for c in rest))
                conns, by_shard = [first] + rest, []
                h.nr_shards = 0
        except BaseException:
            # a failed open never leaks what it already opened (each reconnect would pile up)
            for c in opened:
                c.close()
            raise
        for c in h.conns:
            c.close()
        h.conns = conns
        h.shard_conns = by_shard
        h.up = True
        h.failures = 0

    async def _open_shards(self, h: Host, first: CqlConnection, nr: int, opened: List[CqlConnection]):
        """``per_shard`` connections to every shard of a Scylla node.  With a shard-aware
        port the local port picks the shard (``port % nr == shard``); without one — or when
        the advertised aware port is refused, filtered or times out (e.g. a Service that
        only exposes 9042), as the scylladb gocql fork does — keep reconnecting to the
        regular port until each shard has been handed out.  Connections that land on a
        shard that already has its ``per_shard`` are closed, not kept (NAT-rewritten source
        ports would otherwise pile up ~nr_shards×32 of them); every connection opened is
        recorded in ``opened`` so the caller can close them all if the open fails."""
        by_shard: List[List[CqlConnection]] = [[] for _ in range(nr)]
        by_shard[int(first.scylla("SCYLLA_SHARD") or 0) % nr].append(first)
        aware = [int(first.scylla("SCYLLA_SHARD_AWARE_PORT") or 0)] if self.shard_aware_port else [0]

        async def one(shard: int) -> None:
            for attempt in range(32):
                lp = 0
                port = aware[0]
                if port:
                    base = random.randrange(32768, 60000)
                    lp = base - base % nr + shard
                c = self._new_conn(h, port=port or None, local_port=lp)
                opened.append(c)
                try:
                    await c.connect(self.keyspace)
                except (OSError, asyncio.TimeoutError) as exc:
                    c.close()
                    if port and getattr(exc, "errno", None) in (98, 99):  # EADDRINUSE / EADDRNOTAVAIL
                        continue
                    if port:
                        log.warning("CQL host %s:%s: shard-aware port %d unusable (%r); falling back to the "
                                    "regular port", h.address[0], h.address[1], port, exc)
                        aware[0] = 0
                        self.stats["shard_port_fallbacks"] = self.stats.get("shard_port_fallbacks", 0) + 1
                        continue
                    raise
                got = int(c.scylla("SCYLLA_SHARD") or 0) % nr
                if len(by_shard[got]) >= self.per_shard:
                    c.close()  # a stray connection to a shard that is already served
                else:
                    by_shard[got].append(c)
                if len(by_shard[shard]) >= self.per_shard:
                    return
            log.warning("CQL host %s:%s: no connection to shard %d", h.address[0], h.address[1], shard)

        for shard in range(nr):
            while len(by_shard[shard]) < self.per_shard:
                before = len(by_shard[shard])
                await one(shard)
                if len(by_shard[shard]) == before:
                    break
        conns = [c for lst in by_shard for c in lst]
        return conns, by_shard

    async def connect(self) -> None:
        last: Optional[BaseException] = None
        for addr in self.contact_points:
            h = Host(address=addr, host_id=addr[0] if self.sni_proxy is None else "")
            if self.sni_proxy is not None:
                h.host_id = addr[0]
            try:
                await self._open_host(h)
            except (OSError, asyncio.TimeoutError, StoreError) as exc:
                if isinstance(exc, CqlError) and exc.code in (0x0100, 0x2100):
                    raise  # bad credentials / unauthorized: no point trying other hosts
                last = exc
                log.warning("CQL contact point %s:%s unavailable: %s", addr[0], addr[1], exc)
                continue
            self.hosts[addr] = h
            break
        if not self.hosts:
            raise StoreError(f"could not connect to any CQL contact point: {last}")
        if self.discover:
            try:
                await self._discover()
            except StoreError as exc:  # e.g. a server without system tables
                log.warning("CQL topology discovery failed: %s (routing round-robin)", exc)
        others = [h for h in self.hosts.values() if not h.up]
        if others:
            await asyncio.gather(*(self._try_open(h) for h in others))
        self._reconnector = asyncio.create_task(self._reconnect_loop(), name="cql-reconnect")

    async def _try_open(self, h: Host) -> None:
        try:
            await self._open_host(h)
        except (OSError, asyncio.TimeoutError, StoreError) as exc:
            self._mark_down(h, exc)

    async def _discover(self) -> None:
        first = next(iter(self.hosts.values()))
        local = await self._query_on(first, "SELECT data_center, rack, host_id, tokens, native_port FROM system.local")
        peers_rows: List[Dict[str, Any]] = []
        try:
            peers = await self._query_on(first, "SELECT peer, rpc_address, data_center, rack, host_id, tokens, native_port FROM system.peers")
            peers_rows = peers.dicts()
        except CqlError:  # real Scylla has no native_port column in peers; fall back
            peers = await self._query_on(first, "SELECT peer, rpc_address, data_center, rack, host_id, tokens FROM system.peers")
            peers_rows = peers.dicts()
        lrow = local.dicts()[0] if local.rows else {}
        first.dc = lrow.get("data_center") or ""
        first.rack = lrow.get("rack") or ""
        if self.sni_proxy is None:
            first.host_id = str(lrow.get("host_id") or "")
        first.tokens = [int(t) for t in (lrow.get("tokens") or [])]
        for p in peers_rows:
            addr = p.get("rpc_address") or p.get("peer")
            if not addr or addr == "0.0.0.0":
                addr = p.get("peer")
            port = int(p.get("native_port") or first.address[1])
            key = (addr, port)
            h = self.hosts.get(key) or Host(address=key)
            h.dc, h.rack = p.get("data_center") or "", p.get("rack") or ""
            h.host_id = str(p.get("host_id") or "")
            h.tokens = [int(t) for t in (p.get("tokens") or [])]
            self.hosts[key] = h
        self._build_ring()

    def _build_ring(self) -> None:
        pairs = []
        for h in self.hosts.values():
            if self.local_dc and h.dc and h.dc != self.local_dc:
                continue
            for t in h.tokens:
                pairs.append((t, h))
        pairs.sort(key=lambda p: p[0])
        self._ring = [p[0] for p in pairs]
        self._ring_hosts = [p[1] for p in pairs]

    def owner(self, token: int) -> Optional[Host]:
        """Replica owning ``token``: the first ring token >= it (wrapping)."""
        if not self._ring:
            return None
        i = bisect.bisect_left(self._ring, token)
        return self._ring_hosts[i % len(self._ring)]

    def _mark_down(self, h: Host, exc: BaseException) -> None:
        if h.up:
            log.warning("CQL host %s:%s down: %s", h.address[0], h.address[1], exc)
        h.up = False
        h.failures += 1
        h.next_retry = time.monotonic() + min(30.0, 0.1 * (2 ** min(h.failures, 9))) * (0.8 + 0.4 * random.random())

    async def _reconnect_loop(self) -> None:
        while True:
            await asyncio.sleep(0.05)
            now = time.monotonic()
            for h in list(self.hosts.values()):
                if h.up and all(c.closed for c in h.conns):
                    self._mark_down(h, ConnectionClosed("all connections closed"))
                if not h.up and now >= h.next_retry:
                    await self._try_open(h)
                    if h.up:
                        log.info("CQL host %s:%s back up", *h.address)

    async def close(self) -> None:
        if self._reconnector is not None:
            self._reconnector.cancel()
            try:
                await self._reconnector
            except (asyncio.CancelledError, Exception):
                pass
        for h in self.hosts.values():
            for c in h.conns:
                c.close()
        await asyncio.sleep(0)

    # -------------------------------------------------------------- routing
    def _candidates(self, routing_token: Optional[int]) -> List[Host]:
        """Query plan: the token owner first (token-aware), then the other live local-DC
        hosts round-robin.  Plans are cached until a host flips up/down or joins."""
        key = (_HOST_EPOCH[0], len(self.hosts))
        if self._plan_key != key:
            up = [h for h in self.hosts.values() if h.up and (not self.local_dc or not h.dc or h.dc == self.local_dc)]
            if not up:
                up = [h for h in self.hosts.values() if h.up]
            self._plan_up = up
            self._plan_owner = {}
            self._plan_key = key
        up = self._plan_up
        if routing_token is not None and self.token_aware and self._ring:
            o = self.owner(routing_token)
            if o is not None and o.up:
                self.stats["token_routed"] += 1
                plan = self._plan_owner.get(id(o))
                if plan is None:
                    plan = self._plan_owner[id(o)] = [o] + [h for h in up if h is not o]
                return plan
        if len(up) > 1:
            self._rr = (self._rr + 1) % len(up)
            return up[self._rr:] + up[: self._rr]
        return up

    async def _query_on(self, h: Host, cql: str, values=None) -> Rows:
        conn = h.pick()
        if conn is None:
            raise ConnectionClosed("host has no live connection")
        r = await conn.request(lambda s: N.encode_query(s, cql, values, None, CONSISTENCY["ONE"]))
        return self._result(r)

    @staticmethod
    def _result(r):
        kind = r[0]
        if kind == "rows":
            return Rows(tuple(r[1]), r[2], r[3])
        if kind == "error":
            raise CqlError(r[1], r[2], r[3])
        return r

    # -------------------------------------------------------------- statements
    async def prepare(self, query: str) -> PreparedStatement:
        ps = self._prepared.get(query)
        if ps is not None:
            return ps
        fut = self._preparing.get(query)
        if fut is not None:
            return await fut
        fut = asyncio.get_running_loop().create_future()
        self._preparing[query] = fut
        try:
            last: Optional[BaseException] = None
            for h in self._candidates(None):
                conn = h.pick()
                if conn is None:
                    continue
                try:
                    r = await conn.request(lambda s: N.encode_prepare(s, query))
                except (ConnectionClosed, RequestTimeout, OSError) as exc:
                    last = exc
                    continue
                if r[0] == "error":
                    raise CqlError(r[1], r[2], r[3])
                _, qid, bind, pk, result = r
                ps = PreparedStatement(query, qid, [b[3] for b in bind], list(pk),
                                       tuple(n for n, _ in result) if result is not None else None,
                                       [t for _, t in result] if result is not None else None,
                                       conditional=is_conditional(query))
                conn.prepared_here.add(qid)
                self._prepared[query] = ps
                fut.set_result(ps)
                return ps
            raise StoreError(f"prepare failed on every host: {last}")
        except BaseException as exc:
            if not fut.done():
                fut.set_exception(exc)
                fut.exception()  # consumed
            raise
        finally:
            self._preparing.pop(query, None)

    def routing_token(self, ps: PreparedStatement, values: Sequence[Any]) -> Optional[int]:
        if not ps.pk_indexes or not (self._ring or self._sharded):
            return None
        get = ps._pk_get
        if get is None:
            get = ps._pk_get = _pk_getter(ps.pk_indexes)
        key = get(values)
        tok = self._tokens.get(key)  # a decision reads then writes the same partition
        if tok is not None:
            return tok
        parts = []
        for i in ps.pk_indexes:
            v = values[i]
            if v is None:
                return None
            parts.append(N.serialize(v, ps.bind_types[i]))
        tok = N.token_for(parts)
        if len(self._tokens) > 8192:
            self._tokens.clear()
        self._tokens[key] = tok
        return tok

    def _route(self, ps: PreparedStatement, values: Sequence[Any]):
        """(token, owner host, owner shard) of a statement's partition when token-aware
        routing applies and the owner is up, cached per partition key until a host flips or
        joins; else ``(token, None, None)`` and :meth:`_candidates` plans as usual."""
        if not (self.token_aware or self.shard_aware):
            return None, None, None
        get = ps._pk_get
        if get is None:
            if not ps.pk_indexes:
                return None, None, None
            get = ps._pk_get = _pk_getter(ps.pk_indexes)
        key = get(values)
        epoch = (_HOST_EPOCH[0], len(self.hosts))
        hit = self._routes.get(key)
        if hit is not None and hit[0] == epoch:
            if hit[4]:
                self.stats["token_routed"] += 1
            return hit[1], hit[2], hit[3]
        tok = self.routing_token(ps, values)
        if tok is None:
            return None, None, None
        by_ring = bool(self.token_aware and self._ring)
        if by_ring:
            o = self.owner(tok)
        else:
            # no ring (one node, or token-awareness off): with a single live host every
            # plan starts there, so its shard can be cached the same way
            up = [h for h in self.hosts.values() if h.up]
            o = up[0] if len(up) == 1 else None
        if o is None or not o.up:
            return tok, None, None
        shard = o.shard_of(tok) if o.nr_shards else None
        if len(self._routes) > 8192:
            self._routes.clear()
        self._routes[key] = (epoch, tok, o, shard, by_ring)
        if by_ring:
            self.stats["token_routed"] += 1
        return tok, o, shard

    async def execute(self, ps_or_query, values: Sequence[Any] = (), *, consistency: Optional[int] = None,
                      serial: Optional[int] = None, idempotent: bool = True, timeout: Optional[float] = None):
        ps = ps_or_query if isinstance(ps_or_query, PreparedStatement) else await self.prepare(ps_or_query)
        cl = self.consistency if consistency is None else consistency
        token, owner, owner_shard = self._route(ps, values)
        vals = list(values)
        hint = ps.result_types
        skip = hint is not None and not ps.conditional
        attempts = 0
        sent = False  # a request went onto a connection (it may have landed)
        last: Optional[BaseException] = None
        tried: set = _NO_HOSTS  # replaced by a real set on the first failure
        while attempts <= self.max_retries:
            if owner is not None and not tried:
                h, shard = owner, owner_shard  # cached token-aware route (first attempt)
            else:
                cands = self._candidates(token)
                if tried:
                    cands = [h for h in cands if h.address not in tried] or cands
                if not cands:
                    raise NotSent(f"no CQL host available: {last}")
                h = cands[0]
                shard = h.shard_of(token) if h.nr_shards else None
            conn = h.pick(shard)
            if conn is None:
                self._mark_down(h, ConnectionClosed("no live connection"))
                tried = tried or set()
                tried.add(h.address)
                attempts += 1
                continue
            self.stats["requests"] += 1
            if shard is not None:
                self.stats["shard_routed"] += 1
            sent = True
            try:
                codes = ps.codes
                r = await conn.request_nowait(_build_execute_fast if codes is not None else _build_execute,
                                              hint if skip else None, timeout,
                                              (ps.query_id, vals, codes, ps.bind_types, cl, skip, serial))
            except (ConnectionClosed, OSError) as exc:
                last = exc
                self._mark_down(h, exc)
                tried = tried or set()
                tried.add(h.address)
                attempts += 1
                self.stats["retries"] += 1
                continue
            except RequestTimeout as exc:
                last = exc
                if not idempotent:
                    raise
                tried = tried or set()
                tried.add(h.address)
                attempts += 1
                self.stats["retries"] += 1
                continue
            kind = r[0]
            if kind == "error":
                code = r[1]
                if code == ERR_UNPREPARED:
                    self.stats["reprepares"] += 1
                    rr = await conn.request(lambda s: N.encode_prepare(s, ps.query))
                    if rr[0] == "error":
                        raise CqlError(rr[1], rr[2], rr[3])
                    if rr[1] != ps.query_id:
                        ps.query_id = rr[1]
                    attempts += 1
                    continue
                if code in RETRYABLE and idempotent and attempts < self.max_retries:
                    last = CqlError(code, r[2], r[3])
                    attempts += 1
                    self.stats["retries"] += 1
                    await asyncio.sleep(min(0.2, 0.01 * (2 ** attempts)))
                    continue
                raise CqlError(code, r[2], r[3])
            if kind == "rows":
                names = ps.result_names if skip else tuple(r[1])
                return Rows(names, r[2], r[3])
            return r
        raise (StoreError if sent else NotSent)(f"CQL request failed after {attempts} attempts: {last}")

    async def execute_batch(self, ps: PreparedStatement, rows: Sequence[Sequence[Any]], *,
                            consistency: Optional[int] = None, logged: bool = False,
                            timeout: Optional[float] = None) -> None:
        """One BATCH frame of ``ps`` over many value rows (bulk loads: one round trip and
        one frame instead of one per row).  UNLOGGED unless ``logged``; retried on
        another host after a connection failure, re-prepared once on UNPREPARED."""
        cl = self.consistency if consistency is None else consistency
        kind = 0 if logged else 1
        for attempt in range(self.max_retries + 1):
            cands = self._candidates(None)
            if not cands:
                raise StoreError("no CQL host available")
            h = cands[attempt % len(cands)]
            conn = h.pick()
            if conn is None:
                self._mark_down(h, ConnectionClosed("no live connection"))
                continue
            stmts = [(1, ps.query_id, list(r), ps.bind_types) for r in rows]
            self.stats["requests"] += 1
            try:
                r = await conn.request(lambda s: N.encode_batch(s, kind, stmts, cl, None, None), None, timeout)
            except (ConnectionClosed, OSError) as exc:
                self._mark_down(h, exc)
                self.stats["retries"] += 1
                continue
            if r[0] == "error":
                if r[1] == ERR_UNPREPARED:
                    rr = await conn.request(lambda s: N.encode_prepare(s, ps.query))
                    if rr[0] == "error":
                        raise CqlError(rr[1], rr[2], rr[3])
                    ps.query_id = rr[1]
                    continue
                if r[1] in RETRYABLE:
                    self.stats["retries"] += 1
                    await asyncio.sleep(min(0.2, 0.01 * (2 ** attempt)))
                    continue
                raise CqlError(r[1], r[2], r[3])
            return
        raise StoreError("CQL batch failed after retries")

    async def query(self, cql: str, values: Optional[Sequence[Any]] = None, consistency: Optional[int] = None):
        """Unprepared statement (schema, admin)."""
        cl = self.consistency if consistency is None else consistency
        last: Optional[BaseException] = None
        for h in self._candidates(None):
            conn = h.pick()
            if conn is None:
                continue
            try:
                r = await conn.request(lambda s: N.encode_query(s, cql, list(values) if values else None, None, cl))
            except (ConnectionClosed, RequestTimeout, OSError) as exc:
                last = exc
                self._mark_down(h, exc)
                continue
            return self._result(r)
        raise StoreError(f"no CQL host could run the query: {last}")


# ---------------------------------------------------------------------------- Astra secure connect bundle
@dataclass
class SecureBundle:
    host: str
    port: int
    cql_port: int
    keyspace: str
    local_dc: str
    ssl_ctx: ssl.SSLContext
    raw_config: Dict[str, Any]


def load_secure_bundle(b64: str) -> SecureBundle:
    """Parse an Astra Secure Connect Bundle (base64 zip) into a mutual-TLS context."""
    import os
    import tempfile

    data = base64.b64decode(b64)
    with zipfile.ZipFile(io.BytesIO(data)) as z:
        names = set(z.namelist())
        cfg = json.loads(z.read("config.json"))
        files = {n: z.read(n) for n in ("ca.crt", "cert", "key") if n in names}
    if "ca.crt" not in files:
        raise StoreError("secure connect bundle has no ca.crt")
    ctx = ssl.create_default_context(ssl.Purpose.SERVER_AUTH, cadata=files["ca.crt"].decode())
    ctx.check_hostname = False  # Astra SNI routes by host id; the proxy certificate names the proxy
    if "cert" in files and "key" in files:
        with tempfile.TemporaryDirectory() as d:
            cp, kp = os.path.join(d, "cert"), os.path.join(d, "key")
            with open(cp, "wb") as f:
                f.write(files["cert"])
            with open(kp, "wb") as f:
                f.write(files["key"])
            ctx.load_cert_chain(cp, kp)
    return SecureBundle(host=cfg.get("host", ""), port=int(cfg.get("port", 29080)), cql_port=int(cfg.get("cql_port", 29042)),
                        keyspace=cfg.get("keyspace", ""), local_dc=cfg.get("localDC", ""), ssl_ctx=ctx, raw_config=cfg)


async def astra_contact_info(bundle: SecureBundle, timeout: float = 10.0) -> Dict[str, Any]:
    """Metadata service (``https://host:port/metadata``): SNI proxy address, host ids, local DC."""
    import aiohttp

    url = f"https://{bundle.host}:{bundle.port}/metadata"
    async with aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=timeout)) as s:
        async with s.get(url, ssl=bundle.ssl_ctx) as r:
            r.raise_for_status()
            doc = await r.json(content_type=None)
    return doc.get("contact_info", doc)


# ---------------------------------------------------------------------------- checkpoint store
def _q(name: str) -> str:
    return name


class CqlCheckpointStore(CheckpointStore):
    """``nexus.checkpoints`` over CQL (schema: ``models.checkpoint``; reference schema
    ``/root/reference/test-resources/checkpoints.cql:1-29``)."""

    def __init__(self, session: CqlSession, keyspace: str = KEYSPACE, table: str = TABLE,
                 consistency: str = "LOCAL_QUORUM", serial_consistency: str = "LOCAL_SERIAL"):
        self.session = session
        self.keyspace, self.table = keyspace, table
        self.cl = CONSISTENCY[consistency.upper()]
        self.serial = CONSISTENCY[serial_consistency.upper()]
        ft = f"{keyspace}.{table}"
        cols = ", ".join(COLUMN_NAMES)
        self.q_read = f"SELECT {cols} FROM {ft} WHERE algorithm = ? AND id = ?"
        # projected read for the owned-columns path: one text column instead of 19
        # (no timestamp decoding, ~10x smaller response)
        self.q_read_status = f"SELECT lifecycle_stage FROM {ft} WHERE algorithm = ? AND id = ?"
        self.q_insert = f"INSERT INTO {ft} ({cols}) VALUES ({', '.join('?' for _ in COLUMN_NAMES)})"
        self.q_update_failure = (f"UPDATE {ft} SET lifecycle_stage = ?, algorithm_failure_cause = ?, "
                                 f"algorithm_failure_details = ?, last_modified = ? WHERE algorithm = ? AND id = ?")
        self.q_update_stage = f"UPDATE {ft} SET lifecycle_stage = ?, last_modified = ? WHERE algorithm = ? AND id = ?"
        self.reads = self.writes = 0
        self._cas_q: Dict[Tuple[str, int], str] = {}

    @classmethod
    def from_config(cls, cfg) -> "CqlCheckpointStore":
        """Build from ``SupervisorConfig`` (``cql-store-type`` scylla | astra)."""
        from ..config.schema import CQL_STORE_ASTRA

        if cfg.cql_store_type == CQL_STORE_ASTRA:
            a = cfg.astra_cql_store
            if not a.secure_connection_bundle_base64:
                raise StoreError("astra-cql-store.secure-connection-bundle-base64 is empty")
            bundle = load_secure_bundle(a.secure_connection_bundle_base64)
            store = cls(CqlSession([(bundle.host, bundle.cql_port)], user=a.gateway_user, password=a.gateway_password,
                                   ssl_ctx=bundle.ssl_ctx, local_dc=bundle.local_dc, request_timeout=a.request_timeout,
                                   consistency=a.consistency),
                        keyspace=a.keyspace or bundle.keyspace or KEYSPACE, table=a.table, consistency=a.consistency)
            store._bundle = bundle
            return store
        s = cfg.scylla_cql_store
        hosts = []
        for h in s.hosts:
            host, _, port = h.partition(":")
            hosts.append((host, int(port) if port else s.port))
        sess = CqlSession(hosts, user=s.user, password=s.password, local_dc=s.local_dc,
                          connections_per_host=s.connections_per_host, request_timeout=s.request_timeout,
                          connect_timeout=s.connect_timeout, token_aware=s.token_aware, consistency=s.consistency,
                          shard_aware=s.shard_aware, connections_per_shard=s.connections_per_shard)
        return cls(sess, keyspace=s.keyspace, table=s.table, consistency=s.consistency)

    async def connect(self) -> None:
        bundle = getattr(self, "_bundle", None)
        if bundle is not None:
            info = await astra_contact_info(bundle)
            proxy = info.get("sni_proxy_address", "")
            ph, _, pp = proxy.rpartition(":")
            self.session.sni_proxy = (ph, int(pp))
            self.session.local_dc = info.get("local_dc", self.session.local_dc)
            self.session.contact_points = [(hid, 0) for hid in info.get("contact_points", [])] or self.session.contact_points
        await self.session.connect()
        await asyncio.gather(*(self.session.prepare(q) for q in (self.q_read, self.q_read_status, self.q_insert,
                                                                  self.q_update_failure, self.q_update_stage)))

    async def close(self) -> None:
        await self.session.close()

    async def read_checkpoint(self, algorithm: str, request_id: str) -> Optional[CheckpointedRequest]:
        self.reads += 1
        rows = await self.session.execute(self.q_read, (algorithm, request_id), consistency=self.cl)
        if not rows.rows:
            return None
        return CheckpointedRequest(*rows.rows[0])

    async def read_status(self, algorithm: str, request_id: str) -> Optional[CheckpointedRequest]:
        self.reads += 1
        rows = await self.session.execute(self.q_read_status, (algorithm, request_id), consistency=self.cl)
        if not rows.rows:
            return None
        return StageRow(algorithm, request_id, rows.rows[0][0])

    async def upsert_checkpoint(self, checkpoint: CheckpointedRequest) -> None:
        self.writes += 1
        await self.session.execute(self.q_insert, checkpoint.as_row(), consistency=self.cl)

    async def upsert_many(self, checkpoints: Sequence[CheckpointedRequest], chunk: int = 64) -> None:
        """Bulk full-row upserts as UNLOGGED batches (the receiver's new-run inserts)."""
        ps = await self.session.prepare(self.q_insert)
        for i in range(0, len(checkpoints), chunk):
            part = checkpoints[i:i + chunk]
            self.writes += len(part)
            await self.session.execute_batch(ps, [c.as_row() for c in part], consistency=self.cl)

    async def update_status(self, algorithm, request_id, lifecycle_stage, failure_cause, failure_details, last_modified,
                            only_if_stages=None, set_failure=True) -> bool:
        self.writes += 1
        if set_failure:
            q = self.q_update_failure
            vals: List[Any] = [lifecycle_stage, failure_cause, failure_details, last_modified, algorithm, request_id]
        else:
            q = self.q_update_stage
            vals = [lifecycle_stage, last_modified, algorithm, request_id]
        if only_if_stages is None:
            await self.session.execute(q, vals, consistency=self.cl)
            return True
        applied, _stage = await self._cas(q, vals, only_if_stages)
        return applied

    async def cas_update(self, algorithm, request_id, lifecycle_stage, failure_cause, failure_details, last_modified,
                         only_if_stages, set_failure=True) -> Tuple[bool, Optional[str]]:
        """One lightweight transaction in place of read + write: ``(applied, current stage)``;
        the stage is the row's when the condition failed (None: no such row)."""
        self.writes += 1
        if set_failure:
            return await self._cas(self.q_update_failure, [lifecycle_stage, failure_cause, failure_details,
                                                           last_modified, algorithm, request_id], only_if_stages)
        return await self._cas(self.q_update_stage, [lifecycle_stage, last_modified, algorithm, request_id],
                               only_if_stages)

    async def _cas(self, q: str, vals: List[Any], only_if_stages) -> Tuple[bool, Optional[str]]:
        stages = tuple(only_if_stages)
        cq = self._cas_q.get((q, len(stages)))
        if cq is None:
            cq = self._cas_q[(q, len(stages))] = q + " IF lifecycle_stage IN (" + ", ".join("?" for _ in stages) + ")"
        rows = await self.session.execute(cq, vals + list(stages), consistency=self.cl, serial=self.serial)
        if not rows.rows:
            return False, None
        row = rows.rows[0]
        if row[0]:
            return True, None
        # not applied: Cassandra/Scylla return the current values of the condition's columns
        # (or the whole row); a missing row returns [applied] alone
        try:
            i = rows.names.index("lifecycle_stage")
        except ValueError:
            return False, None
        return False, row[i] if i < len(row) else None

    async def create_schema(self, replication: str = "{'class': 'SimpleStrategy', 'replication_factor': 1}") -> None:
        """Keyspace + table + indexes (what ``prepare-scylla.sh`` applies in the reference)."""
        from ..models.checkpoint import create_index_cql, create_table_cql

        await self.session.query(f"CREATE KEYSPACE IF NOT EXISTS {self.keyspace} WITH replication = {replication}")
        ddl = create_table_cql(self.keyspace, self.table).replace("create table", "CREATE TABLE IF NOT EXISTS", 1)
        await self.session.query(ddl)
        for stmt in create_index_cql(self.keyspace, self.table):
            await self.session.query(stmt.replace("create index", "CREATE INDEX IF NOT EXISTS", 1).rstrip(";"))
