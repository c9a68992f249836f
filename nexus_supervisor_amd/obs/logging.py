"""Structured logging with klog-style verbosity.

The reference logs through slog bridged into klog (``/root/reference/main.go:15,19``)
with V(0) for decisions and errors, V(1) for no-op events and V(4) for every
raw event (``/root/reference/services/supervisor.go:138,162,256``).
``log-level`` (``NEXUS__LOG_LEVEL``, Helm default ``INFO``) maps to a max
verbosity: ERROR/WARN/INFO → V(0), DEBUG → V(4), TRACE → V(9).  Lines are JSON
objects with the reference's structured keys (``requestId``, ``algorithm``,
``reason``, ``message``).
"""
from __future__ import annotations

import json
import logging
import os
import sys
import threading
import time
from typing import Any, Dict, Optional

_LEVELS = {"TRACE": (logging.DEBUG, 9), "DEBUG": (logging.DEBUG, 4), "INFO": (logging.INFO, 0),
           "WARN": (logging.WARNING, 0), "WARNING": (logging.WARNING, 0), "ERROR": (logging.ERROR, 0)}
LOG_LEVELS = tuple(_LEVELS)


def parse_level(level: str):
    """(python level, klog verbosity) of a ``log-level`` string; unknown → ValueError
    (the reference fails start-up on a logger it cannot configure, ``main.go:22-24``)."""
    key = (level or "INFO").strip().upper()
    if key not in _LEVELS:
        raise ValueError(f"unknown log-level {level!r} (one of {', '.join(LOG_LEVELS)})")
    return _LEVELS[key]


class JsonFormatter(logging.Formatter):
    def __init__(self, static: Optional[Dict[str, Any]] = None):
        super().__init__()
        self.static = dict(static or {})

    _sec = -1
    _sec_text = ""

    def format(self, record: logging.LogRecord) -> str:
        error = self.formatException(record.exc_info) if record.exc_info else None
        return self.line(record.created, record.msecs, record.levelname, record.name, record.getMessage(),
                         getattr(record, "v", None), getattr(record, "kv", None), error)

    def line(self, created: float, msecs: float, levelname: str, name: str, msg: str, v=None, kv=None,
             error: Optional[str] = None) -> str:
        """One JSON line (also :meth:`KLogger._emit`'s direct path, which has no record)."""
        sec = int(created)
        if sec != self._sec:  # one strftime per second, not per line
            self._sec, self._sec_text = sec, time.strftime("%Y-%m-%dT%H:%M:%S", time.gmtime(sec))
        doc: Dict[str, Any] = {"time": f"{self._sec_text}.{int(msecs):03d}Z",
                               "level": levelname, "logger": name, "msg": msg}
        if v:
            doc["v"] = v
        if kv:
            doc.update(kv)
        if error is not None:
            doc["error"] = error
        if self.static:
            doc.update(self.static)
        if _dumps is not None:  # one log line per decision (reference V(0)): native encoder
            return _dumps(doc, default=str).decode()
        return json.dumps(doc, default=str, separators=(",", ":"), ensure_ascii=False)


try:
    from .._kube_native import dumps as _dumps
except ImportError:  # pragma: no cover - CPU hosts without the native build
    _dumps = None


class _Record(logging.LogRecord):
    """A :class:`logging.LogRecord` built without the caller lookup (``findCaller`` walks
    the stack and normalises file names) and the process / thread-name probes of
    ``LogRecord.__init__``: the JSON formatter reads none of them, and a decision logged at
    V(0) paid ~40 % of its log line for them.  Handlers and filters see a normal record
    (``pathname``/``lineno`` empty, ``threadName``/``processName`` None)."""

    def __init__(self, name: str, level: int, msg: str, extra: Dict[str, Any]):  # noqa: D107 - no super().__init__
        ct = time.time()
        self.name = name
        self.msg = msg
        self.args = ()
        self.levelno = level
        self.levelname = _LEVEL_NAMES.get(level) or logging.getLevelName(level)
        self.pathname = self.filename = self.module = ""
        self.lineno = 0
        self.funcName = None
        self.exc_info = self.exc_text = self.stack_info = None
        self.created = ct
        self.msecs = (ct - int(ct)) * 1000
        self.relativeCreated = (ct - logging._startTime) * 1000  # type: ignore[attr-defined]
        self.thread = threading.get_ident()
        self.threadName = self.processName = None
        self.process = os.getpid()
        self.__dict__.update(extra)


_LEVEL_NAMES = {logging.DEBUG: "DEBUG", logging.INFO: "INFO", logging.WARNING: "WARNING", logging.ERROR: "ERROR"}


class KLogger:
    """``logger.v(4).info("event received", object=...)`` on top of :mod:`logging`."""

    def __init__(self, name: str = "nexus_supervisor_amd", verbosity: int = 0):
        self._log = logging.getLogger(name)
        self.verbosity = verbosity

    def v(self, level: int) -> "_V":
        return _V(self, level)

    def enabled(self, level: int) -> bool:
        return level <= self.verbosity

    def _emit(self, level: int, msg: str, extra: Dict[str, Any]) -> None:
        lg = self._log
        if lg.isEnabledFor(level):
            hs = lg.handlers
            if len(hs) == 1 and not lg.filters and not lg.propagate:
                h = hs[0]
                if type(h) is BufferedStreamHandler and not h.filters and type(h.formatter) is JsonFormatter \
                        and level >= h.level:
                    # the deployed configuration (configure_logging without a Datadog sink): the
                    # line straight into the handler's buffer — no LogRecord, no filter or
                    # handler-chain walk
                    ct = time.time()
                    h.write_line(h.formatter.line(ct, (ct - int(ct)) * 1000, _LEVEL_NAMES.get(level) or
                                                  logging.getLevelName(level), lg.name, msg, extra.get("v"),
                                                  extra.get("kv")), level)
                    return
            lg.handle(_Record(lg.name, level, msg, extra))

    def info(self, msg: str, **kv) -> None:
        self._emit(logging.INFO, msg, {"kv": kv})

    def warning(self, msg: str, **kv) -> None:
        self._log.warning(msg, extra={"kv": kv})

    def error(self, err: Optional[BaseException], msg: str, **kv) -> None:
        if err is not None:
            kv = dict(kv, err=str(err))
        self._log.error(msg, extra={"kv": kv})


class _V:
    __slots__ = ("parent", "level")

    def __init__(self, parent: KLogger, level: int):
        self.parent = parent
        self.level = level

    def info(self, msg: str, **kv) -> None:
        if self.level <= self.parent.verbosity:
            self.parent._emit(logging.INFO, msg, {"kv": kv, "v": self.level})

    def error(self, err: Optional[BaseException], msg: str, **kv) -> None:
        self.parent.error(err, msg, **kv)

    @property
    def enabled(self) -> bool:
        return self.level <= self.parent.verbosity


try:
    from asyncio import _get_running_loop as _running_loop  # C accessor: no exception when there is none
except ImportError:  # pragma: no cover
    def _running_loop():
        return None


class BufferedStreamHandler(logging.StreamHandler):
    """``StreamHandler`` that does not flush per record: ``StreamHandler.emit`` flushes the
    stream after every line, one ``write`` syscall per decision logged at V(0).  Lines go
    into the stream's buffer and are flushed at most ``interval`` seconds later, at WARNING
    and above immediately, and on shutdown.

    On an asyncio loop the delayed flush is a ``call_later`` timer; elsewhere one long-lived
    flusher thread does it and a line that dirties a clean buffer only sets an event.
    (A ``threading.Timer`` per flush window started a thread
    for the first line of every window: at the north-star churn — a decision every ~60 ms,
    a window every few lines — that was ~130 µs of thread start-up on an MI355X host in
    front of every logged decision's queueing, the largest item of an event-driven
    decision's classification stage.)"""

    def __init__(self, stream=None, interval: float = 0.2):
        super().__init__(stream)
        self.interval = interval
        self._dirty = False
        self._closed = False
        self._wake = threading.Event()
        self._flusher: Optional[threading.Thread] = None

    def emit(self, record: logging.LogRecord) -> None:
        try:
            msg = self.format(record)
            self.stream.write(msg + self.terminator)
        except RecursionError:  # pragma: no cover - as logging.StreamHandler
            raise
        except Exception:  # pragma: no cover
            self.handleError(record)
            return
        self._written(record.levelno)

    def write_line(self, line: str, levelno: int) -> None:
        """A formatted line from :meth:`KLogger._emit`'s direct path (under the handler's
        lock, as ``Handler.handle`` would take it: a flusher thread may flush meanwhile)."""
        lock = self.lock
        if lock is not None:
            lock.acquire()
        try:
            self.stream.write(line + self.terminator)
        except Exception:  # pragma: no cover - a closed stream: as handleError, say nothing
            return
        finally:
            if lock is not None:
                lock.release()
        self._written(levelno)

    def _written(self, levelno: int) -> None:
        if levelno >= logging.WARNING or self.interval <= 0:
            self.flush()
        elif not self._dirty:
            self._dirty = True
            loop = _running_loop()
            if loop is not None:
                # on an event loop (the supervisor's): a timer handle, no thread wake-up
                loop.call_later(self.interval, self._loop_flush)
                return
            if self._flusher is None or not self._flusher.is_alive():
                # (re)started lazily: also after a fork, whose child has no such thread
                self._flusher = threading.Thread(target=self._run, name="log-flush", daemon=True)
                self._flusher.start()
            self._wake.set()

    def _loop_flush(self) -> None:
        self._dirty = False
        try:
            self.flush()
        except Exception:  # noqa: BLE001 - e.g. the stream was closed under us
            pass

    def _run(self) -> None:
        while not self._closed:
            self._wake.wait()
            self._wake.clear()
            if self._closed:
                break
            time.sleep(self.interval)
            self._dirty = False  # before the flush: a line written from here on re-arms
            try:
                self.flush()
            except Exception:  # noqa: BLE001 - e.g. the stream was closed under us
                pass

    def close(self) -> None:
        self._closed = True
        self._wake.set()
        self.flush()
        super().close()


def configure_logging(level: str = "INFO", stream=None, static: Optional[Dict[str, Any]] = None,
                      env: Optional[Dict[str, str]] = None) -> KLogger:
    """Configure the root ``nexus_supervisor_amd`` logger (telemetry.ConfigureLogger analog,
    ``/root/reference/main.go:15``): JSON lines on stdout, plus the batched Datadog HTTP
    sink when the ``DATADOG__*`` variables are set (``obs/datadog.py``)."""
    pylevel, verbosity = parse_level(level)
    root = logging.getLogger("nexus_supervisor_amd")
    root.setLevel(pylevel)
    shutdown_logging()
    h = BufferedStreamHandler(stream or sys.stdout)
    h.setFormatter(JsonFormatter(static))
    root.addHandler(h)
    from .datadog import DatadogLogHandler

    dd = DatadogLogHandler.from_env(env)
    if dd is not None:
        dd.setFormatter(JsonFormatter(static))
        root.addHandler(dd)
    root.propagate = False
    return KLogger("nexus_supervisor_amd", verbosity)


def shutdown_logging() -> None:
    """Flush and detach the handlers (the Datadog sink ships what is still queued)."""
    root = logging.getLogger("nexus_supervisor_amd")
    for h in list(root.handlers):
        root.removeHandler(h)
        if isinstance(h, BufferedStreamHandler):
            h.close()  # flushes; the stream itself (stdout) stays open
        elif not isinstance(h, logging.StreamHandler):
            h.close()
