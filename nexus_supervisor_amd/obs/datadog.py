"""Datadog log shipping (the reference's ``telemetry.ConfigureLogger`` fan-out).

The reference logs through slog with a multi-handler: stdout plus slog-datadog when
``DATADOG__API_KEY``, ``DATADOG__ENDPOINT``, ``DATADOG__APPLICATION_HOST`` and
``DATADOG__SERVICE_NAME`` are set (``/root/reference/main.go:15,22-24``;
``/root/reference/.helm/templates/deployment.yaml:68-87``).  This handler
is the same sink built for a supervisor whose event loop must never wait on HTTPS:

* ``emit`` only formats the record and puts it on a bounded queue (full → the line is
  counted in ``dropped`` and the caller moves on);
* one daemon thread batches up to ``batch_size`` lines or ``flush_interval`` seconds
  and POSTs them gzip-compressed to the v2 HTTP intake
  (``https://http-intake.logs.<site>/api/v2/logs``, header ``DD-API-KEY``);
* 408/429/5xx and connection errors are retried with exponential backoff (3 tries),
  other 4xx drop the batch (a bad key must not wedge the queue);
* ``close()`` drains what is queued within a deadline.

``DATADOG__ENDPOINT`` is the Datadog site (``datadoghq.eu``, the Helm default) or a
full ``http(s)://`` base URL (proxies, tests).
"""
from __future__ import annotations

import gzip
import json
import logging
import os
import queue
import threading
import time
import urllib.error
import urllib.request
from typing import Any, Dict, List, Mapping, Optional

_STATUS = {"DEBUG": "debug", "INFO": "info", "WARNING": "warn", "ERROR": "error", "CRITICAL": "critical"}


def intake_url(endpoint: str) -> str:
    endpoint = endpoint.strip().rstrip("/")
    if "://" in endpoint:
        return endpoint if endpoint.endswith("/api/v2/logs") else endpoint + "/api/v2/logs"
    return f"https://http-intake.logs.{endpoint}/api/v2/logs"


class DatadogLogHandler(logging.Handler):
    def __init__(self, api_key: str, endpoint: str, service: str, host: str = "", *,
                 source: str = "nexus-supervisor", tags: Optional[Mapping[str, str]] = None,
                 batch_size: int = 500, flush_interval: float = 2.0, max_queue: int = 20_000,
                 timeout: float = 5.0, retries: int = 3):
        super().__init__()
        self.url = intake_url(endpoint)
        self.api_key = api_key
        self.service = service
        self.host = host
        self.source = source
        self.tags = ",".join(f"{k}:{v}" for k, v in (tags or {}).items())
        self.batch_size = batch_size
        self.flush_interval = flush_interval
        self.timeout = timeout
        self.retries = retries
        self.q: "queue.Queue[Optional[Dict[str, Any]]]" = queue.Queue(maxsize=max_queue)
        self.dropped = 0
        self.sent = 0
        self.failed_batches = 0
        self._closed = False
        self._thread = threading.Thread(target=self._run, name="datadog-logs", daemon=True)
        self._thread.start()

    @classmethod
    def from_env(cls, env: Optional[Mapping[str, str]] = None, **kw) -> Optional["DatadogLogHandler"]:
        """The handler when all four ``DATADOG__*`` variables are set, else None."""
        env = os.environ if env is None else env
        key, endpoint = env.get("DATADOG__API_KEY", ""), env.get("DATADOG__ENDPOINT", "")
        host, service = env.get("DATADOG__APPLICATION_HOST", ""), env.get("DATADOG__SERVICE_NAME", "")
        if not (key and endpoint and host and service):
            return None
        tags = {}
        if env.get("DD_VERSION"):
            tags["version"] = env["DD_VERSION"]
        if env.get("DD_ENV"):
            tags["env"] = env["DD_ENV"]
        return cls(key, endpoint, service, host, tags=tags, **kw)

    # ---------------------------------------------------------------- producer side
    def emit(self, record: logging.LogRecord) -> None:
        if self._closed:
            return
        try:
            msg = self.format(record)
            entry: Dict[str, Any] = {"message": msg, "ddsource": self.source, "service": self.service,
                                     "hostname": self.host, "status": _STATUS.get(record.levelname, "info")}
            if self.tags:
                entry["ddtags"] = self.tags
            self.q.put_nowait(entry)
        except queue.Full:
            self.dropped += 1
        except Exception:  # noqa: BLE001 - logging must never raise into the caller
            self.handleError(record)

    # ---------------------------------------------------------------- shipper thread
    def _run(self) -> None:
        batch: List[Dict[str, Any]] = []
        deadline = time.monotonic() + self.flush_interval
        while True:
            timeout = max(0.0, deadline - time.monotonic())
            try:
                item = self.q.get(timeout=timeout)
            except queue.Empty:
                item = False
            if item is None:  # close(): ship the rest and stop
                while True:
                    try:
                        rest = self.q.get_nowait()
                    except queue.Empty:
                        break
                    if rest:
                        batch.append(rest)
                    if len(batch) >= self.batch_size:
                        self._ship(batch)
                        batch = []
                if batch:
                    self._ship(batch)
                return
            if item:
                batch.append(item)
            if len(batch) >= self.batch_size or (batch and time.monotonic() >= deadline):
                self._ship(batch)
                batch = []
            if time.monotonic() >= deadline:
                deadline = time.monotonic() + self.flush_interval

    def _ship(self, batch: List[Dict[str, Any]]) -> None:
        body = gzip.compress(json.dumps(batch, separators=(",", ":")).encode())
        delay = 0.2
        for attempt in range(self.retries):
            req = urllib.request.Request(self.url, data=body, method="POST", headers={
                "DD-API-KEY": self.api_key, "Content-Type": "application/json", "Content-Encoding": "gzip"})
            try:
                with urllib.request.urlopen(req, timeout=self.timeout) as resp:  # noqa: S310 - fixed https intake
                    resp.read()
                self.sent += len(batch)
                return
            except urllib.error.HTTPError as exc:
                if exc.code not in (408, 429) and exc.code < 500:
                    break  # bad key / payload: retrying cannot help
            except (urllib.error.URLError, OSError):
                pass
            if attempt + 1 < self.retries:
                time.sleep(delay)
                delay *= 2
        self.failed_batches += 1
        self.dropped += len(batch)

    def close(self, timeout: float = 5.0) -> None:
        if not self._closed:
            self._closed = True
            try:
                self.q.put(None, timeout=timeout)
            except queue.Full:
                pass
            self._thread.join(timeout)
        super().close()
