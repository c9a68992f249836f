"""Metrics registry with Prometheus text exposition and a DogStatsD sink.

The reference attaches a DogStatsD client named ``nexus_receiver`` to its
context (``/root/reference/main.go:17``; socket from ``DD_DOGSTATSD_URL``,
``/root/reference/.helm/templates/deployment.yaml:92-93``) and the nexus-core
actor presumably emits queue metrics through it.  This build keeps the
DogStatsD sink (same env names; namespace configurable, default
``nexus_supervisor``) and adds Prometheus exposition plus HDR latency
histograms for the north-star metric (pod-fail → checkpoint latency).

The registry is loop-confined and lock-free: ``inc``/``observe`` are plain
dict/list updates on the hot path.
"""
from __future__ import annotations

import os
import socket
import time
from typing import Dict, Iterable, Optional, Tuple

from .histogram import LatencyHistogram

LabelKey = Tuple[Tuple[str, str], ...]


_LK_MEMO: Dict[Tuple, LabelKey] = {}


def _lk(labels: Optional[Dict[str, str]]) -> LabelKey:
    """Canonical (sorted) label key; memoised on the items in call order, since the hot
    counters pass the same few label sets (action, stage × class) once per decision."""
    if not labels:
        return ()
    raw = tuple(labels.items())
    try:
        k = _LK_MEMO.get(raw)
    except TypeError:  # an unhashable label value
        return tuple(sorted(raw))
    if k is None:
        if len(_LK_MEMO) > 4096:
            _LK_MEMO.clear()
        k = _LK_MEMO[raw] = tuple(sorted(raw))
    return k


class Metrics:
    def __init__(self, namespace: str = "nexus_supervisor", static_tags: Optional[Dict[str, str]] = None):
        self.namespace = namespace
        self.static_tags = dict(static_tags or {})
        self.counters: Dict[str, Dict[LabelKey, float]] = {}
        self.gauges: Dict[str, Dict[LabelKey, float]] = {}
        self.hists: Dict[str, Dict[LabelKey, LatencyHistogram]] = {}
        self.help: Dict[str, str] = {}
        self.statsd: Optional["DogStatsd"] = None
        self._h0: Dict[str, LatencyHistogram] = {}  # unlabelled series: one dict probe per observation

    def describe(self, name: str, text: str) -> None:
        self.help[name] = text

    def inc(self, name: str, value: float = 1.0, labels: Optional[Dict[str, str]] = None) -> None:
        d = self.counters.get(name)
        if d is None:
            d = self.counters[name] = {}
        k = _lk(labels) if labels else ()
        d[k] = d.get(k, 0.0) + value
        if self.statsd is not None:
            self.statsd.count(name, value, labels)

    def set(self, name: str, value: float, labels: Optional[Dict[str, str]] = None) -> None:
        d = self.gauges.get(name)
        if d is None:
            d = self.gauges[name] = {}
        d[_lk(labels)] = float(value)
        if self.statsd is not None:
            self.statsd.gauge(name, value, labels)

    def observe_seconds(self, name: str, seconds: float, labels: Optional[Dict[str, str]] = None) -> None:
        if not labels:
            h = self._h0.get(name)
            if h is not None:
                h.record(seconds * 1e6)
                if self.statsd is not None:
                    self.statsd.timing(name, seconds * 1e3, None)
                return
        d = self.hists.get(name)
        if d is None:
            d = self.hists[name] = {}
        k = _lk(labels)
        h = d.get(k)
        if h is None:
            h = d[k] = LatencyHistogram()
        if not k:
            self._h0[name] = h
        h.record(seconds * 1e6)
        if self.statsd is not None:
            self.statsd.timing(name, seconds * 1e3, labels)

    def hist0(self, name: str) -> LatencyHistogram:
        """The unlabelled series of ``name`` (created when missing), for a caller that records
        into it directly — only while no DogStatsD sink is attached (``statsd is None``)."""
        h = self._h0.get(name)
        if h is None:
            h = self.hists.setdefault(name, {}).setdefault((), LatencyHistogram())
            self._h0[name] = h
        return h

    def histogram(self, name: str, labels: Optional[Dict[str, str]] = None) -> Optional[LatencyHistogram]:
        return self.hists.get(name, {}).get(_lk(labels))

    def counter(self, name: str, labels: Optional[Dict[str, str]] = None) -> float:
        return self.counters.get(name, {}).get(_lk(labels), 0.0)

    def gauge(self, name: str, labels: Optional[Dict[str, str]] = None) -> float:
        return self.gauges.get(name, {}).get(_lk(labels), 0.0)

    # ------------------------------------------------------------ exposition
    def prometheus_text(self) -> str:
        lines = []
        ns = self.namespace

        def fmt_labels(k: LabelKey, extra: Iterable[Tuple[str, str]] = ()) -> str:
            items = list(self.static_tags.items()) + list(k) + list(extra)
            if not items:
                return ""
            return "{" + ",".join(f'{a}="{_esc(b)}"' for a, b in items) + "}"

        for name, series in sorted(self.counters.items()):
            full = f"{ns}_{name}_total"
            if name in self.help:
                lines.append(f"# HELP {full} {self.help[name]}")
            lines.append(f"# TYPE {full} counter")
            for k, v in series.items():
                lines.append(f"{full}{fmt_labels(k)} {v:g}")
        for name, series in sorted(self.gauges.items()):
            full = f"{ns}_{name}"
            if name in self.help:
                lines.append(f"# HELP {full} {self.help[name]}")
            lines.append(f"# TYPE {full} gauge")
            for k, v in series.items():
                lines.append(f"{full}{fmt_labels(k)} {v:g}")
        for name, series in sorted(self.hists.items()):
            full = f"{ns}_{name}_seconds"
            if name in self.help:
                lines.append(f"# HELP {full} {self.help[name]}")
            lines.append(f"# TYPE {full} summary")
            for k, h in series.items():
                for q in (0.5, 0.9, 0.99, 0.999):
                    lines.append(f"{full}{fmt_labels(k, [('quantile', str(q))])} {h.percentile(q * 100) / 1e6:.9g}")
                lines.append(f"{full}_sum{fmt_labels(k)} {h.sum / 1e6:.9g}")
                lines.append(f"{full}_count{fmt_labels(k)} {h.total}")
        return "\n".join(lines) + "\n"

    def snapshot(self) -> Dict[str, object]:
        out: Dict[str, object] = {}
        for name, series in self.counters.items():
            for k, v in series.items():
                out[name + _suffix(k)] = v
        for name, series in self.gauges.items():
            for k, v in series.items():
                out[name + _suffix(k)] = v
        for name, series in self.hists.items():
            for k, h in series.items():
                out[name + _suffix(k)] = {kk: (vv / 1e6 if kk.startswith("p") or kk in ("mean", "max", "min") else vv)
                                          for kk, vv in h.summary().items()}
        return out


def _suffix(k: LabelKey) -> str:
    return "" if not k else "{" + ",".join(f"{a}={b}" for a, b in k) + "}"


def _esc(s: str) -> str:
    return str(s).replace("\\", "\\\\").replace('"', '\\"').replace("\n", "\\n")


class DogStatsd:
    """Minimal DogStatsD datagram client (``udp://host:port`` or ``unix:///path``)."""

    def __init__(self, url: str, namespace: str = "nexus_supervisor", tags: Optional[Dict[str, str]] = None,
                 max_buffer: int = 8192, flush_interval: float = 0.25):
        self.namespace = namespace
        self.tags = dict(tags or {})
        self.max_buffer = max_buffer
        self.flush_interval = flush_interval
        self._buf: list = []
        self._size = 0
        self._last_flush = time.monotonic()
        self.dropped = 0
        if url.startswith("unix://"):
            self.sock = socket.socket(socket.AF_UNIX, socket.SOCK_DGRAM)
            self.addr = url[len("unix://"):]
        else:
            hostport = url[len("udp://"):] if url.startswith("udp://") else url
            host, _, port = hostport.rpartition(":")
            self.sock = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
            self.addr = (host or "127.0.0.1", int(port or 8125))
        self.sock.setblocking(False)

    @classmethod
    def from_env(cls, namespace: str, env=None) -> Optional["DogStatsd"]:
        env = os.environ if env is None else env
        url = env.get("DD_DOGSTATSD_URL")
        if not url:
            return None
        tags = {}
        for key, tag in (("DD_SERVICE", "service"), ("DD_VERSION", "version"), ("DD_ENV", "env")):
            if env.get(key):
                tags[tag] = env[key]
        if env.get("DD_ENTITY_ID"):
            tags["dd.internal.entity_id"] = env["DD_ENTITY_ID"]
        return cls(url, namespace, tags)

    def _emit(self, name: str, value, mtype: str, labels: Optional[Dict[str, str]]):
        tags = dict(self.tags)
        if labels:
            tags.update(labels)
        tag_s = ("|#" + ",".join(f"{k}:{v}" for k, v in tags.items())) if tags else ""
        line = f"{self.namespace}.{name}:{value:g}|{mtype}{tag_s}"
        self._buf.append(line)
        self._size += len(line) + 1
        now = time.monotonic()
        if self._size >= self.max_buffer or now - self._last_flush >= self.flush_interval:
            self.flush()

    def count(self, name, value, labels=None):
        self._emit(name, value, "c", labels)

    def gauge(self, name, value, labels=None):
        self._emit(name, value, "g", labels)

    def timing(self, name, ms, labels=None):
        self._emit(name, ms, "d", labels)

    def flush(self) -> None:
        if not self._buf:
            return
        payload = "\n".join(self._buf).encode()
        self._buf.clear()
        self._size = 0
        self._last_flush = time.monotonic()
        try:
            self.sock.sendto(payload, self.addr)
        except OSError:
            self.dropped += 1

    def attach(self, loop) -> None:
        """Flush on a timer too (not only when the next metric is emitted), so the tail of a
        burst reaches the agent within ``flush_interval`` even if the process goes idle."""
        self._loop = loop

        def tick():
            if self.sock.fileno() < 0:
                return
            if self._buf and time.monotonic() - self._last_flush >= self.flush_interval:
                self.flush()
            self._timer = loop.call_later(self.flush_interval, tick)

        self._timer = loop.call_later(self.flush_interval, tick)

    def close(self) -> None:
        timer = getattr(self, "_timer", None)
        if timer is not None:
            timer.cancel()
        self.flush()
        self.sock.close()
