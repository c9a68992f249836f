"""HDR-style log-linear latency histogram (O(1) record; the hot path records a handful
per decision).

Values are recorded in integer microseconds.  Buckets have a fixed relative
precision: each power-of-two range ``[2^k, 2^(k+1))`` is split into
``2**sub_bits`` linear sub-buckets (sub_bits=7 → <0.8% error), like
HdrHistogram with 2 significant digits.  Recording is O(1), percentile query
O(#buckets).

The record path is native (``csrc/kube/histogram.cpp``, ``_kube_native.LatencyHist``)
when the extension is built — six stage latencies per decision made the pure-Python
record ~3 % of a shard worker's CPU; :class:`PyLatencyHistogram` is the same histogram in
Python (CPU hosts without the build, and the reference the native one is tested against).
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Optional, Tuple


MAX_US = 1 << 53  # recorded values are clamped here (~285 years), as in the native histogram


class _HistMath:
    """Queries shared by both implementations (they only read ``counts`` and the stats)."""

    sub_bits: int
    sub: int

    def _bounds(self, idx: int):
        if idx < self.sub:
            return idx, idx + 1
        e = idx // self.sub - 1
        top = self.sub + idx % self.sub
        return top << e, (top + 1) << e

    def _value_at(self, idx: int) -> int:
        lo, hi = self._bounds(idx)
        return (lo + hi - 1) // 2

    def record_seconds(self, seconds: float) -> None:
        self.record(seconds * 1e6)  # type: ignore[attr-defined]

    def percentile(self, p: float) -> float:
        """Value (µs) at percentile ``p`` in [0, 100]."""
        total = self.total  # type: ignore[attr-defined]
        if total == 0:
            return 0.0
        target = max(1, int(round(p / 100.0 * total + 0.4999999)))
        run = 0
        mx = self.max  # type: ignore[attr-defined]
        for i, c in enumerate(self.counts):  # type: ignore[attr-defined]
            if c:
                run += c
                if run >= target:
                    return float(min(self._value_at(i), mx))
        return float(mx)

    def mean(self) -> float:
        total = self.total  # type: ignore[attr-defined]
        return self.sum / total if total else 0.0  # type: ignore[attr-defined]

    def summary(self, ps: Iterable[float] = (50, 90, 99, 99.9)) -> Dict[str, float]:
        out = {f"p{p:g}": self.percentile(p) for p in ps}
        out.update(count=self.total, mean=self.mean(), max=float(self.max), min=float(self.min or 0))  # type: ignore[attr-defined]
        return out

    def buckets(self) -> List[Tuple[int, int]]:
        """Non-empty (upper_bound_us, count) pairs."""
        return [(self._bounds(i)[1], c) for i, c in self.sparse()]  # type: ignore[attr-defined]


class PyLatencyHistogram(_HistMath):
    # slots: record() reads and writes six attributes, a handful of times per decision
    __slots__ = ("sub_bits", "sub", "max_exp", "counts", "total", "sum", "min", "max")

    def __init__(self, sub_bits: int = 7, max_exp: int = 40):
        self.sub_bits = sub_bits
        self.sub = 1 << sub_bits
        self.max_exp = max_exp
        self.counts: List[int] = [0] * ((max_exp + 1) * self.sub)
        self.total = 0
        self.sum = 0
        self.min: Optional[int] = None
        self.max = 0

    def _index(self, v: int) -> int:
        if v < self.sub:
            return v
        e = v.bit_length() - self.sub_bits - 1  # >= 0; (v >> e) in [sub, 2*sub)
        if e >= self.max_exp:
            return len(self.counts) - 1
        return e * self.sub + (v >> e)

    def record(self, value_us: float, count: int = 1) -> None:
        v = int(value_us) if value_us < MAX_US else MAX_US
        if v < self.sub:  # _index inlined: a handful of records per decision on the hot path
            if v < 0:
                v = 0
            idx = v
        else:
            e = v.bit_length() - self.sub_bits - 1
            idx = e * self.sub + (v >> e) if e < self.max_exp else len(self.counts) - 1
        self.counts[idx] += count
        self.total += count
        self.sum += v * count
        m = self.min
        if m is None or v < m:
            self.min = v
        if v > self.max:
            self.max = v

    def sparse(self) -> List[List[int]]:
        return [[i, c] for i, c in enumerate(self.counts) if c]

    def merge_state(self, sparse, total: int, hsum: int, hmin: Optional[int], hmax: int) -> None:
        for i, c in sparse:
            self.counts[i] += c
        self.total += total
        self.sum += hsum
        if hmin is not None and (self.min is None or hmin < self.min):
            self.min = hmin
        self.max = max(self.max, hmax)

    def merge(self, other) -> None:
        assert other.sub_bits == self.sub_bits and len(other.counts) == len(self.counts)
        self.merge_state(other.sparse(), other.total, other.sum, other.min, other.max)

    def reset(self) -> None:
        self.counts = [0] * len(self.counts)
        self.total = self.sum = self.max = 0
        self.min = None


try:
    from .._kube_native import LatencyHist as _NativeHist
except ImportError:  # pragma: no cover - CPU hosts without the native build
    _NativeHist = None


class NativeLatencyHistogram(_HistMath):
    """:class:`PyLatencyHistogram` with its state and ``record`` in C."""

    __slots__ = ("_h", "record", "sub_bits", "sub", "max_exp")

    def __init__(self, sub_bits: int = 7, max_exp: int = 40):
        self._h = _NativeHist(sub_bits, max_exp)
        self.record = self._h.record  # bound C method: no Python frame per sample
        self.sub_bits = sub_bits
        self.sub = 1 << sub_bits
        self.max_exp = max_exp

    @property
    def counts(self) -> List[int]:
        return self._h.counts()

    @property
    def total(self) -> int:
        return self._h.total

    @property
    def sum(self) -> int:
        return self._h.sum

    @property
    def min(self) -> Optional[int]:
        return self._h.min

    @property
    def max(self) -> int:
        return self._h.max

    def sparse(self) -> List[List[int]]:
        return self._h.sparse()

    def merge_state(self, sparse, total: int, hsum: int, hmin: Optional[int], hmax: int) -> None:
        h = self._h
        for i, c in sparse:
            h.add_bucket(i, c)
        mn = h.min
        if hmin is not None and (mn is None or hmin < mn):
            mn = hmin
        h.set_stats(h.total + total, h.sum + hsum, mn, max(h.max, hmax))

    def merge(self, other) -> None:
        if isinstance(other, NativeLatencyHistogram):
            self._h.merge(other._h)
        else:
            self.merge_state(other.sparse(), other.total, other.sum, other.min, other.max)

    def reset(self) -> None:
        self._h.reset()


LatencyHistogram = NativeLatencyHistogram if _NativeHist is not None else PyLatencyHistogram
