"""HDR-style log-linear latency histogram (pure Python, O(1) record; the hot path
records a handful per decision).

Values are recorded in integer microseconds.  Buckets have a fixed relative
precision: each power-of-two range ``[2^k, 2^(k+1))`` is split into
``2**sub_bits`` linear sub-buckets (sub_bits=7 → <0.8% error), like
HdrHistogram with 2 significant digits.  Recording is O(1), percentile query
O(#buckets).
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Tuple


class LatencyHistogram:
    # slots: record() reads and writes six attributes, a handful of times per decision
    __slots__ = ("sub_bits", "sub", "max_exp", "counts", "total", "sum", "min", "max")

    def __init__(self, sub_bits: int = 7, max_exp: int = 40):
        self.sub_bits = sub_bits
        self.sub = 1 << sub_bits
        self.max_exp = max_exp
        self.counts: List[int] = [0] * ((max_exp + 1) * self.sub)
        self.total = 0
        self.sum = 0
        self.min = None
        self.max = 0

    def _index(self, v: int) -> int:
        if v < self.sub:
            return v
        e = v.bit_length() - self.sub_bits - 1  # >= 0; (v >> e) in [sub, 2*sub)
        if e >= self.max_exp:
            return len(self.counts) - 1
        return e * self.sub + (v >> e)

    def _bounds(self, idx: int):
        if idx < self.sub:
            return idx, idx + 1
        e = idx // self.sub - 1
        top = self.sub + idx % self.sub
        return top << e, (top + 1) << e

    def _value_at(self, idx: int) -> int:
        lo, hi = self._bounds(idx)
        return (lo + hi - 1) // 2

    def record(self, value_us: float, count: int = 1) -> None:
        v = int(value_us)
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

    def record_seconds(self, seconds: float) -> None:
        self.record(seconds * 1e6)

    def percentile(self, p: float) -> float:
        """Value (µs) at percentile ``p`` in [0, 100]."""
        if self.total == 0:
            return 0.0
        target = max(1, int(round(p / 100.0 * self.total + 0.4999999)))
        run = 0
        for i, c in enumerate(self.counts):
            if c:
                run += c
                if run >= target:
                    return float(min(self._value_at(i), self.max))
        return float(self.max)

    def mean(self) -> float:
        return self.sum / self.total if self.total else 0.0

    def merge(self, other: "LatencyHistogram") -> None:
        assert other.sub_bits == self.sub_bits and len(other.counts) == len(self.counts)
        for i, c in enumerate(other.counts):
            if c:
                self.counts[i] += c
        self.total += other.total
        self.sum += other.sum
        if other.min is not None and (self.min is None or other.min < self.min):
            self.min = other.min
        self.max = max(self.max, other.max)

    def reset(self) -> None:
        self.counts = [0] * len(self.counts)
        self.total = self.sum = self.max = 0
        self.min = None

    def summary(self, ps: Iterable[float] = (50, 90, 99, 99.9)) -> Dict[str, float]:
        out = {f"p{p:g}": self.percentile(p) for p in ps}
        out.update(count=self.total, mean=self.mean(), max=float(self.max), min=float(self.min or 0))
        return out

    def buckets(self) -> List[Tuple[int, int]]:
        """Non-empty (upper_bound_us, count) pairs."""
        out = []
        for i, c in enumerate(self.counts):
            if c:
                out.append((self._bounds(i)[1], c))
        return out
