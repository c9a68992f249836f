"""Go ``time.Duration`` string parsing / formatting.

The reference config surface uses Go duration syntax (``100ms``, ``1s``,
``1m30s``) for ``failure-rate-base-delay`` / ``failure-rate-max-delay``
(``/root/reference/.helm/values.yaml:143-149``) and the checkpoint column
``payload_valid_for`` holds the same syntax (``'1h'``, ``'15m'`` in
``/root/reference/test-resources/checkpoints.cql:38,47``).  Durations are kept
as float seconds internally.
"""
from __future__ import annotations

import re

_UNITS = {
    "ns": 1e-9,
    "us": 1e-6,
    "µs": 1e-6,
    "μs": 1e-6,
    "ms": 1e-3,
    "s": 1.0,
    "m": 60.0,
    "h": 3600.0,
}
_PART = re.compile(r"(\d+(?:\.\d*)?|\.\d+)(ns|us|µs|μs|ms|s|m|h)")


def parse_duration(value) -> float:
    """Parse a Go duration (``"1h2m3.5s"``, ``"-100ms"``, ``"0"``) into seconds.

    Numbers (int/float) are accepted as seconds.  Raises ``ValueError`` on
    malformed input, matching ``time.ParseDuration`` strictness (a bare
    non-zero number without unit is rejected).
    """
    if isinstance(value, bool):
        raise ValueError(f"invalid duration {value!r}")
    if isinstance(value, (int, float)):
        return float(value)
    s = str(value).strip()
    if not s:
        raise ValueError("empty duration")
    sign = 1.0
    if s[0] in "+-":
        sign = -1.0 if s[0] == "-" else 1.0
        s = s[1:]
    if s == "0":
        return 0.0
    pos = 0
    total = 0.0
    while pos < len(s):
        m = _PART.match(s, pos)
        if not m:
            raise ValueError(f"invalid duration {value!r}")
        total += float(m.group(1)) * _UNITS[m.group(2)]
        pos = m.end()
    if pos == 0:
        raise ValueError(f"invalid duration {value!r}")
    return sign * total


def format_duration(seconds: float) -> str:
    """Format seconds the way Go's ``Duration.String()`` does (``1m30s``, ``100ms``)."""
    if seconds == 0:
        return "0s"
    neg = seconds < 0
    ns = round(abs(seconds) * 1e9)
    sign = "-" if neg else ""
    if ns < 1000:
        return f"{sign}{ns}ns"
    if ns < 1_000_000:
        return f"{sign}{_trim(ns / 1e3)}µs"
    if ns < 1_000_000_000:
        return f"{sign}{_trim(ns / 1e6)}ms"
    h, rem = divmod(ns, 3_600_000_000_000)
    m, rem = divmod(rem, 60_000_000_000)
    sec = rem / 1e9
    out = sign
    if h:
        out += f"{h}h"
    if h or m:
        out += f"{m}m"
    out += f"{_trim(sec)}s"
    return out


def _trim(x: float) -> str:
    s = f"{x:.9f}".rstrip("0").rstrip(".")
    return s or "0"
