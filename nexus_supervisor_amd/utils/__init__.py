"""Small shared helpers (durations, clocks, coalescing)."""
from .durations import format_duration, parse_duration


def coalesce(*values):
    """Return the first argument that is not ``None`` (nexus-core ``util.CoalescePointer``,
    used at ``/root/reference/services/supervisor.go:71``)."""
    for v in values:
        if v is not None:
            return v
    return None


__all__ = ["parse_duration", "format_duration", "coalesce"]
