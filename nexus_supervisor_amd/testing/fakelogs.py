"""A fake kubelet log directory (``/var/log/pods``) for the node agent's log-tail reader.

The container runtime writes one file per container instance,
``<root>/<ns>_<pod>_<uid>/<container>/<restartCount>.log``, each line in the CRI format
``<RFC3339Nano> <stdout|stderr> <P|F> <text>`` (``P``: a partial line continued by the
next record).  :func:`write_cri_log` lays a process's captured output out the same way,
so CPU tests and the GPU-box test (real stderr of a real HIP/torch OOM) read exactly what
a node would hold.
"""
from __future__ import annotations

import datetime as _dt
import os
from typing import Iterable, Optional, Tuple

from ..gpu.logtail import container_log_dir


def _ts(t: Optional[float] = None) -> str:
    d = _dt.datetime.fromtimestamp(t if t is not None else _dt.datetime.now().timestamp(), _dt.timezone.utc)
    return d.strftime("%Y-%m-%dT%H:%M:%S.%f000Z")


def cri_lines(text: str, stream: str = "stderr", split_at: int = 0) -> Iterable[str]:
    """CRI records of ``text`` (``split_at`` > 0: lines longer than that are written as
    ``P`` partials, as runtimes do above their 16 KiB line buffer)."""
    for line in text.splitlines():
        if split_at and len(line) > split_at:
            parts = [line[i:i + split_at] for i in range(0, len(line), split_at)]
            for p in parts[:-1]:
                yield f"{_ts()} {stream} P {p}"
            yield f"{_ts()} {stream} F {parts[-1]}"
        else:
            yield f"{_ts()} {stream} F {line}"


def write_cri_log(root: str, namespace: str, pod: str, uid: str, container: str, restart: int = 0,
                  streams: Iterable[Tuple[str, str]] = (), split_at: int = 0) -> str:
    """Write ``(stream, text)`` chunks as container instance ``restart``'s log; returns the path."""
    d = container_log_dir(root, namespace, pod, uid, container)
    if d is None:
        raise ValueError("namespace / pod / uid / container must be plain path components")
    os.makedirs(d, exist_ok=True)
    path = os.path.join(d, f"{int(restart)}.log")
    with open(path, "a", encoding="utf-8") as f:
        for stream, text in streams:
            for rec in cri_lines(text, stream, split_at):
                f.write(rec + "\n")
    return path
