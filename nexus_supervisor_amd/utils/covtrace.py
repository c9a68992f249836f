"""Line coverage of child processes for the coverage gate (``tools/coverage_gate.py``).

The gate traces the pytest process itself; shard workers (``python -m
nexus_supervisor_amd worker``) and other package entry points run in processes of
their own.  With ``NEXUS_COVERAGE_DIR`` set, :func:`install_from_env` traces every
frame of this package in the current process and writes the executed lines to
``<dir>/cov-<pid>.json`` at exit; the gate merges those files.  Off (a single env
lookup) otherwise.
"""
from __future__ import annotations

import atexit
import json
import os
import sys
import threading
from typing import Dict, Set

ENV = "NEXUS_COVERAGE_DIR"


def install_from_env() -> bool:
    out_dir = os.environ.get(ENV)
    if not out_dir:
        return False
    pkg = os.path.dirname(os.path.dirname(os.path.realpath(__file__))) + os.sep
    hits: Dict[str, Set[int]] = {}

    def trace(frame, event, arg):
        fn = frame.f_code.co_filename
        if not fn.startswith(pkg):
            return None
        lines = hits.get(fn)
        if lines is None:
            lines = hits[fn] = set()
        lines.add(frame.f_lineno)

        def local(frame, event, arg):
            if event == "line":
                lines.add(frame.f_lineno)
            return local

        return local

    def dump() -> None:
        sys.settrace(None)
        path = os.path.join(out_dir, f"cov-{os.getpid()}.json")
        try:
            with open(path, "w") as f:
                json.dump({k: sorted(v) for k, v in hits.items()}, f)
        except OSError:
            pass

    threading.settrace(trace)
    sys.settrace(trace)
    atexit.register(dump)
    return True
