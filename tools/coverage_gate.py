#!/usr/bin/env python3
"""Line-coverage gate for the CPU test suite (reference ``.testcoverage.yml:1-19``:
file 70 / package 70 / total 75, with excluded paths).

``coverage.py`` is not part of this image, so this is a small self-contained
tracer: executable lines come from the compiled code objects of every module
under ``nexus_supervisor_amd/`` (``co_lines``), executed lines from a
``sys.settrace``/``threading.settrace`` hook that only instruments frames of
those files.  pytest runs in-process; package child processes (``python -m
nexus_supervisor_amd …``: shard workers) trace themselves when ``NEXUS_COVERAGE_DIR``
is set (``nexus_supervisor_amd/utils/covtrace.py``) and their lines are merged.

    python tools/coverage_gate.py [--config .testcoverage.yml] [--report FILE] [-- pytest args]

Exit status 0 when every threshold holds, 1 otherwise (2 when the tests fail).
"""
from __future__ import annotations

import argparse
import json
import os
import re
import sys
import threading
from collections import defaultdict
from types import CodeType
from typing import Dict, Iterable, List, Set

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "nexus_supervisor_amd")


def _code_lines(code: CodeType, out: Set[int]) -> None:
    for _s, _e, line in code.co_lines():
        if line is not None:
            out.add(line)
    for c in code.co_consts:
        if isinstance(c, CodeType):
            _code_lines(c, out)


_PRAGMA = re.compile(r"#\s*pragma:\s*no\s*cover")


def executable_lines(path: str) -> Set[int]:
    with open(path, encoding="utf-8") as f:
        src = f.read()
    lines: Set[int] = set()
    _code_lines(compile(src, path, "exec"), lines)
    text = src.splitlines()
    # module docstrings / bare string constants are "executed" at import; drop the
    # explicitly excluded lines
    return {n for n in lines if n <= len(text) and not _PRAGMA.search(text[n - 1])}


class Tracer:
    def __init__(self, files: Iterable[str]):
        self.files = set(files)
        self.hits: Dict[str, Set[int]] = defaultdict(set)

    def _global(self, frame, event, arg):
        fn = frame.f_code.co_filename
        if fn not in self.files:
            return None
        hits = self.hits[fn]
        hits.add(frame.f_lineno)

        def local(frame, event, arg):
            if event == "line":
                hits.add(frame.f_lineno)
            return local

        return local

    def start(self) -> None:
        threading.settrace(self._global)
        sys.settrace(self._global)

    def stop(self) -> None:
        sys.settrace(None)
        threading.settrace(None)


def load_config(path: str) -> dict:
    import yaml

    with open(path) as f:
        return yaml.load(f, Loader=yaml.SafeLoader) or {}


def main(argv: List[str] = None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    pytest_args = ["tests", "-q", "-x", "-m", "not gpu", "-p", "no:cacheprovider"]
    if "--" in argv:
        i = argv.index("--")
        pytest_args = argv[i + 1:]
        argv = argv[:i]
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default=os.path.join(ROOT, ".testcoverage.yml"))
    ap.add_argument("--report", default="")
    args = ap.parse_args(argv)
    cfg = load_config(args.config)
    th = cfg.get("threshold", {})
    excludes = [re.compile(p) for p in (cfg.get("exclude", {}) or {}).get("paths", [])]

    files = {}
    for d, _dirs, names in os.walk(PKG):
        for n in names:
            if n.endswith(".py"):
                p = os.path.join(d, n)
                rel = os.path.relpath(p, ROOT)
                if any(e.search(rel) for e in excludes):
                    continue
                files[p] = rel

    tracer = Tracer(files)
    import tempfile

    child_dir = tempfile.mkdtemp(prefix="nexus-cov-")
    os.environ["NEXUS_COVERAGE_DIR"] = child_dir
    # line tracing slows everything 3-10x: the lease-timing tests scale their clocks
    os.environ.setdefault("NEXUS_TEST_TIME_SCALE", "3")
    os.chdir(ROOT)
    sys.path.insert(0, ROOT)
    import pytest

    tracer.start()
    try:
        rc = pytest.main(pytest_args)
    finally:
        tracer.stop()

    real = {os.path.realpath(p): p for p in files}
    for name in os.listdir(child_dir):
        try:
            with open(os.path.join(child_dir, name)) as f:
                doc = json.load(f)
        except (OSError, ValueError):
            continue
        for fn, lines in doc.items():
            p = real.get(os.path.realpath(fn))
            if p is not None:
                tracer.hits[p].update(lines)

    per_file = {}
    missing: Dict[str, List[int]] = {}
    per_pkg: Dict[str, List[int]] = defaultdict(lambda: [0, 0])
    tot_hit = tot_all = 0
    for p, rel in sorted(files.items(), key=lambda kv: kv[1]):
        lines = executable_lines(p)
        if not lines:
            continue
        got = lines & tracer.hits.get(p, set())
        hit = len(got)
        missing[rel] = sorted(lines - got)
        per_file[rel] = (hit, len(lines))
        pk = per_pkg[os.path.dirname(rel)]
        pk[0] += hit
        pk[1] += len(lines)
        tot_hit += hit
        tot_all += len(lines)

    pct = lambda h, n: 100.0 * h / n if n else 100.0  # noqa: E731
    fails = []
    print(f"\n{'file':60s} {'lines':>6s} {'cover':>7s}")
    for rel, (h, n) in per_file.items():
        flag = ""
        if pct(h, n) < th.get("file", 0):
            flag = "  < file threshold"
            fails.append(f"file {rel}: {pct(h, n):.1f}%")
        print(f"{rel:60s} {n:6d} {pct(h, n):6.1f}%{flag}")
    print()
    for pk, (h, n) in sorted(per_pkg.items()):
        if pct(h, n) < th.get("package", 0):
            fails.append(f"package {pk}: {pct(h, n):.1f}%")
        print(f"package {pk:52s} {n:6d} {pct(h, n):6.1f}%")
    total = pct(tot_hit, tot_all)
    print(f"\ntotal {tot_all} lines, {total:.1f}% covered "
          f"(thresholds: file {th.get('file', 0)}, package {th.get('package', 0)}, total {th.get('total', 0)})")
    if total < th.get("total", 0):
        fails.append(f"total: {total:.1f}%")
    if args.report:
        with open(args.report, "w") as f:
            json.dump({"total": round(total, 2), "thresholds": th,
                       "packages": {k: round(pct(*v), 2) for k, v in per_pkg.items()},
                       "files": {k: round(pct(*v), 2) for k, v in per_file.items()}, "failures": fails,
                       "missing_lines": missing}, f, indent=1)
    if rc != 0:
        print(f"tests failed (pytest exit {rc})")
        return 2
    for f_ in fails:
        print("BELOW THRESHOLD:", f_)
    return 1 if fails else 0


if __name__ == "__main__":
    sys.exit(main())
