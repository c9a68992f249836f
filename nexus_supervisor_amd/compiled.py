"""Hot-path modules compiled to C extensions (Cython, pure-Python mode), loaded only when
they were built from the source that is on disk.

Per pod failure a shard worker spends most of its CPU in CPython bytecode spread thin
over dict-heavy helpers — object accessors, the classifier, OOM scoring, topology, the
actuator, the CQL and HTTP clients (``profiles/r3_cpu_ab/``: no single function over a
few percent).  Compiling those modules as they are removes the interpreter's dispatch
from all of them at once.  MI355X box, interleaved (``profiles/r4_compiled_ab/``): the
socket-free hot path 60–65 µs per failure against 83–84 µs, the driver-like bench 38.3k
failures/s at 120 µs of replica CPU per failure against 33.3k at 157 µs.  Nothing about
them changes: the ``.py`` file stays the source of truth, the compiled module behaves the
same (the whole test suite runs against it; Cython's annotation typing is off, so
annotations stay hints), and a tree without the build, or with a module edited since,
simply imports the ``.py``.

* :data:`MODULES` — what is compiled (``python -m nexus_supervisor_amd._build --only
  compiled``; ``__graft_entry__.build()`` builds it too).  Each extension lands in
  ``_compiled/<module>.<ext>`` with ``<module>.sha256``, the hash of the source it was
  built from.
* :func:`install` (called by the package's ``__init__``) puts a finder at the front of
  ``sys.meta_path`` that serves a listed module from its extension when that hash matches
  the ``.py`` on disk, else lets the normal import take it.
* ``NEXUS_PURE_PYTHON=1`` (or a coverage run: ``NEXUS_COVERAGE_DIR``) imports the sources
  only — line coverage, ``/debug/pprof`` frames and debuggers see Python code.

:func:`loaded` names the modules running compiled in this process (the bench line's
``config.compiled_modules`` counts the replica parent's).
"""
from __future__ import annotations

import hashlib
import importlib.abc
import importlib.machinery
import importlib.util
import os
import sys
from typing import Dict, List, Optional

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
DIR = os.path.join(PKG_DIR, "_compiled")
EXT = importlib.machinery.EXTENSION_SUFFIXES[0]

MODULES = (
    "nexus_supervisor_amd.models.kube",
    "nexus_supervisor_amd.models.decisions",
    "nexus_supervisor_amd.models.checkpoint",
    "nexus_supervisor_amd.classify.classifier",
    "nexus_supervisor_amd.classify.reference_rules",
    "nexus_supervisor_amd.gpu.oom",
    "nexus_supervisor_amd.gpu.topology",
    "nexus_supervisor_amd.gpu.logtail",
    "nexus_supervisor_amd.gpu.telemetry",
    "nexus_supervisor_amd.gpu.collective",
    "nexus_supervisor_amd.obs.metrics",
    "nexus_supervisor_amd.obs.delivery",
    "nexus_supervisor_amd.obs.logging",
    "nexus_supervisor_amd.supervisor",
    "nexus_supervisor_amd.parallel.pipeline",
    "nexus_supervisor_amd.parallel.ratelimit",
    "nexus_supervisor_amd.parallel.breaker",
    "nexus_supervisor_amd.parallel.watchhub",
    "nexus_supervisor_amd.informer.informer",
    "nexus_supervisor_amd.informer.store",
    "nexus_supervisor_amd.store.cql",
    "nexus_supervisor_amd.kube.client",
    "nexus_supervisor_amd.kube.fasthttp",
    "nexus_supervisor_amd.kube.flowcontrol",
    "nexus_supervisor_amd.kube.errors",
    "nexus_supervisor_amd.store.base",
    "nexus_supervisor_amd.parallel.sharding",
    "nexus_supervisor_amd.parallel.workers",
)

_LOADED: List[str] = []


def source_path(name: str) -> str:
    """The ``.py`` of a listed module."""
    rel = name.split(".", 1)[1].replace(".", os.sep) + ".py"
    return os.path.join(PKG_DIR, rel)


def extension_path(name: str) -> str:
    return os.path.join(DIR, name + EXT)


def hash_path(name: str) -> str:
    return os.path.join(DIR, name + ".sha256")


def source_hash(path: str) -> str:
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def fresh(name: str) -> bool:
    """Was this module's extension built from the source on disk?"""
    so, sha = extension_path(name), hash_path(name)
    if not (os.path.exists(so) and os.path.exists(sha)):
        return False
    try:
        with open(sha) as f:
            return f.read().strip() == source_hash(source_path(name))
    except OSError:
        return False


def disabled() -> bool:
    return bool(os.environ.get("NEXUS_PURE_PYTHON") or os.environ.get("NEXUS_COVERAGE_DIR"))


class _Finder(importlib.abc.MetaPathFinder):
    def __init__(self):
        self.names = frozenset(MODULES)
        self.checked: Dict[str, bool] = {}

    def find_spec(self, fullname, path=None, target=None):
        if fullname not in self.names:
            return None
        ok = self.checked.get(fullname)
        if ok is None:
            ok = self.checked[fullname] = fresh(fullname)
        if not ok:
            return None  # not built, or the source changed since: the .py
        so = extension_path(fullname)
        spec = importlib.util.spec_from_file_location(
            fullname, so, loader=importlib.machinery.ExtensionFileLoader(fullname, so))
        if fullname not in _LOADED:
            _LOADED.append(fullname)
        return spec


_FINDER: Optional[_Finder] = None


def install() -> bool:
    """Serve the listed modules compiled when they are fresh (no-op when disabled)."""
    global _FINDER
    if _FINDER is not None or disabled():
        return False
    _FINDER = _Finder()
    sys.meta_path.insert(0, _FINDER)
    return True


def loaded() -> List[str]:
    """The listed modules this process imported compiled."""
    return [n for n in _LOADED if n in sys.modules]
