"""Compiled hot-path modules (``nexus_supervisor_amd/compiled.py``): served from
``_compiled/`` only when built from the source on disk; a stale or missing build, or
``NEXUS_PURE_PYTHON=1``, imports the ``.py``."""
import os
import subprocess
import sys

import pytest

from nexus_supervisor_amd import compiled

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _built() -> bool:
    return all(compiled.fresh(n) for n in compiled.MODULES)


def _probe(env_extra):
    code = ("import nexus_supervisor_amd.supervisor as s, nexus_supervisor_amd.compiled as c; "
            "print(s.__file__); print(len(c.loaded()))")
    env = {k: v for k, v in os.environ.items() if k not in ("NEXUS_COVERAGE_DIR", "NEXUS_PURE_PYTHON")}
    env.update(env_extra)
    out = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    path, n = out.stdout.split()
    return path, int(n)


def test_every_listed_module_exists_and_imports():
    for name in compiled.MODULES:
        assert os.path.exists(compiled.source_path(name)), name
        __import__(name)


@pytest.mark.skipif(not _built(), reason="compiled modules not built (python -m nexus_supervisor_amd._build)")
def test_fresh_build_is_loaded_and_pure_python_opt_out():
    path, n = _probe({})
    assert path.endswith(compiled.EXT) and n >= 1
    path, n = _probe({"NEXUS_PURE_PYTHON": "1"})
    assert path.endswith("supervisor.py") and n == 0


def test_a_stale_build_is_never_loaded(tmp_path, monkeypatch):
    """An extension whose recorded source hash differs from the .py on disk (the module was
    edited after the build) is skipped: the edit runs, not the old machine code."""
    name = "nexus_supervisor_amd.gpu.oom"
    monkeypatch.setattr(compiled, "DIR", str(tmp_path))
    so = compiled.extension_path(name)
    with open(so, "wb") as f:
        f.write(b"not an extension")
    with open(compiled.hash_path(name), "w") as f:
        f.write("0" * 64 + "\n")
    assert not compiled.fresh(name)
    finder = compiled._Finder()
    assert finder.find_spec(name) is None
    with open(compiled.hash_path(name), "w") as f:
        f.write(compiled.source_hash(compiled.source_path(name)) + "\n")
    assert compiled.fresh(name)
    spec = compiled._Finder().find_spec(name)
    assert spec is not None and spec.origin == so
    assert compiled._Finder().find_spec("nexus_supervisor_amd.app") is None  # not listed


def test_coverage_runs_import_the_sources(monkeypatch):
    monkeypatch.setenv("NEXUS_COVERAGE_DIR", "/tmp/x")
    assert compiled.disabled()
    monkeypatch.delenv("NEXUS_COVERAGE_DIR")
    monkeypatch.setenv("NEXUS_PURE_PYTHON", "1")
    assert compiled.disabled()
