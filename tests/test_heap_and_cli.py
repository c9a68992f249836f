"""``/debug/heap`` helpers (``obs/heap.py``) directly, the ``shadow-report`` CLI entry and the
compiled-module build step."""
import json
import os
import tracemalloc

import pytest

from nexus_supervisor_amd.obs import heap


class _Idx:
    def __init__(self, items):
        self._items = items


class _Inf:
    def __init__(self, items):
        self.indexer = _Idx(items)


class _Factory:
    def __init__(self, items):
        self.informers = {"Pod": _Inf(items)}


class _Sup:
    def __init__(self, items):
        self.factory = _Factory(items)


def test_census_with_tracemalloc_growth_and_trim():
    tracemalloc.start(4)
    try:
        first = heap.census(None, top=5, trim=True)
        keep = [{"kind": "Pod", "metadata": {"name": f"p{i}"}} for i in range(2000)]  # noqa: F841 - grows
        second = heap.census(None, top=5)
    finally:
        tracemalloc.stop()
        heap._LAST = None
    assert first["gc_objects"] > 0 and len(first["types"]) <= 5
    assert "rss_before_trim_mb" in first and "tracemalloc_mb" in first
    assert second["tracemalloc_growth"] and "stack" in second["tracemalloc_growth"][0]
    assert isinstance(heap.malloc_trim(), bool)


def test_retainers_finds_what_holds_a_deleted_object():
    cached = {"ns/a": {"kind": "Pod", "metadata": {"name": "a"}}}
    holder = {"leak": [{"kind": "Pod", "metadata": {"name": "gone", "resourceVersion": "7"}}]}
    out = heap.retainers(_Sup(cached), "Pod", samples=5)
    assert out[0]["stray"] >= 1
    gone = [r for r in out[1:] if r["name"] == "gone"]
    assert gone and gone[0]["rv"] == "7" and gone[0]["chain"]
    assert any("list[1]" in c for lvl in gone[0]["chain"] for c in lvl)
    del holder
    assert heap._desc({"b": 1, "a": 2}) == "dict{a,b}" and heap._desc((1, 2)) == "tuple[2]"


def test_shadow_report_cli(tmp_path, capsys, monkeypatch):
    from nexus_supervisor_amd import shadow

    assert shadow.main([]) == 2
    log = tmp_path / "shadow.log"
    log.write_text(json.dumps({"msg": "dry run: would write", "algorithm": "alg", "requestId": "r1",
                               "stage": "FAILED", "class": "host-oom"}) + "\n")
    monkeypatch.setenv("NEXUS__CQL_STORE_TYPE", "memory")
    assert shadow.main([str(log)]) == 0
    doc = json.loads(capsys.readouterr().out)
    assert isinstance(doc, dict)


def test_compile_one_module_into_a_scratch_dir(tmp_path, monkeypatch):
    pytest.importorskip("Cython")
    from nexus_supervisor_amd import _build, compiled

    monkeypatch.setattr(compiled, "DIR", str(tmp_path))
    name = "nexus_supervisor_amd.obs.delivery"
    assert _build._compile_module(name) == f"compiled {name}"
    assert compiled.fresh(name) and os.path.exists(compiled.extension_path(name))
    assert _build._compile_module(name) is None  # fresh: nothing to do
    assert [p for p in os.listdir(tmp_path) if ".tmp" in p] == []  # no leftovers
