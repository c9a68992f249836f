"""Native informer apply (``_kube_native.apply_lines``, csrc/kube/informer_apply.cpp) against
the Python loop it replaces (``SharedInformer._apply_lines``, ``NEXUS_PY_INFORMER_APPLY=1``):
the same cache, the same label index, the same handler calls in the same order, the same
resourceVersion bookkeeping, an ERROR line stopping the batch, handler exceptions logged
and swallowed."""
import pytest

from nexus_supervisor_amd import _kube_native
from nexus_supervisor_amd.informer import informer as I
from nexus_supervisor_amd.informer.store import Indexer, label_index

LABEL = "batch.kubernetes.io/job-name"


def _pod(name, rv, job=None, ns="nexus"):
    md = {"name": name, "namespace": ns, "resourceVersion": str(rv)}
    if job is not None:
        md["labels"] = {LABEL: job}
    return {"kind": "Pod", "metadata": md}


def _batch():
    return [("ADDED", _pod("a", 1, "j1")), ("ADDED", _pod("b", 2, "j1")), ("BOOKMARK", {"metadata": {"resourceVersion": "3"}}),
            ("MODIFIED", _pod("a", 4, "j2")), ("MODIFIED", _pod("b", 5, None)), ("DELETED", _pod("a", 6)),
            ("ADDED", _pod("c", 7, "j3", ns="")), ("DELETED", _pod("zz", 8)), ("ADDED", _pod("boom", 9, "j9")),
            ("ERROR", {"kind": "Status", "code": 410}), ("ADDED", _pod("never", 11, "jx"))]


def _run(native, monkeypatch):
    monkeypatch.setattr(I, "_NATIVE_APPLY", [(_kube_native.apply_lines if native else None)])
    inf = I.SharedInformer.__new__(I.SharedInformer)
    inf.kind, inf.watch_events, inf._rv, inf.stamp = "Pod", 0, "", lambda: 0.0
    ix = Indexer()
    ix.add_indexer("job-name", label_index(LABEL))
    inf.indexer = ix
    calls = []

    def add(o):
        calls.append(("add", o["metadata"]["name"]))
        if o["metadata"]["name"] == "boom":
            raise RuntimeError("handler bug")

    inf.handlers = [I.Handler(on_add=add, on_update=lambda o, n: calls.append(("upd", o["metadata"]["resourceVersion"],
                                                                                n["metadata"]["resourceVersion"])),
                              on_delete=lambda o: calls.append(("del", o["metadata"]["name"], o["metadata"]["resourceVersion"])))]
    err = inf._apply_lines(_batch(), 0, 64)
    return err, calls, dict(ix._items), {k: {v: set(s) for v, s in d.items()} for k, d in ix._indices.items()}, \
        inf._rv, inf.watch_events


def test_native_apply_matches_python(monkeypatch):
    py = _run(False, monkeypatch)
    nat = _run(True, monkeypatch)
    assert nat == py
    err, calls, items, indices, rv, seen = nat
    assert err == {"kind": "Status", "code": 410}
    assert ("add", "boom") in calls and ("add", "never") not in calls  # an ERROR stops the batch
    assert calls[3] == ("upd", "2", "5") and calls[4] == ("del", "a", "4")  # deletes see the cached version
    assert set(items) == {"nexus/b", "c", "nexus/boom"} and indices == {"job-name": {"j3": {"c"}, "j9": {"nexus/boom"}}}
    assert rv == "9" and seen == 9


def test_native_apply_rejects_bad_input():
    with pytest.raises(TypeError):
        _kube_native.apply_lines([("ADDED",)], 0, 1, {}, None, {}, [], [], [], print, "Pod")
