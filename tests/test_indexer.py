"""Informer cache (client-go ``cache.Indexer`` equivalent): the single-label fast path keeps
exactly the index the generic path keeps, over random add / relabel / status-update / delete
sequences."""
import random

from hypothesis import given, settings
from hypothesis import strategies as st

from nexus_supervisor_amd.informer.store import Indexer, label_index

LABEL = "job-name"


def _generic(label):
    fn = label_index(label)

    def plain(obj):  # same function without the fast-path marker
        return fn(obj)

    return plain


def _pod(name, job, rv, ns="ns"):
    labels = {"app": "x"}
    if job is not None:
        labels[LABEL] = job
    return {"metadata": {"name": name, "namespace": ns, "resourceVersion": str(rv), "labels": labels},
            "status": {"phase": random.choice(["Pending", "Running", "Failed"])}}


def _snapshot(ix):
    return {v: set(ks) for v, ks in ix._indices["job"].items()}


ops = st.lists(st.tuples(st.sampled_from(["upsert", "delete"]), st.integers(0, 7),
                         st.one_of(st.none(), st.sampled_from(["j0", "j1", "j2"]))), max_size=80)


@settings(max_examples=200, deadline=None)
@given(ops)
def test_label_fast_path_matches_generic_index(seq):
    fast = Indexer({"job": label_index(LABEL)})
    slow = Indexer({"job": _generic(LABEL)})
    assert fast._labels is not None and slow._labels is None
    for rv, (op, i, job) in enumerate(seq):
        name = f"p{i}"
        if op == "upsert":
            a = fast.upsert(_pod(name, job, rv))
            b = slow.upsert(_pod(name, job, rv))
            assert (a is None) == (b is None)
        else:
            assert (fast.delete(f"ns/{name}") is None) == (slow.delete(f"ns/{name}") is None)
        assert _snapshot(fast) == _snapshot(slow)
        assert all(ks for ks in fast._indices["job"].values())  # no empty buckets left behind
    for job in ("j0", "j1", "j2"):
        got = sorted(o["metadata"]["name"] for o in fast.by_index("job", job))
        assert got == sorted(o["metadata"]["name"] for o in slow.by_index("job", job))


def test_status_update_leaves_index_bucket_untouched():
    ix = Indexer({"job": label_index(LABEL)})
    ix.upsert(_pod("a", "j", 1))
    bucket = ix._indices["job"]["j"]
    ix.upsert(_pod("a", "j", 2))
    assert ix._indices["job"]["j"] is bucket and bucket == {"ns/a"}
    ix.upsert(_pod("a", "k", 3))  # relabelled: moves buckets
    assert "j" not in ix._indices["job"] and ix._indices["job"]["k"] == {"ns/a"}
    ix.add_indexer("other", lambda o: ())  # a non-label indexer turns the fast path off
    assert ix._labels is None
    ix.upsert(_pod("b", "k", 4))
    assert ix._indices["job"]["k"] == {"ns/a", "ns/b"}
