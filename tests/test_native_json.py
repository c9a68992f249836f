"""Native compact JSON encoder (``csrc/kube/json_encode.cpp``) against the json module:
property test over arbitrary JSON documents, sort_keys, default=, errors."""
import json
import math

import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

K = pytest.importorskip("nexus_supervisor_amd._kube_native")

scalars = st.none() | st.booleans() | st.integers(min_value=-(2 ** 70), max_value=2 ** 70) | \
    st.floats(allow_nan=False, allow_infinity=False) | st.text(max_size=20)
docs = st.recursive(scalars, lambda c: st.lists(c, max_size=5) | st.dictionaries(st.text(max_size=8), c, max_size=5),
                    max_leaves=40)


@settings(max_examples=300, deadline=None)
@given(docs)
def test_roundtrip_matches_json(doc):
    out = K.dumps(doc)
    assert json.loads(out) == json.loads(json.dumps(doc))
    assert out == json.dumps(doc, separators=(",", ":"), ensure_ascii=False).encode()


@settings(max_examples=200, deadline=None)
@given(st.dictionaries(st.text(max_size=8), scalars, max_size=8))
def test_sort_keys_matches_json(doc):
    assert K.dumps(doc, sort_keys=True) == json.dumps(doc, sort_keys=True, separators=(",", ":"),
                                                      ensure_ascii=False).encode()


def test_specials_default_and_errors():
    assert K.dumps({"a": (1, 2)}, newline=True) == b'{"a":[1,2]}\n'
    assert K.dumps([math.nan, math.inf, -math.inf]) == b"[NaN,Infinity,-Infinity]"
    assert K.dumps({1: "x", None: 2, False: 3}) == b'{"1":"x","null":2,"false":3}'
    assert K.dumps({"s": {1, 2}}, default=sorted) == b'{"s":[1,2]}'
    with pytest.raises(TypeError):
        K.dumps({"s": object()})
    a = []
    a.append(a)
    with pytest.raises(ValueError):
        K.dumps(a)
    assert K.dumps("\x01 é") == json.dumps("\x01 é", ensure_ascii=False).encode()


def test_deleted_watch_events_decode_identity_only():
    """DELETED envelopes project "object" to identity + labels (Events keep involvedObject
    for the shard filter); other types, and envelopes with "object" first, keep the full
    projection."""
    import json as _json

    from nexus_supervisor_amd import _kube_native as K
    from nexus_supervisor_amd.models import kube

    pod = {"kind": "Pod", "apiVersion": "v1",
           "metadata": {"name": "p", "namespace": "ns", "uid": "u", "resourceVersion": "5", "labels": {"a": "b"},
                        "annotations": {"x": "y"}},
           "spec": {"nodeName": "n", "containers": [{"name": "c", "env": [{"name": "X", "value": "1"}]}]},
           "status": {"phase": "Failed"}}
    d = K.ProjectedDecoder(kube.watch_projection("Pod"))
    (full,) = d.feed((_json.dumps({"type": "MODIFIED", "object": pod}) + "\n").encode())
    (gone,) = d.feed((_json.dumps({"type": "DELETED", "object": pod}) + "\n").encode())
    assert full["object"]["spec"]["nodeName"] == "n" and full["object"]["status"]["phase"] == "Failed"
    assert gone["type"] == "DELETED" and set(gone["object"]) == {"kind", "apiVersion", "metadata"}
    assert gone["object"]["metadata"] == {"name": "p", "namespace": "ns", "uid": "u", "resourceVersion": "5",
                                          "labels": {"a": "b"}}
    (late,) = d.feed((_json.dumps({"object": pod, "type": "DELETED"}) + "\n").encode())
    assert late["object"]["spec"]["nodeName"] == "n"  # type after object: cannot know, keep all
    ev = {"kind": "Event", "metadata": {"name": "e", "namespace": "ns", "resourceVersion": "7"},
          "involvedObject": {"kind": "Job", "name": "j"}, "reason": "BackoffLimitExceeded", "count": 3,
          "source": {"component": "job-controller"}}
    (ge,) = K.ProjectedDecoder(kube.watch_projection("Event")).feed((_json.dumps({"type": "DELETED", "object": ev}) + "\n").encode())
    assert ge["object"]["involvedObject"] == {"kind": "Job", "name": "j"}
    assert "source" not in ge["object"] and "count" not in ge["object"]


def test_kv_env_projection_keeps_what_topology_reads():
    """Pods decode their container env into a filtered {name: value} dict; every variable
    gpu/topology.py reads must survive it (models/kube.py ENV_KEEP / ENV_PREFIXES)."""
    import json as _json

    from nexus_supervisor_amd.gpu import topology as T
    from nexus_supervisor_amd.models import kube as KM
    from nexus_supervisor_amd.models.kube import watch_projection

    read = {v for v, _k in T._INT_VARS} | set(T.RANK_VARS) | set(T.DEVICE_VARS) | {"MASTER_ADDR"}
    assert read <= set(KM.ENV_KEEP)
    assert T.COLLECTIVE_PREFIXES == KM.ENV_PREFIXES
    env = [{"name": "RANK", "value": "3"}, {"name": "PATH", "value": "/bin"}, {"name": "NCCL_DEBUG", "value": "INFO"},
           {"name": "RANK", "value": "9"}, {"name": "SECRET", "valueFrom": {"secretKeyRef": {"name": "s"}}},
           {"name": "HIP_VISIBLE_DEVICES", "value": "4,5,6,7"}, {"name": "MASTER_ADDR", "value": "h\\u00e9st"}]
    pod = {"kind": "Pod", "metadata": {"name": "p", "resourceVersion": "1"},
           "spec": {"containers": [{"name": "a", "env": env}, {"name": "b", "env": [{"name": "LOCAL_RANK", "value": "1"},
                                                                                    {"name": "RANK", "value": "7"}]}]}}
    line = (_json.dumps({"type": "ADDED", "object": pod}) + "\n").encode()
    out = K.ProjectedDecoder(watch_projection("Pod")).feed(line)[0]["object"]
    c0 = out["spec"]["containers"][0]["env"]
    assert c0 == {"RANK": "3", "NCCL_DEBUG": "INFO", "HIP_VISIBLE_DEVICES": "4,5,6,7", "MASTER_ADDR": "h\\u00e9st"}
    merged = KM.pod_env(out)
    assert merged["RANK"] == "3" and merged["LOCAL_RANK"] == "1" and "PATH" not in merged
    # the same pod in API shape folds to the same topology
    raw = _json.loads(line)["object"]
    t1 = T.topology_from_env(KM.pod_env(out), 1, "")
    t2 = T.topology_from_env({k: v for k, v in KM.pod_env(raw).items()}, 1, "")
    assert t1 == t2 and t1["visible_devices"] == ["4", "5", "6", "7"] and t1["rank"] == 3


def test_raw_json_splice_and_trace_equivalence():
    from nexus_supervisor_amd.classify.classifier import RawJSON, _json_default

    inner = {"links": [{"gpu": 0, "peer": 1}], "fully_connected": True}
    raw = RawJSON(K.dumps(inner))
    doc = {"a": 1, "topology": {"xgmi": raw}, "b": b"plain"}
    out = K.dumps(doc, default=str)
    back = json.loads(out)
    assert back["topology"]["xgmi"] == inner and back["b"] == "b'plain'"
    assert json.loads(json.dumps(doc, default=_json_default)) == back


def test_feed_events_matches_python_envelope_unpacking():
    """``feed_events(bytes, kind)`` = ``[(ev.get("type", ""), ev.get("object") or {})]`` with the
    object's missing / null kind set to ``kind`` (the hub feed's batched informer path)."""
    import json as _json

    from nexus_supervisor_amd import _kube_native as K
    from nexus_supervisor_amd.models import kube

    lines = [{"type": "ADDED", "object": {"metadata": {"name": "a", "namespace": "ns"}}},
             {"type": "MODIFIED", "object": {"kind": "Pod", "metadata": {"name": "b"}}},
             {"type": "DELETED", "object": {"kind": None, "metadata": {"name": "c"}}},
             {"type": "BOOKMARK", "object": {}},
             {"object": {"metadata": {"name": "d"}}},
             {"type": "ERROR"}]
    data = b"".join((_json.dumps(x) + "\n").encode() for x in lines)
    proj = kube.watch_projection("Pod")
    want = []
    for ev in K.ProjectedDecoder(proj).feed(data):
        obj = ev.get("object") or {}
        if obj.get("kind") is None:
            obj["kind"] = "Pod"
        want.append((ev.get("type", ""), obj))
    d = K.ProjectedDecoder(proj)
    got = d.feed_events(data[:37], "Pod") + d.feed_events(data[37:], "Pod")  # split mid-line
    assert got == want
    assert [t for t, _ in got] == ["ADDED", "MODIFIED", "DELETED", "BOOKMARK", "", "ERROR"]
    assert all(o["kind"] == "Pod" for _, o in got)
    with pytest.raises(ValueError):
        K.ProjectedDecoder(True).feed_events(b"[1, 2]\n", "Pod")


def test_numbers_and_strings_match_json_module_exactly():
    """The fast paths (std::to_chars for ints and for floats in Python repr's fixed range,
    an 8-byte clean-run scan for strings) produce the json module's exact bytes."""
    import json
    import random
    import struct

    from nexus_supervisor_amd._kube_native import dumps

    rng = random.Random(11)
    floats = [0.0, -0.0, 1.0, -1.0, 0.5, 1e-4, 9.999e-5, 1e16, 9999999999999998.0, 1792219597.431, 0.1, 1 / 3,
              5e-324, 1.7976931348623157e308]
    while len(floats) < 20000:
        v = struct.unpack("d", struct.pack("Q", rng.getrandbits(64)))[0] if rng.random() < 0.5 else \
            rng.uniform(-1e17, 1e17) * 10 ** rng.randint(-25, 0)
        if v == v and abs(v) != float("inf"):
            floats.append(v)
    ints = [0, -1, 2 ** 63 - 1, -2 ** 63, 2 ** 64, 10 ** 30] + [rng.randint(-10 ** 18, 10 ** 18) for _ in range(2000)]
    alphabet = [chr(c) for c in range(128)] + ["é", "☃", "𝄞"]
    strs = ["".join(rng.choice(alphabet) for _ in range(rng.randint(0, 40))) for _ in range(3000)]
    for doc in ([floats], [ints], [strs], {s: i for s, i in zip(strs, ints)}):
        assert dumps(doc).decode() == json.dumps(doc, separators=(",", ":"), ensure_ascii=False)
