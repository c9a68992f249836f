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
