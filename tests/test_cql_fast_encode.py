"""``encode_execute_fast`` (the scalar EXECUTE encoder of every decision's read and write)
produces the same frame bytes as the general ``encode_execute``, and declines — returns
NotImplemented, so the session falls back — for anything outside its scalar set."""
import datetime as dt

import pytest

N = pytest.importorskip("nexus_supervisor_amd._cql_native")

QID = bytes(range(16))
NOW = dt.datetime(2026, 10, 17, 6, 30, 1, 250000, tzinfo=dt.timezone.utc)

CASES = [
    # the owned-columns write: stage, cause, a 2 KB trace with non-ASCII text, timestamp, key
    (["FAILED", "Algorithm encountered a fatal error", "trace ✓ " + "x" * 2000, NOW, "algo", "id-1"],
     [0x0D, 0x0D, 0x0D, 0x0B, 0x0D, 0x0D]),
    (["algo", "id-1"], [0x0D, 0x0D]),  # the status read
    ([None, 5, -7, 2.5, True, False, b"\x00\x01", 1_700_000_000_123, 12.5, 3], [0x0D, 0x09, 0x02, 0x07, 0x04, 0x04, 0x03, 0x0B, 0x0B, 0x12]),
    ([b"raw-bytes-as-text", "ascii"], [0x0D, 0x01]),
    ([], []),
]


@pytest.mark.parametrize("values,types", CASES)
@pytest.mark.parametrize("skip,serial", [(True, None), (False, 9)])
def test_fast_matches_general(values, types, skip, serial):
    slow = N.encode_execute(17, QID, values, types, 6, skip, -1, None, serial, None)
    fast = N.encode_execute_fast(17, QID, values, bytes(types), 6, skip, serial)
    assert fast == slow


@pytest.mark.parametrize("values,types", [
    ([object()], [0x0D]),        # not str / bytes
    (["x"], [0x20]),             # a collection type
    ([2 ** 40], [0x09]),         # out of int range
    (["1"], [0x09]),             # str for an int column
    (["a", "b"], [0x0D]),        # arity mismatch
])
def test_fast_declines(values, types):
    assert N.encode_execute_fast(1, QID, values, bytes(types), 1, True, None) is NotImplemented


def test_prepared_codes_only_for_scalar_statements():
    from nexus_supervisor_amd.store.cql import PreparedStatement

    ps = PreparedStatement("q", QID, [0x0D, 0x0B], [0], None, None)
    assert ps.codes == b"\x0d\x0b"
    assert PreparedStatement("q", QID, [0x0D, (0x20, 0x0D)], [0], None, None).codes is None
