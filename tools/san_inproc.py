"""Run native-extension tests in a process whose in-process extensions are the
sanitizer builds (``build/san/<sanitizer>/``, via ``NEXUS_NATIVE_DIR``) with the
sanitizer runtime LD_PRELOADed; tests/test_sanitizers.py drives it and fails on any
sanitizer report.  Refuses to run if the instrumented modules are not the ones loaded.

    NEXUS_NATIVE_DIR=build/san/address LD_PRELOAD=$(g++ -print-file-name=libasan.so) \
        python tools/san_inproc.py <pytest args>
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    d = os.environ.get("NEXUS_NATIVE_DIR")
    assert d, "NEXUS_NATIVE_DIR must name the instrumented build"
    from nexus_supervisor_amd import _cql_native, _kube_native  # noqa: F401

    mods = [_cql_native, _kube_native]
    try:
        from nexus_supervisor_amd import _amdsmi_monitor_stub

        mods.append(_amdsmi_monitor_stub)
    except ImportError:
        pass
    for m in mods:
        assert os.path.realpath(m.__file__).startswith(os.path.realpath(d)), (m.__name__, m.__file__)
    print("instrumented:", ", ".join(os.path.basename(m.__file__) for m in mods), flush=True)
    import pytest

    return pytest.main(["-q", "-p", "no:cacheprovider", "-p", "no:xdist", *sys.argv[1:]])


if __name__ == "__main__":
    sys.exit(main())
