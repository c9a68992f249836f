"""Sanitizer and fuzz coverage for the native code (host code only — GPU sanitizers are
not available on the pool).  The reference has no race/sanitizer testing at all
(CI runs `go test` without `-race`).

* ``nexus-cqlsrv`` built with ``-fsanitize=address`` / ``undefined`` and driven through the
  real client (schema, seed, prepared reads/writes, LWT, WAL restart, malformed frames);
  the test fails on any sanitizer report in the server's stderr.
* random / truncated inputs into the in-process decoders (``_cql_native.FrameReader``,
  ``_kube_native.ProjectedDecoder``) must raise ``ValueError`` — never crash.
* the in-process extensions themselves (``_kube_native``, ``_cql_native`` and the GPU
  monitor over the stub amd-smi) built with ``-fsanitize=address,undefined`` and loaded
  into a child Python with the runtime preloaded (``tools/san_inproc.py``): the fuzzers,
  the native JSON tests, the monitor tests and the reference-parity scenario over HTTP +
  CQL run there; any ASan / UBSan report fails the test.
* the GPU monitor's sampler + event-listener threads under ThreadSanitizer
  (``bin/monitor_selftest-thread`` over the stub amd-smi and a fake procfs), and the
  monitor module itself under TSan in a child Python.
"""
import asyncio
import json
import os
import random
import socket
import struct

import subprocess
import sys

import pytest

from nexus_supervisor_amd import _build
from nexus_supervisor_amd import _cql_native as N
from nexus_supervisor_amd import _kube_native as K
from nexus_supervisor_amd.models import kube
from nexus_supervisor_amd.testing.seed import ALGORITHM, seed_cql_statements, seed_rows

pytestmark = pytest.mark.slow


@pytest.fixture(scope="module", params=["address", "undefined", "thread"])
def sanitized_server(request):
    try:
        _build.build(sanitize=request.param)
    except RuntimeError as exc:  # pragma: no cover - toolchain without the runtime
        pytest.skip(f"sanitizer build unavailable: {exc}")
    exe = os.path.join(_build.BIN, f"nexus-cqlsrv-{request.param}")
    os.environ["NEXUS_CQLSRV_BINARY"] = exe
    yield request.param
    os.environ.pop("NEXUS_CQLSRV_BINARY", None)


def _garbage_frames(port: int, seed: int = 0) -> None:
    rng = random.Random(seed)
    for i in range(60):
        s = socket.create_connection(("127.0.0.1", port), timeout=2)
        try:
            kind = i % 4
            if kind == 0:  # random bytes
                s.sendall(bytes(rng.getrandbits(8) for _ in range(rng.randint(1, 200))))
            elif kind == 1:  # valid header, lying length, truncated body
                body = bytes(rng.getrandbits(8) for _ in range(rng.randint(0, 40)))
                s.sendall(struct.pack(">BBhBI", 4, 0, 1, rng.choice([1, 5, 7, 9, 10, 13, 15]), len(body) + 100) + body)
            elif kind == 2:  # valid frame, garbage body
                body = bytes(rng.getrandbits(8) for _ in range(rng.randint(0, 60)))
                s.sendall(struct.pack(">BBhBI", 4, 0, 1, rng.choice([7, 9, 10, 13]), len(body)) + body)
            else:  # STARTUP then a QUERY with random CQL text
                s.sendall(N.encode_startup(1, {"CQL_VERSION": "3.0.0"}))
                q = "".join(rng.choice("SELECT *FROM nexus.checkpoints WHERE id='x' AND (?,) ;\"") for _ in range(60))
                s.sendall(N.encode_query(2, q, None, None, 1))
            s.settimeout(0.05)
            try:
                s.recv(65536)
            except OSError:
                pass
        finally:
            s.close()


def test_cqlsrv_under_sanitizer(sanitized_server, arun):
    from nexus_supervisor_amd.store.cql import CqlCheckpointStore, CqlError, CqlSession
    from nexus_supervisor_amd.testing.cqlsrv import CqlServer
    import datetime as dt

    # TSan: the shard threads (Scylla emulation) serve concurrent clients on every shard
    shards = 4 if sanitized_server == "thread" else 0
    srv = CqlServer(persist=True, exec_statements=seed_cql_statements(), user="u", password="p",
                    shards=shards).start(timeout=30)
    try:
        async def go():
            st = CqlCheckpointStore(CqlSession([srv.address], user="u", password="p", request_timeout=3.0))
            await st.connect()
            for row in seed_rows():
                assert await st.read_checkpoint(ALGORITHM, row.id) == row
            burst = [r.deep_copy() for r in seed_rows()]
            for i, r in enumerate(burst):
                r.id = f"burst-{i}"
            many = [dict(r=r, i=k) for k in range(40) for r in burst]
            for m in many:
                m["r"] = m["r"].deep_copy()
                m["r"].id = f"{m['r'].id}-{m['i']}"
            await asyncio.gather(*(st.upsert_checkpoint(m["r"]) for m in many))
            got = await asyncio.gather(*(st.read_status(ALGORITHM, m["r"].id) for m in many))
            assert all(g is not None for g in got)
            now = dt.datetime.now(dt.timezone.utc)
            assert await st.update_status(ALGORITHM, seed_rows()[0].id, "FAILED", "c" * 5000, "d☃", now)
            assert not await st.update_status(ALGORITHM, seed_rows()[0].id, "RUNNING", None, None, now,
                                              only_if_stages=["BUFFERED"])
            with pytest.raises(CqlError):
                await st.session.query("SELECT FROM WHERE")
            await st.close()

        arun(go())
        _garbage_frames(srv.port)
        srv.restart(timeout=30)  # WAL replay under the sanitizer
        _garbage_frames(srv.port, seed=1)
    finally:
        srv.stop()
    log = srv.log()
    assert "AddressSanitizer" not in log and "runtime error" not in log and "LeakSanitizer" not in log, log[-3000:]
    assert "ThreadSanitizer" not in log, log[-3000:]


def test_frame_reader_fuzz():
    rng = random.Random(42)
    ok = bad = 0
    for _ in range(3000):
        r = N.FrameReader()
        n = rng.randint(0, 64)
        data = bytes([0x84, 0, 0, 1, rng.choice([0, 2, 3, 6, 8, 0x0C, 0x10, 0x55])]) + struct.pack(">I", n)
        data += bytes(rng.getrandbits(8) for _ in range(n))
        try:
            r.feed(data)
            ok += 1
        except ValueError:
            bad += 1
    assert ok + bad == 3000 and bad > 0


def test_projected_decoder_fuzz():
    rng = random.Random(7)
    d = K.ProjectedDecoder(kube.watch_projection("Pod"))
    base = json.dumps({"type": "ADDED", "object": {"metadata": {"name": "x☃", "labels": {"a": "b"}},
                                                   "status": {"phase": "Running", "containerStatuses": [{"name": "c"}]}}}).encode()
    ok = bad = 0
    for _ in range(5000):
        b = bytearray(base)
        for _ in range(rng.randint(1, 6)):
            op = rng.random()
            i = rng.randrange(len(b))
            if op < 0.4:
                b[i] = rng.getrandbits(8)
            elif op < 0.7:
                del b[i]
            else:
                b.insert(i, rng.choice(b'{}[]",:\\u0'))
        d.reset()
        line = bytes(b).replace(b"\n", b" ") + b"\n"
        try:
            d.feed(line)
            ok += 1
        except ValueError:
            bad += 1
        d.reset()
        try:
            d.feed_events(line, "Pod")  # same bytes through the (type, object) pair builder
        except ValueError:
            pass
    assert ok + bad == 5000 and bad > 0 and ok > 0


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_REPORTS = ("ERROR: AddressSanitizer", "runtime error:", "WARNING: ThreadSanitizer", "ERROR: LeakSanitizer")


def _sanitized(sanitize):
    try:
        _build.build(sanitize=sanitize)
    except RuntimeError as exc:  # pragma: no cover - toolchain without the runtime
        pytest.skip(f"sanitizer build unavailable: {exc}")
    rt = _build.sanitizer_runtime(sanitize)
    if rt is None:  # pragma: no cover
        pytest.skip(f"no {sanitize} runtime library")
    return rt


@pytest.mark.parametrize("sanitize", ["thread", "address"])
def test_gpu_monitor_threads_under_sanitizer(sanitize, tmp_path):
    """Sampler + event listener + every reader of the native monitor, concurrently, over
    the stub amd-smi and a fake procfs in all three process-source modes."""
    from nexus_supervisor_amd.testing.fakeprocfs import FakeProcFs

    _sanitized(sanitize)
    fs = FakeProcFs(str(tmp_path), n_gpus=2)
    fs.add_process(4242, {0: 8 << 30, 1: 1 << 30}, env={"RANK": "1"}, pod_uid="0f3e2b6a-1111-2222-3333-444455556666")
    exe = os.path.join(_build.BIN, f"monitor_selftest-{sanitize}")
    p = subprocess.run([exe, fs.proc, fs.sys, "1.5"], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, TSAN_OPTIONS="halt_on_error=0", ASAN_OPTIONS="detect_leaks=1"))
    out = p.stdout + p.stderr
    assert p.returncode == 0 and not any(r in out for r in _REPORTS), out[-4000:]
    assert out.count("mode=") == 3


@pytest.mark.parametrize("sanitize", ["address", "thread"])
def test_inprocess_extensions_under_sanitizer(sanitize):
    rt = _sanitized(sanitize)
    if sanitize == "address":
        tests = ["tests/test_sanitizers.py::test_frame_reader_fuzz", "tests/test_sanitizers.py::test_projected_decoder_fuzz",
                 "tests/test_native_json.py", "tests/test_gpu_monitor_native.py",
                 "tests/test_kube_wire.py::test_reference_parity_over_http_and_cql", "tests/test_cql.py",
                 "tests/test_workers.py::test_router_forgets_deleted_pods_by_generation",
                 "tests/test_workers.py::test_watch_splitter_routes_lines_and_list_items"]
    else:
        tests = ["tests/test_gpu_monitor_native.py"]
    env = dict(os.environ, NEXUS_NATIVE_DIR=os.path.join(_build.SAN_DIR, sanitize), LD_PRELOAD=rt,
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1",
               TSAN_OPTIONS="halt_on_error=0:report_signal_unsafe=0", PYTHONDONTWRITEBYTECODE="1")
    env.pop("PYTEST_XDIST_WORKER", None)
    # the servers these tests start run uninstrumented (a module-scoped sanitized_server
    # parametrisation may still have its TSan binary selected in this process)
    env.pop("NEXUS_CQLSRV_BINARY", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "san_inproc.py"), *tests], cwd=ROOT,
                       capture_output=True, text=True, timeout=600, env=env)
    out = p.stdout + p.stderr
    assert "instrumented:" in out, out[-3000:]
    assert p.returncode == 0, out[-4000:]
    assert not any(r in out for r in _REPORTS), out[-4000:]


@pytest.mark.parametrize("sanitize", ["thread", "address"])
def test_kubesim_threaded_apply_under_sanitizer(sanitize, arun):
    """``nexus-kubesim`` with apply and fan-out threads: bulk applies of the lifecycle
    workload (lines prepared on threads, kinds committed on threads) while three watches
    stream and Job DELETEs cascade to their pods on another connection (on the GC thread:
    ``--async-gc``, as the bench runs it)."""
    from nexus_supervisor_amd.bench.workload import Workload
    from nexus_supervisor_amd.kube.client import KubeClient, KubeConfig
    from nexus_supervisor_amd.testing.kubesim import KubeSim, SimControl, encode_events

    _sanitized(sanitize)
    os.environ["NEXUS_KUBESIM_BINARY"] = os.path.join(_build.BIN, f"nexus-kubesim-{sanitize}")
    try:
        sim = KubeSim(apply_threads=4, flush_threads=2, history=2_000, async_gc=True).start(timeout=30)  # history overflows: ring pops are buried
    finally:
        os.environ.pop("NEXUS_KUBESIM_BINARY", None)
    try:
        async def go():
            ctl = SimControl(sim.url, sim.apply_url)
            wl = Workload(concurrent_jobs=300, hbm_shape="default-pod")
            objs, _rows = wl.initial()
            await ctl.apply([("ADDED", o) for o in objs])
            rv = str((await ctl.stats())["rv"])
            kc = KubeClient(KubeConfig(sim.url))
            seen = {"Event": 0, "Pod": 0, "Job": 0}

            async def watch(kind):
                async for _t, _o in kc.watch(kind, "nexus", rv, timeout_seconds=30):
                    seen[kind] += 1

            tasks = [asyncio.ensure_future(watch(k)) for k in seen]
            await asyncio.sleep(0.3)
            lines = 0
            for _ in range(8):
                st = wl.step(60)
                body = encode_events([(t, o) for t, o in st.traffic])
                lines += body.count(b"\n")
                await ctl.apply_pipelined([body[:body.index(b"\n", len(body) // 2) + 1],
                                           body[body.index(b"\n", len(body) // 2) + 1:]])
                await asyncio.gather(*(kc.delete_job("nexus", rid) for rid in st.failed))
            for _ in range(200):
                if seen["Event"] and seen["Pod"] and seen["Job"]:
                    break
                await asyncio.sleep(0.05)
            await asyncio.sleep(0.5)
            for t in tasks:
                t.cancel()
            await asyncio.gather(*tasks, return_exceptions=True)
            stats = await ctl.stats()
            await kc.close()
            await ctl.close()
            return seen, lines, stats

        seen, lines, stats = arun(go(), timeout=240)
    finally:
        sim.stop()
    log = sim.log()
    assert not any(r in log for r in _REPORTS), log[-4000:]
    assert all(seen.values()), seen
    assert stats.get("commit_parallel", 0) > 0, stats  # the kinds were committed on threads
    assert stats.get("gc_pods", 0) > 0, stats  # the deleted Jobs' pods went on the GC thread
