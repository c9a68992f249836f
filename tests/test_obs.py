"""Observability sinks: DogStatsD over UDP and UDS with the reference's env names
(``DD_DOGSTATSD_URL``, ``DD_SERVICE``, ``DD_VERSION``, ``DD_ENTITY_ID``:
``/root/reference/.helm/templates/deployment.yaml:68-94``), Prometheus text, latency histograms."""
import os
import socket
import tempfile

from nexus_supervisor_amd.obs.histogram import LatencyHistogram
from nexus_supervisor_amd.obs.metrics import DogStatsd, Metrics


def _recv_all(sock):
    out = []
    sock.settimeout(0.5)
    try:
        while True:
            out += sock.recv(65536).decode().split("\n")
    except OSError:
        pass
    return out


def test_dogstatsd_udp_env_tags():
    rx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    rx.bind(("127.0.0.1", 0))
    port = rx.getsockname()[1]
    d = DogStatsd.from_env("nexus_supervisor", env={"DD_DOGSTATSD_URL": f"udp://127.0.0.1:{port}", "DD_SERVICE": "svc",
                                                    "DD_VERSION": "v1", "DD_ENTITY_ID": "uid-1"})
    m = Metrics("nexus_supervisor")
    m.statsd = d
    m.inc("decisions", labels={"action": "ToFailFatalError"})
    m.set("queue_depth", 3)
    m.observe_seconds("event_to_checkpoint", 0.0125)
    d.flush()
    lines = _recv_all(rx)
    assert "nexus_supervisor.decisions:1|c|#service:svc,version:v1,dd.internal.entity_id:uid-1,action:ToFailFatalError" in lines
    assert any(line.startswith("nexus_supervisor.queue_depth:3|g") for line in lines)
    assert any(line.startswith("nexus_supervisor.event_to_checkpoint:12.5|d") for line in lines)
    d.close()
    rx.close()
    assert DogStatsd.from_env("x", env={}) is None


def test_dogstatsd_unix_socket():
    with tempfile.TemporaryDirectory() as tmp:
        path = os.path.join(tmp, "dsd.socket")
        rx = socket.socket(socket.AF_UNIX, socket.SOCK_DGRAM)
        rx.bind(path)
        d = DogStatsd(f"unix://{path}", "nexus_receiver")  # reference namespace kept configurable
        d.count("events_received", 5)
        d.flush()
        assert _recv_all(rx) == ["nexus_receiver.events_received:5|c"]
        d.close()
        rx.close()


def test_prometheus_exposition_and_histogram():
    m = Metrics("nexus_supervisor", {"version": "0.1.0"})
    m.describe("event_to_checkpoint", "latency")
    for ms in range(1, 101):
        m.observe_seconds("event_to_checkpoint", ms / 1000)
    m.inc("decisions", 2, {"action": "ToRunning"})
    text = m.prometheus_text()
    assert "# TYPE nexus_supervisor_decisions_total counter" in text
    assert 'nexus_supervisor_decisions_total{version="0.1.0",action="ToRunning"} 2' in text
    assert 'nexus_supervisor_event_to_checkpoint_seconds_count{version="0.1.0"} 100' in text
    h = m.histogram("event_to_checkpoint")
    assert abs(h.percentile(50) / 1000 - 50) < 2 and abs(h.percentile(99) / 1000 - 99) < 3


def test_histogram_merge_and_bounds():
    a, b = LatencyHistogram(), LatencyHistogram()
    for v in range(1000):
        a.record(v)
        b.record(v * 10)
    a.merge(b)
    s = a.summary()
    assert s["count"] == 2000 and s["max"] >= 9990 * 0.99


# ----------------------------------------------------------------------------- Datadog logs
import gzip  # noqa: E402
import http.server  # noqa: E402
import json  # noqa: E402
import logging  # noqa: E402
import threading  # noqa: E402
import time  # noqa: E402

import pytest  # noqa: E402


class _Intake(http.server.BaseHTTPRequestHandler):
    batches: list = []
    codes: list = []

    def do_POST(self):  # noqa: N802
        body = self.rfile.read(int(self.headers["Content-Length"]))
        code = self.codes.pop(0) if self.codes else 202
        if code == 202:
            assert self.headers["DD-API-KEY"] == "k3y" and self.headers["Content-Encoding"] == "gzip"
            self.batches.append((self.path, json.loads(gzip.decompress(body))))
        self.send_response(code)
        self.send_header("Content-Length", "0")
        self.end_headers()

    def log_message(self, *a):
        pass


@pytest.fixture
def intake():
    _Intake.batches, _Intake.codes = [], []
    srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), _Intake)
    t = threading.Thread(target=srv.serve_forever, daemon=True)
    t.start()
    yield srv, _Intake
    srv.shutdown()


def _env(srv):
    return {"DATADOG__API_KEY": "k3y", "DATADOG__ENDPOINT": f"http://127.0.0.1:{srv.server_address[1]}",
            "DATADOG__APPLICATION_HOST": "node-7", "DATADOG__SERVICE_NAME": "nexus-supervisor", "DD_VERSION": "v9"}


def test_datadog_log_sink_batches_and_retries(intake):
    """Logs fan out to Datadog when DATADOG__* are set (the
    reference's telemetry.ConfigureLogger, main.go:15; deployment.yaml:68-87)."""
    from nexus_supervisor_amd.obs.datadog import DatadogLogHandler, intake_url
    from nexus_supervisor_amd.obs.logging import configure_logging, shutdown_logging

    srv, h = intake
    assert intake_url("datadoghq.eu") == "https://http-intake.logs.datadoghq.eu/api/v2/logs"
    assert DatadogLogHandler.from_env({"DATADOG__API_KEY": "x"}) is None  # all four needed
    h.codes = [503]  # first POST fails: retried
    import io

    log = configure_logging("INFO", stream=io.StringIO(), static={"service": "nexus-supervisor"}, env=_env(srv))
    dd = [x for x in logging.getLogger("nexus_supervisor_amd").handlers if isinstance(x, DatadogLogHandler)][0]
    dd.flush_interval = 0.1
    for i in range(5):
        log.info("Algorithm run failed", requestId=f"r{i}")
    log.v(4).info("not shipped at INFO")
    deadline = time.monotonic() + 5
    while sum(len(b) for _p, b in h.batches) < 5 and time.monotonic() < deadline:
        time.sleep(0.05)
    shutdown_logging()
    entries = [e for _p, b in h.batches for e in b]
    assert len(entries) == 5 and all(p == "/api/v2/logs" for p, _b in h.batches)
    e = entries[0]
    assert e["service"] == "nexus-supervisor" and e["hostname"] == "node-7" and e["status"] == "info"
    assert e["ddtags"] == "version:v9" and json.loads(e["message"])["requestId"] == "r0"
    assert dd.dropped == 0 and dd.sent == 5


def test_datadog_sink_never_blocks_and_drops_on_bad_key(intake):
    from nexus_supervisor_amd.obs.datadog import DatadogLogHandler

    srv, h = intake
    h.codes = [403] * 10
    dd = DatadogLogHandler("bad", f"http://127.0.0.1:{srv.server_address[1]}", "svc", "host", flush_interval=0.05,
                           max_queue=3)
    dd.setFormatter(logging.Formatter("%(message)s"))
    t0 = time.monotonic()
    for i in range(50):  # a full queue drops instead of blocking the caller
        dd.emit(logging.LogRecord("x", logging.INFO, "f", 1, f"m{i}", None, None))
    assert time.monotonic() - t0 < 0.5
    dd.close()
    assert dd.dropped > 0 and dd.sent == 0 and not h.batches


def test_unknown_log_level_fails_start():
    from nexus_supervisor_amd.config import load_config
    from nexus_supervisor_amd.config.schema import ConfigError

    with pytest.raises(ConfigError):
        load_config(path=None, env={"NEXUS__LOG_LEVEL": "LOUD"})
    assert load_config(path=None, env={"NEXUS__LOG_LEVEL": "debug"}).log_level == "debug"


def test_dogstatsd_timer_flush_after_idle(arun):
    """The tail of a burst reaches the agent without a further metric."""
    import asyncio

    rx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    rx.bind(("127.0.0.1", 0))
    d = DogStatsd(f"udp://127.0.0.1:{rx.getsockname()[1]}", flush_interval=0.05)

    async def go():
        d.attach(asyncio.get_running_loop())
        d.count("decisions", 1)  # first emit flushes (interval since construction elapsed?) or buffers
        d.count("decisions", 2)
        await asyncio.sleep(0.2)  # idle: only the timer can flush
        d.close()

    d._last_flush = time.monotonic()  # start inside the interval so the emits buffer
    arun(go())
    lines = [x for x in _recv_all(rx) if x]
    assert "nexus_supervisor.decisions:2|c" in lines


def test_buildmeta_stamp(tmp_path):
    import importlib.util

    from nexus_supervisor_amd import buildmeta

    p = buildmeta.write("v1.4.2", "20261016120000", str(tmp_path / "_bi.py"))
    spec = importlib.util.spec_from_file_location("_bi", p)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    assert mod.APP_VERSION == "1.4.2" and mod.BUILD_NUMBER == "20261016120000"
    with pytest.raises(ValueError):
        buildmeta.write("latest", "1", str(tmp_path / "x.py"))
    import nexus_supervisor_amd as pkg

    assert pkg.__version__ == buildmeta.APP_VERSION and pkg.__build__ == buildmeta.BUILD_NUMBER


def test_buffered_log_handler_flushes_on_timer_warning_and_shutdown():
    """V(0) decision lines are not flushed one syscall each: they reach the stream within
    the flush interval, at once for WARNING and above, and on shutdown."""
    import io
    import time

    from nexus_supervisor_amd.obs.logging import BufferedStreamHandler, configure_logging, shutdown_logging

    raw = io.BytesIO()
    stream = io.TextIOWrapper(io.BufferedWriter(raw, buffer_size=1 << 16), encoding="utf-8")
    log = configure_logging("INFO", stream=stream)
    log.info("Algorithm run failed", requestId="r1")
    assert raw.getvalue() == b""  # buffered
    time.sleep(0.5)
    assert b'"requestId":"r1"' in raw.getvalue()  # timer flush
    log.info("second")
    log.warning("loud")
    assert b"loud" in raw.getvalue() and b"second" in raw.getvalue()
    log.info("last")
    shutdown_logging()
    assert b"last" in raw.getvalue()
    assert isinstance(BufferedStreamHandler(io.StringIO()), BufferedStreamHandler)


def test_native_histogram_matches_python():
    """``_kube_native.LatencyHist`` (the record path in C) keeps exactly the Python
    histogram's buckets and statistics, and merges across both."""
    import random

    import pytest

    from nexus_supervisor_amd.obs import histogram as H

    if H._NativeHist is None:
        pytest.skip("native extension not built")
    rng = random.Random(3)
    py, nat = H.PyLatencyHistogram(), H.NativeLatencyHistogram()
    vals = [rng.choice([-5.0, 0.0, 0.4, 127.9, 128.0]) for _ in range(50)] + \
        [rng.lognormvariate(6, 3) for _ in range(20000)] + [2.0 ** 45, 1e30]
    for v in vals:
        py.record(v)
        nat.record(v)
    nat.record(7, 3)
    py.record(7, 3)
    assert nat.counts == py.counts and nat.sparse() == py.sparse()
    assert (nat.total, nat.sum, nat.min, nat.max) == (py.total, py.sum, py.min, py.max)
    assert nat.summary() == py.summary() and nat.buckets() == py.buckets()
    both = H.NativeLatencyHistogram()
    both.merge(nat)
    both.merge(py)
    ref = H.PyLatencyHistogram()
    ref.merge(py)
    ref.merge(py)
    assert both.counts == ref.counts and (both.total, both.sum, both.min, both.max) == (ref.total, ref.sum, ref.min, ref.max)
    both.reset()
    assert both.total == 0 and both.min is None and both.percentile(99) == 0.0


def test_buffered_log_handler_flushes_late_without_a_thread_per_window(arun):
    """Lines are flushed within the interval — by a loop timer on an event loop, by one
    long-lived flusher thread elsewhere — and no thread is started per flush window (a
    threading.Timer per window cost ~130 µs of thread start-up per decision at 1000
    failures/min)."""
    import asyncio
    import io
    import logging
    import threading
    import time as _t

    from nexus_supervisor_amd.obs.logging import BufferedStreamHandler, JsonFormatter

    class Stream(io.StringIO):
        flushed = 0

        def flush(self):
            Stream.flushed += 1

    s = Stream()
    h = BufferedStreamHandler(s, interval=0.05)
    h.setFormatter(JsonFormatter())
    lg = logging.getLogger("test_buffered_handler")
    lg.propagate = False
    lg.addHandler(h)
    lg.setLevel(logging.INFO)
    try:
        before = threading.active_count()
        for _ in range(3):  # off-loop: one flusher thread, reused
            lg.info("x")
            _t.sleep(0.12)
        assert Stream.flushed >= 3 and threading.active_count() <= before + 1

        async def on_loop():
            n0, threads = Stream.flushed, threading.active_count()
            for _ in range(3):
                lg.info("y")
                await asyncio.sleep(0.12)
            assert Stream.flushed >= n0 + 3 and threading.active_count() == threads

        arun(on_loop())
        assert s.getvalue().count("\n") == 6
    finally:
        lg.removeHandler(h)
        h.close()


def test_direct_log_path_writes_the_record_paths_line():
    """KLogger's direct path (one BufferedStreamHandler, no filters: the deployed setup)
    writes the same JSON line the LogRecord path does; a filter or a second handler puts
    every line back on the record path."""
    import io
    import json as _json
    import logging as _logging

    from nexus_supervisor_amd.obs.logging import configure_logging, shutdown_logging

    def lines(extra_handler):
        buf = io.StringIO()
        log = configure_logging("DEBUG", stream=buf, static={"service": "s"})
        root = _logging.getLogger("nexus_supervisor_amd")
        if extra_handler:
            root.addHandler(_logging.NullHandler())
        log.info("Algorithm run failed", requestId="r1", reason="OOMKilled")
        log.v(4).info("event received", object="ns/e")
        root.handlers[0].flush()
        shutdown_logging()
        out = [_json.loads(x) for x in buf.getvalue().splitlines()]
        for d in out:
            d.pop("time")
        return out

    direct, via_record = lines(False), lines(True)
    assert direct == via_record
    assert direct[0] == {"level": "INFO", "logger": "nexus_supervisor_amd", "msg": "Algorithm run failed",
                         "requestId": "r1", "reason": "OOMKilled", "service": "s"}
    assert direct[1]["v"] == 4
