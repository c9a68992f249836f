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
