"""Process entry (C1 / N1-N3: ``/root/reference/main.go:12-43``): signal-driven shutdown
with drain, ``NEXUS__`` env config, JSON klog-style logging, and the ``python -m
nexus_supervisor_amd supervisor`` process against a real HTTP apiserver and the
native CQL server."""
import asyncio
import io
import json
import os
import signal
import socket
import subprocess
import sys
import threading
import time
import urllib.request

from nexus_supervisor_amd import app as app_mod
from nexus_supervisor_amd.config import load_config
from nexus_supervisor_amd.models import LifecycleStage as S
from nexus_supervisor_amd.obs.logging import configure_logging
from nexus_supervisor_amd.store.cql import CqlCheckpointStore, CqlSession
from nexus_supervisor_amd.testing.cqlsrv import CqlServer
from nexus_supervisor_amd.testing.fake_apiserver import FakeApiServer
from nexus_supervisor_amd.testing.seed import ALGORITHM, make_job, make_pod, seed_cql_statements, seed_rows
from nexus_supervisor_amd.utils import coalesce

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RUNNING_ROW = seed_rows()[1]


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _kubeconfig(path, url, token=""):
    user = f"{{token: {token}}}" if token else "{}"
    with open(path, "w") as f:
        f.write(f"""apiVersion: v1
kind: Config
current-context: t
clusters: [{{name: c, cluster: {{server: "{url}"}}}}]
contexts: [{{name: t, context: {{cluster: c, user: u, namespace: nexus}}}}]
users: [{{name: u, user: {user}}}]
""")


def _get(url, timeout=1.0):
    try:
        with urllib.request.urlopen(url, timeout=timeout) as r:
            return r.status, r.read().decode()
    except Exception:  # noqa: BLE001
        return 0, ""


def _wait_ready(port, deadline_s=30.0):
    deadline = time.monotonic() + deadline_s
    while time.monotonic() < deadline:
        if _get(f"http://127.0.0.1:{port}/readyz")[0] == 200:
            return True
        time.sleep(0.05)
    return False


def test_json_logging_levels_and_static_tags():
    buf = io.StringIO()
    log = configure_logging("DEBUG", stream=buf, static={"service": "nexus-supervisor"})
    log.info("decision", requestId="r1", algorithm="a")
    log.v(4).info("event received", reason="Failed")
    log.v(9).info("too verbose")
    try:
        raise RuntimeError("boom")
    except RuntimeError as exc:
        log.error(exc, "write failed", requestId="r2")
    log.warning("slow")
    lines = [json.loads(x) for x in buf.getvalue().splitlines()]
    assert [x["msg"] for x in lines] == ["decision", "event received", "write failed", "slow"]
    assert lines[0]["requestId"] == "r1" and lines[0]["service"] == "nexus-supervisor" and lines[0]["level"] == "INFO"
    assert lines[1]["v"] == 4 and lines[2]["err"] == "boom" and lines[2]["level"] == "ERROR"
    assert log.v(4).enabled and not log.v(5).enabled and log.enabled(4)
    quiet = configure_logging("ERROR", stream=io.StringIO())
    assert not quiet.v(1).enabled
    assert coalesce(None, 0, 3) == 0 and coalesce(None, None) is None


def test_main_sigterm_drains_and_exits_zero(monkeypatch, tmp_path):
    """``app.main()`` in-process: env config, ready probe, SIGTERM → drain → exit 0."""
    api = FakeApiServer()
    loop = asyncio.new_event_loop()
    started = threading.Event()
    box = {}

    def serve():
        asyncio.set_event_loop(loop)
        box["url"] = loop.run_until_complete(api.start())
        started.set()
        loop.run_forever()

    th = threading.Thread(target=serve, daemon=True)
    th.start()
    assert started.wait(10)
    labels = load_config(path=None, env={}).labels
    loop.call_soon_threadsafe(api.create, make_pod(RUNNING_ROW.id, labels))
    kc = tmp_path / "kubeconfig"
    _kubeconfig(kc, box["url"])
    obs = _free_port()
    for k, v in {"NEXUS__CQL_STORE_TYPE": "memory", "NEXUS__KUBE_CONFIG_PATH": str(kc),
                 "NEXUS__OBSERVABILITY__HTTP_PORT": str(obs), "NEXUS__OBSERVABILITY__HTTP_HOST": "127.0.0.1",
                 "NEXUS__LOG_LEVEL": "DEBUG", "NEXUS__RESYNC_PERIOD": "0s", "NEXUS_CONFIG_DIR": str(tmp_path)}.items():
        monkeypatch.setenv(k, v)
    seen = {}

    def driver():
        seen["ready"] = _wait_ready(obs)
        upd = make_pod(RUNNING_ROW.id, labels, rv="9")
        upd["status"] = {"phase": "Failed", "containerStatuses": [
            {"name": "algorithm", "state": {"terminated": {"reason": "OOMKilled", "exitCode": 137}}}]}
        loop.call_soon_threadsafe(lambda: api.update(upd))
        deadline = time.monotonic() + 10
        while time.monotonic() < deadline:
            code, text = _get(f"http://127.0.0.1:{obs}/metrics")
            if "decisions_missing_checkpoint" in text:  # memory store: no row → skipped
                seen["metrics"] = text
                break
            time.sleep(0.05)
        os.kill(os.getpid(), signal.SIGTERM)

    d = threading.Thread(target=driver, daemon=True)
    d.start()
    try:
        rc = app_mod.main([])
    finally:
        d.join(15)
        asyncio.run_coroutine_threadsafe(api.stop(), loop).result(10)
        loop.call_soon_threadsafe(loop.stop)
        th.join(5)
        loop.close()
    assert rc == 0 and seen.get("ready") and "metrics" in seen


def test_main_fatal_init_exits_one(monkeypatch, tmp_path):
    """Unloadable kube config → logged fatal error, exit 1 (``klog.FlushAndExit(…, 1)``)."""
    monkeypatch.setenv("NEXUS__CQL_STORE_TYPE", "memory")
    monkeypatch.setenv("NEXUS__KUBE_CONFIG_PATH", str(tmp_path / "missing"))
    monkeypatch.setenv("NEXUS_CONFIG_DIR", str(tmp_path))
    monkeypatch.delenv("KUBERNETES_SERVICE_HOST", raising=False)
    assert app_mod.main([]) == 1


def test_supervisor_process_end_to_end(arun, tmp_path):
    """``python -m nexus_supervisor_amd supervisor`` as a real process: HTTP watch in,
    CQL write out, SIGTERM → graceful exit 0."""
    srv = CqlServer(exec_statements=seed_cql_statements()).start()
    obs = _free_port()

    async def go():
        api = FakeApiServer(token="tok")
        url = await api.start()
        labels = load_config(path=None, env={}).labels
        api.create(make_pod(RUNNING_ROW.id, labels))
        api.create(make_job(RUNNING_ROW.id, labels))
        kc = tmp_path / "kubeconfig"
        _kubeconfig(kc, url, token="tok")
        env = dict(os.environ, NEXUS__CQL_STORE_TYPE="scylla", NEXUS__SCYLLA_CQL_STORE__HOSTS=f"127.0.0.1:{srv.port}",
                   NEXUS__KUBE_CONFIG_PATH=str(kc), NEXUS__OBSERVABILITY__HTTP_PORT=str(obs),
                   NEXUS__OBSERVABILITY__HTTP_HOST="127.0.0.1", NEXUS__WORKERS="4", NEXUS_CONFIG_DIR=str(tmp_path),
                   PYTHONPATH=ROOT)
        proc = subprocess.Popen([sys.executable, "-m", "nexus_supervisor_amd", "supervisor"], env=env, cwd=str(tmp_path),
                                stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
        store = CqlCheckpointStore(CqlSession([srv.address]))
        try:
            loop = asyncio.get_running_loop()
            assert await loop.run_in_executor(None, _wait_ready, obs, 60.0), "supervisor never became ready"
            upd = make_pod(RUNNING_ROW.id, labels, rv="9")
            upd["status"] = {"phase": "Failed", "containerStatuses": [
                {"name": "algorithm", "state": {"terminated": {"reason": "OOMKilled", "exitCode": 137}}}]}
            api.update(upd)
            await store.connect()
            row = None
            for _ in range(200):
                row = await store.read_checkpoint(ALGORITHM, RUNNING_ROW.id)
                if row is not None and row.lifecycle_stage == S.FAILED and api.get("Job", "nexus", RUNNING_ROW.id) is None:
                    break
                await asyncio.sleep(0.05)
            assert row is not None and row.lifecycle_stage == S.FAILED
            assert "OOMKilled" in row.algorithm_failure_cause
            assert ("Job", "nexus", RUNNING_ROW.id, "Background") in api.deleted
            proc.send_signal(signal.SIGTERM)
            rc = await loop.run_in_executor(None, proc.wait, 20)
            out = proc.stdout.read().decode()
            assert rc == 0, out[-2000:]
            logs = [json.loads(x) for x in out.splitlines() if x.startswith("{")]
            msgs = [x["msg"] for x in logs]
            assert "Starting Nexus Supervisor" in msgs and any("draining" in m for m in msgs)
        finally:
            if proc.poll() is None:
                proc.kill()
                proc.wait(5)
            await store.close()
            await api.stop()

    try:
        arun(go(), timeout=120)
    finally:
        srv.stop()


def test_gc_tuner_freezes_after_sync_and_restores(arun):
    import gc

    from nexus_supervisor_amd.obs.metrics import Metrics
    from nexus_supervisor_amd.utils.gctune import GcTuner

    saved = gc.get_threshold()
    cache = [{"metadata": {"name": f"r{i}"}} for i in range(1000)]  # long-lived, acyclic

    async def go():
        m = Metrics("t")
        t = GcTuner(thresholds=(12345, 11, 7), refreeze_interval=0.01, metrics=m)
        t.after_sync()
        assert gc.get_threshold() == (12345, 11, 7) and gc.get_freeze_count() >= len(cache)
        await asyncio.sleep(0.05)
        assert t.freezes >= 2 and m.gauge("gc_frozen_objects") > 0
        t.stop()
        assert gc.get_freeze_count() == 0 and gc.get_threshold() == saved

    arun(go())
    cfg = load_config(path=None, env={"NEXUS__RUNTIME__GC_THRESHOLD0": "5000", "NEXUS__RUNTIME__GC_FREEZE": "false"})
    t = GcTuner.from_config(cfg.runtime)
    assert t.thresholds[0] == 5000 and not t.freeze_enabled
    del cache
