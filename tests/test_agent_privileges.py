"""The node agent as deployed: it must run as root, and when it does not, every refused
read is counted and logged instead of silently degrading attribution.

A non-root UID gets no effective capabilities even in a ``privileged: true`` container,
so it is refused other users' ``/proc/<pid>/fd`` / ``fdinfo`` / ``environ`` (the
per-process VRAM and rank env of the supervised job), root-owned 0640 container logs
under ``/var/log/pods`` and the root-only kubelet pod-resources socket.  The reference has
no node agent; its one Deployment runs as ``nonroot``
(``/root/reference/.container/Dockerfile:45``), which is right for the supervisor and is
kept for it here.
"""
import json
import os
import socket
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deploy"))

from render import render_docs  # noqa: E402

from nexus_supervisor_amd.gpu import logtail  # noqa: E402
from nexus_supervisor_amd.gpu.agent import NodeAgent, process_privileges  # noqa: E402
from nexus_supervisor_amd.gpu.podresources import PodResourcesClient  # noqa: E402
from nexus_supervisor_amd.gpu.telemetry import FakeTelemetry  # noqa: E402

CHART = os.path.join(ROOT, "deploy", "helm", "nexus-supervisor-amd")
NOBODY = 65532
FDINFO = ("pos:\t0\nflags:\t02100002\nmnt_id:\t25\ndrm-driver:\tamdgpu\ndrm-pdev:\t0000:05:00.0\n"
          "drm-client-id:\t7\ndrm-memory-vram:\t104857600 KiB\ndrm-memory-gtt:\t2048 KiB\n")


def test_chart_runs_the_agent_as_root_and_the_supervisor_not():
    docs = render_docs(CHART)
    ds = [d for d in docs if d["kind"] == "DaemonSet"][0]
    c = ds["spec"]["template"]["spec"]["containers"][0]
    sc = c["securityContext"]
    assert sc["runAsUser"] == 0 and sc["runAsGroup"] == 0 and sc["runAsNonRoot"] is False and sc["privileged"] is True
    env = {e["name"]: e.get("value") for e in c["env"]}
    assert env["NEXUS_AGENT_METRICS_PORT"] == "9102" and c["ports"][0]["containerPort"] == 9102
    dep = [d for d in docs if d["kind"] == "Deployment"][0]
    dsc = dep["spec"]["template"]["spec"]["containers"][0]["securityContext"]
    assert dsc["runAsNonRoot"] is True and dsc["runAsUser"] == NOBODY and dsc["capabilities"] == {"drop": ["ALL"]}


def test_process_privileges_reads_capeff(tmp_path):
    st = tmp_path / "status"
    st.write_text("Name:\tpython\nCapEff:\t0000000000000000\n")
    p = process_privileges(str(st))
    assert not p["sufficient"] and set(p["missing"]) == {"CAP_SYS_PTRACE", "CAP_DAC_READ_SEARCH"}
    st.write_text("CapEff:\t000001ffffffffff\n")  # every capability (root in a privileged container)
    assert process_privileges(str(st))["sufficient"]
    st.write_text(f"CapEff:\t{(1 << 19) | (1 << 2):016x}\n")  # ptrace + dac_read_search
    assert process_privileges(str(st))["sufficient"]


def _fixtures(tmp_path):
    """A root-owned fake /proc (one PID whose fd table is 0700, one whose fdinfo is 0600)
    and a kubelet log tree with a 0640 container log, as a node holds them."""
    proc = tmp_path / "proc"
    for pid, fd_mode, info_mode in ((4101, 0o700, 0o644), (4102, 0o755, 0o600)):
        base = proc / str(pid)
        (base / "fd").mkdir(parents=True)
        (base / "fdinfo").mkdir()
        os.symlink("/dev/dri/renderD128", base / "fd" / "5")
        (base / "fdinfo" / "5").write_text(FDINFO)
        (base / "stat").write_text(f"{pid} (python) S 1 1 1 0 -1 0 0 0 0 0 0 0 0 0 20 0 1 0 777 0 0\n")
        os.chmod(base / "fdinfo" / "5", info_mode)
        os.chmod(base / "fd", fd_mode)
    logs = tmp_path / "pods"
    d = logs / "nexus_run-w0_uid-1" / "algorithm"
    d.mkdir(parents=True)
    f = d / "0.log"
    f.write_text("2026-01-01T00:00:00Z stderr F torch.OutOfMemoryError: HIP out of memory. GPU 0 has a total "
                 "capacity of 287.98 GiB\n")
    os.chmod(f, 0o640)
    for p in (tmp_path, proc, logs, logs / "nexus_run-w0_uid-1", d):
        os.chmod(p, 0o755)
    pod = {"metadata": {"name": "run-w0", "namespace": "nexus", "uid": "uid-1"},
           "status": {"phase": "Failed", "containerStatuses": [{"name": "algorithm", "restartCount": 0, "state": {
               "terminated": {"reason": "Error", "exitCode": 1, "message": ""}}}]}}
    return str(proc), str(logs), pod


class _NullFactory:
    def informer(self, kind, **kw):
        return None


class _NativeTel(FakeTelemetry):
    """Fake GPU backend whose denial counters are the native monitor's (procscan.hpp)."""

    def __init__(self, mod):
        super().__init__(n_gpus=1)
        self.mod = mod

    def denials(self):
        return dict(self.mod.denials())


def _scan_and_read(proc, logs, pod, sock):
    from nexus_supervisor_amd import _amdsmi_monitor_stub as mod

    mod.reset_denials()
    uses = mod.DrmScanner(proc, 1).scan()
    agent = NodeAgent(None, _NativeTel(mod), "n", "nexus", factory=_NullFactory(), log_root=logs,
                      pod_resources=PodResourcesClient(sock))
    agent.privileges = process_privileges()
    recs = agent.log_evidence(pod)
    if agent.podres.check() == "denied":
        agent._denied("podresources")
    agent.check_denials()
    counters = {k: {",".join(f"{a}={b}" for a, b in sorted(lab)): v for lab, v in vals.items()}
                for k, vals in agent.metrics.counters.items()}
    return {"uses": uses, "recs": recs, "counters": counters, "privileges": agent.privileges,
            "denials": dict(mod.denials())}


@pytest.mark.skipif(os.geteuid() != 0, reason="needs root to build root-owned fixtures and drop to another uid")
def test_non_root_agent_reports_denials_root_agent_attributes():
    import pathlib
    import shutil
    import tempfile

    # not pytest's tmp_path: its parents are 0700, the dropped child could not reach it
    tmp_path = pathlib.Path(tempfile.mkdtemp(prefix="nexus-agent-priv-"))
    try:
        _non_root_vs_root(tmp_path)
    finally:
        shutil.rmtree(tmp_path, ignore_errors=True)


def _non_root_vs_root(tmp_path):
    proc, logs, pod = _fixtures(tmp_path)
    sock_path = str(tmp_path / "kubelet.sock")
    srv = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    srv.bind(sock_path)
    srv.listen(4)
    os.chmod(sock_path, 0o600)  # the kubelet's pod-resources socket: root only
    try:
        # root: everything readable, the HIP OOM text and the pod's VRAM are attributed
        root = _scan_and_read(proc, logs, pod, sock_path)
        assert {u["pid"] for u in root["uses"]} == {4101, 4102}
        assert all(u["bdf"] == "0000:05:00.0" and u["vram_bytes"] == 100 << 30 for u in root["uses"])
        assert root["recs"][0]["match"] == "hbm" and not root["recs"][0].get("denied")
        assert not any(root["denials"].values()) and "agent_proc_scan_denied" not in root["counters"]
        assert root["privileges"]["sufficient"]
        # the same agent code as uid 65532 (the image's default user) in a forked child
        r, w = os.pipe()
        pid = os.fork()
        if pid == 0:  # pragma: no cover - child
            try:
                os.close(r)
                os.setgroups([])
                os.setgid(NOBODY)
                os.setuid(NOBODY)
                out = _scan_and_read(proc, logs, pod, sock_path)
                os.write(w, json.dumps(out, default=str).encode())
            finally:
                os._exit(0)
        os.close(w)
        data = b""
        while True:
            chunk = os.read(r, 65536)
            if not chunk:
                break
            data += chunk
        os.close(r)
        os.waitpid(pid, 0)
        child = json.loads(data)
    finally:
        srv.close()
    assert child["uses"] == []  # nothing attributed ...
    assert child["denials"]["fd"] >= 1 and child["denials"]["fdinfo"] >= 1  # ... and it says why
    c = child["counters"]
    assert c["agent_proc_scan_denied"]["source=fd"] >= 1 and c["agent_proc_scan_denied"]["source=fdinfo"] >= 1
    assert c["agent_log_read_denied"][""] == 1 and child["recs"][0]["denied"] is True
    assert c["agent_podresources_denied"][""] == 1
    assert not child["privileges"]["sufficient"] and child["privileges"]["euid"] == NOBODY
    assert "CAP_SYS_PTRACE" in child["privileges"]["missing"]


def test_log_reader_marks_unreadable_directory(tmp_path):
    d = tmp_path / "nexus_run-w0_uid-1"
    d.mkdir()
    pod = {"metadata": {"name": "run-w0", "namespace": "nexus", "uid": "uid-1"},
           "status": {"phase": "Failed", "containerStatuses": [{"name": "algorithm", "restartCount": 0, "state": {
               "terminated": {"reason": "Error", "exitCode": 1, "message": ""}}}]}}
    recs = logtail.node_log_evidence(str(tmp_path), pod)
    assert recs[0]["error"] == "no log file" and not recs[0].get("denied")
