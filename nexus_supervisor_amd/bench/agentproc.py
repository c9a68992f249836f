"""The node agent as its own process for benchmarks and scenarios: ``python -m
nexus_supervisor_amd agent`` against a test apiserver, configured the way the chart's
DaemonSet configures it (``NODE_NAME``, ``NEXUS__*`` settings, metrics port), ready once
its pod informer has listed the node's pods (``/healthz``)."""
from __future__ import annotations

import asyncio
import json
import os
import socket
import subprocess
import sys
import time
from typing import Any, Dict, Optional

from ..utils.proc import die_with_parent


def free_port() -> int:
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def write_kubeconfig(path: str, server: str) -> str:
    with open(path, "w") as f:
        json.dump({"apiVersion": "v1", "kind": "Config", "current-context": "bench",
                   "clusters": [{"name": "bench", "cluster": {"server": server}}],
                   "contexts": [{"name": "bench", "context": {"cluster": "bench", "user": "bench"}}],
                   "users": [{"name": "bench", "user": {}}]}, f)
    return path


class AgentProcess:
    """``start()`` / ``stop()`` one node agent; ``cpu_s()`` its CPU time so far."""

    def __init__(self, api_url: str, workdir: str, node: str, *, namespace: str = "nexus", backend: str = "fake",
                 sample_interval: float = 0.5, kube_qps: float = 50.0, kube_burst: int = 100,
                 log_root: Optional[str] = None, env: Optional[Dict[str, str]] = None):
        self.api_url, self.workdir, self.node, self.namespace = api_url, workdir, node, namespace
        self.backend, self.sample_interval = backend, sample_interval
        self.kube_qps, self.kube_burst = kube_qps, kube_burst
        self.log_root = log_root
        self.extra_env = dict(env or {})
        self.port = 0
        self.proc: Optional[subprocess.Popen] = None
        self.log_path = os.path.join(workdir, f"agent-{node}.log")

    def _env(self) -> Dict[str, str]:
        kcfg = write_kubeconfig(os.path.join(self.workdir, f"agent-{self.node}.kubeconfig"), self.api_url)
        env = dict(os.environ, NODE_NAME=self.node, NEXUS__KUBE_CONFIG_PATH=kcfg,
                   NEXUS__RESOURCE_NAMESPACE=self.namespace, NEXUS__GPU__BACKEND=self.backend,
                   NEXUS__GPU__SAMPLE_INTERVAL=f"{int(round(self.sample_interval * 1000))}ms",
                   NEXUS__KUBE_QPS=str(self.kube_qps), NEXUS__KUBE_BURST=str(int(self.kube_burst)),
                   NEXUS_AGENT_METRICS_PORT=str(self.port))
        if self.log_root:
            env["NEXUS_AGENT_LOG_ROOT"] = self.log_root
        else:
            env["NEXUS__GPU__LOG_TAIL"] = "off"
        # the package this process runs, whatever the caller's working directory
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        env["PYTHONPATH"] = os.pathsep.join(x for x in (root, env.get("PYTHONPATH", "")) if x)
        env.update(self.extra_env)
        return env

    async def start(self, timeout: float = 120.0) -> "AgentProcess":
        import aiohttp

        self.port = free_port()
        logf = open(self.log_path, "wb")
        self.proc = subprocess.Popen([sys.executable, "-m", "nexus_supervisor_amd", "agent"], env=self._env(),
                                     stdout=logf, stderr=subprocess.STDOUT, preexec_fn=die_with_parent())
        logf.close()
        deadline = time.monotonic() + timeout
        async with aiohttp.ClientSession() as http:
            while True:
                if self.proc.poll() is not None:
                    raise RuntimeError(f"node agent exited rc={self.proc.returncode}: {self.log()}")
                try:
                    async with http.get(f"http://127.0.0.1:{self.port}/healthz") as r:
                        if r.status == 200:
                            return self
                except aiohttp.ClientError:
                    pass
                if time.monotonic() > deadline:
                    raise RuntimeError(f"node agent not ready after {timeout:.0f}s: {self.log()}")
                await asyncio.sleep(0.1)

    async def metrics(self) -> Dict[str, float]:
        """The agent's Prometheus counters and gauges, by name (labels summed)."""
        import aiohttp

        out: Dict[str, float] = {}
        async with aiohttp.ClientSession() as http:
            async with http.get(f"http://127.0.0.1:{self.port}/metrics") as r:
                text = await r.text()
        for line in text.splitlines():
            if not line or line.startswith("#"):
                continue
            name, _, val = line.rpartition(" ")
            name = name.split("{", 1)[0]
            try:
                out[name] = out.get(name, 0.0) + float(val)
            except ValueError:
                pass
        return out

    def cpu_s(self) -> float:
        try:
            with open(f"/proc/{self.proc.pid}/stat") as f:
                fields = f.read().rsplit(")", 1)[1].split()
            return (int(fields[11]) + int(fields[12])) / os.sysconf("SC_CLK_TCK")
        except (OSError, IndexError, ValueError, AttributeError):
            return 0.0

    def log(self) -> str:
        try:
            with open(self.log_path, "rb") as f:
                return f.read()[-2000:].decode(errors="replace")
        except OSError:
            return ""

    def stop(self) -> Dict[str, Any]:
        if self.proc is not None and self.proc.poll() is None:
            self.proc.terminate()
            try:
                self.proc.wait(10)
            except subprocess.TimeoutExpired:
                self.proc.kill()
                self.proc.wait(5)
        return {"rc": self.proc.returncode if self.proc else None}
