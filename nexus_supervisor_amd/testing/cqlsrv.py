"""Process wrapper for the native CQL server (``csrc/cqlsrv`` → ``bin/nexus-cqlsrv``).

Stands in for the reference's docker-compose Scylla + ``prepare-scylla.sh``
(``/root/reference/docker-compose.yaml:4-29``): start on an ephemeral port, seed
with the checkpoint schema + rows, and inject faults (latency, Overloaded errors,
dropped connections, kill/restart with the write-ahead log).
"""
from __future__ import annotations

import os
import signal
import subprocess
import tempfile
import time
from typing import List, Optional, Sequence

from ..utils.proc import die_with_parent


class CqlServer:
    def __init__(self, *, user: str = "", password: str = "", latency_us: int = 0, error_rate: float = 0.0,
                 persist: bool = False, tokens: Sequence[int] = (), peers: Sequence[str] = (), exec_statements: Sequence[str] = (),
                 dc: str = "datacenter1", host: str = "127.0.0.1", port: int = 0, extra_args: Sequence[str] = (),
                 shards: int = 0, shard_aware_port: int = 0, lwt_latency_us: int = -1):
        from .._build import binary

        # NEXUS_CQLSRV_BINARY selects e.g. a sanitizer build (bin/nexus-cqlsrv-address)
        self.exe = os.environ.get("NEXUS_CQLSRV_BINARY") or binary("nexus-cqlsrv")
        self.dir = tempfile.mkdtemp(prefix="nexus-cqlsrv-")
        self.host = host
        self.port = port
        self.user, self.password = user, password
        self.latency_us, self.error_rate = latency_us, error_rate
        self.lwt_latency_us = lwt_latency_us  # extra for a conditional write (Paxos); -1 = server default 3 x latency
        self.data = os.path.join(self.dir, "wal.bin") if persist else ""
        self.tokens = [str(t) for t in tokens]
        self.peers = list(peers)
        self.dc = dc
        self.extra = list(extra_args)
        # Scylla shard emulation: shard threads + SCYLLA_* SUPPORTED keys + shard-aware port
        self.shards = shards
        self.shard_aware_port = shard_aware_port
        self.exec_file = ""
        if exec_statements:
            self.exec_file = os.path.join(self.dir, "init.cql")
            with open(self.exec_file, "w") as f:
                for s in exec_statements:
                    f.write(s.rstrip().rstrip(";") + ";\n")
        self.proc: Optional[subprocess.Popen] = None
        self.log_path = os.path.join(self.dir, "server.log")

    def _argv(self) -> List[str]:
        ready = os.path.join(self.dir, "ready")
        argv = [self.exe, "--host", self.host, "--port", str(self.port), "--ready-file", ready, "--dc", self.dc]
        if self.user:
            argv += ["--user", self.user, "--password", self.password]
        if self.latency_us:
            argv += ["--latency-us", str(self.latency_us)]
        if self.lwt_latency_us >= 0:
            argv += ["--lwt-latency-us", str(self.lwt_latency_us)]
        if self.error_rate:
            argv += ["--error-rate", str(self.error_rate)]
        if self.data:
            argv += ["--data", self.data]
        if self.tokens:
            argv += ["--tokens", ",".join(self.tokens)]
        for p in self.peers:
            argv += ["--peer", p]
        if self.exec_file:
            argv += ["--exec", self.exec_file]
        if self.shards:
            argv += ["--shards", str(self.shards), "--shard-aware-port", str(self.shard_aware_port)]
        return argv + self.extra

    def start(self, timeout: float = 10.0) -> "CqlServer":
        ready = os.path.join(self.dir, "ready")
        if os.path.exists(ready):
            os.unlink(ready)
        logf = open(self.log_path, "ab")
        self.proc = subprocess.Popen(self._argv(), stdout=logf, stderr=logf, start_new_session=True, preexec_fn=die_with_parent())
        logf.close()
        deadline = time.monotonic() + timeout
        while time.monotonic() < deadline:
            if os.path.exists(ready):
                with open(ready) as f:
                    lines = f.read().split()
                self.port = int(lines[0])
                if len(lines) > 1 and int(lines[1]):
                    self.shard_aware_port = int(lines[1])  # kept across restarts
                # a restarted persistent server with --exec must not re-run the seed
                if self.exec_file and self.data:
                    self.exec_file = ""
                return self
            if self.proc.poll() is not None:
                raise RuntimeError(f"nexus-cqlsrv exited rc={self.proc.returncode}: {self.log()}")
            time.sleep(0.01)
        self.stop()
        raise RuntimeError("nexus-cqlsrv did not become ready")

    def log(self) -> str:
        try:
            with open(self.log_path) as f:
                return f.read()[-4000:]
        except OSError:
            return ""

    @property
    def address(self):
        return (self.host, self.port)

    def drop_connections(self) -> None:
        if self.proc is not None:
            self.proc.send_signal(signal.SIGUSR1)

    def kill(self) -> None:
        """Hard crash (SIGKILL): the WAL keeps what was acknowledged."""
        if self.proc is not None and self.proc.poll() is None:
            self.proc.kill()
            self.proc.wait(5)

    def restart(self, timeout: float = 10.0) -> "CqlServer":
        self.kill()
        return self.start(timeout)

    def stop(self) -> None:
        if self.proc is not None and self.proc.poll() is None:
            self.proc.terminate()
            try:
                self.proc.wait(5)
            except subprocess.TimeoutExpired:
                self.proc.kill()
                self.proc.wait(5)

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()
