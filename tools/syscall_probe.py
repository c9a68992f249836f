#!/usr/bin/env python3
"""Syscall cost probe: what one kernel crossing costs on this host.

The supervisor's hot path is loopback/remote socket I/O (CQL + HTTP), so the
per-syscall price decides whether batching requests per write pays.  Prints one
JSON object with ns per call for: a trivial syscall, send/recv on a UNIX socket
pair, a TCP loopback send, and a TCP loopback one-byte ping-pong (two processes).
"""
from __future__ import annotations

import json
import os
import select
import socket
import sys
import time


def per_call(fn, n):
    t = time.perf_counter_ns()
    for _ in range(n):
        fn()
    return (time.perf_counter_ns() - t) / n


def main() -> int:
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
    out = {}
    out["python_noop_call_ns"] = per_call(lambda: None, n)
    out["getppid_ns"] = per_call(os.getppid, n)
    a, b = socket.socketpair()
    msg = b"x" * 100

    def unix_rt():
        a.send(msg)
        b.recv(4096)
    out["unix_send_recv_100B_ns"] = per_call(unix_rt, n)

    srv = socket.socket()
    srv.bind(("127.0.0.1", 0))
    srv.listen(1)
    c = socket.create_connection(srv.getsockname())
    s, _ = srv.accept()
    for sk in (c, s):
        sk.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)

    def tcp_rt():
        c.send(msg)
        s.recv(4096)
    out["tcp_send_recv_100B_ns"] = per_call(tcp_rt, n)
    big = b"x" * 16384

    def tcp_big():
        c.send(big)
        got = 0
        while got < len(big):
            got += len(s.recv(65536))
    out["tcp_send_recv_16KiB_ns"] = per_call(tcp_big, n // 4)
    ep = select.epoll()
    ep.register(s.fileno(), select.EPOLLIN)
    out["epoll_wait0_ns"] = per_call(lambda: ep.poll(0), n)

    # cross-process ping-pong (wakeup cost)
    pid = os.fork()
    if pid == 0:
        try:
            while True:
                d = s.recv(1)
                if not d or d == b"q":
                    break
                s.send(d)
        finally:
            os._exit(0)

    def pingpong():
        c.send(b"p")
        c.recv(1)
    out["tcp_pingpong_xproc_ns"] = per_call(pingpong, n // 4)
    c.send(b"q")
    os.waitpid(pid, 0)
    out = {k: round(v, 1) for k, v in out.items()}
    out["cpus"] = os.cpu_count()
    try:
        with open("/proc/version") as f:
            out["kernel"] = f.read().strip()[:120]
    except OSError:
        pass
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
