"""CPU cost per pod failure of the native apiserver simulator alone (``nexus-kubesim``).

The wire bench shares the box's CPUs between the supervisor workers and the harness, so
the simulator's own busy-time counters swing with contention.  This driver isolates it:
the bench workload's traffic is applied (``/sim/apply``), the failed runs' Jobs are
DELETEd over pipelined keep-alive connections (Background propagation, as the
supervisor does), and ``--watchers`` watch streams per kind are drained by threads that
only read bytes.  Reported: simulator CPU µs per failure (utime + stime from /proc).

    python tools/kubesim_bench.py [--steps 60] [--events 1000] [--watchers 1]
"""
import argparse
import asyncio
import json
import os
import socket
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nexus_supervisor_amd.bench.workload import Workload  # noqa: E402
from nexus_supervisor_amd.testing.kubesim import KubeSim, SimControl, encode_events  # noqa: E402

PATHS = {"Pod": "/api/v1/namespaces/nexus/pods", "Job": "/apis/batch/v1/namespaces/nexus/jobs",
         "Event": "/api/v1/namespaces/nexus/events"}


def cpu_s(pid):
    with open(f"/proc/{pid}/stat") as f:
        parts = f.read().rsplit(")", 1)[1].split()
    return (int(parts[11]) + int(parts[12])) / os.sysconf("SC_CLK_TCK")


def drain(host, port, path, stop, counter):
    s = socket.create_connection((host, port))
    s.sendall(f"GET {path}?watch=1&resourceVersion=0 HTTP/1.1\r\nHost: x\r\n\r\n".encode())
    s.settimeout(0.2)
    while not stop.is_set():
        try:
            b = s.recv(1 << 20)
        except socket.timeout:
            continue
        if not b:
            break
        counter[0] += len(b)
    s.close()


def delete_all(host, port, names, conns=4):
    """Pipelined DELETEs over ``conns`` keep-alive connections; waits for every response."""
    body = b'{"kind":"DeleteOptions","apiVersion":"v1","propagationPolicy":"Background"}'
    socks = [socket.create_connection((host, port)) for _ in range(conns)]
    per = [names[i::conns] for i in range(conns)]
    for s, ns in zip(socks, per):
        reqs = b"".join(f"DELETE {PATHS['Job']}/{n} HTTP/1.1\r\nHost: x\r\nContent-Type: application/json\r\n"
                        f"Content-Length: {len(body)}\r\n\r\n".encode() + body for n in ns)
        s.sendall(reqs)
    for s, ns in zip(socks, per):
        want, got, buf = len(ns), 0, b""
        while got < want:
            buf += s.recv(1 << 16)
            got = buf.count(b"HTTP/1.1 ")
        s.close()


async def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--events", type=int, default=1000)
    ap.add_argument("--jobs", type=int, default=10_000)
    ap.add_argument("--watchers", type=int, default=1, help="watch streams per kind (replicas watching the namespace)")
    ap.add_argument("--flush-threads", type=int, default=0, help="simulator fan-out threads (0 = one per watcher, ≤ 8)")
    ap.add_argument("--async-gc", action="store_true", help="the simulator's GC thread (as the bench runs it)")
    args = ap.parse_args(argv)
    wl = Workload(concurrent_jobs=args.jobs)
    objs, _ = wl.initial()
    steps = [wl.step(args.events) for _ in range(args.steps + 2)]
    bodies = [(failed, encode_events(traffic)) for failed, traffic, _ in steps]
    ft = args.flush_threads or max(1, min(8, args.watchers))
    with KubeSim(history=50_000, flush_threads=ft, prefault_mb=int(os.environ.get("NEXUS_KUBESIM_PREFAULT_MB", "0")),
                 apply_threads=int(os.environ.get("NEXUS_KUBESIM_APPLY_THREADS", "1")), async_gc=args.async_gc) as sim:
        host, port = sim.url.split("//")[1].split(":")
        port = int(port)
        ctl = SimControl(sim.url, sim.apply_url)
        await ctl.apply_raw(encode_events(("ADDED", o) for o in objs))
        stop, counter = threading.Event(), [0]
        ths = [threading.Thread(target=drain, args=(host, port, p, stop, counter), daemon=True)
               for p in PATHS.values() for _ in range(args.watchers)]
        for t in ths:
            t.start()
        await asyncio.sleep(0.5)
        for failed, body in bodies[:2]:  # warmup
            await ctl.apply_raw(body)
            delete_all(host, port, failed)
        c0, t0 = cpu_s(sim.proc.pid), time.monotonic()
        st0 = await ctl.stats()
        b0, l0 = st0.get("busy_ns", 0), st0.get("lock_ns", 0)
        for failed, body in bodies[2:]:
            await ctl.apply_raw(body)
            await asyncio.get_running_loop().run_in_executor(None, delete_all, host, port, failed)
        await asyncio.sleep(0.3)
        c1, t1 = cpu_s(sim.proc.pid), time.monotonic()
        st = await ctl.stats()
        stop.set()
        await ctl.close()
    n = args.steps * args.events
    print(json.dumps({"failures": n, "kubesim_cpu_us_per_failure": round(1e6 * (c1 - c0) / n, 2),
                      "event_loop_busy_us_per_failure": round((st.get("busy_ns", 0) - b0) / 1e3 / n, 2), "flush_threads": ft,
                      # time holding the store mutex: the serial part, the simulator's ceiling
                      "store_lock_us_per_failure": round((st.get("lock_ns", 0) - l0) / 1e3 / n, 2),
                      "threads": st.get("threads"),
                      "wall_s": round(t1 - t0, 2), "watch_bytes": counter[0], "watchers_per_kind": args.watchers,
                      "sim": {k: st.get(k) for k in ("requests", "deleted", "applied", "sends")},
                      "us_per_failure": {k[:-3]: round((st.get(k, 0) - st0.get(k, 0)) / 1000 / n, 2) for k in st if k.endswith("_ns") and isinstance(st[k], (int, float))}}))


if __name__ == "__main__":
    asyncio.run(main())
