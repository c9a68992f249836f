"""Measure a supervisor replica's own memory against the number of concurrent jobs
(VERDICT r3 weak #7 / next #8).

The bench's ``replica_rss_mb`` includes the bench driver and torch's HIP context in the same
process.  This tool runs the replica the way production does — ``python -m
nexus_supervisor_amd supervisor`` as its own process tree (coordinating parent + shard
workers) — against the native apiserver simulator and CQL server holding N live runs
(Job + Pod with torchrun env, one RUNNING checkpoint row each, the bench workload's shape),
waits for ``/readyz`` (caches synced), then fails runs with the bench's failure mix for a
while (churn: every failed run is replaced by a fresh one) and samples RSS of every
process of the replica (``/proc/<pid>/status`` VmRSS / VmHWM).

    python tools/replica_memory.py --jobs 0 5000 10000 20000 --procs 1 6 --out profiles/r4_memory/replica_memory.json

Output: per (procs, jobs) the parent's and the workers' RSS after sync and after churn,
plus the least-squares slope in MB per 1k jobs — what ``values.yaml`` ``resources`` cites.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import subprocess
import sys
import tempfile
import time
import urllib.request

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from nexus_supervisor_amd.bench.wire import schema_statements  # noqa: E402
from nexus_supervisor_amd.bench.workload import Workload  # noqa: E402
from nexus_supervisor_amd.store.cql import CqlCheckpointStore, CqlSession  # noqa: E402
from nexus_supervisor_amd.testing.cqlsrv import CqlServer  # noqa: E402
from nexus_supervisor_amd.testing.kubesim import KubeSim, SimControl  # noqa: E402


def _rss(pid: int):
    out = {}
    try:
        with open(f"/proc/{pid}/status") as f:
            for ln in f:
                if ln.startswith(("VmRSS:", "VmHWM:")):
                    k, v = ln.split(":", 1)
                    out[k] = int(v.split()[0]) / 1024.0
    except OSError:
        return None
    return out


def _children(pid: int):
    kids = []
    try:
        for t in os.listdir(f"/proc/{pid}/task"):
            with open(f"/proc/{pid}/task/{t}/children") as f:
                kids += [int(x) for x in f.read().split()]
    except OSError:
        pass
    return kids


def _tree(pid: int):
    parent = _rss(pid) or {}
    workers = [r for r in (_rss(k) for k in _children(pid)) if r]
    return {"parent_rss_mb": round(parent.get("VmRSS", 0.0), 1), "parent_hwm_mb": round(parent.get("VmHWM", 0.0), 1),
            "workers": len(workers), "workers_rss_mb": round(sum(w.get("VmRSS", 0.0) for w in workers), 1),
            "workers_hwm_mb": round(sum(w.get("VmHWM", 0.0) for w in workers), 1),
            "total_rss_mb": round(parent.get("VmRSS", 0.0) + sum(w.get("VmRSS", 0.0) for w in workers), 1)}


async def measure(jobs: int, procs: int, churn_events: int, workdir: str, trace: int = 0, rate: float = 0.0):
    sim = KubeSim(history=50_000, bookmark_ms=2000).start()
    cql = CqlServer(exec_statements=schema_statements(), shards=2).start()
    ctl = SimControl(sim.url)
    wl = Workload(max(jobs, 1) if jobs else 0)
    objs, rows = wl.initial() if jobs else ([], [])
    store = CqlCheckpointStore(CqlSession([("127.0.0.1", cql.port)], connections_per_host=2, consistency="ONE"),
                               consistency="ONE")
    await store.connect()
    for i in range(0, len(rows), 500):
        await asyncio.gather(*(store.upsert_checkpoint(r) for r in rows[i:i + 500]))
    for i in range(0, len(objs), 4096):
        await ctl.apply([("ADDED", o) for o in objs[i:i + 4096]])
    kcfg = os.path.join(workdir, "kubeconfig")
    with open(kcfg, "w") as f:
        json.dump({"apiVersion": "v1", "kind": "Config", "current-context": "m",
                   "clusters": [{"name": "m", "cluster": {"server": sim.url}}],
                   "contexts": [{"name": "m", "context": {"cluster": "m", "user": "m"}}],
                   "users": [{"name": "m", "user": {}}]}, f)
    port = 19000 + (os.getpid() % 1000)
    env = dict(os.environ, PYTHONPATH=ROOT, NEXUS__KUBE_CONFIG_PATH=kcfg, NEXUS__CQL_STORE_TYPE="scylla",
               NEXUS__SCYLLA_CQL_STORE__HOSTS=f"127.0.0.1:{cql.port}", NEXUS__SCYLLA_CQL_STORE__CONSISTENCY="ONE",
               NEXUS__RESOURCE_NAMESPACE="nexus", NEXUS__RUNTIME__WORKER_PROCESSES=str(procs),
               NEXUS__OBSERVABILITY__HTTP_PORT=str(port), NEXUS__OBSERVABILITY__HTTP_HOST="127.0.0.1",
               NEXUS__RATE_LIMIT_ELEMENTS_PER_SECOND="0", NEXUS__WORKERS="64", NEXUS__KUBE_QPS="0",
               NEXUS__LOG_LEVEL="ERROR", NEXUS__GPU__BACKEND="none")
    if trace:
        env["PYTHONTRACEMALLOC"] = str(trace)
    log = open(os.path.join(workdir, f"sup_{procs}_{jobs}.log"), "wb")
    proc = subprocess.Popen([sys.executable, "-m", "nexus_supervisor_amd", "supervisor"], env=env, stdout=log,
                            stderr=log, start_new_session=True)
    out = {"jobs": jobs, "procs": procs}
    try:
        t0 = time.monotonic()
        while True:
            try:
                with urllib.request.urlopen(f"http://127.0.0.1:{port}/readyz", timeout=2) as r:
                    if r.status == 200:
                        break
            except Exception:  # noqa: BLE001 - not up yet
                pass
            if proc.poll() is not None or time.monotonic() - t0 > 300:
                raise RuntimeError(f"supervisor did not become ready (rc={proc.poll()})")
            await asyncio.sleep(0.2)
        out["sync_s"] = round(time.monotonic() - t0, 2)
        await asyncio.sleep(2.0)
        out["after_sync"] = _tree(proc.pid)
        heap0 = _heap(port) if procs == 1 else None
        done = 0
        if jobs:
            while done < churn_events:
                n = min(500, churn_events - done)
                failed, traffic, new_rows = wl.step(n)
                await asyncio.gather(*(store.upsert_checkpoint(r) for r in new_rows))
                await ctl.apply(traffic)
                done += n
                await asyncio.sleep(max(0.05, n / rate) if rate else 0.05)
            await asyncio.sleep(3.0)
        out["churn_events"] = done
        out["after_churn"] = _tree(proc.pid)
        if heap0 is not None:
            heap1 = _heap(port, "&trim=1")
            out["heap_after_churn"] = {"structures": heap1.get("structures"), "rss_mb": heap1.get("rss_mb"),
                                       "rss_before_trim_mb": heap1.get("rss_before_trim_mb"),
                                       "rss_after_trim_mb": heap1.get("rss_after_trim_mb"),
                                       "tracemalloc_mb": [heap0.get("tracemalloc_mb"), heap1.get("tracemalloc_mb")],
                                       "tracemalloc_growth": (heap1.get("tracemalloc_growth") or [])[:12]}
            out["heap_growth"] = {
                "types": _grow(heap0.get("types", {}), heap1.get("types", {})),
                "dict_shapes": _grow(heap0.get("dict_shapes", {}), heap1.get("dict_shapes", {}))}
    finally:
        proc.terminate()
        try:
            proc.wait(20)
        except subprocess.TimeoutExpired:
            proc.kill()
        log.close()
        await store.close()
        await ctl.close()
        sim.stop()
        cql.stop()
    return out


def _heap(port: int, extra: str = ""):
    with urllib.request.urlopen(f"http://127.0.0.1:{port}/debug/heap?top=60{extra}", timeout=60) as r:
        return json.loads(r.read())


def _grow(a, b, n: int = 8):
    d = {k: b.get(k, 0) - a.get(k, 0) for k in set(a) | set(b)}
    return dict(sorted(((k, v) for k, v in d.items() if v), key=lambda kv: -kv[1])[:n])


def _slope(points):
    n = len(points)
    if n < 2:
        return None
    mx = sum(x for x, _ in points) / n
    my = sum(y for _, y in points) / n
    sxx = sum((x - mx) ** 2 for x, _ in points)
    return round(sum((x - mx) * (y - my) for x, y in points) / sxx * 1000.0, 2) if sxx else None


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, nargs="+", default=[0, 5000, 10000, 20000])
    ap.add_argument("--procs", type=int, nargs="+", default=[1, 6])
    ap.add_argument("--churn", type=int, default=20000, help="failed runs (each replaced) after the sync")
    ap.add_argument("--out", default="")
    ap.add_argument("--churn-rate", type=float, default=0.0, help="failures per second during the churn (0 = ~10k/s)")
    ap.add_argument("--tracemalloc", type=int, default=0, help="PYTHONTRACEMALLOC frames in the replica (diagnosis)")
    a = ap.parse_args(argv)
    results = []
    with tempfile.TemporaryDirectory(prefix="nexus-mem-") as wd:
        for procs in a.procs:
            for jobs in a.jobs:
                r = asyncio.run(measure(jobs, procs, a.churn, wd, a.tracemalloc, a.churn_rate))
                print(json.dumps(r), flush=True)
                results.append(r)
    summary = {}
    for procs in a.procs:
        rs = [r for r in results if r["procs"] == procs]
        for phase in ("after_sync", "after_churn"):
            for part in ("parent_rss_mb", "workers_rss_mb", "total_rss_mb"):
                summary.setdefault(f"procs{procs}", {})[f"{phase}.{part}.per_1k_jobs"] = _slope(
                    [(r["jobs"], r[phase][part]) for r in rs])
        base = next((r for r in rs if r["jobs"] == 0), None)
        if base:
            summary[f"procs{procs}"]["base_total_rss_mb"] = base["after_churn"]["total_rss_mb"]
    doc = {"tool": "tools/replica_memory.py", "python": sys.version.split()[0], "runs": results, "summary": summary}
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(doc, f, indent=1)
    print(json.dumps(summary, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
