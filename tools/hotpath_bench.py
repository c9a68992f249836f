"""Shard-worker hot path without sockets: CPU per pod failure, reproducible to ~2 %.

The wire bench measures the whole replica next to an apiserver simulator, a CQL server
and a traffic generator on the same cores, so a few-percent change of the supervisor's
own cost drowns in box-to-box and run-to-run noise.  This drives ONE supervisor exactly
as a shard worker is driven — the hub's SNAPSHOT / LINES frames into
:class:`..parallel.watchhub.HubListWatch` (native projected decode, batched informer
apply), the bench's failure mix, its supervisor config and GPU evidence provider — with
an in-memory store and Job client, and echoes each Job DELETE back as the DELETED lines
of the Job and its Pod (what the API server's garbage collector sends).  It reports the
main thread's CPU per failure (``time.thread_time``) over the timed steps.

    python tools/hotpath_bench.py [--jobs 10000] [--events 1000] [--steps 20] [--warmup 3]
                                  [--repeat 3] [--pprof OUT.pb.gz] [--cprofile OUT.prof]

Not covered (the wire bench's job): CQL encode / socket I/O, the HTTP DELETE, the hub.
"""
import argparse
import asyncio
import gc
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from nexus_supervisor_amd.bench.runner import BenchConfig, supervisor_config  # noqa: E402

try:  # absent from older trees (the harness is also run against _ab/base snapshots)
    from nexus_supervisor_amd.bench.runner import _stage_counts, _stage_delta  # noqa: E402
except ImportError:  # pragma: no cover
    def _stage_counts(sup):
        return {}

    def _stage_delta(before, after):
        return {}
from nexus_supervisor_amd.bench.workload import Workload  # noqa: E402
from nexus_supervisor_amd.gpu.telemetry import FakeTelemetry, pod_evidence_provider  # noqa: E402
from nexus_supervisor_amd.informer import InformerFactory  # noqa: E402
from nexus_supervisor_amd.obs.logging import configure_logging  # noqa: E402
from nexus_supervisor_amd.parallel.watchhub import KINDS, LINES, SNAPSHOT, HubListWatch  # noqa: E402
from nexus_supervisor_amd.store.memory import MemoryStore  # noqa: E402
from nexus_supervisor_amd.supervisor import Supervisor  # noqa: E402
from nexus_supervisor_amd.testing.inproc import RecordingJobs  # noqa: E402

FRAME_LINES = 16  # watch lines per LINES frame (the hub's frames carry a few lines each)


def _containers(obj, prefix="sup.", depth=0, seen=None):
    """(size, path) of every dict / set / list / deque over 100 entries reachable from the
    supervisor's attributes (three levels): a structure that grows step after step is a
    leak, and a growing per-event cost usually is one."""
    seen = set() if seen is None else seen
    out = []
    for k, v in list(vars(obj).items()):
        if id(v) in seen:
            continue
        seen.add(id(v))
        if isinstance(v, (dict, set, list)) or type(v).__name__ in ("deque", "OrderedDict"):
            if len(v) > 100:
                out.append((len(v), prefix + k))
        elif depth < 3 and hasattr(v, "__dict__") and type(v).__module__.startswith("nexus_supervisor_amd"):
            out += _containers(v, f"{prefix}{k}.", depth + 1, seen)
    return out


def _lines(events, logs=None):
    out = {k: [] for k in KINDS}
    for etype, obj in events:
        if etype == "LOG":  # default-pod HBM OOM: the text the pods/log read returns
            if logs is not None:
                logs[(obj["namespace"], obj["pod"], obj["container"])] = obj["text"].encode()
            continue
        out[obj["kind"]].append(json.dumps({"type": etype, "object": obj}, separators=(",", ":")).encode())
    return out


async def run(args) -> dict:
    sc = supervisor_config(BenchConfig())
    try:
        wl = Workload(args.jobs, seed=args.seed, hbm_shape=args.hbm_shape)
    except TypeError:  # pragma: no cover - older trees (_ab/base snapshots)
        wl = Workload(args.jobs, seed=args.seed)
    objs, rows = wl.initial()
    store = MemoryStore(rows)
    queues = {k: asyncio.Queue() for k in KINDS}
    factory = InformerFactory(lambda kind: HubListWatch(kind, queues[kind]), resync_period=0.0)
    jobs = RecordingJobs(o["metadata"]["name"] for o in objs if o["kind"] == "Job")
    # the worker's logging (JSON lines, buffered), into /dev/null: one line per decision
    logger = configure_logging("INFO", stream=open(os.devnull, "w"))
    sup = Supervisor(sc, store, jobs, factory, logger=logger)
    tel = FakeTelemetry()
    sup.classifier.evidence_provider = pod_evidence_provider(tel)
    for k in KINDS:
        items = [o for o in objs if o["kind"] == k]
        queues[k].put_nowait((SNAPSHOT, b"1\n" + json.dumps(items, separators=(",", ":")).encode()))
    latest = {(o["kind"], o["metadata"]["name"]): o for o in objs if o["kind"] in ("Job", "Pod")}
    waiting: set = set()
    all_decided = asyncio.Event()

    def on_decision(d):
        waiting.discard(d.result.request_id)
        if not waiting:
            all_decided.set()

    sup.decision_hooks.append(on_decision)
    sup.init()
    await sup.start(wait_sync_timeout=60)

    from nexus_supervisor_amd import _kube_native
    from nexus_supervisor_amd.classify.classifier import EVENT_REASONS_READ

    ev_router = _kube_native.ShardRouter(0, 1, 0, sc.labels.job_name_label)
    ev_router.set_event_reasons(sorted(EVENT_REASONS_READ))
    ev_splitter = _kube_native.WatchSplitter(ev_router, "event")

    def push(lines_by_kind):
        for k, lines in lines_by_kind.items():
            for i in range(0, len(lines), FRAME_LINES):
                queues[k].put_nowait((LINES, b"\n".join(lines[i:i + FRAME_LINES]) + b"\n"))

    def gen():
        """One step's inputs, encoded up front (outside the timed region): the failure
        traffic, and the DELETED echo of each failed run's Job and Pod."""
        failed, traffic, new_rows = wl.step(args.events)
        for etype, o in traffic:
            if o.get("kind") in ("Job", "Pod"):
                latest[(o["kind"], o["metadata"]["name"])] = o
        echo = []
        for name in failed:
            for kind, key in (("Job", name), ("Pod", f"{name}-w0")):
                o = latest.pop((kind, key), None)
                if o is not None:
                    echo.append(("DELETED", dict(o, metadata=dict(o["metadata"], resourceVersion=wl._next_rv()))))
        by_kind = _lines(traffic, getattr(jobs, "logs", None))
        if by_kind.get("Event"):
            # the watch hub's splitter (parent process) drops the Events no rule reads
            outs, _, _ = ev_splitter.feed(b"\n".join(by_kind["Event"]) + b"\n")
            by_kind["Event"] = outs[0].splitlines()
        return failed, new_rows, by_kind, _lines(echo)

    async def step(data):
        failed, new_rows, traffic, echo = data
        for r in new_rows:
            store.rows[r.key] = r
        waiting.update(failed)
        all_decided.clear()
        push(traffic)
        try:
            await asyncio.wait_for(all_decided.wait(), 60)
        except asyncio.TimeoutError:
            raise RuntimeError(f"{len(waiting)} failures undecided") from None
        while sup._deletes:
            await asyncio.wait(list(sup._deletes), timeout=10)
        push(echo)  # the API server's answer to the DELETEs
        for rid in failed:  # finished runs leave the store (a real worker's heap does not hold them)
            store.rows.pop((wl.algorithm, rid), None)
        jobs.deleted.clear()
        getattr(store, "write_log", []).clear()
        await asyncio.sleep(0)
        while any(not q.empty() for q in queues.values()):
            await asyncio.sleep(0.002)
        return len(failed)

    for _ in range(args.warmup):
        await step(gen())
    results = []
    for _ in range(args.repeat):
        batch = [gen() for _ in range(args.steps)]
        gc.collect()
        sampler = prof = None
        if args.pprof:
            from nexus_supervisor_amd.obs.pprof import Sampler

            sampler = Sampler(hz=499).start()
        if args.cprofile:
            import cProfile

            prof = cProfile.Profile()
            prof.enable()
        gc_t = {0: 0.0, 1: 0.0, 2: 0.0}
        gc_n = {0: 0, 1: 0, 2: 0}
        gc_start = [0.0]

        def gc_cb(phase, info):
            if phase == "start":
                gc_start[0] = time.thread_time()
            else:
                g = info.get("generation", 0)
                gc_t[g] += time.thread_time() - gc_start[0]
                gc_n[g] += 1

        gc.callbacks.append(gc_cb)
        lws = [inf.lw for inf in factory.informers.values()]
        d0 = sum(lw.decode_seconds for lw in lws)
        l0 = {inf.kind: inf.lw.decoded_lines for inf in factory.informers.values()}
        stages0 = _stage_counts(sup)
        c0, t0, n = time.thread_time(), time.perf_counter(), 0
        for data in batch:
            n += await step(data)
            if args.gap:
                await asyncio.sleep(args.gap)
        cpu, wall = time.thread_time() - c0, time.perf_counter() - t0
        gc.callbacks.remove(gc_cb)
        if prof is not None:
            prof.disable()
            prof.dump_stats(args.cprofile)
        if sampler is not None:
            with open(args.pprof, "wb") as f:
                f.write(sampler.stop().encode_gz())
        results.append({"cpu_us_per_event": round(1e6 * cpu / n, 1), "events_per_s_cpu": round(n / cpu),
                        "wall_s": round(wall, 2), "events": n,
                        "decode_us_per_event": round(1e6 * (sum(lw.decode_seconds for lw in lws) - d0) / n, 1),
                        "lines_per_event": {inf.kind: round((inf.lw.decoded_lines - l0[inf.kind]) / n, 2)
                                            for inf in factory.informers.values()},
                        "gc_us_per_event": {g: round(1e6 * gc_t[g] / n, 2) for g in gc_t},
                        "gc_collections": dict(gc_n),
                        "stages_ms": _stage_delta(stages0, _stage_counts(sup))})
        del batch
        if args.sizes:
            results[-1]["containers"] = sorted(_containers(sup), reverse=True)[:12]
    await sup.stop(drain=True, timeout=5)
    us = [r["cpu_us_per_event"] for r in results]
    return {"cpu_us_per_event_median": statistics.median(us), "cpu_us_per_event": us, "runs": results,
            "config": {"jobs": args.jobs, "events": args.events, "steps": args.steps, "frame_lines": FRAME_LINES}}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=10_000)
    ap.add_argument("--events", type=int, default=1000)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--repeat", type=int, default=3)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--pprof", default="")
    ap.add_argument("--cprofile", default="")
    ap.add_argument("--gap", type=float, default=0.0,
                    help="idle seconds between steps (low-rate mode: with --events 1, what one failure costs when "
                         "nothing is batched and every telemetry snapshot is stale)")
    ap.add_argument("--sizes", action="store_true", help="report the supervisor's large containers per repeat")
    ap.add_argument("--hbm-shape", default="default-pod", choices=("default-pod", "termination-message"),
                    help="HBM-OOM failures as the wire bench's default (the text in the container log, read over "
                         "pods/log: served here from memory) or in the termination message")
    args = ap.parse_args(argv)
    out = asyncio.run(run(args))
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
