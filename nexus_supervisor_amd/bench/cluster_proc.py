"""Synthetic cluster process for the wire-mode benchmark.

Runs, in its own process (so its CPU does not count against the supervisor's
event loop): the kube-apiserver (the native ``nexus-kubesim`` child by default,
``--api python`` for the Python fake), the :class:`~.workload.Workload`
generator, and the "receiver" role that inserts each new run's checkpoint row
into the CQL store before the run's pods exist (what nexus's receiver does
upstream of the supervisor).  A small control API drives it:

``POST /bench/init {"jobs": N, "seed": s, "shards": S, "shard_indexes": [k, ...],
                   "pregen": P, "events": E}``
                                                    one workload per listed replica shard
                                                    (N live runs each, + rows) and P
                                                    pre-generated steps of E failures each
``POST /bench/step {"events": E, "shard": k}``    fail E runs of shard k, start the previous
                                                    step's new runs, create E new ones;
                                                    ``{"rids": [...], "t_push": monotonic,
                                                    "expected": {rid: stage}, "started": [...],
                                                    "start_expected": {rid: "RUNNING"}}``
``POST /bench/probe {"n": N, "rate_per_min": R, "seed": s, "shard": k}``
                                                    the open-loop probe: N one-failure steps
                                                    at Poisson arrivals, ``{"steps": [...]}``

Per-rank mode lists one shard (the rank's own cluster); shared mode (``bench.py
--cluster shared``) lists every shard: one apiserver and one CQL server for the whole
node, every replica watching the whole namespace and owning its shard of it.

``python -m nexus_supervisor_amd.bench.cluster_proc --ready-file F --cql HOST:PORT``
"""
from __future__ import annotations

import argparse
import asyncio
import collections
import gc
import json
import os
import sys
import time

from aiohttp import web


# watch lines per /sim/apply request: the simulator applies a request in one pass of its
# event loop, so a whole 20k-line step in one request would hold every watch flush, Job
# DELETE and pods/log answer for its duration (tens of ms); chunks interleave with them
APPLY_CHUNK = int(os.environ.get("NEXUS_BENCH_APPLY_CHUNK", "1024"))
# chunks sent ahead of their answers on the generator's apply connection (HTTP/1.1
# pipelining; 1 = one request per round trip): the apply port then never idles between two
# chunks of a step waiting for this process to read an answer and send the next
APPLY_DEPTH = int(os.environ.get("NEXUS_BENCH_APPLY_DEPTH", "3"))


async def amain(args) -> None:
    from ..store.cql import CqlCheckpointStore, CqlSession
    from ..testing.fake_apiserver import FakeApiServer
    from .workload import DEFAULT_HIP_OOM, Workload

    sim = simctl = api = None
    if args.api == "kubesim":
        # native apiserver simulator: the generator below only produces traffic
        from ..testing.kubesim import KubeSim, SimControl, encode_events

        sim = KubeSim(host=args.host, port=args.port, history=args.history, bookmark_ms=2000,
                      flush_threads=args.flush_threads, api_latency_us=args.api_latency_us,
                      write_qps=args.write_qps, write_burst=args.write_burst,
                      prefault_mb=int(os.environ.get("NEXUS_KUBESIM_PREFAULT_MB", "768")),
                      apply_threads=int(os.environ.get("NEXUS_KUBESIM_APPLY_THREADS", "6")),
                      log_root=args.log_root,
                      # Job DELETEs answered before their pods go, as a real API server does (its
                      # GC deletes them afterwards): the pod cascade is off the simulator's loop
                      async_gc=os.environ.get("NEXUS_KUBESIM_ASYNC_GC", "1") == "1").start()
        simctl = SimControl(sim.url, sim.apply_url)
    else:
        api = FakeApiServer(history=args.history, bookmark_interval=2.0)

    async def apply_chunks(bodies):
        """Apply pre-encoded chunks in order; the step's push time is the first commit."""
        if APPLY_DEPTH > 1:
            docs = await simctl.apply_pipelined(list(bodies), APPLY_DEPTH)
            return docs[0]["t_push"] if docs else time.monotonic()
        t = None
        for b in bodies:
            doc = await simctl.apply_raw(b)
            t = doc["t_push"] if t is None else t
        return t if t is not None else time.monotonic()

    async def apply(events):
        """Commit watch traffic to the API server; returns the commit (push) time."""
        if simctl is not None:
            return await apply_chunks([encode_events(events[i:i + APPLY_CHUNK])
                                       for i in range(0, len(events), APPLY_CHUNK)])
        t = time.monotonic()
        for i, (etype, obj) in enumerate(events):
            api.apply(etype, obj, copy_obj=False)
            if i % 256 == 255:
                await asyncio.sleep(0)  # keep serving DELETEs / watch writes during a burst
        return t
    host, _, port = args.cql.partition(":")
    store = CqlCheckpointStore(CqlSession([(host, int(port))], connections_per_host=2, consistency="ONE"), consistency="ONE")
    await store.connect()
    shards = {}  # replica shard → _Shard
    state = {}

    class _Shard:
        def __init__(self, wl):
            self.wl = wl
            self.pregen = collections.deque()
            self.next = None
            self.lock = asyncio.Lock()

    async def write_rows(rows):
        # the receiver's inserts as UNLOGGED batches of 64 rows, 8 batches in flight
        chunk = 64 * 8
        await asyncio.gather(*(store.upsert_many(rows[i:i + chunk]) for i in range(0, len(rows), chunk)))

    async def h_init(req):
        p = await req.json()
        n_shards = int(p.get("shards", 1))
        indexes = p.get("shard_indexes")
        if indexes is None:
            indexes = [int(p.get("shard_index", 0))]
        node_slots = int(p.get("node_slots", 0))
        if node_slots:
            indexes = list(range(node_slots))  # node mode: one workload per GPU slot, one replica
        total = 0
        for k in indexes:
            # per-rank mode: the rank's workload (rank = its shard); shared mode: one per shard;
            # node mode: slot k's runs on GPU k (one replica owns every slot: no shard filter)
            wl = Workload(p.get("jobs", 10_000), rank=k if len(indexes) > 1 else p.get("rank", 0),
                          world=p.get("world", 1), seed=p.get("seed", 0),
                          hip_oom_message=p.get("hip_oom_message") or DEFAULT_HIP_OOM,
                          shards=1 if node_slots else n_shards, shard_index=0 if node_slots else k,
                          shard_label=p.get("shard_label") or "", hbm_shape=p.get("hbm_shape") or "termination-message",
                          run_starts=bool(p.get("run_starts", True)), visible_devices=str(k) if node_slots else None)
            objs, rows = wl.initial()
            await write_rows(rows)
            await apply([("ADDED", o) for o in objs])
            sh = shards[k] = _Shard(wl)
            total += len(objs)
            # synthetic input generated up front (like a data loader's pre-built batches): the
            # failures of the next `pregen` steps of `events` each, their replacement runs' rows
            # inserted (the receiver writes a run's row before its pods exist) and their watch
            # traffic encoded, so a timed step costs the generator one HTTP request
            pregen, events = int(p.get("pregen", 0)), int(p.get("events", 0))
            if pregen and events and simctl is not None:
                for _ in range(pregen):
                    st = wl.step(events)
                    await write_rows(st.rows)
                    sh.pregen.append((events, st, [encode_events(st.traffic[i:i + APPLY_CHUNK])
                                                   for i in range(0, len(st.traffic), APPLY_CHUNK)]))
                    st.traffic = None  # encoded: only the ids and expected stages are kept
        # the simulated cluster holds the same 10k-run heap as the supervisor: keep it out
        # of full collections so the generator never paces the measured process
        gc.collect()
        gc.freeze()
        gc.set_threshold(20000, 20, 20)
        return web.json_response({"objects": total, "shards": sorted(shards)})

    async def prepare(wl, events: int):
        # generate the next step's traffic and insert its replacement runs' rows ahead of
        # time (overlapped with the supervisor working on the current step)
        st = wl.step(events)
        await write_rows(st.rows)
        return st

    async def h_step(req):
        cp = state.pop("cprof", None)
        if cp is not None:
            cp.enable()
        p = await req.json()
        events = int(p["events"])
        sh = shards[int(p["shard"])] if "shard" in p else next(iter(shards.values()))
        async with sh.lock:  # one step of a shard at a time (shards run concurrently)
            doc = await _step(sh, events)
        hold = float(p.get("respond_after_ms") or 0.0)
        if hold > 0:
            # latency probe: answer after the failure has been delivered and decided, so the
            # bench driver's handling of this answer never shares the replica parent's loop
            # with the watch line it is timing (the driver is not part of the supervisor)
            await asyncio.sleep(hold / 1000.0)
        return web.json_response(doc)

    async def h_probe(req):
        """The open-loop latency probe, played here: ``n`` single failures of shard ``shard``
        at Poisson arrivals of mean rate ``rate_per_min`` (``seed``: the same schedule every
        run), each one step; answers once every arrival is applied, with each step's
        ``{"rids", "t_push", "expected"}`` in arrival order.  The bench driver makes ONE
        request for the whole probe, so nothing of the driver runs on the replica parent's
        loop while failures are in flight (an HTTP round trip per arrival there cost 1–4 ms
        of that loop, overlapping the next arrivals' watch delivery)."""
        import random

        p = await req.json()
        n = int(p["n"])
        rate = float(p.get("rate_per_min", 1000.0)) / 60.0
        rng = random.Random(int(p.get("seed", 0)))
        sh = shards[int(p["shard"])] if "shard" in p else next(iter(shards.values()))
        loop = asyncio.get_running_loop()
        docs = [None] * n
        async with sh.lock:
            # the saturated steps left a prefetched 1000-failure step (and maybe pre-generated
            # ones) whose replacement runs are live in the workload: create them in the cluster
            # now and let the supervisor absorb that burst (thousands of ADDED lines) before the
            # first timed arrival, instead of inside it
            while sh.pregen:
                await apply_chunks(sh.pregen.popleft()[2])
            nxt, sh.next = sh.next, None
            if nxt is not None:
                # its runs' starts and failures are part of the workload's state now: the
                # cluster must see them (their decisions are absorbed in the settle below)
                stale = await nxt[1]
                await apply(stale.traffic)
            # the saturated steps' Events reach their TTL now, not in the first arrival's step
            expired = sh.wl.expire_all()
            if expired:
                await apply(expired)
        await asyncio.sleep(float(p.get("settle_s", 2.0)))

        async def one(i):
            async with sh.lock:
                docs[i] = await _step(sh, 1)

        tasks = []
        start = loop.time()
        at = 0.0
        for i in range(n):
            at += rng.expovariate(rate)
            delay = start + at - loop.time()
            if delay > 0:
                await asyncio.sleep(delay)
            tasks.append(asyncio.ensure_future(one(i)))  # open loop: the next arrival never waits
        await asyncio.gather(*tasks)
        return web.json_response({"steps": docs})

    async def _step(sh, events):
        wl = sh.wl
        queue = sh.pregen
        if queue and queue[0][0] == events and sh.next is None:
            _, st, body = queue.popleft()
            t_push = await apply_chunks(body)
            return st.doc(t_push)
        if queue:
            # a step of another size (latency probe): the pre-generated steps' runs are live
            # in the workload already, so they must exist in the cluster before we diverge
            while queue:
                await apply_chunks(queue.popleft()[2])
        nxt, sh.next = sh.next, None
        if nxt is not None and nxt[0] == events:
            st = await nxt[1]
        else:
            if nxt is not None:
                # a prefetched step of another size is dropped: its starts and failures are
                # already part of the workload's state, so the cluster must see them too
                # (untimed: nobody waits for their decisions)
                stale = await nxt[1]
                await apply(stale.traffic)
            st = await prepare(wl, events)
        t_push = await apply(st.traffic)
        sh.next = (events, asyncio.ensure_future(prepare(wl, events)))
        return st.doc(t_push)

    async def h_oom(req):
        """One running run of slot ``slot`` dies of an HBM-OOM whose text is ``message`` (a
        real OOM's, from that slot's GPU): ``{"rids", "t_push", "expected"}``."""
        p = await req.json()
        sh = shards[int(p["slot"])]
        async with sh.lock:
            # the slot's pending steps must exist in the cluster before the workload diverges
            while sh.pregen:
                await apply_chunks(sh.pregen.popleft()[2])
            nxt, sh.next = sh.next, None
            if nxt is not None:
                stale = await nxt[1]
                await apply(stale.traffic)
            st = sh.wl.fail_with("hbm-oom", p.get("message"))
            await write_rows(st.rows)
            t_push = await apply(st.traffic)
        return web.json_response(st.doc(t_push))

    async def h_stats(req):
        if simctl is not None:
            return web.json_response(await simctl.stats())
        return web.json_response({"requests": api.requests, "watch_requests": api.watch_requests, "rv": api.rv,
                                  "deleted": len(api.deleted)})

    url = sim.url if sim is not None else await api.start(args.host, args.port)
    # control routes live on a second tiny app (the apiserver app is frozen once started)
    ctl = web.Application(client_max_size=64 << 20)
    ctl.router.add_post("/bench/init", h_init)
    ctl.router.add_post("/bench/step", h_step)
    ctl.router.add_post("/bench/probe", h_probe)
    ctl.router.add_post("/bench/oom", h_oom)
    ctl.router.add_get("/bench/stats", h_stats)
    runner = web.AppRunner(ctl, access_log=None)
    await runner.setup()
    site = web.TCPSite(runner, args.host, 0, backlog=1024)
    await site.start()
    ctl_port = site._server.sockets[0].getsockname()[1]  # noqa: SLF001
    tmp = args.ready_file + ".tmp"
    with open(tmp, "w") as f:
        json.dump({"api": url, "ctl": f"http://{args.host}:{ctl_port}", "pid": os.getpid(),
                   "sim_pid": sim.proc.pid if sim is not None else None}, f)
    os.replace(tmp, args.ready_file)
    stop = asyncio.Event()
    loop = asyncio.get_running_loop()
    import signal

    for sig in (signal.SIGTERM, signal.SIGINT):
        loop.add_signal_handler(sig, stop.set)
    sampler = cprof = None
    if os.environ.get("NEXUS_CLUSTER_PPROF"):
        from ..obs.pprof import Sampler

        sampler = Sampler(hz=199).start()
    if os.environ.get("NEXUS_CLUSTER_CPROFILE"):
        import cProfile

        cprof = state["cprof"] = cProfile.Profile()  # enabled by the first step (init excluded)
    await stop.wait()
    if sampler is not None:
        prof = sampler.stop()
        with open(os.environ["NEXUS_CLUSTER_PPROF"], "w") as f:
            f.write(prof.top(40))
    if cprof is not None:
        import io
        import pstats

        cprof.disable()
        buf = io.StringIO()
        pstats.Stats(cprof, stream=buf).sort_stats("tottime").print_stats(40)
        with open(os.environ["NEXUS_CLUSTER_CPROFILE"], "w") as f:
            f.write(buf.getvalue())
    await runner.cleanup()
    if api is not None:
        await api.stop()
    if simctl is not None:
        await simctl.close()
    if sim is not None:
        sim.stop()
    await store.close()


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=0)
    ap.add_argument("--cql", required=True)
    ap.add_argument("--ready-file", required=True)
    # watch-resume window per kind (the apiserver's watch cache): ~15 saturating steps of
    # backlog.  A bigger window only grows the simulator's heap line by line (each line a
    # fresh page-faulted allocation instead of a recycled one) and costs it throughput.
    ap.add_argument("--history", type=int, default=50_000)
    ap.add_argument("--flush-threads", type=int, default=1, help="simulator watch fan-out threads")
    ap.add_argument("--api-latency-us", type=int, default=0, help="simulated API answer latency (kubesim)")
    ap.add_argument("--write-qps", type=float, default=0.0, help="APF-like cap on mutating requests (kubesim)")
    ap.add_argument("--write-burst", type=int, default=0)
    ap.add_argument("--log-root", default="", help="kubesim: write LOG lines as CRI files here (/var/log/pods)")
    ap.add_argument("--api", choices=("kubesim", "python"), default="kubesim",
                    help="native apiserver simulator (default) or the Python fake")
    args = ap.parse_args(argv)
    asyncio.run(amain(args))
    return 0


if __name__ == "__main__":
    sys.exit(main())
