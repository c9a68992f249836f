"""HTTP observability endpoints (absent in the reference: its Deployment defines no
ports and no probes, ``/root/reference/.helm/templates/deployment.yaml:37-120``).

``/metrics``               Prometheus text exposition (counters, gauges, latency histograms)
``/healthz``               liveness: the event loop answers and workers are alive
``/readyz``                readiness: informer caches synced (and, with leader election, reports role)
``/debug/pprof/profile``   ``?seconds=N`` sampling profile in pprof ``profile.proto`` (gzip)
``/debug/pprof/top``       same sample, rendered as a flat/cumulative text table
``/debug/vars``            JSON snapshot: pipeline stats, store stats, queue depth, leadership
``/debug/heap``            heap census of this process (Go's ``/debug/pprof/heap`` role): RSS, live
                           objects by type and dict shape, the supervisor's bounded caches, and
                           with ``PYTHONTRACEMALLOC`` set the top allocation sites (``?top=N``)
"""
from __future__ import annotations

import asyncio
import threading
from typing import Optional

from aiohttp import web

from .pprof import Sampler


class ObsServer:
    def __init__(self, app):
        self.app = app
        self._runner: Optional[web.AppRunner] = None
        self.port = 0
        self._loop_thread = threading.get_ident()

    async def _metrics(self):
        pool = getattr(self.app, "pool", None)
        if pool is not None:  # process-per-core replica: merge the shard workers' registries
            await pool.refresh_metrics(2.0)
            m = pool.merged_metrics(self.app.metrics)
            m.set("active", 1.0 if pool.active else 0.0)
            m.set("worker_processes_alive", sum(1 for w in pool.workers if w.proc is not None and w.proc.poll() is None))
            return m
        from ..parallel.workers import collect_gauges

        collect_gauges(self.app.supervisor, self.app.metrics)
        return self.app.metrics

    async def h_metrics(self, req):
        m = await self._metrics()
        return web.Response(text=m.prometheus_text(), content_type="text/plain", charset="utf-8",
                            headers={"X-Content-Type-Options": "nosniff"})

    async def h_healthz(self, req):
        pool = getattr(self.app, "pool", None)
        if pool is not None:
            ok = pool.alive()
            return web.Response(status=200 if ok else 503, text="ok" if ok else "worker process exited")
        sup = self.app.supervisor
        ok = sup.pipeline is not None and any(not t.done() for t in sup.pipeline._tasks)  # noqa: SLF001
        return web.Response(status=200 if ok else 503, text="ok" if ok else "workers stopped")

    async def h_readyz(self, req):
        ready = self.app.ready()
        role = "leader" if self.app.supervisor.active else "standby"
        return web.Response(status=200 if ready else 503, text=f"{'ready' if ready else 'syncing'} ({role})")

    async def _sample(self, req) -> "Sampler":
        seconds = min(float(req.query.get("seconds", "10")), 120.0)
        hz = int(req.query.get("hz", str(self.app.cfg.observability.profiler_hz)))
        s = Sampler(hz, thread_id=self._loop_thread).start()
        await asyncio.sleep(seconds)
        s.stop()
        return s

    async def h_profile(self, req):
        s = await self._sample(req)
        return web.Response(body=s.profile.encode_gz(), content_type="application/octet-stream",
                            headers={"Content-Disposition": 'attachment; filename="profile.pb.gz"'})

    async def h_top(self, req):
        s = await self._sample(req)
        return web.Response(text=s.profile.top(int(req.query.get("n", "30"))))

    async def h_vars(self, req):
        pool = getattr(self.app, "pool", None)
        if pool is not None:
            m = await self._metrics()
            doc = {"active": pool.active, "worker_processes": pool.count, "restarts": pool.restarts,
                   "workers": [{"index": w.index, "pid": w.proc.pid if w.proc else None, "synced": w.synced.is_set(),
                                "alive": w.proc is not None and w.proc.poll() is None} for w in pool.workers],
                   "metrics": m.snapshot()}
            if self.app.elector is not None:
                doc["leader"] = {"identity": self.app.elector.identity, "leader": self.app.elector.leader,
                                 "observed_holder": self.app.elector.observed_holder}
            return web.json_response(doc, dumps=lambda o: __import__("json").dumps(o, default=str))
        sup = self.app.supervisor
        doc = {"active": sup.active, "namespace": sup.namespace,
               "pipeline": sup.pipeline.stats.as_dict() if sup.pipeline else {},
               "queue_depth": sup.pipeline.depth() if sup.pipeline else 0,
               "informers": {k: {"objects": len(i.indexer), "relists": i.relists, "watch_events": i.watch_events}
                             for k, i in sup.factory.informers.items()},
               "metrics": self.app.metrics.snapshot()}
        store = self.app.store
        sess = getattr(store, "session", None)
        if sess is not None:
            doc["cql"] = dict(sess.stats, hosts={f"{h.address[0]}:{h.address[1]}": h.up for h in sess.hosts.values()})
        if self.app.elector is not None:
            doc["leader"] = {"identity": self.app.elector.identity, "leader": self.app.elector.leader,
                             "observed_holder": self.app.elector.observed_holder}
        return web.json_response(doc, dumps=lambda o: __import__("json").dumps(o, default=str))

    async def h_heap(self, req):
        import json

        from .heap import census

        top = int(req.query.get("top", "25"))
        sup = getattr(self.app, "supervisor", None)
        doc = census(sup, top=top, trim=req.query.get("trim") == "1")
        probe = req.query.get("retainers")
        if probe:
            from .heap import retainers

            doc["retainers"] = retainers(sup, probe)
        return web.Response(text=json.dumps(doc, indent=1, default=str), content_type="application/json")

    async def start(self, host: str, port: int) -> int:
        self._loop_thread = threading.get_ident()
        app = web.Application()
        app.router.add_get("/metrics", self.h_metrics)
        app.router.add_get("/healthz", self.h_healthz)
        app.router.add_get("/readyz", self.h_readyz)
        app.router.add_get("/debug/pprof/profile", self.h_profile)
        app.router.add_get("/debug/pprof/top", self.h_top)
        app.router.add_get("/debug/vars", self.h_vars)
        app.router.add_get("/debug/heap", self.h_heap)
        self._runner = web.AppRunner(app, access_log=None)
        await self._runner.setup()
        site = web.TCPSite(self._runner, host, port)
        await site.start()
        self.port = site._server.sockets[0].getsockname()[1]  # noqa: SLF001
        return self.port

    async def stop(self) -> None:
        if self._runner is not None:
            await self._runner.cleanup()
            self._runner = None
