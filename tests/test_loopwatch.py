"""``obs/loopwatch.py``: the opt-in slow-callback watch behind ``bench.py
--diag-slow-callback-ms`` — which callbacks held a process's loop at least the threshold."""
import asyncio
import asyncio.events
import gc
import time

import pytest

from nexus_supervisor_amd.obs import loopwatch
from nexus_supervisor_amd.obs.metrics import Metrics


@pytest.fixture(autouse=True)
def _drop_gc_hook(monkeypatch):
    monkeypatch.setattr(loopwatch, "_GC_HOOK", None)
    yield
    if loopwatch._GC_HOOK in gc.callbacks:
        gc.callbacks.remove(loopwatch._GC_HOOK)


def test_slow_callbacks_are_counted_by_name(monkeypatch):
    monkeypatch.setattr(asyncio.events.Handle, "_run", asyncio.events.Handle._run)  # restored afterwards
    monkeypatch.setattr(loopwatch, "_INSTALLED", False)
    m = Metrics("t")
    assert loopwatch.install(m, 2.0, "worker")
    assert not loopwatch.install(m, 2.0, "worker")  # once per process

    def slow():
        time.sleep(0.004)

    def fast():
        pass

    async def busy():
        time.sleep(0.004)

    async def go():
        loop = asyncio.get_running_loop()
        loop.call_soon(slow)
        loop.call_soon(fast)
        await asyncio.ensure_future(busy())
        await asyncio.sleep(0.01)

    asyncio.run(go())
    counts = {dict(k)["name"]: v for k, v in m.counters["slow_callbacks"].items()}
    assert counts.get("test_slow_callbacks_are_counted_by_name.<locals>.slow") == 1
    assert counts.get("task:test_slow_callbacks_are_counted_by_name.<locals>.busy") == 1
    assert not any("fast" in k for k in counts)
    assert all(dict(k)["where"] == "worker" for k in m.counters["slow_callbacks"])
    secs = sum(m.counters["slow_callback_seconds"].values())
    assert 0.007 < secs < 0.5
    assert m.histogram("slow_callback").total == 2


def test_gc_time_inside_slow_callbacks(monkeypatch):
    monkeypatch.setattr(asyncio.events.Handle, "_run", asyncio.events.Handle._run)
    monkeypatch.setattr(loopwatch, "_INSTALLED", False)
    m = Metrics("t")
    assert loopwatch.install(m, 1.0, "parent")

    def collects():
        junk = []
        for _ in range(20000):  # reference cycles for the collector to walk
            a = []
            a.append(a)
            junk.append(a)
        del junk
        gc.collect()
        time.sleep(0.002)

    def plain():
        time.sleep(0.002)

    async def go():
        loop = asyncio.get_running_loop()
        loop.call_soon(collects)
        loop.call_soon(plain)
        await asyncio.sleep(0.01)

    asyncio.run(go())
    gc_ms = {dict(k)["name"].rsplit(".", 1)[-1]: v * 1e3 for k, v in m.counters["slow_callback_gc_seconds"].items()}
    assert gc_ms["collects"] > 0.0
    assert gc_ms["plain"] == 0.0


def test_install_from_env(monkeypatch):
    monkeypatch.setattr(asyncio.events.Handle, "_run", asyncio.events.Handle._run)
    monkeypatch.setattr(loopwatch, "_INSTALLED", False)
    m = Metrics("t")
    monkeypatch.delenv("NEXUS_SLOW_CALLBACK_MS", raising=False)
    assert loopwatch.install_from_env(m) is None
    monkeypatch.setenv("NEXUS_SLOW_CALLBACK_MS", "bogus")
    assert loopwatch.install_from_env(m) is None
    monkeypatch.setenv("NEXUS_SLOW_CALLBACK_MS", "0.5")
    assert loopwatch.install_from_env(m, "parent") == 0.5


def test_names_never_raise():
    class Coro:  # a compiled module's finished coroutine: no name to report
        def __getattribute__(self, name):
            if name in ("__qualname__", "__name__"):
                return None
            return object.__getattribute__(self, name)

    class NoName:
        def get_coro(self):
            return Coro()

    class H:
        def __init__(self, cb):
            self._callback = cb

    assert loopwatch._name(H(NoName().get_coro)).startswith("task:")

    class Broken:
        @property
        def __self__(self):
            raise RuntimeError("boom")

    assert loopwatch._name(H(Broken())) == "?"


def test_bench_slow_callback_rows_carry_gc_time():
    from nexus_supervisor_amd.bench.runner import _slow_callbacks

    k = frozenset({"name": "task:WatchHub._pump", "where": "parent"}.items())
    before = {"slow_callbacks": {k: 2.0}, "slow_callback_seconds": {k: 0.002}, "slow_callback_gc_seconds": {k: 0.0}}
    after = {"slow_callbacks": {k: 5.0}, "slow_callback_seconds": {k: 0.0062}, "slow_callback_gc_seconds": {k: 0.003}}
    (row,) = _slow_callbacks(before, after)
    assert row == {"where": "parent", "name": "task:WatchHub._pump", "count": 3, "total_ms": 4.2, "gc_ms": 3.0}
