"""``obs/loopwatch.py``: the opt-in slow-callback watch behind ``bench.py
--diag-slow-callback-ms`` — which callbacks held a process's loop at least the threshold."""
import asyncio
import asyncio.events
import time

from nexus_supervisor_amd.obs import loopwatch
from nexus_supervisor_amd.obs.metrics import Metrics


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
