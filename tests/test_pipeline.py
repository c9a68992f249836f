"""Keyed pipeline: per-key ordering, coalescing, backoff, dead-letter, rate limit."""
import asyncio
import time
from dataclasses import dataclass

import pytest

from nexus_supervisor_amd.parallel.pipeline import PipelineStage
from nexus_supervisor_amd.parallel.ratelimit import ExponentialBackoff, TokenBucket


@dataclass
class Item:
    key: tuple
    val: int
    action: str = "a"


def test_token_bucket_rate():
    t = [0.0]
    b = TokenBucket(10, 5, clock=lambda: t[0])
    waits = [b.reserve() for _ in range(7)]
    assert waits[:5] == [0, 0, 0, 0, 0]
    assert waits[5] == pytest.approx(0.1) and waits[6] == pytest.approx(0.2)
    t[0] = 10.0
    assert b.reserve() == 0
    assert TokenBucket(0, 1).reserve() == 0  # unlimited


def test_exponential_backoff():
    b = ExponentialBackoff(0.1, 1.0)
    assert [b.when("k") for _ in range(6)] == pytest.approx([0.1, 0.2, 0.4, 0.8, 1.0, 1.0])
    b.forget("k")
    assert b.when("k") == pytest.approx(0.1)


def test_per_key_order_and_parallel_keys(arun):
    seen = []
    inflight = {}
    max_conc = [0]

    async def proc(it):
        inflight[it.key] = inflight.get(it.key, 0) + 1
        assert inflight[it.key] == 1, "same key processed concurrently"
        max_conc[0] = max(max_conc[0], sum(inflight.values()))
        await asyncio.sleep(0.001)
        seen.append((it.key, it.val))
        inflight[it.key] -= 1
        return it.val

    async def go():
        p = PipelineStage("t", proc, workers=8, elements_per_second=0, burst=1, key_fn=lambda x: x.key)
        await p.start()
        for v in range(20):
            for k in range(5):
                p.receive(Item((k,), v))
        assert await p.join(5)
        await p.stop()
        return p

    p = arun(go())
    for k in range(5):
        vals = [v for kk, v in seen if kk == (k,)]
        assert vals == list(range(20))
    assert max_conc[0] > 1
    assert p.stats.processed == 100


def test_coalescing(arun):
    calls = []

    async def proc(it):
        calls.append(it)
        await asyncio.sleep(0.01)

    async def go():
        p = PipelineStage("t", proc, workers=1, elements_per_second=0, burst=1, key_fn=lambda x: x.key,
                          coalesce_key=lambda x: x.action)
        await p.start()
        p.receive(Item(("k",), 1, "fail"))
        await asyncio.sleep(0.002)  # first is in flight; the next three coalesce into one
        p.receive(Item(("k",), 2, "run"))
        p.receive(Item(("k",), 3, "run"))
        p.receive(Item(("k",), 4, "run"))
        assert await p.join(5)
        await p.stop()
        return p

    p = arun(go())
    assert [c.val for c in calls] == [1, 2]
    assert p.stats.coalesced == 2


def test_retry_blocks_key_then_succeeds(arun):
    attempts = {}
    order = []

    async def proc(it):
        attempts[it.val] = attempts.get(it.val, 0) + 1
        if it.val == 1 and attempts[1] < 3:
            raise RuntimeError("transient")
        order.append(it.val)

    async def go():
        p = PipelineStage("t", proc, workers=4, elements_per_second=0, burst=1, base_delay=0.01, max_delay=0.02,
                          key_fn=lambda x: x.key)
        await p.start()
        p.receive(Item(("k",), 1))
        p.receive(Item(("k",), 2))
        assert await p.join(5)
        await p.stop()
        return p

    p = arun(go())
    assert order == [1, 2]
    assert attempts[1] == 3 and p.stats.retries == 2


def test_dead_letter(arun):
    dead = []

    async def proc(it):
        raise RuntimeError("poison")

    async def go():
        p = PipelineStage("t", proc, workers=2, elements_per_second=0, burst=1, base_delay=0.001, max_delay=0.002,
                          max_retries=3, key_fn=lambda x: x.key, on_dead_letter=lambda it, e: dead.append(it.val))
        await p.start()
        p.receive(Item(("k",), 7))
        assert await p.join(5)
        await p.stop()
        return p

    p = arun(go())
    assert dead == [7] and p.stats.dead_lettered == 1 and p.stats.failed_attempts == 4


def test_rate_limit_applies(arun):
    async def proc(it):
        return None

    async def go():
        p = PipelineStage("t", proc, workers=4, elements_per_second=100, burst=5, key_fn=lambda x: x.key)
        await p.start()
        t0 = time.monotonic()
        for i in range(25):
            p.receive(Item((i,), i))
        assert await p.join(5)
        dt = time.monotonic() - t0
        await p.stop()
        return dt

    dt = arun(go())
    assert dt >= 0.15  # 20 tokens beyond the burst at 100/s


def test_stop_drains(arun):
    done = []

    async def proc(it):
        await asyncio.sleep(0.005)
        done.append(it.val)

    async def go():
        p = PipelineStage("t", proc, workers=2, elements_per_second=0, burst=1, key_fn=lambda x: x.key)
        await p.start()
        for i in range(10):
            p.receive(Item((i,), i))
        await p.stop(drain=True, timeout=5)
        assert not p.receive(Item((99,), 99))

    arun(go())
    assert sorted(done) == list(range(10))
