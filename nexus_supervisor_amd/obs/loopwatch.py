"""Opt-in event-loop watch: which callbacks hold a process's loop for longer than a
threshold (``NEXUS_SLOW_CALLBACK_MS``).

A watch line that reaches a worker while its loop runs something else waits for it; the
bench probe's delivery split (:mod:`.delivery`) shows *that* a stage was late, this shows
*what* held the loop.  :func:`install` wraps ``asyncio.Handle._run`` (every callback and
task step of the process's loops): one ``perf_counter`` pair per callback — a diagnostic,
not for production — and for each callback at or over the threshold increments
``slow_callbacks{name, where}`` / ``slow_callback_seconds{name, where}`` and records its
duration in the ``slow_callback`` histogram.  ``slow_callback_gc_seconds{name, where}`` is
the part of those callbacks the cyclic garbage collector ran in (a ``gc.callbacks`` clock):
a collection triggered by whatever allocation crossed the threshold holds the loop as
long as the callback's own work.
asyncio's own debug mode does the same but slows every coroutine down.
"""
from __future__ import annotations

import asyncio.events as _events
import gc
import os
import time
from typing import Optional

_INSTALLED = False
_GC_HOOK = None  # the gc.callbacks entry of install()


def _name(handle) -> str:
    """A readable name of what a handle runs; never raises (a compiled module's finished
    coroutine may report no ``__qualname__``)."""
    try:
        cb = handle._callback
        owner = getattr(cb, "__self__", None)
        if owner is not None and hasattr(owner, "get_coro"):  # a Task step: the coroutine's name
            coro = owner.get_coro()
            q = getattr(coro, "__qualname__", None) or getattr(coro, "__name__", None) or type(coro).__name__
            return f"task:{q}"
        name = getattr(cb, "__qualname__", None) or getattr(cb, "__name__", None) or type(cb).__name__
        return name if owner is None else f"{type(owner).__name__}.{str(name).rsplit('.', 1)[-1]}"
    except Exception:  # noqa: BLE001 - a diagnostic must never take the loop down
        return "?"


def install(metrics, threshold_ms: float, where: str = "") -> bool:
    """Watch every loop of this process (``where`` labels it: the replica parent's watch hub
    or a shard worker); False when already installed or disabled."""
    global _INSTALLED, _GC_HOOK
    if _INSTALLED or threshold_ms <= 0:
        return False
    threshold = threshold_ms / 1000.0
    orig = _events.Handle._run
    # NEXUS_SLOW_CALLBACK_LOG=1: also one stderr line per slow callback, with its
    # CLOCK_MONOTONIC end time (lines up with the bench's push stamps across processes)
    log_each = os.environ.get("NEXUS_SLOW_CALLBACK_LOG", "") not in ("", "0")
    clock = time.perf_counter
    gc_s = [0.0, 0.0]  # [GC seconds so far, start of the running collection]

    def _gc_clock(phase, _info):
        if phase == "start":
            gc_s[1] = clock()
        else:
            gc_s[0] += clock() - gc_s[1]

    def _run(self):
        g0 = gc_s[0]
        t0 = clock()
        orig(self)
        d = clock() - t0
        if d >= threshold:
            try:
                labels = {"name": _name(self), "where": where}
                metrics.inc("slow_callbacks", labels=labels)
                metrics.inc("slow_callback_seconds", d, labels=labels)
                metrics.inc("slow_callback_gc_seconds", gc_s[0] - g0, labels=labels)
                metrics.observe_seconds("slow_callback", d)
                if log_each:
                    import sys

                    owner = getattr(self._callback, "__self__", None)
                    task = owner.get_name() if hasattr(owner, "get_name") else ""
                    sys.stderr.write(f"SLOWCB {time.monotonic():.4f} {where} pid={os.getpid()} {labels['name']} "
                                     f"{task} {d * 1e3:.2f}ms gc={(gc_s[0] - g0) * 1e3:.2f}ms\n")
            except Exception:  # noqa: BLE001 - never let the watch break the loop it watches
                pass

    gc.callbacks.append(_gc_clock)
    _GC_HOOK = _gc_clock
    _events.Handle._run = _run
    _INSTALLED = True
    return True


def install_from_env(metrics, where: str = "") -> Optional[float]:
    """:func:`install` with ``NEXUS_SLOW_CALLBACK_MS`` (unset or 0: nothing)."""
    raw = os.environ.get("NEXUS_SLOW_CALLBACK_MS", "")
    try:
        ms = float(raw) if raw else 0.0
    except ValueError:
        return None
    return ms if install(metrics, ms, where) else None
