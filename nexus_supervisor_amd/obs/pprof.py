"""Sampling profiler that writes pprof ``profile.proto`` (gzip).

The north star says the hot path (informer → classify → CQL write) is
"profiled with pprof rather than rocprof"; the reference itself exposes no
profiling (no ``net/http/pprof``, no HTTP server).  This sampler
walks the target thread's Python stack ``hz`` times a second from a background
thread and emits the standard pprof format (samples/count + cpu/nanoseconds,
function + line locations) so ``go tool pprof`` / ``pprof -top`` read it
directly.  The protobuf is hand-encoded (no generated code needed).
"""
from __future__ import annotations

import gzip
import signal
import sys
import threading
import time
from collections import Counter
from typing import Dict, List, Optional, Tuple

Frame = Tuple[str, str, int, int]  # (filename, function, first line, line)


def _varint(v: int) -> bytes:
    v &= (1 << 64) - 1
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _key(field: int, wt: int) -> bytes:
    return _varint((field << 3) | wt)


def _f_varint(field: int, v: int) -> bytes:
    return _key(field, 0) + _varint(v)


def _f_bytes(field: int, b: bytes) -> bytes:
    return _key(field, 2) + _varint(len(b)) + b


def _f_packed(field: int, vals) -> bytes:
    return _f_bytes(field, b"".join(_varint(v) for v in vals))


class Profile:
    """Aggregated stacks → profile.proto."""

    def __init__(self, period_ns: int):
        self.period_ns = period_ns
        self.stacks: Counter = Counter()
        self.start_ns = time.time_ns()
        self.duration_ns = 0

    def add(self, stack: Tuple[Frame, ...], n: int = 1) -> None:
        self.stacks[stack] += n

    def encode(self) -> bytes:
        strings: List[str] = [""]
        sidx: Dict[str, int] = {"": 0}

        def s(x: str) -> int:
            i = sidx.get(x)
            if i is None:
                i = sidx[x] = len(strings)
                strings.append(x)
            return i

        funcs: Dict[Tuple[str, str, int], int] = {}
        locs: Dict[Tuple[int, int], int] = {}
        out = bytearray()
        # sample_type: samples/count, cpu/nanoseconds
        out += _f_bytes(1, _f_varint(1, s("samples")) + _f_varint(2, s("count")))
        out += _f_bytes(1, _f_varint(1, s("cpu")) + _f_varint(2, s("nanoseconds")))
        func_msgs = bytearray()
        loc_msgs = bytearray()
        for stack, n in self.stacks.items():
            loc_ids = []
            for filename, name, first, line in stack:  # leaf first
                fk = (filename, name, first)
                fid = funcs.get(fk)
                if fid is None:
                    fid = funcs[fk] = len(funcs) + 1
                    func_msgs += _f_bytes(5, _f_varint(1, fid) + _f_varint(2, s(name)) + _f_varint(3, s(name))
                                          + _f_varint(4, s(filename)) + _f_varint(5, first))
                lk = (fid, line)
                lid = locs.get(lk)
                if lid is None:
                    lid = locs[lk] = len(locs) + 1
                    line_msg = _f_varint(1, fid) + _f_varint(2, line)
                    loc_msgs += _f_bytes(4, _f_varint(1, lid) + _f_bytes(4, line_msg))
                loc_ids.append(lid)
            out += _f_bytes(2, _f_packed(1, loc_ids) + _f_packed(2, [n, n * self.period_ns]))
        out += loc_msgs
        out += func_msgs
        for st in strings:
            out += _f_bytes(6, st.encode())
        out += _f_varint(9, self.start_ns)
        out += _f_varint(10, self.duration_ns)
        out += _f_bytes(11, _f_varint(1, sidx["cpu"]) + _f_varint(2, sidx["nanoseconds"]))
        out += _f_varint(12, self.period_ns)
        out += _f_varint(14, sidx["cpu"])
        return bytes(out)

    def encode_gz(self) -> bytes:
        return gzip.compress(self.encode())

    def top(self, n: int = 25) -> str:
        """Flat + cumulative table (what ``pprof -top`` shows), for committed summaries."""
        total = sum(self.stacks.values()) or 1
        flat: Counter = Counter()
        cum: Counter = Counter()
        for stack, c in self.stacks.items():
            if stack:
                flat[_fmt(stack[0])] += c
            for fr in set(_fmt(f) for f in stack):
                cum[fr] += c
        lines = [f"samples: {total}  period: {self.period_ns / 1e6:.2f} ms  duration: {self.duration_ns / 1e9:.2f} s",
                 f"{'flat':>8} {'flat%':>6} {'cum':>8} {'cum%':>6}  function"]
        for fn, c in flat.most_common(n):
            lines.append(f"{c:8d} {100 * c / total:5.1f}% {cum[fn]:8d} {100 * cum[fn] / total:5.1f}%  {fn}")
        lines.append("")
        lines.append("top cumulative:")
        for fn, c in cum.most_common(n):
            lines.append(f"{c:8d} {100 * c / total:5.1f}%  {fn}")
        return "\n".join(lines)


def _fmt(fr: Frame) -> str:
    filename, name, _first, _line = fr
    short = filename.rsplit("/site-packages/", 1)[-1].rsplit("/repo/", 1)[-1]
    return f"{name} ({short})"


class Sampler:
    """Samples one thread's stack at ``hz`` into a :class:`Profile`.

    ``mode="signal"`` (the default when started on the main thread for the main thread):
    ``ITIMER_PROF`` delivers SIGPROF every 1/hz s of *process CPU time* and the handler
    records the interrupted frame.  CPython runs a signal handler only between bytecodes,
    so the ticks that fall inside one long C call (the native watch decoder, a socket
    write) coalesce into a single delivery; each sample is therefore weighted by the
    thread CPU time since the previous one, in sampling periods (profiles/r2: unweighted,
    12 workers at 499 Hz kept ~2.8k of ~15k ticks each and under-counted native calls).
    ``mode="thread"``: a sampler thread reads ``sys._current_frames()`` on a wall clock;
    it only gets the GIL when the target releases it, so it over-samples frames that sit
    in syscalls (socket writes, epoll) — use it for non-main threads only.
    """

    def __init__(self, hz: int = 97, thread_id: Optional[int] = None, max_depth: int = 64, mode: str = "auto"):
        self.hz = max(1, hz)
        self.thread_id = thread_id if thread_id is not None else threading.main_thread().ident
        self.max_depth = max_depth
        self.profile = Profile(int(1e9 / self.hz))
        self._stop = threading.Event()
        self._t: Optional[threading.Thread] = None
        self._t0 = 0.0
        on_main = threading.current_thread() is threading.main_thread()
        target_main = self.thread_id == threading.main_thread().ident
        if mode == "auto":
            mode = "signal" if (on_main and target_main and hasattr(signal, "setitimer")) else "thread"
        self.mode = mode
        self._prev_handler = None
        self._period = 1.0 / self.hz
        self._last_cpu = 0.0

    def start(self) -> "Sampler":
        self._t0 = time.monotonic()
        self._last_cpu = time.thread_time()
        if self.mode == "signal":
            self._prev_handler = signal.signal(signal.SIGPROF, self._on_signal)
            period = 1.0 / self.hz
            signal.setitimer(signal.ITIMER_PROF, period, period)
            return self
        self._t = threading.Thread(target=self._loop, name="pprof-sampler", daemon=True)
        self._t.start()
        return self

    def stop(self) -> Profile:
        if self.mode == "signal":
            signal.setitimer(signal.ITIMER_PROF, 0, 0)
            if self._prev_handler is not None:
                signal.signal(signal.SIGPROF, self._prev_handler)
                self._prev_handler = None
        self._stop.set()
        if self._t is not None:
            self._t.join()
        self.profile.duration_ns = int((time.monotonic() - self._t0) * 1e9)
        return self.profile

    def _record(self, frame, n: int = 1) -> None:
        stack = []
        f = frame
        while f is not None and len(stack) < self.max_depth:
            co = f.f_code
            stack.append((co.co_filename, co.co_name, co.co_firstlineno, f.f_lineno or 0))
            f = f.f_back
        if stack:
            self.profile.add(tuple(stack), n)

    def _on_signal(self, signum, frame) -> None:
        now = time.thread_time()
        n = max(1, int((now - self._last_cpu) / self._period + 0.5))
        self._last_cpu = now
        self._record(frame, n)

    def _loop(self) -> None:
        period = 1.0 / self.hz
        nxt = time.monotonic()
        tid = self.thread_id
        while not self._stop.is_set():
            frame = sys._current_frames().get(tid)  # noqa: SLF001
            if frame is not None:
                self._record(frame)
            del frame
            nxt += period
            delay = nxt - time.monotonic()
            if delay > 0:
                self._stop.wait(delay)
            else:
                nxt = time.monotonic()


def profile_for(seconds: float, hz: int = 97, thread_id: Optional[int] = None) -> Profile:
    s = Sampler(hz, thread_id).start()
    time.sleep(seconds)
    return s.stop()


def decode_profile(data: bytes) -> Dict[str, object]:
    """Minimal protobuf reader for tests: string table + sample count + locations."""
    if data[:2] == b"\x1f\x8b":
        data = gzip.decompress(data)

    def read_varint(b, i):
        shift = v = 0
        while True:
            c = b[i]
            i += 1
            v |= (c & 0x7F) << shift
            if not c & 0x80:
                return v, i
            shift += 7

    def fields(b):
        i = 0
        while i < len(b):
            k, i = read_varint(b, i)
            f, wt = k >> 3, k & 7
            if wt == 0:
                v, i = read_varint(b, i)
                yield f, v
            elif wt == 2:
                ln, i = read_varint(b, i)
                yield f, b[i:i + ln]
                i += ln
            else:
                raise ValueError(f"unsupported wire type {wt}")

    strings, samples, locations, functions = [], 0, 0, 0
    values = 0
    period = 0
    for f, v in fields(data):
        if f == 6:
            strings.append(v.decode())
        elif f == 2:
            samples += 1
            for sf, sv in fields(v):
                if sf == 2:
                    j = 0
                    first = True
                    while j < len(sv):
                        x, j = read_varint(sv, j)
                        if first:
                            values += x
                            first = False
        elif f == 4:
            locations += 1
        elif f == 5:
            functions += 1
        elif f == 12:
            period = v
    return {"strings": strings, "samples": samples, "sample_count": values, "locations": locations,
            "functions": functions, "period": period}


def _pb_fields(b: bytes):
    i = 0
    while i < len(b):
        k, i = _read_varint(b, i)
        f, wt = k >> 3, k & 7
        if wt == 0:
            v, i = _read_varint(b, i)
            yield f, v
        elif wt == 2:
            ln, i = _read_varint(b, i)
            yield f, b[i:i + ln]
            i += ln
        else:
            raise ValueError(f"unsupported wire type {wt}")


def _read_varint(b: bytes, i: int):
    shift = v = 0
    while True:
        c = b[i]
        i += 1
        v |= (c & 0x7F) << shift
        if not c & 0x80:
            return v, i
        shift += 7


def _packed(v) -> List[int]:
    if isinstance(v, int):
        return [v]
    out, j = [], 0
    while j < len(v):
        x, j = _read_varint(v, j)
        out.append(x)
    return out


def load_profile(data: bytes) -> Profile:
    """Decode a profile written by :meth:`Profile.encode` back into stacks (merging)."""
    if data[:2] == b"\x1f\x8b":
        data = gzip.decompress(data)
    strings: List[str] = []
    funcs: Dict[int, Tuple[int, int, int]] = {}
    locs: Dict[int, Tuple[int, int]] = {}
    samples: List[Tuple[List[int], int]] = []
    period = duration = 0
    for f, v in _pb_fields(data):
        if f == 6:
            strings.append(v.decode())
        elif f == 2:
            ids: List[int] = []
            n = 0
            for sf, sv in _pb_fields(v):
                if sf == 1:
                    ids += _packed(sv)
                elif sf == 2:
                    n = _packed(sv)[0]
            samples.append((ids, n))
        elif f == 4:
            lid = fid = line = 0
            for sf, sv in _pb_fields(v):
                if sf == 1:
                    lid = sv
                elif sf == 4:
                    for lf, lv in _pb_fields(sv):
                        if lf == 1:
                            fid = lv
                        elif lf == 2:
                            line = lv
            locs[lid] = (fid, line)
        elif f == 5:
            fid = name = fname = first = 0
            for sf, sv in _pb_fields(v):
                if sf == 1:
                    fid = sv
                elif sf == 2:
                    name = sv
                elif sf == 4:
                    fname = sv
                elif sf == 5:
                    first = sv
            funcs[fid] = (name, fname, first)
        elif f == 10:
            duration = v
        elif f == 12:
            period = v
    prof = Profile(period or 1)
    prof.duration_ns = duration
    for ids, n in samples:
        stack = []
        for lid in ids:
            fid, line = locs[lid]
            name, fname, first = funcs[fid]
            stack.append((strings[fname], strings[name], first, line))
        prof.add(tuple(stack), n)
    return prof


def merge_profiles(profiles) -> Profile:
    """Sum several profiles (e.g. every shard worker of a replica) into one."""
    profiles = list(profiles)
    out = Profile(profiles[0].period_ns if profiles else 1)
    for p in profiles:
        out.stacks.update(p.stacks)
        out.duration_ns = max(out.duration_ns, p.duration_ns)
    return out
