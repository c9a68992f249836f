"""Symbolise a native CPU-sampler dump (``NEXUS_KUBESIM_PROF=<file>``, see
``csrc/kubesim/kubesim.cpp`` ``namespace prof``) into flat / cumulative tables.

    python tools/native_prof.py <dump> [--top 30]

Each dump line is one sample: ``module+0xoffset`` frames, leaf first.  Offsets are
resolved with ``addr2line -f -C`` per module (one process per module).
"""
import argparse
import collections
import subprocess


def symbolise(frames):
    by_mod = collections.defaultdict(set)
    for fr in frames:
        mod, _, off = fr.rpartition("+")
        by_mod[mod].add(off)
    names = {}
    for mod, offs in by_mod.items():
        offs = sorted(offs)
        if mod == "?":
            names.update({f"?+{o}": f"?{o}" for o in offs})
            continue
        try:
            out = subprocess.run(["addr2line", "-f", "-C", "-e", mod, *offs], capture_output=True, text=True,
                                 timeout=120).stdout.splitlines()
        except (OSError, subprocess.TimeoutExpired):
            out = []
        short = mod.rsplit("/", 1)[-1]
        for i, o in enumerate(offs):
            fn = out[2 * i] if 2 * i < len(out) else "??"
            if fn == "??":
                fn = f"{short}+{o}"
            names[f"{mod}+{o}"] = fn[:110]
    return names


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dump")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--thread", choices=("all", "event-loop", "helper-thread"), default="all",
                    help="only the samples of the event loop / the apply and fan-out threads")
    a = ap.parse_args()
    samples = [line.split() for line in open(a.dump) if line.strip()]
    if a.thread != "all":
        samples = [s for s in samples if s and s[-1] == f"[{a.thread}]+0x0"]
    names = symbolise({f for s in samples for f in s})
    flat, cum = collections.Counter(), collections.Counter()
    for s in samples:
        syms = [names.get(f, f) for f in s]
        flat[syms[0]] += 1
        for fn in set(syms):
            cum[fn] += 1
    n = max(len(samples), 1)
    print(f"samples: {len(samples)}")
    print("   flat  flat%  function")
    for fn, c in flat.most_common(a.top):
        print(f"{c:7d} {100.0 * c / n:5.1f}%  {fn}")
    print("\n    cum   cum%  function")
    for fn, c in cum.most_common(a.top):
        print(f"{c:7d} {100.0 * c / n:5.1f}%  {fn}")


if __name__ == "__main__":
    main()
