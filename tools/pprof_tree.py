"""Where does a function's time go?  Sums pprof profiles (e.g. every shard worker of a
run) and prints, for each function matching ROOT, its callees by cumulative samples and
the root's own lines by flat samples.

    python tools/pprof_tree.py ROOT PROFILE.pb.gz [PROFILE.pb.gz ...] [--depth N]

ROOT matches the function name, or ``name@file-substring``.  ``--depth N`` expands the
callee table N levels (default 1).
"""
import os
import sys
from collections import Counter

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nexus_supervisor_amd.obs.pprof import load_profile, merge_profiles  # noqa: E402


def _match(fr, root: str) -> bool:
    name, _, file_part = root.partition("@")
    return fr[1] == name and (not file_part or file_part in fr[0])


def _short(fr) -> str:
    return f"{fr[1]} ({fr[0].rsplit('/repo/', 1)[-1].rsplit('/python3.10/', 1)[-1]})"


def tree(prof, root: str, depth: int = 1):
    total = 0
    callees: Counter = Counter()
    lines: Counter = Counter()
    for stack, c in prof.stacks.items():
        # leaf first: the outermost matching frame owns the sample (no double count on recursion)
        idx = [i for i, fr in enumerate(stack) if _match(fr, root)]
        if not idx:
            continue
        i = idx[-1]
        total += c
        lines[stack[i][3]] += c
        path = tuple(_short(stack[j]) for j in range(i - 1, max(i - 1 - depth, -1), -1))
        callees[path or ("<self>",)] += c
    return total, callees, lines


def main(argv) -> int:
    depth = 1
    if "--depth" in argv:
        k = argv.index("--depth")
        depth = int(argv[k + 1])
        argv = argv[:k] + argv[k + 2:]
    root, paths = argv[0], argv[1:]
    profs = []
    for p in paths:
        with open(p, "rb") as f:
            profs.append(load_profile(f.read()))
    merged = merge_profiles(profs)
    all_samples = sum(merged.stacks.values()) or 1
    total, callees, lines = tree(merged, root, depth)
    print(f"{root}: {total} samples, {100 * total / all_samples:.1f}% of all")
    for path, c in callees.most_common(40):
        print(f"{c:8d} {100 * c / max(total, 1):5.1f}%  {' > '.join(path)}")
    print("by line of the root (inclusive):")
    for ln, c in lines.most_common(15):
        print(f"{c:8d} {100 * c / max(total, 1):5.1f}%  line {ln}")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
