"""Sum pprof profiles (e.g. the shard workers of one replica) and print the top table.

    python tools/pprof_merge.py OUT.top.txt PROFILE.pb.gz [PROFILE.pb.gz ...]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nexus_supervisor_amd.obs.pprof import load_profile, merge_profiles  # noqa: E402


def main(argv) -> int:
    out, paths = argv[0], argv[1:]
    profs = []
    for p in paths:
        with open(p, "rb") as f:
            profs.append(load_profile(f.read()))
    merged = merge_profiles(profs)
    per = [sum(p.stacks.values()) for p in profs]
    text = f"merged {len(profs)} profiles; samples per profile: min {min(per)} max {max(per)}\n" + merged.top(60)
    with open(out, "w") as f:
        f.write(text + "\n")
    print(text[:2000])
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
