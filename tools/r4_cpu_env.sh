#!/bin/bash
# The box's CPU share as the bench sees it: affinity, cgroup CPU quota and throttling
# counters around one driver-like bench run (is a tail a CFS throttle?).
set -o pipefail
OUT=${OUT:-gpurun_out/r4_cpu_env}
mkdir -p "$OUT"
{
  echo "nproc=$(nproc)"
  python -c 'import os; print("affinity", len(os.sched_getaffinity(0)), "cpu_count", os.cpu_count())'
  for f in /sys/fs/cgroup/cpu.max /sys/fs/cgroup/cpu.weight /sys/fs/cgroup/cpuset.cpus.effective; do
    [ -r "$f" ] && echo "$f: $(tr '\n' ' ' < "$f")"
  done
  echo "cpu.stat before:"; [ -r /sys/fs/cgroup/cpu.stat ] && cat /sys/fs/cgroup/cpu.stat
  lscpu | grep -E '^(Model name|Thread|Core|Socket|CPU\(s\)|NUMA node\(s\)|CPU max MHz|CPU min MHz)' || true
} > "$OUT/env.txt" 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 1
{ echo "cpu.stat after:"; [ -r /sys/fs/cgroup/cpu.stat ] && cat /sys/fs/cgroup/cpu.stat; } >> "$OUT/env.txt" 2>&1
cat "$OUT/env.txt"
