#!/bin/bash
# Shard-worker count on the final tree (default-pod HBM shape): 6 / 8 / 10 workers,
# interleaved, two rounds, driver-like runs.  Each step under its own time limit; the first
# failure ends the batch.
set -o pipefail
OUT=${OUT:-gpurun_out/r4_sweep_final}
mkdir -p "$OUT"
for r in 1 2; do
  for p in 6 8 10; do
    echo "== procs $p round $r"
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --procs "$p" --probe-events 0 \
      > "$OUT/procs${p}_$r.json" 2> "$OUT/procs${p}_$r.err" || exit 1
  done
done
