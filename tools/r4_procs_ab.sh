#!/bin/bash
# 6 vs 8 shard workers with the latency probe on: driver-like runs interleaved on one box.
set -o pipefail
OUT=${OUT:-gpurun_out/r4_procs_ab}
N=${N:-3}
mkdir -p "$OUT"
for i in $(seq 1 "$N"); do
  for p in 6 8; do
    echo "== procs $p run $i"
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --procs "$p" \
      > "$OUT/procs${p}_$i.json" 2> "$OUT/procs${p}_$i.err" || exit 1
  done
done
