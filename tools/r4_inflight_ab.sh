#!/bin/bash
# Steps in flight (bench.py --inflight) 4 vs 8: is the saturated line capacity-bound or
# pipeline-bound?  Driver-like runs, probe off, interleaved on one box.
set -o pipefail
OUT=${OUT:-gpurun_out/r4_inflight_ab}
N=${N:-3}
mkdir -p "$OUT"
for i in $(seq 1 "$N"); do
  for f in 4 8; do
    echo "== inflight $f run $i"
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --inflight "$f" --probe-events 0 \
      > "$OUT/inflight${f}_$i.json" 2> "$OUT/inflight${f}_$i.err" || exit 1
  done
done
