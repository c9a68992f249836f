#!/bin/bash
# What the default-pod HBM-OOM shape (empty termination message, the HIP OOM text read
# over pods/log) costs against the termination-message shape, on one box: driver-like
# bench runs interleaved A/B, then the socket-free hot path for each shape.
set -o pipefail
OUT=${OUT:-gpurun_out/r4_shape_ab}
N=${N:-3}
mkdir -p "$OUT"
for i in $(seq 1 "$N"); do
  for s in default-pod termination-message; do
    echo "== bench $s $i"
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --hbm-shape "$s" > "$OUT/bench_${s}_$i.json" \
      2> "$OUT/bench_${s}_$i.err" || exit 1
  done
done
for i in 1 2; do
  for s in default-pod termination-message; do
    echo "== hotpath $s $i"
    timeout -k 10 300 python tools/hotpath_bench.py --steps 20 --warmup 3 --repeat 1 --hbm-shape "$s" \
      > "$OUT/hotpath_${s}_$i.json" 2> "$OUT/hotpath_${s}_$i.err" || exit 1
  done
done
