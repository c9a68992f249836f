#!/bin/bash
# Compiled hot-path modules vs the same sources in CPython (NEXUS_PURE_PYTHON=1), one box,
# interleaved: the socket-free hot path, then driver-like bench runs.
set -o pipefail
OUT=${OUT:-gpurun_out/r4_compiled_ab}
N=${N:-3}
mkdir -p "$OUT"
for i in $(seq 1 "$N"); do
  for m in compiled pure; do
    echo "== hotpath $m $i"
    if [ "$m" = pure ]; then export NEXUS_PURE_PYTHON=1; else unset NEXUS_PURE_PYTHON; fi
    timeout -k 10 300 python tools/hotpath_bench.py --steps 20 --warmup 3 --repeat 1 \
      > "$OUT/hotpath_${m}_$i.json" 2> "$OUT/hotpath_${m}_$i.err" || exit 1
  done
done
for i in $(seq 1 "$N"); do
  for m in compiled pure; do
    echo "== bench $m $i"
    if [ "$m" = pure ]; then export NEXUS_PURE_PYTHON=1; else unset NEXUS_PURE_PYTHON; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$OUT/bench_${m}_$i.json" 2> "$OUT/bench_${m}_$i.err" || exit 1
  done
done
unset NEXUS_PURE_PYTHON
