#!/bin/bash
# N driver-like bench runs of the current tree back to back (median and range of the
# published numbers: VERDICT r3 next #3), then the hot-path A/B of the native informer apply.
set -o pipefail
OUT=${OUT:-gpurun_out/r4_repeat}
N=${N:-5}
mkdir -p "$OUT"
for i in $(seq 1 "$N"); do
  echo "== bench $i"
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$OUT/bench_$i.json" 2> "$OUT/bench_$i.err" || exit 1
done
if [ "${HOTPATH:-1}" = 1 ]; then
  for i in 1 2 3; do
    for m in 0 1; do
      echo "== hotpath py_apply=$m round $i"
      NEXUS_PY_INFORMER_APPLY=$m timeout -k 10 300 python tools/hotpath_bench.py --steps 20 --warmup 3 --repeat 1 \
        > "$OUT/hotpath_py${m}_$i.json" 2> "$OUT/hotpath_py${m}_$i.err" || exit 1
    done
  done
fi
