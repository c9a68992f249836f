#!/bin/bash
# One gpurun call: shard-worker count sweep on the final tree (6 / 8 / 10 / 12 workers, two
# 30-step runs each, interleaved so box drift hits every setting alike).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/sweep
for r in 1 2; do
  for p in 6 8 10 12; do
    timeout -k 10 300 python bench.py --steps 30 --warmup 2 --procs $p > gpurun_out/sweep/procs${p}_$r.log 2> gpurun_out/sweep/procs${p}_$r.err || exit $?
  done
done
for f in gpurun_out/sweep/*.log; do echo "$f $(tail -1 $f | cut -c1-100)"; done
