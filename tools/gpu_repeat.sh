#!/bin/bash
# One gpurun call: GPU tests + smoke, then the north-star bench five times back to back (12
# shard workers, the default) and three times with 6 saturated workers, for a median per
# configuration on one box instead of a single sample.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/rep
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
for i in 1 2 3 4 5; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 2 > gpurun_out/rep/default_$i.log 2> gpurun_out/rep/default_$i.err || exit $?
done
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 2 --procs 6 > gpurun_out/rep/procs6_$i.log 2> gpurun_out/rep/procs6_$i.err || exit $?
done
tail -2 gpurun_out/pytest_gpu.log; tail -1 gpurun_out/smoke.log | cut -c1-120
for f in gpurun_out/rep/*.log; do echo "$f $(tail -1 $f | cut -c1-120)"; done
