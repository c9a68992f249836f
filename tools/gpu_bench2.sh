#!/bin/bash
# One gpurun call: two back-to-back runs of the north-star bench (30 steps) to gauge box noise.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
python -m nexus_supervisor_amd._build > gpurun_out/build.log 2>&1 &&
timeout -k 10 600 python bench.py --steps 30 --warmup 2 > gpurun_out/bench_a.log 2> gpurun_out/bench_a.err &&
timeout -k 10 600 python bench.py --steps 30 --warmup 2 --no-real-oom > gpurun_out/bench_b.log 2> gpurun_out/bench_b.err
rc=$?
for f in gpurun_out/bench_a.log gpurun_out/bench_b.log; do tail -1 $f | cut -c1-300; done
exit $rc
