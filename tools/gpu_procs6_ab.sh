#!/bin/bash
# One gpurun call: CPU per failure with the shard workers saturated (6 worker processes, so the
# apiserver simulator is not the bound), fused conditional write vs the reference's read + write,
# then the default 12-worker north-star line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python bench.py --steps 30 --warmup 2 --procs 6 > gpurun_out/p6_fused.log 2> gpurun_out/p6_fused.err &&
timeout -k 10 600 python bench.py --steps 30 --warmup 2 --procs 6 --two-step-write > gpurun_out/p6_two_step.log 2> gpurun_out/p6_two_step.err &&
timeout -k 10 600 python bench.py --steps 30 --warmup 2 --procs 6 > gpurun_out/p6_fused_b.log 2> gpurun_out/p6_fused_b.err &&
timeout -k 10 600 python bench.py --steps 30 --warmup 2 --procs 6 --two-step-write > gpurun_out/p6_two_step_b.log 2> gpurun_out/p6_two_step_b.err &&
timeout -k 10 600 python bench.py --steps 30 --warmup 2 > gpurun_out/default.log 2> gpurun_out/default.err
rc=$?
for f in p6_fused p6_two_step p6_fused_b p6_two_step_b default; do tail -1 gpurun_out/$f.log | cut -c1-160; done
exit $rc
