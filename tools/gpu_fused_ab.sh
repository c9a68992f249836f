#!/bin/bash
# One gpurun call: A/B of the actuation path on the north-star bench (fused conditional write,
# the default, vs the reference's read + write), then a ~30 s pprof run of the default with the
# shard workers' profiles summed.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 600 python bench.py --steps 30 --warmup 2 > gpurun_out/bench_fused.log 2> gpurun_out/bench_fused.err &&
timeout -k 10 600 python bench.py --steps 30 --warmup 2 --two-step-write > gpurun_out/bench_two_step.log 2> gpurun_out/bench_two_step.err &&
timeout -k 10 600 python bench.py --steps 30 --warmup 2 > gpurun_out/bench_fused_b.log 2> gpurun_out/bench_fused_b.err &&
timeout -k 10 600 python bench.py --steps ${PROF_STEPS:-1200} --warmup 2 --probe-events 0 --no-real-oom \
    --pprof-out gpurun_out/prof/bench.pb.gz --pprof-hz 499 > gpurun_out/prof_bench.log 2> gpurun_out/prof_bench.err &&
python tools/pprof_merge.py gpurun_out/prof/workers_merged.top.txt gpurun_out/prof/bench.pb.gz.w*.pb.gz > /dev/null
rc=$?
for f in bench_fused bench_two_step bench_fused_b prof_bench; do tail -1 gpurun_out/$f.log | cut -c1-200; done
exit $rc
