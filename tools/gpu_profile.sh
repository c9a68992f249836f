#!/bin/bash
# One gpurun call: a long saturated bench with pprof in every process (>=30 s timed,
# >=5k samples per shard worker), then the workers' profiles summed.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
python -m nexus_supervisor_amd._build > gpurun_out/build.log 2>&1 &&
timeout -k 10 900 python bench.py --steps ${PROF_STEPS:-2200} --warmup 2 --probe-events 0 \
    --pprof-out gpurun_out/prof/bench.pb.gz --pprof-hz ${PPROF_HZ:-499} ${BENCH_ARGS:-} > gpurun_out/prof_bench.log 2> gpurun_out/prof_bench.err &&
python tools/pprof_merge.py gpurun_out/prof/workers_merged.top.txt gpurun_out/prof/bench.pb.gz.w*.pb.gz > /dev/null
rc=$?
tail -3 gpurun_out/prof_bench.err; tail -1 gpurun_out/prof_bench.log | cut -c1-600
exit $rc
