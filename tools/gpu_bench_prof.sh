#!/bin/bash
# One gpurun call: the north-star bench (30 steps), then a 1200-step run with pprof in every
# process (~30 s timed) and the shard workers' profiles summed.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
python -m nexus_supervisor_amd._build > gpurun_out/build.log 2>&1 &&
timeout -k 10 600 python bench.py --steps 30 --warmup 2 > gpurun_out/bench.log 2> gpurun_out/bench.err &&
timeout -k 10 600 python bench.py --steps ${PROF_STEPS:-1200} --warmup 2 --probe-events 0 --no-real-oom \
    --pprof-out gpurun_out/prof/bench.pb.gz --pprof-hz 499 > gpurun_out/prof_bench.log 2> gpurun_out/prof_bench.err &&
python tools/pprof_merge.py gpurun_out/prof/workers_merged.top.txt gpurun_out/prof/bench.pb.gz.w*.pb.gz > /dev/null
rc=$?
tail -1 gpurun_out/bench.log | cut -c1-400; tail -1 gpurun_out/prof_bench.log | cut -c1-300
exit $rc
