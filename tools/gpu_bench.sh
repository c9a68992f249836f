#!/bin/bash
# One gpurun call: build, then the wire-mode bench (default config) with a pprof profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
python -m nexus_supervisor_amd._build > gpurun_out/build.log 2>&1 &&
NEXUS_CLUSTER_PPROF=$PWD/gpurun_out/cluster_profile.top.txt timeout -k 10 900 python bench.py --steps ${BENCH_STEPS:-10} --warmup 2 --pprof-out gpurun_out/bench_profile.pb.gz ${BENCH_ARGS:-} > gpurun_out/bench.log 2> gpurun_out/bench.err
rc=$?
tail -5 gpurun_out/bench.err; tail -1 gpurun_out/bench.log
exit $rc
