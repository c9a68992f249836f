#!/bin/bash
# One gpurun call: GPU tests, smoke, short benches, rocprofv3 kernel stats of the
# HIP stress workload. Every GPU step has its own time limit; steps chain with &&.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
python -m nexus_supervisor_amd._build > gpurun_out/build.log 2>&1 &&
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 600 python bench.py --steps ${BENCH_STEPS:-10} --warmup 2 ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1 &&
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/rocprof" -o stress \
    -- "$GRAFT_REPO_ROOT/nexus_supervisor_amd/bin/gpu_stress" hold --gib 32 --seconds 3 ) > gpurun_out/rocprof.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log; tail -2 gpurun_out/smoke.log; tail -1 gpurun_out/bench.log
exit $rc
