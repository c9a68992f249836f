#!/bin/bash
# One gpurun call: GPU tests (incl. BASELINE config 3 on the real MI355X), the BASELINE
# scenario table (configs 1,2,4,5 at reference limits and uncapped), then bench.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
python -m nexus_supervisor_amd._build > gpurun_out/build.log 2>&1 &&
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 900 python -m nexus_supervisor_amd.bench.scenarios --only 1,2,4,5 --seconds ${SCEN_SECONDS:-30} \
    --json-out gpurun_out/scenarios.json > gpurun_out/scenarios.log 2>&1 &&
timeout -k 10 600 python bench.py --steps ${BENCH_STEPS:-10} --warmup 2 ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log; grep '^{' gpurun_out/scenarios.log; tail -1 gpurun_out/bench.log
exit $rc
