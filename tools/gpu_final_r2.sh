#!/bin/bash
# One gpurun call: GPU tests, smoke, the north-star bench (30 steps) and BASELINE config 5s
# (sharded replicas under chaos, incl. the crashed replica's return and rebalancing).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
python -m nexus_supervisor_amd._build > gpurun_out/build.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 600 python bench.py --steps 30 --warmup 2 > gpurun_out/bench.log 2> gpurun_out/bench.err &&
timeout -k 10 600 python -u -m nexus_supervisor_amd.bench.scenarios --only 5s --seconds 30 \
    --json-out gpurun_out/scenarios_5s.json > gpurun_out/scenarios_5s.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log; tail -2 gpurun_out/smoke.log; tail -1 gpurun_out/bench.log | cut -c1-600
grep '^{' gpurun_out/scenarios_5s.log | cut -c1-300
exit $rc
