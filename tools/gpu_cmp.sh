#!/bin/bash
# One gpurun call: GPU tests, smoke, then the default bench (10 steps, as the driver) and a
# 30-step run for a steadier number.  Every GPU step has its own limit; steps chain with &&.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
python -m nexus_supervisor_amd._build > gpurun_out/build.log 2>&1 &&
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/b_default.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 30 --warmup 3 > gpurun_out/b_30.log 2>&1
