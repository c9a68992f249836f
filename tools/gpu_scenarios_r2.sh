#!/bin/bash
# One gpurun call: the BASELINE scenario table on the MI355X box — configs 1, 2, 4, 5 and
# 5s (sharded replicas with per-shard Leases under chaos), each at reference limits and
# uncapped, plus config 3 (real HBM-OOM on the GPU with per-GPU attribution).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
python -m nexus_supervisor_amd._build > gpurun_out/build.log 2>&1 &&
timeout -k 10 1000 python -u -m nexus_supervisor_amd.bench.scenarios --only 1,2,3,4,5,5s --gpu --seconds ${SCEN_SECONDS:-30} \
    --json-out gpurun_out/scenarios_r2.json > gpurun_out/scenarios_r2.log 2>&1
rc=$?
grep '^{' gpurun_out/scenarios_r2.log | cut -c1-400
exit $rc
