set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6t
timeout -k 10 1050 python -u -m nexus_supervisor_amd.bench.scenarios --gpu --json-out gpurun_out/r6t/scenarios.json > gpurun_out/r6t/scenarios.log 2>&1 || { tail -40 gpurun_out/r6t/scenarios.log; exit 1; }
tail -40 gpurun_out/r6t/scenarios.log
