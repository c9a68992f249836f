#!/bin/bash
# One gpurun call: the default bench at several shard-worker counts (is 12 still the
# knee now that the simulator has headroom?).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/sweep
python -m nexus_supervisor_amd._build > gpurun_out/build.log 2>&1 || exit 1
rc=0
for p in ${SWEEP_PROCS:-10 12 13 14}; do
  timeout -k 10 240 python bench.py --steps 10 --warmup 2 --procs $p --no-real-oom > gpurun_out/sweep/procs$p.log 2> gpurun_out/sweep/procs$p.err || { rc=$?; break; }
  echo "procs $p: $(tail -1 gpurun_out/sweep/procs$p.log | cut -c1-120)"
done
exit $rc
