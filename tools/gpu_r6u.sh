set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6u
# the generator's apply connection: one chunk per round trip (d1) vs three chunks ahead (d3)
for tag in d3a d1a d3b d1b; do
  d=${tag:1:1}
  NEXUS_BENCH_APPLY_DEPTH=$d timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --diag-step-timeline > gpurun_out/r6u/bench_$tag.json 2> gpurun_out/r6u/bench_$tag.err || { tail -30 gpurun_out/r6u/bench_$tag.err; exit 1; }
  tail -c 100 gpurun_out/r6u/bench_$tag.json
done
