set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6p
# event noise selector on: the default config, then 7 and 8 shard workers, interleaved
for tag in p6a p7a p8a p6b p7b p8b; do
  n=${tag:1:1}
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --procs $n --probe-events 0 --diag-step-timeline > gpurun_out/r6p/bench_$tag.json 2> gpurun_out/r6p/bench_$tag.err || { tail -30 gpurun_out/r6p/bench_$tag.err; exit 1; }
  tail -c 120 gpurun_out/r6p/bench_$tag.json
done
