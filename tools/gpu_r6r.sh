set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6r
# decisions in flight per replica (--workers, split over the shard workers) x shard workers
for tag in p7w256 p7w512 p8w512 p8w1024 p7w1024 p7w512b; do
  n=${tag:1:1}; w=${tag:3}; w=${w%b}
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --procs $n --workers $w --probe-events 0 --diag-step-timeline > gpurun_out/r6r/bench_$tag.json 2> gpurun_out/r6r/bench_$tag.err || { tail -30 gpurun_out/r6r/bench_$tag.err; exit 1; }
  tail -c 100 gpurun_out/r6r/bench_$tag.json
done
