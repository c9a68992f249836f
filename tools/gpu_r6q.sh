set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6q
# steps in flight x shard workers, interleaved (probe off: throughput only)
for tag in p7i4 p7i6 p6i6 p7i8 p6i4 p7i6b; do
  n=${tag:1:1}; i=${tag:3:1}
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --procs $n --inflight $i --probe-events 0 --diag-step-timeline > gpurun_out/r6q/bench_$tag.json 2> gpurun_out/r6q/bench_$tag.err || { tail -30 gpurun_out/r6q/bench_$tag.err; exit 1; }
  tail -c 100 gpurun_out/r6q/bench_$tag.json
done
