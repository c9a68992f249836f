set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6m
export NEXUS_SLOW_CALLBACK_LOG=1
for tag in a b; do
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --diag-slow-callback-ms 0.5 > gpurun_out/r6m/bench_$tag.json 2> gpurun_out/r6m/bench_$tag.err || { tail -30 gpurun_out/r6m/bench_$tag.err; exit 1; }
  d=$(ls -dt /tmp/nexus-bench-r0-* | head -1)
  cat $d/worker-*.log 2>/dev/null | grep SLOWCB > gpurun_out/r6m/worker_slowcb_$tag.txt || true
  tail -c 150 gpurun_out/r6m/bench_$tag.json
done
