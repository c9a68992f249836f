set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6aa
# lines per /sim/apply chunk (the store lock is held for one chunk's commit): 1024 (default) vs 512 vs 2048
for tag in c1024a c512a c2048a c1024b c512b c2048b; do
  c=${tag:1}; c=${c%?}
  NEXUS_BENCH_APPLY_CHUNK=$c timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --probe-events 0 --diag-step-timeline > gpurun_out/r6aa/bench_$tag.json 2> gpurun_out/r6aa/bench_$tag.err || { tail -30 gpurun_out/r6aa/bench_$tag.err; exit 1; }
  tail -c 100 gpurun_out/r6aa/bench_$tag.json
done
