set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6w
# async GC frees removed objects off the loop: 8 vs 7 shard workers (a: probe on, b: off)
for tag in p8a p7a p8b p7b; do
  n=${tag:1:1}; pe=600; case $tag in *b) pe=0;; esac
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --procs $n --probe-events $pe --diag-step-timeline > gpurun_out/r6w/bench_$tag.json 2> gpurun_out/r6w/bench_$tag.err || { tail -30 gpurun_out/r6w/bench_$tag.err; exit 1; }
  tail -c 100 gpurun_out/r6w/bench_$tag.json
done
