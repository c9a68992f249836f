set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6v
# the simulator's Job-DELETE pod cascade: on its GC thread (g1) vs inside the DELETE (g0); then 8 workers
for tag in g1a g0a g1b g0b g1p8 g1p8b; do
  g=${tag:1:1}; procs=0; case $tag in *p8*) procs=8;; esac
  NEXUS_KUBESIM_ASYNC_GC=$g timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --procs $procs --probe-events 0 --diag-step-timeline > gpurun_out/r6v/bench_$tag.json 2> gpurun_out/r6v/bench_$tag.err || { tail -30 gpurun_out/r6v/bench_$tag.err; exit 1; }
  tail -c 100 gpurun_out/r6v/bench_$tag.json
done
