set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6f
for v in "p6 --procs 6" "p7 --procs 7" "p6b --procs 6"; do
  set -- $v; tag=$1; shift
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --diag-step-timeline "$@" > gpurun_out/r6f/bench_$tag.json 2> gpurun_out/r6f/bench_$tag.err || { tail -30 gpurun_out/r6f/bench_$tag.err; exit 1; }
  tail -c 200 gpurun_out/r6f/bench_$tag.json
done
