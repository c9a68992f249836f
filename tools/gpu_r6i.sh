set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6i
for v in "n1 --cpu-affinity none" "a1 --cpu-affinity auto" "n2 --cpu-affinity none" "a2 --cpu-affinity auto"; do
  set -- $v; tag=$1; shift
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --diag-step-timeline "$@" > gpurun_out/r6i/bench_$tag.json 2> gpurun_out/r6i/bench_$tag.err || { tail -30 gpurun_out/r6i/bench_$tag.err; exit 1; }
  tail -c 120 gpurun_out/r6i/bench_$tag.json
done
