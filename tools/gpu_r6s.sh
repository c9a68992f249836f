set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6s
for tag in a b; do
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6s/bench_$tag.json 2> gpurun_out/r6s/bench_$tag.err || { tail -30 gpurun_out/r6s/bench_$tag.err; exit 1; }
  tail -c 100 gpurun_out/r6s/bench_$tag.json
done
