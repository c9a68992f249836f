set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6e
for i in a b; do
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6e/bench_$i.json 2> gpurun_out/r6e/bench_$i.err || { tail -30 gpurun_out/r6e/bench_$i.err; exit 1; }
  tail -c 300 gpurun_out/r6e/bench_$i.json
done
