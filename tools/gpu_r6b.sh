set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6b
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r6b/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r6b/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r6b/pytest_gpu.log
cp gpurun_out/hip_runtime_oom.json gpurun_out/r6b/ 2>/dev/null
for i in a b; do
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6b/bench_$i.json 2> gpurun_out/r6b/bench_$i.err || { tail -30 gpurun_out/r6b/bench_$i.err; exit 1; }
  tail -c 300 gpurun_out/r6b/bench_$i.json
done
