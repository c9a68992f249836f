set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6a
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r6a/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r6a/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r6a/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6a/smoke.log 2>&1 || { tail -30 gpurun_out/r6a/smoke.log; exit 1; }
tail -2 gpurun_out/r6a/smoke.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6a/bench.json 2> gpurun_out/r6a/bench.err || { tail -30 gpurun_out/r6a/bench.err; exit 1; }
tail -c 1500 gpurun_out/r6a/bench.json
grep -c "Unable to open queues" gpurun_out/r6a/bench.err gpurun_out/r6a/pytest_gpu.log || true
