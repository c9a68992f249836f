set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6fin2
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r6fin2/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r6fin2/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r6fin2/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6fin2/smoke.log 2>&1 || { tail -30 gpurun_out/r6fin2/smoke.log; exit 1; }
tail -2 gpurun_out/r6fin2/smoke.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6fin2/bench.json 2> gpurun_out/r6fin2/bench.err || { tail -30 gpurun_out/r6fin2/bench.err; exit 1; }
tail -c 200 gpurun_out/r6fin2/bench.json
