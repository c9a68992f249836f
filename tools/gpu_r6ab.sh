set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6ab
# final tree with the node agent compiled (gpu.agent in compiled.MODULES): GPU tests, smoke, agent path
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r6ab/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r6ab/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r6ab/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6ab/smoke.log 2>&1 || { tail -30 gpurun_out/r6ab/smoke.log; exit 1; }
tail -1 gpurun_out/r6ab/smoke.log
timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 --gpu-evidence agent --events 300 > gpurun_out/r6ab/bench_agent_a.json 2> gpurun_out/r6ab/bench_agent_a.err || { tail -30 gpurun_out/r6ab/bench_agent_a.err; exit 1; }
tail -c 150 gpurun_out/r6ab/bench_agent_a.json
