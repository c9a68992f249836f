set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6c
timeout -k 10 400 python -u -m pytest tests/test_gpu_box.py -m gpu -x -v --timeout 300 --timeout-method thread -k rebuilt > gpurun_out/r6c/pytest_rebuild.log 2>&1 || { tail -40 gpurun_out/r6c/pytest_rebuild.log; exit 1; }
tail -3 gpurun_out/r6c/pytest_rebuild.log
cp gpurun_out/box_rebuild.json gpurun_out/r6c/
export NEXUS_SLOW_CALLBACK_LOG=1
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --diag-probe-timeline --diag-slow-callback-ms 0.7 > gpurun_out/r6c/bench_diag.json 2> gpurun_out/r6c/bench_diag.err || { tail -30 gpurun_out/r6c/bench_diag.err; exit 1; }
tail -c 300 gpurun_out/r6c/bench_diag.json
