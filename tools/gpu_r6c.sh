set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6c
export NEXUS_SLOW_CALLBACK_LOG=1
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --diag-probe-timeline --diag-slow-callback-ms 0.7 > gpurun_out/r6c/bench_diag.json 2> gpurun_out/r6c/bench_diag.err || { tail -30 gpurun_out/r6c/bench_diag.err; exit 1; }
tail -c 300 gpurun_out/r6c/bench_diag.json
