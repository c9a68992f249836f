set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6y
# a longer run of the final harness (pipelined applies, async GC): 40 timed steps, 240k failures
timeout -k 10 600 python bench.py --gpus 1 --steps 40 --warmup 5 --diag-step-timeline > gpurun_out/r6y/bench_s40.json 2> gpurun_out/r6y/bench_s40.err || { tail -30 gpurun_out/r6y/bench_s40.err; exit 1; }
tail -c 300 gpurun_out/r6y/bench_s40.json
