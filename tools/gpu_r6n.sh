set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6n
timeout -k 10 900 python bench.py --gpus 1 --steps 100 --warmup 5 --no-pregen > gpurun_out/r6n/bench_soak100.json 2> gpurun_out/r6n/bench_soak100.err || { tail -30 gpurun_out/r6n/bench_soak100.err; exit 1; }
tail -c 300 gpurun_out/r6n/bench_soak100.json
