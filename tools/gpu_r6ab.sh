set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6ab
# the node agent compiled with Cython (gpu.agent in compiled.MODULES): agent path on default pods
for tag in a b; do
  timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 --gpu-evidence agent --events 300 > gpurun_out/r6ab/bench_agent_$tag.json 2> gpurun_out/r6ab/bench_agent_$tag.err || { tail -30 gpurun_out/r6ab/bench_agent_$tag.err; exit 1; }
  tail -c 150 gpurun_out/r6ab/bench_agent_$tag.json
done
