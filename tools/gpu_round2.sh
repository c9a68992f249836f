#!/bin/bash
# One gpurun call: default bench (1 slot), the same with 500 us of injected CQL latency,
# the shared-cluster mode rehearsed at 2 ranks on the box's CPUs (gloo: the 8-GPU run
# uses the same code over RCCL), then the long profiled run.  Each step has its own
# time limit; steps chain with &&.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
python -m nexus_supervisor_amd._build > gpurun_out/build.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/bench_default.log 2> gpurun_out/bench_default.err &&
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cql-latency-us 500 > gpurun_out/bench_cql500.log 2> gpurun_out/bench_cql500.err &&
HIP_VISIBLE_DEVICES= CUDA_VISIBLE_DEVICES= timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 2 --no-real-oom \
    > gpurun_out/bench_shared2.log 2> gpurun_out/bench_shared2.err &&
timeout -k 10 600 python bench.py --steps ${PROF_STEPS:-2200} --warmup 2 --probe-events 0 \
    --pprof-out gpurun_out/prof/bench.pb.gz --pprof-hz 499 > gpurun_out/prof_bench.log 2> gpurun_out/prof_bench.err &&
python tools/pprof_merge.py gpurun_out/prof/workers_merged.top.txt gpurun_out/prof/bench.pb.gz.w*.pb.gz > /dev/null
rc=$?
for f in bench_default bench_cql500 bench_shared2 prof_bench; do echo "== $f"; tail -1 gpurun_out/$f.log | cut -c1-400; done
exit $rc
