#!/bin/bash
# Round-4 measurement batch for one MI355X box (gpurun): shared-namespace replicas with and
# without shard-narrowed watches (gloo ranks: the supervisor does no GPU compute), and the
# priced apiserver + CQL runs.  Every step under its own timeout,
# chained so the first failure ends the batch.
set -o pipefail
OUT=${OUT:-gpurun_out/r4_box}
mkdir -p "$OUT"
run_shared() {  # $1 = ranks, $2 = tag, $3.. = extra bench args
  local n=$1 tag=$2
  shift 2
  CUDA_VISIBLE_DEVICES= HIP_VISIBLE_DEVICES= timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node "$n" --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus "$n" \
    --cluster shared --steps 20 --warmup 3 --probe-events 0 "$@" > "$OUT/shared_${tag}.json" 2> "$OUT/shared_${tag}.err"
}
step() { echo "== $*"; "$@"; }
if [ "${1:-shared}" = shared ]; then
  step run_shared 2 n2_label &&
  step run_shared 2 n2_nolabel --no-shard-label &&
  step run_shared 4 n4_label &&
  step run_shared 4 n4_nolabel --no-shard-label
elif [ "$1" = priced ]; then
  step timeout -k 10 300 python bench.py --cql-latency-us 500 --api-latency-us 2000 --actuation two-step \
      > "$OUT/priced_two_step.json" 2> "$OUT/priced_two_step.err" &&
  step timeout -k 10 300 python bench.py --cql-latency-us 500 --api-latency-us 2000 --actuation fused \
      > "$OUT/priced_fused.json" 2> "$OUT/priced_fused.err" &&
  step timeout -k 10 300 python bench.py --cql-latency-us 500 --api-latency-us 2000 --actuation two-step \
      --kube-qps 50 > "$OUT/priced_two_step_qps50.json" 2> "$OUT/priced_two_step_qps50.err"
fi
