set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6z
# replaced objects and watch-history pops freed on the GC thread (new) vs under the store lock
# (prev: bin/nexus-kubesim-prev, built from the previous commit's source), 7 and 8 workers
for tag in n7a p7a n8a p8a n7b p7b; do
  n=${tag:1:1}; bin=""; case $tag in p*) bin="$PWD/nexus_supervisor_amd/bin/nexus-kubesim-prev";; esac
  NEXUS_KUBESIM_BINARY=$bin timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --procs $n --probe-events 0 --diag-step-timeline > gpurun_out/r6z/bench_$tag.json 2> gpurun_out/r6z/bench_$tag.err || { tail -30 gpurun_out/r6z/bench_$tag.err; exit 1; }
  tail -c 100 gpurun_out/r6z/bench_$tag.json
done
