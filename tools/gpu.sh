#!/bin/bash
# One parameterised gpurun driver (replaces the round-2 one-off gpu_*.sh scripts).
#
#   gpurun -- bash tools/gpu.sh STEP [STEP ...]
#
# Steps run in order, each under its own time limit; the first failing step ends the
# call (no GPU step starts after a fault, abort, time limit or hang).  Output goes to
# gpurun_out/<step>*.log; the last line of each bench is echoed at the end.
#
#   build                 in-tree native build (normally already done on the CPU side)
#   topo                  CPU / NUMA / cgroup layout and the GPU's PCI locality (gpurun_out/topo.log)
#   tests[=EXPR]          pytest -m gpu (optionally -k EXPR), per-test 120 s timeout
#   smoke                 __graft_entry__.smoke()
#   bench[=ARGS]          python bench.py --steps ${BENCH_STEPS:-30} --warmup 2 ARGS
#                         (ARGS: commas become spaces, e.g. bench=--procs,6)
#   variant=NAME:ARGS     one bench logged as gpurun_out/var_NAME.log (A/B runs)
#   repeat=N[:ARGS]       N benches in a row (median spread)
#   sweep=P1,P2,..        one bench per --procs value
#   profile[=ARGS]        long pprof bench (${PROF_STEPS:-1200} steps) + merged worker profile
#   scenarios=IDS         python -m nexus_supervisor_amd.bench.scenarios --only IDS
#   rocprof               rocprofv3 kernel stats of the HIP stress workload
#   hotpath[=N]           tools/hotpath_bench.py (one shard worker's CPU per failure, no sockets)
#                         N rounds, alternating with the _ab/base tree when it exists (A/B)
#   basebench[=ARGS]      bench.py of the _ab/base tree (A/B against bench)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
STEPS_N=${BENCH_STEPS:-30}
summary=()

run_bench() {  # name, timeout, extra args...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" python bench.py --steps "$STEPS_N" --warmup 2 "$@" > "gpurun_out/$name.log" 2> "gpurun_out/$name.err"
  local rc=$?
  summary+=("$name: $(tail -1 "gpurun_out/$name.log" | cut -c1-240)")
  return $rc
}

for step in "$@"; do
  key=${step%%=*}
  val=""
  [[ "$step" == *=* ]] && val=${step#*=}
  echo "== $step ($(date +%T))"
  case "$key" in
    build)
      python -m nexus_supervisor_amd._build > gpurun_out/build.log 2>&1 ;;
    topo)
      { lscpu; echo "== cpu.max"; cat /sys/fs/cgroup/cpu.max; echo "== cpuset";
        cat /sys/fs/cgroup/cpuset.cpus.effective 2>/dev/null;
        echo "== affinity"; python -c 'import os; print(sorted(os.sched_getaffinity(0)))';
        for d in /sys/class/drm/card*/device; do echo "== $d $(readlink -f $d)";
          cat $d/numa_node $d/local_cpulist 2>/dev/null; done;
        timeout -k 10 120 python -c 'import torch; p=torch.cuda.get_device_properties(0); print("pci", p.pci_domain_id, p.pci_bus_id, p.pci_device_id)';
      } > gpurun_out/topo.log 2>&1 ;;
    tests)
      if [ -n "$val" ]; then
        timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$val" \
          > gpurun_out/pytest_gpu.log 2>&1
      else
        timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
          > gpurun_out/pytest_gpu.log 2>&1
      fi
      rc=$?; summary+=("tests: $(tail -1 gpurun_out/pytest_gpu.log)"); [ $rc -eq 0 ] ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
      rc=$?; summary+=("smoke: $(tail -1 gpurun_out/smoke.log | cut -c1-160)"); [ $rc -eq 0 ] ;;
    bench)
      run_bench bench 600 ${val//,/ } ;;
    variant)
      name=${val%%:*}; args=""; [[ "$val" == *:* ]] && args=${val#*:}
      run_bench "var_$name" 300 ${args//,/ } ;;
    repeat)
      n=${val%%:*}; args=""; [[ "$val" == *:* ]] && args=${val#*:}
      mkdir -p gpurun_out/rep
      for i in $(seq 1 "$n"); do run_bench "rep/run_$i" 300 ${args//,/ } || break; done ;;
    sweep)
      mkdir -p gpurun_out/sweep
      for p in ${val//,/ }; do run_bench "sweep/procs$p" 300 --procs "$p" || break; done ;;
    profile)
      mkdir -p gpurun_out/prof
      timeout -k 10 900 python bench.py --steps "${PROF_STEPS:-1200}" --warmup 2 --probe-events 0 --no-real-oom \
        --pprof-out gpurun_out/prof/bench.pb.gz --pprof-hz "${PPROF_HZ:-499}" ${val//,/ } \
        > gpurun_out/prof/bench.log 2> gpurun_out/prof/bench.err &&
      python tools/pprof_merge.py gpurun_out/prof/workers_merged.top.txt gpurun_out/prof/bench.pb.gz.w*.pb.gz > /dev/null
      rc=$?; summary+=("profile: $(tail -1 gpurun_out/prof/bench.log | cut -c1-200)"); [ $rc -eq 0 ] ;;
    scenarios)
      gpuflag=""; [[ ",$val," == *",3,"* ]] && gpuflag="--gpu"
      timeout -k 10 900 python -u -m nexus_supervisor_amd.bench.scenarios --only "$val" $gpuflag \
        --json-out "gpurun_out/scenarios_${val//,/_}.json" > "gpurun_out/scenarios_${val//,/_}.log" 2>&1 ;;
    rocprof)
      ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
          -d "$GRAFT_REPO_ROOT/gpurun_out/rocprof" -o stress \
          -- "$GRAFT_REPO_ROOT/nexus_supervisor_amd/bin/gpu_stress" hold --gib 32 --seconds 3 ) > gpurun_out/rocprof.log 2>&1 ;;
    hotpath)
      mkdir -p gpurun_out/hotpath
      rc=0
      for i in $(seq 1 "${val:-3}"); do
        if [ -d _ab/base ]; then
          ( cd _ab/base && timeout -k 10 300 python tools/hotpath_bench.py --steps 10 --repeat 1 ) \
            > "gpurun_out/hotpath/base_$i.json" 2> "gpurun_out/hotpath/base_$i.err" || { rc=$?; break; }
        fi
        timeout -k 10 300 python tools/hotpath_bench.py --steps 10 --repeat 1 \
          > "gpurun_out/hotpath/new_$i.json" 2> "gpurun_out/hotpath/new_$i.err" || { rc=$?; break; }
      done
      summary+=("hotpath: $(cat gpurun_out/hotpath/*.json | python -c 'import sys,json; print([json.loads(l)["cpu_us_per_event_median"] for l in sys.stdin if l.strip()])')")
      [ $rc -eq 0 ] ;;
    basebench)
      ( cd _ab/base && timeout -k 10 600 python bench.py --steps "$STEPS_N" --warmup 2 ${val//,/ } ) \
        > gpurun_out/basebench.log 2> gpurun_out/basebench.err
      rc=$?; summary+=("basebench: $(tail -1 gpurun_out/basebench.log | cut -c1-240)"); [ $rc -eq 0 ] ;;
    *)
      echo "unknown step $step"; false ;;
  esac
  rc=$?
  if [ $rc -ne 0 ]; then
    echo "step $step failed rc=$rc"
    printf '%s\n' "${summary[@]}"
    exit $rc
  fi
done
printf '%s\n' "${summary[@]}"
exit 0
