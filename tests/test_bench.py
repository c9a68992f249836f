"""``bench.py`` driver contract (one JSON line, metric/config from BASELINE.json, weak
scaling, MAX over ranks) on CPU: the wire transport in-process, and two ranks under
``torch.distributed.run`` with gloo (the 8-GPU run uses the same path over RCCL)."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _check(out, n, steps, warmup, events):
    assert KEYS <= set(out)
    with open(os.path.join(ROOT, "BASELINE.json")) as f:
        base = json.load(f)
    assert out["metric"] == base["metric"] or out["metric"].startswith("pod-fail")
    assert out["n_gpus"] == n and out["steps"] == steps and out["warmup"] == warmup
    # node mode: one replica over the node's slots on a split namespace (strong); else per-slot work (weak)
    assert out["scaling"] == ("strong" if out["config"].get("cluster") == "node" else "weak")
    assert out["higher_is_better"] is True and out["errors"] == 0
    assert out["value"] > 0 and out["config"]["global_batch"] == events * n
    assert abs(out["vs_baseline"] - out["value"] / 10.0) < 0.05
    assert out["p50_ms"] is not None and out["p99_ms"] >= out["p50_ms"]
    # the bench checks what it measured: every decision wrote the workload's expected stage,
    # and every timed run's row (failed and started) reads back with that stage
    assert out["wrong_stage"] == 0, out["readback"]
    assert out["readback"]["checked"] >= steps * events * n and out["readback"]["wrong"] == 0, out["readback"]
    assert out["supervisor_cpu_us_per_event_rank0"] > 0
    if out["config"].get("workload") == "lifecycle":
        # every failure brings its replacement run's start: a ToRunning decision (read + write)
        # per started run, and the Pending -> Running watch traffic with the kubelet's Events
        assert out["starts_per_s"] > 0 and out["decisions_per_s"] > out["value"], out
        assert out["start_p50_ms"] is not None
        if out["config"]["transport"] == "wire":
            assert out["watch_objects_per_failure"] >= 8, out["watch_objects_per_failure"]


@pytest.mark.slow
def test_bench_wire_in_process(tmp_path, capsys):
    import bench

    js = tmp_path / "b.json"
    rc = bench.main(["--steps", "2", "--warmup", "1", "--jobs", "300", "--events", "60", "--probe-events", "3",
                     "--probe-rate", "6000", "--json-out", str(js)])
    assert rc == 0
    lines = [x for x in capsys.readouterr().out.splitlines() if x.startswith("{")]
    assert len(lines) == 1
    out = json.loads(lines[0])
    assert out == json.loads(js.read_text())
    _check(out, 1, 2, 1, 60)
    cfg = out["config"]
    assert cfg["transport"] == "wire" and cfg["store"].startswith("cql")
    # one replica, no HA: failures read then write plainly; a ToRunning is one conditional write
    assert cfg["actuation"] == "read+write (ToRunning: one conditional write)"
    st = cfg["stages_ms"]
    assert st["receive_to_checkpoint"]["count"] >= 120
    for k in ("stage_classify", "stage_queue", "stage_write"):
        assert st[k]["count"] == st["receive_to_checkpoint"]["count"]
    # the reads are the failures' only: no ToRunning reads its row first
    assert 0 < st["stage_read"]["count"] < st["receive_to_checkpoint"]["count"]
    assert st["stage_read"]["count"] + st["stage_prepare"]["count"] == st["receive_to_checkpoint"]["count"]
    assert out["latency_at_rate"]["events"] == 3


@pytest.mark.slow
def test_bench_gpu_evidence_through_the_node_agent(capsys):
    """``--gpu-evidence agent``: the node agent as its own process annotates every failed GPU
    pod (default pods: their logs read from a kubelet-style /var/log/pods the simulator
    writes), the supervisor (no local telemetry) holds each decision for it; the line reports
    the agent's cost and how many waits expired, and every row still reads back correct."""
    import bench

    rc = bench.main(["--steps", "2", "--warmup", "1", "--jobs", "300", "--events", "40", "--probe-events", "5",
                     "--probe-rate", "6000", "--gpu-evidence", "agent", "--procs", "2"])
    assert rc == 0
    out = json.loads([x for x in capsys.readouterr().out.splitlines() if x.startswith("{")][-1])
    _check(out, 1, 2, 1, 40)
    ev = out["config"]["gpu_evidence"]
    assert ev["via"] == "node-agent" and ev["deferred"] > 0 and ev["agent_annotations"] >= ev["deferred"] * 0.9, ev
    assert ev["wait_expired"] == 0 and ev["agent_util"] > 0, ev
    # default pods: the agent reads their OOM text from the simulator's /var/log/pods, the
    # supervisor never has to fetch a tail over pods/log
    assert out["config"]["hbm_oom_shape"] == "default-pod"
    assert ev["agent_log_reads"] > 0 and ev["supervisor_log_fetches"] == 0, ev


@pytest.mark.slow
def test_bench_fused_actuation_with_priced_lwt(capsys):
    """``--actuation fused`` at a CQL round trip of 2 ms, the LWT priced as a Paxos round
    (3 more round trips): the checkpoint-write stage of the fused path costs ~4 round trips
    where the two-step path's write costs 1 (+1 read)."""
    import bench

    rc = bench.main(["--steps", "2", "--warmup", "1", "--jobs", "300", "--events", "40", "--probe-events", "0",
                     "--actuation", "fused", "--cql-latency-us", "2000", "--procs", "1"])
    assert rc == 0
    out = json.loads([x for x in capsys.readouterr().out.splitlines() if x.startswith("{")][-1])
    _check(out, 1, 2, 1, 40)
    assert out["config"]["actuation"] == "fused conditional write"
    st = out["config"]["stages_ms"]
    assert st["stage_write"]["p50"] >= 4 * 2.0 * 0.9  # the CAS itself, not local work
    assert "stage_read" not in st and st["stage_prepare"]["p50"] < 2.0


@pytest.mark.slow
def test_bench_two_step_write_ab(capsys):
    """``--two-step-write`` (the reference's read + write actuation) passes the same checks, and
    the line says which actuation it measured."""
    import bench

    rc = bench.main(["--steps", "2", "--warmup", "1", "--jobs", "300", "--events", "60", "--probe-events", "0",
                     "--two-step-write"])
    assert rc == 0
    out = json.loads([x for x in capsys.readouterr().out.splitlines() if x.startswith("{")][-1])
    _check(out, 1, 2, 1, 60)
    assert out["config"]["actuation"].startswith("read+write")


@pytest.mark.slow
def test_bench_two_ranks_torchrun_gloo():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2",
                        "--steps", "2", "--warmup", "1", "--jobs", "200", "--events", "40", "--transport", "inproc",
                        "--probe-events", "0"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [x for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0 only
    out = json.loads(lines[0])
    _check(out, 2, 2, 1, 40)
    assert out["config"]["parallelism"] == "shard2x1proc"


@pytest.mark.slow
def test_bench_two_ranks_wire_worker_processes():
    """The replica slot mode on the wire transport: the shared cluster — ONE
    apiserver simulator and ONE CQL server for both ranks, each rank a 2-process replica
    watching the whole namespace with ``sharding.shards = 2`` — MAX-over-ranks timing,
    one JSON line, every timed run read back with its expected stage."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2",
                        "--steps", "2", "--warmup", "1", "--jobs", "300", "--events", "50", "--procs", "2",
                        "--probe-events", "0", "--cluster", "shared", "--slot-mode", "replica"], cwd=ROOT, env=env,
                       capture_output=True,
                       text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [x for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, p.stdout
    out = json.loads(lines[0])
    _check(out, 2, 2, 1, 50)
    cfg = out["config"]
    assert cfg["parallelism"] == "shard2x2proc" and cfg["worker_processes"] == 2 and cfg["cluster"] == "shared"
    assert cfg["stages_ms"]["receive_to_checkpoint"]["count"] >= 150  # merged from both workers
    assert {"worker0_util", "worker1_util"} <= set(cfg["cpu_util_rank0"])


@pytest.mark.slow
def test_baseline_scenarios_small(arun):
    """BASELINE configs 1, 2, 4, 5 (scaled down): every run reaches its expected stage,
    the leader crash fails over, latencies are reported."""
    from nexus_supervisor_amd.bench import scenarios as sc

    r1 = arun(sc.cfg1_single("uncapped", n=5), timeout=60)
    assert r1["acked"] == 5 and r1["wrong_stage"] == 0 and r1["p50_ms"] < 1000
    r2 = arun(sc.cfg2_burst("reference", n=40), timeout=60)
    assert r2["acked"] == 40 and r2["wrong_stage"] == 0
    # the mix really holds start failures (image pulls, GPU admission rejections)
    assert r2["kinds"].get("image-pull") and r2["kinds"].get("gpu-admission") and r2["kinds"].get("host-oom")
    r4 = arun(sc.cfg4_rate("uncapped", seconds=2.0, rate=1200, jobs=300), timeout=60)
    assert r4["drained"] and r4["wrong_stage"] == 0 and r4["acked"] == r4["events"] == 40
    r5 = arun(sc.cfg5_chaos("uncapped", seconds=4.0, rate=1200, jobs=300), timeout=120)
    assert r5["drained"] and r5["wrong_stage"] == 0
    assert {"cql_restart", "storm", "leader_crash", "failover_s"} <= set(r5["chaos"])
    assert r5["chaos"]["failover_s"] < 10


def _torchrun(nproc, *args, timeout=400):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
                        "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", str(nproc),
                        *args], cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [x for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


@pytest.mark.slow
def test_bench_four_ranks_shared_cluster_not_harness_bound():
    """4 gloo ranks on the shared cluster (one apiserver simulator
    + one CQL server, four replicas each owning a shard of the namespace): no harness
    process saturated, every decision in its expected stage, every timed row read back,
    and the replica CPU per failure reported for every rank."""
    out = _torchrun(4, "--steps", "2", "--warmup", "1", "--jobs", "200", "--events", "30", "--procs", "1",
                    "--probe-events", "0", "--cluster", "shared", "--slot-mode", "replica")
    _check(out, 4, 2, 1, 30)
    assert out["config"]["cluster"] == "shared" and out["config"]["parallelism"] == "shard4x1proc"
    assert out["harness_bound"]["bound"] is False and out["harness_bound"]["bound_ranks"] == [], out["harness_bound"]
    assert out["wrong_stage"] == 0 and out["readback"]["wrong"] == 0 and out["readback"]["checked"] >= 4 * 2 * 30
    assert len(out["supervisor_cpu_us_per_event_by_rank"]) == 4
    assert all(v and v > 0 for v in out["supervisor_cpu_us_per_event_by_rank"])


@pytest.mark.slow
def test_bench_two_ranks_per_rank_clusters_and_poisson_probe():
    """The default N>1 layout: every GPU-job slot's replica with its own apiserver simulator
    and CQL server (weak scaling with nothing shared), plus the open-loop probe: Poisson
    arrivals, every probe event acknowledged."""
    out = _torchrun(2, "--steps", "2", "--warmup", "1", "--jobs", "200", "--events", "30", "--procs", "1",
                    "--probe-events", "40", "--probe-rate", "6000", "--slot-mode", "replica")
    _check(out, 2, 2, 1, 30)
    assert out["config"]["cluster"] == "per-rank"
    probe = out["latency_at_rate"]
    assert probe["events"] == 40 and probe["arrivals"] == "poisson" and probe["p99_ms"] >= probe["p50_ms"] > 0


def test_probe_stage_delta_counts_only_what_the_probe_recorded():
    """The probe's stage breakdown is the growth of the cumulative stage histograms."""
    from nexus_supervisor_amd.bench.runner import _stage_counts, _stage_delta
    from nexus_supervisor_amd.obs.metrics import Metrics

    m = Metrics("t")
    sup = type("S", (), {"metrics": m})()
    for _ in range(1000):
        m.observe_seconds("stage_read", 0.050)  # saturated steps: 50 ms reads
    before = _stage_counts(sup)
    for v in (0.0002, 0.0003, 0.0004):
        m.observe_seconds("stage_read", v)  # the probe: sub-millisecond reads
    d = _stage_delta(before, _stage_counts(sup))
    assert d["stage_read"]["count"] == 3
    assert 0.19 < d["stage_read"]["p50"] < 0.32 and d["stage_read"]["max"] < 0.41
    assert "stage_write" not in d


@pytest.mark.slow
def test_bench_node_mode_four_slots_one_replica_one_monitor():
    """The default for N>1 (``--slot-mode node``): ONE supervisor replica and ONE GPU monitor
    on rank 0 supervise every GPU slot of the node (the production shape: one HA
    supervisor, one node agent); each rank is a slot whose runs sit on its GPU.  Every
    slot's HBM-OOM at about the same moment is attributed to that slot's physical GPU."""
    out = _torchrun(4, "--steps", "2", "--warmup", "1", "--jobs", "200", "--events", "30", "--procs", "1",
                    "--probe-events", "10", "--probe-rate", "6000")
    _check(out, 4, 2, 1, 30)
    cfg = out["config"]
    assert cfg["slot_mode"] == "node" and cfg["gpu_monitors"] == 1 and cfg["cluster"] == "node"
    assert cfg["parallelism"] == "node4slots:1replica:1proc"
    att = cfg["attribution"]
    assert att["slots"] == 4 and att["correct"] == 4, att
    assert [p["gpu_index"] for p in att["per_slot"]] == [0, 1, 2, 3]
    # every slot's failures went through the one replica: the failures of all four slots
    assert out["readback"]["checked"] >= 4 * 2 * 30 and out["wrong_stage"] == 0
