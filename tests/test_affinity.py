"""CPU placement (utils/affinity.py) over a fake sysfs: the GPU's NUMA node, one hardware
thread per core, the cgroup's allowed set, and the too-small fallback."""
import os

import pytest

from nexus_supervisor_amd.utils import affinity


def _sysfs(root, gpus, nodes, siblings):
    for bdf, (vendor, cls, node) in gpus.items():
        d = root / "bus" / "pci" / "devices" / bdf
        d.mkdir(parents=True)
        (d / "vendor").write_text(vendor + "\n")
        (d / "class").write_text(cls + "\n")
        (d / "numa_node").write_text(f"{node}\n")
    for n, cpulist in nodes.items():
        d = root / "devices" / "system" / "node" / f"node{n}"
        d.mkdir(parents=True)
        (d / "cpulist").write_text(cpulist + "\n")
    for cpu, sib in siblings.items():
        d = root / "devices" / "system" / "cpu" / f"cpu{cpu}" / "topology"
        d.mkdir(parents=True)
        (d / "thread_siblings_list").write_text(sib + "\n")


@pytest.fixture
def box(tmp_path):
    # 2 nodes x 4 cores x 2 threads: node0 = cpus 0-3 + 8-11, node1 = 4-7 + 12-15
    sib = {c: f"{c % 8},{c % 8 + 8}" for c in range(16)}
    _sysfs(tmp_path,
           {"0000:05:00.0": ("0x1002", "0x038000", 0), "0000:75:00.0": ("0x1002", "0x120000", 1),
            "0000:01:00.0": ("0x8086", "0x020000", 0)},  # a NIC: not a GPU
           {0: "0-3,8-11", 1: "4-7,12-15"}, sib)
    return str(tmp_path)


def test_cpulist_parsing():
    assert affinity.parse_cpulist("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]
    assert affinity.parse_cpulist("") == []


def test_plan_picks_the_gpus_node_one_thread_per_core(box):
    assert affinity.amd_gpu_nodes(box) == [0, 1]
    p = affinity.plan("auto", gpu_index=1, allowed=set(range(16)), min_cpus=4, sys_root=box)
    assert p == {"mode": "numa-cores", "node": 1, "cpus": [4, 5, 6, 7]}
    p = affinity.plan("numa", gpu_index=0, allowed=set(range(16)), min_cpus=4, sys_root=box)
    assert p["cpus"] == [0, 1, 2, 3, 8, 9, 10, 11]


def test_plan_respects_the_allowed_set_and_falls_back(box):
    # a cgroup cpuset with only the SMT siblings of node 0: numa-cores keeps none of them
    # (each is the higher thread of its core), auto falls back to every thread
    p = affinity.plan("auto", gpu_index=0, allowed={8, 9, 10, 11}, min_cpus=4, sys_root=box)
    assert p == {"mode": "numa", "node": 0, "cpus": [8, 9, 10, 11]}
    assert affinity.plan("auto", gpu_index=0, allowed={0, 1}, min_cpus=4, sys_root=box) is None
    assert affinity.plan("none", sys_root=box) is None
    with pytest.raises(ValueError):
        affinity.plan("everywhere", sys_root=box)


def test_unknown_gpu_index_uses_node_zero(box):
    p = affinity.plan("numa-cores", gpu_index=7, allowed=set(range(16)), min_cpus=2, sys_root=box)
    assert p["node"] == 0 and p["cpus"] == [0, 1, 2, 3]


def test_apply_restricts_this_process():
    before = os.sched_getaffinity(0)
    try:
        one = min(before)
        assert affinity.apply({"mode": "numa", "node": 0, "cpus": [one]}) == {"mode": "numa", "node": 0, "cpus": 1}
        assert os.sched_getaffinity(0) == {one}
        assert affinity.apply(None) is None
    finally:
        os.sched_setaffinity(0, before)


def test_busy_cores_are_left_out_while_enough_remain(box):
    # core 1 (cpus 1 + 9) is busy on one thread, core 2 on both together, core 3 quiet
    busy = {1: 0.9, 9: 0.0, 2: 0.3, 10: 0.3, 0: 0.1, 8: 0.1}
    p = affinity.plan("numa-cores", gpu_index=0, allowed=set(range(16)), min_cpus=2, sys_root=box, busy=busy)
    assert p["cpus"] == [0, 3] and p["busy_cores_skipped"] == 2
    assert affinity.apply(None) is None
    # too few quiet cores: the whole node, nothing skipped
    p = affinity.plan("numa-cores", gpu_index=0, allowed=set(range(16)), min_cpus=3, sys_root=box, busy=busy)
    assert p["cpus"] == [0, 1, 2, 3] and "busy_cores_skipped" not in p


def test_cpu_busy_reads_proc_stat(tmp_path):
    import threading

    stat = tmp_path / "stat"
    stat.write_text("cpu  10 0 10 100 0 0 0 0 0 0\ncpu0 5 0 5 50 0 0 0 0 0 0\ncpu1 5 0 5 50 0 0 0 0 0 0\n")

    def later():
        stat.write_text("cpu  30 0 10 120 0 0 0 0 0 0\ncpu0 25 0 5 50 0 0 0 0 0 0\ncpu1 5 0 5 70 0 0 0 0 0 0\n")

    t = threading.Timer(0.05, later)
    t.start()
    busy = affinity.cpu_busy(0.2, proc_root=str(tmp_path))
    t.join()
    assert busy == {0: 1.0, 1: 0.0}
