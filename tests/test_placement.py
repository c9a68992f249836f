"""GPU-local CPU placement (utils.placement) over a fake sysfs: two NUMA nodes, four
GPUs each, 2-way SMT."""
import os

from nexus_supervisor_amd.utils import placement as P


def _fake_sys(tmp_path, cores=32, smt=2):
    pci = tmp_path / "pci"
    cpu = tmp_path / "cpu"
    ncpu = cores * smt
    for c in range(ncpu):
        d = cpu / f"cpu{c}" / "topology"
        d.mkdir(parents=True)
        core = c % cores
        d.joinpath("thread_siblings_list").write_text(",".join(str(core + k * cores) for k in range(smt)) + "\n")
    bdfs = []
    half = cores // 2
    for g in range(8):
        bdf = P.pci_bdf(0, 0x10 + g * 0x10, 0)
        d = pci / bdf
        d.mkdir(parents=True)
        node = 0 if g < 4 else 1
        d.joinpath("numa_node").write_text(f"{node}\n")
        lo = node * half
        d.joinpath("local_cpulist").write_text(f"{lo}-{lo + half - 1},{cores + lo}-{cores + lo + half - 1}\n")
        bdfs.append(bdf)
    return str(pci), str(cpu), bdfs, list(range(ncpu))


def test_cpulist_roundtrip():
    assert P.parse_cpulist("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]
    assert P.format_cpulist([11, 0, 1, 2, 3, 8, 10]) == "0-3,8,10-11"
    assert P.parse_cpulist("") == []


def test_eight_ranks_get_disjoint_gpu_local_core_blocks(tmp_path):
    pci, cpu, bdfs, allowed = _fake_sys(tmp_path)
    blocks = [P.plan(r, 8, bdfs, allowed, per_rank=4, sys_pci=pci, sys_cpu=cpu) for r in range(8)]
    for r, b in enumerate(blocks):
        assert b["how"] == "gpu-local"
        assert b["numa_node"] == (0 if r < 4 else 1)
        assert len(b["cpus"]) == 4
        lo = 0 if r < 4 else 16
        assert all(lo <= c < lo + 16 for c in b["cpus"])  # node-local, first SMT thread only
    flat = [c for b in blocks for c in b["cpus"]]
    assert len(flat) == len(set(flat))


def test_oversubscribed_node_splits_evenly(tmp_path):
    pci, cpu, bdfs, allowed = _fake_sys(tmp_path, cores=8)
    # 4 cores per node, 4 ranks per node, 16 wanted each: one core per rank
    blocks = [P.plan(r, 8, bdfs, allowed, per_rank=16, sys_pci=pci, sys_cpu=cpu)["cpus"] for r in range(4)]
    assert all(len(b) == 1 for b in blocks) and len({b[0] for b in blocks}) == 4


def test_single_gpu_box_restricted_affinity(tmp_path):
    pci, cpu, bdfs, _ = _fake_sys(tmp_path)
    # the process may only use node 1's cores: GPU 0 (node 0) has no allowed local CPU
    allowed = list(range(16, 32))
    b = P.plan(0, 1, bdfs[:1], allowed, per_rank=6, sys_pci=pci, sys_cpu=cpu)
    assert b["how"] == "split" and b["cpus"] == list(range(16, 22))


def test_unknown_locality_falls_back_to_split(tmp_path):
    b = P.plan(1, 2, ["0000:ff:00.0", "0000:fe:00.0"], list(range(8)), per_rank=3,
               sys_pci=str(tmp_path / "nope"), sys_cpu=str(tmp_path / "nope"))
    assert b["how"] == "split" and b["cpus"] == [3, 4, 5]
    # no GPU at all (CPU rehearsal): still disjoint blocks per local rank
    got = [P.plan(r, 4, [], list(range(8)), per_rank=2, sys_pci=str(tmp_path), sys_cpu=str(tmp_path))["cpus"]
           for r in range(4)]
    assert got == [[0, 1], [2, 3], [4, 5], [6, 7]]


def test_apply_pins_calling_thread():
    before = os.sched_getaffinity(0)
    try:
        one = min(before)
        assert P.apply([one])
        assert os.sched_getaffinity(0) == {one}
    finally:
        os.sched_setaffinity(0, before)
    assert not P.apply([])
