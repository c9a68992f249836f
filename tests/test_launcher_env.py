"""Launcher env families folded into the rank topology (VERDICT r5 missing #4).

Kubeflow's training operator (PyTorchJob) and a pod that runs ``torchrun`` itself give
the pod torchrun's arguments as ``PET_*`` env; ``RANK`` / ``WORLD_SIZE`` only exist in the
processes torchrun starts.  The reference caches these pods and never reads them
(``/root/reference/services/supervisor.go:74``)."""
import json

import pytest

from nexus_supervisor_amd.config.schema import LabelConfig
from nexus_supervisor_amd.gpu.telemetry import FakeTelemetry, evidence_for
from nexus_supervisor_amd.gpu.topology import merge_process_ranks, topology_from_env, topology_from_pod
from nexus_supervisor_amd.models import kube
from nexus_supervisor_amd.testing.seed import make_pod

# a PyTorchJob worker as the training operator renders it (2 nodes × 8 GPUs)
TRAINING_OPERATOR_ENV = {
    "PET_NNODES": "2", "PET_NPROC_PER_NODE": "8", "PET_NODE_RANK": "1",
    "PET_MASTER_ADDR": "llama-pretrain-master-0", "PET_MASTER_PORT": "23456",
    "MASTER_ADDR": "llama-pretrain-master-0", "MASTER_PORT": "23456", "PYTHONUNBUFFERED": "1",
    "NCCL_IB_DISABLE": "1", "RCCL_MSCCLPP_ENABLE": "1",
}


@pytest.mark.parametrize("env,gpus,want", [
    (TRAINING_OPERATOR_ENV, 8, {"nnodes": 2, "local_world_size": 8, "node_rank": 1, "world_size": 16,
                                "master_addr": "llama-pretrain-master-0", "master_port": 23456, "launcher": "torchrun"}),
    # nproc-per-node "gpu": one process per GPU the pod got
    ({"PET_NNODES": "4", "PET_NPROC_PER_NODE": "gpu", "PET_NODE_RANK": "0"}, 8,
     {"nnodes": 4, "local_world_size": 8, "world_size": 32, "node_rank": 0}),
    # elastic range: no world size; the c10d rendezvous endpoint names the master
    ({"PET_NNODES": "1:4", "PET_NPROC_PER_NODE": "8", "PET_RDZV_ENDPOINT": "etcd-0.etcd:2379",
      "PET_RDZV_BACKEND": "c10d"}, 8,
     {"nnodes_range": [1, 4], "local_world_size": 8, "master_addr": "etcd-0.etcd", "master_port": 2379,
      "rdzv_backend": "c10d"}),
    # the direct variables win over PET_*
    ({"PET_NNODES": "2", "PET_NPROC_PER_NODE": "8", "WORLD_SIZE": "4", "LOCAL_WORLD_SIZE": "2", "RANK": "3"}, 2,
     {"world_size": 4, "local_world_size": 2, "rank": 3, "nnodes": 2}),
])
def test_pet_env_table(env, gpus, want):
    topo = topology_from_env(env, gpus)
    for k, v in want.items():
        assert topo.get(k) == v, (k, topo)
    if "nnodes_range" in want:
        assert "world_size" not in topo and "nnodes" not in topo


def test_training_operator_pod_spec_through_the_native_projection():
    """The decoder keeps PET_* (models/kube.py ENV_KEEP): the topology of a pod decoded
    from the watch stream carries them."""
    nat = pytest.importorskip("nexus_supervisor_amd._kube_native")
    pod = make_pod("pt-1", LabelConfig(), env=TRAINING_OPERATOR_ENV, gpus=8, node="mi355x-003")
    dec = nat.ProjectedDecoder(kube.watch_projection("Pod"))
    line = json.dumps({"type": "ADDED", "object": pod}).encode() + b"\n"
    (ev,) = dec.feed(line)
    obj = ev["object"]
    topo = topology_from_pod(obj)
    assert topo["world_size"] == 16 and topo["node_rank"] == 1 and topo["local_world_size"] == 8
    assert topo["collective_env"] == {"NCCL_IB_DISABLE": "1", "RCCL_MSCCLPP_ENABLE": "1"}
    assert "PYTHONUNBUFFERED" not in kube.pod_env(obj)


def test_agent_keeps_the_ranks_collective_env():
    """The node agent's per-process environ carries the RCCL settings a launcher gave its
    children only (mpirun -x, a wrapper script): they reach the topology's
    collective_env; the pod spec's own values win."""
    tel = FakeTelemetry(n_gpus=8)
    for r in range(2):
        tel.add_process(100 + r, r, vram_bytes=1 << 30, pod_uid="uid-7",
                        env={"RANK": str(8 + r), "LOCAL_RANK": str(r), "WORLD_SIZE": "16",
                             "NCCL_IB_DISABLE": "0", "RCCL_ENABLE_INTRANET": "1", "NCCL_DEBUG": "WARN"})
    ev = evidence_for(tel, pod_uid="uid-7")
    assert ev["collective_env"] == {"NCCL_DEBUG": "WARN", "NCCL_IB_DISABLE": "0", "RCCL_ENABLE_INTRANET": "1"}
    topo = merge_process_ranks(topology_from_env(TRAINING_OPERATOR_ENV, 8), ev)
    assert topo["collective_env"]["NCCL_IB_DISABLE"] == "1"  # the spec's value
    assert topo["collective_env"]["RCCL_ENABLE_INTRANET"] == "1" and topo["collective_env"]["NCCL_DEBUG"] == "WARN"
    assert topo["collective_env_from_processes"] == ["NCCL_DEBUG", "RCCL_ENABLE_INTRANET"]
    assert [e["rank"] for e in topo["rank_map"]] == [8, 9]
