"""8-GPU node trace fixture (pins the trace-row size bound): the native monitor over the stub amd-smi
(``NEXUS_STUB_GPUS=8``, every GPU pair xGMI-linked) watches an 8-rank job — several
processes per GPU, a burst of GPU events — and one rank dies of an HBM-OOM.  Prints the
rendered trace row and its size as one JSON line.  Run as its own process: the stub's GPU
count is fixed when the library first initialises.

    NEXUS_STUB_GPUS=8 python -m nexus_supervisor_amd.testing.trace8 <scratch dir> [max_bytes]
"""
from __future__ import annotations

import json
import sys
import tempfile
import time


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    root = argv[0] if argv else tempfile.mkdtemp(prefix="trace8-")
    cap = int(argv[1]) if len(argv) > 1 else 8192
    from .. import _amdsmi_monitor_stub as M
    from ..classify import Classifier, render_trace
    from ..config.schema import LabelConfig
    from ..gpu.telemetry import AmdSmiTelemetry, pod_evidence_provider
    from .fakeprocfs import FakeProcFs
    from .seed import make_pod

    uid = "0f3e2b6a-8888-2222-3333-444455556666"
    fs = FakeProcFs(root, n_gpus=8)
    pid = 5000
    for g in range(8):
        for k in range(6):  # the rank's process + dataloader workers / helpers
            env = {"RANK": str(g), "LOCAL_RANK": str(g), "WORLD_SIZE": "8", "LOCAL_WORLD_SIZE": "8",
                   "HIP_VISIBLE_DEVICES": "0,1,2,3,4,5,6,7", "MASTER_ADDR": "10.0.0.1", "MASTER_PORT": "29500",
                   "NCCL_SOCKET_IFNAME": "eth0", "NCCL_IB_HCA": "mlx5"}
            fs.add_process(pid, {g: (200 << 30) if k == 0 else (1 + k) << 30}, env=env, pod_uid=uid)
            pid += 1
    tel = AmdSmiTelemetry(interval=0.01, proc_source="drm", proc_root=fs.proc, sys_root=fs.sys, stub=True)
    tel.start()
    try:
        M.stub_set_vram(3, 294_000)
        for i in range(40):
            M.stub_push_event(i % 8, "QUEUE_EVICTION", f"queue eviction #{i} " + "x" * 60)
        deadline = time.time() + 10
        while time.time() < deadline and sum(len(g["procs"]) for g in tel.snapshot()) < 48:
            time.sleep(0.02)
        time.sleep(0.2)
        labels = LabelConfig()
        c = Classifier(labels)
        c.evidence_provider = pod_evidence_provider(tel, lookback=30)
        env = {"RANK": "3", "LOCAL_RANK": "3", "WORLD_SIZE": "8", "LOCAL_WORLD_SIZE": "8",
               "HIP_VISIBLE_DEVICES": "0,1,2,3,4,5,6,7"}
        pod = make_pod("trace8-run", labels, gpus=8, rv="2", env=env, status={
            "phase": "Failed", "containerStatuses": [{"name": "algorithm", "restartCount": 0, "state": {"terminated": {
                "reason": "Error", "exitCode": 1,
                "message": "torch.OutOfMemoryError: HIP out of memory. Tried to allocate 20.00 GiB. GPU 3 has a total "
                           "capacity of 287.98 GiB of which 1.00 GiB is free."}}}]})
        pod["metadata"]["uid"] = uid
        r = c.classify_pod(pod)[0]
        untrimmed = render_trace(r, max_bytes=0)
        trace = render_trace(r, max_bytes=cap)
        print(json.dumps({"bytes": len(trace.encode()), "untrimmed_bytes": len(untrimmed.encode()),
                          "trace": json.loads(trace)}))
    finally:
        tel.stop()
    return 0


if __name__ == "__main__":
    sys.exit(main())
