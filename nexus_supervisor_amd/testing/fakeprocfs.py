"""Fake ``/proc`` and ``/sys`` trees for the native attribution scanners
(``csrc/amdsmi/procscan.hpp``): processes with amdgpu render-node fds (DRM fdinfo),
their cgroup (→ pod UID) and environment, and the KFD sysfs view (topology nodes with
PCI locations, per-process ``vram_<gpu_id>``).  The GPUs default to the stub amd-smi's
BDFs (``0000:0a:00.0``, ``0000:0b:00.0``, …; ``csrc/amdsmi/amdsmi_stub.cpp``).
"""
from __future__ import annotations

import os
from typing import Dict, Optional


def stub_bdf(i: int) -> str:
    return f"0000:{0x0a + i:02x}:00.0"


def _location_id(bdf: str) -> int:
    _dom, bus, devfn = bdf.split(":")
    dev, fn = devfn.split(".")
    return (int(bus, 16) << 8) | (int(dev, 16) << 3) | int(fn, 16)


def fdinfo_text(bdf: str, vram_bytes: int, client_id: int = 1, gtt_bytes: int = 8 << 20) -> str:
    """An amdgpu render-node fdinfo as the kernel prints it (fields the scanner reads plus noise)."""
    kib = vram_bytes // 1024
    return (f"pos:\t0\nflags:\t02100002\nmnt_id:\t2524\nino:\t11\ndrm-driver:\tamdgpu\n"
            f"drm-client-id:\t{client_id}\ndrm-pdev:\t{bdf}\npasid:\t62450\n"
            f"drm-total-cpu:\t21588 KiB\ndrm-total-gtt:\t{gtt_bytes // 1024} KiB\n"
            f"drm-total-vram:\t{kib} KiB\ndrm-resident-vram:\t{kib} KiB\n"
            f"drm-memory-vram:\t{kib} KiB\ndrm-memory-gtt: \t{gtt_bytes // 1024} KiB\n"
            f"amd-evicted-vram:\t0 KiB\namd-requested-vram:\t{kib} KiB\n")


class FakeProcFs:
    def __init__(self, root: str, n_gpus: int = 2):
        self.proc = os.path.join(root, "proc")
        self.sys = os.path.join(root, "sys")
        os.makedirs(os.path.join(self.proc, "self", "ns"), exist_ok=True)
        self.gpu_ids: Dict[int, int] = {}
        nodes = os.path.join(self.sys, "class", "kfd", "kfd", "topology", "nodes")
        os.makedirs(os.path.join(nodes, "0"), exist_ok=True)  # CPU node: gpu_id 0
        with open(os.path.join(nodes, "0", "gpu_id"), "w") as f:
            f.write("0\n")
        for i in range(n_gpus):
            gid = 27852 + 1000 * i
            self.gpu_ids[i] = gid
            d = os.path.join(nodes, str(i + 1))
            os.makedirs(d, exist_ok=True)
            with open(os.path.join(d, "gpu_id"), "w") as f:
                f.write(f"{gid}\n")
            with open(os.path.join(d, "properties"), "w") as f:
                f.write(f"cpu_cores_count 0\nsimd_count 1024\nlocation_id {_location_id(stub_bdf(i))}\ndomain 0\n"
                        f"drm_render_minor {128 + i}\n")
        os.makedirs(os.path.join(self.sys, "class", "kfd", "kfd", "proc"), exist_ok=True)

    def add_process(self, pid: int, gpus: Dict[int, int], env: Optional[Dict[str, str]] = None,
                    pod_uid: str = "", comm: str = "python3", start: int = 1000, kfd: bool = True) -> None:
        """``gpus``: GPU index → VRAM bytes (one render fd per GPU, plus a /dev/kfd fd)."""
        d = os.path.join(self.proc, str(pid))
        os.makedirs(os.path.join(d, "fd"), exist_ok=True)
        os.makedirs(os.path.join(d, "fdinfo"), exist_ok=True)
        with open(os.path.join(d, "stat"), "w") as f:
            f.write(f"{pid} ({comm}) S 1 1 1 0 -1 4194560 0 0 0 0 0 0 0 0 20 0 1 0 {start} 0 0\n")
        with open(os.path.join(d, "comm"), "w") as f:
            f.write(comm + "\n")
        cg = (f"0::/kubepods.slice/kubepods-burstable.slice/kubepods-burstable-pod{pod_uid.replace('-', '_')}.slice/"
              f"cri-containerd-abc.scope\n") if pod_uid else "0::/user.slice\n"
        with open(os.path.join(d, "cgroup"), "w") as f:
            f.write(cg)
        with open(os.path.join(d, "environ"), "wb") as f:
            f.write(b"".join(f"{k}={v}".encode() + b"\0" for k, v in (env or {}).items()))
        self._link(os.path.join(d, "fd", "3"), "/dev/kfd")
        with open(os.path.join(d, "fdinfo", "3"), "w") as f:
            f.write("pos:\t0\nflags:\t02100002\n")
        for k, (gpu, vram) in enumerate(sorted(gpus.items())):
            fd = 7 + k
            self._link(os.path.join(d, "fd", str(fd)), f"/dev/dri/renderD{128 + gpu}")
            self.set_vram(pid, gpu, vram, fd=fd)
            if kfd:
                kd = os.path.join(self.sys, "class", "kfd", "kfd", "proc", str(pid))
                os.makedirs(kd, exist_ok=True)
                with open(os.path.join(kd, f"vram_{self.gpu_ids[gpu]}"), "w") as f:
                    f.write(f"{vram}\n")

    def set_vram(self, pid: int, gpu: int, vram: int, fd: Optional[int] = None) -> None:
        d = os.path.join(self.proc, str(pid))
        if fd is None:
            fd = next(int(x) for x in os.listdir(os.path.join(d, "fd"))
                      if os.readlink(os.path.join(d, "fd", x)) == f"/dev/dri/renderD{128 + gpu}")
        tmp = os.path.join(d, "fdinfo", f".{fd}.tmp")
        with open(tmp, "w") as f:
            f.write(fdinfo_text(stub_bdf(gpu), vram, client_id=pid * 10 + gpu))
        os.replace(tmp, os.path.join(d, "fdinfo", str(fd)))
        kf = os.path.join(self.sys, "class", "kfd", "kfd", "proc", str(pid), f"vram_{self.gpu_ids[gpu]}")
        if os.path.exists(kf):
            with open(kf + ".tmp", "w") as f:
                f.write(f"{vram}\n")
            os.replace(kf + ".tmp", kf)

    def end_process(self, pid: int) -> None:
        import shutil

        shutil.rmtree(os.path.join(self.proc, str(pid)), ignore_errors=True)
        shutil.rmtree(os.path.join(self.sys, "class", "kfd", "kfd", "proc", str(pid)), ignore_errors=True)

    @staticmethod
    def _link(path: str, target: str) -> None:
        if os.path.lexists(path):
            os.remove(path)
        os.symlink(target, path)
