"""Probe what the MI355X box exposes to an unprivileged process.

Records amd-smi capabilities (VRAM usage, process list, event notification,
xGMI / ECC queries), the cgroup layout of /proc/self, and the HIP OOM
message a too-large allocation produces.  Output: gpurun_out/probe.json.
"""
import json
import os
import subprocess
import sys
import time

out = {"uid": os.getuid(), "cpu_count": os.cpu_count()}
try:
    out["sched_affinity"] = len(os.sched_getaffinity(0))
except Exception as e:  # pragma: no cover
    out["sched_affinity"] = repr(e)
try:
    with open("/proc/self/cgroup") as f:
        out["cgroup"] = f.read()
except Exception as e:
    out["cgroup"] = repr(e)

try:
    import amdsmi as a

    a.amdsmi_init()
    hs = a.amdsmi_get_processor_handles()
    out["n_gpus"] = len(hs)
    gpus = []
    for h in hs:
        g = {}
        for name, fn in [
            ("bdf", lambda: a.amdsmi_get_gpu_device_bdf(h)),
            ("uuid", lambda: a.amdsmi_get_gpu_device_uuid(h)),
            ("vram", lambda: a.amdsmi_get_gpu_vram_usage(h)),
            ("enum", lambda: a.amdsmi_get_gpu_enumeration_info(h)),
            ("kfd", lambda: a.amdsmi_get_gpu_kfd_info(h)),
            ("procs", lambda: a.amdsmi_get_gpu_process_list(h)),
            ("ecc_total", lambda: a.amdsmi_get_gpu_total_ecc_count(h)),
            ("xgmi_link", lambda: a.amdsmi_get_gpu_xgmi_link_status(h)),
            ("xgmi_info", lambda: a.amdsmi_get_xgmi_info(h)),
            ("asic", lambda: a.amdsmi_get_gpu_asic_info(h)),
        ]:
            try:
                g[name] = fn()
            except Exception as e:
                g[name] = "ERR " + repr(e)
        gpus.append(g)
    out["gpus"] = gpus
    try:
        out["compute_procs"] = a.amdsmi_get_gpu_compute_process_info()
    except Exception as e:
        out["compute_procs"] = "ERR " + repr(e)
    a.amdsmi_shut_down()
except Exception as e:
    out["amdsmi"] = "ERR " + repr(e)

# HIP OOM message from a child process (a too-large allocation fails fast).
code = (
    "import torch,sys\n"
    "free,total=torch.cuda.mem_get_info(0)\n"
    "print('MEM',free,total,flush=True)\n"
    "x=torch.empty(int(total*1.5),dtype=torch.uint8,device='cuda')\n"
)
p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
out["oom_child"] = {"rc": p.returncode, "stdout": p.stdout[-2000:], "stderr": p.stderr[-4000:]}

os.makedirs("gpurun_out", exist_ok=True)
with open("gpurun_out/probe.json", "w") as f:
    json.dump(out, f, indent=1, default=str)
print(json.dumps(out, default=str)[:3000])
