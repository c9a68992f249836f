"""Probe the per-process GPU attribution sources on a box (round 2, VERDICT weak #2).

While a HIP workload (``gpu_stress hold``) runs as a child, record:
  * ``/proc/<child>/fd`` links to ``/dev/kfd`` / ``/dev/dri/renderD*`` and the DRM
    ``fdinfo`` of the render fds (``drm-pdev``, ``drm-memory-vram`` …);
  * ``/sys/class/kfd/kfd/proc/*`` (KFD per-process dirs: keyed by the *init-namespace* PID)
    and their ``vram_<gpu_id>`` files;
  * the KFD topology (``gpu_id`` → PCI location) and the PID namespace of this process;
  * amd-smi's process list (python bindings) at the same moment.
Output: gpurun_out/probe_kfd.json
"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def rd(p, cap=4096):
    try:
        with open(p, "rb") as f:
            return f.read(cap).decode(errors="replace")
    except Exception as e:  # noqa: BLE001
        return "ERR " + repr(e)


def main():
    from nexus_supervisor_amd._build import binary

    out = {"self_pid": os.getpid(), "pidns": rd("/proc/self/status").split("NSpid:")[-1].split("\n")[0].strip()}
    try:
        out["pidns_link"] = os.readlink("/proc/self/ns/pid")
    except OSError as e:
        out["pidns_link"] = repr(e)
    exe = binary("gpu_stress")
    p = subprocess.Popen([exe, "hold", "--gib", "8", "--seconds", "4"], stdout=subprocess.PIPE, stderr=subprocess.PIPE)
    out["child_pid"] = p.pid
    time.sleep(2.0)
    fds = {}
    try:
        for fd in os.listdir(f"/proc/{p.pid}/fd"):
            try:
                tgt = os.readlink(f"/proc/{p.pid}/fd/{fd}")
            except OSError as e:
                tgt = repr(e)
            if "/dev/" in tgt:
                fds[fd] = {"target": tgt, "fdinfo": rd(f"/proc/{p.pid}/fdinfo/{fd}")}
    except OSError as e:
        fds["error"] = repr(e)
    out["child_fds"] = fds
    out["child_status_nspid"] = rd(f"/proc/{p.pid}/status").split("NSpid:")[-1].split("\n")[0].strip()
    kp = "/sys/class/kfd/kfd/proc"
    procs = {}
    try:
        for d in os.listdir(kp):
            ent = {}
            try:
                for f in sorted(os.listdir(f"{kp}/{d}")):
                    full = f"{kp}/{d}/{f}"
                    ent[f] = sorted(os.listdir(full))[:20] if os.path.isdir(full) else rd(full, 256).strip()
            except OSError as e:
                ent["error"] = repr(e)
            procs[d] = ent
    except OSError as e:
        procs["error"] = repr(e)
    out["kfd_proc"] = procs
    topo = {}
    tp = "/sys/class/kfd/kfd/topology/nodes"
    try:
        for n in sorted(os.listdir(tp)):
            props = rd(f"{tp}/{n}/properties")
            keep = {ln.split()[0]: ln.split()[1] for ln in props.splitlines() if len(ln.split()) == 2 and ln.split()[0] in
                    ("location_id", "domain", "simd_count", "unique_id", "drm_render_minor", "num_xgmi_links",
                     "hive_id", "gfx_target_version", "mem_banks_count")}
            topo[n] = {"gpu_id": rd(f"{tp}/{n}/gpu_id").strip(), "props": keep,
                       "io_links": sorted(os.listdir(f"{tp}/{n}/io_links")) if os.path.isdir(f"{tp}/{n}/io_links") else [],
                       "p2p_links": sorted(os.listdir(f"{tp}/{n}/p2p_links")) if os.path.isdir(f"{tp}/{n}/p2p_links") else []}
            for kind in ("io_links", "p2p_links"):
                for l in topo[n][kind][:8]:
                    topo[n].setdefault(kind + "_props", {})[l] = rd(f"{tp}/{n}/{kind}/{l}/properties", 1024)
    except OSError as e:
        topo["error"] = repr(e)
    out["kfd_topology"] = topo
    try:
        import amdsmi as a

        a.amdsmi_init()
        hs = a.amdsmi_get_processor_handles()
        lst = []
        for h in hs:
            try:
                lst.append({"bdf": a.amdsmi_get_gpu_device_bdf(h), "procs": a.amdsmi_get_gpu_process_list(h)})
            except Exception as e:  # noqa: BLE001
                lst.append("ERR " + repr(e))
            for name, fn in (("topo_numa", lambda: a.amdsmi_get_gpu_topo_numa_affinity(h)),
                             ("xgmi_info", lambda: a.amdsmi_get_xgmi_info(h)),
                             ("link_metrics", lambda: a.amdsmi_get_link_metrics(h)),
                             ("xgmi_link_status", lambda: a.amdsmi_get_gpu_xgmi_link_status(h))):
                try:
                    lst[-1][name] = fn() if isinstance(lst[-1], dict) else None
                except Exception as e:  # noqa: BLE001
                    if isinstance(lst[-1], dict):
                        lst[-1][name] = "ERR " + repr(e)
        out["amdsmi"] = lst
        a.amdsmi_shut_down()
    except Exception as e:  # noqa: BLE001
        out["amdsmi"] = "ERR " + repr(e)
    o, e = p.communicate(timeout=60)
    out["child_rc"] = p.returncode
    out["child_stderr"] = e.decode(errors="replace")[-500:]
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/probe_kfd.json", "w") as f:
        json.dump(out, f, indent=1, default=str)
    print(json.dumps(out, default=str)[:4000])


if __name__ == "__main__":
    main()
