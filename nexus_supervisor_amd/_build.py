"""Build the native components in-tree (no pip install; the .so files travel with
the repo snapshot to GPU boxes).

=====================  ======================================  ==================
artefact               sources                                 toolchain
=====================  ======================================  ==================
``_cql_native``        ``csrc/cql/cql_native.cpp`` (+ proto)   g++ + pybind11
``_amdsmi_monitor``    ``csrc/amdsmi/gpu_monitor.cpp``         g++ + libamd_smi
``bin/nexus-cqlsrv``   ``csrc/cqlsrv/*.cpp`` (+ proto)         g++ (epoll)
``bin/nexus-kubesim``  ``csrc/kubesim/*.cpp`` (+ json.hpp)     g++ (epoll)
``bin/gpu_stress``     ``csrc/stress/gpu_stress.hip``          hipcc gfx950
``_amdsmi_monitor_stub`` monitor over ``amdsmi_stub.cpp``      g++ (CPU tests)
``bin/monitor_selftest`` monitor threads over the stub          g++ (TSan/ASan)
``_certgen``           ``csrc/certgen/certgen.cpp``            g++ + libcrypto
=====================  ======================================  ==================

Every C++ target builds with ``-Wall -Wextra -Werror`` (the CI static-analysis gate).
``--sanitize address|undefined|thread`` also builds the in-process extensions with the
sanitizer into ``build/san/<name>/``; tests load them in a subprocess via
``NEXUS_NATIVE_DIR`` with the runtime LD_PRELOADed (:func:`sanitizer_runtime`).

``python -m nexus_supervisor_amd._build [--force] [--only NAME] [--sanitize thread|address]``
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import sysconfig
from typing import Dict, List, Optional

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(ROOT, "csrc")
BIN = os.path.join(PKG, "bin")
SAN_DIR = os.path.join(ROOT, "build", "san")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")


def _pybind_includes() -> List[str]:
    import pybind11

    return [f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}"]


def _cxx() -> str:
    return os.environ.get("CXX", "g++")


def targets(sanitize: Optional[str] = None, out_root: Optional[str] = None) -> Dict[str, Dict]:
    """Every native artefact.  With ``sanitize`` the in-process extensions are built into
    ``SAN_DIR/<sanitizer>/`` (loaded in a subprocess through ``NEXUS_NATIVE_DIR``) and the
    executables get a ``-<sanitizer>`` suffix.  ``out_root``: extensions and executables
    all go there instead (a from-source rebuild beside the in-tree artefacts, loaded the
    same way — ``tests/test_gpu_box.py`` rebuilds on the GPU box itself)."""
    common = ["-O2", "-g", "-std=c++17", "-Wall", "-Wextra", "-Werror", "-Wno-unused-parameter", "-fvisibility=hidden"]
    san = []
    if sanitize:
        flags = "address,undefined" if sanitize in ("address", "undefined") else sanitize
        san = [f"-fsanitize={flags}", "-fno-omit-frame-pointer", "-fno-sanitize-recover=undefined"
               if sanitize != "thread" else "-fno-omit-frame-pointer"]
    proto = os.path.join(CSRC, "cql", "cql_proto.hpp")
    amd = os.path.join(CSRC, "amdsmi")
    mon_deps = [os.path.join(amd, "monitor_core.hpp"), os.path.join(amd, "procscan.hpp"),
                os.path.join(amd, "stderr_filter.hpp")]
    ext_dir = out_root or (os.path.join(SAN_DIR, sanitize) if sanitize else PKG)
    bin_dir = out_root or BIN
    sfx = f"-{sanitize}" if sanitize else ""
    return {
        "cql_native": {
            "out": os.path.join(ext_dir, "_cql_native" + EXT),
            "srcs": [os.path.join(CSRC, "cql", "cql_native.cpp")],
            "deps": [proto],
            "cmd": lambda out, srcs: [_cxx(), *common, *san, "-shared", "-fPIC", *_pybind_includes(), *srcs, "-o", out],
            "inproc": True,
        },
        "kube_native": {
            "out": os.path.join(ext_dir, "_kube_native" + EXT),
            "srcs": [os.path.join(CSRC, "kube", "watch_decoder.cpp"), os.path.join(CSRC, "kube", "json_encode.cpp"),
                     os.path.join(CSRC, "kube", "histogram.cpp"), os.path.join(CSRC, "kube", "informer_apply.cpp"),
                     os.path.join(CSRC, "kube", "shared_bucket.cpp")],
            "deps": [],
            "cmd": lambda out, srcs: [_cxx(), *common, "-O3", *san, "-shared", "-fPIC",
                                      f"-I{sysconfig.get_paths()['include']}", *srcs, "-o", out],
            "inproc": True,
        },
        # the shard-label webhook's self-signed CA + serving certificate (libcrypto)
        "certgen": {
            "out": os.path.join(ext_dir, "_certgen" + EXT),
            "srcs": [os.path.join(CSRC, "certgen", "certgen.cpp")],
            "deps": [],
            "cmd": lambda out, srcs: [_cxx(), *common, *san, "-shared", "-fPIC", *_pybind_includes(), *srcs, "-lcrypto",
                                      "-o", out],
            "requires": "/usr/include/openssl/x509v3.h",
            "inproc": True,
        },
        "amdsmi_monitor": {
            "out": os.path.join(ext_dir, "_amdsmi_monitor" + EXT),
            "srcs": [os.path.join(amd, "gpu_monitor.cpp")],
            "deps": mon_deps,
            "cmd": lambda out, srcs: [_cxx(), *common, *san, "-shared", "-fPIC", *_pybind_includes(), f"-I{ROCM}/include",
                                      *srcs, f"-L{ROCM}/lib", "-lamd_smi", f"-Wl,-rpath,{ROCM}/lib", "-pthread", "-o", out],
            "requires": os.path.join(ROCM, "include", "amd_smi", "amdsmi.h"),
        },
        # the same monitor over the stub amd-smi: CPU tests of the sampler / attribution path
        "amdsmi_monitor_stub": {
            "out": os.path.join(ext_dir, "_amdsmi_monitor_stub" + EXT),
            "srcs": [os.path.join(amd, "gpu_monitor.cpp"), os.path.join(amd, "amdsmi_stub.cpp")],
            "deps": mon_deps,
            "cmd": lambda out, srcs: [_cxx(), *common, *san, "-shared", "-fPIC", *_pybind_includes(), f"-I{ROCM}/include",
                                      "-DNEXUS_AMDSMI_STUB", "-DNEXUS_MONITOR_MODULE=_amdsmi_monitor_stub", *srcs,
                                      "-pthread", "-o", out],
            "requires": os.path.join(ROCM, "include", "amd_smi", "amdsmi.h"),
            "inproc": True,
        },
        "monitor_selftest": {
            "out": os.path.join(bin_dir, "monitor_selftest" + sfx),
            "srcs": [os.path.join(amd, "monitor_selftest.cpp"), os.path.join(amd, "amdsmi_stub.cpp")],
            "deps": mon_deps,
            "cmd": lambda out, srcs: [_cxx(), *common, *san, f"-I{ROCM}/include", *srcs, "-pthread", "-o", out],
            "requires": os.path.join(ROCM, "include", "amd_smi", "amdsmi.h"),
            "exe": True,
        },
        "cqlsrv": {
            "out": os.path.join(bin_dir, "nexus-cqlsrv" + sfx),
            "srcs": [os.path.join(CSRC, "cqlsrv", "cqlsrv.cpp")],
            "deps": [proto],
            "cmd": lambda out, srcs: [_cxx(), *common, *san, "-pthread", f"-I{os.path.join(CSRC, 'cql')}", *srcs, "-o", out],
            "exe": True,
        },
        "kubesim": {
            "out": os.path.join(bin_dir, "nexus-kubesim" + sfx),
            "srcs": [os.path.join(CSRC, "kubesim", "kubesim.cpp")],
            "deps": [os.path.join(CSRC, "kubesim", "json.hpp")],
            "cmd": lambda out, srcs: [_cxx(), *common, "-O3", *san, "-pthread", *srcs, "-o", out],
            "exe": True,
        },
        "gpu_stress": {
            "out": os.path.join(bin_dir, "gpu_stress"),
            "srcs": [os.path.join(CSRC, "stress", "gpu_stress.hip")],
            "deps": [],
            "cmd": lambda out, srcs: [os.path.join(ROCM, "bin", "hipcc"), f"--offload-arch={ARCH}", "-O3", "-std=c++17",
                                      "-Wall", "-Werror", *srcs, "-o", out],
            "requires": os.path.join(ROCM, "bin", "hipcc"),
        },
    }


def sanitizer_runtime(sanitize: str) -> Optional[str]:
    """``LD_PRELOAD`` value for an uninstrumented Python that loads instrumented
    extensions: the compiler's sanitizer runtime first, then libstdc++ (the runtime
    resolves its ``__cxa_throw`` interceptor at startup; Python itself does not link
    libstdc++, so without it the first C++ exception aborts the process)."""
    libs = []
    for lib in ({"address": "libasan.so", "undefined": "libasan.so", "thread": "libtsan.so"}[sanitize], "libstdc++.so"):
        p = subprocess.run([_cxx(), f"-print-file-name={lib}"], capture_output=True, text=True)
        path = p.stdout.strip()
        if not (path and os.path.isabs(path) and os.path.exists(path)):
            return None
        libs.append(os.path.realpath(path))
    return " ".join(libs)


def _stale(t: Dict) -> bool:
    out = t["out"]
    if not os.path.exists(out):
        return True
    m = os.path.getmtime(out)
    return any(os.path.getmtime(s) > m for s in t["srcs"] + t["deps"] + [__file__])


def build_one(name: str, t: Dict, force: bool = False, verbose: bool = False) -> str:
    if t.get("requires") and not os.path.exists(t["requires"]):
        return f"{name}: skipped (missing {t['requires']})"
    missing = [s for s in t["srcs"] if not os.path.exists(s)]
    if missing:
        return f"{name}: skipped (no sources {missing})"
    if not force and not _stale(t):
        return f"{name}: up to date"
    os.makedirs(os.path.dirname(t["out"]), exist_ok=True)
    tmp = f"{t['out']}.tmp{os.getpid()}"  # concurrent builders (test workers) never share a temp file
    cmd = t["cmd"](tmp, t["srcs"])
    if verbose:
        print(" ".join(cmd), flush=True)
    p = subprocess.run(cmd, capture_output=True, text=True)
    if p.returncode != 0:
        raise RuntimeError(f"{name}: build failed\n$ {' '.join(cmd)}\n{p.stdout}\n{p.stderr}")
    os.replace(tmp, t["out"])
    return f"{name}: built {os.path.relpath(t['out'], ROOT)}"


def _compile_module(name: str, force: bool = False, verbose: bool = False) -> Optional[str]:
    """One hot-path module through Cython (pure-Python mode) and the C compiler into
    ``_compiled/`` with the hash of its source (:mod:`.compiled`); None when fresh."""
    from . import compiled

    if not force and compiled.fresh(name):
        return None
    src = compiled.source_path(name)
    digest = compiled.source_hash(src)
    os.makedirs(compiled.DIR, exist_ok=True)
    tag = f"{name}.tmp{os.getpid()}"
    c_file = os.path.join(compiled.DIR, tag + ".c")
    so_tmp = os.path.join(compiled.DIR, tag + compiled.EXT)
    steps = [
        [sys.executable, "-m", "cython", "-3", "--module-name", name, "-X", "binding=True",
         "-X", "embedsignature=False",
         # annotations stay hints: as C types they would be enforced (a frozenset bound to a
         # name annotated `set` raises) — Python semantics exactly, only the dispatch removed
         "-X", "annotation_typing=False", "-o", c_file, src],
        [os.environ.get("CC", "gcc"), "-O2", "-fPIC", "-shared", "-fno-strict-aliasing", "-fwrapv", "-w",
         f"-I{sysconfig.get_paths()['include']}", c_file, "-o", so_tmp],
    ]
    try:
        for cmd in steps:
            if verbose:
                print(" ".join(cmd), flush=True)
            p = subprocess.run(cmd, capture_output=True, text=True)
            if p.returncode != 0:
                raise RuntimeError(f"compiled {name}: build failed\n$ {' '.join(cmd)}\n{p.stdout}\n{p.stderr}")
        os.replace(so_tmp, compiled.extension_path(name))
        with open(compiled.hash_path(name) + ".tmp", "w") as f:
            f.write(digest + "\n")
        os.replace(compiled.hash_path(name) + ".tmp", compiled.hash_path(name))
    finally:
        for leftover in (c_file, so_tmp):
            if os.path.exists(leftover):
                os.remove(leftover)
    return f"compiled {name}"


def build_compiled(force: bool = False, verbose: bool = False) -> str:
    """Every :data:`.compiled.MODULES` entry whose extension is missing or stale."""
    from . import compiled

    try:
        import Cython  # noqa: F401
    except ImportError:
        return "compiled: skipped (Cython not importable)"
    with cf.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        done = [r for r in ex.map(lambda n: _compile_module(n, force, verbose), compiled.MODULES) if r]
    return f"compiled: {len(done)} built, {len(compiled.MODULES) - len(done)} up to date"


def build(force: bool = False, only: Optional[List[str]] = None, sanitize: Optional[str] = None, verbose: bool = False,
          out_root: Optional[str] = None) -> List[str]:
    ts = targets(sanitize, out_root)
    names = [n for n in ts if not only or n in only]
    if sanitize:
        names = [n for n in names if ts[n].get("exe") or ts[n].get("inproc")]
    with cf.ThreadPoolExecutor(max_workers=min(4, len(names) or 1)) as ex:
        futs = {ex.submit(build_one, n, ts[n], force, verbose): n for n in names}
        out = [f.result() for f in cf.as_completed(futs)]
    if not sanitize and not out_root and (not only or "compiled" in only):
        out.append(build_compiled(force, verbose))
    return out


def binary(name: str) -> str:
    """Path of a built helper binary, building it on demand."""
    ts = targets()
    key = {"nexus-cqlsrv": "cqlsrv", "gpu_stress": "gpu_stress", "nexus-kubesim": "kubesim",
           "monitor_selftest": "monitor_selftest"}[name]
    t = ts[key]
    if _stale(t):
        build_one(key, t)
    return t["out"]


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--only", action="append")
    ap.add_argument("--sanitize", choices=("thread", "address", "undefined"))
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args(argv)
    for line in build(a.force, a.only, a.sanitize, a.verbose):
        print(line)
    return 0


if __name__ == "__main__":
    sys.exit(main())
