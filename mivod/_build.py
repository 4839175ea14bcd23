"""In-tree native build for mivod (no hipify, no JIT cache).

Two shared objects are produced next to this file:

* ``mivod/_mvk*.so``    – hand-written gfx950 HIP kernels (``csrc/kernels``) +
  PyTorch bindings.  Device code is compiled by ``hipcc --offload-arch=gfx950``;
  the torch-facing binding TU is host-only C++.
* ``mivod/_mvcore*.so`` – the C++ engine core (``csrc/engine``): TCP control
  plane / coordinator, stall inspector, timeline writer, fusion planner,
  rendezvous store.  Pure C++17 + pybind11, no GPU dependency, so the CPU test
  tier loads it too.

``python -m mivod._build`` (or ``__graft_entry__.build()``) rebuilds whatever is
out of date.  Objects are cached under ``build/`` keyed by source mtime.
"""
from __future__ import annotations

import os
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "mivod")
CSRC = os.path.join(ROOT, "csrc")
BUILD = os.path.join(ROOT, "build", "native")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("MIVOD_OFFLOAD_ARCH", "gfx950")
EXT_SUFFIX = sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def _hipcc() -> str:
    return os.path.join(ROCM, "bin", "hipcc")


def _py_includes() -> list[str]:
    import pybind11

    return [sysconfig.get_paths()["include"], pybind11.get_include()]


def _torch_flags():
    import torch
    from torch.utils import cpp_extension as ce

    inc = []
    for p in ce.include_paths(device_type="cuda"):
        inc += ["-I", p]
    libdirs = ce.library_paths(device_type="cuda")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    defs = [
        f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
        "-DTORCH_API_INCLUDE_EXTENSION_H",
        "-DTORCH_EXTENSION_NAME=_mvk",
        "-DUSE_ROCM=1",
        "-D__HIP_PLATFORM_AMD__=1",
    ]
    ldflags = []
    for d in libdirs:
        ldflags += ["-L", d, f"-Wl,-rpath,{d}"]
    ldflags += ["-lc10", "-ltorch", "-ltorch_cpu", "-ltorch_python", "-lc10_hip", "-ltorch_hip"]
    return inc, defs, ldflags


def _stale(target: str, deps: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd: list[str], verbose: bool) -> None:
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError(f"mivod native build failed: {' '.join(cmd[:3])} ...")


def _headers(d: str) -> list[str]:
    return [os.path.join(d, f) for f in os.listdir(d) if f.endswith((".h", ".hpp"))]


def kernels_so() -> str:
    return os.path.join(PKG, "_mvk" + EXT_SUFFIX)


def core_so() -> str:
    return os.path.join(PKG, "_mvcore" + EXT_SUFFIX)


def build_kernels(verbose: bool = False, force: bool = False) -> str:
    kdir = os.path.join(CSRC, "kernels")
    os.makedirs(BUILD, exist_ok=True)
    hdrs = _headers(kdir)
    inc, defs, ld = _torch_flags()
    hip_srcs = sorted(f for f in os.listdir(kdir) if f.endswith(".hip"))
    cpp_srcs = sorted(f for f in os.listdir(kdir) if f.endswith(".cpp"))
    objs, jobs = [], []
    for f in hip_srcs:
        src = os.path.join(kdir, f)
        obj = os.path.join(BUILD, f + ".o")
        objs.append(obj)
        if force or _stale(obj, [src] + hdrs):
            jobs.append([_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
                         "-munsafe-fp-atomics", "-I", kdir, "-c", src, "-o", obj])
    for f in cpp_srcs:
        src = os.path.join(kdir, f)
        obj = os.path.join(BUILD, f + ".o")
        objs.append(obj)
        if force or _stale(obj, [src] + hdrs):
            jobs.append(["g++", "-O2", "-std=c++17", "-fPIC", "-I", kdir,
                         "-I", os.path.join(ROCM, "include")]
                        + [x for p in _py_includes() for x in ("-I", p)] + inc + defs
                        + ["-c", src, "-o", obj])
    _parallel(jobs, verbose)
    so = kernels_so()
    if force or jobs or _stale(so, objs):
        _run([_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", so] + objs + ld
             + ["-L", os.path.join(ROCM, "lib"), f"-Wl,-rpath,{os.path.join(ROCM, 'lib')}",
                "-lamdhip64", "-lrocprofiler-sdk-roctx"], verbose)
    return so


def build_core(verbose: bool = False, force: bool = False) -> str:
    edir = os.path.join(CSRC, "engine")
    os.makedirs(BUILD, exist_ok=True)
    hdrs = _headers(edir)
    srcs = sorted(f for f in os.listdir(edir) if f.endswith(".cc"))
    objs, jobs = [], []
    for f in srcs:
        src = os.path.join(edir, f)
        obj = os.path.join(BUILD, "core_" + f + ".o")
        objs.append(obj)
        if force or _stale(obj, [src] + hdrs):
            jobs.append(["g++", "-O2", "-std=c++17", "-fPIC", "-Wall", "-fvisibility=hidden",
                         "-I", edir] + [x for p in _py_includes() for x in ("-I", p)]
                        + ["-c", src, "-o", obj])
    _parallel(jobs, verbose)
    so = core_so()
    if force or jobs or _stale(so, objs):
        _run(["g++", "-shared", "-fPIC", "-o", so] + objs + ["-lpthread"], verbose)
    return so


def comm_so() -> str:
    return os.path.join(PKG, "_mvcomm" + EXT_SUFFIX)


def _torch_libdir() -> str:
    import torch
    return os.path.join(os.path.dirname(torch.__file__), "lib")


def build_comm(verbose: bool = False, force: bool = False) -> str:
    """``mivod/_mvcomm*.so`` — mivod's RCCL data plane (csrc/comm).  Host code
    only; linked against the librccl / libamdhip64 that PyTorch-ROCm itself
    loads (same SONAMEs), so one RCCL and one HIP runtime live in the process."""
    cdir = os.path.join(CSRC, "comm")
    os.makedirs(BUILD, exist_ok=True)
    hdrs = _headers(cdir)
    srcs = sorted(f for f in os.listdir(cdir) if f.endswith((".cc", ".hip")))
    kern_hdrs = _headers(os.path.join(CSRC, "kernels"))
    objs, jobs = [], []
    for f in srcs:
        src = os.path.join(cdir, f)
        obj = os.path.join(BUILD, "comm_" + f + ".o")
        objs.append(obj)
        if force or _stale(obj, [src] + hdrs + kern_hdrs):
            dev = [f"--offload-arch={ARCH}"] if f.endswith(".hip") else []
            jobs.append([_hipcc()] + dev + ["-O3", "-std=c++17", "-fPIC", "-Wall",
                                            "-fvisibility=hidden", "-I", cdir,
                                            "-I", os.path.join(ROCM, "include")]
                        + [x for p in _py_includes() for x in ("-I", p)]
                        + ["-c", src, "-o", obj])
    _parallel(jobs, verbose)
    so = comm_so()
    tl = _torch_libdir()
    if force or jobs or _stale(so, objs):
        _run([_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", so] + objs
             + ["-L", tl, f"-Wl,-rpath,{tl}", "-l:librccl.so", "-l:libamdhip64.so",
                "-lpthread"], verbose)
    return so


def _parallel(jobs, verbose):
    if not jobs:
        return
    n = max(1, min(len(jobs), int(os.environ.get("MAX_JOBS", "8"))))
    with ThreadPoolExecutor(n) as ex:
        list(ex.map(lambda c: _run(c, verbose), jobs))


def build_all(verbose: bool = False, force: bool = False) -> list[str]:
    out = []
    if os.path.isdir(os.path.join(CSRC, "engine")) and any(
            f.endswith(".cc") for f in os.listdir(os.path.join(CSRC, "engine"))):
        out.append(build_core(verbose, force))
    out.append(build_comm(verbose, force))
    out.append(build_kernels(verbose, force))
    return out


if __name__ == "__main__":
    force = "--force" in sys.argv
    for p in build_all(verbose=True, force=force):
        print("built", p)
