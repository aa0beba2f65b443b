"""In-tree native build for deeplearning_mpi_amd.

Three artefacts, all written next to this file so they travel with the repo snapshot:

* ``csrc/kernels/*.hip`` -> ``build/obj/*.o`` with ``hipcc --offload-arch=gfx950`` (pure HIP,
  no torch headers, seconds per file);
* ``_C.*.so``  = torch binding (``csrc/binding/*.cpp``, g++ against the torch headers) linked
  with the kernel objects, ``libamdhip64`` and the RCCL that torch itself loads;
* ``_mpi.*.so`` = MPI bootstrap (``csrc/mpi/mpi_boot.cpp``, pybind11 + libmpi).

Rebuilds only what changed (mtime of the source and of every header in ``csrc``).
Usage: ``python -m deeplearning_mpi_amd.build [-j N] [--force]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(HERE, "build", "obj")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("DLMPI_ARCH", "gfx950")
MPI_PREFIX = os.environ.get("DLMPI_MPI_PREFIX", "/opt/conda")

EXT_SUFFIX = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
C_SO = os.path.join(HERE, "_C" + EXT_SUFFIX)
MPI_SO = os.path.join(HERE, "_mpi" + EXT_SUFFIX)


def _headers():
    return glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True)


def _stale(target, sources):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in sources)


def _run(cmd, verbose=False):
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("build step failed:\n" + " ".join(cmd) + "\n" + r.stdout)
    return r.stdout


def _torch_flags():
    import torch
    from torch.utils import cpp_extension

    inc = cpp_extension.include_paths()
    tlib = os.path.join(os.path.dirname(torch.__file__), "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    cflags = [f"-I{p}" for p in inc] + [
        f"-I{sysconfig.get_paths()['include']}",
        f"-I{ROCM}/include",
        f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
        "-D__HIP_PLATFORM_AMD__=1",
        "-DUSE_ROCM=1",
        "-DTORCH_API_INCLUDE_EXTENSION_H",
        "-DTORCH_EXTENSION_NAME=_C",
        "-std=c++17",
        "-O2",
        "-fPIC",
        "-Wno-unused-result",
    ]
    ldflags = [
        f"-L{tlib}",
        f"-L{ROCM}/lib",
        "-lc10",
        "-ltorch",
        "-ltorch_cpu",
        "-ltorch_python",
        "-lc10_hip",
        "-ltorch_hip",
        "-lamdhip64",
        f"{tlib}/librccl.so",
        f"-Wl,-rpath,{tlib}",
        f"-Wl,-rpath,{ROCM}/lib",
    ]
    return cflags, ldflags


def build_kernels(jobs=8, force=False, verbose=False):
    os.makedirs(OBJ, exist_ok=True)
    hdrs = _headers()
    srcs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    todo = []
    objs = []
    for s in srcs:
        o = os.path.join(OBJ, os.path.basename(s)[:-4] + ".o")
        objs.append(o)
        if force or _stale(o, [s] + hdrs):
            todo.append((s, o))
    hipcc = os.path.join(ROCM, "bin", "hipcc")

    def one(so):
        s, o = so
        extra = os.environ.get("DLMPI_HIPCC_FLAGS", "").split()   # experiments: extra hipcc flags
        _run([hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-munsafe-fp-atomics", *extra,
              "-c", s, "-o", o], verbose)
        return o

    if todo:
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            list(ex.map(one, todo))
    return objs


def build_binding(objs, jobs=8, force=False, verbose=False):
    cflags, ldflags = _torch_flags()
    hdrs = _headers()
    srcs = sorted(glob.glob(os.path.join(CSRC, "binding", "*.cpp")))
    bobjs, todo = [], []
    for s in srcs:
        o = os.path.join(OBJ, "binding_" + os.path.basename(s)[:-4] + ".o")
        bobjs.append(o)
        if force or _stale(o, [s] + hdrs):
            todo.append((s, o))

    def one(so):
        s, o = so
        _run(["g++"] + cflags + ["-c", s, "-o", o], verbose)

    if todo:
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            list(ex.map(one, todo))
    if force or _stale(C_SO, bobjs + objs):
        _run(["g++", "-shared", "-o", C_SO] + bobjs + objs + ldflags, verbose)
    return C_SO


def build_mpi(force=False, verbose=False):
    src = os.path.join(CSRC, "mpi", "mpi_boot.cpp")
    if not os.path.exists(os.path.join(MPI_PREFIX, "include", "mpi.h")):
        print(f"[dlmpi.build] no MPI under {MPI_PREFIX}; skipping _mpi", file=sys.stderr)
        return None
    if not (force or _stale(MPI_SO, [src])):
        return MPI_SO
    import pybind11

    _run(["g++", "-O2", "-shared", "-fPIC", "-std=c++17", f"-I{pybind11.get_include()}",
          f"-I{sysconfig.get_paths()['include']}", f"-I{MPI_PREFIX}/include", src, "-o", MPI_SO,
          f"-L{MPI_PREFIX}/lib", "-lmpi", f"-Wl,-rpath,{MPI_PREFIX}/lib"], verbose)
    return MPI_SO


def build(jobs=8, force=False, verbose=False):
    objs = build_kernels(jobs, force, verbose)
    build_binding(objs, jobs, force, verbose)
    build_mpi(force, verbose)
    return C_SO


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", "--jobs", type=int, default=min(8, os.cpu_count() or 4))
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args()
    so = build(a.jobs, a.force, a.verbose)
    print(f"[dlmpi.build] ok: {so}")


if __name__ == "__main__":
    main()
