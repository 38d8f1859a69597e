"""Build liblsr.so (HIP, gfx950) in-tree with hipcc.

Usage: python -m langsplat_amd.build [--force] [--debug]

The library is a plain extern "C" shared object (include/lsr.h); no torch headers are involved,
so it travels to the GPU box as a single prebuilt file.  Compile flags:
  --offload-arch=gfx950   MI355X only
  -ffp-contract=off       explicit fma only: matches oracle/lsr_oracle.c operation order
  -munsafe-fp-atomics     float atomicAdd -> global_atomic_add_f32 (no CAS loop)
"""
from __future__ import annotations

import argparse
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
ROOT = os.path.dirname(HERE)
BUILD_DIR = os.path.join(ROOT, "build", "lsr")
LIB_PATH = os.path.join(HERE, "liblsr.so")
SOURCES = ["lsr_preprocess.hip", "lsr_binning.hip", "lsr_render.hip", "lsr_loss.hip", "lsr_optim.hip", "lsr_knn.hip", "lsr_api.hip"]
HEADERS = ["lsr_device.h", "lsr_internal.h"]
# per-source extra flags: the render kernels write their packed (v_pk_*) arithmetic explicitly; the
# SLP vectorizer would re-pack their scalar remainder across list entries at the cost of register
# moves (forward walk 70 -> 75 VALU per entry pair)
EXTRA_FLAGS = {"lsr_render.hip": ["-fno-slp-vectorize"]}
ARCH = os.environ.get("LSR_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the HIP toolchain (ROCm) is required to build liblsr.so")


def cflags(debug: bool = False):
    f = [f"--offload-arch={ARCH}", "-std=c++17", "-fPIC", "-ffp-contract=off", "-munsafe-fp-atomics",
         "-Wall", "-Wno-unused-function", "-Wno-unused-result"]
    f += ["-O1", "-g"] if debug else ["-O3"]
    return f


def _stale(lib: str, deps) -> bool:
    if not os.path.exists(lib):
        return True
    t = os.path.getmtime(lib)
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, debug: bool = False, verbose: bool = False) -> str:
    deps = [os.path.join(CSRC, s) for s in SOURCES + HEADERS] + [os.path.join(ROOT, "include", "lsr.h"), __file__]
    if not force and not _stale(LIB_PATH, deps):
        return LIB_PATH
    os.makedirs(BUILD_DIR, exist_ok=True)
    cc = hipcc()
    objs = []
    for src in SOURCES:
        obj = os.path.join(BUILD_DIR, src.replace(".hip", ".o"))
        cmd = [cc] + cflags(debug) + EXTRA_FLAGS.get(src, []) + ["-c", os.path.join(CSRC, src), "-o", obj]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        objs.append(obj)
    tmp = LIB_PATH + ".tmp"
    cmd = [cc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB_PATH)
    return LIB_PATH


AUTOGRAD_SRC = os.path.join(CSRC, "lsr_autograd.cpp")
AUTOGRAD_LIB = os.path.join(HERE, "_lsr_autograd.so")


def build_autograd_helper(force: bool = False, verbose: bool = False) -> str:
    """_lsr_autograd.so: a CPython extension over torch's autograd C++ API (host code, g++; no HIP),
    used by the captured steps to release stale AccumulateGrad nodes (csrc/lsr_autograd.cpp)."""
    if not force and not _stale(AUTOGRAD_LIB, [AUTOGRAD_SRC, __file__]):
        return AUTOGRAD_LIB
    import sysconfig

    import torch
    from torch.utils import cpp_extension
    incs = cpp_extension.include_paths() + [sysconfig.get_paths()["include"]]
    libdir = os.path.join(os.path.dirname(torch.__file__), "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    cmd = [os.environ.get("CXX", "g++"), "-O2", "-std=c++17", "-shared", "-fPIC", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
           "-w"] + [f"-I{d}" for d in incs] + [AUTOGRAD_SRC, f"-L{libdir}", "-lc10", "-ltorch", "-ltorch_cpu",
                                               "-ltorch_python", f"-Wl,-rpath,{libdir}", "-o", AUTOGRAD_LIB + ".tmp"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(AUTOGRAD_LIB + ".tmp", AUTOGRAD_LIB)
    return AUTOGRAD_LIB


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--debug", action="store_true")
    args = ap.parse_args(argv)
    print(build(force=args.force, debug=args.debug, verbose=True))
    print(build_autograd_helper(force=args.force, verbose=True))


if __name__ == "__main__":
    sys.exit(main())
