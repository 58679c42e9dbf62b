"""Build libcsg.so (HIP, gfx950) with hipcc and libcsgio.so (host writers)
with g++, both in-tree.

``python -m constructionsceneposeestimation_amd.build`` — cross-compiles
without a GPU.  The .so files are git-ignored but travel to the GPU box with
the repo snapshot.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
LIB = os.path.join(PKG, "libcsg.so")
SOURCES = [os.path.join(PKG, "csrc", "csg_kernels.hip"), os.path.join(PKG, "csrc", "csg_encode.hip"),
           os.path.join(PKG, "csrc", "csg_api.cpp")]
DEPS = SOURCES + [os.path.join(PKG, "csrc", "csg_kernels.h"), os.path.join(PKG, "csrc", "csg_encode.h"),
                  os.path.join(PKG, "csrc", "csg_deflate.h"), os.path.join(PKG, "csrc", "csg_widen.h"),
                  os.path.join(ROOT, "include", "csg_api.h")]
ARCH = os.environ.get("CSG_OFFLOAD_ARCH", "gfx950")
IO_LIB = os.path.join(PKG, "libcsgio.so")
IO_SOURCES = [os.path.join(PKG, "csrc", "csg_io.cpp")]
IO_DEPS = IO_SOURCES + [os.path.join(ROOT, "include", "csg_io.h"), os.path.join(PKG, "csrc", "csg_repr.h")]
IO_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-shared", "-Wall", "-pthread"]
# _csgjson: the label-JSON encoder (CPython extension module)
JSON_EXT = os.path.join(PKG, "_csgjson.so")
JSON_SOURCES = [os.path.join(PKG, "csrc", "csg_json.cpp"), os.path.join(PKG, "csrc", "csg_repr.h")]

# -ffp-contract=off: the raster spec's float expressions must round exactly as
# written (bit-exact with the CPU oracle).  HIP keeps fp32 '/' and sqrtf
# correctly rounded by default; do not add -ffast-math.
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", f"--offload-arch={ARCH}", "-Wall", "-pthread"]


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm required to build libcsg.so)")


def needs_build(lib: str = LIB, deps=None) -> bool:
    deps = DEPS if deps is None else deps
    if not os.path.exists(lib):
        return True
    t = os.path.getmtime(lib)
    return any(os.path.getmtime(p) > t for p in deps)


def build(force: bool = False, verbose: bool = False) -> str:
    if force or needs_build():
        cmd = [hipcc(), *FLAGS, "-o", LIB + ".tmp", *SOURCES]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
        os.replace(LIB + ".tmp", LIB)
    return LIB


def build_io(force: bool = False, verbose: bool = False) -> str:
    if force or needs_build(IO_LIB, IO_DEPS):
        cxx = os.environ.get("CXX") or shutil.which("g++") or "g++"
        cmd = [cxx, *IO_FLAGS, "-o", IO_LIB + ".tmp", *IO_SOURCES, "-lz"]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
        os.replace(IO_LIB + ".tmp", IO_LIB)
    return IO_LIB


def build_json(force: bool = False, verbose: bool = False) -> str:
    if force or needs_build(JSON_EXT, JSON_SOURCES):
        import sysconfig
        cxx = os.environ.get("CXX") or shutil.which("g++") or "g++"
        cmd = [cxx, "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", f"-I{sysconfig.get_paths()['include']}", "-o",
               JSON_EXT + ".tmp", JSON_SOURCES[0]]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
        os.replace(JSON_EXT + ".tmp", JSON_EXT)
    return JSON_EXT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
    print(build_io(force="--force" in sys.argv, verbose=True))
    print(build_json(force="--force" in sys.argv, verbose=True))
