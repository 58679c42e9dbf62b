"""Build libcsg.so (HIP, gfx950) in-tree with hipcc.

``python -m constructionsceneposeestimation_amd.build`` — cross-compiles
without a GPU.  The .so is git-ignored but travels to the GPU box with the
repo snapshot.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
LIB = os.path.join(PKG, "libcsg.so")
SOURCES = [os.path.join(PKG, "csrc", "csg_kernels.hip"), os.path.join(PKG, "csrc", "csg_api.cpp")]
DEPS = SOURCES + [os.path.join(PKG, "csrc", "csg_kernels.h"), os.path.join(ROOT, "include", "csg_api.h")]
ARCH = os.environ.get("CSG_OFFLOAD_ARCH", "gfx950")

# -ffp-contract=off: the raster spec's float expressions must round exactly as
# written (bit-exact with the CPU oracle).  HIP keeps fp32 '/' and sqrtf
# correctly rounded by default; do not add -ffast-math.
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", f"--offload-arch={ARCH}", "-Wall"]


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm required to build libcsg.so)")


def needs_build() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(p) > t for p in DEPS)


def build(force: bool = False, verbose: bool = False) -> str:
    if force or needs_build():
        cmd = [hipcc(), *FLAGS, "-o", LIB + ".tmp", *SOURCES]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
        os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
