"""ctypes binding of libcsgio.so (include/csg_io.h): native writers of the
generator's on-disk formats (generate_construction_data.py: PNG :1672-1673,
``.npy`` :2066-2069, depth CSV :1688, point-cloud TXT :769-770).

Each call encodes and writes one file with the GIL released, so a thread
pool of writers runs in parallel with the GPU rendering the next batch.  The
text formats are byte-identical to the ``np.savetxt`` calls of the reference.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional

import numpy as np

from .build import IO_LIB, build_io, needs_build, IO_DEPS

ABI_VERSION = 2  # CSGIO_ABI_VERSION in include/csg_io.h
EXPORTED = ("csgio_abi_version", "csgio_write_png_rgb", "csgio_write_npy", "csgio_write_depth_csv",
            "csgio_write_pointcloud_txt", "csgio_depth_stats")
PNG_STRATEGY = {"default": 0, "rle": 1, "huffman": 2}
_lib: Optional[C.CDLL] = None


class CsgIoError(OSError):
    pass


def load() -> C.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if needs_build(IO_LIB, IO_DEPS):
        try:
            build_io()
        except Exception as e:  # pragma: no cover - surfaced below
            if not os.path.exists(IO_LIB):
                raise CsgIoError(f"libcsgio.so missing and could not be built: {e}") from e
    lib = C.CDLL(IO_LIB)
    vp, u32, u64, cp = C.c_void_p, C.c_uint32, C.c_uint64, C.c_char_p
    lib.csgio_abi_version.argtypes = []
    lib.csgio_write_png_rgb.argtypes = [cp, vp, u32, u32, C.c_int, C.c_int]
    lib.csgio_depth_stats.argtypes = [vp, u64, vp]
    lib.csgio_write_npy.argtypes = [cp, vp, u64, cp, vp, u32]
    lib.csgio_write_depth_csv.argtypes = [cp, vp, u32, u32]
    lib.csgio_write_pointcloud_txt.argtypes = [cp, vp, vp, u64]
    if lib.csgio_abi_version() != ABI_VERSION:
        raise CsgIoError(f"libcsgio.so ABI {lib.csgio_abi_version()} != binding ABI {ABI_VERSION}; rebuild")
    _lib = lib
    return lib


def _check(rc: int, what: str, path: str) -> None:
    if rc != 0:
        raise CsgIoError(-rc, f"{what} failed: {os.strerror(-rc)}", path)


def write_png(path: str, rgb: np.ndarray, level: int = 1, strategy: str = "default") -> None:
    a = np.ascontiguousarray(rgb, np.uint8)
    assert a.ndim == 3 and a.shape[2] == 3, a.shape
    _check(load().csgio_write_png_rgb(path.encode(), a.ctypes.data, a.shape[1], a.shape[0], level,
                                      PNG_STRATEGY[strategy]), "write_png", path)


def depth_stats(depth: np.ndarray) -> dict:
    """Counts of one depth image in one native pass (GIL released):
    valid (finite, > 0), zero and infinite pixels, sum / min / max of the valid."""
    a = np.ascontiguousarray(depth, np.float32)
    out = np.zeros(6, np.float64)
    _check(load().csgio_depth_stats(a.ctypes.data, a.size, out.ctypes.data), "depth_stats", "")
    return {"valid": int(out[0]), "zero": int(out[1]), "inf": int(out[2]), "total": int(a.size),
            "sum": float(out[3]), "min": float(out[4]), "max": float(out[5])}


def write_npy(path: str, arr: np.ndarray) -> None:
    a = np.ascontiguousarray(arr)
    descr = np.lib.format.dtype_to_descr(a.dtype)
    shape = (C.c_uint64 * max(a.ndim, 1))(*a.shape)
    _check(load().csgio_write_npy(path.encode(), a.ctypes.data, a.nbytes, descr.encode(), shape, a.ndim),
           "write_npy", path)


def write_depth_csv(path: str, depth: np.ndarray) -> None:
    a = np.ascontiguousarray(depth, np.float32)
    _check(load().csgio_write_depth_csv(path.encode(), a.ctypes.data, a.shape[1], a.shape[0]), "write_depth_csv", path)


def write_pointcloud_txt(path: str, points: np.ndarray, rgb: np.ndarray) -> None:
    """``points`` (..., 3) float32 world xyz (NaN = no hit), ``rgb`` (..., 3) uint8."""
    p = np.ascontiguousarray(points, np.float32).reshape(-1, 3)
    c = np.ascontiguousarray(rgb, np.uint8).reshape(-1, 3)
    assert p.shape == c.shape
    _check(load().csgio_write_pointcloud_txt(path.encode(), p.ctypes.data, c.ctypes.data, p.shape[0]),
           "write_pointcloud_txt", path)
