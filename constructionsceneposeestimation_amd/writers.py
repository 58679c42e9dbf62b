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

ABI_VERSION = 4  # CSGIO_ABI_VERSION in include/csg_io.h
EXPORTED = ("csgio_abi_version", "csgio_write_png_rgb", "csgio_write_npy", "csgio_write_depth_csv",
            "csgio_write_pointcloud_txt", "csgio_depth_stats", "csgio_write_label_json")
PNG_STRATEGY = {"default": 0, "rle": 1, "huffman": 2}
_lib: Optional[C.CDLL] = None


class CsgIoError(OSError):
    pass


class Label(C.Structure):   # csgio_label
    _fields_ = [("frame_id", C.c_uint32), ("height", C.c_uint32), ("width", C.c_uint32),
                ("n_objects", C.c_uint32), ("n_labels", C.c_uint32), ("n_kp", C.c_uint32),
                ("camera_pose", C.c_void_p), ("camera_params", C.c_char_p), ("class_mapping", C.c_char_p),
                ("obj_head", C.c_void_p), ("obj_label", C.c_void_p), ("obj_kp_off", C.c_void_p),
                ("obj_kp", C.c_void_p), ("inst_stats", C.c_void_p), ("covered", C.c_void_p),
                ("kp_uv", C.c_void_p), ("kp_vis", C.c_void_p), ("kp_name", C.c_void_p),
                ("obj_listed", C.c_void_p)]


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
    lib.csgio_write_label_json.argtypes = [cp, C.POINTER(Label)]
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


class LabelWriter:
    """Label files written natively (csgio_write_label_json, GIL released):
    byte-identical to ``save_label_json(label_record(...))`` (labels.py) for
    one workload's keypoint table and camera intrinsics.  The fixed JSON
    pieces are rendered once (per workload; object poses once per epoch) with
    the same encoder that writes the Python path."""

    def __init__(self, kp_table, camera_params: dict, n_labels: int, height: int, width: int):
        from .identity import CONSTRUCTION_CLASS
        from .labels import label_json_bytes
        self._enc = label_json_bytes
        self.height, self.width, self.n_labels = int(height), int(width), int(n_labels)
        self.camera_params = label_json_bytes(camera_params).replace(b"\n", b"\n  ")
        self.class_mapping = label_json_bytes(dict(CONSTRUCTION_CLASS)).replace(b"\n", b"\n  ")
        names = [label_json_bytes(n) for _, n in kp_table]
        self._names = names
        self.kp_name = (C.c_char_p * max(len(names), 1))(*names)
        self.n_kp = len(names)
        n_obj = max([j for j, _ in kp_table] + [-1]) + 1
        self._kp_by_obj = [[] for _ in range(n_obj)]
        for k, (j, _) in enumerate(kp_table):
            self._kp_by_obj[j].append(k)
        self._epochs = {}

    def epoch(self, e: int, poses):
        """The per-epoch pieces for ``object_poses`` of epoch e (cached)."""
        hit = self._epochs.get(e)
        if hit is not None:
            return hit
        heads = []
        for p in poses:
            t = self._enc(p)                       # {\n  "inst_idx": ..\n}
            heads.append(b"    " + t[2:-2].replace(b"\n", b"\n    "))
        n = len(poses)
        kp_lists = [self._kp_by_obj[j] if j < len(self._kp_by_obj) else [] for j in range(n)]
        off = np.zeros(n + 1, np.uint32)
        off[1:] = np.cumsum([len(x) for x in kp_lists])
        idx = np.array([k for x in kp_lists for k in x] or [0], np.uint32)
        labels = np.array([p["inst_idx"] for p in poses] or [0], np.int32)
        labels = np.where(labels < 0, labels + self.n_labels, labels).astype(np.int32)   # Python indexing
        st = {"heads": heads, "head_arr": (C.c_char_p * max(n, 1))(*heads), "n": n, "off": off, "idx": idx,
              "labels": labels}
        if len(self._epochs) >= 64:
            self._epochs.pop(next(iter(self._epochs)))
        self._epochs[e] = st
        return st

    def n_visible(self, ep: dict, inst_stats: np.ndarray, listed: Optional[np.ndarray] = None) -> int:
        """Objects the label file lists: those with visible pixels (and, with
        ``listed``, those flagged there; labels.label_record's rule)."""
        lab = ep["labels"][:ep["n"]]
        ok = (lab >= 0) & (lab < inst_stats.shape[0])
        vis = np.zeros(ep["n"], bool)
        vis[ok] = inst_stats[lab[ok], 0] != 0
        if listed is not None:
            vis |= ok & np.asarray(listed, bool)[:ep["n"]]
        return int(np.count_nonzero(vis))

    def write(self, path: str, frame_id: int, camera_pose, ep: dict, inst_stats: np.ndarray,
              covered: Optional[np.ndarray], kp_uv: np.ndarray, kp_vis: np.ndarray,
              listed: Optional[np.ndarray] = None) -> None:
        pose = np.ascontiguousarray(np.asarray(camera_pose, np.float64).reshape(7))
        st = np.ascontiguousarray(inst_stats, np.uint32)
        cv = np.ascontiguousarray(covered, np.uint32) if covered is not None else None
        uv = np.ascontiguousarray(kp_uv, np.float32)
        vis = np.ascontiguousarray(kp_vis, np.int32)
        lst = np.ascontiguousarray(listed, np.uint8) if listed is not None else None
        if lst is not None and lst.shape[0] < ep["n"]:
            raise CsgIoError(f"write_label_json: listed has {lst.shape[0]} entries, {ep['n']} objects")
        L = Label(int(frame_id), self.height, self.width, ep["n"], st.shape[0], self.n_kp, pose.ctypes.data,
                  self.camera_params, self.class_mapping, C.cast(ep["head_arr"], C.c_void_p).value,
                  ep["labels"].ctypes.data, ep["off"].ctypes.data, ep["idx"].ctypes.data, st.ctypes.data,
                  cv.ctypes.data if cv is not None else None, uv.ctypes.data, vis.ctypes.data,
                  C.cast(self.kp_name, C.c_void_p).value, lst.ctypes.data if lst is not None else None)
        _check(load().csgio_write_label_json(path.encode(), C.byref(L)), "write_label_json", path)
