"""ctypes binding of libcsg.so (include/csg_api.h).

The product path has no CPU fallback: if the HIP library is missing or fails
to load, every call raises :class:`CsgError`.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional

PKG = os.path.dirname(os.path.abspath(__file__))
# CSG_LIB names an alternative build of the same ABI (A/B timing of kernel variants)
LIB_PATH = os.environ.get("CSG_LIB") or os.path.join(PKG, "libcsg.so")
ABI_VERSION = 11  # CSG_ABI_VERSION in include/csg_api.h
KEEP_TEXTURE = -2  # CSG_KEEP_TEXTURE
COVERED_UNKNOWN = 0x80000000  # csg_outputs.label_covered flag: a tile held more than 32 labels
ERR_CAPACITY = -6  # CSG_ERR_CAPACITY
# csg_outputs.file_kinds (CSG_FILE_*): files encoded on the GPU, one per kind per frame, in bit order
FILE_KINDS = {"rgb_png": 1, "depth_csv": 2, "depth_png": 4, "pointcloud_txt": 8}

EXPORTED = (
    "csg_create", "csg_destroy", "csg_last_error", "csg_abi_version", "csg_upload_scene",
    "csg_upload_texture", "csg_set_light", "csg_set_instance_transforms", "csg_set_keypoints",
    "csg_render_batch", "csg_render_batch_async", "csg_synchronize", "csg_get_batch_stats",
    "csg_project_keypoints", "csg_timing_reset", "csg_timing_read", "csg_set_dr_light", "csg_set_dr_textures",
    "csg_instance_bounds", "csg_copy_files", "csg_host_alloc", "csg_host_free", "csg_size_work",
    "csg_get_work_info", "csg_host_id_bytes",
)


class CsgError(RuntimeError):
    pass


class Config(C.Structure):
    _fields_ = [("device", C.c_int32), ("width", C.c_uint32), ("height", C.c_uint32),
                ("max_frames", C.c_uint32), ("near_clip", C.c_float), ("far_clip", C.c_float),
                ("records_per_frame", C.c_uint32), ("bins_per_frame", C.c_uint32),
                ("frames_per_launch", C.c_uint32)]


class Mesh(C.Structure):
    _fields_ = [("positions", C.c_void_p), ("n_vertices", C.c_uint32), ("indices", C.c_void_p),
                ("n_tris", C.c_uint32), ("uvs", C.c_void_p), ("n_uvs", C.c_uint32),
                ("uv_indices", C.c_void_p), ("material", C.c_uint32)]


class Material(C.Structure):
    _fields_ = [("base_color", C.c_uint8 * 4), ("texture", C.c_int32), ("alpha_test", C.c_uint32),
                ("alpha_threshold", C.c_uint32)]


class Instance(C.Structure):
    _fields_ = [("model", C.c_float * 16), ("mesh", C.c_uint32), ("inst_idx", C.c_int32),
                ("reserved", C.c_uint32 * 2)]


class Light(C.Structure):
    _fields_ = [("ambient", C.c_float * 3), ("sun", C.c_float * 3), ("sun_dir", C.c_float * 3),
                ("sky", C.c_uint8 * 4)]


class Frame(C.Structure):
    _fields_ = [("view", C.c_float * 16), ("proj", C.c_float * 16), ("xform_set", C.c_uint32),
                ("frame_id", C.c_uint32), ("records_hint", C.c_uint32), ("bins_hint", C.c_uint32)]


class Outputs(C.Structure):
    _fields_ = [("rgb", C.c_void_p), ("instance", C.c_void_p), ("depth", C.c_void_p),
                ("keypoints_uv", C.c_void_p), ("keypoints_vis", C.c_void_p), ("inst_stats", C.c_void_p),
                ("n_labels", C.c_uint32), ("on_device", C.c_int32), ("normals", C.c_void_p),
                ("points", C.c_void_p), ("depth_vis", C.c_void_p), ("depth_range", C.c_void_p),
                ("label_covered", C.c_void_p), ("file_kinds", C.c_uint32), ("pad_files", C.c_uint32),
                ("files", C.c_void_p), ("files_cap", C.c_uint64), ("file_offsets", C.c_void_p),
                ("depth_stats", C.c_void_p)]


class BatchStats(C.Structure):
    _fields_ = [("records", C.c_uint64), ("bin_entries", C.c_uint64), ("frames", C.c_uint32),
                ("pad", C.c_uint32), ("ms_setup", C.c_float),
                ("ms_bin", C.c_float), ("ms_raster", C.c_float), ("ms_keypoints", C.c_float),
                ("ms_total", C.c_float)]


class Timing(C.Structure):
    _fields_ = [("batches", C.c_uint32), ("frames", C.c_uint32), ("ms_setup", C.c_double),
                ("ms_bin", C.c_double), ("ms_raster", C.c_double), ("ms_keypoints", C.c_double)]


class WorkInfo(C.Structure):
    _fields_ = [("records_per_frame", C.c_uint32), ("bins_per_frame", C.c_uint32),
                ("frames_per_launch", C.c_uint32), ("sized_frames", C.c_uint32), ("max_records", C.c_uint32),
                ("max_bins", C.c_uint32), ("mean_records", C.c_double), ("mean_bins", C.c_double),
                ("work_bytes", C.c_uint64), ("pool_records", C.c_uint64), ("pool_bins", C.c_uint64),
                ("hinted", C.c_uint32), ("hint_retries", C.c_uint32)]


_lib: Optional[C.CDLL] = None


def _share_hip_runtime() -> None:
    """One HIP runtime per process.  PyTorch-ROCm ships its own
    libamdhip64.so (soname libamdhip64.so.7, the one libcsg.so needs): loaded
    first, it also serves libcsg.so.  If libcsg.so came first, /opt/rocm's
    copy would be loaded and a later ``import torch`` would load a second
    runtime, whose GPU initialisation then fails ("No HIP GPUs are
    available").  So when torch is installed it is imported before libcsg.so
    (CSG_OWN_HIP_RUNTIME=1 skips this for processes that never use torch)."""
    import sys
    if "torch" in sys.modules or os.environ.get("CSG_OWN_HIP_RUNTIME") == "1":
        return
    import importlib.util
    if importlib.util.find_spec("torch") is not None:
        import torch  # noqa: F401


def load(path: str = LIB_PATH) -> C.CDLL:
    """Load libcsg.so, building it first when the sources are newer (needs hipcc)."""
    global _lib
    if _lib is not None:
        return _lib
    if path == os.path.join(PKG, "libcsg.so") and (not os.path.exists(path) or
                                                   os.environ.get("CSG_AUTOBUILD", "1") == "1"):
        try:
            from .build import build, needs_build
            if needs_build():
                build()
        except Exception as e:  # pragma: no cover - surfaced below
            if not os.path.exists(path):
                raise CsgError(f"libcsg.so missing and could not be built: {e}") from e
    if not os.path.exists(path):
        raise CsgError(f"libcsg.so not found at {path}; run python -m constructionsceneposeestimation_amd.build")
    _share_hip_runtime()
    lib = C.CDLL(path)
    vp, u32, i32 = C.c_void_p, C.c_uint32, C.c_int32
    lib.csg_create.argtypes = [C.POINTER(Config), C.POINTER(vp)]
    lib.csg_destroy.argtypes = [vp]
    lib.csg_destroy.restype = None
    lib.csg_last_error.argtypes = [vp]
    lib.csg_last_error.restype = C.c_char_p
    lib.csg_abi_version.argtypes = []
    lib.csg_host_id_bytes.argtypes = [vp]
    lib.csg_upload_scene.argtypes = [vp, C.POINTER(Mesh), u32, C.POINTER(Material), u32, C.POINTER(Instance), u32]
    lib.csg_upload_texture.argtypes = [vp, u32, vp, u32, u32]
    lib.csg_set_light.argtypes = [vp, C.POINTER(Light)]
    lib.csg_set_instance_transforms.argtypes = [vp, u32, vp, u32]
    lib.csg_set_keypoints.argtypes = [vp, u32, vp, u32]
    lib.csg_render_batch.argtypes = [vp, vp, u32, C.POINTER(Outputs)]
    lib.csg_render_batch_async.argtypes = [vp, vp, u32, i32, C.POINTER(Outputs), vp]
    lib.csg_synchronize.argtypes = [vp]
    lib.csg_get_batch_stats.argtypes = [vp, C.POINTER(BatchStats)]
    lib.csg_project_keypoints.argtypes = [vp, vp, u32, vp, vp, vp, vp]
    lib.csg_timing_reset.argtypes = [vp]
    lib.csg_timing_read.argtypes = [vp, C.POINTER(Timing)]
    lib.csg_copy_files.argtypes = [vp, vp, C.c_uint64, vp]
    lib.csg_host_alloc.argtypes = [vp, C.c_uint64, C.POINTER(vp)]
    lib.csg_host_free.argtypes = [vp, vp]
    lib.csg_set_dr_light.argtypes = [vp, u32, C.POINTER(Light)]
    lib.csg_set_dr_textures.argtypes = [vp, u32, vp, u32]
    lib.csg_instance_bounds.argtypes = [vp, u32, vp]
    lib.csg_size_work.argtypes = [vp, vp, u32, i32, C.c_float, C.POINTER(WorkInfo)]
    lib.csg_get_work_info.argtypes = [vp, C.POINTER(WorkInfo)]
    if lib.csg_abi_version() != ABI_VERSION:
        raise CsgError(f"libcsg.so ABI {lib.csg_abi_version()} != binding ABI {ABI_VERSION}; rebuild")
    _lib = lib
    return lib
