"""Writer pool of the generator: frames rendered on the GPU are encoded and
written to disk by worker processes (or threads), the role of the
reference's per-frame cv2.imwrite / np.save / np.savetxt / json.dump calls
(generate_construction_data.py:1668-1711, :2055-2072), run in parallel with
the GPU.

Threads (the default) or processes: a frame's files are encoded by the
native writers (libcsgio.so, GIL released), but its label JSON
(``json.dump(indent=2)``, about 80 KB with keypoints) is pure Python and
holds the GIL for ~4 ms.  Worker processes have a GIL each; measured on C3
at 1080p with 16 writers they are nevertheless slower (184 vs 233 frames/s:
every worker page-faults the shared slots it reads, and each task is
pickled), so threads are the default and processes an option for heavier
per-frame Python work.

Frames reach the workers through shared memory: the renderer writes each
batch's outputs straight into one slot of a ring of ``n_slots`` shared
batch buffers (:meth:`Renderer.render` ``out=``), a task names (slot, frame)
plus the frame's small label dict, and a slot is reused only after every
task that reads it has finished.  The processes are spawned before the
parent touches the GPU and never use it.
"""
from __future__ import annotations

import multiprocessing as mp
import os
import threading
import time
from concurrent.futures import Future, ProcessPoolExecutor, ThreadPoolExecutor
from typing import Dict, List, Optional, Tuple

import numpy as np

Layout = Dict[str, Tuple[int, tuple, str]]     # name -> (byte offset in a slot, shape, dtype)


SINKS = ("disk", "discard")


def _atomic(path: str, fn, *args, sink: str = "disk") -> None:
    """Write through ``path + '.tmp'`` and rename: a crash never leaves a
    truncated file under the final name.  Sink "discard" writes the same
    bytes to /dev/null instead (the whole pipeline but the file system: a
    steady-state measurement of render, encode, copy and writer threads)."""
    if sink == "discard":
        fn(os.devnull, *args)
        return
    tmp = path + ".tmp"
    fn(tmp, *args)
    os.replace(tmp, path)


def _write_png(path: str, rgb: np.ndarray) -> None:
    from . import writers as fileio
    # zlib level 1 with run-length matches only: ~2x faster than the default
    # strategy on rendered frames for ~2% more bytes (tools/gen_bench.py)
    fileio.write_png(path, rgb, level=1, strategy="rle")


def _write_bytes(path: str, data) -> None:
    """Write a buffer (os.write releases the GIL)."""
    fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
    try:
        mv = memoryview(data)
        while mv:
            n = os.write(fd, mv)
            mv = mv[n:]
    finally:
        os.close(fd)


POINTCLOUD_HEADER = b"x y z r g b\n"   # the TXT's first line (np.savetxt header, GDP:766-770)


def write_frame(arrays: Dict[str, np.ndarray], k: int, files: List[Tuple[str, str, Tuple[str, ...]]],
                label: dict, label_path: str, sink: str = "disk") -> Optional[dict]:
    """Every file of frame ``k`` of a batch, then its label JSON (the resume
    marker, GDP:1357-1367 scans labels/).  ``files`` = (path, kind, array
    names); kind "encoded" names the file index j in the batch's files
    encoded on the GPU (arrays "files" + "file_offsets"); ``label`` is the
    label dict, or a callable that writes the label file to the path it is
    given (writers.LabelWriter); returns the frame's depth counts for the
    quality log.  ``sink`` "discard": every file goes to /dev/null."""
    from . import writers as fileio
    from .labels import label_json_bytes
    for path, kind, keys in files:
        if kind in ("encoded", "encoded_pointcloud"):
            off = arrays["file_offsets"]
            j = keys[0]
            data = arrays["files"][int(off[j]):int(off[j + 1])]
            # a frame without a single point gets no point-cloud file, as in the
            # reference (save_pointcloud_with_rgb returns on an empty cloud,
            # GDP:723-725; the depth fallback saves only len(xyzrgb) > 0, :1755)
            if kind == "encoded_pointcloud" and len(data) <= len(POINTCLOUD_HEADER):
                continue
            _atomic(path, _write_bytes, data, sink=sink)
            continue
        a = [arrays[x][k] for x in keys]
        if kind == "pointcloud" and np.isnan(a[0]).all():   # no point: no file (GDP:723-725, :1755)
            continue
        if kind == "png":
            _atomic(path, _write_png, *a, sink=sink)
        elif kind == "npy":
            _atomic(path, fileio.write_npy, *a, sink=sink)
        elif kind == "csv":
            _atomic(path, fileio.write_depth_csv, *a, sink=sink)
        elif kind == "pointcloud":
            _atomic(path, fileio.write_pointcloud_txt, *a, sink=sink)
        else:
            raise ValueError(kind)
    if callable(label):   # a native label writer job (writers.LabelWriter.write bound to the frame)
        _atomic(label_path, label, sink=sink)
    else:
        _atomic(label_path, _write_bytes, label_json_bytes(label), sink=sink)
    return fileio.depth_stats(arrays["depth"][k]) if "depth" in arrays else None


# -- worker-process side ---------------------------------------------------------
_ATTACHED: Dict[str, object] = {}


def _views(shm_name: str, slot_bytes: int, layout: Layout, slot: int) -> Dict[str, np.ndarray]:
    from multiprocessing import shared_memory
    shm = _ATTACHED.get(shm_name)
    if shm is None:
        # (attaching registers the name with the parent's resource tracker
        # again, a no-op: the parent unlinks it and unregisters it once)
        shm = shared_memory.SharedMemory(name=shm_name)
        _ATTACHED[shm_name] = shm
    base = slot * slot_bytes
    return {k: np.ndarray(shape, np.dtype(dt), buffer=shm.buf, offset=base + off)
            for k, (off, shape, dt) in layout.items()}


def _task(shm_name, slot_bytes, layout, slot, k, files, label, label_path, sink):
    return write_frame(_views(shm_name, slot_bytes, layout, slot), k, files, label, label_path, sink)


def _ping() -> int:
    return os.getpid()


# -- parent side -----------------------------------------------------------------
class WriterPool:
    """``n_slots`` batch buffers shaped by ``spec`` (name -> (shape, dtype) of
    one batch, Renderer.output_spec) and ``workers`` writer processes (mode
    "process") or threads (mode "thread")."""

    def __init__(self, spec: Dict[str, tuple], workers: int, n_slots: int = 3, mode: str = "process",
                 sink: str = "disk"):
        if sink not in SINKS:
            raise ValueError(f"sink {sink!r}: choose from {SINKS}")
        self.mode = mode
        self.sink = sink
        self.workers = workers
        self.task_s, self.tasks = 0.0, 0   # thread mode: summed wall time of the frame tasks
        self.layout: Layout = {}
        off = 0
        for k, (shape, dt) in spec.items():
            off = (off + 255) & ~255
            self.layout[k] = (off, tuple(int(x) for x in shape), np.dtype(dt).str)
            off += int(np.prod(shape)) * np.dtype(dt).itemsize
        self.slot_bytes = (off + 4095) & ~4095
        self.n_slots = n_slots
        self.busy: List[List[Future]] = [[] for _ in range(n_slots)]
        self.shm = None
        if mode == "process":
            from multiprocessing import shared_memory
            self.shm = shared_memory.SharedMemory(create=True, size=max(self.slot_bytes * n_slots, 1))
            self.pool = ProcessPoolExecutor(max_workers=workers, mp_context=mp.get_context("spawn"))
            # start every worker now, before the parent initialises the GPU
            for f in [self.pool.submit(_ping) for _ in range(workers)]:
                f.result()
            self._local = None
        elif mode == "thread":
            self.pool = ThreadPoolExecutor(max_workers=workers)
            self._task_lock = threading.Lock()
            self._local = [{k: np.empty(shape, np.dtype(dt)) for k, (_, shape, dt) in self.layout.items()}
                           for _ in range(n_slots)]
        else:
            raise ValueError(f"writer mode {mode!r}: 'process' or 'thread'")

    def use_pinned(self, alloc, files_bytes: int = 0, free=None) -> None:
        """Thread mode: the slots' arrays in page-locked memory from
        ``alloc(nbytes)`` (Renderer.host_buffer: device-to-host copies at full
        PCIe rate), plus a ``files`` buffer of ``files_bytes`` per slot for the
        files the GPU encodes (Renderer.render_files); ``free(array)``
        (Renderer.free_host_buffer) releases a replaced files buffer."""
        assert self._local is not None, "pinned slots need writer threads"
        self.free = free
        self._grow_lock = threading.Lock()
        self._files_free = {}          # slot -> free() of its current files buffer's renderer
        self._retired = []             # (replaced files buffer, its free()): release_retired() / close()
        for slot in range(self.n_slots):
            buf = alloc(self.slot_bytes)
            d = {k: np.ndarray(shape, np.dtype(dt), buffer=buf, offset=off)
                 for k, (off, shape, dt) in self.layout.items()}
            if files_bytes:
                d["files"] = alloc(files_bytes)
            self._local[slot] = d
        self.alloc = alloc

    def grow_files(self, slot: int, nbytes: int, alloc=None, free=None) -> np.ndarray:
        """A larger ``files`` buffer for a slot (the batch's files did not
        fit), from ``alloc`` / to be released by ``free``: the growing
        renderer's own (Renderer.host_buffer / free_host_buffer), so a
        renderer context is only touched by the thread that renders with it.
        The replaced buffer is retired, not freed here (hipHostFree waits
        for the device, which would stall the other renderer's batch in the
        middle of this one's copy): its owning renderer's thread releases it
        at its next batch (:meth:`release_retired`), and :meth:`close` releases
        whatever is left, so pinned memory does not pile up over a run.
        The lock orders concurrent grows of the renderers' threads."""
        alloc = alloc or self.alloc
        with self._grow_lock:
            old = self._local[slot].get("files")
            self._local[slot]["files"] = alloc(nbytes)
            if old is not None:
                owner = self._files_free.get(slot, self.free)
                if owner is not None:
                    self._retired.append((old, owner))
            self._files_free[slot] = free or self.free
        return self._local[slot]["files"]

    def release_retired(self, free) -> int:
        """Free the retired files buffers whose owner is ``free`` (the calling
        render thread's Renderer.free_host_buffer); returns how many.  A
        retired buffer is no longer any slot's, and the tasks that read it
        finished before its slot was handed out again (:meth:`arrays`)."""
        if not getattr(self, "_retired", None):
            return 0
        with self._grow_lock:
            mine = [a for a, f in self._retired if f == free]
            self._retired = [(a, f) for a, f in self._retired if f != free]
        for a in mine:
            free(a)
        return len(mine)

    @property
    def retired(self) -> int:
        """Files buffers replaced by a grow and not yet released."""
        return len(getattr(self, "_retired", []))

    def arrays(self, slot: int) -> Dict[str, np.ndarray]:
        """The slot's arrays, to render into (waits until no task reads it)."""
        for f in self.busy[slot]:
            f.result()
        self.busy[slot] = []
        if self.shm is not None:
            base = slot * self.slot_bytes
            return {k: np.ndarray(shape, np.dtype(dt), buffer=self.shm.buf, offset=base + off)
                    for k, (off, shape, dt) in self.layout.items()}
        return self._local[slot]

    def submit(self, slot: int, k: int, files, label: dict, label_path: str) -> Future:
        if self.shm is not None:
            f = self.pool.submit(_task, self.shm.name, self.slot_bytes, self.layout, slot, k, files, label,
                                 label_path, self.sink)
        else:
            f = self.pool.submit(self._timed_write, self._local[slot], k, files, label, label_path, self.sink)
        self.busy[slot].append(f)
        return f

    def _timed_write(self, *args):
        """write_frame in a writer thread, its wall time added to ``task_s``."""
        t0 = time.perf_counter()
        try:
            return write_frame(*args)
        finally:
            dt = time.perf_counter() - t0
            with self._task_lock:
                self.task_s += dt
                self.tasks += 1

    def close(self) -> None:
        for fs in self.busy:
            for f in fs:
                f.result()
        self.pool.shutdown()
        for arr, free in getattr(self, "_retired", []):
            free(arr)
        self._retired = []
        if self.shm is not None:
            try:
                self.shm.close()
            except BufferError:   # a caller still holds a view of a slot: the mapping goes with it
                pass
            self.shm.unlink()
            self.shm = None
