"""ctypes binding of the gfx950 vector-search core (include/vdb.h, lib/libvdb_amd.so).

This is the only way the store reaches the device.  There is no CPU fallback:
if the shared library is missing, or no gfx950 device is visible, every
constructor here raises.  (The CPU oracle under ``oracle/`` is test
infrastructure and is never imported by this package.)
"""
from __future__ import annotations

import ctypes
import os
import threading
from pathlib import Path
from typing import Optional, Tuple

import numpy as np

_PKG_ROOT = Path(__file__).resolve().parent.parent
_DEFAULT_LIB = _PKG_ROOT / "lib" / "libvdb_amd.so"

VDB_OK = 0
VDB_ERR_INVALID = -1
VDB_ERR_HIP = -2
VDB_ERR_OOM = -3
VDB_ERR_NONFINITE = -4
VDB_ERR_UNSUPPORTED = -5
VDB_ERR_NODEVICE = -6

METRIC_IDS = {"cosine": 0, "euclidean": 1}
# candidate-pass arithmetic (include/vdb.h VDB_PREC_*); results are identical, speed differs
PRECISION_IDS = {"fp32": 0, "bf16x3": 1, "bf16": 2, "auto": 3, "i8": 4, "i8x3": 5, "i8q": 6}
MEM_HOST = 0
MEM_DEVICE = 1
# largest beam (ef) vdb_graph_search accepts (csrc/vdb_graph.hip GS_EF_MAX)
GRAPH_EF_MAX = 256

# Every symbol include/vdb.h declares (tests/test_abi.py checks the .so exports them).
EXPORTED_SYMBOLS = (
    "vdb_last_error", "vdb_version", "vdb_device_count",
    "vdb_index_create", "vdb_index_destroy", "vdb_index_reserve",
    "vdb_index_set_param", "vdb_index_get_stat",
    "vdb_index_add", "vdb_index_count", "vdb_index_clear", "vdb_index_get_vectors",
    "vdb_index_search", "vdb_merge_topk", "vdb_similarity_matrix", "vdb_normalize_rows", "vdb_topk_scores",
    "vdb_graph_build", "vdb_graph_import", "vdb_graph_export", "vdb_graph_add", "vdb_graph_info", "vdb_graph_search",
    "vdb_graph_stat", "vdb_graph_set_param", "vdb_graph_destroy",
    "vdb_shards_create", "vdb_shards_destroy", "vdb_shards_add", "vdb_shards_count", "vdb_shards_shard_count",
    "vdb_shards_search", "vdb_shards_search_device", "vdb_shards_get_vectors", "vdb_shards_clear", "vdb_shards_reserve",
    "vdb_shards_set_param", "vdb_shards_get_stat", "vdb_shutdown",
)

_lib = None
_lib_lock = threading.Lock()


class VDBError(RuntimeError):
    """A failing vdb_* call (HIP error, out of memory, no device)."""


def library_path() -> Path:
    return Path(os.environ.get("VDB_LIB", str(_DEFAULT_LIB)))


def _prefer_torch_runtime() -> None:
    # torch bundles its own libamdhip64.so.7; load it first so the process has
    # one HIP runtime whichever of torch / this library is imported first.
    try:  # pragma: no cover - depends on the environment
        import torch  # noqa: F401
    except Exception:
        pass


def load_library():
    """Load (once) and type the C-ABI.  Raises ImportError if it is not built."""
    global _lib
    with _lib_lock:
        if _lib is not None:
            return _lib
        path = library_path()
        if not path.exists():
            raise ImportError(
                f"vdb HIP library not found at {path}; build it with "
                f"`make -C {_PKG_ROOT}` (hipcc --offload-arch=gfx950)")
        _prefer_torch_runtime()
        lib = ctypes.CDLL(str(path))
        c_i32, c_i64, c_vp = ctypes.c_int32, ctypes.c_int64, ctypes.c_void_p
        p_i64 = ctypes.POINTER(ctypes.c_int64)
        sig = {
            "vdb_last_error": (ctypes.c_char_p, []),
            "vdb_version": (c_i32, []),
            "vdb_device_count": (c_i32, [ctypes.POINTER(ctypes.c_int32)]),
            "vdb_index_create": (c_i32, [c_i32, c_i32, c_i32, ctypes.POINTER(c_vp)]),
            "vdb_index_destroy": (c_i32, [c_vp]),
            "vdb_index_reserve": (c_i32, [c_vp, c_i64]),
            "vdb_index_set_param": (c_i32, [c_vp, ctypes.c_char_p, c_i64]),
            "vdb_index_get_stat": (c_i32, [c_vp, ctypes.c_char_p, p_i64]),
            "vdb_index_add": (c_i32, [c_vp, c_vp, c_i64, c_i32, c_vp]),
            "vdb_index_count": (c_i32, [c_vp, p_i64]),
            "vdb_index_clear": (c_i32, [c_vp]),
            "vdb_index_get_vectors": (c_i32, [c_vp, c_i64, c_i64, c_vp]),
            "vdb_index_search": (c_i32, [c_vp, c_vp, c_i32, c_i32, c_vp, c_i32, c_vp, c_vp, c_vp, c_i64, c_vp]),
            "vdb_merge_topk": (c_i32, [c_vp, c_vp, c_i32, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp]),
            "vdb_similarity_matrix": (c_i32, [c_vp, c_i64, c_i32, c_vp, c_i32, c_i32, c_vp, c_vp]),
            "vdb_normalize_rows": (c_i32, [c_vp, c_i64, c_i32, c_vp, c_vp]),
            "vdb_topk_scores": (c_i32, [c_vp, c_i32, c_i64, c_i32, c_i32, c_vp, c_vp, c_vp]),
            "vdb_graph_build": (c_i32, [c_vp, c_i32, c_i32, c_i32, ctypes.POINTER(c_vp)]),
            "vdb_graph_import": (c_i32, [c_vp, c_i32, c_i64, c_vp, c_i32, c_vp, ctypes.POINTER(c_vp)]),
            "vdb_graph_export": (c_i32, [c_vp, c_vp, c_vp]),
            "vdb_graph_add": (c_i32, [c_vp]),
            "vdb_graph_info": (c_i32, [c_vp, p_i64, ctypes.POINTER(c_i32), ctypes.POINTER(c_i32)]),
            "vdb_graph_search": (c_i32, [c_vp, c_vp, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp, c_vp]),
            "vdb_graph_stat": (c_i32, [c_vp, ctypes.c_char_p, p_i64]),
            "vdb_graph_set_param": (c_i32, [c_vp, ctypes.c_char_p, c_i64]),
            "vdb_graph_destroy": (c_i32, [c_vp]),
            "vdb_shards_create": (c_i32, [c_i32, c_i32, c_vp, c_i32, ctypes.POINTER(c_vp)]),
            "vdb_shards_destroy": (c_i32, [c_vp]),
            "vdb_shards_add": (c_i32, [c_vp, c_vp, c_i64]),
            "vdb_shards_count": (c_i32, [c_vp, p_i64]),
            "vdb_shards_shard_count": (c_i32, [c_vp, c_i32, p_i64]),
            "vdb_shards_search": (c_i32, [c_vp, c_vp, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp]),
            "vdb_shards_search_device": (c_i32, [c_vp, c_vp, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp]),
            "vdb_shards_get_vectors": (c_i32, [c_vp, c_i64, c_i64, c_vp]),
            "vdb_shards_clear": (c_i32, [c_vp]),
            "vdb_shards_reserve": (c_i32, [c_vp, c_i64]),
            "vdb_shards_set_param": (c_i32, [c_vp, ctypes.c_char_p, c_i64]),
            "vdb_shards_get_stat": (c_i32, [c_vp, ctypes.c_char_p, p_i64]),
            "vdb_shutdown": (c_i32, []),
        }
        for name, (res, args) in sig.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


def _check(rc: int) -> None:
    if rc == VDB_OK:
        return
    msg = _lib.vdb_last_error().decode("utf-8", "replace")
    if rc in (VDB_ERR_INVALID, VDB_ERR_NONFINITE):
        raise ValueError(msg)
    raise VDBError(f"vdb error {rc}: {msg}")


def device_count() -> int:
    lib = load_library()
    n = ctypes.c_int32(0)
    lib.vdb_device_count(ctypes.byref(n))
    return int(n.value)


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


class NativeIndex:
    """One device-resident corpus (tiled fp32 + norms) on one GPU."""

    def __init__(self, dim: int, metric: str = "cosine", device: int = 0, precision: Optional[str] = None):
        if metric not in METRIC_IDS:
            raise ValueError(f"unsupported metric {metric!r}; the vdb core implements {sorted(METRIC_IDS)}")
        self._lib = load_library()
        self.dim = int(dim)
        self.metric = metric
        self.device = int(device)
        h = ctypes.c_void_p()
        _check(self._lib.vdb_index_create(self.dim, METRIC_IDS[metric], self.device, ctypes.byref(h)))
        self._h = h
        if precision is not None:
            self.set_precision(precision)

    # -- lifecycle -------------------------------------------------------------
    def close(self) -> None:
        h, self._h = getattr(self, "_h", None), None
        if h:
            self._lib.vdb_index_destroy(h)

    def __del__(self):  # pragma: no cover - GC timing
        try:
            self.close()
        except Exception:
            pass

    def reserve(self, rows: int) -> None:
        _check(self._lib.vdb_index_reserve(self._h, int(rows)))

    def set_param(self, name: str, value: int) -> None:
        _check(self._lib.vdb_index_set_param(self._h, name.encode(), int(value)))

    def set_precision(self, precision: str) -> None:
        if precision not in PRECISION_IDS:
            raise ValueError(f"precision must be one of {sorted(PRECISION_IDS)}, got {precision!r}")
        self.set_param("precision", PRECISION_IDS[precision])

    @property
    def precision(self) -> str:
        v = self.stat("precision")
        return next(k for k, i in PRECISION_IDS.items() if i == v)

    def stat(self, name: str) -> int:
        v = ctypes.c_int64(0)
        _check(self._lib.vdb_index_get_stat(self._h, name.encode(), ctypes.byref(v)))
        return int(v.value)

    # -- data ------------------------------------------------------------------
    def add(self, vectors: np.ndarray) -> None:
        v = np.ascontiguousarray(vectors, dtype=np.float32)
        if v.ndim != 2 or v.shape[1] != self.dim:
            raise ValueError(f"vectors must have shape (n, {self.dim}), got {v.shape}")
        if v.shape[0] == 0:
            return
        _check(self._lib.vdb_index_add(self._h, _ptr(v), v.shape[0], MEM_HOST, None))

    def add_device(self, ptr: int, n: int, stream: int = 0) -> None:
        _check(self._lib.vdb_index_add(self._h, ctypes.c_void_p(ptr), int(n), MEM_DEVICE, ctypes.c_void_p(stream)))

    def count(self) -> int:
        n = ctypes.c_int64(0)
        _check(self._lib.vdb_index_count(self._h, ctypes.byref(n)))
        return int(n.value)

    def clear(self) -> None:
        _check(self._lib.vdb_index_clear(self._h))

    def get_vectors(self, start: int = 0, n: Optional[int] = None) -> np.ndarray:
        total = self.count()
        n = total - start if n is None else n
        out = np.empty((max(n, 0), self.dim), dtype=np.float32)
        if n > 0:
            _check(self._lib.vdb_index_get_vectors(self._h, int(start), int(n), _ptr(out)))
        return out

    # -- search ----------------------------------------------------------------
    def search(self, queries: np.ndarray, k: int, row_mask: Optional[np.ndarray] = None,
               with_keys: bool = False, index_offset: int = 0):
        """Host-memory search.  Returns (scores f32 [B,k], indices i64 [B,k][, keys f64 [B,k]])."""
        q = np.ascontiguousarray(queries, dtype=np.float32)
        if q.ndim == 1:
            q = q[None, :]
        if q.ndim != 2 or q.shape[1] != self.dim:
            raise ValueError(f"queries must have shape (B, {self.dim}), got {np.shape(queries)}")
        B = q.shape[0]
        k = int(k)
        scores = np.empty((B, k), dtype=np.float32)
        idx = np.empty((B, k), dtype=np.int64)
        keys = np.empty((B, k), dtype=np.float64) if with_keys else None
        mask_p = None
        if row_mask is not None:
            m = np.ascontiguousarray(row_mask, dtype=np.uint32)
            need = (self.count() + 31) // 32
            if m.size < need:
                raise ValueError(f"row_mask needs {need} uint32 words, got {m.size}")
            mask_p = _ptr(m)
        _check(self._lib.vdb_index_search(self._h, _ptr(q), B, k, mask_p, MEM_HOST, _ptr(scores), _ptr(idx),
                                          _ptr(keys) if keys is not None else None, int(index_offset), None))
        return (scores, idx, keys) if with_keys else (scores, idx)

    def search_device(self, q_ptr: int, n_queries: int, k: int, out_scores_ptr: int, out_idx_ptr: int,
                      out_keys_ptr: int = 0, mask_ptr: int = 0, index_offset: int = 0, stream: int = 0) -> None:
        """Device-memory search (pointers from torch tensors); stream-ordered."""
        _check(self._lib.vdb_index_search(
            self._h, ctypes.c_void_p(q_ptr), int(n_queries), int(k), ctypes.c_void_p(mask_ptr or None),
            MEM_DEVICE, ctypes.c_void_p(out_scores_ptr), ctypes.c_void_p(out_idx_ptr),
            ctypes.c_void_p(out_keys_ptr or None), int(index_offset), ctypes.c_void_p(stream or None)))


class NativeShards:
    """One corpus row-sharded over several GPUs of this process (include/vdb.h vdb_shards_*):
    the same interface as NativeIndex for the store; results identical to one index."""

    def __init__(self, dim: int, metric: str = "cosine", devices=(0,), precision: Optional[str] = None):
        if metric not in METRIC_IDS:
            raise ValueError(f"unsupported metric {metric!r}; the vdb core implements {sorted(METRIC_IDS)}")
        devices = [int(d) for d in devices]
        if not devices:
            raise ValueError("devices must name at least one GPU")
        self._lib = load_library()
        self.dim = int(dim)
        self.metric = metric
        self.devices = devices
        dv = (ctypes.c_int32 * len(devices))(*devices)
        h = ctypes.c_void_p()
        _check(self._lib.vdb_shards_create(self.dim, METRIC_IDS[metric], dv, len(devices), ctypes.byref(h)))
        self._h = h
        if precision is not None:
            self.set_param("precision", PRECISION_IDS[precision])

    def close(self) -> None:
        h, self._h = getattr(self, "_h", None), None
        if h:
            self._lib.vdb_shards_destroy(h)

    def __del__(self):  # pragma: no cover - GC timing
        try:
            self.close()
        except Exception:
            pass

    def reserve(self, rows: int) -> None:
        _check(self._lib.vdb_shards_reserve(self._h, int(rows)))

    def set_param(self, name: str, value: int) -> None:
        _check(self._lib.vdb_shards_set_param(self._h, name.encode(), int(value)))

    def stat(self, name: str) -> int:
        v = ctypes.c_int64(0)
        _check(self._lib.vdb_shards_get_stat(self._h, name.encode(), ctypes.byref(v)))
        return int(v.value)

    def shard_counts(self):
        out = []
        for g in range(len(self.devices)):
            v = ctypes.c_int64(0)
            _check(self._lib.vdb_shards_shard_count(self._h, g, ctypes.byref(v)))
            out.append(int(v.value))
        return out

    def add(self, vectors: np.ndarray) -> None:
        v = np.ascontiguousarray(vectors, dtype=np.float32)
        if v.ndim != 2 or v.shape[1] != self.dim:
            raise ValueError(f"vectors must have shape (n, {self.dim}), got {v.shape}")
        if v.shape[0]:
            _check(self._lib.vdb_shards_add(self._h, _ptr(v), v.shape[0]))

    def count(self) -> int:
        n = ctypes.c_int64(0)
        _check(self._lib.vdb_shards_count(self._h, ctypes.byref(n)))
        return int(n.value)

    def clear(self) -> None:
        _check(self._lib.vdb_shards_clear(self._h))

    def get_vectors(self, start: int = 0, n: Optional[int] = None) -> np.ndarray:
        total = self.count()
        n = total - start if n is None else n
        out = np.empty((max(n, 0), self.dim), dtype=np.float32)
        if n > 0:
            _check(self._lib.vdb_shards_get_vectors(self._h, int(start), int(n), _ptr(out)))
        return out

    def search(self, queries: np.ndarray, k: int, row_mask: Optional[np.ndarray] = None, with_keys: bool = False):
        q = np.ascontiguousarray(queries, dtype=np.float32)
        if q.ndim == 1:
            q = q[None, :]
        if q.ndim != 2 or q.shape[1] != self.dim:
            raise ValueError(f"queries must have shape (B, {self.dim}), got {np.shape(queries)}")
        B, k = q.shape[0], int(k)
        scores = np.empty((B, k), dtype=np.float32)
        idx = np.empty((B, k), dtype=np.int64)
        keys = np.empty((B, k), dtype=np.float64) if with_keys else None
        mask_p = None
        if row_mask is not None:
            m = np.ascontiguousarray(row_mask, dtype=np.uint32)
            need = (self.count() + 31) // 32
            if m.size < need:
                raise ValueError(f"row_mask needs {need} uint32 words, got {m.size}")
            mask_p = _ptr(m)
        _check(self._lib.vdb_shards_search(self._h, _ptr(q), B, k, mask_p, _ptr(scores), _ptr(idx),
                                           _ptr(keys) if keys is not None else None))
        return (scores, idx, keys) if with_keys else (scores, idx)


def _shards_search_device(self, q_ptr: int, n_queries: int, k: int, out_scores_ptr: int, out_idx_ptr: int,
                          out_keys_ptr: int = 0, mask_ptr: int = 0, stream: int = 0) -> None:
    """Stream-ordered search of every shard (all pointers on devices[0], no host wait)."""
    _check(self._lib.vdb_shards_search_device(
        self._h, ctypes.c_void_p(q_ptr), int(n_queries), int(k), ctypes.c_void_p(mask_ptr or None),
        ctypes.c_void_p(out_scores_ptr), ctypes.c_void_p(out_idx_ptr), ctypes.c_void_p(out_keys_ptr or None),
        ctypes.c_void_p(stream or None)))


NativeShards.search_device = _shards_search_device


def shutdown() -> None:
    """include/vdb.h vdb_shutdown: release idle workspaces of every live index."""
    _check(load_library().vdb_shutdown())


class NativeGraph:
    """The graph index over a NativeIndex's rows (include/vdb.h vdb_graph_*):
    hnswlib-style search results (labels, distances: cosine 1 - cos, L2 squared)."""

    def __init__(self, index: "NativeIndex", handle):
        self.index = index  # keeps the corpus alive
        self._lib = index._lib
        self._h = handle

    @classmethod
    def build(cls, index: "NativeIndex", degree: int = 32, knn: int = 32, n_entries: int = 256) -> "NativeGraph":
        h = ctypes.c_void_p()
        _check(index._lib.vdb_graph_build(index._h, int(degree), int(knn), int(n_entries), ctypes.byref(h)))
        return cls(index, h)

    @classmethod
    def from_arrays(cls, index: "NativeIndex", neighbors: np.ndarray, entries: np.ndarray) -> "NativeGraph":
        nb = np.ascontiguousarray(neighbors, dtype=np.int32)
        en = np.ascontiguousarray(entries, dtype=np.int32)
        if nb.ndim != 2:
            raise ValueError(f"neighbors must be [n, degree], got {nb.shape}")
        h = ctypes.c_void_p()
        _check(index._lib.vdb_graph_import(index._h, nb.shape[1], nb.shape[0], _ptr(nb) if nb.size else None,
                                           en.size, _ptr(en) if en.size else None, ctypes.byref(h)))
        return cls(index, h)

    def add(self) -> None:
        """include/vdb.h vdb_graph_add: insert the rows the index gained since the last
        build / add (incremental, instead of a rebuild)."""
        _check(self._lib.vdb_graph_add(self._h))

    def info(self) -> Tuple[int, int, int]:
        n, d, e = ctypes.c_int64(0), ctypes.c_int32(0), ctypes.c_int32(0)
        _check(self._lib.vdb_graph_info(self._h, ctypes.byref(n), ctypes.byref(d), ctypes.byref(e)))
        return int(n.value), int(d.value), int(e.value)

    def to_arrays(self) -> Tuple[np.ndarray, np.ndarray]:
        n, d, e = self.info()
        nb = np.empty((n, d), np.int32)
        en = np.empty(e, np.int32)
        _check(self._lib.vdb_graph_export(self._h, _ptr(nb) if nb.size else None, _ptr(en) if en.size else None))
        return nb, en

    def search(self, queries: np.ndarray, k: int, ef: int = 100):
        q = np.ascontiguousarray(queries, dtype=np.float32)
        if q.ndim == 1:
            q = q[None, :]
        if q.ndim != 2 or q.shape[1] != self.index.dim:
            raise ValueError(f"queries must have shape (n, {self.index.dim}), got {np.shape(queries)}")
        labels = np.empty((q.shape[0], int(k)), np.int64)
        dist = np.empty((q.shape[0], int(k)), np.float32)
        _check(self._lib.vdb_graph_search(self._h, _ptr(q), q.shape[0], int(k), int(ef), MEM_HOST, _ptr(labels),
                                          _ptr(dist), None))
        return labels, dist

    def search_device(self, q_ptr: int, n_queries: int, k: int, ef: int, labels_ptr: int, dist_ptr: int,
                      stream: int = 0) -> None:
        _check(self._lib.vdb_graph_search(self._h, ctypes.c_void_p(q_ptr), int(n_queries), int(k), int(ef), MEM_DEVICE,
                                          ctypes.c_void_p(labels_ptr), ctypes.c_void_p(dist_ptr),
                                          ctypes.c_void_p(stream or None)))

    def stat(self, name: str) -> int:
        v = ctypes.c_int64(0)
        _check(self._lib.vdb_graph_stat(self._h, name.encode(), ctypes.byref(v)))
        return int(v.value)

    def set_param(self, name: str, value: int) -> None:
        """include/vdb.h vdb_graph_set_param ("teams": workgroups per query)."""
        _check(self._lib.vdb_graph_set_param(self._h, name.encode(), int(value)))

    def close(self) -> None:
        h, self._h = getattr(self, "_h", None), None
        if h:
            self._lib.vdb_graph_destroy(h)

    def __del__(self):  # pragma: no cover - GC timing
        try:
            self.close()
        except Exception:
            pass


def merge_topk_device(keys_ptr: int, idx_ptr: int, n_lists: int, n_queries: int, k_in: int, k_out: int,
                      metric: str, out_scores_ptr: int, out_idx_ptr: int, out_keys_ptr: int = 0,
                      stream: int = 0) -> None:
    lib = load_library()
    _check(lib.vdb_merge_topk(ctypes.c_void_p(keys_ptr), ctypes.c_void_p(idx_ptr), int(n_lists), int(n_queries),
                              int(k_in), int(k_out), METRIC_IDS[metric], ctypes.c_void_p(out_scores_ptr),
                              ctypes.c_void_p(out_idx_ptr), ctypes.c_void_p(out_keys_ptr or None),
                              ctypes.c_void_p(stream or None)))


# the operator slot also serves the dot product (performance/mlx_optimized.py:150-156)
OP_METRIC_IDS = dict(METRIC_IDS, dot_product=2)


def similarity_matrix_device(corpus_ptr: int, n: int, dim: int, q_ptr: int, n_queries: int, metric: str,
                             out_ptr: int, stream: int = 0) -> None:
    lib = load_library()
    _check(lib.vdb_similarity_matrix(ctypes.c_void_p(corpus_ptr), int(n), int(dim), ctypes.c_void_p(q_ptr),
                                     int(n_queries), OP_METRIC_IDS[metric], ctypes.c_void_p(out_ptr),
                                     ctypes.c_void_p(stream or None)))


def normalize_rows_device(in_ptr: int, n: int, dim: int, out_ptr: int, stream: int = 0) -> None:
    _check(load_library().vdb_normalize_rows(ctypes.c_void_p(in_ptr), int(n), int(dim), ctypes.c_void_p(out_ptr),
                                             ctypes.c_void_p(stream or None)))


def topk_scores_device(scores_ptr: int, rows: int, n: int, k: int, largest: bool, out_idx_ptr: int,
                       out_val_ptr: int = 0, stream: int = 0) -> None:
    _check(load_library().vdb_topk_scores(ctypes.c_void_p(scores_ptr), int(rows), int(n), int(k), int(bool(largest)),
                                          ctypes.c_void_p(out_idx_ptr), ctypes.c_void_p(out_val_ptr or None),
                                          ctypes.c_void_p(stream or None)))
