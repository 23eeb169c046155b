"""The reference's compiled-operator module (performance/mlx_optimized.py) on the gfx950 core.

Same function names, argument meaning, return shapes and ValueError checks as
/root/reference/performance/mlx_optimized.py; each function runs device kernels through the
C-ABI (include/vdb.h), never a CPU path:

  compute_cosine_similarity_single / _batch   vdb_similarity_matrix, cosine (fp32 MFMA GEMM)
  compute_euclidean_distance                  vdb_similarity_matrix, euclidean
  compute_dot_product                         vdb_similarity_matrix, dot product
  fast_top_k_indices                          vdb_topk_scores (ties -> lower index)
  normalize_vectors                           vdb_normalize_rows
  optimized_similarity_search / _batch_...    the fused search itself: a device index
                                              (norms once, MFMA candidate pass, exact rerank)
  fast_vector_concatenation, optimized_vector_addition, PerformanceMonitor,
  warmup_compiled_functions                   as in the reference

Arrays: numpy arrays (or anything np.asarray takes) in -> numpy arrays out; torch CUDA
tensors in -> torch CUDA tensors out (device resident, no host round trip: a CUDA corpus is
ingested device to device into an index cached per tensor version, _device_index).  PyTorch
is only the device-memory container here.
"""
from __future__ import annotations

import logging
import threading
import time
from typing import Dict, Tuple

import numpy as np

from service import _vdb

logger = logging.getLogger("mlx_vector_db.optimized")


def _torch():
    import torch
    return torch


def _ndim(a) -> int:
    return len(a.shape) if hasattr(a, "shape") else np.ndim(a)


def _is_dev(a) -> bool:
    return hasattr(a, "is_cuda") and bool(a.is_cuda)


def _dev(a):
    """(device fp32 contiguous tensor, returned-as-torch flag)."""
    torch = _torch()
    if _is_dev(a):
        return a.detach().to(torch.float32).contiguous(), True
    arr = np.ascontiguousarray(np.asarray(a, dtype=np.float32))
    return torch.from_numpy(arr).cuda(), False


def _out(t, as_torch: bool):
    return t if as_torch else t.cpu().numpy()


def _stream(t) -> int:
    return _torch().cuda.current_stream(t.device).cuda_stream


def _matrix(queries2d, db, metric: str):
    q, qt = _dev(queries2d)
    x, xt = _dev(db)
    torch = _torch()
    out = torch.empty((q.shape[0], x.shape[0]), dtype=torch.float32, device=x.device)
    if x.shape[0] and q.shape[0]:
        _vdb.similarity_matrix_device(x.data_ptr(), x.shape[0], x.shape[1], q.data_ptr(), q.shape[0], metric,
                                      out.data_ptr(), _stream(x))
    return out, (qt or xt)


def compute_cosine_similarity_single(query_vector, db_vectors):
    """mlx_optimized.py:26-57: 1-D scores of one query (1-D or one-row 2-D)."""
    q = query_vector
    shape = tuple(q.shape) if hasattr(q, "shape") else np.shape(q)
    if len(shape) == 1:
        q = q.reshape(1, -1)
    elif not (len(shape) == 2 and shape[0] == 1):
        raise ValueError(f"query_vector muss 1D oder 2D mit einer Zeile sein, erhielt Shape {shape}")
    out, t = _matrix(q, db_vectors, "cosine")
    return _out(out.reshape(-1), t)


def compute_cosine_similarity_batch(query_vectors, db_vectors):
    """mlx_optimized.py:59-88: [B, N] scores, with the reference's shape checks."""
    qs = tuple(query_vectors.shape) if hasattr(query_vectors, "shape") else np.shape(query_vectors)
    ds = tuple(db_vectors.shape) if hasattr(db_vectors, "shape") else np.shape(db_vectors)
    if len(qs) != 2:
        raise ValueError(f"query_vectors muss 2D sein, erhielt Shape {qs}")
    if len(ds) != 2:
        raise ValueError(f"db_vectors muss 2D sein, erhielt Shape {ds}")
    if qs[1] != ds[1]:
        raise ValueError(f"Dimension Mismatch: query_vectors Dim {qs[1]}, db_vectors Dim {ds[1]}")
    out, t = _matrix(query_vectors, db_vectors, "cosine")
    return _out(out, t)


def fast_top_k_indices(scores, k: int):
    """mlx_optimized.py:90-108: indices of the k highest scores, best first (ties to the lower
    index); empty for k <= 0."""
    s, t = _dev(scores)
    if s.ndim != 1:
        raise ValueError("scores muss ein 1D mx.array sein.")
    torch = _torch()
    kk = min(int(k), s.shape[0])
    if k <= 0 or kk == 0:
        return _out(torch.zeros(0, dtype=torch.int32, device=s.device), t)
    idx = torch.empty(kk, dtype=torch.int64, device=s.device)
    _vdb.topk_scores_device(s.data_ptr(), 1, s.shape[0], kk, True, idx.data_ptr(), 0, _stream(s))
    return _out(idx.to(torch.int32), t)


def normalize_vectors(vectors):
    """mlx_optimized.py:110-125."""
    v, t = _dev(vectors)
    if v.ndim != 2:
        raise ValueError(f"vectors muss 2D sein für Normalisierung, erhielt Shape {tuple(v.shape)}")
    out = _torch().empty_like(v)
    if v.shape[0]:
        _vdb.normalize_rows_device(v.data_ptr(), v.shape[0], v.shape[1], out.data_ptr(), _stream(v))
    return _out(out, t)


def fast_vector_concatenation(existing_vectors, new_vectors):
    """mlx_optimized.py:127-137 (an O(N) copy; the store appends in place instead)."""
    if existing_vectors.shape[0] == 0:
        return new_vectors
    if new_vectors.shape[0] == 0:
        return existing_vectors
    if existing_vectors.shape[1] != new_vectors.shape[1]:
        raise ValueError("Dimensionen der zu konkatenierenden Vektoren stimmen nicht überein.")
    if _is_dev(existing_vectors) or _is_dev(new_vectors):
        a, _ = _dev(existing_vectors)
        b, _ = _dev(new_vectors)
        return _torch().cat([a, b], dim=0)
    return np.concatenate([np.asarray(existing_vectors), np.asarray(new_vectors)], axis=0)


def compute_euclidean_distance(query_vector, db_vectors):
    """mlx_optimized.py:139-148: sqrt(sum((db - q)^2, axis=1)) for one query."""
    q = query_vector.reshape(1, -1) if _ndim(query_vector) == 1 else query_vector
    out, t = _matrix(q, db_vectors, "euclidean")
    return _out(out.reshape(-1) if out.shape[0] == 1 else out, t)


def compute_dot_product(query_vector, db_vectors):
    """mlx_optimized.py:150-156: db @ q for a 1-D query; (db @ Q^T).flatten() ([N, B] order)
    for a 2-D one."""
    nd = _ndim(query_vector)
    q = query_vector.reshape(1, -1) if nd == 1 else query_vector
    out, t = _matrix(q, db_vectors, "dot_product")  # [B, N]
    res = out.reshape(-1) if nd == 1 else out.t().contiguous().reshape(-1)
    return _out(res, t)


class PerformanceMonitor:
    """mlx_optimized.py:159-196."""

    def __init__(self):
        self.call_counts: Dict[str, int] = {}
        self.total_times: Dict[str, float] = {}
        self._lock = threading.Lock()

    def record_call(self, func_name: str, duration: float):
        with self._lock:
            self.call_counts[func_name] = self.call_counts.get(func_name, 0) + 1
            self.total_times[func_name] = self.total_times.get(func_name, 0.0) + duration

    def get_stats(self) -> dict:
        with self._lock:
            stats = {}
            for name, calls in self.call_counts.items():
                if calls == 0:
                    continue
                avg = self.total_times[name] / calls
                stats[name] = {"calls": calls, "total_time_seconds": round(self.total_times[name], 4),
                               "avg_time_ms": round(avg * 1000, 4),
                               "calls_per_second": round(1.0 / avg if avg > 0 else 0, 2)}
            return stats

    def reset(self):
        with self._lock:
            self.call_counts.clear()
            self.total_times.clear()
        logger.info("PerformanceMonitor has been reset.")


performance_monitor = PerformanceMonitor()


# Device corpora (torch CUDA tensors) are ingested device to device into an index that is kept
# for the next call with the same tensor (same object, storage, shape and version counter:
# an in-place write bumps `_version`), so a caller searching one corpus tensor repeatedly --
# what the reference's batched search is for -- pays the ingest (norms, split copy) once.
_DEV_CACHE_SIZE = 2
_dev_cache: "OrderedDict" = None
_dev_lock = threading.Lock()


def _device_index(db):
    """A device index holding the rows of CUDA tensor `db` (cached, see above)."""
    import weakref
    from collections import OrderedDict
    global _dev_cache
    torch = _torch()
    key = (db.data_ptr(), tuple(db.shape), tuple(db.stride()), str(db.dtype), db.device.index, db._version)
    with _dev_lock:
        if _dev_cache is None:
            _dev_cache = OrderedDict()
        hit = _dev_cache.get(key)
        if hit is not None and hit[0]() is db:
            _dev_cache.move_to_end(key)
            return hit[1]
    x = db.detach().to(torch.float32).contiguous()
    ix = _vdb.NativeIndex(x.shape[1], "cosine", x.device.index)
    ix.reserve(x.shape[0])
    ix.add_device(x.data_ptr(), x.shape[0], _stream(x))  # device to device, after the caller's stream
    with _dev_lock:
        _dev_cache[key] = (weakref.ref(db), ix)
        # an evicted index is only dropped, never closed here: another thread may have taken it
        # from the cache a moment ago and be searching it; the last reference frees it
        while len(_dev_cache) > _DEV_CACHE_SIZE:
            _dev_cache.popitem(last=False)
    return ix


def _search(query_vectors, db_vectors, k: int):
    """The fused device search (norms once, candidate pass, exact rerank); (indices int64
    [B, k'], scores fp32 [B, k']) with k' = min(k, N).  A CUDA-tensor corpus stays on the
    device (device-to-device ingest, device queries and outputs, torch tensors returned); a
    host corpus goes through a transient index (numpy out)."""
    if _is_dev(db_vectors):
        torch = _torch()
        N = db_vectors.shape[0]
        q, _ = _dev(query_vectors)
        q = q.to(db_vectors.device)
        B = q.shape[0]
        kk = min(int(k), N)
        if N == 0 or kk <= 0:
            z = dict(device=db_vectors.device)
            return torch.zeros((B, 0), dtype=torch.int64, **z), torch.zeros((B, 0), dtype=torch.float32, **z)
        ix = _device_index(db_vectors)
        s = torch.empty((B, kk), dtype=torch.float32, device=q.device)
        i = torch.empty((B, kk), dtype=torch.int64, device=q.device)
        ix.search_device(q.data_ptr(), B, kk, s.data_ptr(), i.data_ptr(), 0, stream=_stream(q))
        return i, s
    x = np.asarray(db_vectors, np.float32)
    q = query_vectors.detach().cpu().numpy() if _is_dev(query_vectors) else np.asarray(query_vectors, np.float32)
    B = q.shape[0]
    kk = min(int(k), x.shape[0])
    if x.shape[0] == 0 or kk <= 0:
        return np.zeros((B, 0), np.int64), np.zeros((B, 0), np.float32)
    ix = _vdb.NativeIndex(x.shape[1], "cosine", _torch().cuda.current_device())
    try:
        ix.add(x)
        s, i = ix.search(q, kk)
    finally:
        ix.close()
    return i, s


def optimized_similarity_search(query_vector, db_vectors, k: int = 10) -> Tuple:
    """mlx_optimized.py:199-215: (top_k_indices, top_k_scores) of one cosine query."""
    shape = tuple(query_vector.shape) if hasattr(query_vector, "shape") else np.shape(query_vector)
    if len(shape) == 2 and shape[0] == 1:
        q = query_vector.reshape(-1)
    elif len(shape) == 1:
        q = query_vector
    else:
        raise ValueError(f"query_vector muss 1D oder 2D (1 Zeile) sein, Shape: {shape}")
    t0 = time.perf_counter()
    i, s = _search(q.reshape(1, -1), db_vectors, k)
    performance_monitor.record_call("optimized_similarity_search", time.perf_counter() - t0)
    if _is_dev(query_vector) and not _is_dev(db_vectors):
        torch = _torch()
        return torch.from_numpy(i[0]).to(query_vector.device), torch.from_numpy(s[0]).to(query_vector.device)
    return i[0], s[0]


def optimized_batch_similarity_search(query_vectors, db_vectors, k: int = 10) -> Tuple:
    """mlx_optimized.py:217-248: (all_top_k_indices [B, k'], all_top_k_scores [B, k'])."""
    t0 = time.perf_counter()
    i, s = _search(query_vectors, db_vectors, k)
    performance_monitor.record_call("optimized_batch_similarity_search", time.perf_counter() - t0)
    if _is_dev(query_vectors) and not _is_dev(db_vectors):
        torch = _torch()
        return torch.from_numpy(i).to(query_vectors.device), torch.from_numpy(s).to(query_vectors.device)
    return i, s


def optimized_vector_addition(existing_vectors, new_vectors, normalize: bool = False):
    """mlx_optimized.py:250-255."""
    combined = fast_vector_concatenation(existing_vectors, new_vectors)
    return normalize_vectors(combined) if normalize else combined


def warmup_compiled_functions(dimension: int = 384, n_vectors: int = 100):
    """mlx_optimized.py:257-287: run every operator once (loads the code objects)."""
    logger.info("warming up the device operators (dim %d, n %d)", dimension, n_vectors)
    try:
        rng = np.random.default_rng(0)
        db = rng.standard_normal((max(n_vectors, 1), dimension)).astype(np.float32)
        q1 = rng.standard_normal(dimension).astype(np.float32)
        qb = rng.standard_normal((min(10, max(n_vectors, 1)), dimension)).astype(np.float32)
        k = min(5, max(n_vectors, 1))
        compute_cosine_similarity_single(q1, db)
        compute_cosine_similarity_batch(qb, db)
        fast_top_k_indices(rng.standard_normal(max(n_vectors, 1)).astype(np.float32), k)
        normalize_vectors(db)
        fast_vector_concatenation(db[: n_vectors // 2], db[n_vectors // 2:])
        optimized_batch_similarity_search(qb, db, k)
        logger.info("device operator warmup done")
    except Exception as e:  # the reference logs and continues (:286-287)
        logger.error("device operator warmup failed: %s", e, exc_info=True)
