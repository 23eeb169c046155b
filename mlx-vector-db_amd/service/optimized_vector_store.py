"""Drop-in store for the brute-force hot path, backed by the gfx950 vdb core.

Mirrors the reference module ``service/optimized_vector_store.py`` (same class
and function names, argument meaning, return shapes and error behaviour) so
that existing callers — the REST routes (api/routes/vectors.py:57-64, :193,
:229-233, :291), the admin routes, the RAG pipeline and the benchmarks — run
unchanged with ``mlx-vector-db_amd/`` first on ``sys.path``.

What differs underneath:
  * the corpus lives on the GPU as row-major fp32 rows plus an int8 copy of the
    centred rows (two planes in MFMA operand tiles; a split-bf16 copy is built
    only if a search needs one), with norms computed once at ingest (the
    reference re-normalises every row on every query,
    service/optimized_vector_store.py:31-41);
  * search is a fused int8-MFMA candidate pass (I8 for k <= 16, I8X3 above;
    uncertified queries re-passed or sent to the exact scan) + exact fp64 rerank
    and certificate instead of a full argsort (:176-183); ranking is exact with
    ties to the lower row;
  * ``batch_query``, ``optimize`` and ``health_check`` exist (callers expect
    them: api/routes/vectors.py:291, api/routes/admin.py:230, tests/demo.py:134,
    :248, :254) and the functional API of tests/test_vector_store.py:15-18.
"""
from __future__ import annotations

import json
import logging
import os
import collections
import shutil
import threading
import time
from dataclasses import dataclass
from pathlib import Path
from typing import Any, Dict, List, Optional, Tuple, Union

import numpy as np

from . import _vdb
from .metadata_index import MetadataIndex
from .persistence import StoreFiles

logger = logging.getLogger("mlx_vector_db.optimized_store")

# Raised by the reference when no similarity operator exists (jit_compile=False
# or metric="dot_product"): service/optimized_vector_store.py:153-154.
_NO_OPERATOR_MSG = "Keine kompilierte Ähnlichkeitsfunktion verfügbar."


@dataclass
class MLXVectorStoreConfig:
    """service/optimized_vector_store.py:51-56, plus two MI355X knobs."""
    dimension: int = 384
    metric: str = "cosine"
    enable_hnsw: bool = False
    jit_compile: bool = True
    device: int = 0          # GPU ordinal holding this store's corpus
    persist: bool = True     # persist every add (append log + periodic compaction, service/persistence.py)
    # several GPUs of this process: the corpus is row-sharded over them, each query batch is
    # searched on every shard at once and the per-shard top-k lists are gathered and merged
    # on the first device (service/_vdb.py NativeShards); None = the single `device`
    devices: Optional[List[int]] = None
    # concurrent single-vector queries (the REST executor's 4 threads, api/routes/vectors.py:43)
    # join one batched device search instead of one corpus scan each (_QueryCoalescer)
    coalesce: bool = True
    coalesce_inflight: int = 2  # coalesced batches running at once (each on its own stream)
    # a batch leader's wait for the rest of a wave of callers (C2, 4 threads, 2 in flight: 8.6-8.9 K
    # QPS at 300 us against 8.3 K without, profiles/r06_serve/serving.txt; a lone caller never waits)
    coalesce_linger_us: float = 300.0


def _as_matrix(vectors: Any) -> np.ndarray:
    """mx.array(vectors, float32) restated (service/optimized_vector_store.py:215-216)."""
    if hasattr(vectors, "detach") and hasattr(vectors, "cpu"):  # torch tensor
        vectors = vectors.detach().cpu().numpy()
    a = np.asarray(vectors, dtype=np.float32)
    return a


class _RWLock:
    """Many readers (queries) or one writer (add / clear / optimize).  The reference
    takes an RLock in add_vectors and clear but none in query
    (service/optimized_vector_store.py:97,116,199) and is served from a 4-thread
    executor (api/routes/vectors.py:43); here queries still run concurrently with each
    other (ctypes releases the GIL inside the C-ABI), but always see a consistent
    (rows, metadata) snapshot instead of a half-applied add."""

    def __init__(self):
        self._cond = threading.Condition(threading.Lock())
        self._readers = 0
        self._writer = False
        self._waiting_writers = 0

    def acquire_read(self):
        with self._cond:
            while self._writer or self._waiting_writers:
                self._cond.wait()
            self._readers += 1

    def release_read(self):
        with self._cond:
            self._readers -= 1
            if self._readers == 0:
                self._cond.notify_all()

    def acquire_write(self):
        with self._cond:
            self._waiting_writers += 1
            while self._writer or self._readers:
                self._cond.wait()
            self._waiting_writers -= 1
            self._writer = True

    def release_write(self):
        with self._cond:
            self._writer = False
            self._cond.notify_all()


class _Read:
    def __init__(self, lk: _RWLock):
        self.lk = lk

    def __enter__(self):
        self.lk.acquire_read()

    def __exit__(self, *a):
        self.lk.release_read()


class _Write(_Read):
    def __enter__(self):
        self.lk.acquire_write()

    def __exit__(self, *a):
        self.lk.release_write()


class _QueryCoalescer:
    """Continuous batching of concurrent single-vector queries, pipelined.

    The reference serves /vectors/query one vector per request from a 4-thread executor
    (api/routes/vectors.py:43, :226-234): each call is a full scan of the corpus
    (service/optimized_vector_store.py:149-192).  A scan costs about the same for 1 query as
    for 64 (the corpus read dominates), so the queries that arrive while batches
    run wait and then run together as the next batch: no artificial delay when a query arrives
    alone, up to ``max_batch`` queries per scan under load.  Up to ``max_inflight`` batches
    run at once (each on its own workspace stream of the index, so one batch's host work and
    tail kernels overlap another's scan; with one batch in flight the device idled during the
    host side and 4 direct callers beat the coalescer).  A batch holds requests of
    one k class (k <= 16 / <= 200 / larger: the candidate pass a batch runs depends on its
    largest k, so one caller's large k does not move its co-batched callers to a slower pass);
    each caller gets its own row and k (the exact order makes every caller's top-k the prefix
    of the batch's).  Callers hold the store's read lock while they wait, so every query of a
    batch sees the same rows."""

    def __init__(self, run, max_batch: int = 64, max_inflight: int = 2, linger_us: float = 0.0):
        self._run = run            # run(Q [B, D], k) -> [(indices, scores, metadata)] * B
        self._max = max_batch
        self._inflight = max(1, int(max_inflight))
        # adaptive linger: callers come back in waves (each waits for its own result), so a leader
        # that finds fewer pending queries than the recent batches held waits up to linger_us for
        # the rest of the wave; a lone caller (recent batches of 1) never waits
        self._linger = max(0.0, float(linger_us)) * 1e-6
        self._recent = collections.deque(maxlen=8)
        self._cv = threading.Condition(threading.Lock())
        self._pending: List[list] = []
        self._running = 0
        self.batches = 0
        self.queries = 0

    @staticmethod
    def _kclass(k: int) -> int:
        return 0 if k <= 16 else 1 if k <= 200 else 2

    def query(self, q: np.ndarray, k: int):
        req = [q, int(k), None, None]  # query, k, result, error
        self._cv.acquire()
        try:
            self._pending.append(req)
            # wait for a result; whenever fewer than max_inflight batches run, lead the next one:
            # the oldest pending request's k class, FIFO (a leader may serve others before its own)
            lingered = False
            while req[2] is None and req[3] is None:
                if self._running >= self._inflight or not self._pending:
                    self._cv.wait()
                    continue
                expect = min(self._max, max(self._recent)) if self._recent else 1
                if self._linger > 0.0 and not lingered and len(self._pending) < expect:
                    lingered = True
                    deadline = time.perf_counter() + self._linger
                    while len(self._pending) < expect and req[2] is None and req[3] is None:
                        rem = deadline - time.perf_counter()
                        if rem <= 0.0:
                            break
                        self._cv.wait(rem)
                    continue  # (another leader may have taken the requests meanwhile)
                kc = self._kclass(self._pending[0][1])
                batch, rest = [], []
                for r in self._pending:
                    (batch if len(batch) < self._max and self._kclass(r[1]) == kc else rest).append(r)
                self._pending = rest
                self._running += 1
                self._cv.release()
                try:
                    kmax = max(r[1] for r in batch)
                    res = self._run(np.stack([r[0] for r in batch]), kmax)
                    for r, (ix, sc, md) in zip(batch, res):
                        r[2] = (ix[:r[1]], sc[:r[1]], md[:r[1]])
                except BaseException as e:  # every caller of the batch sees the failure
                    for r in batch:
                        r[3] = e
                finally:
                    self._cv.acquire()
                    self._running -= 1
                    self.batches += 1
                    self.queries += len(batch)
                    self._recent.append(len(batch))
                    self._cv.notify_all()
        finally:
            self._cv.release()
        if req[3] is not None:
            raise req[3]
        return req[2]


class MLXVectorStore:
    """service/optimized_vector_store.py:59-242, MI355X-native."""

    def __init__(self, store_path: str, config: Optional[MLXVectorStoreConfig] = None):
        self.store_path = Path(store_path).expanduser()
        self.config = config or MLXVectorStoreConfig()
        self._lock = threading.RLock()  # serialises writers (the reference's lock, :97, :199)
        self._rw = _RWLock()            # queries (shared) vs adds / clear (exclusive)
        self.store_path.mkdir(parents=True, exist_ok=True)
        self._is_dirty = False
        self._compiled_similarity_fn = None
        self._index = None  # _vdb.NativeIndex, or _vdb.NativeShards over config.devices
        self._dim: Optional[int] = None
        self._metadata: List[Dict] = []
        self._meta_index = MetadataIndex()
        self._vector_count = 0
        self._hnsw_index = None
        self._files = StoreFiles(self.store_path)
        self._coalescer = _QueryCoalescer(lambda Q, k: self._brute_force_search(Q, k, None),
                                          max_inflight=self.config.coalesce_inflight,
                                          linger_us=self.config.coalesce_linger_us)
        if self.config.enable_hnsw:  # service/optimized_vector_store.py:72-78
            from performance.hnsw_index import ProductionHNSWIndex
            self._hnsw_index = ProductionHNSWIndex(self.config.dimension, self.store_path, self.config.metric,
                                                   device=self._devices()[0])
        self._initialize_store()
        if self.config.jit_compile:
            self._compile_critical_functions()
        logger.info("vdb store initialised: %s | HNSW: %s", self.store_path, self.config.enable_hnsw)

    # ---- state -----------------------------------------------------------------
    def _devices(self) -> List[int]:
        return list(self.config.devices) if self.config.devices else [self.config.device]

    def _create_empty_store(self):
        if self._index is not None:
            self._index.clear()
        self._metadata = []
        self._meta_index.clear()
        self._vector_count = 0
        self._is_dirty = False

    def _initialize_store(self):
        self._load_store()

    def _compile_critical_functions(self):
        # the operator slot: which device kernel family serves brute force (:211-213)
        if self.config.metric in _vdb.METRIC_IDS:
            self._compiled_similarity_fn = self.config.metric

    def _ensure_index(self, dim: int):
        if self._index is None:
            metric = self.config.metric if self.config.metric in _vdb.METRIC_IDS else "cosine"
            devs = self._devices()
            if len(devs) > 1:
                # row shards over several GPUs of this process (service/_vdb.py NativeShards)
                self._index = _vdb.NativeShards(dim, metric, devs)
            else:
                self._index = _vdb.NativeIndex(dim, metric, devs[0])
            self._dim = dim
        elif dim != self._dim:
            raise ValueError(f"Dimension mismatch: store holds {self._dim}-d vectors, got {dim}-d")
        return self._index

    @property
    def _vectors(self) -> Optional[np.ndarray]:
        """The corpus as [N, D] float32 (copied back from the GPU), or None if empty."""
        if self._index is None or self._vector_count == 0:
            return None
        return self._index.get_vectors()

    # ---- ingest ------------------------------------------------------------------
    def add_vectors(self, vectors: Union[np.ndarray, Any], metadata: List[Dict]):
        """service/optimized_vector_store.py:96-114."""
        with self._lock, _Write(self._rw):
            v = _as_matrix(vectors)
            if v.ndim == 1:
                v = v[None, :]
            if v.ndim != 2:
                raise ValueError(f"vectors must be 2-D (n, dim), got shape {v.shape}")
            n0 = self._vector_count
            if v.shape[0] > 0:
                self._ensure_index(v.shape[1]).add(v)
            self._metadata.extend(metadata)
            # the filter postings index exactly the rows' metadata (row r <-> metadata[r])
            self._meta_index.extend(self._metadata[len(self._meta_index):])
            self._vector_count = self._index.count() if self._index is not None else 0
            self._is_dirty = True
            if self.config.persist and v.shape[0] > 0:
                # O(new rows) append instead of the reference's full rewrite per add (:113, :218-223)
                self._files.append(v, metadata)
                if self._files.needs_compaction():
                    self._save_store(force=True)
                else:
                    self._is_dirty = False
            if self.config.enable_hnsw and self._hnsw_index is not None and self._index is not None:
                # the reference rebuilds the graph from scratch on every add (:110-112); the graph
                # path inserts the new rows into the existing graph instead (performance/hnsw_index.py)
                self._hnsw_index.add_rows(self._index, n0)
            return {"vectors_added": len(metadata), "total_vectors": self._vector_count}

    # ---- query ---------------------------------------------------------------------
    def query(self, query_vector: Union[np.ndarray, Any], k: int = 10,
              filter_metadata: Optional[Dict] = None, use_hnsw: bool = True) -> Tuple:
        """service/optimized_vector_store.py:116-145 -> (indices, scores, metadata)."""
        with _Read(self._rw):
            if self._vector_count == 0:
                return [], [], []
            q = _as_matrix(query_vector)
            if q.ndim == 2 and q.shape[0] == 1:
                q = q[0]
            if q.ndim != 1:
                raise ValueError(f"query takes one vector of shape (dim,) or (1, dim), got {q.shape}; "
                                 "use batch_query for several")
            h = self._hnsw_index
            if use_hnsw and self.config.enable_hnsw and h is not None and h.is_loaded:
                # service/optimized_vector_store.py:120-143: hnswlib distances, k*10 candidates
                # when filtering, brute force on any failure
                try:
                    candidate_k = k * 10 if filter_metadata else k
                    indices, distances = h.search(q[None, :], k=candidate_k)
                    indices, distances = indices[0], distances[0]
                    if not filter_metadata:
                        return ([int(i) for i in indices], distances.tolist(),
                                [self._metadata[int(i)] for i in indices])
                    hits = []
                    for i, idx in enumerate(indices):
                        if idx < len(self._metadata):
                            meta = self._metadata[int(idx)]
                            if all(meta.get(key) == value for key, value in filter_metadata.items()):
                                hits.append((int(idx), float(distances[i]), meta))
                        if len(hits) == k:
                            break
                    if not hits:
                        return [], [], []
                    fi, fd, fm = zip(*hits)
                    return list(fi), list(fd), list(fm)
                except Exception as e:
                    logger.warning("HNSW-Suche fehlgeschlagen, falle auf Brute-Force zurück: %s", e)
            # k above the device limit is not coalesced: its error is the caller's alone
            if (self.config.coalesce and not filter_metadata and self._compiled_similarity_fn
                    and 0 < int(k) <= 1024):
                if q.shape[0] != self._dim:
                    raise ValueError(f"Dimension mismatch: query has {q.shape[0]} dims, store holds {self._dim}")
                return self._coalescer.query(q, k)
            return self._brute_force_search(q[None, :], k, filter_metadata)[0]

    def batch_query(self, query_vectors: Union[np.ndarray, Any], k: int = 10,
                    filter_metadata: Optional[Dict] = None) -> List[Tuple]:
        """The batched path (performance/mlx_optimized.py:217-248) behind the store API that
        api/routes/vectors.py:291 and tests/demo.py:134-137 call: one (indices, distances,
        metadata) tuple per query, same rows and order as ``query`` for that vector.

        The second element is a DISTANCE, because that is how its only caller reads it:
        /vectors/batch_query unpacks ``indices, distances, metadata_list`` and scores cosine
        as ``max(0, 1.0 - dist)`` and euclidean as ``1 / (1 + dist)``
        (api/routes/vectors.py:300-306).  So cosine returns ``1 - cos`` and euclidean the
        sqrt-L2 distance (which is what ``query`` already returns for euclidean)."""
        q = _as_matrix(query_vectors)
        if q.ndim == 1:
            q = q[None, :]
        if q.ndim != 2:
            raise ValueError(f"query_vectors must be 2-D (B, dim), got {q.shape}")
        with _Read(self._rw):
            if self._vector_count == 0 or q.shape[0] == 0:
                return [([], [], []) for _ in range(q.shape[0])]
            res = self._brute_force_search(q, k, filter_metadata)
        if self.config.metric == "cosine":
            res = [(i, [1.0 - s for s in sc], m) for i, sc, m in res]
        return res

    def _brute_force_search(self, Q: np.ndarray, k: int, filter_metadata: Optional[Dict] = None):
        """service/optimized_vector_store.py:149-192 for a [B, D] block of queries
        (called with the read lock held)."""
        if not self._compiled_similarity_fn:
            raise RuntimeError(_NO_OPERATOR_MSG)
        B = Q.shape[0]
        empty = [([], [], []) for _ in range(B)]
        if Q.shape[1] != self._dim:
            raise ValueError(f"Dimension mismatch: query has {Q.shape[1]} dims, store holds {self._dim}")
        k = int(k)
        if k <= 0:
            return empty
        n = self._vector_count
        mask = None
        eligible = n
        if filter_metadata:
            # posting lists maintained at add time, not the reference's O(N) scan (:159-165)
            mask, eligible = self._meta_index.bitmap(filter_metadata, n)
            if eligible == 0:
                return empty
        kk = min(k, eligible)
        if kk > 1024:
            raise ValueError(f"k={k} exceeds the device top-k limit of 1024")
        scores, idx = self._index.search(Q, kk, row_mask=mask)
        out = []
        meta = self._metadata
        for b in range(B):
            valid = idx[b] >= 0
            ib = idx[b][valid].tolist()
            sb = scores[b][valid].astype(np.float64).tolist()
            out.append((ib, sb, [meta[i] if i < len(meta) else {} for i in ib]))
        return out

    # ---- misc API ----------------------------------------------------------------------
    def _warmup_kernels(self):
        """service/optimized_vector_store.py:194-196 (a no-op there); here: one tiny search."""
        if self._vector_count and self._compiled_similarity_fn:
            self._index.search(np.zeros((1, self._dim), np.float32) + 1.0, 1)

    def clear(self):
        """service/optimized_vector_store.py:198-209."""
        with self._lock, _Write(self._rw):
            try:
                if self.store_path.exists():
                    shutil.rmtree(self.store_path)
                self.store_path.mkdir(parents=True, exist_ok=True)
                self._files = StoreFiles(self.store_path)
                self._create_empty_store()
                if self.config.enable_hnsw:  # :205-206
                    from performance.hnsw_index import ProductionHNSWIndex
                    self._hnsw_index = ProductionHNSWIndex(self.config.dimension, self.store_path,
                                                           self.config.metric, device=self._devices()[0])
            except Exception as e:  # the reference logs and swallows (:208-209)
                logger.error("clearing store %s failed: %s", self.store_path, e)

    def optimize(self) -> Dict[str, Any]:
        """Callers: api/routes/admin.py:230, api/routes/performance.py:188, tests/demo.py:248.
        Flushes persistence and pre-sizes the device corpus to a 256-row multiple."""
        t0 = time.time()
        with self._lock, _Write(self._rw):
            if self._index is not None:
                self._index.reserve(self._vector_count)
            self._is_dirty = True
            self._save_store(force=True)
        with _Read(self._rw):
            self._warmup_kernels()
        return {"optimized": True, "vector_count": self._vector_count,
                "optimization_time_ms": (time.time() - t0) * 1000.0}

    def health_check(self) -> Dict[str, Any]:
        """Caller: tests/demo.py:254 (reads 'healthy' and 'issues')."""
        issues = []
        if len(self._metadata) != self._vector_count:
            issues.append(f"metadata rows ({len(self._metadata)}) != vectors ({self._vector_count})")
        if self._vector_count and self._index is None:
            issues.append("device index missing")
        if self._index is not None and self._index.count() != self._vector_count:
            issues.append("device row count out of sync")
        if not self._compiled_similarity_fn:
            issues.append(_NO_OPERATOR_MSG)
        return {"healthy": not issues, "issues": issues, "vector_count": self._vector_count,
                "metric": self.config.metric, "devices": self._devices()}

    def get_stats(self):
        """service/optimized_vector_store.py:241-242 (+ memory_usage_mb, read by
        api/routes/monitoring.py:153 and tests/demo.py:146)."""
        mem = 0.0
        if self._index is not None:
            mem = self._index.stat("device_bytes") / (1024.0 * 1024.0)
        return {"vector_count": self._vector_count, "dimension": self.config.dimension,
                "metric": self.config.metric,
                "index_type": "hnsw" if self.config.enable_hnsw else "flat",
                "memory_usage_mb": mem}

    # ---- persistence: vectors.npz + metadata.jsonl (service/optimized_vector_store.py:218-239)
    # plus an append log between compactions (service/persistence.py)
    def _save_store(self, force: bool = False):
        """Compaction: the whole store as the reference's two files (log dropped)."""
        if not (self.config.persist or force):
            return
        if self._vector_count == 0 or not (self._is_dirty or self._files.log_rows):
            return
        self._files.compact(self._index.get_vectors(), self._metadata[: self._vector_count])
        self._is_dirty = False

    def _load_store(self):
        try:
            vecs, meta = self._files.load()
            if vecs.shape[0] == 0:
                self._create_empty_store()
                return
            self._ensure_index(vecs.shape[1]).add(vecs)
            self._metadata = meta
            self._meta_index.clear()
            self._meta_index.extend(meta)
            self._vector_count = self._index.count()
            if self._hnsw_index is not None:
                if not self._hnsw_index.attach(self._index):
                    self._hnsw_index.build(None, native_index=self._index)
        except Exception as e:  # reference: log and start empty (:237-239)
            logger.error("loading store %s failed, starting empty: %s", self.store_path, e)
            self._create_empty_store()


def create_optimized_vector_store(store_path: str, dimension: int = 384, jit_compile: bool = True,
                                  enable_hnsw: bool = False, **kwargs) -> MLXVectorStore:
    """service/optimized_vector_store.py:244-246."""
    config = MLXVectorStoreConfig(dimension=dimension, jit_compile=jit_compile, enable_hnsw=enable_hnsw, **kwargs)
    return MLXVectorStore(store_path, config)


# ---- functional API (tests/test_vector_store.py:15-43 imports these) -----------------------
_STORES: Dict[str, MLXVectorStore] = {}
_STORES_LOCK = threading.Lock()


def _base_dir() -> Path:
    # the REST manager's layout, api/routes/vectors.py:57
    return Path(os.environ.get("VECTOR_STORE_BASE", "~/.team_mind_data/vector_stores")).expanduser()


def _store_path(user_id: str, model_id: str) -> Path:
    return _base_dir() / user_id / model_id


def _key(user_id: str, model_id: str) -> str:
    return f"{user_id}_{model_id}"  # api/routes/vectors.py:45-46


def store_exists(user_id: str, model_id: str) -> bool:
    return _key(user_id, model_id) in _STORES or _store_path(user_id, model_id).exists()


def create_store(user_id: str, model_id: str, dimension: int = 384, metric: str = "cosine",
                 **kwargs) -> MLXVectorStore:
    with _STORES_LOCK:
        key = _key(user_id, model_id)
        if key not in _STORES:
            cfg = MLXVectorStoreConfig(dimension=dimension, metric=metric, **kwargs)
            _STORES[key] = MLXVectorStore(str(_store_path(user_id, model_id)), cfg)
        return _STORES[key]


def _get_store(user_id: str, model_id: str) -> MLXVectorStore:
    key = _key(user_id, model_id)
    if key not in _STORES:
        return create_store(user_id, model_id)  # lazy creation, api/routes/vectors.py:53-69
    return _STORES[key]


def add_vectors(user_id: str, model_id: str, vectors, metadata: List[Dict]) -> Dict[str, int]:
    return _get_store(user_id, model_id).add_vectors(vectors, metadata)


def query_vectors(user_id: str, model_id: str, query_vector, k: int = 10,
                  filter_metadata: Optional[Dict] = None) -> List[Dict[str, Any]]:
    """-> [{"index", "score", "metadata"}] (service/models.py SearchResult shape)."""
    idx, scores, meta = _get_store(user_id, model_id).query(query_vector, k=k, filter_metadata=filter_metadata)
    return [{"index": i, "score": s, "metadata": m} for i, s, m in zip(idx, scores, meta)]


def count_vectors(user_id: str, model_id: str) -> Dict[str, int]:
    st = _get_store(user_id, model_id)
    return {"vectors": st._vector_count, "metadata": len(st._metadata)}


def delete_store(user_id: str, model_id: str) -> bool:
    with _STORES_LOCK:
        st = _STORES.pop(_key(user_id, model_id), None)
    path = _store_path(user_id, model_id)
    if st is not None and st._index is not None:
        st._index.close()
    if path.exists():
        shutil.rmtree(path)
        return True
    return st is not None
