"""Graph index with the interface of the reference's ProductionHNSWIndex
(performance/hnsw_index.py:23-129), served by the gfx950 graph path
(include/vdb.h vdb_graph_*, mlx-vector-db_amd/csrc/vdb_graph.hip).

What is the same: constructor arguments, ``build(data, M, ef_construction,
num_threads)``, ``search(query_data, k, ef_search) -> (labels, distances)`` with
hnswlib's conventions (labels uint64 [n, k]; distances fp32: cosine -> 1 - cos,
l2 -> squared L2, hnsw_index.py:35,101), ``save_index`` / ``_load_index``,
``is_loaded``, ``RuntimeError`` when searched before it is built (:91-92).

What differs: the graph is one level of out-degree 2M (hnswlib's
level-0 degree) built on the GPU from the exact kNN of every row — hnswlib's
neighbour heuristic selects <= M out-edges, then <= 2M of out- and in-edges —
instead of hnswlib's one-at-a-time insertion, so ``ef_construction`` and
``num_threads`` have nothing to control; rows added later are inserted as a batch
(``add_rows``, vdb_graph_add) instead of rebuilding; the upper levels' job (a good
start) is done by scoring spread entry rows -- N_ENTRIES of them, each of the TEAMS
workgroups that search a query scoring its own spread slice of <= 256 (the kNN graph of
clustered rows has no edges between clusters: the entries must reach the query's).
The file is ``hnsw_graph.npz`` (neighbour array + entry rows); hnswlib's
``hnsw_index.bin`` format is not produced (its compatibility is unpinned,
SURVEY.md §8f).  The graph refers to the corpus rows of a device index: ``build``
creates one from ``data`` unless ``native_index`` (e.g. the store's) is given,
and a saved graph is re-attached with ``attach(native_index)``.
"""
from __future__ import annotations

import logging
import time
from pathlib import Path
from typing import Optional, Tuple

import numpy as np

from service import _vdb

logger = logging.getLogger("mlx_hnsw_lib")

GRAPH_FILE = "hnsw_graph.npz"
# entry rows (capped at the row count): 256 teams x 256 per team's slice
N_ENTRIES = 65536
# workgroups per query (include/vdb.h vdb_graph_set_param "teams"): at batch 1 the query
# gets every CU, each searching from its own slice of the entry rows.  5M x 384, ef 128
# (profiles/r05_c5): clustered rows recall@10 0.997 at p50 0.56 ms (the exact path 0.66 ms;
# 256 entries: 0.03); BASELINE's uniform rows 0.56 at 0.76 ms (64 teams 0.39 at 0.63 ms; the
# exact path 0.41 ms: on such data it is the right tool)
TEAMS = 256


class ProductionHNSWIndex:
    def __init__(self, dimension: int, store_path: Path, metric: str = "cosine", max_elements: int = 10000,
                 device: int = 0):
        self.dimension = int(dimension)
        self.store_path = Path(store_path)
        self.index_file_path = self.store_path / GRAPH_FILE
        # hnswlib naming: 'l2' for euclidean (hnsw_index.py:35)
        self.metric = "l2" if metric == "euclidean" else metric
        self.device = device
        self.index: Optional[_vdb.NativeGraph] = None
        self.is_loaded = False
        self.max_elements = max_elements
        self._native: Optional[_vdb.NativeIndex] = None
        self._pending = None  # arrays of a saved graph waiting for attach()
        self._load_index()

    @property
    def _vdb_metric(self) -> str:
        return "euclidean" if self.metric == "l2" else self.metric

    def build(self, data: Optional[np.ndarray], M: int = 16, ef_construction: int = 200, num_threads: int = -1,
              native_index: Optional[_vdb.NativeIndex] = None):
        """hnsw_index.py:44-77.  `data` [n, dim] fp32, or None with `native_index`."""
        if native_index is None:
            data = np.asarray(data, dtype=np.float32)
            if data.ndim != 2 or data.shape[0] == 0:
                logger.warning("Keine Vektoren zum Indexieren vorhanden.")
                return
            native_index = _vdb.NativeIndex(data.shape[1], self._vdb_metric, self.device)
            native_index.add(data)
        n = native_index.count()
        if n == 0:
            logger.warning("Keine Vektoren zum Indexieren vorhanden.")
            return
        t0 = time.time()
        if self.index is not None:
            self.index.close()
        degree = 2 * int(M)
        self.index = _vdb.NativeGraph.build(native_index, degree=degree, knn=degree, n_entries=N_ENTRIES)
        self.index.set_param("teams", TEAMS)
        self._native = native_index
        self.max_elements = max(self.max_elements, n)
        self.is_loaded = True
        logger.info("graph index over %d vectors built in %.2f s (degree %d)", n, time.time() - t0, degree)
        self.save_index()

    def add_rows(self, native_index: _vdb.NativeIndex, first_new_row: int):
        """The store appended rows [first_new_row, count) to `native_index`: insert them into
        the graph (vdb_graph_add: kNN of the new rows, hnswlib's heuristic, re-selection of
        the lists they link into) instead of the reference's rebuild from scratch on every
        add (service/optimized_vector_store.py:110-112).  Builds when there is no graph on
        these rows yet."""
        if not isinstance(native_index, _vdb.NativeIndex):
            logger.warning("graph path needs a single-device index; queries use brute force")
            return
        if self.index is None or self._native is not native_index or self.index.info()[0] != first_new_row:
            self.build(None, native_index=native_index)
            return
        t0 = time.time()
        self.index.add()
        self.max_elements = max(self.max_elements, native_index.count())
        logger.info("graph index: %d rows inserted in %.2f s", native_index.count() - first_new_row, time.time() - t0)
        self.save_index()

    def search(self, query_data: np.ndarray, k: int, ef_search: int = 100) -> Tuple[np.ndarray, np.ndarray]:
        """hnsw_index.py:79-103: (labels uint64 [n, k], distances fp32 [n, k])."""
        if not self.is_loaded or self.index is None:
            raise RuntimeError("HNSW-Index ist nicht gebaut oder geladen.")
        if self._native.count() == 0:
            return np.array([]), np.array([])
        q = np.asarray(query_data, dtype=np.float32)
        if q.ndim == 1:
            q = q[None, :]
        k = int(k)
        if k > self._native.count():
            # hnswlib raises when it cannot return k results
            raise RuntimeError("Cannot return the results in a contigious 2D array. Probably ef or M is too small")
        if k > _vdb.GRAPH_EF_MAX:
            raise RuntimeError(f"k={k} exceeds the graph path's beam limit {_vdb.GRAPH_EF_MAX}")
        # hnswlib searches with max(ef, k); the device beam holds at most GRAPH_EF_MAX
        ef = min(max(int(ef_search), k), _vdb.GRAPH_EF_MAX)
        labels, dist = self.index.search(q, k, ef)
        if (labels < 0).any():
            # hnswlib raises when it cannot return k results (e.g. k > count)
            raise RuntimeError("Cannot return the results in a contigious 2D array. Probably ef or M is too small")
        return labels.astype(np.uint64), dist

    def save_index(self):
        if self.index is None:
            return
        nbr, ent = self.index.to_arrays()
        self.store_path.mkdir(parents=True, exist_ok=True)
        np.savez(str(self.index_file_path), neighbors=nbr, entries=ent, metric=np.array(self.metric),
                 dimension=np.int64(self.dimension))
        logger.info("graph index saved: %s", self.index_file_path)

    def _load_index(self):
        if not self.index_file_path.exists():
            logger.info("Keine Index-Datei unter %s gefunden.", self.index_file_path)
            return
        try:
            with np.load(str(self.index_file_path), allow_pickle=False) as z:
                self._pending = (np.asarray(z["neighbors"], np.int32), np.asarray(z["entries"], np.int32))
        except Exception as e:  # reference: log, stay unloaded (:126-129)
            logger.error("Fehler beim Laden des HNSW-Index: %s. Index wird neu erstellt.", e)
            self._pending = None

    def attach(self, native_index: _vdb.NativeIndex) -> bool:
        """Re-attach a saved graph to the device rows it was built on."""
        if self._pending is None:
            return False
        nbr, ent = self._pending
        if nbr.shape[0] != native_index.count():
            logger.warning("saved graph has %d rows, corpus %d: rebuild needed", nbr.shape[0], native_index.count())
            return False
        self.index = _vdb.NativeGraph.from_arrays(native_index, nbr, ent)
        self.index.set_param("teams", TEAMS)
        self._native = native_index
        self.is_loaded = True
        self._pending = None
        return True
