"""On-disk format of a store: the reference's files plus an append log.

The reference persists a store as ``vectors.npz`` (key ``vectors``, f32 [N, D])
and ``metadata.jsonl`` (one JSON object per row), rewriting BOTH in full on
every ``add_vectors`` (service/optimized_vector_store.py:218-223, called from
:113), i.e. O(N) bytes per add.  SURVEY.md §8f(2): keep those files, replace the
rewrite with an append log and periodic compaction.

Layout of a store directory:

  vectors.npz, metadata.jsonl   the compacted base, exactly the reference's files
                                (a reference process reading the directory sees a
                                consistent, possibly older, snapshot)
  vectors.append.f32            rows added since the last compaction, raw
                                little-endian f32, row-major
  metadata.append.jsonl         their metadata, one JSON object per line
  append.json                   {"dim": D, "base_rows": rows of vectors.npz the
                                log continues}

An add appends to the two log files (O(new rows) bytes); metadata is kept one
line per row (padded with {} / truncated when a caller passes a different
count, which the reference would store as is).  Compaction (when the
log holds more than max(base / 4, 65536) rows, on ``optimize()``, or on demand)
writes a new base through temporary files + atomic renames, then deletes the
log.  Loading reads base + log; a torn last row / line (crash mid-append) is
dropped, a log whose ``base_rows`` no longer matches the base (crash between the
base rename and the log removal) is discarded because the base already holds it.
"""
from __future__ import annotations

import json
import logging
import os
from pathlib import Path
from typing import Dict, List, Tuple

import numpy as np

logger = logging.getLogger("mlx_vector_db.persistence")

BASE_VECTORS = "vectors.npz"
BASE_META = "metadata.jsonl"
LOG_VECTORS = "vectors.append.f32"
LOG_META = "metadata.append.jsonl"
LOG_INFO = "append.json"
MIN_COMPACT_ROWS = 65536


def _write_atomic(path: Path, write) -> None:
    tmp = path.with_name(path.name + ".tmp")
    with open(tmp, "wb") as f:
        write(f)
        f.flush()
        os.fsync(f.fileno())
    os.replace(tmp, path)


class StoreFiles:
    """Base files + append log of one store directory (no device state)."""

    def __init__(self, path: Path):
        self.path = Path(path)
        self.base_rows = 0
        self.log_rows = 0
        self.dim = None

    # ---- read -------------------------------------------------------------------
    def load(self) -> Tuple[np.ndarray, List[Dict]]:
        """(vectors f32 [N, D], metadata) of base + log; empty arrays if nothing is stored."""
        vecs = np.zeros((0, 0), np.float32)
        meta: List[Dict] = []
        bv = self.path / BASE_VECTORS
        if bv.exists():
            with np.load(str(bv), allow_pickle=False) as z:
                vecs = np.asarray(z["vectors"], dtype=np.float32)
            if vecs.ndim != 2:
                raise ValueError(f"{BASE_VECTORS} holds shape {vecs.shape}")
            bm = self.path / BASE_META
            if bm.exists():
                meta = self._read_jsonl(bm)
        self.base_rows = vecs.shape[0]
        self.dim = vecs.shape[1] if vecs.shape[0] else None
        self.log_rows = 0
        info = self._read_info()
        if info is None:
            return vecs, meta
        if info.get("base_rows") == self.base_rows and len(meta) != self.base_rows:
            # a compaction stopped between its two renames (metadata.jsonl is renamed first,
            # see compact): the new metadata already covers the log's rows; or the base was
            # written with a different metadata count.  Row r's metadata is line r either way.
            meta = (meta + [{}] * self.base_rows)[: self.base_rows]
        if info.get("base_rows") != self.base_rows:
            logger.warning("append log continues %s base rows, base holds %d: already compacted, dropped",
                           info.get("base_rows"), self.base_rows)
            self._remove_log()
            return vecs, meta
        D = int(info["dim"])
        raw = np.fromfile(str(self.path / LOG_VECTORS), dtype="<f4") if (self.path / LOG_VECTORS).exists() \
            else np.zeros(0, np.float32)
        n_vec = raw.size // D
        lmeta = self._read_jsonl(self.path / LOG_META) if (self.path / LOG_META).exists() else []
        n = min(n_vec, len(lmeta))
        if n != n_vec or n != len(lmeta) or raw.size != n_vec * D:
            logger.warning("append log torn (%d rows, %d metadata lines): keeping %d", n_vec, len(lmeta), n)
        rows = raw[: n * D].reshape(n, D).astype(np.float32)
        if vecs.shape[0] == 0:
            vecs = rows
        else:
            if D != vecs.shape[1]:
                raise ValueError(f"append log dim {D} != base dim {vecs.shape[1]}")
            vecs = np.concatenate([vecs, rows])
        meta = meta + lmeta[:n]
        self.log_rows = n
        self.dim = D
        if n != n_vec or n != len(lmeta):
            self._rewrite_log(rows, lmeta[:n])  # drop the torn tail so later appends line up
        return vecs, meta

    # ---- write ------------------------------------------------------------------
    def append(self, vectors: np.ndarray, metadata: List[Dict]) -> None:
        """Append rows (and their metadata) to the log: O(new rows) bytes."""
        v = np.ascontiguousarray(vectors, dtype="<f4")
        if v.ndim != 2 or v.shape[0] == 0:
            return
        if self.dim is None:
            self.dim = v.shape[1]
        elif v.shape[1] != self.dim:
            raise ValueError(f"append of {v.shape[1]}-d rows to a {self.dim}-d store")
        self.path.mkdir(parents=True, exist_ok=True)
        if self._read_info() is None:  # a new log: no stale tail of an interrupted removal
            for name in (LOG_VECTORS, LOG_META):
                try:
                    (self.path / name).unlink()
                except FileNotFoundError:
                    pass
            _write_atomic(self.path / LOG_INFO,
                          lambda f: f.write(json.dumps({"dim": self.dim, "base_rows": self.base_rows}).encode()))
        with open(self.path / LOG_VECTORS, "ab") as f:
            f.write(v.tobytes())
        with open(self.path / LOG_META, "a") as f:
            for m in metadata[: v.shape[0]]:
                f.write(json.dumps(m) + "\n")
            for _ in range(v.shape[0] - len(metadata)):  # the reference allows fewer metadata than rows
                f.write("{}\n")
        self.log_rows += v.shape[0]

    def needs_compaction(self) -> bool:
        return self.log_rows > max(self.base_rows // 4, MIN_COMPACT_ROWS)

    def compact(self, vectors: np.ndarray, metadata: List[Dict]) -> None:
        """Write `vectors` / `metadata` (the whole store) as the new base, drop the log.

        Crash safety: both files are written to temporaries first; metadata.jsonl is renamed
        before vectors.npz.  Stopped between the renames, the directory holds the old
        vectors.npz, the new (longer) metadata.jsonl and the log, whose base_rows still
        matches the old base: load() keeps the first base_rows metadata lines and appends the
        log's, which is the same store.  Stopped after the vectors rename, the log's
        base_rows no longer matches and load() drops it (the new base holds its rows)."""
        v = np.ascontiguousarray(vectors, dtype=np.float32)
        self.path.mkdir(parents=True, exist_ok=True)
        _write_atomic(self.path / BASE_META,
                      lambda f: f.write("".join(json.dumps(m) + "\n" for m in metadata).encode()))
        _write_atomic(self.path / BASE_VECTORS, lambda f: np.savez(f, vectors=v))
        self.base_rows = v.shape[0]
        self.dim = v.shape[1] if v.ndim == 2 and v.shape[0] else self.dim
        self._remove_log()
        self.log_rows = 0

    # ---- helpers ----------------------------------------------------------------
    def _read_info(self):
        p = self.path / LOG_INFO
        if not p.exists():
            return None
        try:
            return json.loads(p.read_text())
        except ValueError:
            return None

    @staticmethod
    def _read_jsonl(p: Path) -> List[Dict]:
        out = []
        with open(p, "r") as f:
            for line in f:
                if not line.endswith("\n"):
                    break  # torn last line
                out.append(json.loads(line))
        return out

    def _rewrite_log(self, rows: np.ndarray, meta: List[Dict]) -> None:
        _write_atomic(self.path / LOG_VECTORS, lambda f: f.write(np.ascontiguousarray(rows, "<f4").tobytes()))
        _write_atomic(self.path / LOG_META, lambda f: f.write("".join(json.dumps(m) + "\n" for m in meta).encode()))

    def _remove_log(self) -> None:
        for name in (LOG_INFO, LOG_VECTORS, LOG_META):
            try:
                (self.path / name).unlink()
            except FileNotFoundError:
                pass
