"""Metadata filter as row bitmaps, maintained at add time.

The reference filters by scanning every metadata dict on every query
(service/optimized_vector_store.py:159-165: ``[i for i, m in enumerate(meta) if
all(m.get(k) == v for k, v in filter.items())]``), O(N) Python per query.  Here
each (key, value) pair keeps a posting list of the rows holding it, appended
when rows are added; a filter is the AND of its pairs' postings, turned into the
uint32 row bitmap the device top-k consumes (include/vdb.h ``row_mask``) and
cached per (filter, row count).  A filtered query costs O(matching rows), not
O(N) dict lookups.

Semantics are exactly ``meta.get(key) == value``:
  * dict lookup finds equal hashable values (1 == 1.0 == True hash alike, as
    ``==`` treats them);
  * ``value is None`` also matches rows that lack the key (``get`` returns None);
  * a filter value that is unhashable or NaN (where dict lookup and ``==``
    disagree) falls back to the reference's scan for that pair.
"""
from __future__ import annotations

import math
import threading
from array import array
from collections import OrderedDict
from typing import Any, Dict, List, Optional, Tuple

import numpy as np


def _hashable(v: Any) -> bool:
    try:
        hash(v)
    except TypeError:
        return False
    return not (isinstance(v, float) and math.isnan(v))


class MetadataIndex:
    """Posting lists key -> value -> rows (int64), plus rows lacking each key."""

    CACHE = 64  # bitmaps kept (LRU), keyed by (filter, row count)

    def __init__(self):
        self._post: Dict[str, Dict[Any, array]] = {}
        self._seen_rows: Dict[str, int] = {}  # key -> rows holding it (for the None / missing case)
        self._n = 0
        self._rows: List[Dict] = []
        self._lock = threading.Lock()
        self._cache: "OrderedDict[Tuple, Tuple[np.ndarray, int]]" = OrderedDict()

    def __len__(self) -> int:
        return self._n

    def clear(self) -> None:
        with self._lock:
            self._post.clear()
            self._seen_rows.clear()
            self._n = 0
            self._rows = []
            self._cache.clear()

    def extend(self, metadata: List[Dict]) -> None:
        """Index rows [n, n + len(metadata)) (called under the store's write lock)."""
        with self._lock:
            r = self._n
            for m in metadata:
                if isinstance(m, dict):
                    for k, v in m.items():
                        if not _hashable(v):
                            continue  # never equal to a hashable filter value; unhashable filters scan
                        by_val = self._post.get(k)
                        if by_val is None:
                            by_val = self._post[k] = {}
                        lst = by_val.get(v)
                        if lst is None:
                            lst = by_val[v] = array("q")
                        lst.append(r)
                r += 1
            self._rows.extend(metadata)
            self._n = r
            self._cache.clear()

    def _pair_rows(self, key: Any, value: Any, n: int) -> np.ndarray:
        """Sorted rows < n with ``meta.get(key) == value``."""
        # rows past the metadata list (the reference allows fewer metadata entries than vectors;
        # persistence pads them with {} on reload) have no keys: get(key) is None
        m_rows = min(n, len(self._rows))
        if not _hashable(value):
            return np.fromiter((i for i in range(m_rows) if isinstance(self._rows[i], dict)
                                and self._rows[i].get(key) == value), dtype=np.int64)
        lst = self._post.get(key, {}).get(value) if _hashable(key) else None
        rows = np.frombuffer(lst, dtype=np.int64) if lst is not None else np.zeros(0, np.int64)
        if value is None:
            # rows without the key also satisfy get(key) == None
            has = np.zeros(n, bool)
            for vals in (self._post.get(key, {}) if _hashable(key) else {}).values():
                a = np.frombuffer(vals, dtype=np.int64)
                has[a[a < n]] = True
            for i in range(m_rows):  # rows holding the key with an unhashable value
                m = self._rows[i]
                if isinstance(m, dict) and key in m and not _hashable(m[key]):
                    has[i] = True
            missing = np.nonzero(~has)[0]
            rows = np.union1d(rows, missing)
        return rows[rows < n]

    def bitmap(self, filt: Dict, n: int) -> Tuple[np.ndarray, int]:
        """(uint32 words of the rows < n matching every pair, match count)."""
        try:
            ck: Optional[Tuple] = (tuple(sorted(filt.items(), key=lambda kv: repr(kv[0]))), n)
            hash(ck)
        except TypeError:
            ck = None
        with self._lock:
            if ck is not None and ck in self._cache:
                self._cache.move_to_end(ck)
                return self._cache[ck]
            rows = None
            for k, v in filt.items():
                pr = self._pair_rows(k, v, n)
                rows = pr if rows is None else np.intersect1d(rows, pr, assume_unique=True)
                if rows.size == 0:
                    break
            if rows is None:
                rows = np.arange(n, dtype=np.int64)
            bits = np.zeros(((n + 31) // 32) * 32, dtype=bool)
            bits[rows] = True
            words = np.packbits(bits, bitorder="little").view("<u4").astype(np.uint32)
            out = (words, int(rows.size))
            if ck is not None:
                self._cache[ck] = out
                if len(self._cache) > self.CACHE:
                    self._cache.popitem(last=False)
            return out
