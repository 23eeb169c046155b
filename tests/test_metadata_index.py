"""Metadata filter postings (service/metadata_index.py) against the reference's scan
semantics: AND of ``meta.get(key) == value`` over every row
(/root/reference/service/optimized_vector_store.py:159-165).  Host only."""
import time

import numpy as np
import pytest

from service.metadata_index import MetadataIndex


def _scan(meta, filt, n):
    return [i for i, m in enumerate(meta[:n]) if all(m.get(k) == v for k, v in filt.items())]


def _rows_of(words, n):
    bits = np.unpackbits(words.view(np.uint8), bitorder="little")[:n]
    return np.nonzero(bits)[0].tolist()


def _meta(rng, n):
    out = []
    for i in range(n):
        m = {"id": f"doc_{i}", "hash": int(rng.integers(0, 7))}
        r = rng.random()
        if r < 0.2:
            m["kind"] = None
        elif r < 0.5:
            m["kind"] = "a" if rng.random() < 0.5 else "b"
        if rng.random() < 0.1:
            m["tags"] = ["x", "y"]          # unhashable value
        if rng.random() < 0.3:
            m["num"] = [1, 1.0, True, 2, 0, False][int(rng.integers(0, 6))]
        out.append(m)
    return out


@pytest.mark.parametrize("filt", [
    {"hash": 3}, {"hash": 3, "kind": "a"}, {"kind": None}, {"kind": "zzz"}, {"missing": None},
    {"num": 1}, {"num": True}, {"num": 1.0}, {"num": 0}, {"tags": ["x", "y"]}, {"id": "doc_17"},
    {"id": "doc_17", "hash": 99}, {"hash": float("nan")}, {},
])
def test_bitmap_equals_reference_scan(filt):
    rng = np.random.default_rng(0)
    meta = _meta(rng, 1000)
    ix = MetadataIndex()
    ix.extend(meta[:400])
    ix.extend(meta[400:])
    for n in (1000, 999, 37):
        words, cnt = ix.bitmap(filt, n)
        want = _scan(meta, filt, n)
        assert _rows_of(words, n) == want and cnt == len(want)
        assert words.size == (n + 31) // 32


@pytest.mark.parametrize("filt", [{"kind": None}, {"tags": ["x", "y"]}, {"missing": None}, {"hash": 3}])
def test_fewer_metadata_rows_than_vectors(filt):
    """Rows past the metadata list count as {}: no IndexError for None or
    unhashable filter values."""
    rng = np.random.default_rng(1)
    meta = _meta(rng, 50)
    ix = MetadataIndex()
    ix.extend(meta)
    n = 80  # 30 vectors without metadata
    words, cnt = ix.bitmap(filt, n)
    want = _scan(meta + [{}] * 30, filt, n)
    assert _rows_of(words, n) == want and cnt == len(want)


def test_cache_invalidated_by_adds():
    ix = MetadataIndex()
    ix.extend([{"a": 1}, {"a": 2}])
    w, c = ix.bitmap({"a": 1}, 2)
    assert c == 1
    ix.extend([{"a": 1}])
    w, c = ix.bitmap({"a": 1}, 3)
    assert c == 2 and _rows_of(w, 3) == [0, 2]


def test_filtered_bitmap_host_cost_at_1m_rows():
    """a filtered query over 1M rows spends < 1 ms on the host
    (cached per filter and row count; the first, uncached build is bounded too)."""
    n = 1_000_000
    ix = MetadataIndex()
    ix.extend([{"hash": i % 10, "id": i} for i in range(n)])
    t0 = time.perf_counter()
    w, c = ix.bitmap({"hash": 7}, n)
    first = time.perf_counter() - t0
    assert c == n // 10
    t0 = time.perf_counter()
    for _ in range(100):
        ix.bitmap({"hash": 7}, n)
    cached = (time.perf_counter() - t0) / 100
    t0 = time.perf_counter()
    w1, c1 = ix.bitmap({"id": 123456}, n)
    selective = time.perf_counter() - t0
    assert c1 == 1 and _rows_of(w1, n) == [123456]
    assert cached < 1e-3, cached
    assert selective < 5e-3, selective
    assert first < 0.05, first
