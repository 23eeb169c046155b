"""Store files: the reference's vectors.npz / metadata.jsonl plus the append log
(mlx-vector-db_amd/service/persistence.py).  Host only."""
import json

import numpy as np

from service import persistence as P


def _rows(rng, n, d=8):
    return rng.random((n, d), dtype=np.float32)


def test_reference_files_load_as_is(tmp_path):
    rng = np.random.default_rng(0)
    V = _rows(rng, 5)
    np.savez(str(tmp_path / "vectors.npz"), vectors=V)  # what the reference writes (:218-223)
    (tmp_path / "metadata.jsonl").write_text("".join(json.dumps({"id": i}) + "\n" for i in range(5)))
    v, m = P.StoreFiles(tmp_path).load()
    np.testing.assert_array_equal(v, V)
    assert [x["id"] for x in m] == list(range(5))


def test_append_then_load_and_compact(tmp_path):
    rng = np.random.default_rng(1)
    f = P.StoreFiles(tmp_path)
    A, B = _rows(rng, 3), _rows(rng, 4)
    f.append(A, [{"i": i} for i in range(3)])
    f.append(B, [{"i": i} for i in range(3, 7)])
    assert not (tmp_path / "vectors.npz").exists()  # O(new rows): no rewrite per add
    v, m = P.StoreFiles(tmp_path).load()
    np.testing.assert_array_equal(v, np.concatenate([A, B]))
    assert [x["i"] for x in m] == list(range(7))
    f.compact(v, m)
    assert not (tmp_path / P.LOG_VECTORS).exists() and not (tmp_path / P.LOG_INFO).exists()
    with np.load(str(tmp_path / "vectors.npz"), allow_pickle=False) as z:  # the reference's format
        np.testing.assert_array_equal(z["vectors"], v)
    assert len((tmp_path / "metadata.jsonl").read_text().splitlines()) == 7
    C = _rows(rng, 2)
    f.append(C, [{"i": 7}, {"i": 8}])
    v2, m2 = P.StoreFiles(tmp_path).load()
    np.testing.assert_array_equal(v2, np.concatenate([A, B, C]))
    assert [x["i"] for x in m2] == list(range(9))


def test_torn_tail_is_dropped_and_appends_line_up(tmp_path):
    rng = np.random.default_rng(2)
    f = P.StoreFiles(tmp_path)
    A = _rows(rng, 4)
    f.append(A, [{"i": i} for i in range(4)])
    raw = (tmp_path / P.LOG_VECTORS).read_bytes()
    (tmp_path / P.LOG_VECTORS).write_bytes(raw[:-5])           # half-written last row
    meta = (tmp_path / P.LOG_META).read_text()
    (tmp_path / P.LOG_META).write_text(meta + '{"i": 4')       # half-written next line
    g = P.StoreFiles(tmp_path)
    v, m = g.load()
    np.testing.assert_array_equal(v, A[:3])
    assert [x["i"] for x in m] == [0, 1, 2]
    B = _rows(rng, 2)
    g.append(B, [{"i": 10}, {"i": 11}])
    v2, m2 = P.StoreFiles(tmp_path).load()
    np.testing.assert_array_equal(v2, np.concatenate([A[:3], B]))
    assert [x["i"] for x in m2] == [0, 1, 2, 10, 11]


def test_log_of_an_interrupted_compaction_is_not_counted_twice(tmp_path):
    rng = np.random.default_rng(3)
    f = P.StoreFiles(tmp_path)
    A = _rows(rng, 3)
    f.append(A, [{}] * 3)
    log = {n: (tmp_path / n).read_bytes() for n in (P.LOG_VECTORS, P.LOG_META, P.LOG_INFO)}
    f.compact(A, [{}] * 3)
    for n, b in log.items():  # crash after the base rename, before the log removal
        (tmp_path / n).write_bytes(b)
    v, m = P.StoreFiles(tmp_path).load()
    np.testing.assert_array_equal(v, A)
    assert len(m) == 3 and not (tmp_path / P.LOG_INFO).exists()


def test_compaction_threshold(tmp_path):
    f = P.StoreFiles(tmp_path)
    f.base_rows = 1_000_000
    f.log_rows = 200_000
    assert not f.needs_compaction()
    f.log_rows = 250_001
    assert f.needs_compaction()
    f.base_rows, f.log_rows = 0, P.MIN_COMPACT_ROWS + 1
    assert f.needs_compaction()


def test_dimension_mismatch_rejected(tmp_path):
    f = P.StoreFiles(tmp_path)
    f.append(np.zeros((2, 4), np.float32), [{}, {}])
    try:
        f.append(np.zeros((1, 5), np.float32), [{}])
    except ValueError:
        pass
    else:
        raise AssertionError("expected ValueError")


def test_compaction_stopped_between_its_two_renames(tmp_path, monkeypatch):
    """a crash after metadata.jsonl is renamed but before vectors.npz is must not
    lose or shift metadata (compact renames metadata first; load keeps base_rows lines)."""
    import os
    rng = np.random.default_rng(4)
    f = P.StoreFiles(tmp_path)
    A, B = _rows(rng, 5), _rows(rng, 3)
    f.compact(A, [{"i": i} for i in range(5)])
    f.append(B, [{"i": i} for i in range(5, 8)])
    v, m = P.StoreFiles(tmp_path).load()
    real_replace = os.replace
    calls = []

    def crash_on_second(src, dst):
        calls.append(dst)
        if len(calls) == 2:
            raise OSError("simulated crash between the two renames")
        return real_replace(src, dst)

    monkeypatch.setattr(P.os, "replace", crash_on_second)
    try:
        P.StoreFiles(tmp_path).compact(v, m)
    except OSError:
        pass
    monkeypatch.setattr(P.os, "replace", real_replace)
    assert str(calls[0]).endswith(P.BASE_META)
    g = P.StoreFiles(tmp_path)
    v2, m2 = g.load()
    np.testing.assert_array_equal(v2, np.concatenate([A, B]))
    assert [x["i"] for x in m2] == list(range(8))
    C = _rows(rng, 1)
    g.append(C, [{"i": 8}])  # later adds keep row r <-> metadata line r
    v3, m3 = P.StoreFiles(tmp_path).load()
    np.testing.assert_array_equal(v3, np.concatenate([A, B, C]))
    assert [x["i"] for x in m3] == list(range(9))
