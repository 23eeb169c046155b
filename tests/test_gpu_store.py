"""The drop-in boundary on the GPU: the store mirror (service/optimized_vector_store.py)
against the oracle's restatement of the reference store (oracle/ref_cpu.py
reference_store_search = service/optimized_vector_store.py:116-192) and the
reference's own known-answer tests: P1 self-query (tests/test_integration.py:81-136),
P2/P3 filters (test_integration.py:139-160, tests/demo.py:217-243), P4 counts and P5
result length (tests/test_vector_store.py:20-43), P6 batch shape (demo.py:130-139),
P7 empty store (optimized_vector_store.py:117)."""
import numpy as np
import pytest

from oracle import ref_cpu

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def store_mod():
    from service import _vdb, optimized_vector_store
    assert _vdb.device_count() >= 1, "no GPU visible"
    return optimized_vector_store


def _mk(store_mod, path, dim, metric="cosine", **kw):
    return store_mod.MLXVectorStore(str(path), store_mod.MLXVectorStoreConfig(dimension=dim, metric=metric, **kw))


@pytest.mark.parametrize("metric", ["cosine", "euclidean"])
def test_query_matches_reference_store(store_mod, tmp_path, metric):
    rng = np.random.default_rng(41)
    V = rng.random((3000, 48), dtype=np.float32)
    meta = [{"id": f"doc_{i}", "hash": i % 10, "kind": "a" if i % 3 else "b"} for i in range(3000)]
    st = _mk(store_mod, tmp_path / "s", 48, metric)
    r = st.add_vectors(V, meta)
    assert r == {"vectors_added": 3000, "total_vectors": 3000}
    for q, filt in ((rng.random(48, dtype=np.float32), None), (V[5], None),
                    (rng.random(48, dtype=np.float32), {"hash": 7}),
                    (rng.random(48, dtype=np.float32), {"hash": 3, "kind": "b"})):
        gi, gs, gm = st.query(q, k=10, filter_metadata=filt)
        ri, rs, rm = ref_cpu.reference_store_search(q, V, 10, metric, meta, filt)
        assert gi == ri and gm == rm
        np.testing.assert_allclose(gs, rs, rtol=1e-4, atol=1e-5)
        if filt:
            assert all(all(m[a] == b for a, b in filt.items()) for m in gm)  # P2 / P3


def test_self_query_count_length_batch_empty(store_mod, tmp_path):
    rng = np.random.default_rng(42)
    st = _mk(store_mod, tmp_path / "e", 384)
    assert st.query(rng.random(384, dtype=np.float32), k=5) == ([], [], [])           # P7
    assert st.batch_query(rng.random((3, 384), dtype=np.float32), k=5) == [([], [], [])] * 3
    V = rng.random((500, 384), dtype=np.float32)
    st.add_vectors(V, [{"id": i} for i in range(500)])
    i, s, m = st.query(V[123], k=5)
    assert i[0] == 123 and s[0] > 0.999 and m[0]["id"] == 123                         # P1
    assert len(i) == 5                                                                 # P5
    res = st.batch_query(V[:7], k=4)                                                   # P6
    assert len(res) == 7 and all(len(r[0]) == 4 for r in res)
    assert [r[0][0] for r in res] == list(range(7))
    assert st.query(V[0], k=1000)[0][:1] == [0] and len(st.query(V[0], k=1000)[0]) == 500  # min(k, N)
    assert st.query(V[0], k=0) == ([], [], [])
    assert st.query(V[0], k=3, filter_metadata={"id": -1}) == ([], [], [])
    with pytest.raises(ValueError):
        st.add_vectors(rng.random((2, 10), dtype=np.float32), [{}, {}])  # dimension is enforced
    stats = st.get_stats()
    assert stats["vector_count"] == 500 and stats["memory_usage_mb"] > 0
    assert st.health_check()["healthy"]


def test_no_operator_raises_like_reference(store_mod, tmp_path):
    st = _mk(store_mod, tmp_path / "d", 16, "dot_product")
    st.add_vectors(np.ones((4, 16), np.float32), [{}] * 4)
    with pytest.raises(RuntimeError, match="Keine kompilierte"):
        st.query(np.ones(16, np.float32), k=2)


def test_persistence_append_log_and_compaction(store_mod, tmp_path):
    from service import persistence as P
    rng = np.random.default_rng(43)
    path = tmp_path / "p"
    st = _mk(store_mod, path, 32)
    A, B = rng.random((100, 32), dtype=np.float32), rng.random((50, 32), dtype=np.float32)
    st.add_vectors(A, [{"i": i} for i in range(100)])
    st.add_vectors(B, [{"i": i} for i in range(100, 150)])
    assert (path / P.LOG_VECTORS).exists() and not (path / "vectors.npz").exists()  # no rewrite per add
    q = rng.random(32, dtype=np.float32)
    want = st.query(q, k=8)
    st2 = _mk(store_mod, path, 32)                       # reopen: base + log
    assert st2._vector_count == 150 and st2.query(q, k=8) == want
    st2.optimize()                                       # compaction -> the reference's two files
    assert (path / "vectors.npz").exists() and not (path / P.LOG_VECTORS).exists()
    with np.load(str(path / "vectors.npz"), allow_pickle=False) as z:
        np.testing.assert_array_equal(z["vectors"], np.concatenate([A, B]))
    st3 = _mk(store_mod, path, 32)
    assert st3.query(q, k=8) == want
    st3.clear()
    assert st3.query(q, k=8) == ([], [], []) and not (path / "vectors.npz").exists()


def test_functional_api_lifecycle(store_mod, tmp_path, monkeypatch):
    """tests/test_vector_store.py:20-43 of the reference, verbatim in behaviour."""
    monkeypatch.setenv("VECTOR_STORE_BASE", str(tmp_path / "base"))
    sm = store_mod
    if sm.store_exists("test_user", "test_model"):
        sm.delete_store("test_user", "test_model")
    sm.create_store("test_user", "test_model")
    assert sm.store_exists("test_user", "test_model")
    vecs = np.random.rand(5, 384).astype(np.float32)
    sm.add_vectors("test_user", "test_model", vecs, [{"id": f"v{i}", "source": "test"} for i in range(5)])
    stats = sm.count_vectors("test_user", "test_model")
    assert stats["vectors"] == 5 and stats["metadata"] == 5
    assert len(sm.query_vectors("test_user", "test_model", vecs[0], k=3)) == 3
    sm.delete_store("test_user", "test_model")
    assert not sm.store_exists("test_user", "test_model")


@pytest.mark.parametrize("metric", ["cosine", "euclidean"])
def test_multi_device_shards_equal_one_index(store_mod, metric):
    """vdb_shards_* (include/vdb.h): rows dealt to shards in pieces over several adds, two
    and three shards on the one GPU of the box (the code path of distinct devices, with
    device-local peer copies); results, fp64 keys and ties bit-identical to one index."""
    from service import _vdb
    rng = np.random.default_rng(44)
    V = rng.random((30011, 72), dtype=np.float32)
    V[29000:29010] = V[17]          # ties straddling pieces / shards
    V[5:8] = V[20000]
    Q = np.concatenate([V[[17, 20000]], rng.random((20, 72), dtype=np.float32)])
    mask = rng.random(V.shape[0]) < 0.6
    mask[[17, 29003, 20000, 6]] = True
    bits = np.zeros(((V.shape[0] + 31) // 32) * 32, bool)
    bits[:V.shape[0]] = mask
    words = np.packbits(bits, bitorder="little").view("<u4").astype(np.uint32)
    for devs in ([0, 0], [0, 0, 0]):
        sh = _vdb.NativeShards(72, metric, devs)
        for a, b in ((0, 7), (7, 10007), (10007, 10008), (10008, 30011)):
            sh.add(V[a:b])
        assert sh.count() == V.shape[0] and sum(sh.shard_counts()) == V.shape[0]
        assert max(sh.shard_counts()) - min(sh.shard_counts()) <= 10007
        np.testing.assert_array_equal(sh.get_vectors(), V)
        np.testing.assert_array_equal(sh.get_vectors(29990, 21), V[29990:])
        for k, m in ((10, None), (37, words)):
            s, i, kk = sh.search(Q, k, row_mask=m, with_keys=True)
            es, ei, ek = ref_cpu.exact_search(Q, V, k, metric, row_mask=None if m is None else mask)
            np.testing.assert_array_equal(i, ei)
            np.testing.assert_array_equal(kk, ek)
            np.testing.assert_array_equal(s, es)
        sh.clear()
        assert sh.count() == 0
        sh.close()


@pytest.mark.parametrize("metric", ["cosine", "euclidean"])
def test_shards_with_empty_shards(store_mod, metric):
    """Fewer rows than shards: the empty shards' lists carry key -inf, so they rank
    below every real row in the merge (an L2 key is -d^2 <= 0, a cosine score may be negative)."""
    from service import _vdb
    rng = np.random.default_rng(46)
    V = rng.standard_normal((3, 24)).astype(np.float32)
    Q = np.concatenate([V[[2, 0]], rng.standard_normal((2, 24)).astype(np.float32)])
    for rows in (1, 3):
        sh = _vdb.NativeShards(24, metric, [0, 0, 0, 0])
        sh.add(V[:rows])
        assert sorted(sh.shard_counts()) == [0] * (4 - rows) + [1] * rows
        for k in (1, 5):
            s, i, kk = sh.search(Q, k, with_keys=True)
            es, ei, ek = ref_cpu.exact_search(Q, V[:rows], k, metric)
            np.testing.assert_array_equal(i, ei)
            np.testing.assert_array_equal(kk, ek)
            assert ((i >= 0).sum(axis=1) == min(k, rows)).all()
        sh.close()


def test_store_over_devices_list(store_mod, tmp_path):
    """MLXVectorStoreConfig(devices=[0, 0]): the store API over the shard set."""
    rng = np.random.default_rng(45)
    V = rng.random((5000, 40), dtype=np.float32)
    meta = [{"id": i, "g": i % 3} for i in range(5000)]
    st = _mk(store_mod, tmp_path / "m", 40, devices=[0, 0])
    st.add_vectors(V[:1234], meta[:1234])
    st.add_vectors(V[1234:], meta[1234:])
    for q, filt in ((V[4321], None), (rng.random(40, dtype=np.float32), {"g": 1})):
        gi, gs, gm = st.query(q, k=10, filter_metadata=filt)
        ri, rs, rm = ref_cpu.reference_store_search(q, V, 10, "cosine", meta, filt)
        assert gi == ri and gm == rm
        np.testing.assert_allclose(gs, rs, rtol=1e-4, atol=1e-5)
    assert st.batch_query(V[:3], k=2)[1][0][0] == 1
    st2 = _mk(store_mod, tmp_path / "m", 40, devices=[0, 0])  # reload from the append log
    assert st2._vector_count == 5000 and st2.query(V[4321], k=3)[0][0] == 4321
    from service import _vdb
    _vdb.shutdown()  # idle workspaces released; the stores keep working
    assert st.query(V[10], k=1)[0] == [10]


@pytest.mark.parametrize("metric", ["cosine", "euclidean"])
def test_shards_search_device_queued_back_to_back(store_mod, metric):
    """vdb_shards_search_device (include/vdb.h): three batches queued on one stream of
    devices[0] without a host wait (device masks included), each equal to exact_search."""
    import torch
    from service import _vdb
    rng = np.random.default_rng(47)
    V = rng.random((40_003, 48), dtype=np.float32)
    sh = _vdb.NativeShards(48, metric, [0, 0, 0])
    for a, b in ((0, 10_000), (10_000, 40_003)):
        sh.add(V[a:b])
    mask = rng.random(V.shape[0]) < 0.5
    bits = np.zeros(((V.shape[0] + 31) // 32) * 32, bool)
    bits[:V.shape[0]] = mask
    words = torch.from_numpy(np.packbits(bits, bitorder="little").view("<u4").astype(np.int32)).cuda()
    st = torch.cuda.Stream()
    batches = [rng.random((B, 48), dtype=np.float32) for B in (17, 64, 5)]
    outs = []
    with torch.cuda.stream(st):
        for j, Qh in enumerate(batches):
            q = torch.from_numpy(Qh).cuda()
            s_ = torch.empty((q.shape[0], 12), dtype=torch.float32, device="cuda")
            i_ = torch.empty((q.shape[0], 12), dtype=torch.int64, device="cuda")
            k_ = torch.empty((q.shape[0], 12), dtype=torch.float64, device="cuda")
            sh.search_device(q.data_ptr(), q.shape[0], 12, s_.data_ptr(), i_.data_ptr(), k_.data_ptr(),
                             mask_ptr=words.data_ptr() if j == 1 else 0, stream=st.cuda_stream)
            outs.append((q, s_, i_, k_))
    st.synchronize()
    for j, (Qh, (_, s_, i_, k_)) in enumerate(zip(batches, outs)):
        es, ei, ek = ref_cpu.exact_search(Qh, V, 12, metric, row_mask=mask if j == 1 else None)
        np.testing.assert_array_equal(i_.cpu().numpy(), ei)
        np.testing.assert_array_equal(k_.cpu().numpy(), ek)
    sh.close()
