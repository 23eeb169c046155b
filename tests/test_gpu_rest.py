"""The drop-in boundary end to end on the GPU: the /vectors routes
(mlx-vector-db_amd/api/routes/vectors.py) over the device store, at BASELINE.json configs[0]
(C1: 10K x 384 cosine top-10, single query), against the oracle's restatement of the
reference store (oracle/ref_cpu.reference_store_search = service/optimized_vector_store.py:116-192)
with the reference route's S12 formatting (api/routes/vectors.py:236-258, :296-315) written out
here; and the store under the reference's concurrency (4 executor threads, api/routes/vectors.py:43)
while a fifth thread adds rows."""
import threading
import time

import numpy as np
import pytest

from oracle import ref_cpu

pytestmark = pytest.mark.gpu
AUTH = {"Authorization": "Bearer mlx-vector-dev-key-2024"}


@pytest.fixture(scope="module")
def store_mod():
    from service import _vdb, optimized_vector_store
    assert _vdb.device_count() >= 1, "no GPU visible"
    return optimized_vector_store


@pytest.mark.parametrize("metric", ["cosine", "euclidean"])
def test_rest_routes_c1_10k_x_384(store_mod, tmp_path, metric):
    from fastapi.testclient import TestClient
    from api.routes import vectors as routes
    mgr = routes.VectorStoreManager(config_factory=lambda u, m: store_mod.MLXVectorStoreConfig(dimension=384,
                                                                                               metric=metric),
                                    base_dir=str(tmp_path))
    c = TestClient(routes.create_app(mgr))
    rng = np.random.default_rng(100)
    N, D, k = 10_000, 384, 10
    V = rng.random((N, D), dtype=np.float32)  # tests/quick_test.py / large_scale_benchmark.py data
    meta = [{"id": f"doc_{i}", "content_hash": f"hash_{i}", "g": i % 4} for i in range(N)]
    for s in range(0, N, 2500):
        r = c.post("/vectors/add", json={"user_id": "u", "model_id": "m", "vectors": V[s:s + 2500].tolist(),
                                         "metadata": meta[s:s + 2500]}, headers=AUTH)
        assert r.status_code == 200, r.text
    assert r.json()["total_vectors"] == N
    Q = np.concatenate([V[[0, 10, 4321]], rng.random((5, D), dtype=np.float32)])
    for b, q in enumerate(Q):
        for filt in (None, {"g": 2}):
            body = {"user_id": "u", "model_id": "m", "query": q.tolist(), "k": k}
            if filt:
                body["filter_metadata"] = filt
            got = c.post("/vectors/query", json=body, headers=AUTH).json()["results"]
            # the JSON round trip of q is exact (float32 -> double -> float32)
            ii, ss, mm = ref_cpu.reference_store_search(q, V, k, metric, meta, filt)
            assert [x["metadata"]["id"] for x in got] == [m["id"] for m in mm]
            assert [x["rank"] for x in got] == list(range(1, k + 1))
            for x, s in zip(got, ss):
                if metric == "cosine":
                    assert abs(x["similarity_score"] - s) < 1e-4 and abs(x["distance"] - (1.0 - s)) < 1e-4
                else:
                    assert abs(x["distance"] - s) < 1e-4 * max(1.0, s)
                    assert abs(x["similarity_score"] - 1.0 / (1.0 + s)) < 1e-4
            if b < 3 and not filt:
                assert got[0]["metadata"]["id"] == meta[[0, 10, 4321][b]]["id"]          # P1
                if metric == "cosine":
                    assert got[0]["similarity_score"] > 0.999
    # P2: the content_hash filter returns exactly that row (tests/test_integration.py:139-160)
    got = c.post("/vectors/query", json={"user_id": "u", "model_id": "m", "query": V[10].tolist(), "k": 1,
                                         "filter_metadata": {"content_hash": "hash_10"}}, headers=AUTH).json()
    assert [x["metadata"]["id"] for x in got["results"]] == ["doc_10"]
    # /batch_query: every query's list equals /query's, scored from distances (vectors.py:300-315)
    body = {"user_id": "u", "model_id": "m", "queries": Q.tolist(), "k": k}
    res = c.post("/vectors/batch_query", json=body, headers=AUTH)
    assert res.status_code == 200, res.text
    res = res.json()
    assert res["total_queries"] == len(Q)
    for b, q in enumerate(Q):
        ii, ss, mm = ref_cpu.reference_store_search(q, V, k, metric, meta)
        got = res["results"][b]
        assert [x["metadata"]["id"] for x in got] == [m["id"] for m in mm]
        for x, s in zip(got, ss):
            if metric == "cosine":
                assert abs(x["distance"] - (1.0 - s)) < 1e-4 and abs(x["similarity_score"] - max(0.0, s)) < 1e-4
            else:
                assert abs(x["distance"] - s) < 1e-4 * max(1.0, s)
        if b < 3 and metric == "cosine":
            assert got[0]["similarity_score"] > 0.999  # the best match scores ~1, not ~0
    assert c.get("/vectors/count", params={"user_id": "u", "model_id": "m"}, headers=AUTH).json() == {"count": N}


def test_concurrent_queries_during_adds(store_mod, tmp_path):
    """4 threads query / batch_query one store while a fifth appends rows: no errors, and
    every answer equals the oracle over one of the row-count snapshots the store went
    through (queries see whole adds, never half of one)."""
    rng = np.random.default_rng(7)
    D, k, chunk, n_chunks, N0 = 64, 10, 4000, 5, 20_000
    V = rng.random((N0 + chunk * n_chunks, D), dtype=np.float32)
    Q = rng.random((12, D), dtype=np.float32)
    st = store_mod.MLXVectorStore(str(tmp_path / "c"), store_mod.MLXVectorStoreConfig(dimension=D, persist=False))
    st.add_vectors(V[:N0], [{"i": i} for i in range(N0)])
    sizes = [N0 + chunk * j for j in range(n_chunks + 1)]
    want = {n: ref_cpu.exact_search(Q, V[:n], k, "cosine")[1] for n in sizes}
    errors, answers = [], []
    stop = threading.Event()

    def reader(tid):
        r = np.random.default_rng(tid)
        try:
            while not stop.is_set():
                if tid % 2:
                    b = int(r.integers(0, len(Q)))
                    answers.append(((b,), [st.query(Q[b], k=k)[0]]))
                else:
                    bs = tuple(sorted(set(r.integers(0, len(Q), 4).tolist())))
                    answers.append((bs, [x[0] for x in st.batch_query(Q[list(bs)], k=k)]))
        except Exception as e:  # pragma: no cover - reported below
            errors.append(repr(e))

    def wait_answers(n, limit=60.0):
        t0 = time.time()
        while len(answers) < n and time.time() - t0 < limit and not errors:
            time.sleep(0.002)

    def writer():
        try:
            for j in range(n_chunks):
                wait_answers(len(answers) + 8)  # some answers between every two adds
                s = N0 + chunk * j
                st.add_vectors(V[s:s + chunk], [{"i": i} for i in range(s, s + chunk)])
            wait_answers(len(answers) + 8)
        except Exception as e:  # pragma: no cover
            errors.append(repr(e))

    threads = [threading.Thread(target=reader, args=(t,)) for t in range(4)]
    for t in threads:
        t.start()
    w = threading.Thread(target=writer)
    w.start()
    w.join()
    stop.set()
    for t in threads:
        t.join()
    assert not errors, errors
    assert st._vector_count == sizes[-1] and len(answers) > 20
    seen = set()
    for bs, lists in answers:
        ok = [n for n in sizes if all(lst == want[n][b].tolist() for b, lst in zip(bs, lists))]
        assert ok, (bs, lists)
        seen.update(ok)
    assert len(seen) >= 2  # answers were served while the corpus grew
