"""CPU checks of the oracle (oracle/ref_cpu.py) — no GPU.

Pins, in order of strength:
  1. hand-derived known answers (orthogonal / parallel / scaled / zero vectors
     whose cosine and L2 are exact in binary floating point);
  2. the reference's own behavioural known-answer tests, reproduced on the
     oracle:
       P1 self-query top-1, similarity > 0.999   tests/test_integration.py:81-85,115-136
       P2 filter on content_hash -> doc_10        tests/test_integration.py:139-160
       P3 multi-key AND filter / no match -> []   tests/demo.py:217-243
       P4 count == N                              tests/test_integration.py:102-111
       P5 len(results) == k                       tests/test_vector_store.py:39-40
       P6 batch shape                             tests/demo.py:130-139
       P7 empty store -> ([], [], [])             service/optimized_vector_store.py:117
  3. the committed golden fixtures (tests/golden/*.npz): the oracle reproduces
     them, and on them the reference-faithful fp32 path (normalise, matmul,
     stable argsort — the reference's own arithmetic) ranks exactly like the
     fp64 contract.
"""
import glob
import os

import numpy as np
import pytest

from oracle import ref_cpu

GOLDEN = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "*.npz")))


# ---- 1. known answers -----------------------------------------------------------------
def test_known_answers_cosine():
    V = np.array([[1, 0, 0, 0], [0, 1, 0, 0], [2, 0, 0, 0], [1, 1, 0, 0], [0, 0, 0, 0], [-1, 0, 0, 0]],
                 np.float32)
    q = np.array([3, 0, 0, 0], np.float32)
    s = ref_cpu.reference_cosine_scores(q, V)
    np.testing.assert_array_equal(s[[0, 1, 2, 4, 5]], [1, 0, 1, 0, -1])
    assert abs(s[3] - np.float32(1 / np.sqrt(2))) < 1e-7
    keys = ref_cpu.exact_keys(q, V, "cosine")
    np.testing.assert_array_equal(keys[[0, 1, 2, 4, 5]], [1, 0, 1, 0, -1])
    # ties (rows 0 and 2 both exactly 1.0) go to the lower row
    es, ei, ek = ref_cpu.exact_search(q[None], V, 6, "cosine")
    assert ei[0].tolist() == [0, 2, 3, 1, 4, 5]


def test_known_answers_euclidean():
    V = np.array([[0, 0], [3, 4], [6, 8], [-3, -4], [0, 0]], np.float32)
    q = np.array([0, 0], np.float32)
    d = ref_cpu.reference_euclidean_distances(q, V)
    np.testing.assert_array_equal(d, [0, 5, 10, 5, 0])
    es, ei, ek = ref_cpu.exact_search(q[None], V, 5, "euclidean")
    assert ei[0].tolist() == [0, 4, 1, 3, 2]
    np.testing.assert_array_equal(es[0], [0, 0, 5, 5, 10])
    np.testing.assert_array_equal(ek[0], [-0.0, -0.0, -25, -25, -100])


def test_canonical_sums_match_fp64_blas_closely():
    rng = np.random.default_rng(0)
    X = rng.standard_normal((50, 300)).astype(np.float32)
    q = rng.standard_normal(300).astype(np.float32)
    np.testing.assert_allclose(ref_cpu.canonical_dot64(q, X), X.astype(np.float64) @ q.astype(np.float64),
                               rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(ref_cpu.canonical_sumsq64(X), (X.astype(np.float64) ** 2).sum(1), rtol=1e-12)


def test_k_edge_cases():
    V = np.random.default_rng(1).random((7, 5), dtype=np.float32)
    assert ref_cpu.reference_topk_indices(ref_cpu.reference_cosine_scores(V[0], V), 0).size == 0  # k <= 0
    es, ei, ek = ref_cpu.exact_search(V[:2], V, 10, "cosine")  # k > N -> -1 padding
    assert (ei[:, 7:] == -1).all() and (ek[:, 7:] == -np.inf).all() and (ei[:, :7] >= 0).all()
    es, ei, ek = ref_cpu.exact_search(V[:1], V, 3, "cosine", row_mask=np.zeros(7, bool))
    assert (ei == -1).all()


def test_batch_validation_errors_match_reference():
    """performance/mlx_optimized.py:65-72 raise ValueError for bad shapes."""
    with pytest.raises(ValueError):
        ref_cpu.reference_cosine_batch(np.ones(4, np.float32), np.ones((3, 4), np.float32))
    with pytest.raises(ValueError):
        ref_cpu.reference_cosine_batch(np.ones((2, 4), np.float32), np.ones((3, 5), np.float32))


def test_unsupported_metric_raises_like_reference():
    with pytest.raises(RuntimeError, match="Keine kompilierte"):
        ref_cpu.reference_store_search(np.ones(4, np.float32), np.ones((3, 4), np.float32), 1, "dot_product")


# ---- 2. the reference's behavioural pins ----------------------------------------------------
def _docs(n):
    return [{"id": f"doc_{i}", "content_hash": f"hash_{i}", "parity": i % 2, "bucket": i % 5} for i in range(n)]


def test_p1_self_query_and_p5_length():
    V = np.random.default_rng(2).random((100, 384), dtype=np.float32)  # test_integration.py:83
    meta = _docs(100)
    idx, sc, md = ref_cpu.reference_store_search(V[0], V, 5, "cosine", meta)
    assert md[0]["id"] == "doc_0" and sc[0] > 0.999 and len(idx) == 5
    es, ei, ek = ref_cpu.exact_search(V[:1], V, 5, "cosine")
    assert ei[0].tolist() == idx


def test_p2_p3_filters():
    V = np.random.default_rng(3).standard_normal((20, 128)).astype(np.float32)  # demo.py:215
    meta = _docs(20)
    idx, sc, md = ref_cpu.reference_store_search(V[10], V, 1, "cosine", meta, {"content_hash": "hash_10"})
    assert idx == [10] and md[0]["id"] == "doc_10"
    idx, _, md = ref_cpu.reference_store_search(V[0], V, 20, "cosine", meta, {"parity": 1, "bucket": 3})
    assert sorted(idx) == [3, 13] and all(m["parity"] == 1 and m["bucket"] == 3 for m in md)
    assert ref_cpu.reference_store_search(V[0], V, 5, "cosine", meta, {"parity": 7}) == ([], [], [])
    mask = np.array([m["parity"] == 1 and m["bucket"] == 3 for m in meta])
    es, ei, ek = ref_cpu.exact_search(V[:1], V, 20, "cosine", row_mask=mask)
    assert sorted(ei[0][ei[0] >= 0].tolist()) == [3, 13]


def test_p6_batch_shape_and_p7_empty():
    V = np.random.default_rng(4).random((50, 16), dtype=np.float32)
    idx, sc = ref_cpu.reference_batch_search(V[:3], V, 2)
    assert idx.shape == (3, 2) and sc.shape == (3, 2) and idx[:, 0].tolist() == [0, 1, 2]
    assert ref_cpu.reference_store_search(V[0], np.zeros((0, 16), np.float32), 5) == ([], [], [])
    i0, s0 = ref_cpu.reference_batch_search(V[:3], np.zeros((0, 16), np.float32), 5)
    assert i0.shape == (3, 0)


# ---- 3. golden fixtures ------------------------------------------------------------------
@pytest.mark.parametrize("path", GOLDEN, ids=[os.path.basename(p) for p in GOLDEN])
def test_oracle_reproduces_golden(path):
    z = np.load(path, allow_pickle=False)
    V, Q, k, metric = z["vectors"], z["queries"], int(z["k"]), str(z["metric"])
    mask = z["mask"] if z["mask"].size else None
    es, ei, ek = ref_cpu.exact_search(Q, V, k, metric, row_mask=mask)
    np.testing.assert_array_equal(ei, z["exact_idx"])
    np.testing.assert_array_equal(ek, z["exact_keys"])
    np.testing.assert_array_equal(es, z["exact_scores"])
    # the reference's own fp32 arithmetic ranks identically on these inputs and
    # its scores are within the 1e-4 contract of the exact ones
    np.testing.assert_array_equal(z["ref_idx"], z["exact_idx"])
    valid = ei >= 0
    np.testing.assert_allclose(z["ref_scores"][valid], es[valid], atol=1e-4, rtol=0)


def test_golden_prefilter_path_matches_brute_force():
    """exact_search switches to a BLAS prefilter above 4096 eligible rows; it must
    give the same answer as keying every row canonically."""
    rng = np.random.default_rng(5)
    V = rng.random((6000, 64), dtype=np.float32)
    V[4000:4010] = V[17]
    Q = np.stack([V[17], rng.random(64, dtype=np.float32)])
    for metric in ("cosine", "euclidean"):
        es, ei, ek = ref_cpu.exact_search(Q, V, 15, metric)
        for b in range(2):
            keys = ref_cpu.exact_keys(Q[b], V, metric)
            order = ref_cpu.exact_topk_from_keys(keys, 15)
            np.testing.assert_array_equal(ei[b], order)
            np.testing.assert_array_equal(ek[b], keys[order])


def test_merge_of_shards_equals_global():
    rng = np.random.default_rng(6)
    V = rng.random((3000, 32), dtype=np.float32)
    V[2500:2510] = V[5]
    Q = rng.random((4, 32), dtype=np.float32)
    Q[0] = V[5]
    k = 12
    bounds = [0, 700, 1500, 3000]
    keys, idx = [], []
    for g in range(3):
        _, i, kk = ref_cpu.exact_search(Q, V[bounds[g]:bounds[g + 1]], k, "cosine")
        keys.append(kk)
        idx.append(np.where(i >= 0, i + bounds[g], -1))
    mk, mi = ref_cpu.merge_topk(np.stack(keys), np.stack(idx), k)
    es, ei, ek = ref_cpu.exact_search(Q, V, k, "cosine")
    np.testing.assert_array_equal(mi, ei)
    np.testing.assert_array_equal(mk, ek)


def test_select_neighbors_known_answers():
    """hnswlib's heuristic (oracle.select_neighbors, restating getNeighborsByHeuristic2 as
    graph_prune_kernel runs it) on hand-built cases: candidates along one ray from the node
    keep only the nearest (each farther one is closer to a kept one than to the node);
    orthogonal candidates are all kept; keepPrunedConnections (fill) tops up nearest first."""
    D = 8
    X = np.zeros((8, D), np.float32)
    X[0] = 0.0
    X[0, 0] = 1.0            # node at e0
    for i, t in enumerate((2.0, 3.0, 4.0)):   # rows 1..3 on the ray e0 * t
        X[1 + i, 0] = t
    X[4, 1] = 1.0; X[5, 2] = 1.0; X[6, 3] = 1.0  # unit axes, orthogonal to each other
    X[7, 0] = 1.0; X[7, 4] = 0.5
    sc = ref_cpu._row_scales(X, "euclidean")
    out, dist, amb = ref_cpu.select_neighbors(X, sc, 0, [1, 2, 3, -1], 4, "euclidean")
    assert out.tolist() == [1, -1, -1, -1] and not amb
    assert dist[0] == 1.0
    out, _, _ = ref_cpu.select_neighbors(X, sc, 0, [1, 2, 3, -1], 3, "euclidean", fill=True)
    assert out.tolist() == [1, 2, 3]
    # node at the origin direction e0 (cosine): axes e1, e2, e3 all at distance 1, pairwise 1
    # (not < 1): all kept in candidate order
    scc = ref_cpu._row_scales(X, "cosine")
    out, _, _ = ref_cpu.select_neighbors(X, scc, 0, [4, 5, 6], 3, "cosine")
    assert out.tolist() == [4, 5, 6]
    # sort: candidates given far-first come back nearest first
    out, dist, _ = ref_cpu.select_neighbors(X, sc, 0, [3, 7, 4], 3, "euclidean", sort=True)
    assert out[0] == 7 and dist[0] == np.float32(0.25)


def test_graph_build_restatement_small():
    """The restated build: every list holds distinct rows other than the node, at most
    `degree` of them, each node with at least one out-edge, entries evenly spread."""
    rng = np.random.default_rng(3)
    X = rng.integers(0, 4, (300, 16)).astype(np.float32)
    for metric in ("cosine", "euclidean"):
        nbr, ent, amb = ref_cpu.graph_build(X, metric, degree=16, knn=16, n_entries=8)
        assert nbr.shape == (300, 16) and not amb.any()
        for v in range(300):
            row = nbr[v][nbr[v] >= 0]
            assert row.size >= 1 and v not in row and len(set(row.tolist())) == row.size
        assert ent.tolist() == [i * 300 // 8 for i in range(8)]


def test_l2_batch_chunked_equals_the_store_path():
    """The chunked L2 batch (bench.py's C4 CPU baseline) returns exactly what the
    store's per-query path (`_compiled_euclidean_distance` + stable argsort [:k]) returns, ties
    included (duplicate rows straddling chunk boundaries)."""
    rng = np.random.default_rng(3)
    V = rng.random((5000, 24), dtype=np.float32)
    V[1999:2003] = V[10]  # ties at a chunk boundary (chunk 1000 rows)
    V[4500] = V[10]
    Q = rng.random((7, 24), dtype=np.float32)
    Q[0] = V[10]
    for k in (1, 10, 37):
        idx, dist = ref_cpu.reference_l2_batch_chunked(Q, V, k, chunk_rows=1000)
        for b in range(Q.shape[0]):
            ri, rs, _ = ref_cpu.reference_store_search(Q[b], V, k, "euclidean")
            assert idx[b].tolist() == ri
            np.testing.assert_array_equal(dist[b], np.asarray(rs, np.float32))
