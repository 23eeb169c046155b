"""performance/mlx_optimized.py on the device (the reference's operator module,
/root/reference/performance/mlx_optimized.py:26-287), each function against its numpy
restatement: scores within 1e-4 (fp32, the tolerance north_star states), top-k indices
exact with ties to the lower index, the reference's ValueErrors."""
import numpy as np
import pytest

from oracle import ref_cpu

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mo():
    from service import _vdb
    assert _vdb.device_count() >= 1, "no GPU visible"
    from performance import mlx_optimized
    return mlx_optimized


def test_score_operators(mo):
    rng = np.random.default_rng(50)
    for N, D, B in ((3001, 384, 5), (70, 33, 40), (1, 7, 1), (4096, 1536, 3)):
        V = rng.standard_normal((N, D)).astype(np.float32)
        Q = rng.standard_normal((B, D)).astype(np.float32)
        np.testing.assert_allclose(mo.compute_cosine_similarity_batch(Q, V), ref_cpu.reference_cosine_batch(Q, V),
                                   atol=1e-4, rtol=0)
        np.testing.assert_allclose(mo.compute_cosine_similarity_single(Q[0], V),
                                   ref_cpu.reference_cosine_scores(Q[0], V), atol=1e-4, rtol=0)
        np.testing.assert_allclose(mo.compute_euclidean_distance(Q[0], V),
                                   ref_cpu.reference_euclidean_distances(Q[0], V), atol=1e-4, rtol=1e-5)
        d1 = mo.compute_dot_product(Q[0], V)                     # mx.matmul(db, q)
        np.testing.assert_allclose(d1, V.astype(np.float64) @ Q[0], atol=1e-4 * np.sqrt(D), rtol=1e-5)
        d2 = mo.compute_dot_product(Q, V)                        # (db @ Q^T).flatten()
        np.testing.assert_allclose(d2, (V.astype(np.float64) @ Q.T).reshape(-1), atol=1e-4 * np.sqrt(D), rtol=1e-5)
        nv = mo.normalize_vectors(V)
        np.testing.assert_allclose(nv, V / np.maximum(np.linalg.norm(V, axis=1, keepdims=True), 1e-8), atol=1e-6)
    with pytest.raises(ValueError):
        mo.compute_cosine_similarity_batch(np.ones(4, np.float32), np.ones((3, 4), np.float32))
    with pytest.raises(ValueError):
        mo.compute_cosine_similarity_batch(np.ones((2, 4), np.float32), np.ones((3, 5), np.float32))
    with pytest.raises(ValueError):
        mo.compute_cosine_similarity_single(np.ones((2, 4), np.float32), np.ones((3, 4), np.float32))
    with pytest.raises(ValueError):
        mo.fast_vector_concatenation(np.ones((2, 4), np.float32), np.ones((3, 5), np.float32))


def test_topk_and_searches(mo):
    rng = np.random.default_rng(51)
    s = rng.standard_normal(100_000).astype(np.float32)
    s[[5, 700, 99_999]] = 9.0                                    # a three-way tie at the top
    s[1234] = np.nan
    idx = mo.fast_top_k_indices(s, 10)
    ref = ref_cpu.reference_topk_indices(np.where(np.isnan(s), -np.inf, s), 10)
    assert idx.tolist() == ref.tolist() and idx[:3].tolist() == [5, 700, 99_999]
    assert mo.fast_top_k_indices(s, 0).size == 0 and mo.fast_top_k_indices(s[:3], 10).size == 3
    big = rng.random(300_000).astype(np.float32)
    assert mo.fast_top_k_indices(big, 1000).tolist() == ref_cpu.reference_topk_indices(big, 1000).tolist()
    V = rng.random((20000, 96), dtype=np.float32)
    Q = rng.random((7, 96), dtype=np.float32)
    Q[3] = V[4321]
    i, sc = mo.optimized_batch_similarity_search(Q, V, 10)
    es, ei, _ = ref_cpu.exact_search(Q, V, 10, "cosine")
    assert (i == ei).all() and i[3, 0] == 4321
    np.testing.assert_allclose(sc, es, atol=1e-6)
    i1, s1 = mo.optimized_similarity_search(Q[3], V, 5)
    assert i1.tolist() == ei[3, :5].tolist()
    i0, s0 = mo.optimized_batch_similarity_search(Q, V[:0], 10)
    assert i0.shape == (7, 0)
    comb = mo.optimized_vector_addition(V[:10], V[10:20], normalize=True)
    np.testing.assert_allclose(comb, V[:20] / np.linalg.norm(V[:20], axis=1, keepdims=True), atol=1e-6)
    mo.warmup_compiled_functions(64, 100)
    assert "optimized_batch_similarity_search" in mo.performance_monitor.get_stats()


def test_device_tensors_stay_on_device(mo):
    import torch
    rng = np.random.default_rng(52)
    V = torch.from_numpy(rng.random((5000, 64), dtype=np.float32)).cuda()
    Q = torch.from_numpy(rng.random((4, 64), dtype=np.float32)).cuda()
    out = mo.compute_cosine_similarity_batch(Q, V)
    assert out.is_cuda and tuple(out.shape) == (4, 5000)
    np.testing.assert_allclose(out.cpu().numpy(), ref_cpu.reference_cosine_batch(Q.cpu().numpy(), V.cpu().numpy()),
                               atol=1e-4, rtol=0)
    idx = mo.fast_top_k_indices(out[0], 7)
    assert idx.is_cuda and idx.cpu().tolist() == ref_cpu.reference_topk_indices(out[0].cpu().numpy(), 7).tolist()


def test_batch_search_device_corpus_no_host_copy(mo, monkeypatch):
    """optimized_batch_similarity_search (performance/mlx_optimized.py:217-248) on torch CUDA
    tensors at 200K rows: the corpus goes device to device into a cached index (no .cpu() of
    any tensor during the calls, checked by a patched Tensor.cpu), results stay on device and
    match the exact oracle; the reference's fp32 scores within 1e-4; an in-place write to the
    corpus (version bump) is seen by the next call."""
    import torch
    rng = np.random.default_rng(53)
    Vh = rng.random((200_000, 128), dtype=np.float32)
    Qh = rng.random((48, 128), dtype=np.float32)
    Qh[5] = Vh[199_999]
    V, Q = torch.from_numpy(Vh).cuda(), torch.from_numpy(Qh).cuda()
    es, ei, _ = ref_cpu.exact_search(Qh, Vh, 10, "cosine")
    ri, rs = ref_cpu.reference_batch_search(Qh, Vh, 10)
    real_cpu = torch.Tensor.cpu
    copies = []

    def guarded_cpu(self, *a, **kw):
        copies.append(tuple(self.shape))
        return real_cpu(self, *a, **kw)
    monkeypatch.setattr(torch.Tensor, "cpu", guarded_cpu)
    outs = [mo.optimized_batch_similarity_search(Q, V, 10) for _ in range(3)]
    i1, s1 = mo.optimized_similarity_search(Q[5], V, 4)
    torch.cuda.synchronize()
    assert copies == []  # nothing moved to the host inside the mirror
    monkeypatch.setattr(torch.Tensor, "cpu", real_cpu)
    for i, s in outs:
        assert i.is_cuda and s.is_cuda and tuple(i.shape) == (48, 10)
        np.testing.assert_array_equal(i.cpu().numpy(), ei)
        np.testing.assert_allclose(s.cpu().numpy(), rs, atol=1e-4, rtol=0)
    assert i1.is_cuda and i1.cpu().tolist() == ei[5, :4].tolist()
    V[123] = Q[7]  # in place: the cached index must not serve the old rows
    i2, _ = mo.optimized_batch_similarity_search(Q[7:8], V, 1)
    assert i2.cpu().tolist() == [[123]]
