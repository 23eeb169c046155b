"""BASELINE.json's configurations at their full sizes on one GPU, through the C-ABI.

Every query of every batch is checked for the size-independent properties (sorted
output, planted self-queries on top, no invalid slots, fallbacks counted); a spread of
queries across all query blocks is checked exactly (indices and fp64 keys) against the
oracle (oracle/ref_cpu.exact_search, which keys only a prefiltered candidate set, so it
finishes in seconds at these sizes).

The exact-vs-reference-fp32 question (north_star: indices "bit-exact" with the MLX fp32
reference): on the same queries the numpy restatement of the reference's own fp32 path
(cosine: reference_batch_search = performance/mlx_optimized.py:217-248; L2: the store's
per-query operator, service/optimized_vector_store.py:43-48 + :176-178) is run, and every
place its order differs from the returned one must be a near tie -- exact keys closer than
twice the fp32 error bound of the reference's own arithmetic.  The counts go to
$VDB_TEST_REPORT_DIR/<config>_fp32_ref.json.

  C2  1M x 768 cosine, B=64, k=10: all 64 queries exact and against the fp32 order.
  C3  1M x 1536 cosine, B=256, k=10 (4 query blocks).
  C4  10M x 128 L2, B=512, k=100 (8 query blocks), both step-end modes of the scan.
  C6  10M x 128 cosine, B=64, k=10 (the metric's 8-GPU workload, on one GPU).
  C3 / C4 / C6 run the default precision (VDB_PREC_AUTO) twice; both searches are checked
  and the second must certify (<= 2% fallbacks; a fallback is still exact, only slower).
  C5  5M x 384 graph (M=16 -> degree 32, efSearch=128), batch 1: hnswlib's distance
      conventions (performance/hnsw_index.py:35,101) checked against exact keys of the
      returned rows, recall@10 against the exact path on 100 queries.
"""
import json
import os
import time

import numpy as np
import pytest

from oracle import ref_cpu

pytestmark = [pytest.mark.gpu, pytest.mark.slow]


@pytest.fixture(scope="module")
def vdb():
    from service import _vdb
    assert _vdb.device_count() >= 1, "no GPU visible"
    return _vdb


def _report(name, obj):
    d = os.environ.get("VDB_TEST_REPORT_DIR")
    if d:
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, name), "w") as f:
            json.dump(obj, f, indent=1)
    print(name, json.dumps(obj))


def _properties(s, i, metric, N):
    assert (i >= 0).all() and (i < N).all()
    if metric == "cosine":
        assert (np.diff(s, axis=1) <= 0).all()
    else:
        assert (np.diff(s, axis=1) >= 0).all()
    for row in i:  # no row twice in one list
        assert np.unique(row).size == row.size


def _fp32_order(Q, V, i, sub, k, metric):
    """Positions where the reference's fp32 order differs from ours, each checked to be a near
    tie of the exact keys (< 2x the fp32 bound); returns the report fields."""
    D = V.shape[1]
    if metric == "cosine":
        ri, rs = ref_cpu.reference_batch_search(Q[sub], V, k)
        # one fp32 cosine: D additions + the normalisation roundings, relative to |q||x| = 1
        eps32 = 1.01 * (D + 8) * 2.0 ** -24
    else:
        ri, rs = [], []
        for b in sub:
            d = ref_cpu.reference_euclidean_distances(Q[b], V)
            top = ref_cpu.reference_topk_indices(d, k, metric)
            ri.append(top)
            rs.append(d[top])
        ri, rs = np.array(ri), np.array(rs)
        eps32 = None  # per query below: (D + 3) 2^-24 of the largest squared distance compared
    pos_diff, set_diff, worst, bound = 0, 0, 0.0, 0.0
    for r, b in enumerate(sub):
        ours, ref = i[b].tolist(), ri[r].tolist()
        pairs = [(a, c) for a, c in zip(ours, ref) if a != c]
        pos_diff += len(pairs)
        set_diff += len(set(ref) - set(ours))
        rows = sorted(set(ours) | set(ref))
        kx = ref_cpu.exact_keys(Q[b], V[rows], metric)
        key = dict(zip(rows, kx))
        e2 = 2 * eps32 if eps32 is not None else 2 * 1.01 * (D + 3) * 2.0 ** -24 * float(np.max(-kx))
        bound = max(bound, e2)
        for a, c in pairs:
            gap = abs(key[a] - key[c])
            worst = max(worst, gap)
            assert gap < e2, (b, a, c, gap, e2)
        for c in set(ref) - set(ours):  # a reference row we left out ties with our k-th
            assert abs(key[ours[-1]] - key[c]) < e2
    return {"queries": len(sub), "k": k, "positions_differing": pos_diff, "rows_differing": set_diff,
            "max_exact_key_gap_of_a_swap": worst, "fp32_bound_2eps": bound}, rs


def test_c2_exact_vs_reference_fp32_order(vdb):
    N, D, B, k = 1_000_000, 768, 64, 10
    V = np.random.default_rng(0).random((N, D), dtype=np.float32)
    Q = np.random.default_rng(1).random((B, D), dtype=np.float32)
    Q[5], Q[40] = V[777_777], V[3]
    ix = vdb.NativeIndex(D, "cosine")
    ix.add(V)
    s, i, kk = ix.search(Q, k, with_keys=True)
    _properties(s, i, "cosine", N)
    assert i[5, 0] == 777_777 and i[40, 0] == 3
    sub = list(range(B))  # every query of the batch
    es, ei, ek = ref_cpu.exact_search(Q[sub], V, k, "cosine")
    np.testing.assert_array_equal(i[sub], ei)
    np.testing.assert_array_equal(kk[sub], ek)
    rep, rs = _fp32_order(Q, V, i, sub, k, "cosine")
    np.testing.assert_allclose(s[sub], rs, atol=1e-4, rtol=0)
    assert ix.stat("fallback_queries") == 0
    rep.update(precision=ix.precision,
               searches_by_precision={p: ix.stat(f"searches_{p}") for p in ("bf16", "bf16x3", "fp32", "i8", "i8x3", "i8q")})
    _report("c2_fp32_ref.json", rep)


def test_c3_1m_x_1536_b256(vdb):
    N, D, B, k = 1_000_000, 1536, 256, 10
    V = np.random.default_rng(3).random((N, D), dtype=np.float32)
    Q = np.random.default_rng(4).random((B, D), dtype=np.float32)
    plant = {0: 12, 100: 999_999, 200: 500_000, 255: 77}
    for b, r in plant.items():
        Q[b] = V[r]
    ix = vdb.NativeIndex(D, "cosine")
    ix.add(V)
    sub = [0, 1, 63, 64, 100, 127, 128, 191, 200, 255]  # all 4 query blocks
    es, ei, ek = ref_cpu.exact_search(Q[sub], V, k, "cosine")
    fbs, dts = [], []
    for _ in range(2):
        fb0 = ix.stat("fallback_queries")
        t0 = time.perf_counter()
        s, i, kk = ix.search(Q, k, with_keys=True)
        dts.append(time.perf_counter() - t0)
        fbs.append(ix.stat("fallback_queries") - fb0)
        _properties(s, i, "cosine", N)
        for b, r in plant.items():
            assert i[b, 0] == r and s[b, 0] > 0.9999
        np.testing.assert_array_equal(i[sub], ei)
        np.testing.assert_array_equal(kk[sub], ek)
    by_prec = {p: ix.stat(f"searches_{p}") for p in ("bf16", "bf16x3", "fp32", "i8", "i8x3", "i8q")}
    _report("c3.json", {"fallback_queries_per_search": fbs, "host_search_s": dts, "searches_by_precision": by_prec})
    rep, rs = _fp32_order(Q, V, i, sub, k, "cosine")
    np.testing.assert_allclose(s[sub], rs, atol=1e-4, rtol=0)
    _report("c3_fp32_ref.json", rep)
    assert fbs[-1] <= B // 50  # certified by the candidate pass (a fallback is still exact, only slower)


@pytest.mark.parametrize("sync", [0, 1])
def test_c4_10m_x_128_l2_b512_top100(vdb, sync):
    N, D, B, k = 10_000_000, 128, 512, 100
    V = np.random.default_rng(5).random((N, D), dtype=np.float32)
    Q = np.random.default_rng(6).random((B, D), dtype=np.float32)
    plant = {3: 9_999_999, 70: 0, 300: 4_242_424, 511: 1_234_567}
    for b, r in plant.items():
        Q[b] = V[r]
    ix = vdb.NativeIndex(D, "euclidean")
    ix.set_param("scan_sync", sync)  # 0 = auto (flag-gated: int8 pass, Dp = 128), 1 = lockstep
    ix.reserve(N)
    for s0 in range(0, N, 1 << 21):
        ix.add(V[s0:s0 + (1 << 21)])
    sub = [0, 3, 70, 130, 200, 290, 300, 350, 450, 511]  # all 8 query blocks
    es, ei, ek = ref_cpu.exact_search(Q[sub], V, k, "euclidean")
    fbs = []
    for _ in range(2):
        fb0 = ix.stat("fallback_queries")
        s, i, kk = ix.search(Q, k, with_keys=True)
        fbs.append(ix.stat("fallback_queries") - fb0)
        _properties(s, i, "euclidean", N)
        for b, r in plant.items():
            assert i[b, 0] == r and s[b, 0] == 0.0
        np.testing.assert_array_equal(i[sub], ei)
        np.testing.assert_array_equal(kk[sub], ek)
    by_prec = {p: ix.stat(f"searches_{p}") for p in ("bf16", "bf16x3", "fp32", "i8", "i8x3", "i8q")}
    _report(f"c4_sync{sync}.json", {"fallback_queries_per_search": fbs, "searches_by_precision": by_prec})
    assert fbs[-1] <= B // 50
    if sync == 0:
        rep, rs = _fp32_order(Q, V, i, sub, k, "euclidean")
        np.testing.assert_allclose(s[sub], rs, atol=1e-4, rtol=1e-5)
        _report("c4_fp32_ref.json", rep)


def test_c6_10m_x_128_cosine_b64_top10(vdb):
    """The metric's 8-GPU workload (BASELINE.json metric: cosine top-10 batch=64, 10M x 128)
    on one GPU: properties on every query, exact on a spread, fp32-order report."""
    N, D, B, k = 10_000_000, 128, 64, 10
    V = np.random.default_rng(9).random((N, D), dtype=np.float32)
    Q = np.random.default_rng(10).random((B, D), dtype=np.float32)
    plant = {0: 9_999_999, 31: 0, 32: 5_555_555, 63: 123_456}
    for b, r in plant.items():
        Q[b] = V[r]
    ix = vdb.NativeIndex(D, "cosine")
    ix.reserve(N)
    for s0 in range(0, N, 1 << 21):
        ix.add(V[s0:s0 + (1 << 21)])
    sub = list(range(0, B, 4))
    es, ei, ek = ref_cpu.exact_search(Q[sub], V, k, "cosine")
    fbs = []
    for _ in range(2):
        fb0 = ix.stat("fallback_queries")
        s, i, kk = ix.search(Q, k, with_keys=True)
        fbs.append(ix.stat("fallback_queries") - fb0)
        _properties(s, i, "cosine", N)
        for b, r in plant.items():
            assert i[b, 0] == r and s[b, 0] > 0.9999
        np.testing.assert_array_equal(i[sub], ei)
        np.testing.assert_array_equal(kk[sub], ek)
    by_prec = {p: ix.stat(f"searches_{p}") for p in ("bf16", "bf16x3", "fp32", "i8", "i8x3", "i8q")}
    _report("c6.json", {"fallback_queries_per_search": fbs, "searches_by_precision": by_prec})
    assert fbs[-1] <= max(1, B // 50)
    rep, rs = _fp32_order(Q, V, i, sub, k, "cosine")
    np.testing.assert_allclose(s[sub], rs, atol=1e-4, rtol=0)
    _report("c6_fp32_ref.json", rep)


def _hostile_rows(seed, n, D):
    """Heavy-tailed rows (a Gaussian scale mixture: z1 exp(0.75 z2), tails far past a normal's),
    generated per 1 M-row chunk."""
    out = np.empty((n, D), np.float32)
    for s0 in range(0, n, 1 << 20):
        g = np.random.default_rng([seed, s0])
        m = min(1 << 20, n - s0)
        z = g.standard_normal((m, D), dtype=np.float32)
        out[s0:s0 + m] = z * np.exp(np.float32(0.75) * g.standard_normal((m, D), dtype=np.float32))
    return out


@pytest.mark.timeout(900)
@pytest.mark.parametrize("metric", ["cosine", "euclidean"])
def test_certificate_on_data_hostile_to_the_int8_copy(vdb, metric):
    """the headline's exactness rests on the int8 pass's certificate, so run it
    at full size on data hostile to the quantisation: heavy-tailed rows; a first add whose mean
    differs from the later adds' (the centring row and the quantisation step come from the
    first add); 24 rows of 1000x the norm in a later add (they clip in the int8 copy and their
    residual enters the bound).  Cosine at C2's shape (1M x 768, B = 64, k = 10: the I8 pass),
    L2 at C4's (10M x 128, B = 512, k = 100: the wide I8Q pass).  Queries: copies of the big
    rows, copies of ordinary rows, heavy-tailed queries from both means.  Every query's list is
    checked for the properties, a spread of queries (the planted ones included) bit-exact
    against the oracle (indices and fp64 keys) on two searches; fallbacks are counted and
    reported (a fallback is exact, only slower)."""
    if metric == "cosine":
        N, D, B, k = 1_000_000, 768, 64, 10
    else:
        N, D, B, k = 10_000_000, 128, 512, 100
    first = N // 16
    V = _hostile_rows(31, N, D)
    V[:first] += np.float32(4.0)  # the first add's mean differs
    rng = np.random.default_rng(32)
    big = (rng.choice(N - first, 24, replace=False) + first).astype(np.int64)
    V[big] *= np.float32(1000.0)
    Q = _hostile_rows(33, B, D)
    Q[: B // 2] += np.float32(4.0)
    plant = {}
    for j in range(8):  # copies of big rows and of ordinary rows, spread over the query blocks
        b = (j * B) // 8
        r = int(big[j]) if j % 2 == 0 else int(rng.integers(0, N))
        Q[b] = V[r]
        plant[b] = r
    ix = vdb.NativeIndex(D, metric)
    ix.reserve(N)
    ix.add(V[:first])
    for s0 in range(first, N, 1 << 21):
        ix.add(V[s0:s0 + (1 << 21)])
    sub = sorted(set(plant) | set(range(1, B, max(1, B // 12))))
    es, ei, ek = ref_cpu.exact_search(Q[sub], V, k, metric)
    fbs, incons = [], []
    for _ in range(2):
        fb0, ic0 = ix.stat("fallback_queries"), ix.stat("inconsistent_queries")
        s, i, kk = ix.search(Q, k, with_keys=True)
        fbs.append(ix.stat("fallback_queries") - fb0)
        incons.append(ix.stat("inconsistent_queries") - ic0)
        _properties(s, i, metric, N)
        for b, r in plant.items():
            assert i[b, 0] == r, (b, r, i[b, :3])
        np.testing.assert_array_equal(i[sub], ei)
        np.testing.assert_array_equal(kk[sub], ek)
    by_prec = {p: ix.stat(f"searches_{p}") for p in ("bf16", "bf16x3", "fp32", "i8", "i8x3", "i8q")}
    _report(f"hostile_{metric}.json", {"rows": N, "dim": D, "batch": B, "k": k, "queries_checked_exactly": len(sub),
                                       "fallback_queries_per_search": fbs, "inconsistent_queries_per_search": incons,
                                       "searches_by_precision": by_prec, "searches_wide": ix.stat("searches_wide")})
    ix.close()


@pytest.mark.timeout(600)
def test_c5_graph_5m_x_384(vdb):
    from performance.hnsw_index import N_ENTRIES, TEAMS
    N, D, k, ef = 5_000_000, 384, 10, 128
    V = np.random.default_rng(7).random((N, D), dtype=np.float32)
    Q = np.random.default_rng(8).random((100, D), dtype=np.float32)
    Q[0] = V[4_999_999]
    ix = vdb.NativeIndex(D, "cosine")
    ix.reserve(N)
    for s0 in range(0, N, 1 << 20):
        ix.add(V[s0:s0 + (1 << 20)])
    t0 = time.perf_counter()
    g = vdb.NativeGraph.build(ix, degree=32, knn=32, n_entries=N_ENTRIES)
    build_s = time.perf_counter() - t0
    g.set_param("teams", TEAMS)
    lab, dist = g.search(Q, k, ef)
    assert (lab >= 0).all() and (lab < N).all()
    assert (np.diff(dist, axis=1) >= 0).all()
    # hnswlib cosine convention: distance = 1 - cos of the returned row (fp32 of the same products)
    for b in range(0, 100, 10):
        ex = ref_cpu.exact_keys(Q[b], V[lab[b]], "cosine")
        np.testing.assert_allclose(dist[b], 1.0 - ex, atol=2e-6, rtol=0)
    assert lab[0, 0] == 4_999_999 and abs(dist[0, 0]) < 1e-5
    _, ei, _ = ref_cpu.exact_search(Q, V, k, "cosine")
    recall = np.mean([len(set(a) & set(b)) / k for a, b in zip(lab.tolist(), ei.tolist())])
    _report("c5.json", {"recall_at_10": recall, "build_s": build_s, "teams": TEAMS, "ef": ef})
    # parity for the graph is recall, not equality.  The build and search are
    # deterministic on this data: rounds 2-4 measured 0.397 at 64 teams over 256 entries
    # (profiles/r0*/reports/c5.json); round 5's store setting (65536 entries, 256 teams) 0.556
    # (profiles/r05_c5); the bar is that minus 0.05, so a regression of the graph shows
    # 
    assert recall >= 0.50, recall
