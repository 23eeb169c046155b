"""The wide int8 pass (vdb_scan8w.hip, round 6): rows of <= 128 dims, batches of more than 256.

All queries of a 512-query block in one workgroup with their int8 tiles in registers, the corpus
staged once through an LDS ring, candidates straight into per-(workgroup, query) segments of the
global lists.  Parity bar as everywhere: indices and fp64 keys bit-exact against
the oracle's exact contract (oracle/ref_cpu.py exact_search), every precision and both metrics,
ragged batches and row counts, masks, several 512-query blocks, and segments that overflow (the
query then takes the exact path, still exact).
"""
import numpy as np
import pytest

from oracle import ref_cpu

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def vdb():
    from service import _vdb
    assert _vdb.device_count() >= 1, "no GPU visible"
    return _vdb


def _words(mask):
    n = mask.size
    bits = np.zeros(((n + 31) // 32) * 32, bool)
    bits[:n] = mask
    return np.packbits(bits, bitorder="little").view("<u4").astype(np.uint32)


def _search_check(ix, Q, V, k, metric, mask=None):
    s, i, kk = ix.search(Q, k, row_mask=_words(mask) if mask is not None else None, with_keys=True)
    es, ei, ek = ref_cpu.exact_search(Q, V, k, metric, row_mask=mask)
    np.testing.assert_array_equal(i, ei)
    valid = ei >= 0
    np.testing.assert_array_equal(kk[valid], ek[valid])
    np.testing.assert_array_equal(s[valid], es[valid])


@pytest.mark.parametrize("precision", ["i8q", "i8x3", "i8", "auto"])
@pytest.mark.parametrize("metric", ["cosine", "euclidean"])
@pytest.mark.parametrize("N,D,B,k", [(20000, 128, 512, 100), (33333, 100, 300, 10), (9001, 65, 257, 50),
                                     (300, 128, 400, 16), (41000, 128, 1100, 100)])
def test_wide_pass_matches_oracle(vdb, metric, precision, N, D, B, k):
    rng = np.random.default_rng(N + D + B)
    V = rng.random((N, D), dtype=np.float32)
    Q = rng.random((B, D), dtype=np.float32)
    Q[0] = V[N // 2]      # an exact duplicate of a row
    Q[B - 1] = V[N - 1]   # the last row (the ragged last tile)
    ix = vdb.NativeIndex(D, metric, precision=precision)
    ix.set_param("scan_wide", 1)
    ix.add(V)
    _search_check(ix, Q, V, k, metric)
    assert ix.stat("searches_wide") == 1
    print(f"{metric} {precision} N {N} D {D} B {B} k {k}: fallbacks {ix.stat('fallback_queries')}"
          f" overflow {ix.stat('overflow_queries')}")
    ix.close()


@pytest.mark.parametrize("metric", ["cosine", "euclidean"])
def test_wide_pass_mask_and_chunked_adds(vdb, metric):
    rng = np.random.default_rng(5)
    N, D = 70_001, 128
    V = rng.standard_normal((N, D)).astype(np.float32)
    Q = rng.standard_normal((520, D)).astype(np.float32)
    ix = vdb.NativeIndex(D, metric)  # auto: the wide pass from 65 536 rows
    for s in range(0, N, 9999):
        ix.add(V[s:s + 9999])
    mask = rng.random(N) < 0.35
    _search_check(ix, Q, V, 100, metric, mask=mask)
    _search_check(ix, Q[:260], V, 10, metric)
    assert ix.stat("searches_wide") == 2
    # the 64-query shape on the same index gives the same results
    ix.set_param("scan_wide", 0)
    _search_check(ix, Q, V, 100, metric, mask=mask)
    assert ix.stat("searches_wide") == 2
    ix.close()


@pytest.mark.parametrize("metric", ["cosine", "euclidean"])
def test_wide_pass_segment_overflow_takes_the_exact_path(vdb, metric):
    """Without a pilot bound every row passes, so every (workgroup, query) segment overflows its
    32 slots: each query must be flagged (overflow) and answered by the exact path."""
    rng = np.random.default_rng(8)
    N, D, B = 30_000, 128, 300
    V = rng.random((N, D), dtype=np.float32)
    Q = rng.random((B, D), dtype=np.float32)
    ix = vdb.NativeIndex(D, metric, precision="i8q")
    ix.set_param("scan_wide", 1)
    ix.set_param("pilot_tiles", 0)
    ix.add(V)
    _search_check(ix, Q, V, 20, metric)
    assert ix.stat("searches_wide") == 1
    assert ix.stat("overflow_queries") == B
    ix.close()


@pytest.mark.parametrize("metric", ["cosine", "euclidean"])
def test_wide_pass_clustered_rows(vdb, metric):
    """A run of near-duplicates added contiguously (one cluster of 4000 rows): the tiles are
    dealt to the workgroups one at a time, so the cluster spreads over the segments."""
    rng = np.random.default_rng(9)
    N, D = 80_000, 128
    V = rng.random((N, D), dtype=np.float32)
    V[40_000:44_000] = (V[17] + 2e-3 * rng.random((4000, D))).astype(np.float32)
    Q = np.concatenate([V[17:18], V[41_000:41_001], rng.random((510, D), dtype=np.float32)])
    ix = vdb.NativeIndex(D, metric)
    ix.add(V)
    _search_check(ix, Q, V, 100, metric)
    assert ix.stat("searches_wide") == 1
    print(f"{metric} clustered: fallbacks {ix.stat('fallback_queries')} overflow {ix.stat('overflow_queries')}")
    ix.close()


def test_wide_pass_device_memory_queued(vdb):
    """Device-memory searches through the wide pass, queued back to back on one stream."""
    import torch
    rng = np.random.default_rng(10)
    N, D, B, k = 100_000, 128, 512, 100
    V = rng.random((N, D), dtype=np.float32)
    Qs = [rng.random((B, D), dtype=np.float32) for _ in range(3)]
    ix = vdb.NativeIndex(D, "euclidean")
    ix.add(V)
    outs = []
    for Q in Qs:
        qd = torch.from_numpy(Q).cuda()
        sd = torch.empty((B, k), dtype=torch.float32, device="cuda")
        idd = torch.empty((B, k), dtype=torch.int64, device="cuda")
        kd = torch.empty((B, k), dtype=torch.float64, device="cuda")
        ix.search_device(qd.data_ptr(), B, k, sd.data_ptr(), idd.data_ptr(), kd.data_ptr(), stream=0)
        outs.append((qd, sd, idd, kd))
    torch.cuda.synchronize()
    for Q, (_, sd, idd, kd) in zip(Qs, outs):
        es, ei, ek = ref_cpu.exact_search(Q, V, k, "euclidean")
        np.testing.assert_array_equal(idd.cpu().numpy(), ei)
        np.testing.assert_array_equal(kd.cpu().numpy(), ek)
    assert ix.stat("searches_wide") == 3
    ix.close()


# ---- the long-row form (vdb_scan8wl.hip): I8 cosine, 512..1536-dim rows, 129..256 queries ----

@pytest.mark.parametrize("precision", ["i8", "auto"])
@pytest.mark.parametrize("N,D,B,k", [(20000, 1536, 256, 10), (33333, 1500, 200, 10), (9001, 1024, 129, 50),
                                     (300, 768, 256, 16), (41000, 512, 256, 100), (70001, 1536, 256, 10)])
def test_wide_long_pass_matches_oracle(vdb, precision, N, D, B, k):
    rng = np.random.default_rng(N + D + B + 7)
    V = rng.random((N, D), dtype=np.float32)
    Q = rng.random((B, D), dtype=np.float32)
    Q[0] = V[N // 2]
    Q[B - 1] = V[N - 1]
    ix = vdb.NativeIndex(D, "cosine", precision=precision)
    ix.set_param("scan_wide", 1)
    ix.add(V)
    _search_check(ix, Q, V, k, "cosine")
    wide = ix.stat("searches_wide")
    i8 = ix.stat("searches_i8")
    print(f"long D {D} B {B} k {k} {precision}: wide {wide} i8 {i8} fallbacks {ix.stat('fallback_queries')}"
          f" overflow {ix.stat('overflow_queries')}")
    if precision == "i8":
        assert wide == 1
    ix.close()


def test_wide_long_pass_mask_overflow_and_clusters(vdb):
    rng = np.random.default_rng(21)
    N, D, B = 80_000, 1536, 256
    V = rng.random((N, D), dtype=np.float32)
    V[40_000:44_000] = (V[17] + 2e-3 * rng.random((4000, D))).astype(np.float32)  # one cluster of near-duplicates
    Q = np.concatenate([V[17:18], V[41_000:41_001], rng.random((B - 2, D), dtype=np.float32)])
    ix = vdb.NativeIndex(D, "cosine", precision="i8")  # auto rows threshold: the wide pass from 65 536 rows
    for s in range(0, N, 25_000):
        ix.add(V[s:s + 25_000])
    _search_check(ix, Q, V, 10, "cosine")
    mask = rng.random(N) < 0.4
    _search_check(ix, Q, V, 10, "cosine", mask=mask)
    assert ix.stat("searches_wide") == 2
    # without a pilot bound every segment overflows: every query takes the exact path (still exact)
    ix.set_param("pilot_tiles", 0)
    _search_check(ix, Q[:150], V, 10, "cosine")
    assert ix.stat("searches_wide") == 3 and ix.stat("overflow_queries") >= 150
    # the 64-query shape on the same index gives the same results
    ix.set_param("pilot_tiles", -1)
    ix.set_param("scan_wide", 0)
    _search_check(ix, Q, V, 10, "cosine", mask=mask)
    assert ix.stat("searches_wide") == 3
    ix.close()


@pytest.mark.parametrize("B", [1, 2, 5, 8, 16, 33, 64, 100])
@pytest.mark.parametrize("D", [768, 1536, 1000, 512])
def test_wide_long_pass_small_batches_under_auto(vdb, B, D):
    """Auto takes the long-row wide pass from 65 536 rows for every batch of rows of <= 1024 dims
    (two waves per query tile up to 128 queries) and for batches of <= 16 / > 96 at 1536 dims:
    C2's batches and the serving path's single queries."""
    rng = np.random.default_rng(B * 7 + D)
    N = 66_000
    V = rng.random((N, D), dtype=np.float32)
    Q = rng.random((B, D), dtype=np.float32)
    Q[0] = V[12_345]
    ix = vdb.NativeIndex(D, "cosine")
    ix.add(V)
    _search_check(ix, Q, V, 10, "cosine")
    G8 = ((D + 63) // 64 * 64) // 32
    expect = G8 in (16, 24, 32, 48) and (G8 <= 32 or B <= 16 or B > 96) and ix.stat("searches_i8") == 1
    assert ix.stat("searches_wide") == (1 if expect else 0)
    ix.close()


@pytest.mark.parametrize("small", [0, 1])
@pytest.mark.parametrize("N,D,B,k", [(70_001, 768, 64, 10), (66_000, 1000, 8, 10), (70_000, 512, 120, 50)])
def test_finish_small_form_matches_oracle(vdb, small, N, D, B, k):
    """The finish's 4-wave form (4096-entry buffer) beside the long-row wide scan, and the
    16-wave form, give the same exact results; a list past 4096 entries (no pilot bound) goes to
    the exact path."""
    rng = np.random.default_rng(N + D + small)
    V = rng.random((N, D), dtype=np.float32)
    Q = rng.random((B, D), dtype=np.float32)
    Q[0] = V[7]
    ix = vdb.NativeIndex(D, "cosine", precision="i8")
    ix.set_param("scan_wide", 1)
    ix.set_param("finish_small", small)
    ix.add(V)
    _search_check(ix, Q, V, k, "cosine")
    ix.set_param("pilot_tiles", 0)  # every row passes: segments overflow (exact path, still exact)
    _search_check(ix, Q, V, k, "cosine")
    assert ix.stat("overflow_queries") >= B
    ix.close()


@pytest.mark.parametrize("metric,precision", [("cosine", "i8"), ("euclidean", "i8q"), ("euclidean", "i8x3")])
@pytest.mark.parametrize("B", [1, 37, 64, 100, 200, 256])
def test_wide_pass_small_batches_split_tiles(vdb, metric, precision, B):
    """The short-row wide pass forced on for batches of <= 256: rw = 8 / 4 / 2 waves per 64-query
    block share each stage's tiles, their segment counters and checksum words in LDS."""
    rng = np.random.default_rng(B + len(metric) + len(precision))
    N, D, k = 40_003, 128, 20
    V = rng.random((N, D), dtype=np.float32)
    Q = rng.random((B, D), dtype=np.float32)
    Q[0] = V[N - 1]
    ix = vdb.NativeIndex(D, metric, precision=precision)
    ix.set_param("scan_wide", 1)
    ix.add(V)
    _search_check(ix, Q, V, k, metric)
    mask = rng.random(N) < 0.5
    _search_check(ix, Q, V, k, metric, mask=mask)
    assert ix.stat("searches_wide") == 2
    assert ix.stat("inconsistent_queries") == 0
    ix.close()
