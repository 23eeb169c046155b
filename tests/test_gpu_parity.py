"""Parity of the gfx950 path (through the C-ABI) against the CPU oracle.

Bar: indices bit-exact against the exact contract (fp64 keys in
the canonical order, ties to the lower row), fp64 keys bit-exact, returned fp32
scores within 1e-4 of the reference's own fp32 arithmetic.
"""
import glob
import os

import numpy as np
import pytest

from oracle import ref_cpu

pytestmark = pytest.mark.gpu

GOLDEN = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "*.npz")))


@pytest.fixture(scope="module")
def vdb():
    from service import _vdb
    assert _vdb.device_count() >= 1, "no GPU visible"
    return _vdb


def _mask_words(mask_bool):
    n = mask_bool.size
    bits = np.zeros(((n + 31) // 32) * 32, bool)
    bits[:n] = mask_bool
    return np.packbits(bits, bitorder="little").view("<u4").astype(np.uint32)


PRECISIONS = ["bf16x3", "bf16", "fp32", "auto", "i8", "i8x3", "i8q"]


def _check(vdb, V, Q, k, metric, mask=None, force_exact=False, margin=None, chunked_add=False, precision="bf16x3",
           params=None):
    ix = vdb.NativeIndex(V.shape[1], metric, precision=precision)
    for name, value in (params or {}).items():
        ix.set_param(name, value)
    if force_exact:
        ix.set_param("force_exact", 1)
    if margin is not None:
        ix.set_param("margin", margin)
    if chunked_add:
        for s in range(0, V.shape[0], 777):
            ix.add(V[s:s + 777])
    else:
        ix.add(V)
    assert ix.count() == V.shape[0]
    mw = _mask_words(mask) if mask is not None else None
    s, i, kk = ix.search(Q, k, row_mask=mw, with_keys=True)
    es, ei, ek = ref_cpu.exact_search(Q, V, k, metric, row_mask=mask)
    np.testing.assert_array_equal(i, ei)
    valid = ei >= 0
    # fp64 keys: bit-exact with the canonical order
    np.testing.assert_array_equal(kk[valid], ek[valid])
    np.testing.assert_array_equal(s[valid], es[valid])
    return ix, s, i


@pytest.mark.parametrize("precision", PRECISIONS)
@pytest.mark.parametrize("path", GOLDEN, ids=[os.path.basename(p) for p in GOLDEN])
def test_golden_fixtures(vdb, path, precision):
    z = np.load(path, allow_pickle=False)
    V, Q, k, metric = z["vectors"], z["queries"], int(z["k"]), str(z["metric"])
    mask = z["mask"] if z["mask"].size else None
    ix = vdb.NativeIndex(V.shape[1], metric, precision=precision)
    ix.add(V)
    s, i, kk = ix.search(Q, k, row_mask=_mask_words(mask) if mask is not None else None, with_keys=True)
    np.testing.assert_array_equal(i, z["exact_idx"])
    valid = i >= 0
    np.testing.assert_array_equal(kk[valid], z["exact_keys"][valid])
    # scores vs the reference's fp32 arithmetic, same rows
    np.testing.assert_allclose(s[valid], z["ref_scores"][valid], atol=1e-4, rtol=0)


@pytest.mark.parametrize("precision", PRECISIONS)
@pytest.mark.parametrize("metric", ["cosine", "euclidean"])
@pytest.mark.parametrize("N,D,B,k", [(5000, 384, 7, 10), (3000, 100, 3, 5), (4096, 128, 64, 100),
                                     (1234, 33, 65, 32), (700, 1536, 9, 10), (20000, 768, 130, 10),
                                     (9000, 64, 40, 200), (2500, 1100, 17, 150)])
def test_random_uniform(vdb, metric, N, D, B, k, precision):
    rng = np.random.default_rng(N + D)
    V = rng.random((N, D), dtype=np.float32)
    Q = rng.random((B, D), dtype=np.float32)
    _check(vdb, V, Q, k, metric, precision=precision)


@pytest.mark.parametrize("precision", PRECISIONS)
@pytest.mark.parametrize("metric", ["cosine", "euclidean"])
def test_normal_with_mask_and_chunked_add(vdb, metric, precision):
    rng = np.random.default_rng(7)
    V = rng.standard_normal((6000, 200)).astype(np.float32)
    Q = rng.standard_normal((5, 200)).astype(np.float32)
    mask = rng.random(6000) < 0.3
    _check(vdb, V, Q, 10, metric, mask=mask, chunked_add=True, precision=precision)


@pytest.mark.parametrize("split", [2, 4])
@pytest.mark.parametrize("metric", ["cosine", "euclidean"])
def test_finish_split(vdb, split, metric):
    """The finish kernel with several workgroups per query (index param finish_split): the
    shares of the exact rerank are merged by the last workgroup; same results."""
    rng = np.random.default_rng(split)
    V = rng.random((30000, 200), dtype=np.float32)
    Q = rng.random((40, 200), dtype=np.float32)
    _check(vdb, V, Q, 25, metric, params={"finish_split": split})
    _check(vdb, V, Q, 25, metric, precision="bf16", params={"finish_split": split})
    _check(vdb, V, Q, 25, metric, precision="i8", params={"finish_split": split})


@pytest.mark.parametrize("split,D", [(1, 1090), (3, 1090), (1, 1024), (1, 1025)])
@pytest.mark.parametrize("metric", ["cosine", "euclidean"])
def test_finish_long_rows(vdb, split, D, metric):
    """Rows of more than 1024 dims take the 8-wave finish (vdb_exact.hip, launch_finish): ragged
    D = 1090 at KP 64 / 256 (k 25 / 120), alone and split across workgroups, and both sides of
    the switch (1024: 16 waves, 1025: 8)."""
    rng = np.random.default_rng(D + split)
    V = rng.standard_normal((6000, D)).astype(np.float32)
    Q = rng.standard_normal((24, D)).astype(np.float32)
    for k in (25, 120):
        _check(vdb, V, Q, k, metric, params={"finish_split": split})
        _check(vdb, V, Q, k, metric, precision="i8", params={"finish_split": split})


@pytest.mark.parametrize("precision", ["bf16x3", "i8", "i8x3"])
@pytest.mark.parametrize("sync", [1, 2])
@pytest.mark.parametrize("metric", ["cosine", "euclidean"])
@pytest.mark.parametrize("D,B,k", [(128, 150, 100), (384, 70, 10), (1536, 40, 10)])
def test_scan_step_sync_modes(vdb, sync, metric, D, B, k, precision):
    """Both step ends of the scan (lockstep barrier / flag-gated compaction rounds,
    vdb_scan.hip) on data that keeps every workgroup's buffers overflowing: rows
    approach the queries' direction as the row index grows, so each step beats the
    last and compaction rounds run all the way to the end of the row range."""
    rng = np.random.default_rng(D + sync)
    N = 60000
    Q = rng.random((B, D), dtype=np.float32)
    t = (np.arange(N, dtype=np.float32) / N)[:, None]
    V = (Q[rng.integers(0, B, N)] * t + rng.random((N, D), dtype=np.float32) * (1.0 - t)).astype(np.float32)
    ix, _, _ = _check(vdb, V, Q, k, metric, precision=precision, params={"scan_sync": sync})
    with pytest.raises(Exception):
        ix.set_param("scan_sync", 3)


def test_precision_switch_keeps_results(vdb):
    """Switching the candidate-pass arithmetic after ingest builds / drops the split
    copy; results stay identical (the exact rerank decides)."""
    rng = np.random.default_rng(21)
    V = rng.random((7000, 160), dtype=np.float32) * 100.0 - 30.0
    Q = rng.random((9, 160), dtype=np.float32) * 100.0 - 30.0
    ix = vdb.NativeIndex(160, "euclidean", precision="fp32")
    ix.add(V[:3000])
    ix.set_precision("bf16x3")
    ix.add(V[3000:])
    a = ix.search(Q, 17, with_keys=True)
    ix.set_precision("fp32")
    b = ix.search(Q, 17, with_keys=True)
    ix.set_precision("bf16")
    c = ix.search(Q, 17, with_keys=True)
    ix.set_precision("i8")
    d = ix.search(Q, 17, with_keys=True)
    ix.set_precision("i8x3")
    e = ix.search(Q, 17, with_keys=True)
    ix.set_precision("bf16")
    f = ix.search(Q, 17, with_keys=True)
    es, ei, ek = ref_cpu.exact_search(Q, V, 17, "euclidean")
    for s, i, kk in (a, b, c, d, e, f):
        np.testing.assert_array_equal(i, ei)
        np.testing.assert_array_equal(kk, ek)
    assert ix.stat("fallback_queries") == 0


@pytest.mark.parametrize("precision", ["bf16", "i8"])
@pytest.mark.parametrize("metric", ["cosine", "euclidean"])
def test_bf16_directional_residual_bound(vdb, metric, precision):
    """bf16 certificate with the corpus-rounding bound taken along the rows' mean direction
    (|q - c dir| R + |c| M): on uniform rows (one shared direction) it certifies the queries
    that Cauchy-Schwarz's |q| R leaves uncertified; results are exact either way."""
    rng = np.random.default_rng(41)
    N, D, B, k = 300_000, 1536, 32, 10
    V = rng.random((N, D), dtype=np.float32)
    Q = rng.random((B, D), dtype=np.float32)
    es, ei, ek = ref_cpu.exact_search(Q, V, k, metric)
    fb = {}
    for dirb in (1, 0):
        ix = vdb.NativeIndex(D, metric, precision=precision)
        ix.set_param("dir_bound", dirb)
        ix.add(V)
        s, i, kk = ix.search(Q, k, with_keys=True)
        np.testing.assert_array_equal(i, ei)
        np.testing.assert_array_equal(kk, ek)
        fb[dirb] = ix.stat("fallback_queries")
        ix.close()
    print(f"{metric}: {precision} fallbacks with the directional bound {fb[1]}, Cauchy-Schwarz {fb[0]} of {B}")
    assert fb[1] <= fb[0], fb
    if metric == "cosine" and precision == "bf16":  # (1M x 1536, B = 256: 0 vs every query,
        assert fb[1] == 0, fb                          # profiles/r02s_ab/s4_c3_bf16*.json)
    # i8 (8-bit query: a wider bound) leaves a few of these 1536-dim queries to auto's re-pass


@pytest.mark.parametrize("qlds", [-1, 0, 2])
@pytest.mark.parametrize("D", [192, 320])
@pytest.mark.parametrize("metric", ["cosine", "euclidean"])
@pytest.mark.parametrize("precision", ["i8", "i8x3"])
def test_i8_group_counts_not_a_multiple_of_the_prefetch(vdb, precision, metric, D, qlds):
    """Dp / 32 groups is only even (D = 192: 6, D = 320: 10): the int8 passes that keep 4 groups
    in flight cannot step through them, and the launcher falls back to 2 (4 deep, the step's tail
    would read the next row tile's groups into the scores).  With no_fallback the candidate pass
    alone must certify and order every query, with the query block in LDS (-1) and from L2 (0)."""
    rng = np.random.default_rng(D + 5)
    V = rng.random((6000, D), dtype=np.float32)
    Q = rng.random((24, D), dtype=np.float32)
    _check(vdb, V, Q, 10, metric, precision=precision, params={"no_fallback": 1, "scan_qlds": qlds})


@pytest.mark.parametrize("qlds", [1, 2])
@pytest.mark.parametrize("D,B,k", [(768, 64, 10), (1536, 150, 10), (768, 100, 40), (384, 64, 100), (1000, 70, 3)])
@pytest.mark.parametrize("metric", ["cosine", "euclidean"])
@pytest.mark.parametrize("precision", ["i8", "i8x3"])
def test_i8_query_block_in_lds_whenever_it_fits(vdb, precision, metric, D, B, k, qlds):
    """scan_qlds 2: the query block sits in LDS whenever it fits beside the lists (I8 keeps
    the qh plane alone: 64 x 1536 B = 96 KiB beside 56.5 KiB of lists at KP = 256), against
    the round-3 rule (1: short rows only).  Exact either way; the fallback counts are printed."""
    rng = np.random.default_rng(D + B + k)
    V = rng.random((9000, D), dtype=np.float32)
    V[4000:4003] = V[7]
    Q = rng.random((B, D), dtype=np.float32)
    Q[1] = V[7]
    ix, _, _ = _check(vdb, V, Q, k, metric, precision=precision, params={"scan_qlds": qlds})
    print(f"{precision} {metric} D {D} B {B} k {k} qlds {qlds}: fallbacks {ix.stat('fallback_queries')}")


@pytest.mark.parametrize("refine", [-1, 0, 1])
@pytest.mark.parametrize("D,B,k", [(96, 40, 10), (128, 64, 100), (384, 33, 10), (768, 64, 10), (1536, 20, 25)])
@pytest.mark.parametrize("metric", ["cosine", "euclidean"])
def test_i8_refinement_modes(vdb, metric, D, B, k, refine):
    """The finish's I8 refinement (index param i8_refine: -1 auto = rows of 512 padded dims or
    more, 0 off, 1 on) on both sides of the auto rule, with duplicate rows and a query equal to
    a row (ties at the cut): exact either way."""
    rng = np.random.default_rng(D + B + k + refine)
    V = rng.random((12000, D), dtype=np.float32)
    V[5000:5004] = V[11]
    Q = rng.random((B, D), dtype=np.float32)
    Q[2] = V[11]
    ix, _, _ = _check(vdb, V, Q, k, metric, precision="i8", params={"i8_refine": refine})
    with pytest.raises(Exception):
        ix.set_param("i8_refine", 2)


def _auto_index(vdb, D, a8):
    """An auto-precision index with (a8 = 1, the default) or without the int8 copy: its
    one-plane pass is I8 (BF16 during an I8 hold) or BF16; the x3 pass of holds, re-passes and
    retries is BF16X3 either way (k > 16 runs I8X3 with the int8 copy: the test below).
    Returns it and the stat names of its one-plane / x3 passes."""
    ix = vdb.NativeIndex(D, "cosine")
    ix.set_param("auto_int8", a8)
    assert ix.precision == "auto" and ix.stat("auto_int8") == a8
    return ix, ("searches_i8" if a8 else "searches_bf16", "searches_bf16x3")


@pytest.mark.parametrize("a8", [1, 0])
@pytest.mark.parametrize("mem", ["host", "device"])
def test_auto_precision_switches_on_fallbacks(vdb, mem, a8):
    """VDB_PREC_AUTO runs the bf16 pass while it certifies; rows closer together than the
    bf16 residual bound leave most queries uncertified, after which the index runs bf16x3
    until its rows change (host memory: the batch itself is rerun in bf16x3; device memory:
    it falls back, and the switch happens once the earlier search's counts have landed)."""
    import torch
    rng = np.random.default_rng(31)
    D, N, B, k = 256, 8000, 32, 10
    far = rng.random((N, D), dtype=np.float32)
    base = rng.random(D, dtype=np.float32)
    near = (base + 1e-4 * rng.standard_normal((N, D))).astype(np.float32)
    for V, expect_switch in ((far, False), (near, True)):
        Q = (V[rng.integers(0, N, B)] + 1e-5 * rng.standard_normal((B, D))).astype(np.float32)
        ix, (one, x3) = _auto_index(vdb, D, a8)
        ix.add(V)
        es, ei, ek = ref_cpu.exact_search(Q, V, k, "cosine")
        for _ in range(2):
            if mem == "host":
                s, i, kk = ix.search(Q, k, with_keys=True)
            else:
                qd = torch.from_numpy(Q).cuda()
                sd = torch.empty((B, k), dtype=torch.float32, device="cuda")
                idd = torch.empty((B, k), dtype=torch.int64, device="cuda")
                kd = torch.empty((B, k), dtype=torch.float64, device="cuda")
                ix.search_device(qd.data_ptr(), B, k, sd.data_ptr(), idd.data_ptr(), kd.data_ptr(), stream=0)
                torch.cuda.synchronize()
                i, kk = idd.cpu().numpy(), kd.cpu().numpy()
            np.testing.assert_array_equal(i, ei)
            np.testing.assert_array_equal(kk, ek)
        assert ix.stat(one) >= 1
        if expect_switch:
            assert ix.stat("fallback_queries") * 64 > B  # the x3 pass cannot separate these rows either
            if a8:
                # the I8 failure holds BF16 (host: the batch is rerun in BF16X3 at once); the
                # second search runs BF16, fails too and (host) reruns in BF16X3; (device) the
                # first failure seen also arms the device re-pass, so the second search re-passes
                # 16 of its uncertified queries in a BF16X3 sub-search (the rest: the exact path)
                assert ix.stat("searches_bf16") == 1
                assert ix.stat(x3) == (2 if mem == "host" else 0)  # (device re-pass: not a search)
                if mem == "device":
                    assert ix.stat("repass_queries") == 16, ix.stat("repass_queries")
            else:
                # host memory: the uncertified one-plane pass is rerun at once in x3, then the second
                # search runs x3; device memory: the first search falls back, the second runs x3
                assert ix.stat(x3) == (2 if mem == "host" else 1)
            assert ix.stat(one) == 1
            ix.add(V[:1])  # new rows: the one-plane pass gets another chance
            ix.search(Q, k)
            assert ix.stat(one) == 2
        else:
            assert ix.stat(x3) == 0 and ix.stat("fallback_queries") == 0


@pytest.mark.parametrize("a8", [1, 0])
def test_auto_repass_keeps_bf16_for_a_few_uncertified_queries(vdb, a8):
    """One near-duplicate query in a batch of ordinary ones: its bf16 certificate fails, it
    alone is re-passed in bf16x3 (host memory), and the index stays bf16: the next batch
    runs bf16 again (one query no longer pins the index to bf16x3)."""
    rng = np.random.default_rng(41)
    D, N, B, k = 256, 20000, 32, 10
    V = rng.random((N, D), dtype=np.float32)
    base = rng.random(D, dtype=np.float32)
    V[:400] = (base + 1e-4 * rng.standard_normal((400, D))).astype(np.float32)  # a tight cluster
    Q = rng.random((B, D), dtype=np.float32)
    Q[7] = base  # the near-duplicate query: its top-10 sit inside the cluster
    ix, (one, x3) = _auto_index(vdb, D, a8)
    ix.add(V)
    es, ei, ek = ref_cpu.exact_search(Q, V, k, "cosine")
    for _ in range(3):
        s, i, kk = ix.search(Q, k, with_keys=True)
        np.testing.assert_array_equal(i, ei)
        np.testing.assert_array_equal(kk, ek)
    assert ix.stat("searches") == 3 and ix.stat("queries") == 3 * B
    assert ix.stat("repass_queries") >= 3  # query 7, every search
    assert ix.stat(one) == 3  # never switched
    assert ix.stat("auto_hold") == 0


def test_auto_hold8_holds_bf16_until_the_rows_change(vdb):
    """With the int8 copy, an I8 failure too large for a re-pass holds BF16 (the split copy) for
    16 searches instead of dropping to an x3 pass; new rows end the hold."""
    rng = np.random.default_rng(43)
    D, N, B, k = 128, 6000, 16, 10
    base = rng.random(D, dtype=np.float32)
    near = (base + 1e-4 * rng.standard_normal((N, D))).astype(np.float32)
    Q = (near[rng.integers(0, N, B)] + 1e-5 * rng.standard_normal((B, D))).astype(np.float32)
    ix, (one, x3) = _auto_index(vdb, D, 1)
    ix.add(near)
    es, ei, ek = ref_cpu.exact_search(Q, near, k, "cosine")
    s, i, kk = ix.search(Q, k, with_keys=True)  # I8 fails for most queries -> rerun in BF16X3
    np.testing.assert_array_equal(i, ei)
    assert ix.stat("searches_i8") == 1 and ix.stat("auto_hold8") == 16
    s, i, kk = ix.search(Q, k, with_keys=True)  # the hold: BF16
    np.testing.assert_array_equal(kk, ek)
    assert ix.stat("searches_i8") == 1 and ix.stat("searches_bf16") == 1 and ix.stat("auto_hold8") == 15
    ix.add(near[:1])  # new rows: I8 again
    assert ix.stat("auto_hold8") == 0
    ix.search(Q, k)
    assert ix.stat("searches_i8") == 2


def test_auto_l2_k_above_16_runs_i8q_and_turns_it_off_after_a_failure(vdb):
    """L2 with 16 < k <= 100: auto's pass is I8Q (the int8 copy's xh plane against the 16-bit
    query, KP = 256), exact through the certificate.  Rows its 8-bit corpus cannot separate (two
    tight clusters far apart: one quantisation step spans a cluster) leave most queries
    uncertified: the batch takes the exact path and the index runs I8X3 from then on (i8q_off)."""
    rng = np.random.default_rng(53)
    D, N, B, k = 128, 6000, 16, 40
    V = rng.random((N, D), dtype=np.float32)
    Q = rng.random((B, D), dtype=np.float32)
    ix = vdb.NativeIndex(D, "euclidean")
    assert ix.stat("auto_i8q") == 1
    ix.add(V)
    es, ei, ek = ref_cpu.exact_search(Q, V, k, "euclidean")
    s, i, kk = ix.search(Q, k, with_keys=True)
    np.testing.assert_array_equal(i, ei)
    np.testing.assert_array_equal(kk, ek)
    assert ix.stat("searches_i8q") == 1 and ix.stat("searches_i8x3") == 0
    assert ix.stat("fallback_queries") == 0 and ix.stat("i8q_off") == 0
    s, i, kk = ix.search(Q, 120, with_keys=True)  # k > 100: I8X3
    assert ix.stat("searches_i8x3") == 1
    ix.close()

    b1, b2 = rng.random(D, dtype=np.float32), rng.random(D, dtype=np.float32)
    side = rng.random(N) < 0.5
    V = (np.where(side[:, None], b1, b2) + 1e-5 * rng.standard_normal((N, D))).astype(np.float32)
    Q = (V[rng.integers(0, N, B)] + 1e-6 * rng.standard_normal((B, D))).astype(np.float32)
    ix = vdb.NativeIndex(D, "euclidean")
    ix.add(V)
    es, ei, ek = ref_cpu.exact_search(Q, V, k, "euclidean")
    s, i, kk = ix.search(Q, k, with_keys=True)
    np.testing.assert_array_equal(i, ei)
    np.testing.assert_array_equal(kk, ek)
    assert ix.stat("searches_i8q") == 1 and ix.stat("fallback_queries") > B // 8
    assert ix.stat("i8q_off") == 1
    s, i, kk = ix.search(Q, k, with_keys=True)
    np.testing.assert_array_equal(kk, ek)
    assert ix.stat("searches_i8q") == 1 and ix.stat("searches_i8x3") + ix.stat("searches_bf16x3") >= 1
    ix.close()


def test_auto_k_above_16_runs_i8x3_and_holds_bf16x3_after_a_failure(vdb):
    """With the int8 copy, auto's k > 16 pass is I8X3 (exact results through the certificate);
    rows the 16-bit planes cannot separate -- two tight clusters far apart, so the one
    quantisation step is set by the clusters' distance -- leave most queries uncertified: the
    batch falls back to the exact path and the index holds BF16X3 for the next 16 searches."""
    rng = np.random.default_rng(47)
    D, N, B, k = 128, 6000, 16, 40
    V = rng.random((N, D), dtype=np.float32)
    Q = rng.random((B, D), dtype=np.float32)
    ix, _ = _auto_index(vdb, D, 1)
    ix.add(V)
    es, ei, ek = ref_cpu.exact_search(Q, V, k, "cosine")
    s, i, kk = ix.search(Q, k, with_keys=True)
    np.testing.assert_array_equal(i, ei)
    np.testing.assert_array_equal(kk, ek)
    assert ix.stat("searches_i8x3") == 1 and ix.stat("searches_bf16x3") == 0
    assert ix.stat("fallback_queries") == 0 and ix.stat("auto_hold8") == 0
    ix.close()

    b1, b2 = rng.random(D, dtype=np.float32), rng.random(D, dtype=np.float32)
    side = rng.random(N) < 0.5
    V = (np.where(side[:, None], b1, b2) + 1e-5 * rng.standard_normal((N, D))).astype(np.float32)
    Q = (V[rng.integers(0, N, B)] + 1e-6 * rng.standard_normal((B, D))).astype(np.float32)
    ix, _ = _auto_index(vdb, D, 1)
    ix.add(V)
    es, ei, ek = ref_cpu.exact_search(Q, V, k, "cosine")
    s, i, kk = ix.search(Q, k, with_keys=True)
    np.testing.assert_array_equal(i, ei)
    np.testing.assert_array_equal(kk, ek)
    assert ix.stat("searches_i8x3") == 1 and ix.stat("fallback_queries") > B // 8
    assert ix.stat("auto_hold8") == 16
    s, i, kk = ix.search(Q, k, with_keys=True)  # the hold: BF16X3
    np.testing.assert_array_equal(kk, ek)
    assert ix.stat("searches_i8x3") == 1 and ix.stat("searches_bf16x3") == 1 and ix.stat("auto_hold8") == 15
    ix.add(V[:1])  # new rows end the hold
    assert ix.stat("auto_hold8") == 0
    ix.search(Q, k)
    assert ix.stat("searches_i8x3") == 2
    ix.close()


@pytest.mark.parametrize("a8", [1, 0])
def test_auto_hold_expires(vdb, a8):
    """A failure too large for a re-pass starts a hold of 16 bf16x3 searches; after it the
    index probes the one-plane pass again (and, on data that still fails, holds twice as long).
    With the int8 copy (a8) the x3 hold is reached through BF16: the first search's I8 failure
    holds BF16, whose own failure starts the x3 hold."""
    rng = np.random.default_rng(43)
    D, N, B, k = 128, 6000, 16, 10
    base = rng.random(D, dtype=np.float32)
    near = (base + 1e-4 * rng.standard_normal((N, D))).astype(np.float32)
    Q = (near[rng.integers(0, N, B)] + 1e-5 * rng.standard_normal((B, D))).astype(np.float32)
    ix, (one, x3) = _auto_index(vdb, D, a8)
    ix.add(near)
    es, ei, ek = ref_cpu.exact_search(Q, near, k, "cosine")
    if a8:  # I8 fails -> BF16 hold; then the BF16 pass is the one-plane pass probed below
        s, i, kk = ix.search(Q, k, with_keys=True)
        np.testing.assert_array_equal(i, ei)
        assert ix.stat("searches_i8") == 1 and ix.stat("auto_hold8") == 16
        one = "searches_bf16"
    s, i, kk = ix.search(Q, k, with_keys=True)  # one-plane fails for most queries -> rerun in x3
    np.testing.assert_array_equal(i, ei)
    assert ix.stat(one) == 1 and ix.stat("auto_hold") == 16
    for _ in range(16):
        s, i, kk = ix.search(Q, k, with_keys=True)
        np.testing.assert_array_equal(kk, ek)
    assert ix.stat(one) == 1 and ix.stat("auto_hold") == 0
    s, i, kk = ix.search(Q, k, with_keys=True)  # the probe: one-plane again, fails again -> hold 32
    np.testing.assert_array_equal(i, ei)
    assert ix.stat(one) == 2 and ix.stat("auto_hold") == 32
    n = 18 + a8
    assert ix.stat("searches") == n and ix.stat("queries") == n * B


def test_duplicates_force_certificate_fallback(vdb):
    """50 copies of the nearest row: the candidate list cannot certify the top-k,
    so the exact scan must take over and keep the lower-index-first order."""
    rng = np.random.default_rng(3)
    V = rng.random((20000, 64), dtype=np.float32)
    V[1000:1050] = V[7]
    Q = np.stack([V[7], rng.random(64, dtype=np.float32)])
    ix, s, i = _check(vdb, V, Q, 10, "cosine")
    assert i[0, 0] == 7 and list(i[0, 1:]) == list(range(1000, 1009))
    assert ix.stat("fallback_queries") >= 1


@pytest.mark.parametrize("metric", ["cosine", "euclidean"])
def test_exact_path_large_k(vdb, metric):
    rng = np.random.default_rng(11)
    V = rng.random((9000, 96), dtype=np.float32)
    Q = rng.random((3, 96), dtype=np.float32)
    _check(vdb, V, Q, 300, metric)          # k > 200 -> exact path
    _check(vdb, V, Q, 10, metric, force_exact=True)


def test_k_larger_than_n_and_tiny(vdb):
    rng = np.random.default_rng(5)
    V = rng.random((7, 16), dtype=np.float32)
    Q = rng.random((2, 16), dtype=np.float32)
    ix, s, i = _check(vdb, V, Q, 20, "cosine")
    assert (i[:, 7:] == -1).all() and (i[:, :7] >= 0).all()


def test_empty_index_returns_no_results(vdb):
    ix = vdb.NativeIndex(8, "cosine")
    s, i = ix.search(np.ones((3, 8), np.float32), 5)
    assert (i == -1).all()


def test_nonfinite_rejected(vdb):
    ix = vdb.NativeIndex(4, "cosine")
    bad = np.ones((3, 4), np.float32)
    bad[1, 2] = np.nan
    with pytest.raises(ValueError):
        ix.add(bad)
    assert ix.count() == 0
    ix.add(np.ones((2, 4), np.float32))
    with pytest.raises(ValueError):
        ix.search(np.full((1, 4), np.inf, np.float32), 1)


@pytest.mark.parametrize("metric", ["cosine", "euclidean"])
@pytest.mark.parametrize("precision", ["i8", "i8x3", "auto"])
def test_rejected_add_leaves_no_trace(vdb, metric, precision):
    """an add rejected for a NaN row after good rows must leave the int8 copy's
    column sums (the pass's checksum) and the row statistics as they were: the next searches
    certify in the int8 pass with no flagged / inconsistent query, and stay exact after a
    further good add."""
    from oracle import ref_cpu
    rng = np.random.default_rng(41)
    D = 96
    V = rng.random((6000, D), dtype=np.float32)
    Q = rng.random((16, D), dtype=np.float32)
    ix = vdb.NativeIndex(D, metric, precision=precision)
    ix.add(V[:4000])
    bad = rng.random((500, D), dtype=np.float32) * 50.0  # large rows: they would raise the maxima
    bad[321, 7] = np.nan
    with pytest.raises(ValueError):
        ix.add(bad)
    assert ix.count() == 4000
    for rows in (4000, 6000):
        if rows == 6000:
            ix.add(V[4000:])
        _, i, kk = ix.search(Q, 10, with_keys=True)
        _, ei, ek = ref_cpu.exact_search(Q, V[:rows], 10, metric)
        np.testing.assert_array_equal(i, ei)
        np.testing.assert_array_equal(kk, ek)
    assert ix.stat("inconsistent_queries") == 0
    assert ix.stat("fallback_queries") == 0
    ix.close()


def test_export_roundtrip(vdb):
    rng = np.random.default_rng(9)
    V = rng.standard_normal((1000, 77)).astype(np.float32)
    ix = vdb.NativeIndex(77, "euclidean")
    ix.add(V[:300])
    ix.add(V[300:])
    np.testing.assert_array_equal(ix.get_vectors(), V)
    ix.clear()
    assert ix.count() == 0
    ix.add(V[:10])
    np.testing.assert_array_equal(ix.get_vectors(), V[:10])


def test_merge_topk_matches_single_device(vdb):
    """Shard a corpus in 4, search shards with index offsets, merge on device:
    identical to one search over everything."""
    import torch
    rng = np.random.default_rng(13)
    V = rng.random((8000, 128), dtype=np.float32)
    V[5000:5020] = V[123]  # ties across shards
    Q = rng.random((16, 128), dtype=np.float32)
    Q[0] = V[123]
    k, G = 25, 4
    bounds = np.linspace(0, V.shape[0], G + 1).astype(int)
    keys, idx = [], []
    for g in range(G):
        ix = vdb.NativeIndex(128, "euclidean")
        ix.add(V[bounds[g]:bounds[g + 1]])
        _, i, kk = ix.search(Q, k, with_keys=True, index_offset=int(bounds[g]))
        keys.append(kk)
        idx.append(i)
    kd = torch.from_numpy(np.stack(keys)).cuda()
    idd = torch.from_numpy(np.stack(idx)).cuda()
    os_ = torch.empty((16, k), dtype=torch.float32, device="cuda")
    oi = torch.empty((16, k), dtype=torch.int64, device="cuda")
    ok = torch.empty((16, k), dtype=torch.float64, device="cuda")
    vdb.merge_topk_device(kd.data_ptr(), idd.data_ptr(), G, 16, k, k, "euclidean", os_.data_ptr(), oi.data_ptr(),
                          ok.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    es, ei, ek = ref_cpu.exact_search(Q, V, k, "euclidean")
    np.testing.assert_array_equal(oi.cpu().numpy(), ei)
    np.testing.assert_array_equal(ok.cpu().numpy(), ek)


def test_device_pointer_search_matches_host(vdb):
    import torch
    rng = np.random.default_rng(17)
    V = rng.random((10000, 256), dtype=np.float32)
    Q = rng.random((64, 256), dtype=np.float32)
    ix = vdb.NativeIndex(256, "cosine")
    ix.add(V)
    s_h, i_h = ix.search(Q, 10)
    qd = torch.from_numpy(Q).cuda()
    sd = torch.empty((64, 10), dtype=torch.float32, device="cuda")
    idd = torch.empty((64, 10), dtype=torch.int64, device="cuda")
    ix.search_device(qd.data_ptr(), 64, 10, sd.data_ptr(), idd.data_ptr(),
                     stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(idd.cpu().numpy(), i_h)
    np.testing.assert_array_equal(sd.cpu().numpy(), s_h)


def test_device_search_orders_with_torch_default_stream(vdb):
    """stream=0 (PyTorch's default stream) must order the search with the torch work
    around it: no explicit synchronise between the search and the copy that reads it."""
    import torch
    rng = np.random.default_rng(24)
    V = rng.random((50000, 128), dtype=np.float32)
    Q = rng.random((64, 128), dtype=np.float32)
    ix = vdb.NativeIndex(128, "cosine")
    ix.add(V)
    _, ei, _ = ref_cpu.exact_search(Q, V, 10, "cosine")
    qd = torch.from_numpy(Q).cuda()
    for _ in range(3):
        idd = torch.full((64, 10), -7, dtype=torch.int64, device="cuda")
        sd = torch.empty((64, 10), dtype=torch.float32, device="cuda")
        ix.search_device(qd.data_ptr(), 64, 10, sd.data_ptr(), idd.data_ptr(), stream=0)
        got = idd.clone().cpu().numpy()  # torch work on the default stream, no synchronise
        np.testing.assert_array_equal(got, ei)


@pytest.mark.parametrize("metric", ["cosine", "euclidean"])
def test_device_search_gated_fallback(vdb, metric):
    """Device-memory searches do not wait for the certificate: the exact path is
    queued gated on the device's flag count.  Duplicates force some queries onto
    it; several searches are queued back to back before one synchronise."""
    import torch
    rng = np.random.default_rng(23)
    V = rng.random((30000, 96), dtype=np.float32)
    V[2000:2060] = V[11]
    V[9000:9040] = V[29]
    Q = np.concatenate([V[[11, 29]], rng.random((14, 96), dtype=np.float32)])
    ix = vdb.NativeIndex(96, metric, precision="bf16x3")  # KP = 32 < the 60 copies
    ix.add(V)
    es, ei, ek = ref_cpu.exact_search(Q, V, 12, metric)
    qd = torch.from_numpy(Q).cuda()
    outs = []
    st = torch.cuda.Stream()
    torch.cuda.synchronize()
    for _ in range(3):
        sd = torch.empty((16, 12), dtype=torch.float32, device="cuda")
        idd = torch.empty((16, 12), dtype=torch.int64, device="cuda")
        kd = torch.empty((16, 12), dtype=torch.float64, device="cuda")
        ix.search_device(qd.data_ptr(), 16, 12, sd.data_ptr(), idd.data_ptr(), kd.data_ptr(), stream=st.cuda_stream)
        outs.append((sd, idd, kd))
    torch.cuda.synchronize()
    for sd, idd, kd in outs:
        np.testing.assert_array_equal(idd.cpu().numpy(), ei)
        np.testing.assert_array_equal(kd.cpu().numpy(), ek)
    assert ix.stat("fallback_queries") >= 3 * 2  # the two duplicated queries, every search


@pytest.mark.parametrize("metric", ["cosine", "euclidean"])
def test_device_search_several_streams(vdb, metric):
    """Batches queued round-robin on three streams from one host thread (a server's request
    streams; bench.py --streams) get workspaces of their own and run concurrently; every
    batch equals the oracle, including those whose duplicates take the gated fallback."""
    import torch
    rng = np.random.default_rng(31)
    V = rng.random((40000, 160), dtype=np.float32)
    V[3000:3050] = V[17]
    Qs = [rng.random((40, 160), dtype=np.float32) for _ in range(6)]
    Qs[2][5] = V[17]
    ix = vdb.NativeIndex(160, metric)
    ix.add(V)
    streams = [torch.cuda.Stream() for _ in range(3)]
    outs = []
    torch.cuda.synchronize()
    for rep in range(2):
        for j, Q in enumerate(Qs):
            qd = torch.from_numpy(Q).cuda()
            sd = torch.empty((40, 10), dtype=torch.float32, device="cuda")
            idd = torch.empty((40, 10), dtype=torch.int64, device="cuda")
            kd = torch.empty((40, 10), dtype=torch.float64, device="cuda")
            st = streams[(rep * len(Qs) + j) % 3]
            st.wait_stream(torch.cuda.current_stream())  # the query copy
            ix.search_device(qd.data_ptr(), 40, 10, sd.data_ptr(), idd.data_ptr(), kd.data_ptr(),
                             stream=st.cuda_stream)
            outs.append((j, qd, idd, kd))
    torch.cuda.synchronize()
    for j, _, idd, kd in outs:
        _, ei, ek = ref_cpu.exact_search(Qs[j], V, 10, metric)
        np.testing.assert_array_equal(idd.cpu().numpy(), ei)
        np.testing.assert_array_equal(kd.cpu().numpy(), ek)


def test_similarity_matrix_operator_slot(vdb):
    import torch
    rng = np.random.default_rng(19)
    V = rng.random((3000, 384), dtype=np.float32)
    Q = rng.random((4, 384), dtype=np.float32)
    for metric in ("cosine", "euclidean"):
        out = torch.empty((4, 3000), dtype=torch.float32, device="cuda")
        vt, qt = torch.from_numpy(V).cuda(), torch.from_numpy(Q).cuda()
        vdb.similarity_matrix_device(vt.data_ptr(), 3000, 384, qt.data_ptr(), 4, metric, out.data_ptr())
        torch.cuda.synchronize()
        if metric == "cosine":
            ref = ref_cpu.reference_cosine_batch(Q, V)
        else:
            ref = np.stack([ref_cpu.reference_euclidean_distances(q, V) for q in Q])
        np.testing.assert_allclose(out.cpu().numpy(), ref, atol=1e-4, rtol=0)


@pytest.mark.slow
@pytest.mark.parametrize("precision", PRECISIONS)
def test_full_size_c2_subset(vdb, precision):
    """BASELINE.json configs[1]: 1M x 768 fp32 cosine, B=64, k=10.  The oracle
    checks 8 of the 64 queries exactly; every query checks size-independent
    properties (sorted scores, planted self-queries on top)."""
    N, D, B, k = 1_000_000, 768, 64, 10
    V = np.random.default_rng(0).random((N, D), dtype=np.float32)
    Q = np.random.default_rng(1).random((B, D), dtype=np.float32)
    Q[5] = V[777_777]
    Q[6] = V[3]
    ix = vdb.NativeIndex(D, "cosine", precision=precision)
    ix.add(V)
    s, i = ix.search(Q, k)
    assert ix.stat("fallback_queries") == 0  # the candidate pass certified every query
    assert (np.diff(s, axis=1) <= 0).all()
    assert i[5, 0] == 777_777 and i[6, 0] == 3
    sub = [0, 1, 2, 5, 6, 31, 32, 63]
    es, ei, ek = ref_cpu.exact_search(Q[sub], V, k, "cosine")
    np.testing.assert_array_equal(i[sub], ei)
    np.testing.assert_allclose(s[sub], es, atol=1e-6, rtol=0)


@pytest.mark.parametrize("metric", ["cosine", "euclidean"])
def test_scan2_q4_shape(vdb, metric):
    """The split pass's 128-query shape (knob "scan_q4" = 1; D <= 128, KP = 128, B >= 256):
    query block of 128 in LDS, 2 row tiles per wave, 48 kept per query and workgroup with the
    drop bound raising gthr at the end.  Bit-exact vs the oracle for bf16 (k = 10) and bf16x3
    (k = 100), compile-time (D = 128) and runtime (D = 64) group counts, ragged batches, a mask,
    and clustered rows that put more than 48 of a query's top 100 into one workgroup."""
    rng = np.random.default_rng(67)
    for D, N in ((128, 120_000), (64, 50_003)):
        V = rng.random((N, D), dtype=np.float32)
        Q = rng.random((520, D), dtype=np.float32)
        Q[3], Q[519] = V[N - 1], V[777]
        for prec, k in (("bf16", 10), ("bf16x3", 100)):
            ix = vdb.NativeIndex(D, metric, precision=prec)
            ix.set_param("scan_q4", 1)
            ix.add(V)
            for B in (520, 256):
                s, i, kk = ix.search(Q[:B], k, with_keys=True)
                es, ei, ek = ref_cpu.exact_search(Q[:B], V, k, metric)
                np.testing.assert_array_equal(i, ei)
                np.testing.assert_array_equal(kk, ek)
            mask = rng.random(N) < 0.4
            bits = np.zeros(((N + 31) // 32) * 32, bool)
            bits[:N] = mask
            words = np.packbits(bits, bitorder="little").view("<u4").astype(np.uint32)
            s, i, kk = ix.search(Q[:300], k, row_mask=words, with_keys=True)
            es, ei, ek = ref_cpu.exact_search(Q[:300], V, k, metric, row_mask=mask)
            np.testing.assert_array_equal(i, ei)
            np.testing.assert_array_equal(kk, ek)
            assert ix.stat("searches_q4") == 3
            ix.close()
    V = rng.random((60_000, 128), dtype=np.float32)
    V[30_000:30_070] = (V[9] + 1e-3 * rng.random((70, 128))).astype(np.float32)
    Q = np.concatenate([V[9:10], rng.random((299, 128), dtype=np.float32)])
    ix = vdb.NativeIndex(128, metric, precision="bf16x3")
    ix.set_param("scan_q4", 1)
    ix.add(V)
    s, i, kk = ix.search(Q, 100, with_keys=True)
    es, ei, ek = ref_cpu.exact_search(Q, V, 100, metric)
    np.testing.assert_array_equal(i, ei)
    np.testing.assert_array_equal(kk, ek)
    ix.close()


@pytest.mark.parametrize("precision", ["i8", "i8x3"])
@pytest.mark.parametrize("metric", ["cosine", "euclidean"])
def test_i8_quantisation_edges(vdb, metric, precision):
    """The int8 copy (vdb_scan8_kernel.h): centring row and quantisation step come from the
    first add, are derived again as a small index doubles, and rows past the step's range
    clip (their residual enters the certificate); L2 rows far from the origin push the query
    scale up (int32 range of H's start value).  Every result stays exact."""
    rng = np.random.default_rng(77)
    D, k = 200, 12
    cases = []
    V = rng.random((9000, D), dtype=np.float32)
    cases.append(("tiny first add", V, [1, 2, 5, 40, 952, 8000]))
    W = rng.random((9000, D), dtype=np.float32)
    W[5000:] *= 10.0  # past the range fixed by the first 5000 rows... until the re-derivation
    cases.append(("outliers after the setup", W, [5000, 4000]))
    W2 = rng.random((70000, 64), dtype=np.float32)
    W2[66000:] = W2[66000:] * 30.0 - 15.0  # past kDirRows: the setup stays, these rows clip
    cases.append(("outliers past kDirRows", W2, [66000, 4000]))
    F = (1000.0 + rng.random((6000, D), dtype=np.float32)).astype(np.float32)
    cases.append(("far from the origin", F, [6000]))
    Z = rng.random((3000, D), dtype=np.float32)
    Z[100:110] = 0.0
    cases.append(("zero rows", Z, [3000]))
    for name, V, pieces in cases:
        Dv = V.shape[1]
        Q = rng.random((11, Dv), dtype=np.float32) * (V.max() - V.min()) + V.min()
        Q[0] = V[123]
        if name == "zero rows":
            Q[1] = 0.0
        ix = vdb.NativeIndex(Dv, metric, precision=precision)
        r = 0
        for p in pieces:
            ix.add(V[r:r + p])
            r += p
        s, i, kk = ix.search(Q, k, with_keys=True)
        es, ei, ek = ref_cpu.exact_search(Q, V, k, metric)
        np.testing.assert_array_equal(i, ei, err_msg=name)
        valid = ei >= 0
        np.testing.assert_array_equal(kk[valid], ek[valid], err_msg=name)
        print(f"{metric} {precision} {name}: fallbacks {ix.stat('fallback_queries')} of {Q.shape[0]}")
        ix.close()


@pytest.mark.parametrize("metric", ["cosine", "euclidean"])
def test_i8_store_filled_one_add_at_a_time(vdb, metric):
    """A store filled by many small adds (the REST path: one vector per request) gets a
    usable int8 setup: after the re-derivations the int8 pass certifies the batch."""
    rng = np.random.default_rng(5)
    D, k = 96, 10
    V = rng.random((3000, D), dtype=np.float32)
    ix = vdb.NativeIndex(D, metric, precision="i8")
    r = 0
    while r < V.shape[0]:
        n = int(rng.integers(1, 8))
        ix.add(V[r:r + n])
        r += n
    Q = rng.random((16, D), dtype=np.float32)
    s, i, kk = ix.search(Q, k, with_keys=True)
    es, ei, ek = ref_cpu.exact_search(Q, V, k, metric)
    np.testing.assert_array_equal(i, ei)
    np.testing.assert_array_equal(kk, ek)
    assert ix.stat("searches_i8") == 1
    assert ix.stat("fallback_queries") <= 2, ix.stat("fallback_queries")


def _graded_neighbours(rng, x, n, lo=1e-3, hi=4e-3):
    """n rows around x whose cosine to x falls evenly in [1 - hi, 1 - lo] (L2: squared distance
    2 c |x|^2): closer together than the int8 pass can separate (its eps ~4e-3), far enough
    apart for BF16X3 (eps ~1e-4)."""
    c = np.linspace(lo, hi, n)
    u = rng.standard_normal((n, x.size))
    xd = x.astype(np.float64)
    u -= np.outer(u @ xd / (xd @ xd), xd)
    u *= np.linalg.norm(xd) / np.linalg.norm(u, axis=1, keepdims=True)
    return (xd + np.sqrt(2.0 * c)[:, None] * u).astype(np.float32)


@pytest.mark.parametrize("metric", ["cosine", "euclidean"])
def test_device_repass_of_uncertified_queries(vdb, metric):
    """in a device-memory search (the bench's and a GPU-resident server's path)
    the few queries auto's int8 pass leaves uncertified are gathered ON THE DEVICE into a gated
    I8X3 sub-search (KP 128) on the same stream (device_repass 1) -- no exact scan, no host wait.
    A batch of 64 with one query that has 300 close rows (cosine 1 - [1e-3, 4e-3]) searched three
    times back to back on a side stream: every result exact, no fallback, one re-passed query per
    batch.  (GPUTEST_r04 once counted 2: the re-pass counter was zeroed by a hipMemset on the null
    stream, which this non-blocking stream is not ordered after, so the first search's count could
    land first and be wiped -- now zeroed and completed before any search uses it.)"""
    import torch
    rng = np.random.default_rng(47)
    N, D, B, k = 40000, 128, 64, 10
    V = rng.random((N, D), dtype=np.float32)
    V[1000:1300] = _graded_neighbours(rng, V[11], 300)
    Q = rng.random((B, D), dtype=np.float32)
    Q[5] = V[11]
    ix = vdb.NativeIndex(D, metric)  # auto: the I8 pass for k <= 16
    ix.set_param("device_repass", 1)
    ix.add(V)
    _, ei, ek = ref_cpu.exact_search(Q, V, k, metric)
    qd = torch.from_numpy(Q).cuda()
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    outs = []
    for _ in range(3):
        sd = torch.empty((B, k), dtype=torch.float32, device="cuda")
        idd = torch.empty((B, k), dtype=torch.int64, device="cuda")
        kd = torch.empty((B, k), dtype=torch.float64, device="cuda")
        ix.search_device(qd.data_ptr(), B, k, sd.data_ptr(), idd.data_ptr(), kd.data_ptr(), stream=st.cuda_stream)
        outs.append((idd, kd))
    torch.cuda.synchronize()
    for idd, kd in outs:
        np.testing.assert_array_equal(idd.cpu().numpy(), ei)
        np.testing.assert_array_equal(kd.cpu().numpy(), ek)
    assert ix.stat("searches_i8") == 3
    assert ix.stat("fallback_queries") == 0, ix.stat("fallback_queries")
    assert ix.stat("repass_queries") == 3, ix.stat("repass_queries")
    # a batch with no uncertified query: the gated sub-search does nothing
    Q2 = rng.random((B, D), dtype=np.float32)
    _, ei2, ek2 = ref_cpu.exact_search(Q2, V, k, metric)
    q2 = torch.from_numpy(Q2).cuda()
    sd = torch.empty((B, k), dtype=torch.float32, device="cuda")
    idd = torch.empty((B, k), dtype=torch.int64, device="cuda")
    kd = torch.empty((B, k), dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    ix.search_device(q2.data_ptr(), B, k, sd.data_ptr(), idd.data_ptr(), kd.data_ptr(), stream=0)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(idd.cpu().numpy(), ei2)
    np.testing.assert_array_equal(kd.cpu().numpy(), ek2)
    assert ix.stat("repass_queries") == 3 and ix.stat("fallback_queries") == 0


def test_device_repass_more_flagged_than_gathered(vdb):
    """More uncertified queries than the device re-pass gathers (16): the first 16 are
    re-passed, the rest take the gated exact path; all exact."""
    import torch
    rng = np.random.default_rng(53)
    N, D, B, k = 30000, 96, 40, 10
    V = rng.random((N, D), dtype=np.float32)
    Q = rng.random((B, D), dtype=np.float32)
    for j in range(20):  # 20 queries, each with 300 graded close rows
        V[1000 + 300 * j:1300 + 300 * j] = _graded_neighbours(rng, V[j], 300)
        Q[2 * j] = V[j]
    ix = vdb.NativeIndex(D, "cosine")
    ix.set_param("device_repass", 1)
    ix.add(V)
    _, ei, ek = ref_cpu.exact_search(Q, V, k, "cosine")
    qd = torch.from_numpy(Q).cuda()
    sd = torch.empty((B, k), dtype=torch.float32, device="cuda")
    idd = torch.empty((B, k), dtype=torch.int64, device="cuda")
    kd = torch.empty((B, k), dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    ix.search_device(qd.data_ptr(), B, k, sd.data_ptr(), idd.data_ptr(), kd.data_ptr(), stream=0)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(idd.cpu().numpy(), ei)
    np.testing.assert_array_equal(kd.cpu().numpy(), ek)
    rp, fb = ix.stat("repass_queries"), ix.stat("fallback_queries")
    print(f"re-passed {rp}, exact path {fb}")
    assert rp == 16 and fb >= 1


@pytest.mark.parametrize("mem", ["host", "device"])
def test_i8_narrow_kp_on_small_indexes(vdb, mem):
    """auto's I8 pass keeps KP = 128 instead of 256 on indexes of <= 512 K rows (one rank's shard
    of a weak-scaled run) until a search flags a query; from then on 256 (stat i8_wide).  Exact
    either way: a uniform batch (no flag, stays narrow), then a batch with one query among 300
    close rows (flagged: re-passed or sent to the exact path), then uniform again (wide)."""
    import torch
    rng = np.random.default_rng(71)
    N, D, B, k = 60000, 256, 64, 10
    V = rng.random((N, D), dtype=np.float32)
    V[3000:3300] = _graded_neighbours(rng, V[17], 300)
    Q1 = rng.random((B, D), dtype=np.float32)
    Q2 = rng.random((B, D), dtype=np.float32)
    Q2[9] = V[17]
    ix = vdb.NativeIndex(D, "cosine")
    ix.add(V)

    def run(Q):
        _, ei, ek = ref_cpu.exact_search(Q, V, k, "cosine")
        if mem == "host":
            _, i, kk = ix.search(Q, k, with_keys=True)
        else:
            qd = torch.from_numpy(Q).cuda()
            sd = torch.empty((B, k), dtype=torch.float32, device="cuda")
            idd = torch.empty((B, k), dtype=torch.int64, device="cuda")
            kd = torch.empty((B, k), dtype=torch.float64, device="cuda")
            torch.cuda.synchronize()
            ix.search_device(qd.data_ptr(), B, k, sd.data_ptr(), idd.data_ptr(), kd.data_ptr(), stream=0)
            torch.cuda.synchronize()
            i, kk = idd.cpu().numpy(), kd.cpu().numpy()
        np.testing.assert_array_equal(i, ei)
        np.testing.assert_array_equal(kk, ek)

    run(Q1)
    assert ix.stat("i8_wide") == 0
    run(Q2)
    run(Q1)  # (device memory: the flag of the batch before is seen by this search)
    run(Q1)
    assert ix.stat("i8_wide") == 1
    assert ix.stat("searches_i8") >= 2  # (device memory: the seen fallback also starts an I8 hold)
    ix2 = vdb.NativeIndex(D, "cosine")
    ix2.set_param("i8_narrow", 0)
    with pytest.raises(Exception):
        ix2.set_param("i8_narrow", 1)


def test_split_copy_allocated_lazily_under_auto(vdb):
    """under auto (int8 candidate pass) the split-bf16 copy is allocated only when a
    search first runs a split pass -- here the host re-pass of a query the int8 pass leaves
    uncertified (BF16X3) -- so an index that never needs it holds 7 B per element (fp32 rows 4,
    int8 planes 2, row-major xh 1) + 20 B per row.  Results exact before and after."""
    rng = np.random.default_rng(61)
    N, D, B, k = 30000, 128, 32, 10
    V = rng.random((N, D), dtype=np.float32)
    V[2000:2300] = _graded_neighbours(rng, V[3], 300)
    ix = vdb.NativeIndex(D, "cosine")
    ix.add(V)
    cap = ix.stat("capacity")
    Dp = (D + 63) // 64 * 64
    assert ix.stat("split_copy") == 0
    assert ix.stat("device_bytes") == 7 * cap * Dp + 20 * cap, ix.stat("device_bytes")
    Q = rng.random((B, D), dtype=np.float32)
    _, ei, ek = ref_cpu.exact_search(Q, V, k, "cosine")
    _, i, kk = ix.search(Q, k, with_keys=True)
    np.testing.assert_array_equal(i, ei)
    np.testing.assert_array_equal(kk, ek)
    assert ix.stat("split_copy") == 0  # nothing needed it
    Q[4] = V[3]  # 300 rows the int8 pass cannot separate: host re-pass in BF16X3
    _, ei, ek = ref_cpu.exact_search(Q, V, k, "cosine")
    _, i, kk = ix.search(Q, k, with_keys=True)
    np.testing.assert_array_equal(i, ei)
    np.testing.assert_array_equal(kk, ek)
    assert ix.stat("repass_queries") >= 1
    assert ix.stat("split_copy") == 1 and ix.stat("split_copy_builds") == 1
    assert ix.stat("device_bytes") == 11 * cap * Dp + 20 * cap
    # the copy is now kept up to date by adds (and grows with the index)
    V2 = rng.random((40000, D), dtype=np.float32)
    ix.add(V2)
    ix.set_param("precision", 1)  # bf16x3: reads the split copy on every search
    Va = np.concatenate([V, V2])
    _, ei, ek = ref_cpu.exact_search(Q, Va, k, "cosine")
    _, i, kk = ix.search(Q, k, with_keys=True)
    np.testing.assert_array_equal(i, ei)
    np.testing.assert_array_equal(kk, ek)
    assert ix.stat("split_copy_builds") == 1
    # a bf16x3 index allocates it up front
    ix3 = vdb.NativeIndex(D, "euclidean", precision="bf16x3")
    ix3.add(V)
    assert ix3.stat("split_copy") == 1
    _, ei, ek = ref_cpu.exact_search(Q, V, k, "euclidean")
    _, i, kk = ix3.search(Q, k, with_keys=True)
    np.testing.assert_array_equal(i, ei)
    np.testing.assert_array_equal(kk, ek)


def test_device_repass_after_a_search_of_another_shape(vdb):
    """the device re-pass's gathered-query block has slots past the gathered
    count; they are zeroed, not left holding an earlier search's workspace bytes (which would set
    the batch's int8 scale).  L2, a search of another batch size and k on the same stream first,
    then a batch with one query among 300 close rows: re-passed (not the exact path), exact."""
    import torch
    rng = np.random.default_rng(67)
    N, D = 40000, 128
    V = rng.random((N, D), dtype=np.float32) * 4.0
    V[1000:1300] = _graded_neighbours(rng, V[11], 300)
    ix = vdb.NativeIndex(D, "euclidean")
    ix.set_param("device_repass", 1)
    ix.add(V)
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    Q0 = (rng.random((48, D), dtype=np.float32) * 50.0).astype(np.float32)  # large |q|: big workspace values
    q0 = torch.from_numpy(Q0).cuda()
    o0 = [torch.empty((48, 30), dtype=t, device="cuda") for t in (torch.float32, torch.int64, torch.float64)]
    ix.search_device(q0.data_ptr(), 48, 30, o0[0].data_ptr(), o0[1].data_ptr(), o0[2].data_ptr(), stream=st.cuda_stream)
    B, k = 64, 10
    Q = rng.random((B, D), dtype=np.float32) * 4.0
    Q[5] = V[11]
    qd = torch.from_numpy(Q).cuda()
    sd = torch.empty((B, k), dtype=torch.float32, device="cuda")
    idd = torch.empty((B, k), dtype=torch.int64, device="cuda")
    kd = torch.empty((B, k), dtype=torch.float64, device="cuda")
    ix.search_device(qd.data_ptr(), B, k, sd.data_ptr(), idd.data_ptr(), kd.data_ptr(), stream=st.cuda_stream)
    torch.cuda.synchronize()
    _, ei0, ek0 = ref_cpu.exact_search(Q0, V, 30, "euclidean")
    np.testing.assert_array_equal(o0[1].cpu().numpy(), ei0)
    _, ei, ek = ref_cpu.exact_search(Q, V, k, "euclidean")
    np.testing.assert_array_equal(idd.cpu().numpy(), ei)
    np.testing.assert_array_equal(kd.cpu().numpy(), ek)
    assert ix.stat("fallback_queries") == 0, ix.stat("fallback_queries")
