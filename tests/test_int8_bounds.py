"""The int8 candidate pass's error bound (vdb_scan8_kernel.h, vdb_scan8.hip prep8, vdb_api.cpp
finish arguments), checked on the CPU against a numpy model of the kernels' arithmetic.

The certificate (vdb_exact.hip finish_kernel) needs, for every row x and query q,
    |approx(x, q) - (exact(x, q) - shift(q))| <= eps(q)
where approx is the pass's integer-MFMA score, exact the fp64 key the results are ranked by, and
shift the per-query constant the pass leaves out (cosine mu.q, L2 2 mu.q - |q|^2).  This test
rebuilds approx exactly as the kernels do (centred rows, one step s_x, 8-bit / 16-bit planes,
batch query scale, integer sums, fp32 combination) and eps from the same statistics the
ingest and prep kernels measure, and checks the inequality on data where it is tight and where
it is not: uniform, near-duplicate rows, normal, L2 rows far from the origin.
"""
import numpy as np
import pytest

from oracle import ref_cpu


def _i8_model(V, Q, metric, prec):
    f32 = np.float32
    D = V.shape[1]
    nr = np.sqrt((V.astype(np.float64) ** 2).sum(1))
    if metric == "cosine":
        iv = (1.0 / np.maximum(nr, 1e-8)).astype(f32)
        Y = (V * iv[:, None]).astype(f32)
    else:
        Y = V.astype(f32)
    m = min(len(V), 65536)  # setup_direction: the first kDirRows rows
    sums = Y[:m].astype(np.float64).sum(0)
    dirv = (sums / np.sqrt((sums ** 2).sum())).astype(f32)
    mu = (sums / m).astype(f32)
    Z = (Y - mu).astype(f32)
    zmax = np.abs(Z[:m]).max()
    sx = f32(1.25 * zmax / 127) if zmax > 0 else f32(1.0)
    t = Z * (f32(1) / sx)
    xh = np.clip(np.rint(t), -127, 127)
    xl = np.clip(np.rint((t - xh) * f32(256)), -127, 127)
    r8 = Z.astype(np.float64) - np.float64(sx) * xh
    r16 = r8 - np.float64(sx) * xl / 256.0
    R8, R16 = np.sqrt((r8 ** 2).sum(1)).max(), np.sqrt((r16 ** 2).sum(1)).max()
    M8, M16 = np.abs(r8 @ dirv.astype(np.float64)).max(), np.abs(r16 @ dirv.astype(np.float64)).max()
    ZA = np.sqrt(((np.float64(sx) * xh) ** 2).sum(1)).max()
    XL = np.sqrt(((np.float64(sx) * xl / 256.0) ** 2).sum(1)).max()
    xmax = nr.max()
    # queries (prep_queries + prep8)
    qn = np.sqrt((Q.astype(np.float64) ** 2).sum(1))
    q = (Q * (1.0 / np.maximum(qn, 1e-8)).astype(f32)[:, None]).astype(f32) if metric == "cosine" else Q.astype(f32)
    sq = f32(np.abs(q).max() / 127)
    if metric == "euclidean":
        sq = max(sq, f32(0.5 * xmax * xmax / (float(sx) * 1.0e9)))
    tq = q * (f32(1) / sq)
    qh = np.clip(np.rint(tq), -127, 127)
    ql = np.clip(np.rint((tq - qh) * f32(256)), -127, 127)
    uH = f32(sx * sq)
    uL = f32(uH * f32(1.0 / 256.0))
    H = xh.astype(np.int64) @ qh.T.astype(np.int64)
    if metric == "euclidean":  # H starts at rint(-|x|^2/2 / uH) per row (rinit32 in fp32)
        rinit = (f32(-0.5) * (nr ** 2).astype(f32)).astype(f32)
        H = H + np.rint((rinit * (f32(1) / uH)).astype(f32)).astype(np.int64)[:, None]
    if prec == "i8":
        half = (H.astype(f32) * uH).astype(np.float64)
    else:
        L = xh.astype(np.int64) @ ql.T.astype(np.int64) + xl.astype(np.int64) @ qh.T.astype(np.int64)
        half = (H.astype(f32) * uH + L.astype(f32) * uL).astype(np.float64)
    approx = half if metric == "cosine" else 2.0 * half
    # eps (vdb_api.cpp fa.*, finish_kernel, prep8 qerr)
    x3 = prec == "i8x3"
    R, M = (R16, M16) if x3 else (R8, M8)
    qd = q.astype(np.float64)
    c = qd @ dirv.astype(np.float64)
    w = np.sqrt(((qd - c[:, None] * dirv.astype(np.float64)) ** 2).sum(1))
    xres, dres = 1.01 * R, 1.01 * M  # fa.xres / fa.dres; finish_kernel's bq (min of the two bounds)
    bq = np.minimum(xres * (1.0 if metric == "cosine" else qn), (w * xres + np.abs(c) * dres) * (1 + 1e-6) + 1e-6 * xres)
    r8q = np.sqrt(((qd - np.float64(sq) * qh) ** 2).sum(1))
    r16q = np.sqrt(((qd - np.float64(sq) * (qh + ql / 256.0)) ** 2).sum(1))
    qlv = np.sqrt(((np.float64(sq) * ql / 256.0) ** 2).sum(1))
    e = (ZA + (XL if x3 else 0.0)) * (r16q if x3 else r8q) + (XL * qlv if x3 else 0.0)
    e = e + (float(uH) if metric == "euclidean" else 0.0)
    qerr = 1.01 * (e if metric == "cosine" else 2.0 * e)
    eps_rel = 1.01 * 8.0 * 2.0 ** -24
    if metric == "cosine":
        eps = eps_rel + bq + qerr
    else:  # (the finish adds 2.4e-7 max(|a_k|, |acut|) on top: left out here, a stricter check)
        eps = eps_rel * (2.0 * qn * xmax + xmax * xmax) + 2.0 * bq + qerr
    shift = (mu.astype(np.float64) @ qd.T) if metric == "cosine" else (2.0 * (mu.astype(np.float64) @ qd.T) - qn ** 2)
    return approx, eps, shift


def _datasets():
    rng = np.random.default_rng(12)
    D = 192
    yield "uniform", rng.random((3000, D), dtype=np.float32)
    base = rng.random(D, dtype=np.float32)
    yield "near-duplicates", (base + 1e-4 * rng.standard_normal((3000, D))).astype(np.float32)
    yield "normal", rng.standard_normal((3000, D)).astype(np.float32)
    yield "far from the origin", (1000.0 + rng.random((3000, D), dtype=np.float32)).astype(np.float32)


@pytest.mark.parametrize("prec", ["i8", "i8x3"])
@pytest.mark.parametrize("metric", ["cosine", "euclidean"])
def test_int8_error_bound_holds(metric, prec):
    rng = np.random.default_rng(3)
    for name, V in _datasets():
        Q = V[rng.integers(0, len(V), 12)] + 1e-3 * rng.standard_normal((12, V.shape[1])).astype(np.float32)
        Q = np.concatenate([Q, rng.random((4, V.shape[1]), dtype=np.float32) * (V.max() - V.min()) + V.min()])
        Q = Q.astype(np.float32)
        approx, eps, shift = _i8_model(V, Q, metric, prec)
        _, ei, ek = ref_cpu.exact_search(Q, V, len(V), metric)
        exact = np.empty_like(approx)
        for b in range(Q.shape[0]):
            exact[ei[b], b] = ek[b]
        err = np.abs(approx - (exact - shift[None, :]))
        worst = (err.max(0) / eps).max()
        # the (half-)score additions the model leaves out (fp32 evaluation of the start value)
        # are far inside the 1.01 margins: the bound must hold with room to spare
        assert worst <= 1.0, (name, worst)
        print(f"{metric} {prec} {name}: max |err| / eps = {worst:.3f}")


@pytest.mark.parametrize("metric", ["cosine", "euclidean"])
def test_i8_refinement_bound_holds(metric):
    """The finish's I8 refinement (vdb_exact.hip finish_kernel, FinishArgs.xh_rm): each
    candidate's approximate score corrected by the query's rounding residual,
        a' = a + f s_x xh.r,   r = q' - s_q qh,   f = 1 cosine / 2 L2,
    leaves only the corpus rounding (and the L2 start value's rounding, prep8 qerr2) of the
    error; the refinement's own fp32 arithmetic adds a per-row term.  Checked on the CPU model of
    the kernels' arithmetic, on the same datasets as the unrefined bound; and the refined bound is
    far tighter than the unrefined one on uniform data (why C2 / C3 rerank a fraction of KP)."""
    rng = np.random.default_rng(5)
    f32 = np.float32
    for name, V in _datasets():
        Q = V[rng.integers(0, len(V), 12)] + 1e-3 * rng.standard_normal((12, V.shape[1])).astype(np.float32)
        Q = np.concatenate([Q, rng.random((4, V.shape[1]), dtype=np.float32) * (V.max() - V.min()) + V.min()])
        Q = Q.astype(np.float32)
        approx, eps, shift = _i8_model(V, Q, metric, "i8")
        # the model's internals again (same arithmetic as _i8_model)
        D = V.shape[1]
        nr = np.sqrt((V.astype(np.float64) ** 2).sum(1))
        Y = (V * (1.0 / np.maximum(nr, 1e-8)).astype(f32)[:, None]).astype(f32) if metric == "cosine" else V
        m = min(len(V), 65536)
        mu = (Y[:m].astype(np.float64).sum(0) / m).astype(f32)
        Z = (Y - mu).astype(f32)
        sx = f32(1.25 * np.abs(Z[:m]).max() / 127)
        xh = np.clip(np.rint(Z * (f32(1) / sx)), -127, 127)
        qn = np.sqrt((Q.astype(np.float64) ** 2).sum(1))
        q = (Q * (1.0 / np.maximum(qn, 1e-8)).astype(f32)[:, None]).astype(f32) if metric == "cosine" else Q
        sq = f32(np.abs(q).max() / 127)
        if metric == "euclidean":
            sq = max(sq, f32(0.5 * nr.max() ** 2 / (float(sx) * 1.0e9)))
        qh = np.clip(np.rint(q * (f32(1) / sq)), -127, 127)
        r = (q - sq * qh.astype(f32)).astype(f32)
        fs = 1.0 if metric == "cosine" else 2.0
        refined = approx + fs * float(sx) * (xh.astype(np.float64) @ r.T.astype(np.float64))
        _, ei, ek = ref_cpu.exact_search(Q, V, len(V), metric)
        exact = np.empty_like(approx)
        for b in range(Q.shape[0]):
            exact[ei[b], b] = ek[b]
        # eps' = eps without the query's rounding share (its CS term), plus the refinement's fp32
        # rounding as the kernel bounds it (per query, rows stored as xh + 128; + 2.4e-7 |a'| per row)
        qmx = 127.0 * float(sq)
        Dp = (D + 63) // 64 * 64
        rabs = np.abs(r).sum(1)[None, :]
        rnd = fs * float(sx) * ((Dp + 8) * 5.97e-8 * 256.0 * rabs + 1.2e-7 * qmx * 127.0 * D) + 2.4e-7 * np.abs(refined)
        uH = float(sx) * float(sq)
        qerr2 = 1.01 * (2.0 * uH if metric == "euclidean" else 0.0)
        # the corpus share of eps: eps minus the model's qerr (recomputed: |z~|max |q' - q~|)
        ZA = np.sqrt(((np.float64(sx) * xh) ** 2).sum(1)).max()
        r8q = np.sqrt(((q.astype(np.float64) - np.float64(sq) * qh) ** 2).sum(1))
        e8 = ZA * r8q + (uH if metric == "euclidean" else 0.0)
        qerr = 1.01 * (e8 if metric == "cosine" else 2.0 * e8)
        eps2 = eps - qerr + qerr2
        err = np.abs(refined - (exact - shift[None, :]))
        worst = (err / (eps2[None, :] + rnd)).max()
        assert worst <= 1.0, (name, worst)
        print(f"{metric} {name}: refined max |err| / eps' = {worst:.3f}; eps' / eps = {(eps2 / eps).mean():.3f}")
