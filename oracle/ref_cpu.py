"""CPU oracle for the brute-force distance + top-k hot path.  TEST INFRASTRUCTURE.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module, and only as the checker / the timed CPU baseline.
The product (``mlx-vector-db_amd/``) never imports it: its only compute path is
the gfx950 HIP library.

What it restates (reference = /root/reference, Theseus-AT/mlx-vector-db):
  * ``reference_*`` functions: the reference's own fp32 arithmetic, line for
    line, with numpy standing in for MLX (MLX is not installable here:
    ``import performance.mlx_optimized`` -> ModuleNotFoundError 'mlx', an
    ordinary import error, not a permission denial).
  * ``canonical_*`` / ``exact_*``: the ranking contract the GPU path is held to
    bit for bit — fp64 keys in the one summation order the kernels use
    (mlx-vector-db_amd/csrc/vdb_common.h), ties to the lower row index.

Parity pinning.  The reference ships no golden vectors, fixtures or seeded
tests for this path: its known-answer checks are behavioural —
P1 self-query top-1 with similarity > 0.999 (tests/test_integration.py:81-136),
P2/P3 metadata-filter AND semantics (test_integration.py:139-160,
tests/demo.py:217-243), P4 counts, P5 result length k (tests/test_vector_store.py:35-40),
P6 batch shape (demo.py:130-139), P7 empty store.  tests/test_oracle.py checks
this module against all of them, against hand-derived known answers
(orthogonal / parallel / scaled vectors whose cosine and L2 are exact), and
against the committed fixtures in tests/golden/ (made by
tests/golden/gen_golden.py from this module).  MLX's own argsort cannot be run
here, so the reference's order among fp32 near-ties is "parity unpinned"
beyond those pins; the exact fp64 order is the contract instead.
"""
from __future__ import annotations

import numpy as np

EPS = 1e-8  # service/optimized_vector_store.py:36, performance/mlx_optimized.py:45


# =============================================================================
# 1. Reference arithmetic (fp32), restated from the reference sources
# =============================================================================
def reference_cosine_scores(query: np.ndarray, vectors: np.ndarray) -> np.ndarray:
    """`_compiled_cosine_similarity` (service/optimized_vector_store.py:31-41):
    norms (mx.linalg.norm, :34-35), max with 1e-8 (:36-38), divide (:39-40),
    matmul(vectors_normalized, query_normalized.T).flatten() (:41).  fp32."""
    q = np.asarray(query, dtype=np.float32)
    if q.ndim == 1:
        q = q[None, :]
    v = np.asarray(vectors, dtype=np.float32)
    qn = np.maximum(np.linalg.norm(q, axis=1, keepdims=True), np.float32(EPS)).astype(np.float32)
    vn = np.maximum(np.linalg.norm(v, axis=1, keepdims=True), np.float32(EPS)).astype(np.float32)
    return ((v / vn) @ (q / qn).T).reshape(-1).astype(np.float32)


def reference_euclidean_distances(query: np.ndarray, vectors: np.ndarray) -> np.ndarray:
    """`_compiled_euclidean_distance` (service/optimized_vector_store.py:43-48):
    sqrt(sum((vectors - query)^2, axis=1)), fp32."""
    q = np.asarray(query, dtype=np.float32).reshape(1, -1)
    d = np.asarray(vectors, dtype=np.float32) - q
    return np.sqrt(np.sum(d * d, axis=1, dtype=np.float32)).astype(np.float32)


def reference_cosine_batch(queries: np.ndarray, vectors: np.ndarray) -> np.ndarray:
    """`compute_cosine_similarity_batch` (performance/mlx_optimized.py:59-88): [B, N] fp32,
    with its ValueError checks (:65-72)."""
    Q = np.asarray(queries, dtype=np.float32)
    V = np.asarray(vectors, dtype=np.float32)
    if Q.ndim != 2:
        raise ValueError(f"query_vectors muss 2D sein, erhielt Shape {Q.shape}")
    if V.ndim != 2:
        raise ValueError(f"db_vectors muss 2D sein, erhielt Shape {V.shape}")
    if Q.shape[1] != V.shape[1]:
        raise ValueError(f"Dimension Mismatch: query_vectors Dim {Q.shape[1]}, db_vectors Dim {V.shape[1]}")
    qn = np.maximum(np.sqrt(np.sum(Q * Q, axis=1, keepdims=True)), np.float32(EPS))
    vn = np.maximum(np.sqrt(np.sum(V * V, axis=1, keepdims=True)), np.float32(EPS))
    return ((Q / qn) @ (V / vn).T).astype(np.float32)


def reference_topk_indices(scores: np.ndarray, k: int, metric: str = "cosine") -> np.ndarray:
    """mx.argsort(-s)[:k] (cosine, :181) / mx.argsort(s)[:k] (euclidean, :178), as a
    STABLE sort (ties -> lower row); empty for k <= 0
    (performance/mlx_optimized.py:98-105)."""
    if k <= 0:
        return np.zeros(0, dtype=np.int64)
    key = -scores if metric != "euclidean" else scores
    return np.argsort(key, kind="stable")[:k].astype(np.int64)


def reference_store_search(query, vectors, k=10, metric="cosine", metadata=None, filter_metadata=None):
    """`MLXVectorStore.query` -> `_brute_force_search` (service/optimized_vector_store.py:116-192),
    HNSW disabled.  Returns (indices, scores, metadata) Python lists."""
    V = np.asarray(vectors, dtype=np.float32)
    if V.shape[0] == 0:
        return [], [], []
    original = None
    target = V
    if filter_metadata:
        original = [i for i, m in enumerate(metadata) if all(m.get(a) == b for a, b in filter_metadata.items())]
        if not original:
            return [], [], []
        target = V[original]
    if metric == "cosine":
        s = reference_cosine_scores(query, target)
    elif metric == "euclidean":
        s = reference_euclidean_distances(query, target)
    else:
        raise RuntimeError("Keine kompilierte Ähnlichkeitsfunktion verfügbar.")
    local = reference_topk_indices(s, k, metric)
    top = s[local]
    idx = [original[i] for i in local.tolist()] if original is not None else local.tolist()
    meta = [metadata[i] for i in idx] if metadata is not None else [None] * len(idx)
    return idx, top.tolist(), meta


def reference_batch_search(queries, vectors, k=10):
    """`optimized_batch_similarity_search` (performance/mlx_optimized.py:217-248):
    (indices [B,k'], scores [B,k']) with k' = min(k, N)."""
    S = reference_cosine_batch(queries, vectors)
    B, N = S.shape
    if N == 0:
        return np.zeros((B, 0), np.int64), np.zeros((B, 0), np.float32)
    kk = min(k, N)
    if kk <= 0:
        return np.zeros((B, 0), np.int64), np.zeros((B, 0), np.float32)
    idx = np.argsort(-S, axis=1, kind="stable")[:, :kk]
    return idx.astype(np.int64), np.take_along_axis(S, idx, axis=1)


def reference_l2_batch_chunked(queries, vectors, k=10, chunk_rows=1 << 20):
    """A batch of the store's L2 queries (`_compiled_euclidean_distance`,
    service/optimized_vector_store.py:43-48: sqrt(sum((x - q)^2)) per row, fp32) with the full
    stable argsort of `_brute_force_search` (:176-183) replaced by a running top-k over corpus
    chunks (C4's [512, 10M] distance matrix would be 20 GB).  Merging by
    (distance asc, row asc) keeps exactly the rows the full stable argsort's [:k] would, in the
    same order.  Returns (indices int64 [B, k'], distances fp32 [B, k']), k' = min(k, N)."""
    Q = np.asarray(queries, dtype=np.float32)
    V = np.asarray(vectors, dtype=np.float32)
    B, N = Q.shape[0], V.shape[0]
    kk = min(k, N)
    best_d = np.full((B, 0), np.inf, np.float32)
    best_i = np.zeros((B, 0), np.int64)
    for r0 in range(0, N, chunk_rows):
        C = V[r0:r0 + chunk_rows]
        d = np.empty((B, C.shape[0]), np.float32)
        for b in range(B):
            diff = C - Q[b]
            d[b] = np.sqrt(np.sum(diff * diff, axis=1, dtype=np.float32))
        kc = min(kk, C.shape[0])
        vk = np.partition(d, kc - 1, axis=1)[:, kc - 1]  # every row <= the chunk's kc-th distance (ties kept)
        nd = np.full((B, kk), np.inf, np.float32)
        ni = np.zeros((B, kk), np.int64)
        for b in range(B):
            sel = np.flatnonzero(d[b] <= vk[b])
            cd = np.concatenate([best_d[b], d[b, sel]])
            ci = np.concatenate([best_i[b], sel.astype(np.int64) + r0])
            order = np.lexsort((ci, cd))[:kk]  # (distance asc, row asc): lexsort's last key is primary
            nd[b, :order.size], ni[b, :order.size] = cd[order], ci[order]
        best_d, best_i = nd, ni
    return best_i, best_d


# =============================================================================
# 2. The exact ranking contract (fp64, canonical order) the GPU path must match
# =============================================================================
def _pieces(A: np.ndarray) -> np.ndarray:
    """[M, D] -> fp64 [M, np, 64, 4]: zero-pad D to a multiple of 256; lane l of
    pass m owns dims 256 m + 4 l + j (the canonical order, vdb_common.h)."""
    A = np.asarray(A, dtype=np.float32)
    if A.ndim == 1:
        A = A[None, :]
    M, D = A.shape
    Dp = (D + 255) // 256 * 256
    if Dp != D:
        A = np.pad(A, [(0, 0), (0, Dp - D)])
    return A.astype(np.float64).reshape(M, Dp // 256, 64, 4)


def _butterfly(acc: np.ndarray) -> np.ndarray:
    """xor-butterfly over the last axis (64 lanes), offsets 32..1; returns lane 0."""
    lanes = np.arange(64)
    for off in (32, 16, 8, 4, 2, 1):
        acc = acc + acc[..., lanes ^ off]
    return acc[..., 0]


def canonical_sumsq64(A: np.ndarray) -> np.ndarray:
    """Per-row sum of squares in fp64, canonical order (pack_rows_kernel, prep_queries_kernel)."""
    X = _pieces(A)
    acc = np.zeros((X.shape[0], 64))
    for m in range(X.shape[1]):
        for j in range(4):
            v = X[:, m, :, j]
            acc = acc + v * v
    return _butterfly(acc)


def canonical_norm64(A: np.ndarray) -> np.ndarray:
    return np.sqrt(canonical_sumsq64(A))


def canonical_dot64(q: np.ndarray, X: np.ndarray) -> np.ndarray:
    """fp64 q.x for every row of X, canonical order (exact_key<cosine>, vdb_exact.hip)."""
    qp = _pieces(np.asarray(q).reshape(1, -1))[0]
    Xp = _pieces(X)
    acc = np.zeros((Xp.shape[0], 64))
    for m in range(Xp.shape[1]):
        for j in range(4):
            acc = acc + qp[m, :, j] * Xp[:, m, :, j]
    return _butterfly(acc)


def canonical_sqdist64(q: np.ndarray, X: np.ndarray) -> np.ndarray:
    """fp64 sum((x-q)^2) for every row of X, canonical order (exact_key<euclidean>)."""
    qp = _pieces(np.asarray(q).reshape(1, -1))[0]
    Xp = _pieces(X)
    acc = np.zeros((Xp.shape[0], 64))
    for m in range(Xp.shape[1]):
        for j in range(4):
            d = Xp[:, m, :, j] - qp[m, :, j]
            acc = acc + d * d
    return _butterfly(acc)


def exact_keys(q: np.ndarray, X: np.ndarray, metric: str, xnorm64: np.ndarray | None = None) -> np.ndarray:
    """Ranking keys, higher = better: cosine similarity / minus squared L2 (fp64)."""
    if metric == "cosine":
        qn = canonical_norm64(np.asarray(q, np.float32).reshape(1, -1))[0]
        xn = canonical_norm64(X) if xnorm64 is None else xnorm64
        return canonical_dot64(q, X) / (np.maximum(qn, EPS) * np.maximum(xn, EPS))
    if metric == "euclidean":
        return -canonical_sqdist64(q, X)
    raise RuntimeError("Keine kompilierte Ähnlichkeitsfunktion verfügbar.")


def exact_topk_from_keys(keys: np.ndarray, k: int):
    """Stable order by (key desc, row asc); returns local positions."""
    order = np.lexsort((np.arange(keys.shape[0]), -keys))
    return order[:k]


def keys_to_scores(keys: np.ndarray, metric: str) -> np.ndarray:
    """What the store returns: cosine similarity, or sqrt of the squared distance (fp32)."""
    if metric == "cosine":
        return keys.astype(np.float32)
    return np.sqrt(-keys).astype(np.float32)


def exact_search(queries: np.ndarray, vectors: np.ndarray, k: int, metric: str = "cosine",
                 row_mask: np.ndarray | None = None, chunk: int = 1 << 17):
    """The contract for B queries: (scores f32 [B,k], indices i64 [B,k], keys f64 [B,k]);
    slots past the eligible row count are index -1 / score 0 / key -inf.

    Scales to BASELINE.json's full sizes (10M rows): a fp64 BLAS prefilter over row
    chunks (all queries at once; |error| < 1e-9 relative to the score scale) keeps every
    row within a safe margin of each query's k-th prefilter value, and only those rows
    get canonical keys (exact_keys), so the canonical arithmetic never runs over N."""
    Q = np.asarray(queries, dtype=np.float32)
    if Q.ndim == 1:
        Q = Q[None, :]
    V = np.asarray(vectors, dtype=np.float32)
    B, N = Q.shape[0], V.shape[0]
    rows = np.arange(N) if row_mask is None else np.nonzero(row_mask)[0]
    out_s = np.zeros((B, k), np.float32)
    out_i = np.full((B, k), -1, np.int64)
    out_k = np.full((B, k), -np.inf)
    if rows.size == 0:
        return out_s, out_i, out_k
    kk = min(k, rows.size)
    Q64 = Q.astype(np.float64)
    if rows.size <= 4096:
        cands = [np.arange(rows.size)] * B
    else:
        approx = np.empty((rows.size, B))
        xmax2 = 0.0
        for s0 in range(0, rows.size, chunk):
            sel = rows[s0:s0 + chunk]
            blk = V[sel].astype(np.float64) if row_mask is not None else V[s0:s0 + chunk].astype(np.float64)
            dots = blk @ Q64.T
            sq = np.einsum("ij,ij->i", blk, blk)
            xmax2 = max(xmax2, float(sq.max()))
            if metric == "cosine":
                approx[s0:s0 + chunk] = dots / np.maximum(np.sqrt(sq), EPS)[:, None]
            else:
                approx[s0:s0 + chunk] = 2.0 * dots - sq[:, None]
        cands = []
        for b in range(B):
            a = approx[:, b]
            scale = (np.abs(a).max() + (xmax2 if metric != "cosine" else 1.0)) + 1.0
            kth = np.partition(a, -kk)[-kk]
            cands.append(np.nonzero(a >= kth - 1e-9 * scale)[0])
        del approx
    for b in range(B):
        cand = cands[b]
        Vc = V[rows[cand]]
        keys = exact_keys(Q[b], Vc, metric, canonical_norm64(Vc) if metric == "cosine" else None)
        sel = exact_topk_from_keys(keys, kk)
        out_i[b, :kk] = rows[cand[sel]]
        out_k[b, :kk] = keys[sel]
        out_s[b, :kk] = keys_to_scores(keys[sel], metric)
    return out_s, out_i, out_k


def merge_topk(keys_lists: np.ndarray, idx_lists: np.ndarray, k: int):
    """Merge per-shard lists [G, B, k_in] by (key desc, index asc) -> [B, k] (multi-GPU check)."""
    G, B, kin = keys_lists.shape
    keys = np.transpose(keys_lists, (1, 0, 2)).reshape(B, G * kin)
    idx = np.transpose(idx_lists, (1, 0, 2)).reshape(B, G * kin)
    out_k = np.full((B, k), -np.inf)
    out_i = np.full((B, k), -1, np.int64)
    for b in range(B):
        valid = idx[b] >= 0
        kb, ib = keys[b][valid], idx[b][valid]
        order = np.lexsort((ib, -kb))[:k]
        out_k[b, :order.size] = kb[order]
        out_i[b, :order.size] = ib[order]
    return out_k, out_i


# ---------------------------------------------------------------------------------
# Graph path (performance/hnsw_index.py:79-103 -> hnswlib knn_query).  hnswlib is
# absent, so this restates its published level-0 search
# (hnswalg.h searchBaseLayerST: a min-heap of candidates, a bounded max-heap of
# the ef best results, a visited set; stop when the nearest unexpanded candidate
# is farther than the worst result of a full set) over the same flat neighbour
# array and entry rows the GPU path searches.  Parity for HNSW is unpinned: the
# checks are recall against exact search and agreement with this restatement.
# ---------------------------------------------------------------------------------
def graph_search(vectors: np.ndarray, nbr: np.ndarray, entries: np.ndarray, query: np.ndarray, k: int, ef: int,
                 metric: str = "cosine", inv_norms: np.ndarray | None = None):
    """One query.  Returns (labels int64 [k] (-1 padded), distances fp32 [k] with
    hnswlib conventions: cosine 1 - cos, l2 squared), plus the number of rows scored.
    inv_norms: 1 / max(|x|, 1e-8) per row, precomputed once per corpus (cosine)."""
    import heapq
    V = np.asarray(vectors, np.float32)
    q = np.asarray(query, np.float32).reshape(-1)
    if metric == "cosine":
        qn = q / max(float(np.linalg.norm(q)), 1e-8)
        inv = inv_norms if inv_norms is not None else 1.0 / np.maximum(np.linalg.norm(V, axis=1), 1e-8)

        def dist(rows):
            return 1.0 - (V[rows] @ qn) * inv[rows]
    else:
        def dist(rows):
            d = V[rows] - q
            return np.einsum("ij,ij->i", d, d)
    ent = np.asarray(entries, np.int64)
    de = dist(ent)
    visited = set(ent.tolist())
    cand = [(float(d), int(r)) for d, r in zip(de, ent)]
    heapq.heapify(cand)
    res = [(-d, -r) for d, r in sorted(cand)[:ef]]  # max-heap on (dist, row)
    heapq.heapify(res)
    scored = len(ent)
    while cand:
        d, r = heapq.heappop(cand)
        if len(res) >= ef and (d, r) > (-res[0][0], -res[0][1]):
            break
        nb = [int(x) for x in nbr[r] if x >= 0 and int(x) not in visited]
        if not nb:
            continue
        visited.update(nb)
        dn = dist(np.asarray(nb, np.int64))
        scored += len(nb)
        for dv, rv in zip(dn.tolist(), nb):
            if len(res) < ef or (dv, rv) < (-res[0][0], -res[0][1]):
                heapq.heappush(cand, (dv, rv))
                heapq.heappush(res, (-dv, -rv))
                if len(res) > ef:
                    heapq.heappop(res)
    best = sorted((-a, -b) for a, b in res)[:k]
    labels = np.full(k, -1, np.int64)
    dists = np.full(k, np.inf, np.float32)
    for i, (dv, rv) in enumerate(best):
        labels[i], dists[i] = rv, dv
    if metric != "cosine":
        dists = np.maximum(dists, 0.0)
    return labels, dists, scored


# ---------------------------------------------------------------------------------
# Graph build (performance/hnsw_index.py:44-77 -> hnswlib init_index(M=16,
# ef_construction=200) + add_items).  hnswlib is absent (the reference
# does not pin a version: requirements list `hnswlib` unversioned), so this restates
# its published neighbour selection, getNeighborsByHeuristic2 (hnswalg.h: walk the
# candidates nearest first, keep c unless an already kept r is closer to c than the
# node is, dist(c, r) < dist(c, node), stop at M kept; keepPrunedConnections tops the
# list up with the nearest pruned), in the form the device build runs it
# (vdb_graph.hip graph_prune_kernel, vdb_api.cpp vdb_graph_build): one level of
# out-degree R = 2M, pass 1 selects <= M out-edges from each row's exact kNN, pass 2
# re-selects <= R from out- plus in-edges (hnswlib's level-0 lists after the later
# insertions' links), entry rows evenly spread.
#
# Distances come from fp32 dot products of the stored rows, combined in fp32 as the
# kernel does (cosine 1 - (g * s_c) * s_r with s = fp32 1 / max(|x|, 1e-8); L2
# fma(-2, g, |x_c|^2 + |x_r|^2) with fp32 |x|^2).  The dot products are taken in
# fp64 and rounded to fp32: bit-identical to the kernel's MFMA sums whenever they are
# exact (integer-valued rows, the test's pin); otherwise within fp32 rounding, and
# comparisons that close are reported as ambiguous.
# ---------------------------------------------------------------------------------
def _row_scales(X: np.ndarray, metric: str) -> np.ndarray:
    """pack_rows_kernel's fp32 row scale: cosine 1 / max(|x|, 1e-8), L2 |x|^2 (canonical fp64 sums)."""
    ss = canonical_sumsq64(X)
    if metric == "cosine":
        return (1.0 / np.maximum(np.sqrt(ss), EPS)).astype(np.float32)
    return ss.astype(np.float32)


def _fp32_dist_matrix(gram: np.ndarray, sc: np.ndarray, metric: str) -> np.ndarray:
    """D[c, r] = the kernel's fp32 distance between Gram rows c and r with c's scale applied
    first: cosine 1 - (g * s_c) * s_r, L2 fmaf(-2, g, s_c + s_r) (one rounding)."""
    g = gram.astype(np.float32)
    sc = sc.astype(np.float32)
    if metric == "cosine":
        return (np.float32(1.0) - (g * sc[:, None]) * sc[None, :]).astype(np.float32)
    s = (sc[:, None] + sc[None, :]).astype(np.float32)
    return (-2.0 * g.astype(np.float64) + s.astype(np.float64)).astype(np.float32)


def select_neighbors(X: np.ndarray, scales: np.ndarray, node: int, cands, limit: int, metric: str = "cosine",
                     fill: bool = False, sort: bool = False, tol: float = 0.0):
    """hnswlib's getNeighborsByHeuristic2 for one node over <= 63 candidate rows (-1 padded
    at the tail), as graph_prune_kernel: visiting order = candidate order (the kNN lists
    arrive nearest first) or, with sort, by (fp32 distance to the node, position).
    Returns (rows int32 [limit] -1 padded, fp32 distances [limit] inf padded, ambiguous):
    ambiguous = some decision compared two distances within `tol` (fp32 rounding)."""
    cands = [int(c) for c in cands][:63]
    nvalid = 0
    while nvalid < len(cands) and cands[nvalid] >= 0:
        nvalid += 1
    valid_pos = [i for i, c in enumerate(cands) if c >= 0] if sort else list(range(nvalid))
    rows = np.asarray([node] + [cands[i] for i in valid_pos], np.int64)
    Xr = np.asarray(X, np.float32)[rows].astype(np.float64)
    Dm = _fp32_dist_matrix(Xr @ Xr.T, scales[rows], metric).astype(np.float64)
    d0 = Dm[:, 0]  # my_d0 of lane c: (g[0, c] * s_c) * s_node
    amb = False
    order = list(range(1, len(rows)))
    if sort:
        order.sort(key=lambda i: (d0[i], valid_pos[i - 1]))
        if tol > 0:
            ds = d0[order]
            amb |= bool(np.any((np.abs(np.diff(ds)) <= tol) & (np.diff(ds) != 0)))
    kept = []
    for c in order:
        if len(kept) >= limit:
            break
        if kept:
            dcr = Dm[c, kept]
            if tol > 0 and np.any(np.abs(dcr - d0[c]) <= tol):
                amb = True
            if np.any(dcr < d0[c]):
                continue
        kept.append(c)
    if fill:
        for c in order:
            if len(kept) >= limit:
                break
            if c not in kept:
                kept.append(c)
    rank = {c: j for j, c in enumerate(order)}
    kept.sort(key=lambda c: rank[c])  # nearest first = visiting order
    out = np.full(limit, -1, np.int32)
    dist = np.full(limit, np.inf, np.float32)
    for j, c in enumerate(kept):
        out[j] = rows[c]
        dist[j] = d0[c]
    return out, dist, amb


def graph_build(X: np.ndarray, metric: str = "cosine", degree: int = 32, knn: int = 32, n_entries: int = 256,
                fill: bool = False, tol: float = 0.0):
    """vdb_graph_build restated: (neighbours int32 [N, degree], entries int32 [E], ambiguous
    bool [N] = the node's list may differ from the kernel's by fp32 rounding)."""
    X = np.asarray(X, np.float32)
    N = X.shape[0]
    R, F = degree, degree // 2
    scales = _row_scales(X, metric)
    nbr = np.full((N, R), -1, np.int32)
    amb = np.zeros(N, bool)
    if N > 1:
        kk = min(knn + 1, max(N, 1))
        _, kid, _ = exact_search(X, X, kk, metric)
        CW = min(knn, 63)
        fwd = np.full((N, F), -1, np.int32)
        fdist = np.full((N, F), np.inf, np.float32)
        amb1 = np.zeros(N, bool)
        cand1 = []
        for i in range(N):
            c = [int(v) for v in kid[i] if v >= 0 and v != i][:CW]
            cand1.append(c)
            fwd[i], fdist[i], amb1[i] = select_neighbors(X, scales, i, c + [-1] * (CW - len(c)), F, metric,
                                                         tol=tol)
        # pools: out-edges and in-edges, nearest first by (fp32 distance, row), <= 63 distinct
        rev = [[] for _ in range(N)]
        for u in range(N):
            for j in range(F):
                w = int(fwd[u, j])
                if w >= 0:
                    rev[w].append((float(fdist[u, j]), u))
        # a node's pool is uncertain where an ambiguous pass-1 list could have added or dropped it
        touched = np.zeros(N, bool)
        for u in np.nonzero(amb1)[0]:
            touched[u] = True
            for v in cand1[u]:
                touched[v] = True
        for v in range(N):
            pool = [(float(fdist[v, j]), int(fwd[v, j])) for j in range(F) if fwd[v, j] >= 0] + rev[v]
            pool.sort()
            row = []
            for _, u in pool:
                if len(row) >= 63:
                    break
                if u not in row:
                    row.append(u)
            if tol > 0:
                ds = sorted(d for d, _ in pool)
                if any(abs(a - b) <= tol and a != b for a, b in zip(ds, ds[1:])):
                    touched[v] = True
            out, _, a2 = select_neighbors(X, scales, v, row + [-1] * (63 - len(row)), R, metric, fill=fill, tol=tol)
            nbr[v] = out
            amb[v] = a2 or touched[v]
    E = min(n_entries, max(N, 1))
    ent = np.asarray([i * N // E for i in range(E)], np.int32)
    return nbr, ent, amb
