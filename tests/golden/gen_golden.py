"""Generate the committed golden fixtures from the CPU oracle (oracle/ref_cpu.py).

    python tests/golden/gen_golden.py

Each fixture holds inputs (seeded), the exact contract outputs (indices, fp64
keys, fp32 scores) and the reference-arithmetic fp32 outputs.  Inputs follow
the reference harnesses: uniform [0,1) corpus and queries
(benchmarks/large_scale_benchmark.py:59,61; tests/test_integration.py:83), plus
normal data (tests/demo.py:164,215) and crafted ties: duplicate rows, a row
scaled by 2 (same cosine), zero rows and a zero query.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.abspath(os.path.join(HERE, "..", "..")))
from oracle import ref_cpu  # noqa: E402


def make(name, N, D, B, k, metric, dist="uniform", mask_every=0, seed=0):
    rng = np.random.default_rng(seed)
    if dist == "uniform":
        V = rng.random((N, D), dtype=np.float32)
        Q = np.random.default_rng(seed + 1).random((B, D), dtype=np.float32)
    else:
        V = rng.standard_normal((N, D)).astype(np.float32)
        Q = np.random.default_rng(seed + 1).standard_normal((B, D)).astype(np.float32)
    # crafted ties
    V[100:110] = V[50]          # 10 duplicates of row 50 (+ row 50 itself)
    V[200] = 2.0 * V[60]        # same cosine as row 60
    V[300] = 0.0                # zero vector (norm clamped to 1e-8)
    Q[0] = V[50]                # self-query hitting 11 exact ties
    Q[1] = V[60]
    Q[2] = 0.0                  # zero query: every cosine is 0 -> first k eligible rows
    mask = None
    if mask_every:
        mask = (np.arange(N) % mask_every) == 0
    es, ei, ek = ref_cpu.exact_search(Q, V, k, metric, row_mask=mask)
    meta = [{"id": f"doc_{i}"} for i in range(N)]
    filt = None
    rs = np.zeros((B, k), np.float32)
    ri = np.full((B, k), -1, np.int64)
    for b in range(B):
        if mask is not None:
            meta_m = [{"id": f"doc_{i}", "keep": bool(mask[i])} for i in range(N)]
            idx, sc, _ = ref_cpu.reference_store_search(Q[b], V, k, metric, meta_m, {"keep": True})
        else:
            idx, sc, _ = ref_cpu.reference_store_search(Q[b], V, k, metric, meta, filt)
        ri[b, :len(idx)] = idx
        rs[b, :len(sc)] = sc
    path = os.path.join(HERE, f"{name}.npz")
    np.savez_compressed(path, vectors=V, queries=Q, k=np.int64(k), metric=np.array(metric),
                        mask=(mask if mask is not None else np.zeros(0, bool)),
                        exact_idx=ei, exact_keys=ek, exact_scores=es, ref_idx=ri, ref_scores=rs)
    print(name, V.shape, Q.shape, "->", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    make("cosine_2048x384", 2048, 384, 16, 10, "cosine", seed=0)
    make("euclid_2048x128", 2048, 128, 16, 20, "euclidean", seed=10)
    make("cosine_1000x100_normal_mask", 1000, 100, 6, 5, "cosine", dist="normal", mask_every=3, seed=20)
    make("euclid_777x33_normal", 777, 33, 5, 40, "euclidean", dist="normal", seed=30)
