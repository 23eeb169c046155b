"""Write the C5 experiment input for hnsw_cpu.cpp: bench.py's synthetic corpus (first N
rows of the c5 stream), B uniform queries (seed 1, as bench.py's C5 queries), and their
exact cosine top-k from the oracle.

    python profiles/scripts/hnsw_data.py N B OUT.bin
"""
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from oracle import ref_cpu  # noqa: E402

N, B, out = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
_, D, _, k, metric, _ = bench.CONFIGS["c5"]
V = np.concatenate([bench.corpus_rows(N, D, s, min(s + 8 * bench.CHUNK_ROWS, N))
                    for s in range(0, N, 8 * bench.CHUNK_ROWS)])
Q = np.random.default_rng(1).random((B, D), dtype=np.float32)
_, gt, _ = ref_cpu.exact_search(Q, V, k, metric)
with open(out, "wb") as f:
    np.array([N, D, B, k], np.int64).tofile(f)
    V.astype(np.float32).tofile(f)
    Q.astype(np.float32).tofile(f)
    gt.astype(np.int64).tofile(f)
print("wrote", out, V.shape, Q.shape)
