"""C5 question: is the recall gap the graph's or the data's?  The same search
kernel (vdb_graph_search) over (a) the device graph (exact kNN + hnswlib's heuristic, one
level) and (b) an hnswlib-style graph (profiles/scripts/hnsw_cpu.cpp: hierarchical
incremental insertion, M=16, efC=200; level-0 lists uploaded, the top-level nodes as
entries), 1M x 384 uniform rows (bench.py's C5 stream), 100 uniform queries (seed 1),
recall@10 against the exact path.

    python profiles/scripts/graph_compare.py HNSW_GRAPH.npz OUT.json
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(ROOT, "mlx-vector-db_amd"))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from service import _vdb  # noqa: E402

N, B, k = 1_000_000, 100, 10
_, D, _, _, metric, _ = bench.CONFIGS["c5"]
ix = _vdb.NativeIndex(D, metric)
ix.reserve(N)
for s in range(0, N, 8 * bench.CHUNK_ROWS):
    ix.add(bench.corpus_rows(N, D, s, min(s + 8 * bench.CHUNK_ROWS, N)))
Q = np.random.default_rng(1).random((B, D), dtype=np.float32)
_, gt = ix.search(Q, k)


def recall(g, ef, teams):
    g.set_param("teams", teams)
    g.search(Q[:4], k, ef)
    t0 = time.perf_counter()
    lab = np.concatenate([g.search(Q[i:i + 1], k, ef)[0] for i in range(B)])
    dt = (time.perf_counter() - t0) / B
    r = sum(len(set(a.tolist()) & set(b.tolist())) for a, b in zip(lab, gt)) / float(gt.size)
    return {"ef": ef, "teams": teams, "recall_at_10": r, "host_ms_per_query": dt * 1e3}


out = {"n_rows": N, "dim": D, "queries": B}
t0 = time.perf_counter()
g1 = _vdb.NativeGraph.build(ix, degree=32, knn=32, n_entries=256)
out["device_graph_build_s"] = time.perf_counter() - t0
out["device_graph"] = [recall(g1, ef, t) for ef in (128, 256) for t in (1, 64)]
print(json.dumps(out["device_graph"]), flush=True)
g1.close()
z = np.load(sys.argv[1], allow_pickle=False)
g2 = _vdb.NativeGraph.from_arrays(ix, z["neighbors"], z["entries"])
out["hnsw_graph"] = [recall(g2, ef, t) for ef in (128, 256) for t in (1, 64)]
print(json.dumps(out["hnsw_graph"]), flush=True)
json.dump(out, open(sys.argv[2], "w"), indent=1)
