"""Recall / latency of the graph path vs degree, knn and ef (exploration, not a test)."""
import os, sys, time
import numpy as np
ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path[:0] = [os.path.join(ROOT, "mlx-vector-db_amd"), ROOT]
import torch  # noqa
from service import _vdb
from oracle import ref_cpu
N, D, nq, k = int(sys.argv[1]) if len(sys.argv) > 1 else 20000, int(sys.argv[2]) if len(sys.argv) > 2 else 64, 100, 10
rng = np.random.default_rng(31)
V = rng.random((N, D), dtype=np.float32)
Q = rng.random((nq, D), dtype=np.float32)
ix = _vdb.NativeIndex(D, "cosine")
ix.add(V)
t = time.time()
es, ei, ek = ix.search(Q, k, with_keys=True)
cfgs = [tuple(map(int, c.split("/"))) for c in (sys.argv[3].split(",") if len(sys.argv) > 3 else ["32/32", "32/64", "48/48", "64/64"])]
print(f"exact ground truth {time.time() - t:.2f}s", flush=True)
for deg, knn in cfgs:
    t0 = time.time()
    g = _vdb.NativeGraph.build(ix, degree=deg, knn=knn)
    tb = time.time() - t0
    for ef in (64, 128, 256):
        g.search(Q[:2], k, ef)
        t0 = time.time()
        lab, dist = g.search(Q, k, ef)
        tq = time.time() - t0
        lat = []
        for i in range(10):
            t1 = time.time(); g.search(Q[i], k, ef); lat.append(time.time() - t1)
        r = sum(len(set(a.tolist()) & set(b.tolist())) for a, b in zip(lab, ei)) / (nq * k)
        it = g.stat("iterations") / max(g.stat("queries"), 1)
        print(f"N={N} D={D} deg={deg} knn={knn} ef={ef}: recall@10 {r:.3f}  batch100 {tq*1e3:.1f} ms  b1 p50 {np.median(lat)*1e3:.3f} ms  iters/q {it:.0f}  build {tb:.1f}s", flush=True)
    g.close()
