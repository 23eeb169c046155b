"""Round 6 store-level serving A/B: C2's corpus through the drop-in store, 4 query threads,
coalesced with (max_inflight, linger_us) settings against direct calls, interleaved twice.

    python profiles/scripts/serving_ab6.py [n_queries]
"""
import os, sys, time, shutil, tempfile
import numpy as np
ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(ROOT, "mlx-vector-db_amd")); sys.path.insert(0, ROOT)
from concurrent.futures import ThreadPoolExecutor
import bench
from service.optimized_vector_store import MLXVectorStore, MLXVectorStoreConfig

nq = int(sys.argv[1]) if len(sys.argv) > 1 else 800
N, D, B, k, metric, _ = bench.CONFIGS["c2"]
V = bench.corpus_rows(N, D, 0, N)
tmp = tempfile.mkdtemp(prefix="vdb_serving_ab_")
try:
    st = MLXVectorStore(tmp, MLXVectorStoreConfig(dimension=D, metric=metric, persist=False))
    st.add_vectors(V, [{}] * N)
    Qs = np.random.default_rng(2).random((nq, D), dtype=np.float32)
    for q in Qs[:10]:
        st.query(q, k)
    lat = []
    for q in Qs[:100]:
        t0 = time.perf_counter(); st.query(q, k); lat.append(time.perf_counter() - t0)
    print(f"batch-1 p50 {np.median(lat) * 1e3:.3f} ms", flush=True)
    for rep in range(2):
        for mode in ((2, 300), (2, 100), (2, 600), (3, 300), (2, 0), (1, 200)):
            st.config.coalesce = mode != "direct"
            if mode != "direct":
                st._coalescer._inflight, st._coalescer._linger = mode[0], mode[1] * 1e-6
                st._coalescer._recent.clear()
            b0, q0 = st._coalescer.batches, st._coalescer.queries
            with ThreadPoolExecutor(4) as ex:
                t0 = time.perf_counter()
                list(ex.map(lambda q: st.query(q, k), Qs))
                dt = time.perf_counter() - t0
            nb = st._coalescer.batches - b0
            mb = (st._coalescer.queries - q0) / max(nb, 1)
            print(f"rep {rep} {str(mode):10s} {nq / dt:9.0f} QPS  mean batch {mb:.2f}", flush=True)
    st._index.close()
finally:
    shutil.rmtree(tmp, ignore_errors=True)
