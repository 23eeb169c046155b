"""Round 6 serving diagnosis at C2 (1M x 768 cosine, k = 10): where a single-vector query's time
goes -- the store wrapper, the native host-memory search, the device-memory search -- and how
four threads scale on each layer.

    python profiles/scripts/serving_diag6.py
"""
import os, sys, time, shutil, tempfile
import numpy as np
ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(ROOT, "mlx-vector-db_amd")); sys.path.insert(0, ROOT)
from concurrent.futures import ThreadPoolExecutor
import torch
import bench
from service import _vdb
from service.optimized_vector_store import MLXVectorStore, MLXVectorStoreConfig

N, D, B, k, metric, _ = bench.CONFIGS["c2"]
V = bench.corpus_rows(N, D, 0, N)
Qs = np.random.default_rng(2).random((800, D), dtype=np.float32)


def p50(fn, n=200):
    for i in range(10):
        fn(i)
    t = []
    for i in range(n):
        t0 = time.perf_counter(); fn(i); t.append(time.perf_counter() - t0)
    return np.median(t) * 1e3, np.percentile(t, 90) * 1e3


def qps4(fn, n=800):
    with ThreadPoolExecutor(4) as ex:
        t0 = time.perf_counter()
        list(ex.map(fn, range(n)))
        return n / (time.perf_counter() - t0)


ix = _vdb.NativeIndex(D, metric)
ix.add(V)
ix.search(Qs[:64], k)
print("native host B=1     p50 %.3f p90 %.3f ms" % p50(lambda i: ix.search(Qs[i % 800][None], k)), flush=True)
for b in (2, 4, 8):
    print(f"native host B={b}     p50 %.3f p90 %.3f ms" % p50(lambda i: ix.search(Qs[(i * b) % 792:(i * b) % 792 + b], k)), flush=True)
qd = torch.from_numpy(Qs).cuda()
sd = torch.empty((800, k), device="cuda"); idd = torch.empty((800, k), dtype=torch.int64, device="cuda")
st = torch.cuda.Stream()


def dev1(i):
    ix.search_device(qd[i % 800].data_ptr(), 1, k, sd[i % 800].data_ptr(), idd[i % 800].data_ptr(), stream=st.cuda_stream)
    st.synchronize()


print("native device B=1   p50 %.3f p90 %.3f ms" % p50(dev1), flush=True)
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
tl = []
for i in range(100):
    ev[0].record(st); ix.search_device(qd[i].data_ptr(), 1, k, sd[i].data_ptr(), idd[i].data_ptr(), stream=st.cuda_stream)
    ev[1].record(st); st.synchronize(); tl.append(ev[0].elapsed_time(ev[1]))
print("device time B=1     p50 %.3f ms (HIP events around the device-memory search)" % np.median(tl), flush=True)
for rep in range(2):
    print(f"rep {rep}: 4 threads native host B=1 %.0f QPS" % qps4(lambda i: ix.search(Qs[i % 800][None], k)), flush=True)
    strs = [torch.cuda.Stream() for _ in range(4)]
    import threading
    tid = {}

    def devq(i):
        s = strs[tid.setdefault(threading.get_ident(), len(tid)) % 4]
        ix.search_device(qd[i % 800].data_ptr(), 1, k, sd[i % 800].data_ptr(), idd[i % 800].data_ptr(), stream=s.cuda_stream)
        s.synchronize()
    print(f"rep {rep}: 4 threads native device B=1 %.0f QPS" % qps4(devq), flush=True)
ix.close()
tmp = tempfile.mkdtemp(prefix="vdb_serving_diag_")
try:
    store = MLXVectorStore(tmp, MLXVectorStoreConfig(dimension=D, metric=metric, persist=False))
    store.add_vectors(V, [{}] * N)
    store.config.coalesce = False
    print("store direct B=1    p50 %.3f p90 %.3f ms" % p50(lambda i: store.query(Qs[i % 800], k)), flush=True)
    store.config.coalesce = True
    print("store coalesced B=1 p50 %.3f p90 %.3f ms" % p50(lambda i: store.query(Qs[i % 800], k)), flush=True)
    store._index.close()
finally:
    shutil.rmtree(tmp, ignore_errors=True)
