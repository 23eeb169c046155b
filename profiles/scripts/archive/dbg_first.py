"""Debug: the first search of a fresh process (one case per process): precision / metric /
query block in LDS or not; host memory, shard [0, 15000) of test_two_ranks_one_gpu_equal_single."""
import os, sys, subprocess
ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
if len(sys.argv) == 1:
    cases = [("euclidean", "i8", -1)] * 4 + [("cosine", "i8", -1)]
    L = os.path.join(ROOT, "mlx-vector-db_amd", "lib")
    libs = {"fixed": None, "onep+fixed": os.path.join(L, "libvdb_amd_onep.so")}
    for tag, lib in libs.items():
        env = dict(os.environ)
        if lib:
            env["VDB_LIB"] = lib
        for c in cases:
            r = subprocess.run([sys.executable, __file__, *map(str, c)], capture_output=True, text=True, timeout=120, env=env)
            print(tag, r.stdout.strip() or r.stderr[-400:], flush=True)
    sys.exit(0)
import numpy as np
sys.path.insert(0, os.path.join(ROOT, "mlx-vector-db_amd")); sys.path.insert(0, ROOT)
from service import _vdb
from oracle import ref_cpu
metric, prec, qlds = sys.argv[1], sys.argv[2], int(sys.argv[3])
knob = (sys.argv[4], int(sys.argv[5])) if len(sys.argv) > 5 else None
N, D, B, k = 30000, 96, 20, 12
rng = np.random.default_rng(7)
V = rng.random((N, D), dtype=np.float32)
V[N // 2 - 3:N // 2 + 3] = V[11]
Q = rng.random((B, D), dtype=np.float32)
Q[0] = V[11]
S = V[:15000]
es, ei, ek = ref_cpu.exact_search(Q, S, k, metric)
ix = _vdb.NativeIndex(D, metric, 0, precision=prec)
ix.set_param("scan_qlds", qlds)
if knob:
    ix.set_param(*knob)
ix.add(S)
res = []
for _ in range(2):
    s, i, kk = ix.search(Q, k, with_keys=True)
    res.append((i == ei).mean())
print(f"{metric} {prec} qlds {qlds} {knob}: first {res[0]:.3f} second {res[1]:.3f} fallback {ix.stat('fallback_queries')}")
