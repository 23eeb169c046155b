"""finish_kernel phase breakdown (diagnostic stamp build, lib/libvdb_amd_stamp.so).

    python profiles/scripts/fin_stamp.py CONFIG PRECISION
Prints per-query candidate-list length and the cycles of load / select / exact keys /
ranks / certificate, averaged over the batch of the last search.
"""
import ctypes, os, sys
import numpy as np
ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
os.environ.setdefault("VDB_LIB", os.path.join(ROOT, "mlx-vector-db_amd", "lib", "libvdb_amd_st.so"))
sys.path.insert(0, os.path.join(ROOT, "mlx-vector-db_amd")); sys.path.insert(0, ROOT)
import torch  # noqa
from service import _vdb
import bench
cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
prec = sys.argv[2] if len(sys.argv) > 2 else "bf16x3"
N, D, B, k, metric, _ = bench.CONFIGS[cfg]
N = int(os.environ.get("FIN_ROWS", N))  # e.g. one rank's shard of a weak-scaled run
B = int(os.environ.get("FIN_B", B))
ix = _vdb.NativeIndex(D, metric, precision=prec)
if os.environ.get("VDB_FIN_REFINE") is not None:
    ix.set_param("i8_refine", int(os.environ["VDB_FIN_REFINE"]))
ix.reserve(N)
for s in range(0, N, 1 << 19):
    ix.add(bench.corpus_rows(N, D, s, min(s + (1 << 19), N)))
Q = np.random.default_rng(1).random((B, D), dtype=np.float32)
for _ in range(3):
    ix.search(Q, k)
lib = _vdb.load_library()
fb = (ctypes.c_ulonglong * (B * 16))()
lib.vdb_debug_finish_stamps(fb, B)
f = np.array(fb, dtype=np.uint64).reshape(B, 16).astype(np.float64)
rs = f[:, 6].astype(np.uint64) >> np.uint64(40)
rt = (f[:, 6].astype(np.uint64) & np.uint64((1 << 40) - 1)).astype(np.float64)
print(f"{cfg} {prec} N {N} B {B}: list length mean {f[:, 7].mean():.0f} p50 {np.median(f[:, 7]):.0f} max {f[:, 7].max():.0f}; "
      f"rerank set mean {rs.astype(float).mean():.1f} max {rs.max()}")
for i, name in enumerate(["load", "select", "cert+refine+cut", "exact keys", "ranks+write"]):
    d = f[:, i + 1] - f[:, i]
    print(f"  {name:16s} mean {d.mean():9.0f}  max {d.max():9.0f}  (s_memtime ticks)")
print(f"    (of which refinement + cut: mean {rt.mean():.0f})")
sub = [("select end -> a_k counts", 2, 13), ("a_k counts -> pre-cert sync", 13, 14), ("pre-cert sync", 14, 15),
       ("cert (tid 0) + sync + refine setup", 15, 8), ("refine rows (wave 0)", 8, 9), ("refine sync", 9, 10),
       ("a'_k counts + sync", 10, 11), ("e2 (tid 0) + sync", 11, 12), ("cut", 12, 3)]
for name, i, j in sub:
    d = f[:, j] - f[:, i]
    if (f[:, i] > 0).all() and (f[:, j] > 0).all():
        print(f"    {name:36s} mean {d.mean():9.0f}  max {d.max():9.0f}")
