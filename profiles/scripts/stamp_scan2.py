"""Per-wave phase breakdown of scan2_kernel (diagnostic stamp build lib/libvdb_amd_st.so).

Usage: python profiles/scripts/stamp_scan2.py [config] [precision] [param=value ...]
"""
import ctypes, os, sys
import numpy as np
ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
os.environ["VDB_LIB"] = os.path.join(ROOT, "mlx-vector-db_amd", "lib", "libvdb_amd_st.so")
sys.path.insert(0, os.path.join(ROOT, "mlx-vector-db_amd")); sys.path.insert(0, ROOT)
import torch  # noqa
from service import _vdb
import bench

cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
prec = sys.argv[2] if len(sys.argv) > 2 else "bf16"
params = dict(a.split("=") for a in sys.argv[3:])
N, D, B, k, metric, _ = bench.CONFIGS[cfg]
ix = _vdb.NativeIndex(D, metric, precision=prec)
for kk, v in params.items():
    ix.set_param(kk, int(v))
ix.reserve(N)
for s in range(0, N, 1 << 19):
    ix.add(bench.corpus_rows(N, D, s, min(s + (1 << 19), N)))
Q = np.random.default_rng(1).random((B, D), dtype=np.float32)
for _ in range(4):
    ix.search(Q, k)
lib = _vdb.load_library()
n = 1 << 16
a = np.zeros((n, 8))
for unit in ("b3c", "b3l", "b1c", "b1l"):  # one stamp buffer per instantiation unit
    buf = (ctypes.c_ulonglong * (n * 8))()
    getattr(lib, f"vdb_debug_scan2_stamps_{unit}")(buf, n)
    u = np.array(buf, dtype=np.uint64).reshape(n, 8).astype(np.float64)
    if u[:, 3].sum() > a[:, 3].sum():
        a = u
a = a[a[:, 3] > 0]
t0 = a[:, 7] - a[:, 7].min()
end = t0 + a[:, 3]
print(f"{cfg} {prec} {params}: waves {len(a)}, steps/wave mean {a[:, 6].mean():.2f} max {a[:, 6].max():.0f}")
for i, name in enumerate(["prologue", "k-loop", "epilogue", "total", "publish", "flush"]):
    print(f"  {name:10s} mean {a[:, i].mean():10.0f}  max {a[:, i].max():10.0f}  share {a[:, i].sum() / a[:, 3].sum():.3f}")
print(f"  start skew: mean {t0.mean():.0f} max {t0.max():.0f}; end: min {end.min():.0f} mean {end.mean():.0f} max {end.max():.0f}")
per_step = a[:, 1] / np.maximum(a[:, 6], 1)
print(f"  k-loop per step: mean {per_step.mean():.0f} min {per_step.min():.0f} max {per_step.max():.0f}")
