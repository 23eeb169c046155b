"""Per-wave cycle breakdown of scan_topk (diagnostic stamp build, lib/libvdb_amd_stamp.so)."""
import ctypes, os, sys
import numpy as np
ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
os.environ["VDB_LIB"] = os.path.join(ROOT, "mlx-vector-db_amd", "lib", "libvdb_amd_stamp.so")
sys.path.insert(0, os.path.join(ROOT, "mlx-vector-db_amd")); sys.path.insert(0, ROOT)
import torch  # noqa
from service import _vdb
import bench
variant = int(sys.argv[1]) if len(sys.argv) > 1 else 0
nwg = int(sys.argv[2]) if len(sys.argv) > 2 else 0
prec = sys.argv[3] if len(sys.argv) > 3 else "bf16x3"
cfg = sys.argv[4] if len(sys.argv) > 4 else "c2"
N, D, B, k, metric, _ = bench.CONFIGS[cfg]
ix = _vdb.NativeIndex(D, metric, precision=prec)
ix.set_param("scan_variant" if prec == "fp32" else "scan_variant_bf16x3", variant)
if nwg: ix.set_param("n_wg", nwg)
ix.reserve(N)
for s in range(0, N, 1 << 19):
    ix.add(bench.corpus_rows(N, D, s, min(s + (1 << 19), N)))
Q = np.random.default_rng(1).random((B, D), dtype=np.float32)
for _ in range(3):
    ix.search(Q, k)
lib = _vdb.load_library()
n = 1 << 16
buf = (ctypes.c_ulonglong * (n * 8))()
lib.vdb_debug_scan_stamps(buf, n)
a = np.array(buf, dtype=np.uint64).reshape(n, 8).astype(np.float64)
a = a[a[:, 3] > 0]
print(f"{cfg} {prec} variant {variant} nwg {nwg}: waves {len(a)}")
for i, name in enumerate(["k-loop", "epilogue", "publish", "total", "barrier after k-loop", "scoring", "first insert pass", "retry loop (+barrier,-pub)"]):
    print(f"  {name:22s} mean {a[:, i].mean():12.0f}  max {a[:, i].max():12.0f}  (ticks)")
print("  k-loop share", a[:, 0].sum() / a[:, 3].sum(), "epilogue share", a[:, 1].sum() / a[:, 3].sum())

# finish_kernel phases (per query): list length, load, select, exact keys, ranks/write, certificate
m = 64
fb = (ctypes.c_ulonglong * (m * 8))()
lib.vdb_debug_finish_stamps(fb, m)
f = np.array(fb, dtype=np.uint64).reshape(m, 8).astype(np.float64)
print("finish: list length mean %.0f max %.0f" % (f[:, 7].mean(), f[:, 7].max()))
for i, name in enumerate(["load list", "select", "exact keys", "ranks+write", "certificate"]):
    d = f[:, i + 1] - f[:, i]
    print(f"  {name:14s} mean {d.mean():9.0f}  max {d.max():9.0f} ticks")
