"""Per-wave phase breakdown of scan8_kernel, I8 cosine (diagnostic stamp build lib/libvdb_amd_st8.so,
make variant VTAG=st8 VDEFS=-DVDB_STAMP8).

Usage: python profiles/scripts/stamp_scan8.py [config]
"""
import ctypes, os, sys
import numpy as np
ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
os.environ["VDB_LIB"] = os.path.join(ROOT, "mlx-vector-db_amd", "lib", "libvdb_amd_st8.so")
sys.path.insert(0, os.path.join(ROOT, "mlx-vector-db_amd")); sys.path.insert(0, ROOT)
import torch  # noqa
from service import _vdb
import bench

cfg = sys.argv[1] if len(sys.argv) > 1 else "c6"
N, D, B, k, metric, _ = bench.CONFIGS[cfg]
ix = _vdb.NativeIndex(D, metric, precision="i8")
ix.reserve(N)
for s in range(0, N, 1 << 19):
    ix.add(bench.corpus_rows(N, D, s, min(s + (1 << 19), N)))
Q = np.random.default_rng(1).random((B, D), dtype=np.float32)
for _ in range(4):
    ix.search(Q, k)
lib = _vdb.load_library()
n = 1 << 16
buf = (ctypes.c_ulonglong * (n * 10))()
lib.vdb_debug_scan8_stamps_i1c(buf, n)
a = np.array(buf, dtype=np.uint64).reshape(n, 10).astype(np.float64)
a = a[a[:, 0] > 0]
t0 = a[:, 5] - a[:, 5].min()
end = t0 + a[:, 0]
print(f"{cfg} i8: waves {len(a)}, steps/wave mean {a[:, 4].mean():.2f}; ticks (s_memtime) per wave, mean:")
for i, name in ((0, "total"), (1, "stream waits"), (2, "k-loop incl. waits"), (3, "epilogue")):
    print(f"  {name:20s} {a[:, i].mean():12.0f}  per step {a[:, i].mean() / max(a[:, 4].mean(), 1):10.0f}")
sn = max(a[:, 4].mean(), 1)
x, y = a[:, 6].astype(np.uint64), a[:, 7].astype(np.uint64)
print(f"  steps with a passing tile {(x & 0xFFFFF).astype(float).mean() / sn:.3f} of steps; passing tiles per step "
      f"{(x >> 20).astype(float).mean() / sn:.3f}; compaction rounds per wave {(y & 0xFFFFF).astype(float).mean():.1f}")
print(f"  tile tests per step {a[:, 8].mean() / sn:10.0f}; tests + insertions (before the compaction check) per step "
      f"{(y >> 20).astype(float).mean() / sn:10.0f}")
print(f"  start spread {t0.max():.0f} ticks, end spread {end.max() - end.min():.0f}, span {end.max():.0f}")
