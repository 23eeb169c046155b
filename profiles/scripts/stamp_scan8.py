"""Per-wave phase breakdown of scan8_kernel (diagnostic stamp build lib/libvdb_amd_st8.so,
make variant VTAG=st8 VDEFS=-DVDB_STAMP8): I8 cosine (unit i1c) or I8X3 L2 (unit i3l).

Usage: python profiles/scripts/stamp_scan8.py [config] [i8|i8x3]
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
prec = sys.argv[2] if len(sys.argv) > 2 else "i8"
N, D, B, k, metric, _ = bench.CONFIGS[cfg]
unit = {("i8", "cosine"): "i1c", ("i8x3", "euclidean"): "i3l"}[(prec, metric)]
ix = _vdb.NativeIndex(D, metric, precision=prec)
if os.environ.get("STAMP_CHK") is not None:  # the int8 pass's checksum on / off (A/B)
    ix.set_param("scan_checksum", int(os.environ["STAMP_CHK"]))
ix.reserve(N)
for s in range(0, N, 1 << 19):
    ix.add(bench.corpus_rows(N, D, s, min(s + (1 << 19), N)))
Q = np.random.default_rng(1).random((B, D), dtype=np.float32)
for _ in range(4):
    ix.search(Q, k)
lib = _vdb.load_library()
n = 1 << 16
buf = (ctypes.c_ulonglong * (n * 12))()
getattr(lib, f"vdb_debug_scan8_stamps_{unit}")(buf, n)
raw = np.array(buf, dtype=np.uint64).reshape(n, 12)
out = os.environ.get("STAMP_OUT")
if out:
    np.save(out, raw)
a = raw.astype(np.float64)
live = a[:, 0] > 0
a = a[live]
t0 = a[:, 5] - a[:, 5].min()  # s_memrealtime (100 MHz, one clock for the chip)
end = a[:, 9] - a[:, 5].min()
print(f"{cfg} {prec}: waves {len(a)}, steps/wave mean {a[:, 4].mean():.2f}; ticks (s_memtime) per wave, mean:")
for i, name in ((0, "total"), (1, "stream waits"), (2, "k-loop incl. waits"), (3, "epilogue")):
    print(f"  {name:20s} {a[:, i].mean():12.0f}  per step {a[:, i].mean() / max(a[:, 4].mean(), 1):10.0f}")
sn = max(a[:, 4].mean(), 1)
x, y = a[:, 6].astype(np.uint64), a[:, 7].astype(np.uint64)
print(f"  steps with a passing tile {(x & 0xFFFFF).astype(float).mean() / sn:.3f} of steps; passing tiles per step "
      f"{(x >> 20).astype(float).mean() / sn:.3f}; compaction rounds per wave {(y & 0xFFFFF).astype(float).mean():.1f}")
print(f"  tile tests per step {a[:, 8].mean() / sn:10.0f}; tests + insertions (before the compaction check) per step "
      f"{(y >> 20).astype(float).mean() / sn:10.0f}")
print(f"  after the first insertion round: flag checks / rounds / pacing per step {a[:, 11].mean() / sn:10.0f}; "
      f"the start-value wait per step {a[:, 10].mean() / sn:10.0f}")
print(f"  start spread {t0.max() / 100:.1f} us, end spread {(end.max() - end.min()) / 100:.1f} us, span {end.max() / 100:.1f} us")

# drift between the query blocks of a row range (xcd_map: block L -> j = L / 8, qb = j % n_qb,
# range = 8 (j / n_qb) + L % 8): end times of a range's workgroups, in steps of this wave
n_qb = (B + 63) // 64
if n_qb > 1:
    w = np.nonzero(live)[0]
    L = w // int(os.environ.get('STAMP_NW', '8' if prec == 'i8x3' and metric == 'euclidean' else '4'))
    j = L // 8
    rng_id = 8 * (j // n_qb) + L % 8
    endt = a[:, 9]
    step_rt = ((a[:, 9] - a[:, 5]) / np.maximum(a[:, 4], 1)).mean()  # real-time ticks per step
    spans = []
    for r in np.unique(rng_id):
        e = endt[rng_id == r]
        spans.append((e.max() - e.min()) / step_rt)
    spans = np.array(spans)
    print(f"  query blocks per range {n_qb}: end-time spread within a range, in steps: "
          f"mean {spans.mean():.1f}, max {spans.max():.1f} (of {a[:, 4].mean():.0f} steps)")
