"""Debug: rank 1's shard of test_two_ranks_one_gpu_equal_single (euclidean) searched alone, host
and device memory, against the oracle on the shard."""
import os, sys
import numpy as np
ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(ROOT, "mlx-vector-db_amd")); sys.path.insert(0, ROOT)
import torch
from service import _vdb
from oracle import ref_cpu
N, D, B, k = 30000, 96, 20, 12
rng = np.random.default_rng(7)
V = rng.random((N, D), dtype=np.float32)
V[N // 2 - 3:N // 2 + 3] = V[11]
Q = rng.random((B, D), dtype=np.float32)
Q[0] = V[11]
for metric in ("euclidean", "cosine"):
    for lo, hi in ((0, 15000), (15000, 30000)):
        S = V[lo:hi]
        es, ei, ek = ref_cpu.exact_search(Q, S, k, metric)
        for prec in ("auto", "i8", "bf16x3"):
            ix = _vdb.NativeIndex(D, metric, 0, precision=None if prec == "auto" else prec)
            ix.add(S)
            s, i, kk = ix.search(Q, k, with_keys=True)
            h_ok = (i == ei).mean()
            q = torch.from_numpy(Q).cuda()
            sd = torch.empty((B, k), dtype=torch.float32, device="cuda")
            idd = torch.empty((B, k), dtype=torch.int64, device="cuda")
            kd = torch.empty((B, k), dtype=torch.float64, device="cuda")
            ix.search_device(q.data_ptr(), B, k, sd.data_ptr(), idd.data_ptr(), kd.data_ptr(), index_offset=lo)
            torch.cuda.synchronize()
            d_ok = (idd.cpu().numpy() - lo == ei).mean()
            st = {n: ix.stat(n) for n in ("searches_i8", "searches_i8x3", "searches_bf16x3", "fallback_queries")}
            print(f"{metric} shard [{lo},{hi}) {prec}: host match {h_ok:.3f} device match {d_ok:.3f} {st}", flush=True)
            ix.close()
