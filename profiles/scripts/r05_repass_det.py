"""Round 5: is the I8 pass's certificate outcome for one fixed batch timing-dependent?
The scenario of tests/test_gpu_parity.py::test_device_repass_of_uncertified_queries, searched
many times, one search at a time (synchronised), per-search deltas of the flag counters."""
import os, sys, json
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "mlx-vector-db_amd"), ROOT, os.path.join(ROOT, "tests")]
import torch
from service import _vdb as vdb
from test_gpu_parity import _graded_neighbours

def scenario(metric):
    rng = np.random.default_rng(47)
    N, D, B, k = 40000, 128, 64, 10
    V = rng.random((N, D), dtype=np.float32)
    V[1000:1300] = _graded_neighbours(rng, V[11], 300)
    Q = rng.random((B, D), dtype=np.float32)
    Q[5] = V[11]
    return V, Q, k

out = {}
for metric in ("cosine", "euclidean"):
    V, Q, k = scenario(metric)
    B = Q.shape[0]
    for mode in ("device_sync", "device_queued", "host_kp128", "host_kp256"):
        ix = vdb.NativeIndex(V.shape[1], metric)
        if mode.startswith("device"):
            ix.set_param("device_repass", 1)
        if mode == "host_kp128":
            ix.set_param("margin", 118)
        if mode == "host_kp256":
            ix.set_param("margin", 246)
        ix.add(V)
        qd = torch.from_numpy(Q).cuda()
        deltas = []
        prev = (0, 0, 0)
        n = 40
        bufs = []
        for it in range(n):
            if mode.startswith("device"):
                sd = torch.empty((B, k), dtype=torch.float32, device="cuda")
                idd = torch.empty((B, k), dtype=torch.int64, device="cuda")
                kd = torch.empty((B, k), dtype=torch.float64, device="cuda")
                ix.search_device(qd.data_ptr(), B, k, sd.data_ptr(), idd.data_ptr(), kd.data_ptr(), stream=0)
                bufs.append(idd)
                if mode == "device_queued":
                    continue
                torch.cuda.synchronize()
            else:
                ix.search(Q, k, with_keys=True)
            cur = (ix.stat("repass_queries"), ix.stat("fallback_queries"), ix.stat("overflow_queries"))
            deltas.append([c - p for c, p in zip(cur, prev)])
            prev = cur
        torch.cuda.synchronize()
        cur = (ix.stat("repass_queries"), ix.stat("fallback_queries"), ix.stat("overflow_queries"))
        rec = {"per_search": deltas, "totals": cur, "searches_i8": ix.stat("searches_i8"),
               "i8_wide": ix.stat("i8_wide"), "incons": ix.stat("inconsistent_queries")}
        out[f"{metric}/{mode}"] = rec
        print(metric, mode, "totals", cur, "i8", rec["searches_i8"], "distinct per-search",
              sorted({tuple(d) for d in deltas}), flush=True)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
with open(os.path.join(ROOT, "gpurun_out", "repass_det.json"), "w") as f:
    json.dump(out, f, indent=1)
