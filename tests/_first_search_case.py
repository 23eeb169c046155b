"""One case of tests/test_gpu_guards.py::test_first_search_in_a_fresh_process, run in a fresh
process: argv = precision metric qlds D.  The FIRST search of the process must equal the
oracle (indices and fp64 keys); prints 'FIRST OK' and exits 0, else exits 1.

Data: 30 000 uniform rows with planted duplicates, shard [0, 15 000) searched (the round-3
failing case, test_two_ranks_one_gpu_equal_single's rank 0 shard), 20 queries, k = 12.
"""
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
for p in (os.path.join(ROOT, "mlx-vector-db_amd"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402

from oracle import ref_cpu  # noqa: E402
from service import _vdb  # noqa: E402


def main():
    precision, metric, qlds, D = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
    N, B, k = 30000, 20, 12
    rng = np.random.default_rng(7)
    V = rng.random((N, D), dtype=np.float32)
    V[N // 2 - 3:N // 2 + 3] = V[11]
    Q = rng.random((B, D), dtype=np.float32)
    Q[0] = V[11]
    S = V[:15000]
    es, ei, ek = ref_cpu.exact_search(Q, S, k, metric)
    ix = _vdb.NativeIndex(D, metric, 0, precision=precision)
    ix.set_param("scan_qlds", qlds)
    ix.add(S)
    s, i, kk = ix.search(Q, k, with_keys=True)
    wrong = int((i != ei).sum())
    kwrong = int((kk[ei >= 0] != ek[ei >= 0]).sum())
    fb = ix.stat("fallback_queries")
    inc = ix.stat("inconsistent_queries")
    tag = f"{precision} {metric} qlds {qlds} D {D}: wrong {wrong}/{i.size} keys {kwrong} fallback {fb} incons {inc}"
    if wrong or kwrong:
        print("FIRST WRONG", tag)
        return 1
    print("FIRST OK", tag)
    return 0


if __name__ == "__main__":
    sys.exit(main())
