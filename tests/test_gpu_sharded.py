"""The multi-rank searcher (service/sharded.py) with its device parts: two rank processes on
one GPU, each with its own device index over its row shard, device searches with global
row offsets, the all-gather (gloo, host-staged: RCCL refuses two ranks on one device) and the
device merge (vdb_merge_topk).  The result must equal the oracle over the whole corpus bit for
bit, ties across the shard boundary included.  On the 8-GPU node the same code runs with
RCCL taking the device buffers directly (bench.py --gpus N)."""
import os
import socket

import numpy as np
import pytest

from oracle import ref_cpu

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data(N, D, B):
    rng = np.random.default_rng(7)
    V = rng.random((N, D), dtype=np.float32)
    V[N // 2 - 3:N // 2 + 3] = V[11]  # exact ties straddling the shard boundary
    Q = rng.random((B, D), dtype=np.float32)
    Q[0] = V[11]
    return V, Q


def _rank(rank, world, port, metric, N, D, B, k, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from service import _vdb
    from service.sharded import ShardedSearcher, shard_bounds
    V, Q = _data(N, D, B)
    lo, hi = shard_bounds(N, world, rank)
    ix = _vdb.NativeIndex(D, metric, 0)
    ix.add(V[lo:hi])
    sh = ShardedSearcher.from_index(ix, lo)
    q = torch.from_numpy(Q).cuda()
    s = torch.empty((B, k), dtype=torch.float32, device="cuda")
    i = torch.empty((B, k), dtype=torch.int64, device="cuda")
    kk = torch.empty((B, k), dtype=torch.float64, device="cuda")
    sh.search(q, k, s, i, kk)
    torch.cuda.synchronize()
    np.savez(f"{out}.{rank}.npz", s=s.cpu().numpy(), i=i.cpu().numpy(), k=kk.cpu().numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(240)
@pytest.mark.parametrize("metric", ["cosine", "euclidean"])
def test_two_ranks_one_gpu_equal_single(tmp_path, metric):
    import torch.multiprocessing as mp
    N, D, B, k = 30000, 96, 20, 12
    out = str(tmp_path / "res")
    mp.start_processes(_rank, args=(2, _free_port(), metric, N, D, B, k, out), nprocs=2, join=True,
                       start_method="spawn")
    V, Q = _data(N, D, B)
    es, ei, ek = ref_cpu.exact_search(Q, V, k, metric)
    for r in range(2):
        z = np.load(f"{out}.{r}.npz")
        np.testing.assert_array_equal(z["i"], ei)
        np.testing.assert_array_equal(z["k"], ek)
