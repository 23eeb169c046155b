"""Multi-rank plumbing of the row-sharded search (service/sharded.py) on CPU:
world_size 2 (and 3) over gloo, 127.0.0.1.  Each rank's local search and the
merge are the oracle here (the GPU versions are covered by
tests/test_gpu_parity.py::test_merge_topk_matches_single_device); what is under
test is the shard split, the global row offsets, the all-gather layout and
that the merged result equals a single search over the whole corpus — ties
across shards included."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import ref_cpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _oracle_merge(g_keys, g_idx, k, out_s, out_i, out_k, metric):
    mk, mi = ref_cpu.merge_topk(g_keys.numpy(), g_idx.numpy(), k)
    out_i.copy_(torch.from_numpy(mi))
    out_s.copy_(torch.from_numpy(np.where(mi >= 0, ref_cpu.keys_to_scores(np.where(mi >= 0, mk, 0.0), metric), 0)
                                 .astype(np.float32)))
    if out_k is not None:
        out_k.copy_(torch.from_numpy(mk))


def _worker(rank, world, port, metric, N, D, B, k, result_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from service.sharded import ShardedSearcher, shard_bounds
    rng = np.random.default_rng(42)
    V = rng.random((N, D), dtype=np.float32)
    V[N - 5:] = V[3]          # exact ties that straddle shards
    Q = rng.random((B, D), dtype=np.float32)
    Q[0] = V[3]
    lo, hi = shard_bounds(N, world, rank)
    Vs = V[lo:hi]

    def local(q, kk, s, i, keys, off):
        es, ei, ek = ref_cpu.exact_search(q.numpy(), Vs, kk, metric)
        i.copy_(torch.from_numpy(np.where(ei >= 0, ei + off, -1)))
        s.copy_(torch.from_numpy(es))
        keys.copy_(torch.from_numpy(ek))

    sh = ShardedSearcher(lo, metric, local, lambda *a: _oracle_merge(*a, metric))
    out_s = torch.empty((B, k), dtype=torch.float32)
    out_i = torch.empty((B, k), dtype=torch.int64)
    out_k = torch.empty((B, k), dtype=torch.float64)
    sh.search(torch.from_numpy(Q), k, out_s, out_i, out_k)
    np.savez(f"{result_path}.{rank}.npz", s=out_s.numpy(), i=out_i.numpy(), k=out_k.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,metric", [(2, "cosine"), (2, "euclidean"), (3, "cosine")])
def test_sharded_search_equals_single(tmp_path, world, metric):
    N, D, B, k = 301, 24, 5, 9
    path = str(tmp_path / "res")
    mp.start_processes(_worker, args=(world, _free_port(), metric, N, D, B, k, path), nprocs=world,
                       join=True, start_method="spawn")
    rng = np.random.default_rng(42)
    V = rng.random((N, D), dtype=np.float32)
    V[N - 5:] = V[3]
    Q = rng.random((B, D), dtype=np.float32)
    Q[0] = V[3]
    es, ei, ek = ref_cpu.exact_search(Q, V, k, metric)
    for r in range(world):
        z = np.load(f"{path}.{r}.npz")
        np.testing.assert_array_equal(z["i"], ei)
        np.testing.assert_array_equal(z["k"], ek)
        np.testing.assert_array_equal(z["s"], es)
    assert ei[0, :6].tolist() == [3, N - 5, N - 4, N - 3, N - 2, N - 1]


def test_shard_bounds_cover_rows_once():
    from service.sharded import shard_bounds
    for N in (0, 1, 7, 1000, 1001):
        for G in (1, 2, 3, 8):
            seen = []
            for g in range(G):
                lo, hi = shard_bounds(N, G, g)
                assert 0 <= lo <= hi <= N
                seen.extend(range(lo, hi))
            assert seen == list(range(N))
