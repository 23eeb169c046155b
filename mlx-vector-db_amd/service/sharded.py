"""Row-sharded search across the GPUs of one node.

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI).
Rank g of G holds corpus rows [g*ceil(N/G), min((g+1)*ceil(N/G), N)) in its own
device index; queries are replicated; each rank searches its shard for the
per-shard top-k with GLOBAL row ids (index_offset) and the fp64 exact ranking
keys, the lists are all-gathered (keys f64 + ids i64 packed as one [2, B, k] int64
buffer: one collective), and every rank merges them on device by (key desc, row
asc) (vdb_merge_topk).  Because shard offsets preserve row order and the keys are
the exact fp64 values, the merged result is bit-identical to a single-GPU search.

The reference is single-device (no distributed code); this is the
MI355X-native scale-out of `optimized_batch_similarity_search`
(performance/mlx_optimized.py:217-248).  The collective is the path's one real
exchange step; there is no all-reduce.
"""
from __future__ import annotations

from typing import Callable, Optional, Tuple

import torch
import torch.distributed as dist

from . import _vdb


def shard_bounds(n_rows: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous row range of `rank` (ceil split, last shards may be short/empty)."""
    per = (n_rows + world - 1) // world
    return min(rank * per, n_rows), min((rank + 1) * per, n_rows)


class ShardedSearcher:
    """Searches this rank's shard and merges with every other rank's.

    local_search(q, k, out_scores, out_idx, out_keys, index_offset) fills [B, k]
    outputs for this rank's rows (default: the device index through the C-ABI).
    merge(g_keys[G,B,k], g_idx[G,B,k], k, out_scores, out_idx, out_keys) merges the
    gathered lists (default: vdb_merge_topk on device).  Both are injectable so the
    collective plumbing can be tested with gloo on CPU (tests/test_sharded.py).
    """

    def __init__(self, row_offset: int, metric: str, local_search: Callable, merge: Optional[Callable] = None,
                 group=None):
        self.row_offset = int(row_offset)
        self.metric = metric
        self.local_search = local_search
        self.merge = merge or self._device_merge
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self._bufs = {}

    @classmethod
    def from_index(cls, index: "_vdb.NativeIndex", row_offset: int, group=None) -> "ShardedSearcher":
        def local(q, k, s, i, kk, off):
            stream = torch.cuda.current_stream(q.device).cuda_stream
            index.search_device(q.data_ptr(), q.shape[0], k, s.data_ptr(), i.data_ptr(), kk.data_ptr(),
                                index_offset=off, stream=stream)
        return cls(row_offset, index.metric, local, None, group)

    def _device_merge(self, g_keys, g_idx, k, out_s, out_i, out_k):
        stream = torch.cuda.current_stream(g_keys.device).cuda_stream
        _vdb.merge_topk_device(g_keys.data_ptr(), g_idx.data_ptr(), g_keys.shape[0], g_keys.shape[1],
                               g_keys.shape[2], k, self.metric, out_s.data_ptr(), out_i.data_ptr(),
                               out_k.data_ptr() if out_k is not None else 0, stream)

    def _buffers(self, B: int, k: int, device):
        # per stream: searches queued on several streams (bench.py --streams) each need their own.
        # The local keys (f64) and ids (i64) share one [2, B, k] int64 buffer, so ONE all-gather
        # moves both ([G, 2, B, k]): the exchange is latency-bound on xGMI (C4: 819 KB per rank,
        # c6 at 8 GPUs: 10 KB), so one collective instead of two halves its cost per batch.
        stream = torch.cuda.current_stream(device).cuda_stream if device.type == "cuda" else 0
        key = (B, k, str(device), stream)
        if key not in self._bufs:
            f = dict(device=device)
            pack = torch.empty((2, B, k), dtype=torch.int64, **f)
            self._bufs[key] = (
                torch.empty((B, k), dtype=torch.float32, **f), pack,
                torch.empty((self.world, 2, B, k), dtype=torch.int64, **f),
                torch.empty((self.world, B, k), dtype=torch.float64, **f),
                torch.empty((self.world, B, k), dtype=torch.int64, **f))
        return self._bufs[key]

    def search(self, q: torch.Tensor, k: int, out_scores: torch.Tensor, out_idx: torch.Tensor,
               out_keys: Optional[torch.Tensor] = None) -> None:
        """q [B, D] (replicated on every rank) -> global top-k in out_* (every rank)."""
        B = q.shape[0]
        ls, pack, gathered, g_keys, g_idx = self._buffers(B, k, q.device)
        lk, li = pack[0].view(torch.float64), pack[1]  # contiguous [B, k] planes of the pack
        self.local_search(q, k, ls, li, lk, self.row_offset)
        if self.world == 1:
            out_scores.copy_(ls)
            out_idx.copy_(li)
            if out_keys is not None:
                out_keys.copy_(lk)
            return
        # [G*2B, k] view: the output split along dim 0 in input-shaped chunks
        if q.is_cuda and dist.get_backend(self.group) == "gloo":
            # gloo moves host memory only (tests run several ranks on one GPU this way; RCCL
            # takes the device buffers directly)
            hg = gathered.cpu()
            dist.all_gather_into_tensor(hg.view(self.world * 2 * B, k), pack.cpu().view(2 * B, k), group=self.group)
            gathered.copy_(hg)
        else:
            dist.all_gather_into_tensor(gathered.view(self.world * 2 * B, k), pack.view(2 * B, k), group=self.group)
        g_keys.copy_(gathered[:, 0].view(torch.float64))
        g_idx.copy_(gathered[:, 1])
        self.merge(g_keys, g_idx, k, out_scores, out_idx, out_keys)
