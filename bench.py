#!/usr/bin/env python3
"""Headline benchmark: brute-force cosine / L2 top-k on MI355X (BASELINE.json).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c1|c2|c3|c4|c5|c6] [--scaling weak|strong]

One "step" = one batch of queries searched against the whole corpus (fused
MFMA candidate scan + exact fp64 rerank; queries, corpus and outputs resident
in HBM).  The default run measures BASELINE.json's metric, both halves:
  * the line itself: configs[1] (C2: 1M x 768 cosine top-10, batch 64) -- at
    N > 1 row-sharded with the batch per GPU fixed ("weak": global batch 64 N);
  * "metric_workload_10m_x_128": the metric's "10M x 128D @8 GPU" workload (c6:
    cosine top-10, batch 64, row-sharded with the global batch fixed at 64).
N>1 (torchrun, one rank per GPU, RCCL; or --gpus N alone, which spawns the
ranks) row-shards the corpus over the ranks (service/sharded.py): each rank
searches its shard, the per-shard top-k lists (fp64 keys + global row ids) are
all-gathered over xGMI and merged on device, bit-identical to one GPU.
--config c4 / c6 default to "strong" scaling (BASELINE's fixed global batch),
the others to "weak".

Throughput (`value`): the K timed batches are queued back to back on the stream
(device-memory searches return without a host wait) between two synchronises;
latency (`p50_ms`) comes from a separate loop that waits for every batch.
Rank 0 prints one JSON line: QPS (whole job), p50 batch latency, the roofline
of the dominant kernel (the scan kernel, HIP-event timed inside the library on
the stream it runs on; named against the implementation's own work and against
SURVEY.md §8(d)'s) and, at N=1, the CPU baseline: the reference's paths restated
in numpy (oracle/ref_cpu.py), timed on this host on a bounded sample, and for
c1/c2 the store-API serving numbers (batch-1 p50, 4-thread query QPS).
"""
import argparse
import glob
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "mlx-vector-db_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402  (loaded before the HIP library: one HIP runtime per process)
import torch.distributed as dist  # noqa: E402

from service import _vdb  # noqa: E402
from service.sharded import ShardedSearcher, shard_bounds  # noqa: E402

METRIC = "QPS + p50 latency, cosine top-10 batch=64: 1M×768D @1 GPU; 10M×128D @8 GPU"
CONFIGS = {
    # name: (N, D, B, k, metric, description); c1-c5 = BASELINE.json configs[0..4], c6 = the
    # second half of BASELINE.json's metric ("cosine top-10 batch=64: ... 10M x 128D @8 GPU")
    "c1": (10_000, 384, 1, 10, "cosine", "10K x 384 cosine top-10, single query"),
    "c2": (1_000_000, 768, 64, 10, "cosine", "1M x 768 fp32 cosine top-10, batch 64"),
    "c3": (1_000_000, 1536, 256, 10, "cosine", "1M x 1536 cosine top-10, batch 256 (auto: int8 candidate pass)"),
    "c4": (10_000_000, 128, 512, 100, "euclidean", "10M x 128 L2 top-100, batch 512, row-sharded"),
    # graph path (performance/hnsw_index.py): batch 1, hnswlib M=16 -> out-degree 2M, efSearch 128
    "c5": (5_000_000, 384, 1, 10, "cosine", "5M x 384 graph index (HNSW M=16) cosine top-10, efSearch=128, batch 1"),
    "c6": (10_000_000, 128, 64, 10, "cosine", "10M x 128 cosine top-10, batch 64, row-sharded (the metric's 8-GPU workload)"),
}
# --gpus N > 1 without --scaling: the configs BASELINE.json quotes with a fixed global batch sharded
# over the GPUs (configs[3] "batch=512 ... sharded across 8"; the metric's "10M x 128D @8 GPU" at
# batch 64) keep that batch (strong scaling); the single-GPU configs run B per GPU (weak scaling)
DEFAULT_SCALING = {"c4": "strong", "c6": "strong"}
GRAPH_M, GRAPH_EF = 16, 128
FP32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md, Peak FP32 (matrix)
BF16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md, Peak BF16 MFMA, dense
I8_MFMA_PEAK_TOPS = 5000.0      # MI355X_MICROARCH.md, I8 MFMA: 2x BF16 per clock (2x the K), dense
HBM_PEAK_GBS = 8000.0           # MI355X_MICROARCH.md, HBM3E peak (spec)
CHUNK_ROWS = 1 << 16
_HOST_CORPUS = {}  # (N, D, lo, hi) -> host parts of a corpus the next sub-record reuses


def corpus_rows(N, D, start, stop, seed=0):
    """Rows [start, stop) of the synthetic corpus: uniform [0,1) fp32 like the
    reference harness (benchmarks/large_scale_benchmark.py:59), generated per
    65536-row chunk from SeedSequence([seed, chunk]) so any shard is reproducible
    without generating the others."""
    out = np.empty((stop - start, D), np.float32)
    c0, c1 = start // CHUNK_ROWS, (stop - 1) // CHUNK_ROWS
    for c in range(c0, c1 + 1):
        lo, hi = c * CHUNK_ROWS, min((c + 1) * CHUNK_ROWS, N)
        blk = np.random.Generator(np.random.PCG64(np.random.SeedSequence([seed, c]))).random((hi - lo, D),
                                                                                            dtype=np.float32)
        a, b = max(lo, start), min(hi, stop)
        out[a - start:b - start] = blk[a - lo:b - lo]
    return out


CLUSTERS, CLUSTER_SIGMA = 10_000, 0.1


def cluster_centres(D, seed=0):
    return np.random.Generator(np.random.PCG64(np.random.SeedSequence([seed, 1 << 30]))).random((CLUSTERS, D),
                                                                                                dtype=np.float32)


def corpus_rows_clustered(N, D, start, stop, seed=0, centres=None):
    """Rows [start, stop) of a structured corpus (the graph's case): each row a
    uniform centre of CLUSTERS plus N(0, CLUSTER_SIGMA^2) per dimension, chunk-seeded like
    corpus_rows so any shard is reproducible alone."""
    C = cluster_centres(D, seed) if centres is None else centres
    out = np.empty((stop - start, D), np.float32)
    c0, c1 = start // CHUNK_ROWS, (stop - 1) // CHUNK_ROWS
    for c in range(c0, c1 + 1):
        lo, hi = c * CHUNK_ROWS, min((c + 1) * CHUNK_ROWS, N)
        g = np.random.Generator(np.random.PCG64(np.random.SeedSequence([seed, c, 7])))
        lab = g.integers(0, CLUSTERS, hi - lo)
        blk = C[lab] + g.standard_normal((hi - lo, D), dtype=np.float32) * np.float32(CLUSTER_SIGMA)
        a, b = max(lo, start), min(hi, stop)
        out[a - start:b - start] = blk[a - lo:b - lo]
    return out


def cpu_baseline(V, Q, k, metric="cosine", budget_s=10.0):
    """BASELINE.md §2, the reference's CPU paths restated in numpy (oracle/ref_cpu.py), each
    timed for about `budget_s` on this host's cores on a BOUNDED sample of the workload (the
    full corpus, a subset of the batch's queries), so the default bench stays within minutes:
      (ii) batched `optimized_batch_similarity_search` (performance/mlx_optimized.py:217-248),
           cosine only (the module has no batched L2): sub-batches of Bs queries (normalise +
           fp32 BLAS matmul + stable argsort of [Bs, N]); Bs = B up to 64M scores per batch;
      (i)  per-query store path `_brute_force_search` (service/optimized_vector_store.py:149-192):
           one query at a time (re-normalise the corpus / direct differences for L2, full stable
           argsort, [:k]).
    `value` is the faster of the two in queries/s."""
    from oracle import ref_cpu
    try:
        from threadpoolctl import threadpool_info
        threads = max([p.get("num_threads", 1) for p in threadpool_info() if p.get("user_api") == "blas"] or [1])
    except Exception:
        threads = int(os.environ.get("OMP_NUM_THREADS", "1"))
    N = V.shape[0]
    B = Q.shape[0]
    res = {"unit": "queries/s", "cores": threads, "kind": "port"}
    parts = []
    batched_qps = 0.0
    if True:
        # cosine: the reference's batched module; L2 (no batched L2 in the reference): the store's
        # per-query L2 arithmetic over corpus chunks of 1 M rows with a running top-k merge
        # instead of the full argsort, Bs queries at a time
        Bs = int(max(1, min(B, (64 << 20) // max(N, 1)))) if metric == "cosine" else int(max(1, min(B, 2)))
        bt = []
        t0 = time.perf_counter()
        j = 0
        while not bt or (time.perf_counter() - t0 < budget_s and len(bt) < 50):
            t1 = time.perf_counter()
            qs = Q[(j * Bs) % B:(j * Bs) % B + Bs]
            if metric == "cosine":
                ref_cpu.reference_batch_search(qs, V, k)
            else:
                ref_cpu.reference_l2_batch_chunked(qs, V, k)
            bt.append(time.perf_counter() - t1)
            j += 1
        batched_qps = Bs / float(np.mean(bt))
        res["batched"] = {"qps": batched_qps, "p50_ms_per_batch": float(np.median(bt)) * 1e3, "batches": len(bt),
                          "queries_per_batch": Bs}
        parts.append(f"(ii) {len(bt)} batch(es) of {Bs} of the {B} queries x the full {N}x{V.shape[1]} corpus "
                     f"({'batched cosine' if metric == 'cosine' else 'L2 in 1 M-row chunks, top-k merge'}, "
                     f"{sum(bt):.1f} s)")
    qt = []
    t0 = time.perf_counter()
    i = 0
    while not qt or (time.perf_counter() - t0 < budget_s and len(qt) < 50):
        t1 = time.perf_counter()
        ref_cpu.reference_store_search(Q[i % B], V, k, metric)
        qt.append(time.perf_counter() - t1)
        i += 1
    single_qps = 1.0 / float(np.mean(qt))
    res["per_query"] = {"qps": single_qps, "p50_ms": float(np.median(qt)) * 1e3, "queries": len(qt)}
    parts.append(f"(i) {len(qt)} single queries through the store path ({sum(qt):.1f} s)")
    res["value"] = max(batched_qps, single_qps)
    res["sample"] = "numpy restatement on this host: " + " and ".join(parts) + "; value = the faster path"
    return res


def serving_stats(V, metric, k, device, n_queries=400, threads=4):
    """The reference's live path: single-vector `store.query` calls from a 4-thread executor
    (api/routes/vectors.py:43, :226-234 -> service/optimized_vector_store.py:116-192), here
    through the drop-in store (host memory in and out) over the same corpus: batch-1 latency
    (one caller at a time) and the 4-thread throughput with and without the store's query
    coalescer (concurrent callers joining one device search)."""
    import shutil
    import tempfile
    from concurrent.futures import ThreadPoolExecutor
    from service.optimized_vector_store import MLXVectorStore, MLXVectorStoreConfig
    N, D = V.shape
    tmp = tempfile.mkdtemp(prefix="vdb_bench_store_")
    try:
        st = MLXVectorStore(tmp, MLXVectorStoreConfig(dimension=D, metric=metric, persist=False, device=device))
        st.add_vectors(V, [{}] * N)
        Qs = np.random.default_rng(2).random((n_queries, D), dtype=np.float32)
        for q in Qs[:5]:
            st.query(q, k)
        lat = []
        for q in Qs[:100]:
            t0 = time.perf_counter()
            st.query(q, k)
            lat.append(time.perf_counter() - t0)
        out = {"batch1_p50_ms": float(np.median(lat)) * 1e3, "batch1_p99_ms": float(np.percentile(lat, 99)) * 1e3,
               "threads": threads, "queries": n_queries}
        # both modes twice, interleaved, the better of each reported (host-side noise of a
        # Python-threaded client is large against a 0.15 ms scan: profiles/r04_ab/serving)
        for mode in (True, False, True, False):
            st.config.coalesce = mode
            b0, q0 = st._coalescer.batches, st._coalescer.queries
            with ThreadPoolExecutor(threads) as ex:
                t0 = time.perf_counter()
                list(ex.map(lambda q: st.query(q, k), Qs))
                dt = time.perf_counter() - t0
            key = f"store_query_{threads}threads_qps_{'coalesced' if mode else 'direct'}"
            out[key] = max(out.get(key, 0.0), n_queries / dt)
            if mode:
                nb = st._coalescer.batches - b0
                out["coalesced_mean_batch"] = (st._coalescer.queries - q0) / max(nb, 1)
        st._index.close()
        return out
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def cpu_graph_baseline(V, nbr, entries, Q, k, ef, metric, gt, budget_s=15.0):
    """The graph search restated on the CPU (oracle/ref_cpu.graph_search, hnswlib's
    searchBaseLayerST) over the same neighbour array: queries one at a time until
    the time budget is spent."""
    from oracle import ref_cpu
    inv = 1.0 / np.maximum(np.linalg.norm(V, axis=1), 1e-8) if metric == "cosine" else None  # once per corpus
    t0 = time.perf_counter()
    n = hits = 0
    for b in range(Q.shape[0]):
        lab, _, _ = ref_cpu.graph_search(V, nbr, entries, Q[b], k, ef, metric, inv_norms=inv)
        hits += len(set(lab.tolist()) & set(gt[b].tolist()))
        n += 1
        if time.perf_counter() - t0 > budget_s:
            break
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "queries/s", "cores": 1, "kind": "port",
            "sample": f"{n} single queries, numpy/heapq restatement of hnswlib's level-0 search "
                      f"(searchBaseLayerST) over the same graph, ef={ef}; {dt:.2f} s",
            "recall_at_10": hits / float(n * k)}


def bench_graph(args, world, rank, local, dev, primary=True):
    """C5: the graph path at batch 1.  N>1 runs independent replicas (SURVEY.md §8e:
    each GPU holds the whole graph and serves its own queries); value = all queries
    served / the slowest rank's time.  Returns the record on rank 0 (None elsewhere);
    primary=False: the default run's sub-record (BASELINE's rows, no tuning flags)."""
    from performance.hnsw_index import N_ENTRIES, TEAMS
    rec = None
    if args.teams is None:
        args.teams = TEAMS
    N, D, B, k, metric, desc = CONFIGS["c5"]
    N = (args.rows if primary else None) or N
    if rank == 0:
        print("bench: c5 start", file=sys.stderr, flush=True)
    R = 2 * GRAPH_M
    knn = args.graph_knn or R
    ix = _vdb.NativeIndex(D, metric, local)
    ix.reserve(N)
    keep_host = world == 1 and rank == 0 and not args.no_cpu_baseline
    parts = []
    clustered = args.data == "clustered" and primary
    cen = cluster_centres(D) if clustered else None
    for s0 in range(0, N, 8 * CHUNK_ROWS):
        part = (corpus_rows_clustered(N, D, s0, min(s0 + 8 * CHUNK_ROWS, N), centres=cen) if clustered
                else corpus_rows(N, D, s0, min(s0 + 8 * CHUNK_ROWS, N)))
        ix.add(part)
        if keep_host:
            parts.append(part)
    t0 = time.perf_counter()
    n_ent = (args.graph_entries if primary else None) or N_ENTRIES
    g = _vdb.NativeGraph.build(ix, degree=R, knn=knn, n_entries=n_ent)
    build_s = time.perf_counter() - t0
    g.set_param("teams", args.teams)
    nq = args.warmup + args.steps
    qrng = np.random.default_rng(1 + rank)
    if clustered:  # queries from the same distribution: a centre plus the rows' noise
        Q = (cen[qrng.integers(0, CLUSTERS, nq)] + qrng.standard_normal((nq, D), dtype=np.float32) *
             np.float32(CLUSTER_SIGMA)).astype(np.float32)
    else:
        Q = qrng.random((nq, D), dtype=np.float32)
    q_dev = torch.from_numpy(Q).to(dev)
    lab = torch.empty((nq, k), dtype=torch.int64, device=dev)
    dst = torch.empty((nq, k), dtype=torch.float32, device=dev)
    stream = torch.cuda.Stream(dev)  # a real stream: events and the kernel on the same queue
    sp = stream.cuda_stream
    torch.cuda.synchronize()

    def one(i):
        g.search_device(q_dev[i].data_ptr(), 1, k, GRAPH_EF, lab[i].data_ptr(), dst[i].data_ptr(), stream=sp)

    for i in range(args.warmup):
        one(i)
    torch.cuda.synchronize()
    it0, vis0 = g.stat("iterations"), g.stat("visited")
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    lat = []
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for j in range(args.steps):
        t1 = time.perf_counter()
        ev[j][0].record(stream)
        one(args.warmup + j)
        ev[j][1].record(stream)
        torch.cuda.synchronize()
        lat.append(time.perf_counter() - t1)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    iters = (g.stat("iterations") - it0) / args.steps
    visited = (g.stat("visited") - vis0) / args.steps
    # recall@10 of the timed queries against the exact brute-force path
    Qt = Q[args.warmup:]
    _, gt = ix.search(Qt, k)
    got = lab[args.warmup:].cpu().numpy()
    recall = sum(len(set(a.tolist()) & set(b.tolist())) for a, b in zip(got, gt)) / float(gt.size)
    # exact brute force at batch 1 for comparison (same queries, device resident)
    os_, oi_ = torch.empty((1, k), device=dev), torch.empty((1, k), dtype=torch.int64, device=dev)
    for i in range(3):
        ix.search_device(q_dev[i].data_ptr(), 1, k, os_.data_ptr(), oi_.data_ptr(), 0, stream=sp)
    torch.cuda.synchronize()
    bl = []
    for i in range(min(args.steps, 50)):
        t1 = time.perf_counter()
        ix.search_device(q_dev[i].data_ptr(), 1, k, os_.data_ptr(), oi_.data_ptr(), 0, stream=sp)
        torch.cuda.synchronize()
        bl.append(time.perf_counter() - t1)
    # the same queries at other team counts (p50 over <= 100 single queries, recall)
    sweep = []
    for tm in [int(x) for x in (args.teams_sweep if primary else "").split(",") if x.strip()]:
        if tm == args.teams:
            continue
        g.set_param("teams", tm)
        tl = []
        for j in range(min(args.steps, 100)):
            t1 = time.perf_counter()
            one(args.warmup + j)
            torch.cuda.synchronize()
            tl.append(time.perf_counter() - t1)
        gl = lab[args.warmup:args.warmup + len(tl)].cpu().numpy()
        rc = sum(len(set(a.tolist()) & set(b.tolist())) for a, b in zip(gl, gt[:len(tl)])) / float(len(tl) * k)
        sweep.append({"teams": tm, "p50_ms": float(np.median(tl)) * 1e3, "recall_at_10": rc})
    g.set_param("teams", args.teams)
    p50 = float(np.median(lat))
    if world > 1:
        t = torch.tensor([elapsed, p50, kern_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, p50, kern_ms = t.tolist()
    if rank == 0:
        # algorithmic bytes of one search: every scored row (D fp32 + its row scale)
        # plus the neighbour list of every expanded node (<= 4 per iteration)
        q_bytes = visited * (4 * D + 4) + iters * 4 * R * 4  # (visited / iterations summed over the teams)
        achieved = q_bytes / (kern_ms * 1e-3) / 1e9
        rec = {
            "metric": METRIC,
            "value": args.steps * world / elapsed,
            "unit": "queries/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "p50_ms": p50 * 1e3,
            "p99_ms": float(np.percentile(lat, 99)) * 1e3,
            "recall_at_10": recall,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": ("synthetic uniform [0,1) fp32 (numpy PCG64, corpus seed 0 per 65536-row chunk, queries seed 1)"
                     if not clustered else
                     f"synthetic clustered fp32: {CLUSTERS} uniform [0,1) centres + N(0, {CLUSTER_SIGMA}^2) per "
                     "dimension (corpus seed 0 per 65536-row chunk; queries the same distribution, seed 1)"),
            "config": {"workload": f"c5: {desc}" + (" [clustered data]" if clustered else ""), "n_rows": N, "dim": D,
                       "global_batch": 1, "k": k,
                       "metric": metric, "ef": GRAPH_EF, "degree": R, "build_knn": knn, "entries": n_ent,
                       "teams": args.teams,
                       "parallelism": f"replicas x{world}" if world > 1 else "single GPU"},
            "build_s": build_s,
            "iterations_per_query": iters,
            "visited_per_query": visited,
            "exact_b1_p50_ms": float(np.median(bl)) * 1e3,
            "teams_sweep": sweep,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": None, "kernel": "graph_search",
                         "avg_launch_ms": kern_ms, "algorithmic_bytes": q_bytes,
                         "note": f"{args.teams} workgroups per query, each a chain of dependent beam steps: "
                                 "latency-bound, not bandwidth-bound"},
        }
        if keep_host:
            V = np.concatenate(parts) if len(parts) > 1 else parts[0]
            del parts
            nbr, ent = g.to_arrays()
            print("bench: c5 cpu baseline", file=sys.stderr, flush=True)
            rec["cpu_baseline"] = cpu_graph_baseline(V, nbr, ent, Qt, k, GRAPH_EF, metric, gt,
                                                     budget_s=15.0 if primary else 8.0)
    g.close()
    ix.close()
    return rec


def _rank_entry(local_rank, world, port, argv):
    os.environ.update(RANK=str(local_rank), LOCAL_RANK=str(local_rank), WORLD_SIZE=str(world),
                      LOCAL_WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    sys.argv = [sys.argv[0]] + argv
    main()


def spawn_ranks(n):
    """`bench.py --gpus N` without torchrun: start N fresh rank processes (one per GPU,
    torch.multiprocessing spawn) from this parent, which never touches the GPU itself
    (torch.cuda.device_count() does not initialise it), and return their exit status."""
    import socket
    import torch.multiprocessing as mp
    have = torch.cuda.device_count()
    if have < n:
        print(f"bench.py: --gpus {n} but only {have} GPU(s) visible", file=sys.stderr)
        return 2
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    try:
        mp.start_processes(_rank_entry, args=(n, port, sys.argv[1:]), nprocs=n, join=True, start_method="spawn")
    except Exception as e:  # a rank failed: its traceback is already on stderr
        print(f"bench.py: rank process failed: {e}", file=sys.stderr)
        return 1
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 100 batches: with three streams the first batch's pilot and the last one's finish are a
    # visible part of a 20-batch window (C2: 199-203 K QPS at 20, 216-217 K at 100, same box,
    # profiles/r02s_ab/s15/); the timed region is still ~30 ms
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default=None, choices=sorted(CONFIGS),
                    help="default: c2 (BASELINE.json configs[1]) plus the metric's 8-GPU workload c6 as a sub-record")
    ap.add_argument("--no-metric-workload", action="store_true",
                    help="default run: skip the c6 sub-record (the metric's 10M x 128 workload)")
    ap.add_argument("--no-other-configs", action="store_true",
                    help="default run: skip the c3 / c4 sub-records (BASELINE.json configs[2], [3])")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-serving", action="store_true",
                    help="c1/c2 at N=1: skip the store-API serving numbers (batch-1 p50, 4-thread QPS)")
    ap.add_argument("--scaling", default=None, choices=["weak", "strong"],
                    help="N>1: weak = global batch B*N (fixed work per GPU), strong = global batch B "
                         "(default: strong for c4 / c6, whose BASELINE batch is sharded, weak otherwise)")
    ap.add_argument("--precision", default="auto", choices=["auto", "bf16x3", "bf16", "fp32", "i8", "i8x3", "i8q"],
                    help="candidate-pass arithmetic (results identical; DESIGN.md §3)")
    ap.add_argument("--scan-variant", type=int, default=None, help="candidate-pass kernel variant (tuning)")
    ap.add_argument("--n-wg", type=int, default=None, help="candidate-pass workgroups (tuning)")
    ap.add_argument("--scan-sync", type=int, default=None,
                    help="candidate-pass step end: 1 lockstep barrier, 2 flag-gated rounds (tuning; default by D)")
    ap.add_argument("--scan-qlds", type=int, default=None, help="0: query block never in LDS (tuning)")
    ap.add_argument("--scan-q4", type=int, default=None, help="128-query shape: -1 auto, 0 off, 1 on (tuning)")
    ap.add_argument("--scan-wide", type=int, default=None,
                    help="wide int8 pass (D <= 128, B > 256): -1 auto, 0 off, 1 on (tuning)")
    ap.add_argument("--dir-bound", type=int, default=None,
                    help="bf16 certificate: 1 residual bound along the rows' mean direction (default), 0 Cauchy-Schwarz")
    ap.add_argument("--pilot-tiles", type=int, default=None, help="row tiles sampled by the pilot bound (tuning)")
    ap.add_argument("--margin", type=int, default=None, help="candidates beyond k (tuning; default per precision)")
    ap.add_argument("--pilot-rank", type=int, default=None, help="rank of the pilot bound (tuning; default: Poisson rule)")
    ap.add_argument("--k", type=int, default=None, help="tuning: the config at another k (not the config's line)")
    ap.add_argument("--finish-split", type=int, default=None, help="workgroups per query in the finish (tuning)")
    ap.add_argument("--finish-small", type=int, default=None,
                    help="the finish's 4-wave form beside a long-row wide scan: -1 auto, 0 off, 1 on (tuning)")
    ap.add_argument("--i8-refine", type=int, default=None, help="finish's I8 refinement: -1 auto (rows >= 512 dims), 0 off, 1 on (tuning)")
    ap.add_argument("--plant-close", type=int, default=None,
                    help="one GPU: P queries per batch with 300 rows the int8 pass cannot separate (re-pass test)")
    ap.add_argument("--device-repass", type=int, default=None,
                    help="device re-pass of uncertified queries: -1 auto (armed after a fallback), 0 off, 1 always")
    ap.add_argument("--scan-checksum", type=int, default=None,
                    help="int8 pass checksum checked by the finish: 1 on (default), 0 off (A/B of its cost)")
    ap.add_argument("--rows", type=int, default=None, help="override the corpus rows (exploration only)")
    ap.add_argument("--batch", type=int, default=None,
                    help="override the batch (exploration only: e.g. one rank's shape of a weak-scaled run)")
    ap.add_argument("--timing", type=int, default=1,
                    help="1: the library's HIP events around the scan in the timed region (roofline); 0: none "
                         "(A/B of their cost; the roofline then comes from an untimed second loop)")
    ap.add_argument("--streams", type=int, default=3,
                    help="single GPU: batches queued round-robin on this many HIP streams (a server's request "
                         "streams; each batch still runs the whole search)")
    ap.add_argument("--auto-i8q", type=int, default=None,
                    help="auto's L2 pass for 16 < k <= 100: 1 the xh plane x 16-bit query (default), 0 I8X3")
    ap.add_argument("--no-fallback", action="store_true",
                    help="diagnostics only (kernel-variant timing): skip the exact fallback; results may be wrong")
    ap.add_argument("--graph-knn", type=int, default=None, help="c5: kNN candidates per row for the build")
    ap.add_argument("--teams", type=int, default=None,
                    help="c5: workgroups per query (vdb_graph_set_param teams; default performance/hnsw_index.py TEAMS)")
    ap.add_argument("--graph-entries", type=int, default=None,
                    help="c5: entry rows of the graph (default performance/hnsw_index.py N_ENTRIES)")
    ap.add_argument("--teams-sweep", default="16,64", help="c5: extra teams settings reported beside the line")
    ap.add_argument("--no-graph", action="store_true", help="default run: skip the c5 (graph) sub-record")
    ap.add_argument("--data", default="uniform", choices=["uniform", "clustered"],
                    help="c5: the corpus (BASELINE's uniform [0,1) rows, or rows around cluster centres: the "
                         "structured data a graph index is for)")
    ap.add_argument("--pmc-json", default=None,
                    help="HBM traffic of the scan kernel from a separate rocprofv3 --pmc pass "
                         "(default: newest profiles/*/pmc.json for this config, see profiles/scripts/)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus != world:
        if "WORLD_SIZE" in os.environ or args.gpus < 1:
            sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: launch one rank per GPU "
                     f"(torchrun --nproc-per-node {args.gpus}) or run without torchrun")
        sys.exit(spawn_ranks(args.gpus))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    cfg = args.config or "c2"
    if cfg == "c5":
        rec = bench_graph(args, world, rank, local, dev)
    else:
        rec = bench_brute(cfg, args, world, rank, local, dev, primary=True)
    if args.config is None:
        # The default run also measures, on the same ranks, as compact sub-records (so the driver's
        # N = 1, 2, 4, 8 series carries them all):
        #   c6, the second half of BASELINE.json's metric, "10M x 128D @8 GPU" (cosine top-10,
        #       batch 64, row-sharded with the batch fixed);
        #   c3 and c4, BASELINE.json's configs[2] and [3] (the reference's own
        #       harness reports every shape it runs, benchmarks/large_scale_benchmark.py:32-104).
        subs = [] if args.no_metric_workload else [("metric_workload_10m_x_128", "c6")]
        if not args.no_other_configs:
            subs += [("config_c3", "c3"), ("config_c4", "c4")]
        for key, scfg in subs:
            sub = bench_brute(scfg, args, world, rank, local, dev, primary=False)
            if rank == 0:
                rec[key] = {k_: sub[k_] for k_ in ("value", "unit", "n_gpus", "steps", "ms_per_step", "p50_ms",
                                                   "scaling", "dtype", "config", "fallback_queries_timed",
                                                   "fallback_queries_total", "cpu_baseline") if k_ in sub}
                rec[key]["roofline"] = {
                    k_: sub["roofline"][k_] for k_ in ("bound", "achieved", "peak", "unit", "frac", "traffic",
                                                       "traffic_source", "avg_launch_ms", "precision", "basis",
                                                       "kernel", "algorithmic_bytes", "fp32_equivalent")}
        _HOST_CORPUS.clear()
        if not args.no_other_configs and not args.no_graph:
            # c5, BASELINE.json configs[4]: the graph path at batch 1, with the
            # exact path's batch-1 p50 on the same queries beside it
            sub = bench_graph(args, world, rank, local, dev, primary=False)
            if rank == 0:
                rec["config_c5"] = {k_: sub[k_] for k_ in ("value", "unit", "n_gpus", "steps", "ms_per_step", "p50_ms",
                                                           "p99_ms", "recall_at_10", "exact_b1_p50_ms", "scaling",
                                                           "dtype", "config", "build_s", "iterations_per_query",
                                                           "visited_per_query", "roofline", "cpu_baseline") if k_ in sub}
    if rank == 0:
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def bench_brute(cfg, args, world, rank, local, dev, primary=True):
    """One brute-force config: this rank's shard, the timed loop, the record (rank 0; None
    elsewhere).  primary=False: the compact secondary line (no CPU baseline / serving)."""
    rec = None
    N, D, B, k, metric, desc = CONFIGS[cfg]
    if rank == 0:  # progress on stderr (a long default run stays visibly alive)
        print(f"bench: {cfg} start", file=sys.stderr, flush=True)
    if args.k is not None:  # tuning: the config's rows and batch at another k (not a bench line)
        k = int(args.k)
        desc = f"{desc} [k = {k}]"
    N = (args.rows if primary else None) or N
    B = (args.batch if primary else None) or B
    scaling = args.scaling or DEFAULT_SCALING.get(cfg, "weak")
    lo, hi = shard_bounds(N, world, rank)
    n_local = hi - lo

    # ---- data: this rank's shard of the corpus, replicated queries -------------------
    # (every record at N = 1 carries its CPU baseline, VERDICT r5 #4: sub-records on a shorter budget)
    keep_host = world == 1 and rank == 0 and not args.no_cpu_baseline
    ix = _vdb.NativeIndex(D, metric, local, precision=args.precision)
    if args.scan_variant is not None:
        ix.set_param("scan_variant" if args.precision == "fp32" else "scan_variant_bf16x3", args.scan_variant)
    if args.n_wg is not None:
        ix.set_param("n_wg", args.n_wg)
    if args.scan_sync is not None:
        ix.set_param("scan_sync", args.scan_sync)
    if args.pilot_tiles is not None:
        ix.set_param("pilot_tiles", args.pilot_tiles)
    if args.scan_qlds is not None:
        ix.set_param("scan_qlds", args.scan_qlds)
    if args.scan_q4 is not None:
        ix.set_param("scan_q4", args.scan_q4)
    if args.scan_wide is not None:
        ix.set_param("scan_wide", args.scan_wide)
    if args.dir_bound is not None:
        ix.set_param("dir_bound", args.dir_bound)
    if args.margin is not None:
        ix.set_param("margin", args.margin)
    if args.pilot_rank is not None:
        ix.set_param("pilot_rank", args.pilot_rank)
    if args.finish_split is not None:
        ix.set_param("finish_split", args.finish_split)
    if args.finish_small is not None:
        ix.set_param("finish_small", args.finish_small)
    if args.device_repass is not None:
        ix.set_param("device_repass", args.device_repass)
    if args.i8_refine is not None:
        ix.set_param("i8_refine", args.i8_refine)
    if args.scan_checksum is not None:
        ix.set_param("scan_checksum", args.scan_checksum)
    if args.no_fallback:
        ix.set_param("no_fallback", 1)
    if args.auto_i8q is not None:
        ix.set_param("auto_i8q", args.auto_i8q)
    ix.reserve(n_local)
    host_parts = []
    # --plant-close P (one GPU): P query targets, each with 300 rows closer to it than the int8
    # pass can separate (cosine 1 - [1e-3, 4e-3]): those queries come back uncertified from the
    # candidate pass -- the device re-pass's case, measured against the plain line
    plant = int(args.plant_close or 0) if world == 1 else 0
    targets = [7 + 4001 * j for j in range(plant)]
    # the default run's c6 and c4 sub-records share their corpus (10M x 128, seed 0): generated once
    ckey = (N, D, lo, hi)
    cached = _HOST_CORPUS.get(ckey) if not plant else None
    keep_for_next = not plant and not primary and cfg == "c6"
    for s in range(lo, hi, 8 * CHUNK_ROWS):
        part = cached[(s - lo) // (8 * CHUNK_ROWS)] if cached else corpus_rows(N, D, s, min(s + 8 * CHUNK_ROWS, hi))
        if keep_for_next:
            _HOST_CORPUS.setdefault(ckey, []).append(part)
        if plant and s == lo:
            prng = np.random.default_rng(99)
            for j, t in enumerate(targets):
                x = part[t].astype(np.float64)
                c = np.linspace(1e-3, 4e-3, 300)
                u = prng.standard_normal((300, D))
                u -= np.outer(u @ x / (x @ x), x)
                u *= np.linalg.norm(x) / np.linalg.norm(u, axis=1, keepdims=True)
                part[t + 1:t + 301] = (x + np.sqrt(2.0 * c)[:, None] * u).astype(np.float32)
        ix.add(part)
        if keep_host:
            host_parts.append(part)
    assert ix.count() == n_local
    Bg = B * world if (world > 1 and scaling == "weak") else B  # global batch
    Q = np.random.default_rng(1).random((Bg, D), dtype=np.float32)  # large_scale_benchmark.py:61
    for j, t in enumerate(targets):
        Q[(j * Bg) // max(plant, 1)] = host_parts[0][t] if keep_host else corpus_rows(N, D, t, t + 1)[0]
    q_dev = torch.from_numpy(Q).to(dev)
    n_str = max(1, args.streams)
    outs = [(torch.empty((Bg, k), dtype=torch.float32, device=dev), torch.empty((Bg, k), dtype=torch.int64, device=dev))
            for _ in range(n_str)]
    out_s, out_i = outs[0]
    streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(n_str - 1)]
    searcher = ShardedSearcher.from_index(ix, lo) if world > 1 else None
    n_step = [0]

    def step():
        j = n_step[0] % n_str
        n_step[0] += 1
        os_, oi_ = outs[j]
        if searcher is None:
            ix.search_device(q_dev.data_ptr(), Bg, k, os_.data_ptr(), oi_.data_ptr(), 0, stream=streams[j].cuda_stream)
        else:  # the rank's shard search, the RCCL all-gather and the merge, queued on stream j
            with torch.cuda.stream(streams[j]):
                searcher.search(q_dev, k, os_, oi_)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    # Throughput (value): K batches queued back to back on the stream, as a server
    # keeps the device fed; device-memory searches return without a host wait
    # (DESIGN.md §3), so the host runs ahead and no step waits for its launch.
    # HIP events around the scan inside the throughput loop only with one stream: with several,
    # an event pair also spans the other streams' kernels running beside the scan
    ev_in_loop = bool(args.timing) and n_str == 1
    ix.set_param("timing", int(ev_in_loop))
    scan0, pipe0, n0 = ix.stat("scan_ns"), ix.stat("pipeline_ns"), ix.stat("timed_searches")
    by_prec0 = {p: ix.stat(f"searches_{p}") for p in ("fp32", "bf16x3", "bf16", "i8", "i8x3", "i8q")}
    fb0 = ix.stat("fallback_queries")
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    n_t = ix.stat("timed_searches") - n0
    # candidate passes per arithmetic in the timed region (precision "auto" picks per search)
    by_prec = {p: ix.stat(f"searches_{p}") - by_prec0[p] for p in by_prec0}
    fb_timed = ix.stat("fallback_queries") - fb0
    prec = args.precision if args.precision != "auto" else max(by_prec, key=by_prec.get)
    scan_ms = (ix.stat("scan_ns") - scan0) / 1e6 / max(n_t, 1)
    pipe_ms = (ix.stat("pipeline_ns") - pipe0) / 1e6 / max(n_t, 1)
    roof_timing = "hip events in the timed loop"
    if not ev_in_loop:  # the scan's launch time from a second run of the loop on one stream
        roof_timing = "hip events in a one-stream rerun of the timed loop (no events in the timed loop)"
        n_str = 1
        ix.set_param("timing", 1)
        torch.cuda.synchronize()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        n_t = ix.stat("timed_searches") - n0
        scan_ms = (ix.stat("scan_ns") - scan0) / 1e6 / max(n_t, 1)
        pipe_ms = (ix.stat("pipeline_ns") - pipe0) / 1e6 / max(n_t, 1)
    ix.set_param("timing", 0)
    # Latency (p50_ms): one batch at a time, each waited for
    n_str = 1
    lat = []
    for _ in range(min(args.steps, 50)):
        t0 = time.perf_counter()
        step()
        torch.cuda.synchronize()
        lat.append(time.perf_counter() - t0)
    if world > 1:
        t = torch.tensor([elapsed, scan_ms, pipe_ms, float(np.median(lat))], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, scan_ms, pipe_ms, p50 = t.tolist()
    else:
        p50 = float(np.median(lat))

    fallback = ix.stat("fallback_queries")
    overflow = ix.stat("overflow_queries")
    if rank == 0:
        # Two rooflines of the scan kernel, each named:
        # (1) "implementation" (the top-level fields): the work the kernel's own arithmetic must do
        #     per launch -- every corpus row read once at the element size of the candidate copy it
        #     scans (i8: the hi plane, 1 B; bf16 / i8x3: 2 B; bf16x3 / fp32: 4 B), the L2 row start
        #     values, the queries; its own MFMA count (fp32: 2BND on the FP32 peak; bf16 2x and
        #     bf16x3 3x the products on the bf16 peak; i8 1x (xh qh) and i8x3 3x on the int8 peak) -- bound
        #     by whichever floor is longer;
        # (2) "fp32_equivalent": SURVEY.md §8(d)'s algorithmic work for the config (fp32 arithmetic:
        #     2BND flops, 4 B per element; C3 names the bf16 corpus, 2 B) per launch, reported as a
        #     RATE only.  The kernel does not read the fp32 rows nor issue fp32 MFMAs (int8 /
        #     split-bf16 candidates + an exact fp64 rerank), so that work over the
        #     launch time is not a fraction of any roofline (it exceeded 1); the
        #     roofline fraction is the implementation's, above.
        Dp = (D + 63) // 64 * 64
        elem = {"i8": 1, "i8x3": 2, "i8q": 1, "bf16": 2}.get(prec, 4)
        q_elem = {"i8": 1, "i8x3": 2, "i8q": 2}.get(prec, 4)  # query tiles (i8: the hi plane; i8x3 / i8q: both 1-byte planes)
        hbm_bytes = n_local * Dp * elem + (n_local * 4 if metric == "euclidean" else 0) + Bg * Dp * q_elem
        n_mfma = {"fp32": 1, "bf16x3": 3, "bf16": 2, "i8": 1, "i8x3": 3, "i8q": 2}[prec]
        mfma_flops = n_mfma * 2.0 * Bg * n_local * D
        mfma_peak = {"fp32": FP32_MFMA_PEAK_TFLOPS, "bf16x3": BF16_MFMA_PEAK_TFLOPS, "bf16": BF16_MFMA_PEAK_TFLOPS,
                     "i8": I8_MFMA_PEAK_TOPS, "i8x3": I8_MFMA_PEAK_TOPS, "i8q": I8_MFMA_PEAK_TOPS}[prec]
        t_hbm = hbm_bytes / (HBM_PEAK_GBS * 1e9)
        t_mfma = mfma_flops / (mfma_peak * 1e12)
        achieved_gbs = hbm_bytes / (scan_ms * 1e-3) / 1e9
        achieved_tf = mfma_flops / (scan_ms * 1e-3) / 1e12
        if t_hbm >= t_mfma:
            roof = {"bound": "hbm", "achieved": achieved_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": achieved_gbs / HBM_PEAK_GBS}
        else:
            roof = {"bound": "mfma", "achieved": achieved_tf, "peak": mfma_peak, "unit": "TFLOP/s",
                    "frac": achieved_tf / mfma_peak}
        roof["basis"] = (f"implementation: {elem} B per corpus element read once + queries; "
                         f"{n_mfma} MFMA product(s) per fp32 product "
                         f"({ {'fp32': 'fp32', 'i8': 'int8', 'i8x3': 'int8', 'i8q': 'int8'}.get(prec, 'bf16')} peak)")
        s_flops = 2.0 * Bg * n_local * D
        s_bytes = n_local * D * (2 if cfg == "c3" else 4) + 4 * n_local + 4 * Bg * D + 12 * Bg * k
        fp32_eq = {"flops_per_launch": s_flops, "bytes_per_launch": s_bytes,
                   "tflops_equivalent": s_flops / (scan_ms * 1e-3) / 1e12,
                   "gbs_equivalent": s_bytes / (scan_ms * 1e-3) / 1e9,
                   "note": "SURVEY.md §8(d) fp32 work per launch (2BND flops, 4 B/element; c3: 2 B) over the scan's "
                           "launch time: a throughput, not a roofline fraction (the scan reads the int8 / bf16 "
                           "copy, not the fp32 rows)"}
        wide = ix.stat("searches_wide") > 0  # (rows of > 128 dims: the long-row form, vdb_scan8wl.hip)
        G8 = (D + 63) // 64 * 2  # 32-dim groups; the long-row form's two-waves-per-query-tile kernel below 129 queries
        long_k = "scan8wl_kernel" if (Bg + 31) // 32 <= 4 and G8 <= 32 else "scan8wl1_kernel"
        kname = ((long_k if D > 128 else "scan8w_kernel") if wide else "scan8_kernel") \
            if prec in ("i8", "i8x3", "i8q") \
            else {"fp32": "scan_topk"}.get(prec, "scan2_kernel")
        traffic = None
        traffic_src = None
        cands = [args.pmc_json] if (args.pmc_json and primary) else sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "pmc.json")))
        for path in reversed(cands):
            try:
                pm = json.load(open(path))
            except (OSError, ValueError):
                continue
            if (pm.get("config") == cfg and pm.get("n_gpus") == world and "hbm_bytes_per_launch" in pm
                    and pm.get("precision", "fp32") == prec and kname + "<" in pm.get("kernel", kname + "<")):
                traffic = pm["hbm_bytes_per_launch"]
                traffic_src = os.path.relpath(path, ROOT)
                break
        rec = {
            "metric": METRIC,
            "value": Bg * args.steps / elapsed,
            "unit": "queries/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "p50_ms": p50 * 1e3,
            "higher_is_better": True,
            "scaling": scaling if world > 1 else "weak",
            "vs_baseline": None,
            "dtype": {"fp32": "f32", "bf16x3": "f32 (bf16x3 split MFMA candidates, fp64 exact rerank)",
                      "bf16": "f32 (bf16 corpus x split query MFMA candidates, fp64 exact rerank)",
                      "i8": "f32 (int8 centred corpus x int8 query integer-MFMA candidates, fp64 exact rerank)",
                      "i8x3": "f32 (16-bit fixed-point corpus x query integer-MFMA candidates, fp64 exact rerank)",
                      "i8q": "f32 (8-bit centred corpus x 16-bit query integer-MFMA candidates, fp64 exact rerank)"}[prec],
            "data": "synthetic uniform [0,1) fp32 (numpy PCG64, corpus seed 0 per 65536-row chunk, queries seed 1)",
            "config": {"workload": f"{cfg}: {desc}", "n_rows": N, "dim": D, "global_batch": Bg,
                       "batch_per_gpu_equiv": B, "k": k,
                       "metric": metric, "parallelism": f"row-shard x{world}" if world > 1 else "single GPU",
                       "rows_per_gpu": n_local},
            "roofline": dict(roof, traffic=traffic,
                             kernel=kname,
                             fp32_equivalent=fp32_eq, precision=prec,
                             precision_requested=args.precision, searches_by_precision=by_prec,
                             traffic_source=traffic_src, algorithmic_bytes=hbm_bytes, algorithmic_flops=mfma_flops,
                             avg_launch_ms=scan_ms, hbm_gbs=achieved_gbs, mfma_tflops=achieved_tf,
                             hbm_frac=achieved_gbs / HBM_PEAK_GBS, mfma_frac=achieved_tf / mfma_peak),
            "pipeline_ms": pipe_ms,
            "streams": max(1, args.streams),
            "roofline_timing": roof_timing,
            "fallback_queries_total": fallback,
            "fallback_queries_timed": fb_timed,  # (auto's bf16 probe falls back in warm-up at C3 / C4)
            "fallback_list_overflow": overflow,
        }
        if keep_host:
            V = np.concatenate(host_parts) if len(host_parts) > 1 else host_parts[0]
            del host_parts
            if primary and cfg in ("c1", "c2") and not args.no_serving:
                rec["serving"] = serving_stats(V, metric, k, local)
            print(f"bench: {cfg} cpu baseline", file=sys.stderr, flush=True)
            rec["cpu_baseline"] = cpu_baseline(V, Q, k, metric, budget_s=10.0 if primary else 6.0)
    ix.close()
    return rec


if __name__ == "__main__":
    main()
