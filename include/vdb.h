/*
 * vdb.h — C-ABI of the MI355X (gfx950) brute-force vector-search core.
 *
 * This is the drop-in boundary for the hot path of Theseus-AT/mlx-vector-db.
 * The reference has no FFI of its own: its "operator slot" is the Python
 * callable `MLXVectorStore._compiled_similarity_fn(query, vectors) -> scores[N]`
 * followed by `mx.argsort(...)[:k]`
 * (reference service/optimized_vector_store.py:31-48, :149-192, :211-213) and
 * the batched variant in performance/mlx_optimized.py:59-88, :217-248.
 * Each entry point below names the reference interface it replaces.
 * A ctypes binding (mlx-vector-db_amd/service/_vdb.py) is the host side; the
 * binding a maintainer would add to the reference is shown in INTEGRATION.md.
 *
 * Conventions
 *   - Every function returns an int32 status (VDB_OK = 0, negative = error
 *     class); vdb_last_error() returns a thread-local message for the last
 *     failing call on the calling thread.
 *   - Plain pointers and sizes only.  `mem` says whether the query / output
 *     pointers of a call are host (VDB_MEM_HOST) or device (VDB_MEM_DEVICE)
 *     memory.  Device-memory calls are stream-ordered on `stream` (a
 *     hipStream_t; NULL = the null stream, which orders with PyTorch's default
 *     stream) and return without waiting: the results are in device memory
 *     once the stream reaches that point (the exactness certificate is
 *     checked and any fallback queued on the device, see vdb_index_search).
 *     Host-memory calls run on `stream` or, if NULL, on a stream of the
 *     per-search workspace they take (so concurrent host-memory searches from
 *     several threads overlap on the device) and return when the results are
 *     in host memory.
 *   - The library never frees caller memory.  An index owns its device-resident
 *     corpus: row-major fp32 rows (the exact rerank), the int8
 *     candidate copy in MFMA operand tiles (two planes, the default pass) with
 *     its row-major hi plane and column sums, and -- for the bf16 / fp32
 *     precisions, or under auto only once a search first runs a split pass --
 *     a split-bf16 (fp32) candidate copy; plus a per-call workspace pool.
 *   - All entry points are thread-safe; searches on one index may run from
 *     several threads at once (the reference serves from a 4-thread executor,
 *     api/routes/vectors.py:43).
 *
 * Result contract:
 *   cosine    score = (q/max(|q|,1e-8)) . (x/max(|x|,1e-8))   higher first
 *   euclidean score = sqrt(sum((x-q)^2))                        lower first
 *   Ranking is by the exact (fp64, canonical summation order) value with ties
 *   broken by the lower row index; returned scores are that value rounded to
 *   fp32.  Rows beyond the number of eligible rows are returned as index -1.
 */
#ifndef VDB_H
#define VDB_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
    VDB_OK = 0,
    VDB_ERR_INVALID = -1,     /* bad argument -> Python ValueError          */
    VDB_ERR_HIP = -2,         /* HIP runtime error -> RuntimeError          */
    VDB_ERR_OOM = -3,         /* device allocation failed                   */
    VDB_ERR_NONFINITE = -4,   /* NaN/Inf in vectors or queries -> ValueError */
    VDB_ERR_UNSUPPORTED = -5, /* e.g. metric "dot_product" (reference raises,
                                 service/optimized_vector_store.py:153-154)   */
    VDB_ERR_NODEVICE = -6     /* no gfx950 device visible                    */
};

enum { VDB_METRIC_COSINE = 0, VDB_METRIC_EUCLIDEAN = 1, VDB_METRIC_DOT = 2 /* operator slot only */ };
enum { VDB_MEM_HOST = 0, VDB_MEM_DEVICE = 1 };

/* Candidate-pass arithmetic for an index (vdb_index_set_param "precision").
 * The returned results are identical for all (the exact fp64 rerank decides);
 * only the speed of the candidate pass differs.
 *   VDB_PREC_FP32    fp32 v_mfma_f32_32x32x2_f32 (MFMA-bound, 157 TF peak)
 *   VDB_PREC_BF16X3  split-bf16 "x3": x = hi + lo, q = hi + lo,
 *                    x.q ~ xh.qh + xh.ql + xl.qh on v_mfma_f32_32x32x16_bf16,
 *                    fp32 accumulate; error bound of the same order as fp32
 *                    (HBM-bound).  Keeps a split copy of the corpus (same bytes
 *                    as the fp32 copy).
 *   VDB_PREC_BF16    the hi plane of the split copy only: x.q ~ xh.qh + xh.ql,
 *                    half the corpus bytes per search; the certificate adds a bound
 *                    of the corpus rounding q.(x - bf16(x)) measured at ingest:
 *                    min(|q| R, |q - c d| R + |c| M), R the largest row residual,
 *                    d the normalised mean row of the first add, M the largest
 *                    |d.(x - bf16(x))|, c = q.d, so it is wider
 *                    and takes a larger candidate margin.
 *   VDB_PREC_I8      an int8 copy of the CENTRED rows z = y - mu (y the scored row, mu the
 *                    mean row of the first add), 16-bit fixed point in two planes
 *                    z ~ s_x (xh + xl/256); the query 16-bit fixed point per batch.  I8
 *                    reads the hi plane only (1 byte per element, a quarter of the fp32
 *                    copy): x.q ~ s_x s_q (xh.qh + xh.ql/256) on v_mfma_i32_32x32x32_i8
 *                    (exact integer sums, twice the K of a bf16 MFMA per cycle); the
 *                    certificate adds the measured row rounding (as BF16: Cauchy-Schwarz or
 *                    along d) and each query's own rounding (vdb_scan8_kernel.h).
 *   VDB_PREC_I8X3    both planes (2 bytes per element): xh.qh + (xh.ql + xl.qh)/256, an
 *                    error bound of bf16x3's order at half its bytes and MFMA cycles.
 *   VDB_PREC_AUTO    (default) per batch, on the int8 copy (knob "auto_int8" = 1, the
 *                    default; start value from VDB_AUTO_I8): I8 for k <= 16, I8X3 for k > 16
 *                    (a one-plane pass would need 256 candidates per query there); on the split
 *                    copy (auto_int8 = 0): BF16 / BF16X3.  A host-memory search re-passes its
 *                    uncertified one-plane queries (at most 1/8 of the batch, at most 64) in
 *                    BF16X3 as one gathered sub-search and keeps its precision; more than that
 *                    reruns the batch in BF16X3 and starts a HOLD on the next precision down
 *                    the list I8 -> BF16 -> BF16X3 (an I8X3 failure: its batch takes the exact
 *                    path, the hold runs BF16X3) for the next 16 searches, doubling per failed
 *                    probe up to 2048 (reset by 64 certified searches, or when the rows change).
 *                    A device-memory search sees its fallback counts a search or more late (no
 *                    host sync): its flagged queries take the device-gated exact path and the
 *                    next search starts the hold.  Stats "repass_queries", "auto_hold",
 *                    "auto_hold8". */
/*   VDB_PREC_I8Q     the int8 copy's xh plane (1 byte per element) against the 16-bit query:
 *                    xh.qh + xh.ql / 256, two int8 MFMAs per group.  AUTO's pass for L2 with
 *                    16 < k <= 100 (KP = 256) until a batch flags more than 1/8 of its queries
 *                    (then I8X3 for good, stat "i8q_off"). */
enum { VDB_PREC_FP32 = 0, VDB_PREC_BF16X3 = 1, VDB_PREC_BF16 = 2, VDB_PREC_AUTO = 3, VDB_PREC_I8 = 4, VDB_PREC_I8X3 = 5,
       VDB_PREC_I8Q = 6 };

typedef struct vdb_index vdb_index;

/* --- library -------------------------------------------------------------- */
const char* vdb_last_error(void);
int32_t vdb_version(void);
/* Number of visible HIP devices (0 on a host without a GPU). */
int32_t vdb_device_count(int32_t* n);

/* --- index lifecycle -------------------------------------------------------
 * Replaces MLXVectorStore's corpus state `self._vectors` (mx.array [N,D] f32)
 * and `_compile_critical_functions` (service/optimized_vector_store.py:59-83,
 * :211-213).  metric: VDB_METRIC_*.  Any other metric -> VDB_ERR_UNSUPPORTED,
 * matching the reference, where "dot_product" leaves no operator and every
 * query raises. */
int32_t vdb_index_create(int32_t dim, int32_t metric, int32_t device, vdb_index** out);
int32_t vdb_index_destroy(vdb_index* idx);
/* Pre-size the device corpus for `rows` rows (capacity otherwise doubles). */
int32_t vdb_index_reserve(vdb_index* idx, int64_t rows);
/* Knobs.  "precision" (VDB_PREC_*; default VDB_PREC_AUTO), "margin" (extra candidates
 * per query), "force_exact" (0/1), "no_fallback" (diagnostics: flagged queries keep the
 * approximate order), "timing" (0/1: HIP events around the candidate pass; stats "scan_ns",
 * "pipeline_ns", "timed_searches").  Tuning knobs the bench's A/B runs use (results identical,
 * speed differs): "n_wg" (candidate-pass workgroups), "scan_variant" / "scan_variant_bf16x3"
 * (fp32 / split pass tilings), "scan_sync" (0 auto, 1 per-step barrier, 2 flag-gated
 * compaction rounds), "scan_q4" (split pass 128-query shape, -1 auto / 0 / 1), "scan_qlds"
 * (-1 auto: query block in LDS when it fits, 0 never), "scan_wide" (the wide int8 passes, all
 * queries of a batch in one workgroup's registers: -1 auto from 65 536 rows -- rows of <= 128
 * dims with > 256 queries, or <= 256 up to 2.5M rows; I8 cosine rows of 512..1536 dims with
 * <= 256 queries (1536: <= 16 or > 96) -- 0 off, 1 whenever the shape allows),
 * "scan_checksum" (1 default, 0 off, 2 also I8X3's L sums), "pilot_tiles", "pilot_rank",
 * "finish_split", "finish_small" (-1 auto: the finish's 4-wave form beside a long-row
 * wide scan for batches of >= 32, 0 off, 1 on), "i8_refine", "i8_narrow", "device_repass", "auto_int8", "auto_i8q",
 * "dir_bound" (0: BF16 certificate with |q| R only).  Stats also: "searches", "queries",
 * "fallback_queries", "overflow_queries", "inconsistent_queries", "repass_queries",
 * "capacity", "count", "device_bytes", "precision", "searches_fp32" / "searches_bf16x3" /
 * "searches_bf16" / "searches_i8" / "searches_i8x3" / "searches_i8q" (candidate passes run in
 * each; with VDB_PREC_AUTO these show its choices), "searches_q4", "searches_wide",
 * "auto_int8", "i8q_off", "i8_wide", "split_copy", "split_copy_builds". */
int32_t vdb_index_set_param(vdb_index* idx, const char* name, int64_t value);
int32_t vdb_index_get_stat(const vdb_index* idx, const char* name, int64_t* value);

/* --- ingest ------------------------------------------------------------------
 * Replaces MLXVectorStore.add_vectors' `mx.concatenate([old, new])`
 * (service/optimized_vector_store.py:96-106; mlx_optimized.py:127-137).
 * Appends n rows of `dim` fp32 (row-major) in place (capacity doubling), packs
 * them into the MFMA-tiled layout and computes the per-row norms once.
 * Non-finite input -> VDB_ERR_NONFINITE and nothing is appended.  Device-memory rows
 * (mem = VDB_MEM_DEVICE) are read after the work queued on `stream` so far (NULL = the
 * null stream); the call returns when the rows are ingested (the source may be reused). */
int32_t vdb_index_add(vdb_index* idx, const float* vectors, int64_t n, int32_t mem, void* stream);
int32_t vdb_index_count(const vdb_index* idx, int64_t* n);
/* Replaces MLXVectorStore.clear (service/optimized_vector_store.py:198-209). */
int32_t vdb_index_clear(vdb_index* idx);
/* Copy rows [start, start+n) back out, row-major fp32, to host memory (used for
 * vectors.npz persistence, service/optimized_vector_store.py:218-223). */
int32_t vdb_index_get_vectors(vdb_index* idx, int64_t start, int64_t n, float* out_host);

/* --- search ------------------------------------------------------------------
 * Replaces `_brute_force_search`: similarity fn + mx.argsort(...)[:k] + gather
 * (service/optimized_vector_store.py:149-192) for B=1, and
 * `optimized_batch_similarity_search` (performance/mlx_optimized.py:217-248)
 * for B>1.
 *   queries      [n_queries, dim] fp32 row-major (host or device per `mem`)
 *   k            1..1024 results per query (min(k, eligible rows) are valid)
 *   row_mask     NULL, or a bitmap of ceil(count/32) uint32 words (bit r of
 *                word r/32 = row r eligible): the metadata filter
 *                (service/optimized_vector_store.py:159-167); same memory kind
 *                as `mem`.
 *   out_scores   [n_queries, k] fp32 (cosine similarity / euclidean distance)
 *   out_indices  [n_queries, k] int64 row ids (+ index_offset), -1 = no result
 *   out_keys     NULL or [n_queries, k] fp64 exact ranking keys (cosine: the
 *                similarity; euclidean: minus the squared distance) — what a
 *                multi-GPU merge needs to stay bit-identical to one GPU.
 */
int32_t vdb_index_search(vdb_index* idx, const float* queries, int32_t n_queries, int32_t k,
                         const uint32_t* row_mask, int32_t mem,
                         float* out_scores, int64_t* out_indices, double* out_keys,
                         int64_t index_offset, void* stream);

/* --- multi-GPU merge -----------------------------------------------------------
 * Merge per-shard top-k lists (all device memory, already all-gathered):
 *   keys [n_lists, n_queries, k_in] fp64 ranking keys (higher first),
 *   idx  [n_lists, n_queries, k_in] int64 global row ids (-1 = empty)
 * into the global top-k_out per query, ordered by (key desc, index asc) —
 * bit-identical to a single-GPU search.  No reference counterpart (the
 * reference is single device); SURVEY.md §8e. */
int32_t vdb_merge_topk(const double* keys, const int64_t* idx, int32_t n_lists, int32_t n_queries,
                       int32_t k_in, int32_t k_out, int32_t metric,
                       float* out_scores, int64_t* out_indices, double* out_keys, void* stream);

/* --- stateless operator slot ---------------------------------------------------
 * The reference's similarity functions themselves, returning every score
 * (no top-k): `_compiled_cosine_similarity` / `_compiled_euclidean_distance`
 * (service/optimized_vector_store.py:31-48) for n_queries = 1,
 * `compute_cosine_similarity_batch` (performance/mlx_optimized.py:59-88) for
 * n_queries > 1, and `compute_dot_product` (mlx_optimized.py:150-156, metric
 * VDB_METRIC_DOT).  All pointers are device memory: corpus [n, dim] row-major
 * fp32, queries [n_queries, dim], out [n_queries, n] fp32.  cosine / dot: an fp32
 * MFMA GEMM over LDS-staged tiles with the norms applied in the epilogue;
 * euclidean: direct differences (the reference's form).  Within 1e-4 of the
 * reference's fp32 arithmetic. */
int32_t vdb_similarity_matrix(const float* corpus, int64_t n, int32_t dim,
                              const float* queries, int32_t n_queries, int32_t metric,
                              float* out, void* stream);
/* `normalize_vectors` (performance/mlx_optimized.py:110-125): out = x / max(|x|, 1e-8)
 * per row; device memory, in == out allowed. */
int32_t vdb_normalize_rows(const float* in, int64_t n, int32_t dim, float* out, void* stream);
/* `fast_top_k_indices` / `mx.argsort(-scores)[:k]` (mlx_optimized.py:90-108,
 * optimized_vector_store.py:176-183) over `rows` score rows of length n (device
 * memory): the k best per row, largest first (largest = 1) or smallest first, ties to
 * the lower index, NaN last.  out_indices [rows, k] int64, out_values NULL or
 * [rows, k] fp32.  1 <= k <= min(n, 1024). */
int32_t vdb_topk_scores(const float* scores, int32_t rows, int64_t n, int32_t k, int32_t largest,
                        int64_t* out_indices, float* out_values, void* stream);

/* --- graph index (the HNSW path) -------------------------------------------------
 * Replaces ProductionHNSWIndex (performance/hnsw_index.py:23-129: hnswlib
 * build / knn_query / save / load), re-laid out for the GPU: one
 * level of out-degree `degree` (hnswlib's level-0 degree 2M) as a [N][degree]
 * int32 neighbour array, built from the exact kNN of every row (the brute-force
 * path above, `knn` neighbours) as the degree/2 nearest out-edges plus the nearest
 * reverse edges; searches start from the best of `n_entries` spread rows.  The
 * graph refers to the index's rows; adding rows makes it stale (search errors). */
typedef struct vdb_graph vdb_graph;

int32_t vdb_graph_build(vdb_index* idx, int32_t degree, int32_t knn, int32_t n_entries, vdb_graph** out);
/* Persistence: a graph exported by vdb_graph_export (neighbours [n][degree], -1 =
 * none; entry rows) re-attached to an index holding the same rows. */
int32_t vdb_graph_import(vdb_index* idx, int32_t degree, int64_t n, const int32_t* nbr, int32_t n_entries,
                         const int32_t* entries, vdb_graph** out);
int32_t vdb_graph_export(const vdb_graph* g, int32_t* nbr_host, int32_t* entries_host);
/* Incremental maintenance (replaces the rebuild per add of
 * service/optimized_vector_store.py:110-112): inserts the rows the index gained since the
 * graph was built or last extended (exact kNN of the new rows, hnswlib's heuristic for their
 * out-edges, re-selection of every list that gains an in-edge).  A graph must be extended
 * before it is searched again after its index grew (vdb_graph_search reports it stale). */
int32_t vdb_graph_add(vdb_graph* g);
int32_t vdb_graph_info(const vdb_graph* g, int64_t* n_rows, int32_t* degree, int32_t* n_entries);
/* hnswlib knn_query semantics (hnsw_index.py:98-101): labels [n_queries, k] int64
 * (-1 = none), distances [n_queries, k] fp32: cosine 1 - cos, euclidean squared L2;
 * best first.  ef = beam width (search depth), k <= ef <= 256. */
int32_t vdb_graph_search(vdb_graph* g, const float* queries, int32_t n_queries, int32_t k, int32_t ef, int32_t mem,
                         int64_t* labels, float* distances, void* stream);
/* stats: "queries", "iterations" (beam iterations, summed over queries and teams),
 * "visited" (rows scored, summed) */
int32_t vdb_graph_stat(const vdb_graph* g, const char* name, int64_t* value);
/* Graph search knobs: "teams" (1..256, at most the entry rows; default 1): workgroups per query, each
 * searching from a disjoint slice of the entry rows (entry rank r -> team r mod
 * teams) with its own beam of `ef`, merged into the top k distinct rows.  At
 * batch 1 it puts several CUs on the query: more of the graph explored (higher
 * recall) in about the same latency.  Replaces: nothing in hnswlib (its search
 * is single-threaded per query). */
int32_t vdb_graph_set_param(vdb_graph* g, const char* name, int64_t value);

int32_t vdb_graph_destroy(vdb_graph* g);

/* --- multi-device corpus (one process, several GPUs) ------------------------------
 * The store's corpus row-sharded over `n_devices` GPUs of this process (SURVEY.md §8e;
 * the reference serves from one process, main.py:395, with the corpus on one device,
 * service/optimized_vector_store.py:59-114).  Rows keep their global ids (insertion
 * order); each add is cut into contiguous pieces that level the shard sizes.  A search
 * runs on every shard at once (one stream each, device-resident top-k with exact fp64
 * keys and global ids), gathers the G lists to devices[0] by peer copies over xGMI and
 * merges them there by (key desc, row asc): results identical to vdb_index_search on
 * one index holding every row.  Host memory in and out.  A device may repeat. */
typedef struct vdb_shards vdb_shards;
int32_t vdb_shards_create(int32_t dim, int32_t metric, const int32_t* devices, int32_t n_devices, vdb_shards** out);
int32_t vdb_shards_destroy(vdb_shards* s);
int32_t vdb_shards_add(vdb_shards* s, const float* vectors_host, int64_t n);
int32_t vdb_shards_count(const vdb_shards* s, int64_t* n);
int32_t vdb_shards_shard_count(const vdb_shards* s, int32_t shard, int64_t* n);
/* row_mask: NULL or ceil(count/32) host words over GLOBAL rows (as vdb_index_search) */
int32_t vdb_shards_search(vdb_shards* s, const float* queries_host, int32_t n_queries, int32_t k,
                          const uint32_t* row_mask, float* out_scores, int64_t* out_indices, double* out_keys);
/* Stream-ordered form (no host wait): queries [n_queries, dim], row_mask (NULL or
 * ceil(count/32) words over GLOBAL rows) and the outputs are device memory on devices[0];
 * the search is ordered after the work queued on `stream` (a stream of devices[0], NULL = its
 * null stream) and the outputs are ready when `stream` reaches the merge, so batches can be
 * queued back to back.  Per shard: peer copies of the queries (and the mask, whose shard-local
 * bitmap is built on the shard's device), the shard's device search, a peer copy of its lists
 * to devices[0]; the merge runs on `stream`.  vdb_shards_search is the host-memory form of
 * the same path.  Reference constraint: one process serving every device (main.py:395). */
int32_t vdb_shards_search_device(vdb_shards* s, const float* queries, int32_t n_queries, int32_t k,
                                 const uint32_t* row_mask, float* out_scores, int64_t* out_indices,
                                 double* out_keys, void* stream);
int32_t vdb_shards_get_vectors(vdb_shards* s, int64_t start, int64_t n, float* out_host);
int32_t vdb_shards_clear(vdb_shards* s);
int32_t vdb_shards_reserve(vdb_shards* s, int64_t rows);
/* applied to every shard's index (vdb_index_set_param names) */
int32_t vdb_shards_set_param(vdb_shards* s, const char* name, int64_t value);
/* "count", "shards", else the vdb_index_get_stat name summed over the shards */
int32_t vdb_shards_get_stat(const vdb_shards* s, const char* name, int64_t* value);

/* --- lifecycle ------------------------------------------------------------------------
 * Waits for every queued search of every live index, releases their idle per-search
 * workspaces and trims the devices' stream-ordered pools back to the driver.  Indexes
 * stay valid; the next search re-allocates what it needs. */
int32_t vdb_shutdown(void);

#ifdef __cplusplus
}
#endif
#endif /* VDB_H */
