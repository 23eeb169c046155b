// vdb_internal.h — host-side launchers for the kernels in vdb_kernels.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace vdb {

// Tiling constants (layout documented in vdb_common.h / DESIGN.md §2).
constexpr int TILE_ROWS = 32;      // rows per row tile
constexpr int GROUP_DIMS = 8;      // dims per (tile, group) block
constexpr int BLOCK_FLOATS = 256;  // floats per (tile, group) block = 1 KiB
constexpr int QG_EXTRA = 8;        // duplicated leading dim-groups at the end of each query tile
constexpr int ROW_ALIGN = 1024;    // corpus capacity granule (>= rows per scan step of any variant)

// Candidate-pass arithmetic (vdb.h VDB_PREC_*):
//   PREC_FP32   fp32 corpus tiles, v_mfma_f32_32x32x2_f32 (8-dim groups, 4 KiB per super-tile group)
//   PREC_BF16X3 split-bf16 corpus (x = hi + lo + O(2^-16 x)), three v_mfma_f32_32x32x16_bf16 per
//               16-dim group: hi*hi + hi*lo + lo*hi (8 KiB per super-tile group: [plane][sub tile])
constexpr int PREC_FP32 = 0;
constexpr int PREC_BF16X3 = 1;
//   PREC_BF16   the hi plane of the split copy only (x ~ bf16(x), half the bytes), query split:
//               x.q ~ xh.qh + xh.ql, two v_mfma_f32_32x32x16_bf16 per 16-dim group; bounded by the
//               index's largest row residual |x - bf16(x)| (pack_rows)
constexpr int PREC_BF16 = 2;
//   PREC_I8     int8 copy of the centred rows (vdb_scan8_kernel.h): x ~ s_x xh (1 byte per element),
//               query s_q qh (8 bits): one v_mfma_i32_32x32x32_i8 per 32-dim group
//   PREC_I8X3   both planes of the int8 copy, x ~ s_x (xh + xl/256), query 16 bits: three per group
//   PREC_I8Q    the xh plane (8 bits, 1 byte per element) against the 16-bit query: xh.qh + xh.ql /
//               256, two per group (L2, 16 < k <= 100: C4)
constexpr int PREC_I8 = 3;
constexpr int PREC_I8X3 = 4;
constexpr int PREC_I8Q = 5;
constexpr int N_PREC = 6;
inline bool prec_is_i8(int p) { return p == PREC_I8 || p == PREC_I8X3 || p == PREC_I8Q; }

// Per-index constants of the int8 pass (vdb_api.cpp): the quantisation step s_x of the centred
// rows, max |s_x xh| and max |s_x xl / 256| over the rows (row norms), max |x|^2 / 2 (L2 start)
struct Int8Consts {
    float sx;
    double zmax_h, xl_max, rmax_half;
};
// max |y - mu| of rows [row0, row0 + n) as float bits (atomicMax into *out)
hipError_t launch_zmax(const float* X, const float* inv32, const float* mu, int64_t row0, int64_t n, int D, int G,
                       uint32_t* out, hipStream_t st);
// rows [row0, row0 + n) -> the int8 copy Xq (two planes, 32-dim groups, the split layout's block
// order); stats[0..6) running maxima (fp64 bits): |z - s_x xh|, |dir.(z - s_x xh)|, |z - z~|,
// |dir.(z - z~)|, |s_x xh|, |s_x xl / 256|
hipError_t launch_quant_rows(const float* X, const float* inv32, const float* mu, const float* dir, float sx,
                             int64_t row0, int64_t n, int G, float* Xq, unsigned long long* stats, hipStream_t st, int8_t* xh_rm = nullptr);
// queries -> int8 tiles Qq (G8 + QG_EXTRA groups), per query lsl / qerr, per batch qscal[3]
hipError_t launch_prep8(const float* Q, const double* qn64, const float* qmax, int B, int Bp, int D, int G8,
                        int metric, int prec, const Int8Consts& c, float* Qq, float* lsl, float* qerr, float* qscal,
                        hipStream_t st, float* qres = nullptr, float* qerr2 = nullptr);
// The int8 pass's checksum (vdb_scan8.hip): column sums of the int8 copy's two planes over rows
// [row0, row0 + n) added into csum [2][Dp]; the L2 start values' sum for a batch (*out +=); and a
// test-only corpus fault (one row's planes set to -127, the column sums left as they were)
hipError_t launch_colsum8(const float* Xq, int64_t row0, int64_t n, int G8, uint32_t* csum, hipStream_t st);
hipError_t launch_rstart8(const float* rinit, int64_t N, const float* qscal, int* rs, uint32_t* sum, hipStream_t st);
hipError_t launch_sink_row8(float* Xq, int64_t row, int G8, hipStream_t st);
// (csum / chke, optional: the first workgroup of each query block also writes the int8 pass's
// checksum expectations per query, chke [B][2] -- see FinishArgs::chke)
hipError_t launch_pilot8(int prec, int metric, const float* Xq, const float* rinit, const uint32_t* mask,
                         const float* Qq, const float* qscal, int G8, int64_t N, int B, int n_qblocks, int QB,
                         int n_sample, uint32_t* pslots, hipStream_t st, const uint32_t* csum = nullptr,
                         uint32_t* chke = nullptr, bool wide = false);
int scan8_rows_per_step(int prec, int metric);  // (64 queries per block of the int8 pass)
// the wide int8 pass (vdb_scan8w.hip): rows of 4 groups, batches of more than 256; W8_CH slots per
// (workgroup, query) segment of the candidate lists
constexpr int W8_CH = 32;
bool scan8w_ok(int G8, int B);
// its long-row form (vdb_scan8wl.hip): I8 cosine, 16 / 24 / 32 / 48 groups, 129..256 queries
bool scan8wl_ok(int prec, int metric, int G8, int B);
hipError_t launch_scan8wl(int prec, int metric, const float* Xq, const uint32_t* mask, const float* Qq,
                          const float* lsl, const float* qscal, int G8, int64_t N, int B, int n_seg, float* gl_s,
                          uint32_t* gl_i, int64_t gl_cap, uint32_t* seg_cnt, const uint32_t* gthr, uint32_t* chkp,
                          hipStream_t st);
hipError_t launch_scan8w(int prec, int metric, const float* Xq, const int* rs8, const uint32_t* mask, const float* Qq,
                         const float* lsl, const float* qscal, int G8, int64_t N, int B, int Bp, int n_seg,
                         float* gl_s, uint32_t* gl_i, int64_t gl_cap, uint32_t* seg_cnt, const uint32_t* gthr,
                         uint32_t* chkp, int chk_ld, int chk_l, hipStream_t st);
hipError_t launch_scan8(int prec, int metric, int KP, const float* Xq, const float* rinit, const uint32_t* mask,
                        const float* Qq, const float* lsl, const float* qscal, int G8, int64_t N, int B,
                        int n_qblocks, int64_t n_steps, int n_wg, int spw, float* gl_s, uint32_t* gl_i,
                        uint32_t* gl_cnt, int64_t gl_cap, uint32_t* gthr,
                        int lockstep, int qlds, hipStream_t st, const int* gate = nullptr,
                        uint32_t* chkp = nullptr, int chk_ld = 0, int chk_l = 0);

// Ingest: row-major fp32 [n][D] (device) -> the index's row-major fp32 copy X [cap][Dp]
// (zero padded to Dp = 8 G; read by the exact paths, export and the graph) rows [row0, row0+n),
// canonical fp64 norms, fp32 inverse norms and squared norms, running maxima (as
// fp64 bits) xmax_bits[0] = |x|, [1] = |x - bf16(x)| / |x|, [2] = |x - bf16(x)|,
// and a non-finite counter.
// Also rinit32[row] = -|x|^2 / 2 (the split pass's L2 accumulator start, vdb_scan2.hip), and the
// residuals use the row the split copy will hold: x * inv32 for cosine (normalise = 1), x for L2.
hipError_t launch_pack_rows(const float* src, int64_t n, int D, int G, float* X, int64_t row0,
                            double* nrm64, float* inv32, float* sq32, float* rinit32, int normalise,
                            unsigned long long* xmax_bits, int* nonfinite, hipStream_t st);

// Row-major fp32 rows -> split-bf16 tiles (hi = bf16(y), lo = bf16(y - hi)) for the whole row tiles
// covering rows [row0, row0 + n), y = x * inv32[row] (cosine: the normalised row, as the
// candidate pass scores it) or y = x (inv32 == nullptr, L2).  G = fp32 groups (Dp/8); the
// split copy has G/2 groups.
// PREC_BF16 residual bound along a direction (vdb_ingest.hip): column sums of the split
// copy's rows, then max |dir . (y - bf16(y))| over rows.
hipError_t launch_dir_sum(const float* X, const float* inv32, int64_t row0, int64_t n, int D, int G, double* sums,
                          hipStream_t st);
hipError_t launch_resid_dir(const float* X, const float* inv32, int64_t row0, int64_t n, int D, int G,
                            const float* dir, unsigned long long* out, hipStream_t st);
hipError_t launch_split_rows(const float* X, int G, int64_t row0, int64_t n, const float* inv32, float* Xs,
                             hipStream_t st);

// Row-major fp32 rows -> fp32 tiles (the PREC_FP32 candidate copy), whole row tiles.
hipError_t launch_tile_rows(const float* X, int G, int64_t row0, int64_t n, float* Xt, hipStream_t st);

// The index's rows -> row-major fp32 [n][D] (export for persistence).
hipError_t launch_unpack_rows(const float* X, int G, int D, int64_t row0, int64_t n, float* dst, hipStream_t st);

// gthr[B]: per-query shared threshold (order-preserving score key, 0 = none) and
// gslots[B][KP_MAX]: per-query slots of published workgroup bests; both zeroed by
// prep_queries (see the publish step of scan_topk_kernel).
constexpr int KP_MAX = 256;
constexpr int PILOT_SLOTS = 256;  // pilot bound slots per query
// pslots layout: slot-major, [PILOT_SLOTS][B] (a pilot wave's 32 queries of one tile -> one 128-byte
// segment per atomic instruction; query-major, each went to 32 cache lines: the guide's
// 17x-slower scattered-atomic shape, ~100 us of C4's 219 us pilot)
__host__ __device__ inline size_t pslot_at(int q, int slot, int B) { return (size_t)slot * B + q; }
// Queries: row-major [B][D] -> tiled Qt [Bp/32 tiles] with G + QG_EXTRA groups
// (the first QG_EXTRA groups repeated at the end; cosine: pre-normalised in
// fp32; zero padding written) and/or the split-bf16 tiles Qs (G/2 + QG_EXTRA
// groups, same wrap), canonical fp64 norms [Bp]; resets *flag_count and done[Bp] (the
// gated fallback's per-query counters, ExactTail).
// qmax (optional, the int8 pass): per query max |q'| over its dims (q' cosine-normalised).
hipError_t launch_prep_queries(const float* Q, int B, int Bp, int D, int G, int metric,
                               float* Qt, float* Qs, double* qn64, int* flag_count, uint32_t* gthr,
                               uint32_t* gslots, uint32_t* gl_cnt, int* done, hipStream_t st,
                               float* qmax = nullptr, const float* mu = nullptr, const float* dir = nullptr,
                               double* qconst = nullptr);

// Candidate pass: MFMA fp32 scores fused with a per-workgroup top-KP.
// Output lists cand_[s|i][B][n_wg][KP], each sorted best first.
// X / Qt are the fp32 tiles (prec 0, G = Dp/8 groups) or the split tiles (prec 1, G = Dp/16).
int scan_rows_per_step(int prec, int variant);
int scan_wgs_per_cu(int prec, int variant, int KP);  // resident workgroups per CU the variant is built for
bool scan_variant_ok(int prec, int variant, int G);
hipError_t launch_scan_topk(int prec, int metric, int KP, int variant, const float* X, const float* rowscale,
                            const uint32_t* mask, const float* Qt, int G, int64_t N, int B, int n_qblocks, int64_t n_steps,
                            int n_wg, int steps_per_wg, float* gl_s, uint32_t* gl_i, uint32_t* gl_cnt, int64_t gl_cap,
                            uint32_t* gthr, uint32_t* gslots, int lockstep, hipStream_t st);

// Wave-private candidate pass (scan_priv(prec, variant, KP)): entries above the
// shared bound are appended to global per-query lists gl_[s|i][B][gl_cap] (gl_cnt
// zeroed by prep_queries); select_topk takes the sorted top KP of each list.
bool scan_priv(int prec, int variant, int KP);
int scan_priv_capw();
hipError_t launch_scan_topk_priv(int prec, int metric, int KP, const float* X, const float* rowscale,
                                 const uint32_t* mask, const float* Qt, int G, int64_t N, int B, int n_qblocks,
                                 int64_t n_steps, int n_wg, int spw, float* gl_s, uint32_t* gl_i, uint32_t* gl_cnt,
                                 int64_t gl_cap, uint32_t* gthr, uint32_t* gslots, hipStream_t st);
hipError_t launch_select_topk(const float* gl_s, const uint32_t* gl_i, const uint32_t* gl_cnt, int64_t gl_cap, int KP,
                              int B, float* out_s, uint32_t* out_i, hipStream_t st);

// Pilot bound: scan-identical scores of n_sample evenly spaced row tiles; tile i's
// best score per query goes into pilot slot (i mod PILOT_SLOTS) (atomicMax), then
// gthr[q] = max(gthr[q], KP-th largest slot) -- `KP` here is the bound's rank (vdb_api.cpp
// pilot_rank).  pslots zeroed by prep_queries.
hipError_t launch_pilot(int prec, int metric, int KP, const float* X, const float* rowscale, const uint32_t* mask,
                        const float* Qt, int G, int64_t N, int B, int n_qblocks, int QB, int n_sample,
                        uint32_t* pslots, uint32_t* gthr, hipStream_t st);

hipError_t launch_pilot_bound(uint32_t* pslots, int B, int KP, uint32_t* gthr, hipStream_t st);

// Split-bf16 candidate pass (vdb_scan2.hip; PREC_BF16X3 / PREC_BF16): Xs = the split copy
// (cosine: of the NORMALISED rows), rinit = -|x|^2/2 per row (L2 accumulator start), Qs =
// split query tiles (prep_queries), G = 16-dim groups.  Steps of scan2_rows_per_step() rows.
int scan2_rows_per_step(bool q4 = false);
int scan2_qb(int KP);
// q4: the 128-query shape of the split pass (query block in LDS: D <= 128; KP = 128; 2 row
// tiles per wave, steps of scan2_rows_per_step(true) rows; a workgroup keeps 48 per query)
hipError_t launch_scan2(int prec, int metric, int KP, const float* Xs, const float* rinit, const uint32_t* mask,
                        const float* Qs, int G, int64_t N, int B, int n_qblocks, int64_t n_steps, int n_wg, int spw,
                        float* gl_s, uint32_t* gl_i, uint32_t* gl_cnt, int64_t gl_cap, uint32_t* gthr,
                        int lockstep, hipStream_t st, bool q4 = false, int qlds = -1, const int* gate = nullptr);
// Pilot scores for the split pass: fills pslots only; the bound kernel (launch_pilot_bound) takes
// the rank-th best of them into gthr.
hipError_t launch_pilot2(int prec, int metric, int KP, const float* Xs, const float* rinit, const uint32_t* mask,
                         const float* Qs, int G, int64_t N, int B, int n_qblocks, int QB, int n_sample,
                         uint32_t* pslots, uint32_t* gthr, hipStream_t st);

// Merge sorted per-workgroup lists -> sorted top-KP per query (fp32 keys).
hipError_t launch_merge_f32(int KP, const float* ls, const uint32_t* li, int n_lists, int B,
                            float* out_s, uint32_t* out_i, hipStream_t st);

// Exact fp64 rerank of the KP candidates + certificate check.
struct RerankArgs {
    const float* Q; const double* qn64; const float* X; int G; int D;
    const double* nrm64; const float* app_s; const uint32_t* app_i;
    int k; double eps_rel; double xmax;
    float* out_s; int64_t* out_i; double* out_k; int64_t index_offset;
    int* flag_count; int* flag_list;
    const uint32_t* gthr;  // final shared bound per query (rows at or below it may have been discarded)
};
hipError_t launch_rerank(int metric, int KP, const RerankArgs& a, int B, hipStream_t st);

// Fused select (top KP of each global candidate list) + exact rerank + certificate.
struct FinishArgs {
    int small = 0;  // the 4-wave form with a 4096-entry buffer (vdb_exact.hip FIN_CAP_SMALL)
    const float* gl_s; const uint32_t* gl_i; const uint32_t* gl_cnt; int64_t gl_cap;
    const float* Q; const double* qn64; const float* X; int G; int D; const double* nrm64;
    int k; double eps_rel; double xmax;
    double xres;  // PREC_BF16: bound of |q.(x - bf16(x))| per unit |q| (cosine: relative, L2: absolute)
    // PREC_BF16, optional: unit-ish direction dir [D] and M = 1.01 max |dir.(y - bf16(y))|: the
    // bound per query becomes min(|q| R, |q - c dir| R + |c| M), c = q.dir (R = xres)
    const float* dir = nullptr;
    double dres = 0.0;
    // the int8 pass, optional: the query's own share of eps per query (prep8: query rounding,
    // dropped terms, L2 start rounding), added to the certificate's eps
    const float* qerr = nullptr;
    // the int8 pass's centring row (its scores leave out mu.q; the exact-key certificate adds it)
    const float* mu = nullptr;
    // optional, per query [Bp][3] from prep_queries: mu.q', dir.q', |q' - (dir.q') dir|^2 (fp64;
    // q' the pass's query, cosine unit) -- computed there for the whole batch at once instead of
    // by two waves of each finish workgroup (three dependent fp64 passes over the query, ~14 us)
    const double* qconst = nullptr;
    float* out_s; int64_t* out_i; double* out_k; int64_t index_offset;
    int* flag_count; int* flag_list; const uint32_t* gthr;
    int* overflow_count;  // lists longer than the finish kernel holds (they take the exact path)
    int* incons_count = nullptr;  // optional: queries flagged by the approx-vs-exact consistency guard
    const int* gate = nullptr;  // optional (device re-pass): only queries b < *gate are finished
    // optional, the I8 pass: refine each candidate's approximate score with the query's rounding
    // residual (a' = a + f s_x xh.r, f = 1 cosine / 2 L2) before the rerank cut, so only the
    // corpus term is left of eps (qerr2 = the query's share without its rounding term)
    const int8_t* xh_rm = nullptr;  // the xh plane row-major [rows][Dp]
    const float* qres = nullptr;    // r = q' - s_q qh per query [Bp][Dp]
    const float* qerr2 = nullptr;
    const float* qscal = nullptr;   // [0] = s_x s_q
    float sx = 0.0f;
    int Dp = 0;
    const int64_t* row_ids = nullptr;  // global id per row (multi-device shard), else row + index_offset
    // split > 1: split workgroups per query share the exact rerank (rows by row % split); their
    // shares go to sx_* [B][split][KP] (+ counts sx_n [B][split]) and the last one (done[b],
    // zero on entry, reset on exit) ranks and writes
    int split = 1;
    double* sx_ek = nullptr; uint32_t* sx_ck = nullptr; uint32_t* sx_cr = nullptr; int* sx_n = nullptr;
    int* done = nullptr;
    // optional, the int8 pass's checksum (vdb_scan8.hip): per-workgroup partial sums of the H (and
    // L) accumulators chkp [2][chk_ld][chk_nw]; the value the operands imply is computed here from
    // the query's int8 tiles chk_q (prep8's, chk_g8 32-dim groups) and the copy's column sums
    // chk_csum [2][Dp], plus for L2 the start values' sum *chkr; a mismatch flags the query
    const uint32_t* chkp = nullptr;
    const uint32_t* chke = nullptr;  // the expectations from the pilot (else computed here from chk_q)
    const uint32_t* chkr = nullptr;
    const float* chk_q = nullptr;
    const uint32_t* chk_csum = nullptr;
    int chk_nw = 0, chk_ld = 0, chk_g8 = 0;
    bool chk_l = false;
    // optional, the wide int8 pass (vdb_scan8w.hip): the lists are seg_n segments of W8_CH slots
    // per query, one per scan workgroup, with counts seg_cnt [B][seg_n] (> W8_CH: overflowed)
    const uint32_t* seg_cnt = nullptr;
    int seg_n = 0;
};
hipError_t launch_finish(int metric, int KP, const FinishArgs& a, int B, hipStream_t st);

// Exact fp64 scan of the whole corpus for the queries in qlist[0..nq):
// per-workgroup sorted top-KE lists [nq][n_wg][KE] (fp64 keys, local rows).
// Device-gated form (qcount != nullptr): the flagged queries qlist[0 .. *qcount) are
// only known on the device; nq is then the most the lists have room for, and block
// (0, 0) adds *qcount / *ovf to the cumulative totals[0] / totals[1].
// With a tail (device-gated form only), the workgroup that finishes a query slot's lists
// last (done[slot] counts them; zeroed by prep_queries) merges them into mk / mi [nq][KE]
// and writes the query's results: one launch instead of scan + merge + finalize.
// host_totals (optional, bf16 searches of VDB_PREC_AUTO): block (0, 0) adds the flagged
// count to totals[2] too and writes that total to this pinned host word (read by the next
// search, without a copy or a sync).
struct ExactTail {
    int* done; double* mk; uint32_t* mi; int k; int64_t index_offset;
    float* out_s; int64_t* out_i; double* out_k; const int64_t* row_ids;
    unsigned long long* host_totals = nullptr;
};
hipError_t launch_exact_scan(int metric, int KE, const float* Q, const double* qn64, const int* qlist, int nq,
                             const float* X, int G, int D, const double* nrm64, const uint32_t* mask,
                             int64_t N, int n_wg, int64_t rows_per_wg,
                             double* lk, uint32_t* li, hipStream_t st, const int* qcount = nullptr,
                             const int* ovf = nullptr, unsigned long long* totals = nullptr,
                             const ExactTail* tail = nullptr, int gate_slots = 4, char* gscr = nullptr);
// bytes of the device-gated exact scan's global scratch (gscr above): the per-wave top-k buffers
// of slots x n_wg workgroups and one tail-merge scratch per slot
size_t exact_scan_scratch_bytes(int KE, int n_wg, int slots);

// Merge sorted fp64-key lists.  Element (q, j, e) lives at q*sq + j*sj + e, lists
// have Lk entries; output [nq][KP] sorted.
hipError_t launch_merge_f64_u32(int KP, const double* lk, const uint32_t* li, int n_lists, int Lk,
                                int64_t sq, int64_t sj, int nq, double* out_k, uint32_t* out_i, hipStream_t st,
                                const int* qcount = nullptr);
hipError_t launch_merge_f64_i64(int KP, const double* lk, const int64_t* li, int n_lists, int Lk,
                                int64_t sq, int64_t sj, int nq, double* out_k, int64_t* out_i, hipStream_t st);

// Write final results for query rows qmap[q] (or q if qmap == nullptr) from
// sorted [nq][KP] fp64-key lists.
hipError_t launch_finalize_u32(int metric, const double* sk, const uint32_t* si, int KP, int nq, const int* qmap,
                               int k, int64_t index_offset, float* out_s, int64_t* out_i, double* out_k,
                               hipStream_t st, const int* qcount = nullptr, const int64_t* row_ids = nullptr);
hipError_t launch_finalize_i64(int metric, const double* sk, const int64_t* si, int KP, int nq, const int* qmap,
                               int k, float* out_s, int64_t* out_i, double* out_k, hipStream_t st);
// out[r] = Q[list[r]] (rows of D floats), r < n
hipError_t launch_gather_rows(const float* Q, int D, const int* list, int n, float* out, hipStream_t st);
// The device-memory re-pass (vdb_api.cpp): the first min(c, R) of the c = flags[0] flagged queries
// flags[1..c] gathered into out [R][D]; counts[0] = min(c, R) (the sub-search's gate), counts[1] =
// max(c - R, 0) (left to the exact path); totals (optional) += counts[0].
hipError_t launch_repass_gather(const float* Q, int D, const int* flags, int R, float* out, int* counts,
                                unsigned long long* totals, hipStream_t st);
// o*[list[r]][e] = s*[r][e] for r < n, e < k (ok may be NULL)
hipError_t launch_scatter_results(const int* list, int n, int k, const float* ss, const int64_t* si, const double* sk,
                                  float* os, int64_t* oi, double* ok, hipStream_t st, const int* n_dev = nullptr);
// n "no result" entries: score 0, row -1, key -inf (as write_result's invalid entries)
hipError_t launch_empty_results(int64_t n, float* out_s, int64_t* out_i, double* out_k, hipStream_t st);

// Graph search (vdb_graph.hip): one workgroup per query, beam of ef over a [N][R]
// int32 neighbour array (-1 = none), started from the best of n_entries entry rows.
struct GraphSearchArgs {
    const float* rows; int Dp; int D; const float* rowscale; int64_t n_rows;  // rows: the index's row-major X [.][Dp]
    const int32_t* nbr; int R; const int32_t* entries; int n_entries;
    const float* Q; int k; int ef;
    int64_t* out_lab; float* out_dist; unsigned long long* stats;
    int teams = 1;                                          // workgroups per query (disjoint entry slices)
    int64_t* tmp_lab = nullptr; float* tmp_dist = nullptr;  // teams > 1: per-team lists [nq][teams][k]
};
hipError_t launch_graph_search(int metric, const GraphSearchArgs& a, int nq, hipStream_t st);


// Graph build: hnswlib's neighbour-selection heuristic per node over up to 63
// candidates cand[v][0..cw) (nearest first, -1 padded at the tail); out_nbr /
// out_dist [v][rw] get the kept rows (nearest first) and their distances
// (cosine 1 - cos, L2 squared), -1 / +inf padded.  fill: top up with pruned ones.
// nodes (optional): node id of work item i (else i); cand / out rows are per work item.
// sort: visit the candidates by distance to the node (computed in the kernel) instead of
// in the given order (the given order must then be nearest first, -1 padded at the tail).
struct GraphPruneArgs {
    const float* X; int G; const float* rowscale;
    const int32_t* cand; int cw; int64_t n_nodes; int limit; int rw; int fill;
    int32_t* out_nbr; float* out_dist;
    const int32_t* nodes = nullptr; int sort = 0;
};
// nbr[ids[i]][0..R) = rows[i][0..R) for i < n (incremental graph updates)
hipError_t launch_graph_scatter(int32_t* nbr, int R, const int32_t* ids, const int32_t* rows, int64_t n,
                                hipStream_t st);
hipError_t launch_graph_prune(int metric, const GraphPruneArgs& a, hipStream_t st);

// Operator slot (vdb_ops.hip): full score matrix out[B][N] of row-major X [N][D], Q [B][D]:
// metric 0 cosine / 2 dot product (fp32 MFMA GEMM), 1 euclidean (direct differences).
hipError_t launch_similarity_matrix(const float* X, int64_t N, int D, const float* Q, int B, int metric,
                                    float* out, hipStream_t st);
// x / max(|x|, 1e-8) per row
hipError_t launch_normalize_rows(const float* in, int64_t n, int D, float* out, hipStream_t st);
// top-k of each of `rows` score rows of length n (largest or smallest first, ties to the
// lower index, NaN last); ws: topk_workspace_bytes(n, rows, k) bytes of device memory
size_t topk_workspace_bytes(int64_t n, int rows, int k);
hipError_t launch_topk_scores(const float* S, int rows, int64_t n, int k, int largest, int64_t* out_idx,
                              float* out_val, void* ws, hipStream_t st);

}  // namespace vdb
