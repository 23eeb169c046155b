// vdb_api.cpp — the C-ABI (include/vdb.h): index object, workspace pool and the
// search driver that sequences the kernels of vdb_kernels.hip.
//
// Host-side restatement of the reference store's operator flow
// (service/optimized_vector_store.py:96-192): ingest appends rows in place and
// computes norms once (instead of re-normalising the corpus on every query,
// :31-41); search = candidate pass + exact rerank instead of a full argsort
// (:176-183).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <set>
#include <unordered_map>
#include <shared_mutex>
#include <string>
#include <vector>

#include "../../include/vdb.h"
#include "vdb_internal.h"

using namespace vdb;

namespace {

thread_local std::string g_last_error;

int set_error(int code, const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

#define HIP_TRY(expr)                                                                                  \
    do {                                                                                               \
        hipError_t _e = (expr);                                                                        \
        if (_e != hipSuccess)                                                                          \
            return set_error(_e == hipErrorOutOfMemory ? VDB_ERR_OOM : VDB_ERR_HIP, "%s failed: %s (%s:%d)", \
                             #expr, hipGetErrorString(_e), __FILE__, __LINE__);                        \
    } while (0)

constexpr int64_t kRowAlign = ROW_ALIGN;   // capacity granule, a multiple of every scan step

constexpr size_t kGatedExactBytes = 256u << 20;  // device-gated fallback lists sized for every query of a batch
constexpr int kMaxApproxK = 200;          // k above this uses the exact path

inline int64_t round_up(int64_t a, int64_t b) { return (a + b - 1) / b * b; }
inline int next_pow2(int v) {
    int p = 1;
    while (p < v) p <<= 1;
    return p;
}

// Bump allocator over one device buffer (256-B aligned carve).
struct Carver {
    char* base;
    size_t off = 0;
    template <typename T>
    T* take(size_t count) {
        off = (off + 255) & ~size_t(255);
        T* p = reinterpret_cast<T*>(base + off);
        off += count * sizeof(T);
        return p;
    }
};

struct Workspace {
    char* dev = nullptr;
    size_t dev_bytes = 0;
    char* exact = nullptr;  // exact-path lists, grown on demand
    size_t exact_bytes = 0;
    int* host_flag = nullptr;  // pinned
    // pinned staging of a host-memory search: the queries up, the results down (read with the
    // certificate's flags in one synchronisation; grown on demand)
    char* host_io = nullptr;
    size_t host_io_bytes = 0;
    hipEvent_t done = nullptr;
    // timing (vdb_index_set_param "timing"): a ring of event sets, one per timed search
    // (scan start / scan end / finish end / pilot start), read once complete, so timed
    // device-memory searches can be queued back to back without a host wait
    static constexpr int kTRing = 64;
    hipEvent_t tring[kTRing][4] = {};
    int t_head = 0, t_pending = 0;
    bool busy = false;
    bool used = false;
    hipStream_t last_st = nullptr;  // stream of the last search that used it
    // host-memory searches without a caller stream run on their workspace's own stream, so
    // concurrent host searches (the reference's 4-thread executor, api/routes/vectors.py:43)
    // overlap on the device instead of queueing on one index stream
    hipStream_t own = nullptr;
};

}  // namespace

struct vdb_index {
    int dim = 0, metric = 0, device = 0;
    int Dp = 0, G = 0;
    int64_t count = 0;
    int64_t cap_rows = 0;  // multiple of kRowAlign
    float* X = nullptr;   // row-major fp32 [cap_rows][Dp] (rerank, exact scan, export, graph)
    float* Xs = nullptr;  // the candidate pass's copy, same bytes: split-bf16 tiles (PREC_BF16X3 / BF16 /
                          // AUTO) or fp32 tiles (PREC_FP32), rebuilt from X when the precision class changes.
                          // AUTO with the int8 copy allocates it lazily, on the first search that runs a
                          // split pass (a hold, a host re-pass or retry): ensure_xs
    float* Xq = nullptr;  // the int8 copy (PREC_I8 / I8X3, AUTO with auto_i8): half the bytes of X
    // its xh plane row-major [cap][Dp] (with Xq): the finish refines I8 candidates' scores with
    // the query's rounding residual, reading each candidate's row whole (vdb_exact.hip)
    int8_t* Xh = nullptr;
    double* nrm64 = nullptr;
    float* inv32 = nullptr;
    float* sq32 = nullptr;
    float* rinit32 = nullptr;  // -|x|^2 / 2: the split pass's L2 accumulator start (vdb_scan2.hip)
    unsigned long long* d_xmax = nullptr;
    int* d_nonfinite = nullptr;
    double xmax = 0.0;
    double xres_rel = 0.0, xres_abs = 0.0;  // max |x - bf16(x)| / |x| and max |x - bf16(x)| (PREC_BF16 bound)
    // PREC_BF16 bound along a direction: dir = the normalised mean of the split
    // copy's rows of the first add (up to kDirRows of them), frozen until clear();
    // xres_dir = max |dir . (y - bf16(y))| over all rows
    float* d_dir = nullptr;  // [Dp], zero padded
    bool dir_set = false;
    double xres_dir = 0.0;
    // The int8 pass (PREC_I8 / PREC_I8X3, vdb_scan8.hip): the candidate copy holds z = y - mu,
    // mu [Dp] the mean of the first add's candidate rows (set with dir, frozen until clear()),
    // quantised with step sx = 1.25 max |z| / 127 (over those rows; later rows past the range
    // clip, which the residual statistics then show); d_i8 [0..6) the running row statistics of
    // quant_rows (fp64 bits), [6] max |z| (float bits) at setup; i8st = their host copies.
    float* d_mu = nullptr;
    float sx = 0.0f;
    int64_t dir_rows = 0;  // rows dir / mu / sx were derived from (re-derived as the index doubles, up to kDirRows)
    unsigned long long* d_i8 = nullptr;
    double i8st[6] = {0, 0, 0, 0, 0, 0};
    // the int8 pass's checksum (vdb_scan8.hip): column sums (mod 2^32) of the int8 copy's xh and
    // xl planes over rows [0, count), [2][Dp]; kept by build_candidate_rows
    uint32_t* d_csum = nullptr;
    int64_t scan_checksum = 1;  // knob: 1 the pass's sums are checked by the finish, 0 off (A/B)
    // VDB_PREC_AUTO's candidate copy: the int8 one (I8 / I8X3) when set, else the split-bf16 one
    bool auto_i8 = true;
    hipStream_t stream = nullptr;
    int n_cu = 256;
    // knobs
    int64_t precision = VDB_PREC_AUTO;
    // VDB_PREC_AUTO: BF16 by default; a BF16 search whose uncertified queries are
    // too many for a re-pass (host memory: more than 1/8 of the batch; device memory: any, seen
    // lagged through h_totals) starts a HOLD of BF16X3 searches, 16 << (fails - 1) of them
    // (exponential backoff up to 2048 while probes keep failing; `fails` resets after 64 BF16
    // searches without a new failure, and hold and fails reset when the rows change).  So one
    // near-duplicate query no longer pins the index to BF16X3, and a corpus that never certifies
    // in BF16 pays a probe only once per 2048 searches.
    std::atomic<int> auto_hold{0}, auto_fails{0}, auto_ok{0};
    // With auto_i8, the one-plane pass is I8 (the int8 copy); an I8 failure too large for a
    // re-pass holds BF16 (the split copy) instead for 16 << (fails8 - 1) searches (up to 2048;
    // fails8 resets after 64 I8 searches without a new failure, both when the rows change), so
    // data where the 8-bit query's wider bound does not certify (1M x 1536) runs BF16 and probes
    // I8 rarely.  last_i8: the last one-plane pass was I8 (device-memory failures arrive late).
    std::atomic<int> auto_hold8{0}, auto_fails8{0}, auto_ok8{0};
    std::atomic<bool> last_i8{false};
    // The device-gated fallback total last seen: pinned mirror of d_totals[0], written by the
    // gated exact kernel of a device-memory search and read by the next search.
    std::atomic<unsigned long long> auto_seen{0};
    unsigned long long* h_totals = nullptr;
    int64_t margin = -1;  // -1 = default
    int64_t force_exact = 0;
    int64_t n_wg_override = 0;
    int64_t timing = 0;  // record HIP events around the candidate pass
    int64_t pilot_tiles = -1;  // row tiles sampled by the pilot bound (0 = off, -1 = by k)
    int64_t graph_fill = 0;     // graph build: top up pruned neighbour lists (hnswlib keepPrunedConnections)
    int64_t scan_variant = 0;     // fp32 candidate pass variant (vdb_scan.hip)
    int64_t scan_variant_b3 = 0;  // bf16x3 candidate pass variant
    int64_t scan_sync = 0;        // scan step end: 0 auto, 1 lockstep barrier, 2 flag-gated rounds
    int64_t no_fallback = 0;      // diagnostics only: skip the exact fallback (results may be wrong)
    int64_t pilot_rank_override = 0;  // tuning: rank of the pilot bound (0 = the Poisson rule)
    bool no_dir_bound = false;    // diagnostics: PREC_BF16 certificate with Cauchy-Schwarz only
    int64_t finish_split = 1;  // workgroups per query in the finish kernel (tuning)
    // the finish's small form (4 waves, 4096-entry buffer) that fits beside a long-row wide scan:
    // -1 auto (with that scan at <= 1024 dims), 0 off, 1 on
    int64_t finish_small = -1;
    int64_t scan_qlds = -1;    // split pass: query block in LDS when it fits (-1 auto), 0 never
    // the finish's I8 refinement (i8_refine): -1 auto = rows of kRefineMinDp dims or more (C3 +6%,
    // C2 neutral, C6 -1%: shorter rows rerank cheaply; profiles/r04_mx1); 0 off; 1 on
    int i8_refine = -1;
    // device-memory searches: uncertified queries of an I8 / BF16 / I8X3 pass re-passed in BF16X3
    // on the device (gated kernels, no host wait) instead of the fp64 exact scan.  -1 auto: armed
    // for kRepassArm searches once a device fallback has been seen; 0 off; 1 always
    int64_t device_repass = -1;
    std::atomic<int> repass_arm{0};
    // auto's I8 pass on indexes of <= kI8NarrowRows rows: KP = 128 instead of 256 (a weak-scaled
    // rank's shard: the k-th to KP-th gap widens as rows thin out) until any search of this index
    // flags a query, then 256 for good (i8_wide).  Knob "i8_narrow": -1 auto, 0 off.
    int64_t i8_narrow = -1;
    std::atomic<bool> i8_wide{false};
    // auto's L2 pass for 16 < k <= 100: PREC_I8Q (the xh plane against the 16-bit query) unless
    // "auto_i8q" = 0, or once a batch flagged more than 1/8 of its queries (i8q_off: I8X3 after)
    std::atomic<bool> auto_i8q{true};
    std::atomic<bool> i8q_off{false};
    // the last auto pass was I8Q, and its batch size: a device-memory search sees its flags a
    // search or more late (h_totals), and turns I8Q off by the same 1/8 rule
    std::atomic<bool> last_i8q{false};
    std::atomic<int> last_i8q_b{0};
    int64_t scan_q4 = -1;      // split pass 128-query shape (D <= 128, KP = 128, B >= 256): -1 auto, 0 off, 1 on
    // the wide int8 pass (vdb_scan8w.hip: rows of 4 groups, B > 256): -1 auto (from kWideMinRows
    // rows), 0 off, 1 at any row count
    int64_t scan_wide = -1;
    // stats
    std::atomic<int64_t> n_searches{0}, n_queries{0}, n_fallback{0}, n_overflow{0}, n_incons{0}, n_repass{0}, n_q4{0};
    std::atomic<int64_t> n_wide{0};  // searches through the wide int8 pass
    std::atomic<int64_t> n_xs_builds{0};  // lazy builds of the split copy (ensure_xs)
    std::atomic<int64_t> n_by_prec[N_PREC] = {{0}, {0}, {0}, {0}, {0}, {0}};  // candidate passes per PREC_* (VDB_PREC_AUTO's choices)
    std::atomic<int64_t> scan_ns{0}, pipe_ns{0}, n_timed{0};
    unsigned long long* d_totals = nullptr;  // device: flagged / overflowed / flagged-in-bf16 queries of device-gated searches
    std::shared_mutex mu;  // add/clear/reserve exclusive; search shared
    std::mutex xs_mu;      // the lazy split copy's allocation + build (under the shared lock)
    std::mutex ws_mu;
    std::vector<Workspace*> pool;
    // last work queued on each caller stream by searches without a workspace (graph searches):
    // wait_idle() waits for these and the workspaces' events instead of the whole device
    std::unordered_map<hipStream_t, hipEvent_t> uses;
};

namespace {

// Live indexes, for vdb_shutdown().
std::mutex g_reg_mu;
std::set<vdb_index*> g_indices;

void free_workspace_memory(Workspace* w) {
    if (w->dev) (void)hipFree(w->dev);
    if (w->exact) (void)hipFree(w->exact);
    if (w->host_flag) (void)hipHostFree(w->host_flag);
    if (w->host_io) (void)hipHostFree(w->host_io);
    w->dev = nullptr;
    w->exact = nullptr;
    w->host_flag = nullptr;
    w->host_io = nullptr;
    w->dev_bytes = w->exact_bytes = w->host_io_bytes = 0;
}

int wait_idle(vdb_index* ix);

// The candidate copies a precision setting keeps: Xs holds fp32 tiles (FP32), split-bf16 tiles
// (BF16 / BF16X3 / AUTO) or nothing (I8 / I8X3); Xq the int8 copy (I8 / I8X3, AUTO with auto_i8:
// AUTO keeps both and picks per batch, vdb_index_search).
enum XsKind { kXsNone = -1, kXsFp32 = 0, kXsSplit = 1 };
int xs_kind(int64_t precision) {
    if (precision == VDB_PREC_FP32) return kXsFp32;
    if (precision == VDB_PREC_I8 || precision == VDB_PREC_I8X3 || precision == VDB_PREC_I8Q) return kXsNone;
    return kXsSplit;
}
bool needs_i8(int64_t precision, bool auto_i8) {
    return precision == VDB_PREC_I8 || precision == VDB_PREC_I8X3 || precision == VDB_PREC_I8Q ||
           (precision == VDB_PREC_AUTO && auto_i8);
}
// Settings whose candidate pass reads Xs on every search keep it allocated and up to date from the
// start; AUTO with the int8 copy reads it only for holds, host re-passes and retries, so it is
// built on first use (ensure_xs): 7 instead of 11 B per element (fp32 rows 4, int8 planes 2, the
// row-major xh 1) while no search needs it.  I8 / I8X3 never read it.
bool xs_eager(const vdb_index* ix) {
    const int kind = xs_kind(ix->precision);
    return kind == kXsFp32 || (kind == kXsSplit && !(ix->precision == VDB_PREC_AUTO && ix->auto_i8));
}
float* xs_ptr(const vdb_index* ix) { return __atomic_load_n(&ix->Xs, __ATOMIC_ACQUIRE); }

// The candidate copies of rows [row0, row0 + n) from the row-major rows (tiles: whole row tiles;
// the int8 copy row by row, its statistics into d_i8).  xs / xq: which copies to build.
hipError_t build_candidate_rows(const vdb_index* ix, int64_t row0, int64_t n, hipStream_t st, bool xs = true,
                                bool xq = true) {
    const float* inv = ix->metric == VDB_METRIC_COSINE ? ix->inv32 : nullptr;
    hipError_t e = hipSuccess;
    if (xs && ix->Xs && xs_kind(ix->precision) == kXsFp32) e = launch_tile_rows(ix->X, ix->G, row0, n, ix->Xs, st);
    if (xs && ix->Xs && xs_kind(ix->precision) == kXsSplit) e = launch_split_rows(ix->X, ix->G, row0, n, inv, ix->Xs, st);
    if (e == hipSuccess && xq && needs_i8(ix->precision, ix->auto_i8)) {
        // (rows [0, n) rebuild the whole copy: its column sums start again)
        if (row0 == 0) e = hipMemsetAsync(ix->d_csum, 0, (size_t)2 * ix->Dp * sizeof(uint32_t), st);
        if (e == hipSuccess)
            e = launch_quant_rows(ix->X, inv, ix->d_mu, ix->d_dir, ix->sx, row0, n, ix->G, ix->Xq, ix->d_i8, st, ix->Xh);
        if (e == hipSuccess) e = launch_colsum8(ix->Xq, row0, n, ix->G / 4, ix->d_csum, st);
    }
    return e;
}

// Host copies of the int8 copy's row statistics (after the kernels that update them).
hipError_t read_i8_stats(vdb_index* ix, hipStream_t st) {
    unsigned long long b[6];
    hipError_t e = hipMemcpyAsync(b, ix->d_i8, sizeof(b), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e == hipSuccess) std::memcpy(ix->i8st, b, sizeof(b));
    return e;
}

// Device memory zeroed and the zeroing finished when this returns, so work on ANY stream after it
// sees zeros.  (hipMemset enqueues on the null stream, which the library's and the callers'
// non-blocking streams are not ordered after.)
hipError_t zero_now(void* p, size_t bytes, hipStream_t st) {
    hipError_t e = hipMemsetAsync(p, 0, bytes, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    return e;
}

bool debug_knobs_enabled() {
    const char* e = std::getenv("VDB_DEBUG_KNOBS");
    return e && std::strcmp(e, "1") == 0;
}

int ensure_capacity(vdb_index* ix, int64_t rows) {
    if (rows <= ix->cap_rows) return VDB_OK;
    if (ix->X) {  // every search that might read the old buffers is done (callers hold the write lock)
        const int wr = wait_idle(ix);
        if (wr) return wr;
    }
    int64_t cap = std::max<int64_t>(ix->cap_rows * 2, kRowAlign);
    while (cap < rows) cap *= 2;
    cap = round_up(cap, kRowAlign);
    const size_t tile_floats = (size_t)ix->G * BLOCK_FLOATS;
    const size_t x_bytes = (size_t)(cap / 32) * tile_floats * sizeof(float);
    float* X = nullptr;
    float* Xs = nullptr;
    float* Xq = nullptr;
    int8_t* Xh = nullptr;
    double* n64 = nullptr;
    float *i32 = nullptr, *s32 = nullptr, *r32 = nullptr;
    // All new buffers are allocated and filled before the index switches to them; on
    // any failure (typically out of memory while doubling at large N) they are freed
    // and the index keeps its current buffers, so a later retry sees the same HBM.
    auto fail = [&](hipError_t e, const char* what) {
        (void)hipStreamSynchronize(ix->stream);
        for (void* p : {(void*)X, (void*)Xs, (void*)Xq, (void*)Xh, (void*)n64, (void*)i32, (void*)s32, (void*)r32})
            if (p) (void)hipFree(p);
        return set_error(e == hipErrorOutOfMemory ? VDB_ERR_OOM : VDB_ERR_HIP,
                         "growing the index to %lld rows: %s failed: %s", (long long)cap, what, hipGetErrorString(e));
    };
#define CAP_TRY(expr)                          \
    do {                                       \
        hipError_t _e = (expr);                \
        if (_e != hipSuccess) return fail(_e, #expr); \
    } while (0)
    CAP_TRY(hipMalloc(&X, x_bytes));
    if (ix->Xs || xs_eager(ix)) {  // (AUTO with the int8 copy: lazily, ensure_xs)
        CAP_TRY(hipMalloc(&Xs, x_bytes));
        CAP_TRY(hipMemsetAsync(Xs, 0, x_bytes, ix->stream));
    }
    // the int8 copy only where a setting reads it (FP32 / BF16X3 / BF16 / AUTO without
    // auto_int8 never do; set_param allocates it when a setting starts to, ensure_xq)
    const bool with_xq = ix->Xq || needs_i8(ix->precision, ix->auto_i8);
    if (with_xq) {
        CAP_TRY(hipMalloc(&Xq, x_bytes / 2));
        CAP_TRY(hipMemsetAsync(Xq, 0, x_bytes / 2, ix->stream));
        CAP_TRY(hipMalloc(&Xh, x_bytes / 4));
        CAP_TRY(hipMemsetAsync(Xh, 0, x_bytes / 4, ix->stream));
    }
    CAP_TRY(hipMalloc(&n64, cap * sizeof(double)));
    CAP_TRY(hipMalloc(&i32, cap * sizeof(float)));
    CAP_TRY(hipMalloc(&s32, cap * sizeof(float)));
    CAP_TRY(hipMalloc(&r32, cap * sizeof(float)));
    CAP_TRY(hipMemsetAsync(r32, 0, cap * sizeof(float), ix->stream));
    CAP_TRY(hipMemsetAsync(X, 0, x_bytes, ix->stream));
    CAP_TRY(hipMemsetAsync(n64, 0, cap * sizeof(double), ix->stream));
    CAP_TRY(hipMemsetAsync(i32, 0, cap * sizeof(float), ix->stream));
    CAP_TRY(hipMemsetAsync(s32, 0, cap * sizeof(float), ix->stream));
    if (ix->X) {
        const int64_t used_tiles = round_up(ix->count, 128) / 32;  // whole super tiles (prefix of the layout)
        CAP_TRY(hipMemcpyAsync(X, ix->X, (size_t)ix->count * ix->Dp * sizeof(float), hipMemcpyDeviceToDevice,
                               ix->stream));
        if (Xs && ix->Xs)
            CAP_TRY(hipMemcpyAsync(Xs, ix->Xs, (size_t)used_tiles * tile_floats * sizeof(float),
                                   hipMemcpyDeviceToDevice, ix->stream));
        if (Xq && ix->Xq)
            CAP_TRY(hipMemcpyAsync(Xq, ix->Xq, (size_t)used_tiles * tile_floats * sizeof(float) / 2,
                                   hipMemcpyDeviceToDevice, ix->stream));
        if (Xh && ix->Xh)
            CAP_TRY(hipMemcpyAsync(Xh, ix->Xh, (size_t)ix->count * ix->Dp, hipMemcpyDeviceToDevice, ix->stream));
        CAP_TRY(hipMemcpyAsync(n64, ix->nrm64, ix->count * sizeof(double), hipMemcpyDeviceToDevice, ix->stream));
        CAP_TRY(hipMemcpyAsync(i32, ix->inv32, ix->count * sizeof(float), hipMemcpyDeviceToDevice, ix->stream));
        CAP_TRY(hipMemcpyAsync(s32, ix->sq32, ix->count * sizeof(float), hipMemcpyDeviceToDevice, ix->stream));
        CAP_TRY(hipMemcpyAsync(r32, ix->rinit32, ix->count * sizeof(float), hipMemcpyDeviceToDevice, ix->stream));
    }
    CAP_TRY(hipStreamSynchronize(ix->stream));
#undef CAP_TRY
    if (ix->X) {
        (void)hipFree(ix->X);
        if (ix->Xs) (void)hipFree(ix->Xs);
        if (ix->Xq) (void)hipFree(ix->Xq);
        if (ix->Xh) (void)hipFree(ix->Xh);
        (void)hipFree(ix->nrm64);
        (void)hipFree(ix->inv32);
        (void)hipFree(ix->sq32);
        (void)hipFree(ix->rinit32);
    }
    ix->X = X;
    ix->Xs = Xs;
    ix->Xq = Xq;
    ix->Xh = Xh;
    ix->nrm64 = n64;
    ix->inv32 = i32;
    ix->sq32 = s32;
    ix->rinit32 = r32;
    ix->cap_rows = cap;
    return VDB_OK;
}

// The int8 copy for a setting that starts to read it (lazily: ensure_capacity keeps it only
// while a setting does).  Zeroed; the caller rebuilds rows [0, count) (build_candidate_rows).
int ensure_xq(vdb_index* ix) {
    if (ix->Xq || ix->cap_rows == 0) return VDB_OK;
    const size_t bytes = (size_t)(ix->cap_rows / 32) * ix->G * BLOCK_FLOATS * sizeof(float) / 2;
    float* Xq = nullptr;
    int8_t* Xh = nullptr;
    hipError_t e = hipMalloc(&Xq, bytes);
    if (e == hipSuccess) e = hipMalloc(&Xh, bytes / 2);
    if (e == hipSuccess) e = hipMemsetAsync(Xq, 0, bytes, ix->stream);
    if (e == hipSuccess) e = hipMemsetAsync(Xh, 0, bytes / 2, ix->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ix->stream);
    if (e != hipSuccess) {
        if (Xq) (void)hipFree(Xq);
        if (Xh) (void)hipFree(Xh);
        return set_error(e == hipErrorOutOfMemory ? VDB_ERR_OOM : VDB_ERR_HIP, "int8 copy: %s", hipGetErrorString(e));
    }
    ix->Xq = Xq;
    ix->Xh = Xh;
    return VDB_OK;
}

// The candidate copy Xs for a search that runs a split (or fp32) pass while it is not allocated
// (AUTO with the int8 copy: xs_eager).  Called under the index's shared lock (no add, growth or
// clear runs meanwhile); concurrent searches serialise on xs_mu, and the first allocates it, builds
// rows [0, count) on the index's stream and waits, then publishes the pointer.
int ensure_xs(vdb_index* ix) {
    if (xs_ptr(ix) || ix->cap_rows == 0 || xs_kind(ix->precision) == kXsNone) return VDB_OK;
    std::lock_guard<std::mutex> lg(ix->xs_mu);
    if (ix->Xs) return VDB_OK;
    const size_t bytes = (size_t)(ix->cap_rows / 32) * ix->G * BLOCK_FLOATS * sizeof(float);
    float* Xs = nullptr;
    hipError_t e = hipMalloc(&Xs, bytes);
    if (e == hipSuccess) e = hipMemsetAsync(Xs, 0, bytes, ix->stream);
    if (e == hipSuccess && ix->count > 0) {
        const float* inv = ix->metric == VDB_METRIC_COSINE ? ix->inv32 : nullptr;
        e = xs_kind(ix->precision) == kXsFp32 ? launch_tile_rows(ix->X, ix->G, 0, ix->count, Xs, ix->stream)
                                              : launch_split_rows(ix->X, ix->G, 0, ix->count, inv, Xs, ix->stream);
    }
    if (e == hipSuccess) e = hipStreamSynchronize(ix->stream);
    if (e != hipSuccess) {
        if (Xs) (void)hipFree(Xs);
        return set_error(e == hipErrorOutOfMemory ? VDB_ERR_OOM : VDB_ERR_HIP, "split candidate copy: %s",
                         hipGetErrorString(e));
    }
    __atomic_store_n(&ix->Xs, Xs, __ATOMIC_RELEASE);
    ix->n_xs_builds++;
    return VDB_OK;
}

// A free workspace whose last search was queued on the same stream (stream order makes the
// reuse safe without a wait), else one whose last search has finished, else a new one (up to
// kMaxWs; then any free one, its reuse waiting on its last search): searches queued on several
// streams from one host thread (a server's request streams) then run concurrently instead of
// serialising on one workspace.
constexpr size_t kMaxWs = 16;

// own = a host-memory search that runs on the workspace's own stream: any free workspace
// whose last search has finished (or a new one) serves.
Workspace* acquire_ws(vdb_index* ix, hipStream_t st, bool own = false) {
    std::lock_guard<std::mutex> g(ix->ws_mu);
    Workspace* idle = nullptr;
    Workspace* any = nullptr;
    for (Workspace* w : ix->pool) {
        if (w->busy) continue;
        if (!w->used || (!own && w->last_st == st)) {
            w->busy = true;
            return w;
        }
        if (!idle && w->done && hipEventQuery(w->done) == hipSuccess) idle = w;
        if (!any) any = w;
    }
    Workspace* w = idle ? idle : ix->pool.size() >= kMaxWs ? any : nullptr;
    if (!w) {
        w = new Workspace();
        ix->pool.push_back(w);
    }
    w->busy = true;
    return w;
}

// Another search of this index on the device right now (being queued, or queued and not finished):
// the finish's small form pays off only when it can run beside another batch's scan.
bool others_in_flight(vdb_index* ix, const Workspace* self) {
    std::lock_guard<std::mutex> g(ix->ws_mu);
    for (Workspace* w : ix->pool) {
        if (w == self) continue;
        if (w->busy) return true;
        if (w->used && w->done && hipEventQuery(w->done) == hipErrorNotReady) return true;
    }
    return false;
}

void release_ws(vdb_index* ix, Workspace* w, hipStream_t st) {
    if (w->done == nullptr) (void)hipEventCreateWithFlags(&w->done, hipEventDisableTiming);
    (void)hipEventRecord(w->done, st);
    w->used = true;
    w->last_st = st;
    std::lock_guard<std::mutex> g(ix->ws_mu);
    w->busy = false;
}

// Remember the last work a search without a workspace queued on `st` (wait_idle).
int note_use(vdb_index* ix, hipStream_t st) {
    std::lock_guard<std::mutex> g(ix->ws_mu);
    // a server that makes a stream per request would grow this map without bound:
    // past 64 entries, the ones whose last recorded work has completed are dropped
    if (ix->uses.size() >= 64 && !ix->uses.count(st)) {
        for (auto it = ix->uses.begin(); it != ix->uses.end();) {
            if (hipEventQuery(it->second) == hipSuccess) {
                (void)hipEventDestroy(it->second);
                it = ix->uses.erase(it);
            } else {
                ++it;
            }
        }
    }
    hipEvent_t& e = ix->uses[st];
    if (!e) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(e, st));
    return VDB_OK;
}

// Every search queued on this index (any stream) and its own stream are done: what a resize,
// a rebuild of the candidate copy or a clear needs before touching the buffers searches read.
// Waits on this index's events only, not on the whole device (other indexes keep running).
int wait_idle(vdb_index* ix) {
    std::vector<hipEvent_t> evs;
    {
        std::lock_guard<std::mutex> g(ix->ws_mu);
        for (Workspace* w : ix->pool)
            if (w->used && w->done) evs.push_back(w->done);
        for (auto& kv : ix->uses) evs.push_back(kv.second);
    }
    for (hipEvent_t e : evs) HIP_TRY(hipEventSynchronize(e));
    HIP_TRY(hipStreamSynchronize(ix->stream));
    return VDB_OK;
}

// Accumulate the timing events of a search whose host side returned without
// waiting for the device (device-gated fallback).
// Read the `n` oldest pending event sets of the ring (waiting for them if needed).
int flush_timing(vdb_index* ix, Workspace* w, int n = Workspace::kTRing) {
    while (w->t_pending > 0 && n-- > 0) {
        hipEvent_t* ev = w->tring[(w->t_head - w->t_pending + Workspace::kTRing) % Workspace::kTRing];
        HIP_TRY(hipEventSynchronize(ev[2]));
        float ms_scan = 0.f, ms_pipe = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms_scan, ev[0], ev[1]));
        HIP_TRY(hipEventElapsedTime(&ms_pipe, ev[3], ev[2]));
        ix->scan_ns += (int64_t)(ms_scan * 1e6);
        ix->pipe_ns += (int64_t)(ms_pipe * 1e6);
        ix->n_timed++;
        w->t_pending--;
    }
    return VDB_OK;
}

int flush_all_timing(vdb_index* ix) {
    std::lock_guard<std::mutex> g(ix->ws_mu);
    for (Workspace* w : ix->pool)
        if (!w->busy) {
            const int rc = flush_timing(ix, w);
            if (rc) return rc;
        }
    return VDB_OK;
}

// Make the workspace at least `bytes` large and stream-ordered after its last use.
int ws_reserve(Workspace* w, size_t bytes, hipStream_t st) {
    if (w->used && w->done) HIP_TRY(hipStreamWaitEvent(st, w->done, 0));
    if (!w->host_flag) HIP_TRY(hipHostMalloc(&w->host_flag, 64 * sizeof(int), hipHostMallocDefault));
    if (bytes > w->dev_bytes) {
        if (w->dev) {
            HIP_TRY(hipStreamSynchronize(st));
            (void)hipFree(w->dev);
            w->dev = nullptr;
        }
        size_t nb = std::max(bytes, w->dev_bytes * 2);
        HIP_TRY(hipMalloc(&w->dev, nb));
        w->dev_bytes = nb;
    }
    return VDB_OK;
}

// The pinned staging of a host-memory search (the previous host search on this workspace
// synchronised before returning, so nothing reads the old buffer).
int ws_host_io(Workspace* w, size_t bytes) {
    if (bytes > w->host_io_bytes) {
        const size_t nb = std::max(bytes, w->host_io_bytes * 2);
        if (w->host_io) (void)hipHostFree(w->host_io);
        w->host_io = nullptr;
        w->host_io_bytes = 0;
        HIP_TRY(hipHostMalloc(&w->host_io, nb, hipHostMallocDefault));
        w->host_io_bytes = nb;
    }
    return VDB_OK;
}

int ws_reserve_exact(Workspace* w, size_t bytes, hipStream_t st) {
    if (bytes > w->exact_bytes) {
        if (w->exact) {
            HIP_TRY(hipStreamSynchronize(st));
            (void)hipFree(w->exact);
            w->exact = nullptr;
        }
        HIP_TRY(hipMalloc(&w->exact, bytes));
        w->exact_bytes = bytes;
    }
    return VDB_OK;
}

bool all_finite(const float* p, int64_t n) {
    for (int64_t i = 0; i < n; ++i)
        if (!std::isfinite(p[i])) return false;
    return true;
}


// query slots of the device-gated exact scan (each loops over the flagged queries)
constexpr int kGateSlots = 4;

// Exact full scan for queries qlist[0..nq) (device list) -> writes outputs.
// Bytes of the exact path's lists for nq queries (device-gated form: one list per CU).
size_t exact_bytes(vdb_index* ix, int nq, int k, bool gated) {
    const int KE = std::max(32, next_pow2(k));
    const int64_t n_wg = std::min<int64_t>(std::max<int64_t>(1, ix->n_cu * (gated ? 1 : 2)),
                                           std::max<int64_t>(1, ix->count / 256));
    return (size_t)nq * n_wg * KE * (sizeof(double) + sizeof(uint32_t)) + (size_t)nq * KE * 12 + 4096 +
           (gated ? exact_scan_scratch_bytes(KE, (int)n_wg, std::min(nq, kGateSlots)) : 0);
}

// Exact scan of the queries qlist[0..nq) (or 0..nq).  Device-gated form (qcount_dev):
// the flagged count is read on the device, nq is the capacity, and nothing runs
// when no query was flagged.
int run_exact(vdb_index* ix, Workspace* w, const float* Qd, const double* qn64, const int* qlist_dev, int nq, int k,
              const uint32_t* mask_dev, float* out_s, int64_t* out_i, double* out_k, int64_t index_offset,
              const int64_t* row_ids, hipStream_t st, const int* qcount_dev = nullptr, const int* ovf_dev = nullptr,
              int* done_dev = nullptr, unsigned long long* host_totals = nullptr) {
    const int KE = std::max(32, next_pow2(k));
    const int64_t N = ix->count;
    const bool gated = qcount_dev != nullptr;
    // ~2 workgroups per CU of rows (gated: 1, since an empty gated launch still has to find free
    // CUs beside the next batch's scan), at least 64 rows per wave
    const int64_t wg_target = gated ? std::max<int64_t>(1, ix->n_cu) : 2 * ix->n_cu;
    int n_wg = (int)std::min<int64_t>(wg_target, std::max<int64_t>(1, N / 256));
    const int64_t rpw = (N + n_wg - 1) / n_wg;
    n_wg = (int)((N + rpw - 1) / rpw);
    const int n_lists = n_wg;
    const size_t list_elems = (size_t)nq * n_lists * KE;
    // the device-gated form keeps its top-k buffers in the workspace (no LDS, vdb_exact.hip)
    const size_t scr = gated && done_dev ? exact_scan_scratch_bytes(KE, n_wg, std::min(nq, kGateSlots)) : 0;
    const size_t bytes = list_elems * (sizeof(double) + sizeof(uint32_t)) + (size_t)nq * KE * 12 + 4096 + scr;
    int rc = ws_reserve_exact(w, bytes, st);
    if (rc) return rc;
    Carver c{w->exact};
    double* lk = c.take<double>(list_elems);
    uint32_t* li = c.take<uint32_t>(list_elems);
    double* mk = c.take<double>((size_t)nq * KE);
    uint32_t* mi = c.take<uint32_t>((size_t)nq * KE);
    char* gscr = scr ? c.take<char>(scr) : nullptr;
    if (gated && done_dev) {  // one launch: the last workgroup per query merges and writes (ExactTail)
        const ExactTail tail{done_dev, mk, mi, k, index_offset, out_s, out_i, out_k, row_ids, host_totals};
        HIP_TRY(launch_exact_scan(ix->metric, KE, Qd, qn64, qlist_dev, nq, ix->X, ix->G, ix->dim, ix->nrm64, mask_dev,
                                  N, n_wg, rpw, lk, li, st, qcount_dev, ovf_dev, ix->d_totals, &tail, kGateSlots,
                                  gscr));
        return VDB_OK;
    }
    HIP_TRY(launch_exact_scan(ix->metric, KE, Qd, qn64, qlist_dev, nq, ix->X, ix->G, ix->dim, ix->nrm64, mask_dev, N,
                              n_wg, rpw, lk, li, st, qcount_dev, ovf_dev, gated ? ix->d_totals : nullptr));
    HIP_TRY(launch_merge_f64_u32(KE, lk, li, n_lists, KE, (int64_t)n_lists * KE, KE, nq, mk, mi, st, qcount_dev));
    HIP_TRY(launch_finalize_u32(ix->metric, mk, mi, KE, nq, qlist_dev, k, index_offset, out_s, out_i, out_k, st,
                                qcount_dev, row_ids));
    return VDB_OK;
}

}  // namespace

extern "C" {

const char* vdb_last_error(void) { return g_last_error.c_str(); }

int32_t vdb_version(void) { return 1; }

int32_t vdb_device_count(int32_t* n) {
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    if (e != hipSuccess) c = 0;
    if (n) *n = c;
    return VDB_OK;
}

int32_t vdb_index_create(int32_t dim, int32_t metric, int32_t device, vdb_index** out) {
    if (!out) return set_error(VDB_ERR_INVALID, "out is NULL");
    *out = nullptr;
    if (dim <= 0 || dim > 65536) return set_error(VDB_ERR_INVALID, "dimension must be in [1, 65536], got %d", dim);
    if (metric != VDB_METRIC_COSINE && metric != VDB_METRIC_EUCLIDEAN)
        return set_error(VDB_ERR_UNSUPPORTED, "unsupported metric id %d (cosine=0, euclidean=1)", metric);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return set_error(VDB_ERR_NODEVICE, "no HIP device visible: the vdb core needs an MI355X (gfx950)");
    if (device < 0 || device >= ndev) return set_error(VDB_ERR_INVALID, "device %d out of range [0,%d)", device, ndev);
    HIP_TRY(hipSetDevice(device));
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return set_error(VDB_ERR_NODEVICE, "device %d is %s; this build targets gfx950 only", device,
                         prop.gcnArchName);
    vdb_index* ix = new vdb_index();
    ix->dim = dim;
    ix->metric = metric;
    ix->device = device;
    ix->Dp = (int)round_up(dim, 64);  // G = Dp/8 is a multiple of the scan prefetch depth
    ix->G = ix->Dp / GROUP_DIMS;
    ix->n_cu = prop.multiProcessorCount;
    if (const char* q4 = std::getenv("VDB_SCAN_Q4")) ix->scan_q4 = std::min(1, std::max(-1, std::atoi(q4)));
    if (const char* a8 = std::getenv("VDB_AUTO_I8")) ix->auto_i8 = std::atoi(a8) != 0;
    hipError_t e = hipStreamCreateWithFlags(&ix->stream, hipStreamNonBlocking);
    // d_xmax: [0, 32) the residual maxima, [32, 36) the non-finite count, [64, 96) and
    // [128, 192) an add's snapshot of the maxima and of d_i8 (restored when the add is rejected)
    if (e == hipSuccess) e = hipMalloc(&ix->d_xmax, 192);
    if (e == hipSuccess) e = zero_now(ix->d_xmax, 192, ix->stream);
    if (e == hipSuccess) e = hipMalloc(&ix->d_i8, 64);
    if (e == hipSuccess) e = zero_now(ix->d_i8, 64, ix->stream);
    if (e == hipSuccess) e = hipMalloc(&ix->d_csum, (size_t)2 * ix->Dp * sizeof(uint32_t));
    if (e == hipSuccess) e = zero_now(ix->d_csum, (size_t)2 * ix->Dp * sizeof(uint32_t), ix->stream);
    if (e != hipSuccess) {
        delete ix;
        return set_error(VDB_ERR_HIP, "index setup failed: %s", hipGetErrorString(e));
    }
    ix->d_nonfinite = reinterpret_cast<int*>(reinterpret_cast<char*>(ix->d_xmax) + 32);
    {
        std::lock_guard<std::mutex> rg(g_reg_mu);
        g_indices.insert(ix);
    }
    *out = ix;
    return VDB_OK;
}

int32_t vdb_index_destroy(vdb_index* ix) {
    if (!ix) return VDB_OK;
    {
        std::lock_guard<std::mutex> rg(g_reg_mu);
        g_indices.erase(ix);
    }
    (void)hipSetDevice(ix->device);
    (void)wait_idle(ix);
    for (Workspace* w : ix->pool) {
        free_workspace_memory(w);
        if (w->done) (void)hipEventDestroy(w->done);
        if (w->own) (void)hipStreamDestroy(w->own);
        for (int r = 0; r < Workspace::kTRing; ++r)
            for (int e = 0; e < 4; ++e)
                if (w->tring[r][e]) (void)hipEventDestroy(w->tring[r][e]);
        delete w;
    }
    if (ix->X) (void)hipFree(ix->X);
    if (ix->Xs) (void)hipFree(ix->Xs);
    if (ix->Xq) (void)hipFree(ix->Xq);
    if (ix->Xh) (void)hipFree(ix->Xh);
    if (ix->nrm64) (void)hipFree(ix->nrm64);
    if (ix->inv32) (void)hipFree(ix->inv32);
    if (ix->sq32) (void)hipFree(ix->sq32);
    if (ix->rinit32) (void)hipFree(ix->rinit32);
    if (ix->d_xmax) (void)hipFree(ix->d_xmax);
    if (ix->d_dir) (void)hipFree(ix->d_dir);
    if (ix->d_mu) (void)hipFree(ix->d_mu);
    if (ix->d_i8) (void)hipFree(ix->d_i8);
    if (ix->d_csum) (void)hipFree(ix->d_csum);
    if (ix->d_totals) (void)hipFree(ix->d_totals);
    if (ix->h_totals) (void)hipHostFree(ix->h_totals);
    for (auto& kv : ix->uses) (void)hipEventDestroy(kv.second);
    if (ix->stream) (void)hipStreamDestroy(ix->stream);
    delete ix;
    return VDB_OK;
}

int32_t vdb_index_reserve(vdb_index* ix, int64_t rows) {
    if (!ix) return set_error(VDB_ERR_INVALID, "index is NULL");
    if (rows < 0) return set_error(VDB_ERR_INVALID, "rows must be >= 0");
    HIP_TRY(hipSetDevice(ix->device));
    std::unique_lock<std::shared_mutex> g(ix->mu);
    return ensure_capacity(ix, rows);
}

int32_t vdb_index_set_param(vdb_index* ix, const char* name, int64_t value) {
    if (!ix || !name) return set_error(VDB_ERR_INVALID, "NULL argument");
    std::string n(name);
    if (n == "precision") {
        if (value != VDB_PREC_FP32 && value != VDB_PREC_BF16X3 && value != VDB_PREC_BF16 && value != VDB_PREC_AUTO &&
            value != VDB_PREC_I8 && value != VDB_PREC_I8X3 && value != VDB_PREC_I8Q)
            return set_error(VDB_ERR_INVALID,
                             "precision must be %d (fp32), %d (bf16x3), %d (bf16), %d (auto), %d (i8), %d (i8x3) or "
                             "%d (i8q), got %lld",
                             VDB_PREC_FP32, VDB_PREC_BF16X3, VDB_PREC_BF16, VDB_PREC_AUTO, VDB_PREC_I8, VDB_PREC_I8X3,
                             VDB_PREC_I8Q, (long long)value);
        HIP_TRY(hipSetDevice(ix->device));
        std::unique_lock<std::shared_mutex> g(ix->mu);
        if (value == ix->precision) return VDB_OK;
        const int wr = wait_idle(ix);  // queued searches read the candidate copy
        if (wr) return wr;
        // rebuild a copy the new setting reads that the old one did not keep up to date
        const bool xs = xs_kind(value) != kXsNone && xs_kind(value) != xs_kind(ix->precision);
        const bool xq = needs_i8(value, ix->auto_i8) && !needs_i8(ix->precision, ix->auto_i8);
        if (xq) {
            const int xr = ensure_xq(ix);
            if (xr) return xr;
        }
        ix->precision = value;
        bool built = false;
        if (!ix->Xs && xs_eager(ix)) {  // a setting that reads it on every search: allocated + built now
            const int xr = ensure_xs(ix);
            if (xr) return xr;
            built = true;
        }
        if (((xs && !built) || xq) && ix->X && ix->count > 0) {
            HIP_TRY(build_candidate_rows(ix, 0, ix->count, ix->stream, xs && !built, xq));
            HIP_TRY(read_i8_stats(ix, ix->stream));
        }
    } else if (n == "auto_i8q") {
        ix->auto_i8q = value != 0;
    } else if (n == "auto_int8") {  // VDB_PREC_AUTO's candidate copy: 1 int8, 0 split-bf16
        HIP_TRY(hipSetDevice(ix->device));
        std::unique_lock<std::shared_mutex> g(ix->mu);
        const bool v = value != 0;
        if (v == ix->auto_i8) return VDB_OK;
        const int wr = wait_idle(ix);
        if (wr) return wr;
        const bool xq = needs_i8(ix->precision, v) && !needs_i8(ix->precision, ix->auto_i8);
        if (xq) {
            const int xr = ensure_xq(ix);
            if (xr) return xr;
        }
        ix->auto_i8 = v;
        if (!ix->Xs && xs_eager(ix)) {  // AUTO on the split copy alone: reads it on every search
            const int xr = ensure_xs(ix);
            if (xr) return xr;
        }
        if (xq && ix->X && ix->count > 0) {
            HIP_TRY(build_candidate_rows(ix, 0, ix->count, ix->stream, false, true));
            HIP_TRY(read_i8_stats(ix, ix->stream));
        }
    } else if (n == "margin") {
        ix->margin = value;
    } else if (n == "force_exact") {
        ix->force_exact = value != 0;
    } else if (n == "n_wg") {
        ix->n_wg_override = value;
    } else if (n == "scan_sync") {
        if (value < 0 || value > 2) return set_error(VDB_ERR_INVALID, "scan_sync must be 0, 1 or 2");
        ix->scan_sync = value;
    } else if (n == "scan_variant") {
        if (value < 0 || value > 2) return set_error(VDB_ERR_INVALID, "scan_variant must be 0, 1 or 2");
        ix->scan_variant = value;
    } else if (n == "scan_variant_bf16x3") {
        if (value != 0) return set_error(VDB_ERR_INVALID, "the split-bf16 pass has one variant (0)");
        ix->scan_variant_b3 = value;
    } else if (n == "graph_fill") {
        if (value < 0 || value > 1) return set_error(VDB_ERR_INVALID, "graph_fill must be 0 or 1");
        ix->graph_fill = value;
    } else if (n == "pilot_tiles") {
        if (value < -1 || value > 32768) return set_error(VDB_ERR_INVALID, "pilot_tiles must be in [-1, 32768]");
        ix->pilot_tiles = value;
    } else if (n == "timing") {
        ix->timing = value != 0;
    } else if (n == "no_fallback") {
        ix->no_fallback = value != 0;
    } else if (n == "finish_small") {
        if (value < -1 || value > 1) return set_error(VDB_ERR_INVALID, "finish_small must be -1, 0 or 1");
        ix->finish_small = value;
    } else if (n == "finish_split") {
        if (value < 1 || value > 8) return set_error(VDB_ERR_INVALID, "finish_split must be in [1, 8]");
        ix->finish_split = value;
    } else if (n == "scan_qlds") {
        if (value < -1 || value > 2) return set_error(VDB_ERR_INVALID, "scan_qlds must be -1 (auto), 0, 1 or 2");
        ix->scan_qlds = value;
    } else if (n == "scan_wide") {
        if (value < -1 || value > 1) return set_error(VDB_ERR_INVALID, "scan_wide must be -1, 0 or 1");
        ix->scan_wide = value;
    } else if (n == "scan_q4") {
        if (value < -1 || value > 1) return set_error(VDB_ERR_INVALID, "scan_q4 must be -1, 0 or 1");
        ix->scan_q4 = value;
    } else if (n == "dir_bound") {
        ix->no_dir_bound = value == 0;
    } else if (n == "i8_refine") {
        if (value < -1 || value > 1) return set_error(VDB_ERR_INVALID, "i8_refine must be -1, 0 or 1");
        ix->i8_refine = (int)value;
    } else if (n == "i8_narrow") {
        if (value < -1 || value > 0) return set_error(VDB_ERR_INVALID, "i8_narrow must be -1 or 0");
        ix->i8_narrow = value;
    } else if (n == "device_repass") {
        if (value < -1 || value > 1) return set_error(VDB_ERR_INVALID, "device_repass must be -1, 0 or 1");
        ix->device_repass = value;
    } else if (n.rfind("debug_", 0) == 0 && !debug_knobs_enabled()) {
        // test-only knobs corrupt the index on purpose: only with VDB_DEBUG_KNOBS=1
        return set_error(VDB_ERR_INVALID, "'%s' is a test-only knob (set VDB_DEBUG_KNOBS=1)", name);
    } else if (n == "debug_sink_row8") {
        // TEST ONLY: both int8 planes of row `value` := -127 (the column sums untouched): a corpus
        // operand the int8 pass reads wrong that UNDER-scores the row (for queries with
        // non-negative components) -- the side the finish's approx-vs-exact check cannot see; the
        // pass's checksum flags it
        HIP_TRY(hipSetDevice(ix->device));
        std::unique_lock<std::shared_mutex> g(ix->mu);
        if (value < 0 || value >= ix->count || !ix->Xq)
            return set_error(VDB_ERR_INVALID, "debug_sink_row8: no int8 row %lld", (long long)value);
        const int wr = wait_idle(ix);
        if (wr) return wr;
        HIP_TRY(launch_sink_row8(ix->Xq, value, ix->G / 4, ix->stream));
        HIP_TRY(hipStreamSynchronize(ix->stream));
    } else if (n == "scan_checksum") {
        if (value < 0 || value > 2) return set_error(VDB_ERR_INVALID, "scan_checksum must be 0, 1 or 2");
        ix->scan_checksum = value;
    } else if (n == "debug_stale_rinit") {
        // TEST ONLY: plants a stale L2 start value, -|x|^2/2 := 0 for row `value` (the operand a
        // scan read before its load landed in VERDICT r3), so the consistency guard of the
        // finish can be seen to flag the query instead of certifying it
        if (value < 0) return set_error(VDB_ERR_INVALID, "debug_stale_rinit: row must be >= 0");
        HIP_TRY(hipSetDevice(ix->device));
        std::unique_lock<std::shared_mutex> g(ix->mu);
        if (value >= ix->count || !ix->rinit32) return set_error(VDB_ERR_INVALID, "debug_stale_rinit: no row %lld", (long long)value);
        const int wr = wait_idle(ix);
        if (wr) return wr;
        const float zero = 0.0f;
        HIP_TRY(hipMemcpyAsync(ix->rinit32 + value, &zero, sizeof(float), hipMemcpyHostToDevice, ix->stream));
        HIP_TRY(hipStreamSynchronize(ix->stream));
    } else if (n == "pilot_rank") {
        if (value < 0 || value > 256) return set_error(VDB_ERR_INVALID, "pilot_rank must be in [0, 256]");
        ix->pilot_rank_override = value;
    } else {
        return set_error(VDB_ERR_INVALID, "unknown parameter '%s'", name);
    }
    return VDB_OK;
}

int32_t vdb_index_get_stat(const vdb_index* cix, const char* name, int64_t* value) {
    if (!cix || !name || !value) return set_error(VDB_ERR_INVALID, "NULL argument");
    vdb_index* ix = const_cast<vdb_index*>(cix);  // pending device-side counts are folded in
    std::string n(name);
    unsigned long long dt[4] = {0, 0, 0, 0};
    if ((n == "fallback_queries" || n == "overflow_queries" || n == "repass_queries") && ix->d_totals) {
        HIP_TRY(hipSetDevice(ix->device));
        const int wr = wait_idle(ix);  // device-memory searches queued on caller streams
        if (wr) return wr;
        HIP_TRY(hipMemcpy(dt, ix->d_totals, sizeof(dt), hipMemcpyDeviceToHost));
    }
    if (n == "scan_ns" || n == "pipeline_ns" || n == "timed_searches") {
        HIP_TRY(hipSetDevice(ix->device));
        const int rc = flush_all_timing(ix);
        if (rc) return rc;
    }
    if (n == "searches") *value = ix->n_searches.load();
    else if (n == "queries") *value = ix->n_queries.load();
    else if (n == "fallback_queries") *value = ix->n_fallback.load() + (int64_t)dt[0];
    else if (n == "repass_queries") *value = ix->n_repass.load() + (int64_t)dt[3];  // + device re-passes
    else if (n == "searches_q4") *value = ix->n_q4.load();
    else if (n == "searches_wide") *value = ix->n_wide.load();
    else if (n == "auto_hold") *value = ix->auto_hold.load();
    else if (n == "auto_hold8") *value = ix->auto_hold8.load();
    else if (n == "overflow_queries") *value = ix->n_overflow.load() + (int64_t)dt[1];
    else if (n == "inconsistent_queries") *value = ix->n_incons.load();  // host-memory searches
    else if (n == "capacity") *value = ix->cap_rows;
    else if (n == "scan_ns") *value = ix->scan_ns.load();
    else if (n == "pipeline_ns") *value = ix->pipe_ns.load();
    else if (n == "timed_searches") *value = ix->n_timed.load();
    else if (n == "count") *value = ix->count;
    else if (n == "precision") *value = ix->precision;
    else if (n == "searches_fp32") *value = ix->n_by_prec[PREC_FP32].load();
    else if (n == "searches_bf16x3") *value = ix->n_by_prec[PREC_BF16X3].load();
    else if (n == "searches_bf16") *value = ix->n_by_prec[PREC_BF16].load();
    else if (n == "searches_i8") *value = ix->n_by_prec[PREC_I8].load();
    else if (n == "searches_i8x3") *value = ix->n_by_prec[PREC_I8X3].load();
    else if (n == "auto_int8") *value = ix->auto_i8 ? 1 : 0;
    else if (n == "auto_i8q") *value = ix->auto_i8q ? 1 : 0;
    else if (n == "i8q_off") *value = ix->i8q_off.load() ? 1 : 0;
    else if (n == "searches_i8q") *value = ix->n_by_prec[PREC_I8Q].load();
    else if (n == "i8_wide") *value = ix->i8_wide ? 1 : 0;
    else if (n == "device_bytes") {  // the row buffers actually allocated
        const int64_t xb = (int64_t)(ix->cap_rows / 32) * ix->G * BLOCK_FLOATS * 4;  // fp32 X: 4 B per element
        *value = xb + (xs_ptr(ix) ? xb : 0) + (ix->Xq ? xb / 2 : 0) + (ix->Xh ? xb / 4 : 0) + ix->cap_rows * 20;
    } else if (n == "split_copy") *value = xs_ptr(ix) ? 1 : 0;
    else if (n == "split_copy_builds") *value = ix->n_xs_builds.load();
    else return set_error(VDB_ERR_INVALID, "unknown stat '%s'", name);
    return VDB_OK;
}

// Rows [row0, row0 + n) were just packed: on the first add, fix the residual direction
// (normalised column sums of up to kDirRows of these rows; a host round trip, once per
// index); then the maximum of |dir . (y - bf16(y))| over these rows (d_xmax[3]).
constexpr int64_t kDirRows = 65536;

// On the first add also the int8 copy's centring row mu (the mean of the same rows) and its
// quantisation step sx = 1.25 max |y - mu| / 127 over them (vdb_scan8.hip): this runs before
// the candidate copy of the first rows is built.
static hipError_t setup_direction(vdb_index* ix, int64_t row0, int64_t n, hipStream_t st) {
    if (ix->dir_set) return hipSuccess;
    const float* inv = ix->metric == VDB_METRIC_COSINE ? ix->inv32 : nullptr;
    const int D = ix->dim;
    const int64_t m = std::min(n, kDirRows);
    hipError_t e = hipSuccess;
    if (!ix->d_dir) e = hipMalloc(&ix->d_dir, (size_t)ix->Dp * sizeof(float));
    if (e == hipSuccess && !ix->d_mu) e = hipMalloc(&ix->d_mu, (size_t)ix->Dp * sizeof(float));
    double* sums = nullptr;
    if (e == hipSuccess) e = hipMalloc(&sums, (size_t)D * sizeof(double));
    if (e == hipSuccess) e = hipMemsetAsync(sums, 0, (size_t)D * sizeof(double), st);
    if (e == hipSuccess) e = launch_dir_sum(ix->X, inv, row0, m, D, ix->G, sums, st);
    std::vector<double> h(D);
    if (e == hipSuccess) e = hipMemcpyAsync(h.data(), sums, (size_t)D * sizeof(double), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (sums) (void)hipFree(sums);
    if (e != hipSuccess) return e;
    double nn = 0.0;
    for (double v : h) nn += v * v;
    std::vector<float> dir(ix->Dp, 0.0f), mu(ix->Dp, 0.0f);
    if (nn > 0.0 && std::isfinite(nn))
        for (int d = 0; d < D; ++d) dir[d] = (float)(h[d] / std::sqrt(nn));
    for (int d = 0; d < D; ++d) mu[d] = (float)(h[d] / (double)std::max<int64_t>(m, 1));
    e = hipMemcpyAsync(ix->d_dir, dir.data(), (size_t)ix->Dp * sizeof(float), hipMemcpyHostToDevice, st);
    if (e == hipSuccess)
        e = hipMemcpyAsync(ix->d_mu, mu.data(), (size_t)ix->Dp * sizeof(float), hipMemcpyHostToDevice, st);
    uint32_t zb = 0;
    uint32_t* dz = reinterpret_cast<uint32_t*>(ix->d_i8 + 6);
    if (e == hipSuccess) e = hipMemsetAsync(dz, 0, sizeof(uint32_t), st);
    if (e == hipSuccess) e = launch_zmax(ix->X, inv, ix->d_mu, row0, m, D, ix->G, dz, st);
    if (e == hipSuccess) e = hipMemcpyAsync(&zb, dz, sizeof(zb), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);  // dir / mu are stack buffers
    if (e != hipSuccess) return e;
    float zmax = 0.0f;
    std::memcpy(&zmax, &zb, sizeof(zmax));
    ix->sx = zmax > 0.0f && std::isfinite(zmax) ? 1.25f * zmax / 127.0f : 1.0f;
    ix->dir_rows = m;
    ix->dir_set = true;
    return hipSuccess;
}

static hipError_t residual_direction(vdb_index* ix, int64_t row0, int64_t n, hipStream_t st) {
    const float* inv = ix->metric == VDB_METRIC_COSINE ? ix->inv32 : nullptr;
    return launch_resid_dir(ix->X, inv, row0, n, ix->dim, ix->G, ix->d_dir, ix->d_xmax + 3, st);
}

int32_t vdb_index_add(vdb_index* ix, const float* vectors, int64_t n, int32_t mem, void* stream) {
    if (!ix) return set_error(VDB_ERR_INVALID, "index is NULL");
    if (n < 0) return set_error(VDB_ERR_INVALID, "n must be >= 0");
    if (n == 0) return VDB_OK;
    if (!vectors) return set_error(VDB_ERR_INVALID, "vectors is NULL");
    if (ix->count + n > (int64_t)0xFFFFFFFE) return set_error(VDB_ERR_INVALID, "index is limited to 2^32-2 rows");
    HIP_TRY(hipSetDevice(ix->device));
    std::unique_lock<std::shared_mutex> g(ix->mu);
    hipStream_t st = ix->stream;
    int rc = ensure_capacity(ix, ix->count + n);
    if (rc) return rc;
    // While the direction / centring row / int8 step still come from fewer than kDirRows rows,
    // this add may derive them again and rebuild the int8 copy of rows [0, count) in place
    // (below): device-memory searches still running on caller streams read those buffers
    // together with host-captured scalars (sx, i8st) -- wait for them first.  Past
    // that phase an add only writes rows >= count, which no queued search reads.
    if (ix->count > 0 && ix->dir_rows < kDirRows) {
        const int wr = wait_idle(ix);
        if (wr) return wr;
    }
    HIP_TRY(hipMemsetAsync(ix->d_nonfinite, 0, sizeof(int), st));
    // snapshot of the row statistics the kernels below raise over the new rows: a rejected add
    // puts them back (its rows must leave no trace in any statistic or column sum)
    char* bak = reinterpret_cast<char*>(ix->d_xmax);
    HIP_TRY(hipMemcpyAsync(bak + 64, ix->d_xmax, 32, hipMemcpyDeviceToDevice, st));
    HIP_TRY(hipMemcpyAsync(bak + 128, ix->d_i8, 64, hipMemcpyDeviceToDevice, st));
    if (mem == VDB_MEM_DEVICE) {
        // the rows may still be being written on the caller's stream (NULL = the null stream):
        // ingest (on the index's own stream) starts after that work
        hipEvent_t ready = nullptr;
        HIP_TRY(hipEventCreateWithFlags(&ready, hipEventDisableTiming));
        hipError_t e = hipEventRecord(ready, (hipStream_t)stream);
        if (e == hipSuccess) e = hipStreamWaitEvent(st, ready, 0);
        (void)hipEventDestroy(ready);
        HIP_TRY(e);
    }
    const int D = ix->dim;
    const int64_t chunk = std::max<int64_t>(1, (int64_t)(256ll << 20) / ((int64_t)D * 4));
    float* staging = nullptr;
    if (mem == VDB_MEM_HOST) HIP_TRY(hipMalloc(&staging, (size_t)std::min(chunk, n) * D * sizeof(float)));
    for (int64_t r = 0; r < n; r += chunk) {
        const int64_t m = std::min(chunk, n - r);
        const float* src = vectors + r * D;
        if (mem == VDB_MEM_HOST) {
            hipError_t e = hipMemcpyAsync(staging, src, (size_t)m * D * sizeof(float), hipMemcpyHostToDevice, st);
            if (e == hipSuccess)
                e = launch_pack_rows(staging, m, D, ix->G, ix->X, ix->count + r, ix->nrm64, ix->inv32, ix->sq32,
                                     ix->rinit32, ix->metric == VDB_METRIC_COSINE, ix->d_xmax, ix->d_nonfinite, st);
            if (e == hipSuccess) e = setup_direction(ix, ix->count + r, m, st);
            if (e == hipSuccess) e = build_candidate_rows(ix, ix->count + r, m, st);
            if (e == hipSuccess) e = residual_direction(ix, ix->count + r, m, st);
            if (e == hipSuccess) e = hipStreamSynchronize(st);  // staging reuse
            if (e != hipSuccess) {
                (void)hipFree(staging);
                return set_error(VDB_ERR_HIP, "ingest failed: %s", hipGetErrorString(e));
            }
        } else {
            HIP_TRY(launch_pack_rows(src, m, D, ix->G, ix->X, ix->count + r, ix->nrm64, ix->inv32, ix->sq32,
                                     ix->rinit32, ix->metric == VDB_METRIC_COSINE, ix->d_xmax, ix->d_nonfinite, st));
            HIP_TRY(setup_direction(ix, ix->count + r, m, st));
            HIP_TRY(build_candidate_rows(ix, ix->count + r, m, st));
            HIP_TRY(residual_direction(ix, ix->count + r, m, st));
        }
    }
    if (staging) (void)hipFree(staging);  // ingest runs on the index's own stream (serialised with growth)
    int nonfinite = 0;
    unsigned long long xb[4] = {0, 0, 0, 0};
    HIP_TRY(hipMemcpyAsync(&nonfinite, ix->d_nonfinite, sizeof(int), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(xb, ix->d_xmax, sizeof(xb), hipMemcpyDeviceToHost, st));
    HIP_TRY(read_i8_stats(ix, st));
    if (nonfinite) {
        // rows past `count` are never read; the next add overwrites them.  A rejected first add
        // leaves no direction / centring row behind (they would hold its non-finite values).
        if (ix->count == 0) {
            ix->dir_set = false;
            ix->dir_rows = 0;
            HIP_TRY(hipMemsetAsync(ix->d_xmax, 0, 32, st));
            HIP_TRY(hipMemsetAsync(ix->d_i8, 0, 64, st));
            HIP_TRY(hipStreamSynchronize(st));
            std::memset(ix->i8st, 0, sizeof(ix->i8st));
        } else {
            // the rejected rows' statistics and column sums came in with them: the maxima and the
            // int8 statistics go back to the snapshot, the column sums are rebuilt over [0, count)
            HIP_TRY(hipMemcpyAsync(ix->d_xmax, bak + 64, 32, hipMemcpyDeviceToDevice, st));
            HIP_TRY(hipMemcpyAsync(ix->d_i8, bak + 128, 64, hipMemcpyDeviceToDevice, st));
            if (ix->Xq && needs_i8(ix->precision, ix->auto_i8)) {
                HIP_TRY(hipMemsetAsync(ix->d_csum, 0, (size_t)2 * ix->Dp * sizeof(uint32_t), st));
                HIP_TRY(launch_colsum8(ix->Xq, 0, ix->count, ix->G / 4, ix->d_csum, st));
            }
            HIP_TRY(read_i8_stats(ix, st));  // (synchronises)
        }
        return set_error(VDB_ERR_NONFINITE, "%d row(s) contain NaN or Inf; nothing was added", nonfinite);
    }
    // Direction, centring row and quantisation step from a few rows (a store filled one REST add
    // at a time) would stay poor for good: while they came from fewer than kDirRows rows, they
    // are derived again from all rows each time the index doubles, and the int8 copy and the
    // residual maxima along dir are rebuilt (O(kDirRows) work in total).
    if (ix->dir_rows < kDirRows && ix->count + n >= 2 * ix->dir_rows) {
        const int64_t all = ix->count + n;
        ix->dir_set = false;
        HIP_TRY(hipMemsetAsync(ix->d_xmax + 3, 0, 8, st));
        HIP_TRY(hipMemsetAsync(ix->d_i8, 0, 64, st));
        HIP_TRY(setup_direction(ix, 0, all, st));
        if (needs_i8(ix->precision, ix->auto_i8)) HIP_TRY(build_candidate_rows(ix, 0, all, st, false, true));
        HIP_TRY(residual_direction(ix, 0, all, st));
        HIP_TRY(hipMemcpyAsync(xb, ix->d_xmax, sizeof(xb), hipMemcpyDeviceToHost, st));
        HIP_TRY(read_i8_stats(ix, st));
    }
    double xm[4];
    std::memcpy(xm, xb, sizeof(xm));
    ix->xmax = xm[0];
    ix->xres_rel = xm[1];
    ix->xres_abs = xm[2];
    ix->xres_dir = xm[3];
    ix->count += n;
    ix->auto_hold = 0;  // new rows: VDB_PREC_AUTO tries the one-plane passes again
    ix->auto_fails = 0;
    ix->auto_hold8 = 0;
    ix->auto_fails8 = 0;
    // device-memory failures already landed belong to the old rows: they start no hold
    if (ix->h_totals) ix->auto_seen = ix->h_totals[0];
    return VDB_OK;
}

int32_t vdb_index_count(const vdb_index* ix, int64_t* n) {
    if (!ix || !n) return set_error(VDB_ERR_INVALID, "NULL argument");
    *n = ix->count;
    return VDB_OK;
}

int32_t vdb_index_clear(vdb_index* ix) {
    if (!ix) return set_error(VDB_ERR_INVALID, "index is NULL");
    HIP_TRY(hipSetDevice(ix->device));
    std::unique_lock<std::shared_mutex> g(ix->mu);
    {
        const int wr = wait_idle(ix);
        if (wr) return wr;
    }
    if (ix->X) {
        HIP_TRY(hipMemsetAsync(ix->X, 0, (size_t)(ix->cap_rows / 32) * ix->G * BLOCK_FLOATS * sizeof(float),
                               ix->stream));
        HIP_TRY(hipMemsetAsync(ix->nrm64, 0, ix->cap_rows * sizeof(double), ix->stream));
        if (ix->Xs)
            HIP_TRY(hipMemsetAsync(ix->Xs, 0, (size_t)(ix->cap_rows / 32) * ix->G * BLOCK_FLOATS * sizeof(float),
                                   ix->stream));
        if (ix->Xq)
            HIP_TRY(hipMemsetAsync(ix->Xq, 0, (size_t)(ix->cap_rows / 32) * ix->G * BLOCK_FLOATS * sizeof(float) / 2,
                                   ix->stream));
    }
    HIP_TRY(hipMemsetAsync(ix->d_xmax, 0, 64, ix->stream));
    HIP_TRY(hipMemsetAsync(ix->d_i8, 0, 64, ix->stream));
    HIP_TRY(hipMemsetAsync(ix->d_csum, 0, (size_t)2 * ix->Dp * sizeof(uint32_t), ix->stream));
    HIP_TRY(hipStreamSynchronize(ix->stream));
    std::memset(ix->i8st, 0, sizeof(ix->i8st));
    ix->count = 0;
    ix->auto_hold = 0;
    ix->auto_fails = 0;
    ix->auto_hold8 = 0;
    ix->auto_fails8 = 0;
    ix->xmax = 0.0;
    ix->xres_rel = ix->xres_abs = 0.0;
    ix->dir_set = false;  // the next add picks a new direction (xres_dir's bits were cleared above)
    ix->dir_rows = 0;
    ix->xres_dir = 0.0;
    return VDB_OK;
}

int32_t vdb_index_get_vectors(vdb_index* ix, int64_t start, int64_t n, float* out_host) {
    if (!ix || (!out_host && n > 0)) return set_error(VDB_ERR_INVALID, "NULL argument");
    if (start < 0 || n < 0 || start + n > ix->count)
        return set_error(VDB_ERR_INVALID, "rows [%lld, %lld) out of range [0, %lld)", (long long)start,
                         (long long)(start + n), (long long)ix->count);
    if (n == 0) return VDB_OK;
    HIP_TRY(hipSetDevice(ix->device));
    std::shared_lock<std::shared_mutex> g(ix->mu);
    const int D = ix->dim;
    const int64_t chunk = std::max<int64_t>(1, (int64_t)(256ll << 20) / ((int64_t)D * 4));
    float* tmp = nullptr;
    HIP_TRY(hipMalloc(&tmp, (size_t)std::min(chunk, n) * D * sizeof(float)));
    for (int64_t r = 0; r < n; r += chunk) {
        const int64_t m = std::min(chunk, n - r);
        hipError_t e = launch_unpack_rows(ix->X, ix->G, D, start + r, m, tmp, ix->stream);
        if (e == hipSuccess)
            e = hipMemcpyAsync(out_host + r * D, tmp, (size_t)m * D * sizeof(float), hipMemcpyDeviceToHost, ix->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(ix->stream);
        if (e != hipSuccess) {
            (void)hipFree(tmp);
            return set_error(VDB_ERR_HIP, "export failed: %s", hipGetErrorString(e));
        }
    }
    (void)hipFree(tmp);
    return VDB_OK;
}

// vdb_index_search with an optional global id per row (row_ids, device memory, read by
// the result write-out): a shard of a multi-device set holds pieces of the global
// insertion order (vdb_shards_*).
// search_impl's answer when VDB_PREC_AUTO's bf16 pass left too many queries uncertified in a
// host-memory search: nothing was written, the caller runs the search again in bf16x3 (two
// candidate passes cost far less than the exact scan of most of the batch)
constexpr int32_t kRetryBf16x3 = 1 << 20;
// A host-memory bf16 search re-passes its uncertified queries in bf16x3 (gathered into one
// device-memory sub-search) when they are at most 1/8 of the batch and at most this many.
constexpr int kRepassMax = 64;
// Device-memory searches (device_repass): up to this many uncertified queries of a batch are
// gathered into a gated BF16X3 sub-search on the device (more go to the exact path); auto arms
// the re-pass for kRepassArm searches after a device fallback was seen.
constexpr int kRepassDev = 16;
constexpr int kRepassArm = 256;
// auto's I8 pass: KP = 128 up to this many rows (i8_narrow)
constexpr int64_t kI8NarrowRows = 512 * 1024;
constexpr int64_t kI8NarrowRowsShort = 4 * 1024 * 1024;  // rows of <= 128 dims
// the wide int8 pass under scan_wide auto: from this many rows (smaller indexes: the 64-query shape)
constexpr int64_t kWideMinRows = 65536;
// ... and, for batches of <= 256 (a 64-query block's stage tiles split over 2..8 waves), up to this
// many rows: the c6 shard of an 8-way run (1.25M x 128, B = 64) 1.03 -> 1.25 M QPS per rank, scan
// 60 -> 40 us; at 10M rows the scan is faster (0.218 -> 0.206 ms) but the three-stream step slower
// (0.235 -> 0.245: its 134 KiB of LDS leave no room for the other streams' side kernels),
// profiles/r06_c6w2
constexpr int64_t kWideSplitMaxRows = 2500000;
// the finish holds every segment's entries: at most FIN_CAP (16 K) / W8_CH segments
constexpr int FIN_SEG_MAX = 512;
// i8_refine auto: the finish refines I8 candidates' scores for padded rows of this many dims or more
constexpr int64_t kRefineMinDp = 512;
// VDB_PREC_AUTO uses the bf16 pass up to this k (its KP = next_pow2(k + 112) stays 128)
constexpr int kAutoBf16MaxK = 16;

// VDB_PREC_AUTO bookkeeping (vdb_index::auto_hold): a bf16 failure too large for a re-pass
// starts a hold of bf16x3 searches, doubling per failed probe (16 .. 2048).
void auto_fail(vdb_index* ix) {
    const int f = std::min(8, ix->auto_fails.load() + 1);
    ix->auto_fails = f;
    ix->auto_ok = 0;
    ix->auto_hold = 16 << (f - 1);
}

// The precision class of the next auto search: bf16x3 while a hold lasts.
bool auto_take_hold(vdb_index* ix) {
    int h = ix->auto_hold.load();
    while (h > 0)
        if (ix->auto_hold.compare_exchange_weak(h, h - 1)) return true;
    if (++ix->auto_ok >= 64) ix->auto_fails = 0;  // probes have been certifying for a while
    return false;
}

// The same pair for the I8 -> BF16 hold (vdb_index::auto_hold8).
void auto_fail8(vdb_index* ix) {
    const int f = std::min(8, ix->auto_fails8.load() + 1);
    ix->auto_fails8 = f;
    ix->auto_ok8 = 0;
    ix->auto_hold8 = 16 << (f - 1);
}
bool auto_take_hold8(vdb_index* ix) {
    int h = ix->auto_hold8.load();
    while (h > 0)
        if (ix->auto_hold8.compare_exchange_weak(h, h - 1)) return true;
    if (++ix->auto_ok8 >= 64) ix->auto_fails8 = 0;
    return false;
}

static int32_t search_locked(vdb_index* ix, const float* queries, int32_t B, int32_t k, const uint32_t* row_mask,
                             int32_t mem, float* out_scores, int64_t* out_indices, double* out_keys,
                             int64_t index_offset, void* stream, const int64_t* row_ids, struct SearchOpts opt);

// The uncertified queries flag_list[0..n) (device) of a bf16 search, gathered into a
// device-memory bf16x3 sub-search on the same stream (its own certificate and gated exact
// fallback), whose result rows are scattered back into the batch's outputs.
static int repass_flagged(vdb_index* ix, const float* Qd, const int* flag_list, int n, int k, const uint32_t* md,
                          float* out_s, int64_t* out_i, double* out_k, int64_t index_offset, const int64_t* row_ids,
                          hipStream_t st);

struct SearchOpts {
    bool force_b3 = false;  // VDB_PREC_AUTO: this search runs bf16x3 (retry / re-pass)
    bool repass = false;    // an internal sub-search of a re-pass (no search / query counts)
    // device re-pass: the sub-search's query count lives on the device (B is its capacity);
    // its candidate pass and finish are gated on it, and it runs without a pilot
    const int* gate = nullptr;
    bool force_i8x3 = false;  // the re-pass in I8X3 (the int8 copy's two planes: half BF16X3's bytes)
};

static int32_t search_locked(vdb_index* ix, const float* queries, int32_t B, int32_t k, const uint32_t* row_mask,
                             int32_t mem, float* out_scores, int64_t* out_indices, double* out_keys,
                             int64_t index_offset, void* stream, const int64_t* row_ids, SearchOpts opt);

static int32_t search_impl(vdb_index* ix, const float* queries, int32_t B, int32_t k, const uint32_t* row_mask,
                           int32_t mem, float* out_scores, int64_t* out_indices, double* out_keys,
                           int64_t index_offset, void* stream, const int64_t* row_ids, bool force_b3 = false) {
    if (!ix) return set_error(VDB_ERR_INVALID, "index is NULL");
    if (B <= 0) return set_error(VDB_ERR_INVALID, "n_queries must be >= 1, got %d", B);
    if (k <= 0 || k > 1024) return set_error(VDB_ERR_INVALID, "k must be in [1, 1024], got %d", k);
    if (!queries || !out_scores || !out_indices) return set_error(VDB_ERR_INVALID, "NULL query/output pointer");
    if (mem != VDB_MEM_HOST && mem != VDB_MEM_DEVICE) return set_error(VDB_ERR_INVALID, "bad mem kind %d", mem);
    if (mem == VDB_MEM_HOST && !all_finite(queries, (int64_t)B * ix->dim))
        return set_error(VDB_ERR_NONFINITE, "query contains NaN or Inf");
    HIP_TRY(hipSetDevice(ix->device));
    std::shared_lock<std::shared_mutex> g(ix->mu);
    SearchOpts opt;
    opt.force_b3 = force_b3;
    return search_locked(ix, queries, B, k, row_mask, mem, out_scores, out_indices, out_keys, index_offset, stream,
                         row_ids, opt);
}

static int repass_flagged(vdb_index* ix, const float* Qd, const int* flag_list, int n, int k, const uint32_t* md,
                          float* out_s, int64_t* out_i, double* out_k, int64_t index_offset, const int64_t* row_ids,
                          hipStream_t st) {
    const int D = ix->dim;
    const size_t qb = round_up((int64_t)n * D * 4, 256), sb = round_up((int64_t)n * k * 4, 256),
                 lb = round_up((int64_t)n * k * 8, 256);
    char* buf = nullptr;
    HIP_TRY(hipMallocAsync((void**)&buf, qb + sb + 2 * lb, st));
    float* Qs = (float*)buf;
    float* ss = (float*)(buf + qb);
    int64_t* si = (int64_t*)(buf + qb + sb);
    double* sk = (double*)(buf + qb + sb + lb);
    hipError_t e = launch_gather_rows(Qd, D, flag_list, n, Qs, st);
    int rc = e == hipSuccess ? VDB_OK : set_error(VDB_ERR_HIP, "re-pass gather: %s", hipGetErrorString(e));
    if (rc == VDB_OK) {
        SearchOpts o;
        o.force_b3 = true;
        o.repass = true;
        rc = search_locked(ix, Qs, n, k, md, VDB_MEM_DEVICE, ss, si, sk, index_offset, st, row_ids, o);
    }
    if (rc == VDB_OK) {
        e = launch_scatter_results(flag_list, n, k, ss, si, sk, out_s, out_i, out_k, st);
        if (e != hipSuccess) rc = set_error(VDB_ERR_HIP, "re-pass scatter: %s", hipGetErrorString(e));
    }
    (void)hipFreeAsync(buf, st);
    ix->n_repass += n;
    return rc;
}

// The search itself (the caller holds the index's shared lock).
static int32_t search_locked(vdb_index* ix, const float* queries, int32_t B, int32_t k, const uint32_t* row_mask,
                             int32_t mem, float* out_scores, int64_t* out_indices, double* out_keys,
                             int64_t index_offset, void* stream, const int64_t* row_ids, SearchOpts opt) {
    const int D = ix->dim;
    // device memory: the caller's stream, NULL = the null stream (ordered with the caller's
    // default-stream work, e.g. PyTorch's); host memory: the caller's stream, or (NULL) the
    // stream of the workspace this search takes, so concurrent host searches overlap
    const bool own_stream = mem == VDB_MEM_HOST && !stream;
    hipStream_t st = own_stream ? nullptr : (hipStream_t)stream;
    const int64_t N = ix->count;
    if (!opt.repass) {
        ix->n_searches++;
        ix->n_queries += B;
    }

    // ---- sizes ----------------------------------------------------------------
    // candidates beyond k: the certificate needs a gap of 2 eps between the k-th and the
    // KP-th approximate score; bf16x3's bound grows with D (3D additions), so large D
    // gets a wider margin (1M x 1536 uniform: KP = 32 left ~1.5% of queries uncertified)
    const bool auto_prec = ix->precision == VDB_PREC_AUTO;
    if (auto_prec && ix->h_totals && !opt.repass) {  // fallbacks of earlier device-memory searches (lagged)
        const unsigned long long seen = ix->h_totals[0];
        const unsigned long long prev = ix->auto_seen.exchange(seen);
        if (seen > prev) {
            if (ix->last_i8q && seen - prev > (unsigned long long)std::max(1, ix->last_i8q_b.load() / 8))
                ix->i8q_off = true;
            if (ix->last_i8) {
                auto_fail8(ix);
                ix->i8_wide = true;
            } else {
                auto_fail(ix);
            }
            ix->repass_arm = kRepassArm;  // device_repass auto: re-pass on the device for a while
        }
    }
    const bool approx = N > 0 && !(ix->force_exact || k > kMaxApproxK);
    // AUTO takes bf16x3 directly where bf16's wider certificate needs KP = 256 (k > 16): that
    // pass runs 32-query blocks at twice the query-operand traffic and measured 3x slower than
    // bf16x3 (C4, k = 100: 13 vs 3.9 ms, profiles/r02s_ab/s4_c4_str2.json), and in device memory
    // its uncertified queries cost the exact path
    const bool auto_b16 = k <= kAutoBf16MaxK;
    // AUTO keeps both copies with auto_i8: the one-plane pass is I8 unless an I8 hold is on
    // (then BF16); the k > 16 pass is I8X3 unless an I8 hold is on (then BF16X3) -- with the
    // insertion by pass-bit masks I8X3 runs C4 / C3 / C2 at 2.89 / 1.42 / 0.28 ms against BF16X3's
    // 3.41 / 2.17 / 0.47 (profiles/r03_i8/c4prec, x3prec); holds, re-passes and retries stay
    // BF16X3 (per-element relative precision: no dependence on the rows' range)
    const bool x3_i8 = auto_prec && !opt.force_b3 && !auto_b16 && ix->auto_i8;
    const bool auto_x3 = auto_prec && (opt.force_b3 || !auto_b16 || (approx && auto_take_hold(ix)));
    const bool hold8 = auto_prec && ix->auto_i8 && approx && (x3_i8 || !auto_x3) && auto_take_hold8(ix);
    const bool auto_8 = auto_prec && !auto_x3 && ix->auto_i8 && !hold8;
    const bool auto_8x3 = x3_i8 && !hold8;
    // L2, 16 < k <= 100: the xh plane against the 16-bit query (two MFMAs per group, half the
    // corpus bytes of I8X3; its 8-bit corpus bound certifies at KP = 256)
    const bool auto_8q = auto_8x3 && ix->metric == 1 && k <= 100 && ix->auto_i8q && !ix->i8q_off;
    const bool force_8x3 = auto_prec && opt.force_i8x3 && ix->auto_i8 && ix->Xq;
    const int prec_req = !ix->X ? PREC_FP32
                         : force_8x3 ? PREC_I8X3
                         : ix->precision == VDB_PREC_BF16X3 ? PREC_BF16X3
                         : ix->precision == VDB_PREC_BF16 ? PREC_BF16
                         : ix->precision == VDB_PREC_I8X3 ? PREC_I8X3
                         : ix->precision == VDB_PREC_I8Q ? PREC_I8Q
                         : ix->precision == VDB_PREC_I8 ? PREC_I8
                         : auto_prec ? (auto_x3 ? (auto_8x3 ? (auto_8q ? PREC_I8Q : PREC_I8X3) : PREC_BF16X3)
                                                 : auto_8 ? PREC_I8 : PREC_BF16)
                                     : PREC_FP32;
    if (auto_prec && approx && (!auto_x3 || x3_i8)) {
        ix->last_i8 = auto_8 || auto_8x3;
        ix->last_i8q = prec_req == PREC_I8Q;
        ix->last_i8q_b = (int)B;
    }
    // (a device re-pass's gated sub-search is counted by the device: repass_queries)
    if (approx && !opt.gate) ix->n_by_prec[prec_req]++;
    // the "one plane" precisions (a wide certificate: KP = 128 for small k) and their re-pass
    const bool one_plane = prec_req == PREC_BF16 || prec_req == PREC_I8;

    int margin_def = std::max(16, k / 4);
    if ((prec_req == PREC_BF16X3 || prec_req == PREC_I8X3) && D >= 1024) margin_def = std::max(margin_def, 48);
    // bf16 (hi plane only): eps ~ the rows' bf16 residual (~1.5e-3 relative on uniform data),
    // ~30x bf16x3's: 1M x 768 uniform needs KP = 128 for k = 10 (KP = 64 left 26% of the
    // queries uncertified; KP = 128: none of 2560)
    if (one_plane) margin_def = std::max(16, std::min(std::max(112, k / 2), 256 - k));
    // I8 (the 8-bit query's wider bound): KP = 256.  1M x 768 uniform, B = 64: KP = 128 left one
    // query per batch uncertified; 256 none (profiles/r03_i8/c2_i8_kp*)
    // -- except auto on small indexes (i8_narrow): at <= 512 K rows KP = 128 (one rank of an 8-way
    // weak-scaled C2, 125 K rows x 512 queries: step 0.248 -> 0.207 ms, 0 fallbacks; 250 K: 0.181 ->
    // 0.157; KP = 64 failed thousands of queries, profiles/r04_ab/rank*), widened for good at the
    // first flagged query
    // Rows of <= 128 dims (C6's 10M x 128): 0 fallbacks at KP = 128 even at 10 M rows, faster up to
    // the 4-way shard (8-way 1.25 M x 512: 1.38 -> 1.56 M QPS; 4-way 2.5 M x 256: +4%) and slower
    // at 10 M (262 -> 248 K: the KP = 128 scan's 106 KiB of LDS leaves no room beside it for the
    // next batch's pilot, profiles/r04_ab/rank6m, c6m), hence 4 M
    const bool i8_narrow = auto_prec && ix->i8_narrow != 0 && !ix->i8_wide &&
                           (N <= kI8NarrowRows || (ix->Dp <= 128 && N <= kI8NarrowRowsShort));
    if (prec_req == PREC_I8) margin_def = std::max(16, (i8_narrow ? 128 : 256) - k);
    // I8Q (the 8-bit corpus's bound, as I8's): KP = 256
    if (prec_req == PREC_I8Q) margin_def = std::max(16, 256 - k);
    // a re-pass sub-search (host or device) takes KP = 128: its few queries are the ones whose
    // rows sit closer together than the one-plane pass could separate, so they need the wider
    // gap between the k-th and the KP-th candidate (C2 with 300 rows in a 3e-3 cosine band:
    // BF16X3 at KP = 32 left every such query to the exact scan)
    if (opt.repass) margin_def = std::max(margin_def, 128 - k);
    const int margin = ix->margin >= 0 ? (int)ix->margin : margin_def;
    int KP = std::max(32, next_pow2(k + margin));
    const bool exact_all = ix->force_exact || k > kMaxApproxK || KP > 256;
    if (KP > 256) KP = 256;
    const int prec = prec_req;
    const bool i8_pass = prec_is_i8(prec);  // vdb_scan8.hip
    const int Gs = prec == PREC_FP32 ? ix->G : i8_pass ? ix->G / 4 : ix->G / 2;  // scan groups (8, 32 or 16 dims)
    if (!i8_pass && !exact_all && N > 0 && !xs_ptr(ix)) {  // a split pass under AUTO + int8: the lazy copy
        const int xr = ensure_xs(ix);
        if (xr) return xr;
    }
    // fp32: vdb_scan.hip (variants); split-bf16 (bf16x3, bf16): vdb_scan2.hip
    const bool split_pass = prec == PREC_BF16X3 || prec == PREC_BF16;
    // The split pass's 128-query shape (vdb_scan2_kernel.h, q4): short rows whose query block
    // fits LDS at 128 queries (D <= 128), KP = 128, batches of >= 256: half the query blocks, so
    // each row range is re-read from L2 by half as many workgroups (C4: 8 -> 4 blocks)
    const bool q4 = split_pass && !exact_all && !opt.gate && KP == 128 && B >= 256 && Gs <= 8 &&
                    (ix->scan_q4 == 1 || (ix->scan_q4 < 0));
    // The wide int8 pass (vdb_scan8w.hip): rows of 4 groups (D <= 128) and batches of more than 256
    // (C4, and each rank of its row-sharded run): all queries of a 512-query block in one
    // workgroup, the corpus staged once through LDS; one workgroup per CU, tiles dealt round-robin
    const int64_t n_tiles_all = round_up(N, 32) / 32;
    // ... and its long-row form (vdb_scan8wl.hip): the I8 cosine pass for 16..48 groups and up to
    // 256 queries, all of them in one workgroup's registers, two waves per query tile for batches
    // of <= 128 with rows of <= 1024 dims.  Auto (profiles/r06_wl3, r06_rl4): every batch for rows
    // of <= 1024 dims (C2, B = 64: scan 0.142 -> 0.117 ms, 410 -> 432 K QPS; B = 2 / 32 / 128
    // faster too); at 1536 dims batches of <= 16 and > 96 (C3: 420 -> 494 K; B = 32 even, 64
    // slower).
    const bool wide_long = i8_pass && !exact_all && !opt.gate && scan8wl_ok(prec, ix->metric, Gs, B) && N > 0 &&
                           (ix->scan_wide == 1 ||
                            (ix->scan_wide < 0 && N >= kWideMinRows && (Gs <= 32 || B <= 16 || B > 96)));
    const bool wide8 = wide_long || (i8_pass && !exact_all && !opt.gate && scan8w_ok(Gs, B) && N > 0 &&
                                     (ix->scan_wide == 1 ||
                                      (ix->scan_wide < 0 && N >= kWideMinRows && (B > 256 || N <= kWideSplitMaxRows))));
    const int n_seg8 = !wide8 ? 0
                       : ix->n_wg_override > 0 ? (int)std::min<int64_t>(FIN_SEG_MAX, std::min<int64_t>(ix->n_wg_override, n_tiles_all))
                                               : (int)std::min<int64_t>(FIN_SEG_MAX, round_up(std::min<int64_t>(ix->n_cu, n_tiles_all), 8));
    // query rows per candidate-pass block: the int8 pass keeps 64 at KP = 256 (KW = 64 kept per
    // workgroup, vdb_scan8_kernel.h), the split pass 32 there
    const int QB = q4 ? 128 : i8_pass ? 64 : KP == 256 ? 32 : 64;
    const int QB_pilot = i8_pass ? 64 : KP == 256 ? 32 : 64;  // the pilot's own query blocks (instantiations)
    const int Bp = (int)round_up(B, 128);  // whole query super tiles (tiled layout)
    const int n_qblocks = (B + QB - 1) / QB;
    int variant = split_pass || i8_pass ? 0 : (int)ix->scan_variant;
    if (!split_pass && !i8_pass && !scan_variant_ok(prec, variant, Gs)) variant = 0;  // e.g. PX=8 needs Dp % 128 == 0
    const int64_t step_rows = i8_pass ? scan8_rows_per_step(prec, ix->metric)
                              : split_pass ? scan2_rows_per_step(q4) : scan_rows_per_step(prec, variant);
    const int64_t n_steps = std::max<int64_t>(1, round_up(N, step_rows) / step_rows);
    // one 4-wave workgroup per CU (1 wave per SIMD, all of its 512 registers):
    // measured faster than two per CU, whose top-k epilogues then overlap (profiles/)
    int target = ix->n_wg_override > 0 ? (int)ix->n_wg_override : std::max(1, ix->n_cu / n_qblocks);
    int spw = (int)std::max<int64_t>(1, (n_steps + target - 1) / target);
    int n_wg = (int)((n_steps + spw - 1) / spw);
    const int64_t mask_words = round_up(N, 32) / 32;
    // Step end of the scan (vdb_scan.hip): short steps (Dp <= 128: C4's 10M x 128 runs 8 split
    // groups per step, the epilogue ~half of it) gain from dropping the per-step workgroup barrier
    // (C4 scan 7.58 -> 6.22 ms); long steps lose (C2 0.57 -> 0.65 ms, C3 2.62 -> 2.90 ms), measured.
    // The int8 pass drops it at every length: a per-step barrier lines up the 4 waves' epilogues,
    // so the CU's stream idles through all of them at once; flag-gated, one wave's epilogue runs
    // under the others' loads (C2 366 -> 384 K QPS, C3 365 -> 401 K with its scan 0.576 -> 0.487 ms,
    // profiles/r04_ab/sync, same box).
    const int lockstep = ix->scan_sync == 0 ? (!i8_pass && ix->Dp > 128) : ix->scan_sync == 1;

    Workspace* w = acquire_ws(ix, st, own_stream);
    if (own_stream) {
        if (!w->own) {
            const hipError_t e = hipStreamCreateWithFlags(&w->own, hipStreamNonBlocking);
            if (e != hipSuccess) {
                std::lock_guard<std::mutex> lg(ix->ws_mu);
                w->busy = false;
                return set_error(VDB_ERR_HIP, "workspace stream: %s", hipGetErrorString(e));
            }
        }
        st = w->own;
    }
    struct Releaser {
        vdb_index* ix; Workspace* w; hipStream_t st;
        ~Releaser() { release_ws(ix, w, st); }
    } rel{ix, w, st};

    size_t bytes = 0;
    bytes += (size_t)B * D * 4 + 256;                       // Qraw (host mode)
    bytes += (size_t)(mask_words + 64) * 4 + 256;           // mask (host mode)
    bytes += (size_t)Bp * (ix->Dp + 16 * QG_EXTRA) * 4 + 256;  // Qt (tiled fp32 or split, duplicated groups)
    bytes += (size_t)Bp * 8 + 256;                          // qn64
    bytes += (size_t)Bp * 24 + 256;                         // qconst: the finish's per-query constants
    bytes += (size_t)Bp * KP * 8 + 512;                     // merged approx lists
    bytes += (size_t)B * k * 20 + 768;                      // outputs (host mode)
    bytes += (size_t)(B + 64) * 4 + 256;                    // flags
    bytes += (size_t)Bp * 4 + 256;                          // gated fallback: workgroups done per query
    // finish: optionally several workgroups per query share the exact rerank (tuning knob
    // "finish_split"; measured at C2 bf16, B = 64: split 4 took the finish 24.5 -> 45.9 us,
    // profiles/r02_ab, so the default is 1)
    const int fin_split = (int)ix->finish_split;
    bytes += fin_split > 1 ? (size_t)B * fin_split * (KP_MAX * 16 + 4) + 1024 : 0;
    bytes += (size_t)Bp * 4 + 256;                          // shared thresholds
    bytes += (size_t)Bp * (KP_MAX + PILOT_SLOTS) * 4 + 256;  // shared threshold slots + pilot slots
    bytes += (size_t)Bp * 12 + 1024;                          // int8 pass: qmax, lsl, qerr [Bp]; qscal
    // int8 L2 pass: the batch's integer accumulator start values (vdb_scan8.hip rstart8)
    const bool rs8_on = i8_pass && !exact_all && ix->metric == 1;
    bytes += rs8_on ? (size_t)round_up(N, 32) * 4 + 256 : 0;
    const bool i8_refine = prec == PREC_I8 && ix->Xh &&  // the finish's I8 refinement
                           (ix->i8_refine == 1 || (ix->i8_refine == -1 && ix->Dp >= kRefineMinDp));
    bytes += i8_refine ? (size_t)Bp * (ix->Dp + 1) * 4 + 512 : 0;  // query residuals [Bp][Dp] + qerr2 [Bp]
    const int R_rep = std::min(B, kRepassDev);                // device re-pass: gathered queries + results
    bytes += mem == VDB_MEM_DEVICE ? (size_t)R_rep * (D * 4 + (size_t)k * 20) + 1024 : 0;
    // the int8 pass's checksum: partial sums [2][n_wg8][Bp], expected values [Bp][2], L2 start sum
    const bool chk = i8_pass && !exact_all && ix->scan_checksum && ix->d_csum && N > 0;
    // the L sums of I8X3 too (scan_checksum 2): +5% on C4's scan over H alone (the xh plane, the
    // query's hi plane and the start values; an L operand moves a score by at most the slack lsl)
    const bool chk_l = chk && prec == PREC_I8X3 && ix->scan_checksum == 2;
    const int n_wg8 = wide8 ? n_seg8 : (n_wg + 7) / 8 * 8;
    bytes += wide8 ? (size_t)Bp * n_seg8 * 4 + 256 : 0;  // the wide pass's segment counts
    bytes += chk ? ((size_t)2 * n_wg8 * Bp + (size_t)2 * Bp + 64) * 4 + 768 : 0;
    const bool priv = !exact_all && !split_pass && !i8_pass && scan_priv(prec, variant, KP);
    // global per-query candidate lists: at most 512 entries per workgroup and query
    // (the largest LDS buffer of any variant; 4 x 64 for the wave-private one)
    const int64_t gl_cap = exact_all ? 0 : wide8 ? (int64_t)n_seg8 * W8_CH
                                              : (int64_t)((n_wg + 7) / 8 * 8) * 512;
    bytes += (size_t)B * gl_cap * 8 + (size_t)Bp * 4 + 768;
    // Pilot sample: 512 row tiles, more for large k (its bound then saves more insert work than
    // the sample costs: C4, k = 100, 512 -> 4096 tiles: 89.5 K -> 96.4 K QPS, profiles/r02_ab),
    // and at least 1/160 of the rows: the bound's global rank ~ r N / S sets how many entries
    // each workgroup inserts (C6, 10 M rows, int8 pass: 512 -> 2048 tiles, scan 0.329 -> 0.259 ms,
    // 200 K -> 250 K QPS; C2 / C3, 1 M rows: larger samples only add pilot time,
    // profiles/r03_i8/pilot).
    // Rows of 4 groups (D <= 128: the int8 pass's register-resident pilot, vdb_scan8.hip
    // pilot8_g4) take twice the k-based sample, up to 8192 tiles where the rows are many (at most
    // ~2.5% of them): C4 (k = 100) 4096 -> 8192, scan 2.32 -> 2.19 ms, 213 K -> 220 K QPS with
    // the pilot at ~50 -> ~90 us (profiles/r05_ab/ab20)
    const bool cheap_pilot = i8_pass && Gs == 4;
    const int64_t pilot_cap = cheap_pilot ? std::max<int64_t>(4096, std::min<int64_t>(8192, N / (32 * 40))) : 4096;
    const int64_t pilot_def = std::min<int64_t>(pilot_cap,
                                                std::max<int64_t>((cheap_pilot ? 1024 : 512) * std::max(1, k / 12),
                                                                  N / (32 * 160)));
    const int n_pilot = opt.gate ? 0  // a gated re-pass sub-search: no pilot (few queries; its launches stay light)
                                 : (int)std::min<int64_t>(ix->pilot_tiles >= 0 ? ix->pilot_tiles : pilot_def,
                                                          round_up(N, 32) / 32);
    // Rank of the pilot's bound among its sampled scores.  The KP-th best sample is a
    // guaranteed lower bound of the global KP-th best but sits at global rank ~KP N / S (C2:
    // ~2000), so the candidate pass inserts every score above that until its own buffers
    // tighten (the warm-up: 140 us of a 680 us C2 scan without a pilot, ~65 us with one).
    // Instead: the r-th best sample, r the smallest rank such that (1) the sample holds r of
    // the global top k with probability < 1e-6 (Poisson(k S / N) tail; rows in no particular
    // order), so T stays below a_k, and (2) T's expected global rank r N / S is >= 2 KP, so T
    // mostly stays below a_KP too and the certificate's cut max(a_KP, T) is what it would be
    // without a pilot (T near a_k failed bf16's wide certificate: C2 with 2048 tiles and rule
    // (1) alone; the KP-based Poisson rule instead cost C2 bf16 7%, profiles/r02_ab).  C2: r = 5,
    // T at rank ~300 instead of ~2000.  Exactness does not depend on it: rows dropped below the
    // bound are covered by the certificate (acut >= T), which sends a query whose bound was too
    // high to the exact path.
    int pilot_rank = KP;
    if (n_pilot > 0) {
        const double S = (double)std::min<int64_t>((int64_t)n_pilot * 32, N);
        const double x = (double)k * S / (double)N;
        double term = std::exp(-x), cdf = term;
        int r = 1;
        while (1.0 - cdf >= 1e-6 && r < KP) {
            term *= x / r;
            cdf += term;
            ++r;
        }
        const int r_min = (int)std::ceil(2.0 * KP * S / (double)N);
        pilot_rank = std::min(std::max(r, r_min), KP);
    }
    if (ix->pilot_rank_override > 0) pilot_rank = (int)std::min<int64_t>(ix->pilot_rank_override, KP);
    int rc = ws_reserve(w, bytes, st);
    if (rc) return rc;
    Carver c{w->dev};
    float* Qraw = c.take<float>((size_t)B * D);
    uint32_t* maskd = c.take<uint32_t>(mask_words + 64);
    float* Qt = c.take<float>((size_t)Bp * (ix->Dp + 16 * QG_EXTRA));
    double* qn64 = c.take<double>(Bp);
    double* qconst = c.take<double>((size_t)Bp * 3);
    // the finish's centring row and residual direction (the same conditions as its arguments below)
    const float* q_mu = i8_pass ? ix->d_mu : nullptr;
    const float* q_dir = (prec == PREC_BF16 || i8_pass) && ix->dir_set && !ix->no_dir_bound ? ix->d_dir : nullptr;
    float* os = c.take<float>((size_t)B * k);
    int64_t* oi = c.take<int64_t>((size_t)B * k);
    double* ok = c.take<double>((size_t)B * k);
    int* flags = c.take<int>(B + 64);
    int* done = c.take<int>(Bp);
    uint32_t* gthr = c.take<uint32_t>(Bp);
    uint32_t* gslots = c.take<uint32_t>((size_t)Bp * (KP_MAX + PILOT_SLOTS));
    uint32_t* pslots = gslots + (size_t)Bp * KP_MAX;
    float* gl_s = c.take<float>((size_t)B * gl_cap);
    uint32_t* gl_i = c.take<uint32_t>((size_t)B * gl_cap);
    uint32_t* gl_cnt = c.take<uint32_t>(Bp);
    double* fx_ek = fin_split > 1 ? c.take<double>((size_t)B * fin_split * KP_MAX) : nullptr;
    uint32_t* fx_ck = fin_split > 1 ? c.take<uint32_t>((size_t)B * fin_split * KP_MAX) : nullptr;
    uint32_t* fx_cr = fin_split > 1 ? c.take<uint32_t>((size_t)B * fin_split * KP_MAX) : nullptr;
    int* fx_n = fin_split > 1 ? c.take<int>((size_t)B * fin_split) : nullptr;
    float* q8max = c.take<float>(Bp);
    float* q8lsl = c.take<float>(Bp);
    float* q8err = c.take<float>(Bp);
    float* q8scal = c.take<float>(64);
    float* q8res = i8_refine ? c.take<float>((size_t)Bp * ix->Dp) : nullptr;
    float* q8err2 = i8_refine ? c.take<float>(Bp) : nullptr;
    uint32_t* chkp = chk ? c.take<uint32_t>((size_t)2 * n_wg8 * Bp) : nullptr;
    uint32_t* segc = wide8 ? c.take<uint32_t>((size_t)Bp * n_seg8) : nullptr;
    uint32_t* chkr = chk && ix->metric == 1 ? c.take<uint32_t>(64) : nullptr;
    int* rs8 = rs8_on ? c.take<int>((size_t)round_up(N, 32)) : nullptr;
    // (the pilot writes the checksum's expectations when it runs; else the finish computes them)
    uint32_t* chke = chk && n_pilot > 0 ? c.take<uint32_t>((size_t)2 * Bp) : nullptr;
    float* rep_q = mem == VDB_MEM_DEVICE ? c.take<float>((size_t)R_rep * D) : nullptr;
    float* rep_s = mem == VDB_MEM_DEVICE ? c.take<float>((size_t)R_rep * k) : nullptr;
    int64_t* rep_i = mem == VDB_MEM_DEVICE ? c.take<int64_t>((size_t)R_rep * k) : nullptr;
    double* rep_k = mem == VDB_MEM_DEVICE ? c.take<double>((size_t)R_rep * k) : nullptr;

    const float* Qd = queries;
    const uint32_t* md = row_mask;
    float* out_s = out_scores;
    int64_t* out_i = out_indices;
    double* out_k = out_keys;
    // host memory: the queries go up and the results come down through the workspace's pinned
    // staging (asynchronous copies; the results are read in the same synchronisation as the
    // certificate's flags, and copied out on the host when nothing was flagged)
    const size_t io_q = mem == VDB_MEM_HOST ? (size_t)B * D * 4 : 0;
    const size_t io_r = (size_t)B * k * (4 + 8 + (out_keys ? 8 : 0));
    bool staged = false;
    if (mem == VDB_MEM_HOST) {
        rc = ws_host_io(w, io_q + io_r);
        if (rc) return rc;
        std::memcpy(w->host_io, queries, io_q);
        HIP_TRY(hipMemcpyAsync(Qraw, w->host_io, io_q, hipMemcpyHostToDevice, st));
        Qd = Qraw;
        if (row_mask && N > 0) {
            HIP_TRY(hipMemcpyAsync(maskd, row_mask, (size_t)mask_words * 4, hipMemcpyHostToDevice, st));
            md = maskd;
        }
        out_s = os;
        out_i = oi;
        out_k = out_keys ? ok : nullptr;
    }

    if (N == 0) {
        // empty store: every slot "no result" (reference returns ([],[],[]), :117), keys -inf
        // like every other invalid entry, so an empty shard's lists rank last in a merge
        HIP_TRY(launch_empty_results((int64_t)B * k, out_s, out_i, out_k, st));
    } else {
        HIP_TRY(launch_prep_queries(Qd, B, Bp, D, ix->G, ix->metric, prec == PREC_FP32 ? Qt : nullptr,
                                    split_pass ? Qt : nullptr, qn64, flags, gthr, gslots, gl_cnt, done, st,
                                    i8_pass ? q8max : nullptr, q_mu, q_dir, qconst));
        if (i8_pass && !exact_all) {
            Int8Consts c8;
            c8.sx = ix->sx;
            c8.zmax_h = ix->i8st[4];
            c8.xl_max = ix->i8st[5];
            c8.rmax_half = 0.5 * ix->xmax * ix->xmax;
            HIP_TRY(launch_prep8(Qd, qn64, q8max, B, Bp, D, Gs, ix->metric, prec, c8, Qt, q8lsl, q8err, q8scal, st,
                                 q8res, q8err2));
            if (rs8) {  // L2: the start values at this batch's scale (+ their sum, the checksum's)
                if (chkr) HIP_TRY(hipMemsetAsync(chkr, 0, sizeof(uint32_t), st));
                HIP_TRY(launch_rstart8(ix->rinit32, N, q8scal, rs8, chkr, st));
            }
        }
        int n_flag = 0;
        if (!exact_all) {
            const bool timed = ix->timing != 0 && !opt.gate;  // a gated sub-search may not run at all
            hipEvent_t* tev = nullptr;
            if (timed) {
                if (w->t_pending == Workspace::kTRing) {  // ring full: read the oldest set
                    const int frc = flush_timing(ix, w, 1);
                    if (frc) return frc;
                }
                tev = w->tring[w->t_head];
                w->t_head = (w->t_head + 1) % Workspace::kTRing;
                w->t_pending++;
                for (int e = 0; e < 4; ++e)
                    if (!tev[e]) HIP_TRY(hipEventCreate(&tev[e]));
                HIP_TRY(hipEventRecord(tev[3], st));
            }
            const float* rowscale = ix->metric == 0 ? ix->inv32 : ix->sq32;
            const float* Xscan = i8_pass ? ix->Xq : xs_ptr(ix);  // the copy this pass reads
            if (n_pilot > 0) {
                if (i8_pass) {
                    HIP_TRY(launch_pilot8(prec, ix->metric, Xscan, ix->rinit32, md, Qt, q8scal, Gs, N, B,
                                          (B + QB_pilot - 1) / QB_pilot, QB_pilot, n_pilot, pslots, st,
                                          chke ? ix->d_csum : nullptr, chke, wide_long));
                    HIP_TRY(launch_pilot_bound(pslots, B, pilot_rank, gthr, st));
                } else if (split_pass) {
                    HIP_TRY(launch_pilot2(prec, ix->metric, pilot_rank, Xscan, ix->rinit32, md, Qt, Gs, N, B,
                                          (B + QB_pilot - 1) / QB_pilot, QB_pilot, n_pilot, pslots, gthr, st));
                    HIP_TRY(launch_pilot_bound(pslots, B, pilot_rank, gthr, st));
                }
                else
                    HIP_TRY(launch_pilot(prec, ix->metric, pilot_rank, Xscan, rowscale, md, Qt, Gs, N, B,
                                         n_qblocks, QB, n_pilot, pslots, gthr, st));
            }
            // scan_ns times the scan kernel alone (the roofline's kernel); pipeline_ns
            // everything from the pilot to the rerank
            if (opt.gate && (q4 || !(split_pass || i8_pass)))  // only these passes are gated
                return set_error(VDB_ERR_INVALID, "device re-pass: the sub-search has no gated candidate pass");
            if (timed) HIP_TRY(hipEventRecord(tev[0], st));
            if (q4) ix->n_q4++;
            if (wide8) ix->n_wide++;
            if (wide_long)
                HIP_TRY(launch_scan8wl(prec, ix->metric, Xscan, md, Qt, q8lsl, q8scal, Gs, N, B, n_seg8, gl_s, gl_i,
                                       gl_cap, segc, gthr, chkp, st));
            else if (wide8)
                HIP_TRY(launch_scan8w(prec, ix->metric, Xscan, rs8, md, Qt, q8lsl, q8scal, Gs, N, B, Bp, n_seg8, gl_s, gl_i,
                                      gl_cap, segc, gthr, chkp, Bp, chk_l ? 1 : 0, st));
            else if (i8_pass)
                HIP_TRY(launch_scan8(prec, ix->metric, KP, Xscan, (const float*)rs8, md, Qt, q8lsl, q8scal, Gs, N, B,
                                     n_qblocks, n_steps, n_wg, spw, gl_s, gl_i, gl_cnt, gl_cap, gthr, lockstep,
                                     (int)ix->scan_qlds, st, opt.gate, chkp, Bp, chk_l ? 1 : 0));
            else if (split_pass)
                HIP_TRY(launch_scan2(prec, ix->metric, KP, Xscan, ix->rinit32, md, Qt, Gs, N, B, n_qblocks, n_steps,
                                     n_wg, spw, gl_s, gl_i, gl_cnt, gl_cap, gthr, lockstep, st, q4,
                                     (int)ix->scan_qlds, opt.gate));
            else if (priv)
                HIP_TRY(launch_scan_topk_priv(prec, ix->metric, KP, Xscan, rowscale, md, Qt, Gs, N, B, n_qblocks,
                                              n_steps, n_wg, spw, gl_s, gl_i, gl_cnt, gl_cap, gthr, gslots, st));
            else
                HIP_TRY(launch_scan_topk(prec, ix->metric, KP, variant, Xscan, rowscale, md, Qt, Gs, N, B, n_qblocks,
                                         n_steps, n_wg, spw, gl_s, gl_i, gl_cnt, gl_cap, gthr, gslots, lockstep, st));
            if (timed) HIP_TRY(hipEventRecord(tev[1], st));
            FinishArgs fa;
            fa.gl_s = gl_s; fa.gl_i = gl_i; fa.gl_cnt = gl_cnt; fa.gl_cap = gl_cap;
            fa.Q = Qd; fa.qn64 = qn64; fa.X = ix->X; fa.G = ix->G; fa.D = D; fa.nrm64 = ix->nrm64; fa.k = k;
            // |approx - exact| <= eps_rel * sum|q_i x_i| (relative to |q||x|):
            //   fp32:   D fp32 MFMA additions + ~8 roundings of the normalisation / scaling
            //   bf16x3: 3D additions (each counted at 2^-23 in case the bf16 MFMA adds
            //           truncate) + the dropped hi*lo-order terms (< 3.1 2^-16) + the same 8
            //   bf16:   2D additions + the query split (2^-16) + the same 8, plus xres: the
            //           corpus rounding |q.(x - bf16(x))| <= |q| |x - bf16(x)|, bounded by the
            //           largest row residual measured at ingest (relative for cosine)
            // int8: exact integer sums; 8 roundings (normalisation, centring, the fp32 combination)
            fa.eps_rel = i8_pass ? 1.01 * 8.0 * std::ldexp(1.0, -24)
                         : prec == PREC_FP32 ? 1.01 * (double)(D + 8) * std::ldexp(1.0, -24)
                         : prec == PREC_BF16X3
                             ? 1.01 * (3.0 * D * std::ldexp(1.0, -23) + 3.1 * std::ldexp(1.0, -16) +
                                       8.0 * std::ldexp(1.0, -24))
                             : 1.01 * (2.0 * D * std::ldexp(1.0, -23) + 1.1 * std::ldexp(1.0, -16) +
                                       8.0 * std::ldexp(1.0, -24));
            fa.xmax = ix->xmax;
            fa.xres = prec != PREC_BF16 ? 0.0 : 1.01 * (ix->metric == 0 ? ix->xres_rel : ix->xres_abs);
            fa.dir = prec == PREC_BF16 && ix->dir_set && !ix->no_dir_bound ? ix->d_dir : nullptr;
            fa.dres = 1.01 * ix->xres_dir;
            if (i8_pass) {  // the int8 copy's rounding of the centred rows (absolute: cosine rows are unit)
                fa.xres = 1.01 * ix->i8st[prec == PREC_I8X3 ? 2 : 0] + 1e-300;  // (I8 / I8Q: the xh plane's)
                fa.dir = ix->dir_set && !ix->no_dir_bound ? ix->d_dir : nullptr;
                fa.dres = 1.01 * ix->i8st[prec == PREC_I8X3 ? 3 : 1];
                fa.qerr = q8err;
                fa.mu = ix->d_mu;
                if (i8_refine) {
                    fa.xh_rm = ix->Xh;
                    fa.qres = q8res;
                    fa.qerr2 = q8err2;
                    fa.qscal = q8scal;
                    fa.sx = ix->sx;
                    fa.Dp = ix->Dp;
                }
            }
            fa.out_s = out_s; fa.out_i = out_i; fa.out_k = out_k; fa.index_offset = index_offset;
            fa.row_ids = row_ids;
            fa.flag_count = flags; fa.flag_list = flags + 1; fa.gthr = gthr; fa.overflow_count = flags + B + 1;
            fa.incons_count = flags + B + 2;
            fa.gate = opt.gate;
            if (chk) {
                fa.chkp = chkp;
                fa.chke = chke;
                fa.chkr = chkr;
                fa.chk_q = Qt;
                fa.chk_csum = ix->d_csum;
                fa.chk_g8 = Gs;
                fa.chk_nw = n_wg8;
                fa.chk_ld = Bp;
                fa.chk_l = chk_l;
            }
            fa.qconst = fa.mu == q_mu && fa.dir == q_dir ? qconst : nullptr;  // (prep_queries' constants)
            fa.seg_cnt = segc;
            fa.seg_n = n_seg8;
            // auto: batches of >= 32 (throughput: C2 under three streams 437 -> 453 K QPS, the finish
            // beside the next batch's scan), not single queries (one batch alone its 4 waves are
            // slower: C2 B = 2 step 0.195 -> 0.217 ms; B = 64 p50 0.213 -> 0.240; profiles/r06_fs)
            // (and with the short-row wide pass, <= 128 dims: beside its small stage for <= 256
            // queries; for C4's 512 three workgroups per CU instead of one, 366 -> 374 K QPS,
            // profiles/r06_c4f);
            // auto also only while another search of the index is in flight: a batch alone keeps the
            // 16-wave form (its latency, the bench's p50)
            fa.small = D <= 1024 && (ix->finish_small == 1 ||
                                     (ix->finish_small < 0 && B >= 32 &&
                                      ((wide_long && Gs <= 32) || (wide8 && !wide_long)) &&
                                      others_in_flight(ix, w))) ? 1 : 0;
            fa.split = fin_split; fa.sx_ek = fx_ek; fa.sx_ck = fx_ck; fa.sx_cr = fx_cr; fa.sx_n = fx_n; fa.done = done;
            HIP_TRY(launch_finish(ix->metric, KP, fa, B, st));
            if (timed) HIP_TRY(hipEventRecord(tev[2], st));
            // Device-memory searches do not wait for the certificate: the exact path is
            // launched gated on the device's flag count (nothing runs when no query was
            // flagged), so the call returns with the whole search queued.
            if (ix->no_fallback && mem == VDB_MEM_DEVICE) return VDB_OK;
            if (!ix->no_fallback && mem == VDB_MEM_DEVICE && exact_bytes(ix, B, k, true) <= kGatedExactBytes) {
                {
                    std::lock_guard<std::mutex> lg(ix->ws_mu);  // lazily, once (concurrent searches)
                    if (!ix->d_totals) {
                        HIP_TRY(hipHostMalloc(&ix->h_totals, 2 * sizeof(unsigned long long), hipHostMallocDefault));
                        ix->h_totals[0] = ix->h_totals[1] = 0;
                        unsigned long long* d = nullptr;
                        // flagged, overflowed, flagged in a one-plane pass, re-passed on the device
                        HIP_TRY(hipMalloc(&d, 4 * sizeof(unsigned long long)));
                        // zeroed and COMPLETE before any search stream can use it: a plain hipMemset
                        // runs on the null stream, which a non-blocking caller stream does not order
                        // after -- the first search's device re-pass count could land before the
                        // zeroing and be wiped (GPUTEST_r04: repass_queries 2 of 3 on a side stream)
                        HIP_TRY(zero_now(d, 4 * sizeof(unsigned long long), ix->stream));
                        ix->d_totals = d;
                    }
                }
                unsigned long long* htot =
                    auto_prec && (one_plane || prec == PREC_I8X3 || prec == PREC_I8Q) ? ix->h_totals : nullptr;
                // The device re-pass: up to kRepassDev uncertified queries gathered on the
                // device into a BF16X3 sub-search on this stream, gated on their count (its candidate
                // pass and finish exit at once when nothing was flagged), its rows scattered back;
                // the rest, if any, take the gated exact path.  Like the host re-pass (repass_flagged)
                // for auto's one-plane / I8X3 passes, with the split copy kept beside the int8 one.
                const bool can_rep = !opt.repass && auto_prec && (one_plane || prec == PREC_I8X3 || prec == PREC_I8Q) &&
                                     xs_kind(VDB_PREC_BF16X3) == xs_kind(ix->precision) && rep_q &&
                                     k <= kMaxApproxK;
                bool rep = can_rep && ix->device_repass == 1;
                if (can_rep && ix->device_repass < 0) {
                    int a = ix->repass_arm.load();
                    while (a > 0 && !ix->repass_arm.compare_exchange_weak(a, a - 1)) {}
                    rep = a > 0;
                }
                if (rep) {
                    int* counts = flags + B + 3;  // [0] gathered (the sub-search's gate), [1] left over
                    HIP_TRY(launch_repass_gather(Qd, D, flags, R_rep, rep_q, counts, ix->d_totals + 3, st));
                    SearchOpts o;
                    o.force_b3 = true;
                    o.force_i8x3 = true;  // (I8X3 where the int8 copy is kept, else BF16X3)
                    o.repass = true;
                    o.gate = counts;
                    rc = search_locked(ix, rep_q, R_rep, k, md, VDB_MEM_DEVICE, rep_s, rep_i, rep_k, index_offset, st,
                                       row_ids, o);
                    if (rc) return rc;
                    HIP_TRY(launch_scatter_results(flags + 1, R_rep, k, rep_s, rep_i, rep_k, out_s, out_i, out_k, st,
                                                   counts));
                    if (B > R_rep)
                        rc = run_exact(ix, w, Qd, qn64, flags + 1 + R_rep, B - R_rep, k, md, out_s, out_i, out_k,
                                       index_offset, row_ids, st, counts + 1, flags + B + 1, done + R_rep, htot);
                    return rc;
                }
                rc = run_exact(ix, w, Qd, qn64, flags + 1, B, k, md, out_s, out_i, out_k, index_offset, row_ids, st,
                               flags, flags + B + 1, done, htot);
                return rc;
            }
            HIP_TRY(hipMemcpyAsync(w->host_flag, flags, sizeof(int), hipMemcpyDeviceToHost, st));
            HIP_TRY(hipMemcpyAsync(w->host_flag + 1, flags + B + 1, 2 * sizeof(int), hipMemcpyDeviceToHost, st));
            if (mem == VDB_MEM_HOST) {  // (valid when nothing was flagged: nothing rewrites them then)
                char* r = w->host_io + io_q;
                HIP_TRY(hipMemcpyAsync(r, out_s, (size_t)B * k * 4, hipMemcpyDeviceToHost, st));
                HIP_TRY(hipMemcpyAsync(r + (size_t)B * k * 4, out_i, (size_t)B * k * 8, hipMemcpyDeviceToHost, st));
                if (out_keys)
                    HIP_TRY(hipMemcpyAsync(r + (size_t)B * k * 12, out_k, (size_t)B * k * 8, hipMemcpyDeviceToHost, st));
            }
            HIP_TRY(hipStreamSynchronize(st));
            n_flag = w->host_flag[0];
            staged = mem == VDB_MEM_HOST && n_flag == 0;
            if (prec == PREC_I8 && n_flag > 0) ix->i8_wide = true;
            ix->n_overflow += w->host_flag[1];
            ix->n_incons += w->host_flag[2];
            if (auto_prec && one_plane && n_flag > 0 && !ix->no_fallback) {
                if (n_flag <= std::max(1, B / 8) && n_flag <= kRepassMax) {
                    // a few uncertified queries: re-pass just those in bf16x3 (the index stays bf16)
                    if (timed) {
                        const int frc = flush_timing(ix, w);
                        if (frc) return frc;
                    }
                    rc = repass_flagged(ix, Qd, flags + 1, n_flag, k, md, out_s, out_i, out_k, index_offset,
                                        row_ids, st);
                    if (rc) return rc;
                    n_flag = 0;
                } else {
                    if (prec == PREC_I8) auto_fail8(ix);
                    else auto_fail(ix);
                    ix->n_searches--;  // the retry counts this search (no double count)
                    ix->n_queries -= B;
                    return kRetryBf16x3;
                }
            }
            // auto's I8X3 pass: a failure the size of the one-plane passes' retries holds BF16X3
            // for the next searches (this batch's uncertified queries take the exact path below)
            if (auto_prec && prec == PREC_I8X3 && n_flag > std::max(1, B / 8) && !ix->no_fallback) auto_fail8(ix);
            // auto's I8Q pass: such a failure turns it off for this index (I8X3 from then on)
            if (auto_prec && prec == PREC_I8Q && n_flag > std::max(1, B / 8) && !ix->no_fallback) ix->i8q_off = true;
            if (timed) {
                const int frc = flush_timing(ix, w);
                if (frc) return frc;
            }
            if (n_flag > 0 && !ix->no_fallback) {
                ix->n_fallback += n_flag;
                rc = run_exact(ix, w, Qd, qn64, flags + 1, n_flag, k, md, out_s, out_i, out_k, index_offset, row_ids,
                               st);
                if (rc) return rc;
            }
        } else {
            ix->n_fallback += B;
            rc = run_exact(ix, w, Qd, qn64, nullptr, B, k, md, out_s, out_i, out_k, index_offset, row_ids, st);
            if (rc) return rc;
        }
    }
    if (mem == VDB_MEM_HOST && staged) {
        const char* r = w->host_io + io_q;
        std::memcpy(out_scores, r, (size_t)B * k * 4);
        std::memcpy(out_indices, r + (size_t)B * k * 4, (size_t)B * k * 8);
        if (out_keys) std::memcpy(out_keys, r + (size_t)B * k * 12, (size_t)B * k * 8);
    } else if (mem == VDB_MEM_HOST) {
        HIP_TRY(hipMemcpyAsync(out_scores, out_s, (size_t)B * k * 4, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipMemcpyAsync(out_indices, out_i, (size_t)B * k * 8, hipMemcpyDeviceToHost, st));
        if (out_keys) HIP_TRY(hipMemcpyAsync(out_keys, out_k, (size_t)B * k * 8, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
    }
    return VDB_OK;
}

int32_t vdb_shutdown(void) {
    std::vector<vdb_index*> live;
    {
        std::lock_guard<std::mutex> rg(g_reg_mu);
        live.assign(g_indices.begin(), g_indices.end());
    }
    std::set<int> devices;
    for (vdb_index* ix : live) {
        HIP_TRY(hipSetDevice(ix->device));
        devices.insert(ix->device);
        {
            const int wr = wait_idle(ix);  // every queued search of this index is done
            if (wr) return wr;
        }
        const int frc = flush_all_timing(ix);
        if (frc) return frc;
        std::lock_guard<std::mutex> g(ix->ws_mu);
        for (Workspace* w : ix->pool)
            if (!w->busy) free_workspace_memory(w);
    }
    for (int d : devices) {  // stream-ordered allocations (merge / graph scratch) back to the driver
        HIP_TRY(hipSetDevice(d));
        hipMemPool_t pool = nullptr;
        if (hipDeviceGetDefaultMemPool(&pool, d) == hipSuccess && pool) (void)hipMemPoolTrimTo(pool, 0);
    }
    return VDB_OK;
}

int32_t vdb_index_search(vdb_index* ix, const float* queries, int32_t B, int32_t k, const uint32_t* row_mask,
                         int32_t mem, float* out_scores, int64_t* out_indices, double* out_keys,
                         int64_t index_offset, void* stream) {
    int32_t rc = search_impl(ix, queries, B, k, row_mask, mem, out_scores, out_indices, out_keys, index_offset, stream,
                             nullptr);
    if (rc == kRetryBf16x3)
        rc = search_impl(ix, queries, B, k, row_mask, mem, out_scores, out_indices, out_keys, index_offset, stream,
                         nullptr, true);
    return rc;
}

}  // extern "C"

// ---- internal hooks for the multi-device set (vdb_shards.cpp) ----------------------------
namespace vdb {
int32_t index_search_rows(vdb_index* ix, const float* queries, int32_t B, int32_t k, const uint32_t* row_mask,
                          float* out_scores, int64_t* out_indices, double* out_keys, void* stream,
                          const int64_t* row_ids) {
    int32_t rc = search_impl(ix, queries, B, k, row_mask, VDB_MEM_DEVICE, out_scores, out_indices, out_keys, 0,
                             stream, row_ids);
    if (rc == kRetryBf16x3)  // a batch too large for the device-gated fallback: rerun in bf16x3
        rc = search_impl(ix, queries, B, k, row_mask, VDB_MEM_DEVICE, out_scores, out_indices, out_keys, 0, stream,
                         row_ids, true);
    return rc;
}
// Drop rows past `rows` (undo of a partial multi-shard add; rows past count are never read).
int32_t index_truncate(vdb_index* ix, int64_t rows) {
    std::unique_lock<std::shared_mutex> g(ix->mu);
    if (rows < ix->count) ix->count = rows;
    return VDB_OK;
}
int index_device(const vdb_index* ix) { return ix->device; }
int32_t set_error_msg(int code, const char* msg) { return set_error(code, "%s", msg); }
}  // namespace vdb

extern "C" {

int32_t vdb_merge_topk(const double* keys, const int64_t* idx, int32_t n_lists, int32_t nq, int32_t k_in,
                       int32_t k_out, int32_t metric, float* out_scores, int64_t* out_indices, double* out_keys,
                       void* stream) {
    if (!keys || !idx || !out_scores || !out_indices) return set_error(VDB_ERR_INVALID, "NULL argument");
    if (n_lists <= 0 || nq <= 0 || k_in <= 0 || k_out <= 0 || k_out > 1024 || k_in > 1024)
        return set_error(VDB_ERR_INVALID, "bad sizes n_lists=%d nq=%d k_in=%d k_out=%d", n_lists, nq, k_in, k_out);
    if (metric != 0 && metric != 1) return set_error(VDB_ERR_UNSUPPORTED, "metric %d", metric);
    hipStream_t st = (hipStream_t)stream;
    const int KP = std::max(32, next_pow2(std::max(k_in, k_out)));
    double* mk = nullptr;
    int64_t* mi = nullptr;
    HIP_TRY(hipMallocAsync((void**)&mk, (size_t)nq * KP * 8, st));
    HIP_TRY(hipMallocAsync((void**)&mi, (size_t)nq * KP * 8, st));
    // input [n_lists][nq][k_in]: list j of query q at j*nq*k_in + q*k_in
    HIP_TRY(launch_merge_f64_i64(KP, keys, idx, n_lists, k_in, k_in, (int64_t)nq * k_in, nq, mk, mi, st));
    HIP_TRY(launch_finalize_i64(metric, mk, mi, KP, nq, nullptr, k_out, out_scores, out_indices, out_keys, st));
    HIP_TRY(hipFreeAsync(mk, st));
    HIP_TRY(hipFreeAsync(mi, st));
    return VDB_OK;
}

int32_t vdb_similarity_matrix(const float* corpus, int64_t n, int32_t dim, const float* queries, int32_t nq,
                              int32_t metric, float* out, void* stream) {
    if (!corpus || !queries || !out) return set_error(VDB_ERR_INVALID, "NULL argument");
    if (n < 0 || dim <= 0 || nq <= 0) return set_error(VDB_ERR_INVALID, "bad sizes");
    if (metric < 0 || metric > 2) return set_error(VDB_ERR_UNSUPPORTED, "metric %d", metric);
    HIP_TRY(launch_similarity_matrix(corpus, n, dim, queries, nq, metric, out, (hipStream_t)stream));
    return VDB_OK;
}

int32_t vdb_normalize_rows(const float* in, int64_t n, int32_t dim, float* out, void* stream) {
    if ((!in || !out) && n > 0) return set_error(VDB_ERR_INVALID, "NULL argument");
    if (n < 0 || dim <= 0) return set_error(VDB_ERR_INVALID, "bad sizes");
    HIP_TRY(launch_normalize_rows(in, n, dim, out, (hipStream_t)stream));
    return VDB_OK;
}

int32_t vdb_topk_scores(const float* scores, int32_t rows, int64_t n, int32_t k, int32_t largest, int64_t* out_indices,
                        float* out_values, void* stream) {
    if (!scores || !out_indices) return set_error(VDB_ERR_INVALID, "NULL argument");
    if (rows <= 0 || n <= 0 || n > 0xFFFFFFFEll) return set_error(VDB_ERR_INVALID, "bad sizes rows=%d n=%lld", rows,
                                                                   (long long)n);
    if (k <= 0 || k > 1024 || k > n) return set_error(VDB_ERR_INVALID, "k must be in [1, min(n, 1024)], got %d", k);
    hipStream_t st = (hipStream_t)stream;
    void* ws = nullptr;
    HIP_TRY(hipMallocAsync(&ws, topk_workspace_bytes(n, rows, k), st));
    const hipError_t e = launch_topk_scores(scores, rows, n, k, largest, out_indices, out_values, ws, st);
    HIP_TRY(hipFreeAsync(ws, st));
    HIP_TRY(e);
    return VDB_OK;
}

}  // extern "C"

// =============================================================================
// Graph index (HNSW replacement, performance/hnsw_index.py:23-129)
// =============================================================================
struct vdb_graph {
    vdb_index* ix = nullptr;
    int R = 0;
    int knn = 0;                 // kNN candidates per row of the build (vdb_graph_add reuses it)
    int64_t n = 0;
    int64_t cap = 0;             // rows the device neighbour array holds
    int n_entries = 0;
    int32_t* nbr = nullptr;      // device [cap][R]
    int32_t* entries = nullptr;  // device [n_entries]
    std::vector<int32_t> h_nbr;  // host mirror [n][R] (incremental updates re-prune from it)
    int teams = 1;               // workgroups per query (vdb_graph_set_param "teams")
    unsigned long long* d_stats = nullptr;
    std::atomic<int64_t> n_queries{0};
    int device = 0;  // the index's device (the graph may outlive an explicitly closed index)
    // last search queued on each stream (device memory): vdb_graph_destroy waits for these only
    std::mutex use_mu;
    std::unordered_map<hipStream_t, hipEvent_t> uses;
};

namespace {

int graph_upload(vdb_index* ix, int R, int64_t n, const int32_t* nbr_host, const int32_t* ent_host, int n_ent,
                 vdb_graph** out) {
    vdb_graph* g = new vdb_graph();
    g->ix = ix;
    g->device = ix->device;
    g->R = R;
    g->knn = R;
    g->n = n;
    g->cap = std::max<int64_t>(n, 1);
    g->n_entries = n_ent;
    hipError_t e = hipMalloc(&g->nbr, (size_t)g->cap * R * sizeof(int32_t));
    if (e == hipSuccess) e = hipMalloc(&g->entries, (size_t)std::max(n_ent, 1) * sizeof(int32_t));
    if (e == hipSuccess) e = hipMalloc(&g->d_stats, 64);
    if (e == hipSuccess) e = zero_now(g->d_stats, 64, ix->stream);
    if (e == hipSuccess && n > 0) e = hipMemcpy(g->nbr, nbr_host, (size_t)n * R * sizeof(int32_t), hipMemcpyHostToDevice);
    if (e == hipSuccess && n_ent > 0)
        e = hipMemcpy(g->entries, ent_host, (size_t)n_ent * sizeof(int32_t), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        (void)hipFree(g->nbr);
        (void)hipFree(g->entries);
        (void)hipFree(g->d_stats);
        delete g;
        return set_error(e == hipErrorOutOfMemory ? VDB_ERR_OOM : VDB_ERR_HIP, "graph upload failed: %s",
                         hipGetErrorString(e));
    }
    g->h_nbr.assign(nbr_host, nbr_host + (size_t)n * R);
    *out = g;
    return VDB_OK;
}

// Exact kNN (kk incl. the row itself) of rows [r0, r1) over the whole index: the brute-force
// path with the rows as queries, 512 per launch.  kid [(r1 - r0) * kk] on the host.
int graph_knn(vdb_index* ix, int64_t r0, int64_t r1, int kk, std::vector<int64_t>& kid) {
    const int Bq = 512;
    const int D = ix->dim;
    kid.assign((size_t)(r1 - r0) * kk, -1);
    float* qbuf = nullptr;
    float* dsc = nullptr;
    int64_t* did = nullptr;
    hipStream_t st = ix->stream;
    hipError_t e = hipMalloc(&qbuf, (size_t)Bq * D * sizeof(float));
    if (e == hipSuccess) e = hipMalloc(&dsc, (size_t)Bq * kk * sizeof(float));
    if (e == hipSuccess) e = hipMalloc(&did, (size_t)Bq * kk * sizeof(int64_t));
    int rc = e == hipSuccess ? VDB_OK : set_error(VDB_ERR_OOM, "graph build buffers: %s", hipGetErrorString(e));
    for (int64_t q0 = r0; rc == VDB_OK && q0 < r1; q0 += Bq) {
        const int m = (int)std::min<int64_t>(Bq, r1 - q0);
        {
            std::shared_lock<std::shared_mutex> g(ix->mu);
            e = launch_unpack_rows(ix->X, ix->G, D, q0, m, qbuf, st);
        }
        if (e != hipSuccess) {
            rc = set_error(VDB_ERR_HIP, "graph build: %s", hipGetErrorString(e));
            break;
        }
        rc = vdb_index_search(ix, qbuf, m, kk, nullptr, VDB_MEM_DEVICE, dsc, did, nullptr, 0, st);
        if (rc) break;
        e = hipMemcpyAsync(kid.data() + (size_t)(q0 - r0) * kk, did, (size_t)m * kk * sizeof(int64_t),
                           hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) rc = set_error(VDB_ERR_HIP, "graph build: %s", hipGetErrorString(e));
    }
    (void)hipFree(qbuf);
    (void)hipFree(dsc);
    (void)hipFree(did);
    return rc;
}

// graph_prune over n work items: candidate rows cv [n][cw] (-1 padded), optional node ids
// (else items 0..n), results hn [n][limit] (and distances hd).
int graph_prune_host(vdb_index* ix, const std::vector<int32_t>& cv, int cw, const std::vector<int32_t>* nodes,
                     int64_t n, int limit, int fill, int sort, int32_t* hn, float* hd) {
    if (n <= 0) return VDB_OK;
    hipStream_t st = ix->stream;
    int32_t *dcand = nullptr, *dnbr = nullptr, *dnodes = nullptr;
    float* ddist = nullptr;
    hipError_t e = hipMalloc(&dcand, (size_t)n * cw * sizeof(int32_t));
    if (e == hipSuccess) e = hipMalloc(&dnbr, (size_t)n * limit * sizeof(int32_t));
    if (e == hipSuccess) e = hipMalloc(&ddist, (size_t)n * limit * sizeof(float));
    if (e == hipSuccess && nodes) e = hipMalloc(&dnodes, (size_t)n * sizeof(int32_t));
    if (e == hipSuccess) e = hipMemcpyAsync(dcand, cv.data(), (size_t)n * cw * sizeof(int32_t), hipMemcpyHostToDevice, st);
    if (e == hipSuccess && nodes)
        e = hipMemcpyAsync(dnodes, nodes->data(), (size_t)n * sizeof(int32_t), hipMemcpyHostToDevice, st);
    if (e == hipSuccess) {
        GraphPruneArgs pa;
        std::shared_lock<std::shared_mutex> g(ix->mu);
        pa.X = ix->X; pa.G = ix->G;
        pa.rowscale = ix->metric == VDB_METRIC_COSINE ? ix->inv32 : ix->sq32;
        pa.cand = dcand; pa.cw = cw; pa.n_nodes = n; pa.limit = limit; pa.rw = limit; pa.fill = fill;
        pa.out_nbr = dnbr; pa.out_dist = ddist; pa.nodes = dnodes; pa.sort = sort;
        e = launch_graph_prune(ix->metric, pa, st);
    }
    if (e == hipSuccess) e = hipMemcpyAsync(hn, dnbr, (size_t)n * limit * sizeof(int32_t), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess && hd) e = hipMemcpyAsync(hd, ddist, (size_t)n * limit * sizeof(float), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    (void)hipFree(dcand);
    (void)hipFree(dnbr);
    (void)hipFree(ddist);
    (void)hipFree(dnodes);
    return e == hipSuccess ? VDB_OK : set_error(VDB_ERR_HIP, "graph prune: %s", hipGetErrorString(e));
}

// Candidate rows of rows [r0, r1) from their kNN lists (self and -1 dropped), cw per row.
std::vector<int32_t> knn_candidates(const std::vector<int64_t>& kid, int64_t r0, int64_t r1, int kk, int cw) {
    std::vector<int32_t> cand((size_t)(r1 - r0) * cw, -1);
    for (int64_t i = r0; i < r1; ++i) {
        int c = 0;
        for (int j = 0; j < kk && c < cw; ++j) {
            const int64_t v = kid[(size_t)(i - r0) * kk + j];
            if (v < 0 || v == i) continue;
            cand[(size_t)(i - r0) * cw + c++] = (int32_t)v;
        }
    }
    return cand;
}

}  // namespace

extern "C" {

// entry rows of a graph: up to 256 every search team scores all of them; more (up to this many)
// are split into one spread slice of <= 256 per team (vdb_graph.hip)
constexpr int kGraphEntriesMax = 1 << 20;

int32_t vdb_graph_build(vdb_index* ix, int32_t degree, int32_t knn, int32_t n_entries, vdb_graph** out) {
    if (!ix || !out) return set_error(VDB_ERR_INVALID, "NULL argument");
    *out = nullptr;
    if (degree < 2 || degree > 64 || (degree & 1)) return set_error(VDB_ERR_INVALID, "degree must be even in [2, 64]");
    if (knn < degree / 2 || knn > 200) return set_error(VDB_ERR_INVALID, "knn must be in [degree/2, 200]");
    if (n_entries < 1 || n_entries > kGraphEntriesMax)
        return set_error(VDB_ERR_INVALID, "n_entries must be in [1, %d]", kGraphEntriesMax);
    HIP_TRY(hipSetDevice(ix->device));
    const int64_t N = ix->count;
    if (N > 0x7FFFFFFF) return set_error(VDB_ERR_INVALID, "graph rows are int32");
    const int R = degree, F = degree / 2;
    const int kk = (int)std::min<int64_t>(knn + 1, std::max<int64_t>(N, 1));  // + the row itself
    std::vector<int32_t> nbr((size_t)N * R, -1);
    if (N > 1) {
        // 1. exact kNN of every row (the brute-force path, rows as queries)
        std::vector<int64_t> kid;
        int rc = graph_knn(ix, 0, N, kk, kid);
        if (rc) return rc;
        // 2. hnswlib-style selection: pass 1 keeps <= M = R/2 diverse
        //    out-edges from the kNN; pass 2 re-selects <= R from out- plus in-edges
        //    (hnswlib's level-0 lists: the node's own links plus the links of later
        //    insertions that chose it, re-pruned when they exceed 2M).
        const int CW = std::min(knn, 63);
        std::vector<int32_t> cand = knn_candidates(kid, 0, N, kk, CW);
        kid.clear(); kid.shrink_to_fit();
        std::vector<int32_t> fwd((size_t)N * F);
        std::vector<float> fdist((size_t)N * F);
        rc = graph_prune_host(ix, cand, CW, nullptr, N, F, 0, 0, fwd.data(), fdist.data());
        if (rc) return rc;
        cand.clear(); cand.shrink_to_fit();
        // pool of v: out-edges of v and in-edges u -> v, nearest first, <= 63
        std::vector<int64_t> roff(N + 1, 0);
        for (size_t t = 0; t < fwd.size(); ++t)
            if (fwd[t] >= 0) roff[fwd[t] + 1]++;
        for (int64_t i = 0; i < N; ++i) roff[i + 1] += roff[i];
        std::vector<std::pair<float, int32_t>> rev(roff[N]);
        std::vector<int64_t> rpos(roff.begin(), roff.end() - 1);
        for (int64_t u = 0; u < N; ++u)
            for (int j = 0; j < F; ++j) {
                const int32_t w = fwd[(size_t)u * F + j];
                if (w >= 0) rev[rpos[w]++] = {fdist[(size_t)u * F + j], (int32_t)u};
            }
        std::vector<int32_t> cand2((size_t)N * 63, -1);
        std::vector<std::pair<float, int32_t>> pool;
        for (int64_t v = 0; v < N; ++v) {
            pool.clear();
            for (int j = 0; j < F; ++j)
                if (fwd[(size_t)v * F + j] >= 0) pool.push_back({fdist[(size_t)v * F + j], fwd[(size_t)v * F + j]});
            pool.insert(pool.end(), rev.begin() + roff[v], rev.begin() + roff[v + 1]);
            std::sort(pool.begin(), pool.end(), [](const std::pair<float, int32_t>& x, const std::pair<float, int32_t>& y) {
                return x.first < y.first || (x.first == y.first && x.second < y.second);
            });
            int c = 0;
            int32_t* row = cand2.data() + (size_t)v * 63;
            for (size_t t = 0; t < pool.size() && c < 63; ++t) {
                bool dup = false;
                for (int q = c - 1; q >= 0 && !dup; --q) dup = row[q] == pool[t].second;
                if (!dup) row[c++] = pool[t].second;
            }
        }
        rc = graph_prune_host(ix, cand2, 63, nullptr, N, R, (int)ix->graph_fill, 0, nbr.data(), nullptr);
        if (rc) return rc;
    }
    // 3. entry rows: evenly spread
    const int E = (int)std::min<int64_t>(n_entries, std::max<int64_t>(N, 1));
    std::vector<int32_t> ent(E);
    for (int i = 0; i < E; ++i) ent[i] = (int32_t)((int64_t)i * N / E);
    const int rc = graph_upload(ix, R, N, nbr.data(), ent.data(), N > 0 ? E : 0, out);
    if (rc == VDB_OK) (*out)->knn = knn;
    return rc;
}

// Incremental insertion of the rows the index gained since the graph was built (hnswlib
// inserts one row at a time; here a whole batch): exact kNN of the new rows over all rows,
// pass-1 selection of their out-edges, then every node that gains an in-edge (old or new)
// re-selects <= R from its current list plus the new in-edges (pass 2 with the candidates
// ordered by distance in the kernel).  Old rows' other links are kept.
int32_t vdb_graph_add(vdb_graph* g) {
    if (!g) return set_error(VDB_ERR_INVALID, "graph is NULL");
    vdb_index* ix = g->ix;
    HIP_TRY(hipSetDevice(ix->device));
    const int64_t n0 = g->n, N = ix->count;
    if (N < n0) return set_error(VDB_ERR_INVALID, "index has fewer rows (%lld) than the graph (%lld)", (long long)N,
                                 (long long)n0);
    if (N == n0) return VDB_OK;
    if (N > 0x7FFFFFFF) return set_error(VDB_ERR_INVALID, "graph rows are int32");
    const int R = g->R, F = std::max(1, R / 2);
    const int knn = std::max(g->knn, F);
    const int kk = (int)std::min<int64_t>(knn + 1, N);
    const int64_t nn = N - n0;
    // 1. new rows' out-edges
    std::vector<int64_t> kid;
    int rc = graph_knn(ix, n0, N, kk, kid);
    if (rc) return rc;
    const int CW = std::min(knn, 63);
    std::vector<int32_t> cand = knn_candidates(kid, n0, N, kk, CW);
    kid.clear(); kid.shrink_to_fit();
    std::vector<int32_t> nodes(nn);
    for (int64_t i = 0; i < nn; ++i) nodes[i] = (int32_t)(n0 + i);
    std::vector<int32_t> fwd((size_t)nn * F);
    rc = graph_prune_host(ix, cand, CW, &nodes, nn, F, 0, 0, fwd.data(), nullptr);
    if (rc) return rc;
    // 2. pools: affected node v -> its current list (new rows: their out-edges) + in-edges
    std::unordered_map<int32_t, std::vector<int32_t>> in;
    for (int64_t i = 0; i < nn; ++i)
        for (int j = 0; j < F; ++j) {
            const int32_t w = fwd[(size_t)i * F + j];
            if (w >= 0) in[w].push_back((int32_t)(n0 + i));
        }
    std::vector<int32_t> aff(nodes);
    for (const auto& kv : in)
        if (kv.first < n0) aff.push_back(kv.first);
    std::vector<int32_t> cand2(aff.size() * 63, -1);
    for (size_t a = 0; a < aff.size(); ++a) {
        const int32_t v = aff[a];
        int32_t* row = cand2.data() + a * 63;
        int c = 0;
        auto push = [&](int32_t u) {
            if (u < 0 || u == v || c >= 63) return;
            for (int q = 0; q < c; ++q)
                if (row[q] == u) return;
            row[c++] = u;
        };
        if (v >= n0) {
            for (int j = 0; j < F; ++j) push(fwd[(size_t)(v - n0) * F + j]);
        } else {
            for (int j = 0; j < R; ++j) push(g->h_nbr[(size_t)v * R + j]);
        }
        auto it = in.find(v);
        if (it != in.end())
            for (int32_t u : it->second) push(u);
    }
    std::vector<int32_t> upd(aff.size() * R);
    rc = graph_prune_host(ix, cand2, 63, &aff, (int64_t)aff.size(), R, (int)ix->graph_fill, 1, upd.data(), nullptr);
    if (rc) return rc;
    // 3. device array: grow (doubling) and scatter the updated lists
    hipStream_t st = ix->stream;
    if (N > g->cap) {
        int64_t cap = std::max<int64_t>(g->cap * 2, 1024);
        while (cap < N) cap *= 2;
        int32_t* nb = nullptr;
        HIP_TRY(hipMalloc(&nb, (size_t)cap * R * sizeof(int32_t)));
        hipError_t e = hipMemcpyAsync(nb, g->nbr, (size_t)n0 * R * sizeof(int32_t), hipMemcpyDeviceToDevice, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) {
            (void)hipFree(nb);
            return set_error(VDB_ERR_HIP, "graph grow: %s", hipGetErrorString(e));
        }
        {
            const int wr = wait_idle(ix);  // graph searches that read the old array are done
            if (wr) return wr;
        }
        (void)hipFree(g->nbr);
        g->nbr = nb;
        g->cap = cap;
    }
    g->h_nbr.resize((size_t)N * R, -1);
    for (size_t a = 0; a < aff.size(); ++a)
        std::memcpy(g->h_nbr.data() + (size_t)aff[a] * R, upd.data() + a * R, R * sizeof(int32_t));
    int32_t *dids = nullptr, *drows = nullptr;
    hipError_t e = hipMalloc(&dids, aff.size() * sizeof(int32_t));
    if (e == hipSuccess) e = hipMalloc(&drows, upd.size() * sizeof(int32_t));
    if (e == hipSuccess) e = hipMemcpyAsync(dids, aff.data(), aff.size() * sizeof(int32_t), hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = hipMemcpyAsync(drows, upd.data(), upd.size() * sizeof(int32_t), hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = launch_graph_scatter(g->nbr, R, dids, drows, (int64_t)aff.size(), st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    (void)hipFree(dids);
    (void)hipFree(drows);
    if (e != hipSuccess) return set_error(VDB_ERR_HIP, "graph update: %s", hipGetErrorString(e));
    g->n = N;
    return VDB_OK;
}

int32_t vdb_graph_import(vdb_index* ix, int32_t degree, int64_t n, const int32_t* nbr, int32_t n_entries,
                         const int32_t* entries, vdb_graph** out) {
    if (!ix || !out || (n > 0 && !nbr) || (n_entries > 0 && !entries)) return set_error(VDB_ERR_INVALID, "NULL argument");
    *out = nullptr;
    if (degree < 1 || degree > 64) return set_error(VDB_ERR_INVALID, "degree must be in [1, 64]");
    if (n != ix->count) return set_error(VDB_ERR_INVALID, "graph has %lld rows, index %lld", (long long)n, (long long)ix->count);
    if (n_entries < 0 || n_entries > kGraphEntriesMax)
        return set_error(VDB_ERR_INVALID, "n_entries must be in [0, %d]", kGraphEntriesMax);
    for (int64_t i = 0; i < n * degree; ++i)
        if (nbr[i] < -1 || nbr[i] >= n) return set_error(VDB_ERR_INVALID, "neighbour id out of range at %lld", (long long)i);
    for (int i = 0; i < n_entries; ++i)
        if (entries[i] < 0 || entries[i] >= n) return set_error(VDB_ERR_INVALID, "entry id out of range");
    HIP_TRY(hipSetDevice(ix->device));
    return graph_upload(ix, degree, n, nbr, entries, n_entries, out);
}

int32_t vdb_graph_info(const vdb_graph* g, int64_t* n_rows, int32_t* degree, int32_t* n_entries) {
    if (!g) return set_error(VDB_ERR_INVALID, "graph is NULL");
    if (n_rows) *n_rows = g->n;
    if (degree) *degree = g->R;
    if (n_entries) *n_entries = g->n_entries;
    return VDB_OK;
}

int32_t vdb_graph_export(const vdb_graph* g, int32_t* nbr_host, int32_t* entries_host) {
    if (!g) return set_error(VDB_ERR_INVALID, "graph is NULL");
    HIP_TRY(hipSetDevice(g->ix->device));
    if (nbr_host && g->n > 0)
        HIP_TRY(hipMemcpy(nbr_host, g->nbr, (size_t)g->n * g->R * sizeof(int32_t), hipMemcpyDeviceToHost));
    if (entries_host && g->n_entries > 0)
        HIP_TRY(hipMemcpy(entries_host, g->entries, (size_t)g->n_entries * sizeof(int32_t), hipMemcpyDeviceToHost));
    return VDB_OK;
}

int32_t vdb_graph_search(vdb_graph* g, const float* queries, int32_t nq, int32_t k, int32_t ef, int32_t mem,
                         int64_t* labels, float* distances, void* stream) {
    if (!g || !queries || !labels || !distances) return set_error(VDB_ERR_INVALID, "NULL argument");
    if (nq <= 0) return set_error(VDB_ERR_INVALID, "n_queries must be >= 1");
    if (ef < 1 || ef > 256) return set_error(VDB_ERR_INVALID, "ef must be in [1, 256], got %d", ef);
    if (k < 1 || k > ef) return set_error(VDB_ERR_INVALID, "k must be in [1, ef], got k=%d ef=%d", k, ef);
    if (mem != VDB_MEM_HOST && mem != VDB_MEM_DEVICE) return set_error(VDB_ERR_INVALID, "bad mem kind %d", mem);
    vdb_index* ix = g->ix;
    const int D = ix->dim;
    if (mem == VDB_MEM_HOST && !all_finite(queries, (int64_t)nq * D))
        return set_error(VDB_ERR_NONFINITE, "query contains NaN or Inf");
    HIP_TRY(hipSetDevice(ix->device));
    std::shared_lock<std::shared_mutex> lk(ix->mu);
    if (ix->count != g->n) return set_error(VDB_ERR_INVALID, "graph is stale: %lld rows, index %lld", (long long)g->n,
                                            (long long)ix->count);
    // device memory: the caller's stream, NULL = the null stream (ordered with the caller's
    // default-stream work, e.g. PyTorch's); host memory: NULL = the index's own stream
    hipStream_t st = (stream || mem == VDB_MEM_DEVICE) ? (hipStream_t)stream : ix->stream;
    const float* Qd = queries;
    int64_t* ol = labels;
    float* od = distances;
    void* tmp = nullptr;
    const int T = (int)std::min<int64_t>(g->teams, std::max(g->n_entries, 1));
    const size_t qb = mem == VDB_MEM_HOST ? (size_t)nq * D * 4 : 0, lb = (size_t)nq * k * 8, db = (size_t)nq * k * 4;
    const size_t tb = T > 1 ? (size_t)nq * T * k * 12 + 512 : 0;
    if (mem == VDB_MEM_HOST || T > 1) {
        HIP_TRY(hipMallocAsync(&tmp, qb + lb + db + tb + 1024, st));
        char* base = (char*)tmp;
        if (mem == VDB_MEM_HOST) {
            HIP_TRY(hipMemcpyAsync(base, queries, qb, hipMemcpyHostToDevice, st));
            Qd = (const float*)base;
            ol = (int64_t*)(base + ((qb + 255) & ~size_t(255)));
            od = (float*)((char*)ol + ((lb + 255) & ~size_t(255)));
        }
    }
    GraphSearchArgs a;
    a.rows = ix->X; a.Dp = ix->Dp; a.D = D; a.rowscale = ix->metric == 0 ? ix->inv32 : ix->sq32; a.n_rows = g->n;
    a.nbr = g->nbr; a.R = g->R; a.entries = g->entries; a.n_entries = g->n_entries;
    a.Q = Qd; a.k = k; a.ef = ef; a.out_lab = ol; a.out_dist = od; a.stats = g->d_stats;
    a.teams = T;
    if (T > 1) {
        char* tbase = (char*)tmp + ((qb + 255) & ~size_t(255)) + ((lb + 255) & ~size_t(255)) + ((db + 255) & ~size_t(255));
        a.tmp_lab = (int64_t*)tbase;
        a.tmp_dist = (float*)(tbase + (((size_t)nq * T * k * 8 + 255) & ~size_t(255)));
    }
    if (g->n == 0) {
        HIP_TRY(hipMemsetAsync(ol, 0xFF, (size_t)nq * k * 8, st));
    } else {
        HIP_TRY(launch_graph_search(ix->metric, a, nq, st));
    }
    g->n_queries += nq;
    if (mem == VDB_MEM_HOST) {
        HIP_TRY(hipMemcpyAsync(labels, ol, (size_t)nq * k * 8, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipMemcpyAsync(distances, od, (size_t)nq * k * 4, hipMemcpyDeviceToHost, st));
    }
    if (tmp) HIP_TRY(hipFreeAsync(tmp, st));
    if (mem == VDB_MEM_HOST) HIP_TRY(hipStreamSynchronize(st));
    else {
        const int nr = note_use(ix, st);  // a later resize of the index waits for this search
        if (nr) return nr;
        std::lock_guard<std::mutex> lg(g->use_mu);  // and so does the graph's destroy
        hipEvent_t& ev = g->uses[st];
        if (!ev) HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        HIP_TRY(hipEventRecord(ev, st));
    }
    return VDB_OK;
}

int32_t vdb_graph_set_param(vdb_graph* g, const char* name, int64_t value) {
    if (!g || !name) return set_error(VDB_ERR_INVALID, "NULL argument");
    const std::string n(name);
    if (n == "teams") {
        if (value < 1 || value > 256) return set_error(VDB_ERR_INVALID, "teams must be in [1, 256]");
        g->teams = (int)value;
    } else {
        return set_error(VDB_ERR_INVALID, "unknown graph parameter '%s'", name);
    }
    return VDB_OK;
}

int32_t vdb_graph_stat(const vdb_graph* g, const char* name, int64_t* value) {
    if (!g || !name || !value) return set_error(VDB_ERR_INVALID, "NULL argument");
    std::string n(name);
    if (n == "queries") {
        *value = g->n_queries.load();
    } else if (n == "iterations" || n == "visited") {
        unsigned long long v[2] = {0, 0};
        HIP_TRY(hipMemcpy(v, g->d_stats, sizeof(v), hipMemcpyDeviceToHost));
        *value = (int64_t)v[n == "visited" ? 1 : 0];
    } else {
        return set_error(VDB_ERR_INVALID, "unknown graph stat '%s'", name);
    }
    return VDB_OK;
}

int32_t vdb_graph_destroy(vdb_graph* g) {
    if (!g) return VDB_OK;
    (void)hipSetDevice(g->device);
    for (auto& kv : g->uses) {  // its own searches only: the index may already be closed
        (void)hipEventSynchronize(kv.second);
        (void)hipEventDestroy(kv.second);
    }
    (void)hipFree(g->nbr);
    (void)hipFree(g->entries);
    (void)hipFree(g->d_stats);
    delete g;
    return VDB_OK;
}

}  // extern "C"
