// vdb_shards.cpp — one corpus row-sharded over several GPUs of ONE process (include/vdb.h
// vdb_shards_*).  The reference server is a single process (main.py:395, uvicorn
// workers=1) and its store holds the corpus on one device (service/optimized_vector_store.py:59-114);
// this is the same store API over G devices:
//
//   add      rows keep their global ids (insertion order); each add is cut into contiguous
//            pieces that level the shard sizes, and every shard keeps a device array of the
//            global id of each of its rows;
//   search   queued on every shard at once, one stream per shard, without host waits: the
//            shard's device search (candidate pass + exact fp64 rerank, vdb_api.cpp) writes its
//            top-k as (fp64 key, GLOBAL row); the G lists are gathered to the root device by
//            peer copies over xGMI (hipMemcpyPeerAsync on the shard's stream), and merged there
//            by (key desc, row asc) — bit-identical to one device holding every row.
//
// The exchange is a gather of G x B x k (key, id) pairs to one device, the only place the
// results are needed (they go back to the caller's host buffers): point-to-point copies
// are that gather.  (Across processes, one per GPU, the same lists travel by an RCCL
// all-gather instead: service/sharded.py.)  A device may appear more than once (tests run
// two shards on one GPU); the copies are then device-local.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <functional>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <vector>

#include "../../include/vdb.h"
#include "vdb_internal.h"

namespace vdb {
int32_t index_search_rows(vdb_index* ix, const float* queries, int32_t B, int32_t k, const uint32_t* row_mask,
                          float* out_scores, int64_t* out_indices, double* out_keys, void* stream,
                          const int64_t* row_ids);
int32_t index_truncate(vdb_index* ix, int64_t rows);
int index_device(const vdb_index* ix);
int32_t set_error_msg(int code, const char* msg);
}  // namespace vdb

using namespace vdb;

namespace {

struct Piece {
    int64_t g0;  // first global row
    int64_t l0;  // first local row
    int64_t n;
};

struct Shard {
    int device = 0;
    vdb_index* ix = nullptr;
    hipStream_t st = nullptr;
    hipEvent_t done = nullptr;
    std::vector<Piece> pieces;
    int64_t count = 0;
    int64_t* gid = nullptr;  // device: global id of every local row
    int64_t gid_cap = 0;
};

int fail(int code, const std::string& msg) { return set_error_msg(code, msg.c_str()); }

#define SH_TRY(expr)                                                                                          \
    do {                                                                                                      \
        hipError_t _e = (expr);                                                                               \
        if (_e != hipSuccess)                                                                                 \
            return fail(_e == hipErrorOutOfMemory ? VDB_ERR_OOM : VDB_ERR_HIP,                                \
                        std::string(#expr) + " failed: " + hipGetErrorString(_e));                            \
    } while (0)

int next_pow2(int v) {
    int p = 1;
    while (p < v) p <<= 1;
    return p;
}

}  // namespace

struct vdb_shards {
    int dim = 0, metric = 0;
    std::vector<Shard> sh;
    int64_t count = 0;
    std::shared_mutex mu;  // add / clear exclusive, search shared
};

extern "C" {

int32_t vdb_shards_create(int32_t dim, int32_t metric, const int32_t* devices, int32_t n_devices, vdb_shards** out) {
    if (!out || !devices) return fail(VDB_ERR_INVALID, "NULL argument");
    *out = nullptr;
    if (n_devices < 1 || n_devices > 64) return fail(VDB_ERR_INVALID, "n_devices must be in [1, 64]");
    vdb_shards* s = new vdb_shards();
    s->dim = dim;
    s->metric = metric;
    for (int g = 0; g < n_devices; ++g) {
        Shard sd;
        sd.device = devices[g];
        int rc = vdb_index_create(dim, metric, devices[g], &sd.ix);
        hipError_t e = hipSuccess;
        if (rc == VDB_OK) {
            e = hipSetDevice(devices[g]);
            if (e == hipSuccess) e = hipStreamCreateWithFlags(&sd.st, hipStreamNonBlocking);
            if (e == hipSuccess) e = hipEventCreateWithFlags(&sd.done, hipEventDisableTiming);
        }
        s->sh.push_back(sd);
        if (rc != VDB_OK || e != hipSuccess) {
            vdb_shards_destroy(s);
            return rc != VDB_OK ? rc : fail(VDB_ERR_HIP, std::string("shard setup: ") + hipGetErrorString(e));
        }
    }
    // direct xGMI peer access root <-> every other device (a no-op for repeated devices)
    const int root = devices[0];
    for (int g = 1; g < n_devices; ++g) {
        const int d = devices[g];
        if (d == root) continue;
        int can = 0;
        if (hipDeviceCanAccessPeer(&can, root, d) == hipSuccess && can) {
            (void)hipSetDevice(root);
            (void)hipDeviceEnablePeerAccess(d, 0);
            (void)hipSetDevice(d);
            (void)hipDeviceEnablePeerAccess(root, 0);
        }
    }
    (void)hipGetLastError();  // "already enabled" is not an error here
    *out = s;
    return VDB_OK;
}

int32_t vdb_shards_destroy(vdb_shards* s) {
    if (!s) return VDB_OK;
    for (Shard& sd : s->sh) {
        (void)hipSetDevice(sd.device);
        if (sd.st) (void)hipStreamSynchronize(sd.st);
        if (sd.gid) (void)hipFree(sd.gid);
        if (sd.done) (void)hipEventDestroy(sd.done);
        if (sd.st) (void)hipStreamDestroy(sd.st);
        if (sd.ix) vdb_index_destroy(sd.ix);
    }
    delete s;
    return VDB_OK;
}

int32_t vdb_shards_count(const vdb_shards* s, int64_t* n) {
    if (!s || !n) return fail(VDB_ERR_INVALID, "NULL argument");
    *n = s->count;
    return VDB_OK;
}

int32_t vdb_shards_add(vdb_shards* s, const float* vectors, int64_t n) {
    if (!s) return fail(VDB_ERR_INVALID, "shard set is NULL");
    if (n < 0) return fail(VDB_ERR_INVALID, "n must be >= 0");
    if (n == 0) return VDB_OK;
    if (!vectors) return fail(VDB_ERR_INVALID, "vectors is NULL");
    std::unique_lock<std::shared_mutex> lk(s->mu);
    const int G = (int)s->sh.size();
    const int D = s->dim;
    for (int64_t i = 0; i < n * D; ++i)  // checked before any shard appends (an add is all or nothing)
        if (!std::isfinite(vectors[i])) return fail(VDB_ERR_NONFINITE, "rows contain NaN or Inf; nothing was added");
    // level the shard sizes: target ceil(total / G) rows each, filled in shard order
    const int64_t total = s->count + n;
    const int64_t target = (total + G - 1) / G;
    std::vector<int64_t> take(G, 0);
    int64_t left = n;
    for (int g = 0; g < G && left > 0; ++g) {
        take[g] = std::min<int64_t>(left, std::max<int64_t>(0, target - s->sh[g].count));
        left -= take[g];
    }
    std::vector<int64_t> before(G);
    for (int g = 0; g < G; ++g) before[g] = s->sh[g].count;
    int64_t off = 0;
    int rc = VDB_OK;
    std::vector<int64_t> ids;
    for (int g = 0; g < G && rc == VDB_OK; ++g) {
        if (take[g] == 0) continue;
        Shard& sd = s->sh[g];
        rc = vdb_index_add(sd.ix, vectors + off * D, take[g], VDB_MEM_HOST, nullptr);
        if (rc != VDB_OK) break;
        const int64_t need = sd.count + take[g];
        hipError_t e = hipSetDevice(sd.device);
        if (e == hipSuccess && need > sd.gid_cap) {
            int64_t cap = std::max<int64_t>(1024, sd.gid_cap);
            while (cap < need) cap *= 2;
            int64_t* ng = nullptr;
            e = hipMalloc(&ng, (size_t)cap * sizeof(int64_t));
            if (e == hipSuccess && sd.count) e = hipMemcpy(ng, sd.gid, (size_t)sd.count * 8, hipMemcpyDeviceToDevice);
            if (e == hipSuccess) {
                if (sd.gid) (void)hipFree(sd.gid);
                sd.gid = ng;
                sd.gid_cap = cap;
            } else if (ng) {
                (void)hipFree(ng);
            }
        }
        if (e == hipSuccess) {
            ids.resize(take[g]);
            for (int64_t i = 0; i < take[g]; ++i) ids[i] = s->count + off + i;
            e = hipMemcpy(sd.gid + sd.count, ids.data(), (size_t)take[g] * 8, hipMemcpyHostToDevice);
        }
        if (e != hipSuccess) {
            rc = fail(e == hipErrorOutOfMemory ? VDB_ERR_OOM : VDB_ERR_HIP,
                      std::string("shard row ids: ") + hipGetErrorString(e));
            index_truncate(sd.ix, sd.count);
            break;
        }
        sd.pieces.push_back({s->count + off, sd.count, take[g]});
        sd.count += take[g];
        off += take[g];
    }
    if (rc != VDB_OK) {  // undo the shards that already took their piece
        for (int g = 0; g < G; ++g) {
            Shard& sd = s->sh[g];
            if (sd.count != before[g]) {
                index_truncate(sd.ix, before[g]);
                sd.pieces.pop_back();
                sd.count = before[g];
            }
        }
        return rc;
    }
    s->count = total;
    return VDB_OK;
}

}  // extern "C"

namespace {

// The shard-local bitmap of a global one: bit l <- bit gid[l] of the global mask (both on the
// shard's device); one thread per local word.
__global__ void __launch_bounds__(256) shard_mask_kernel(const uint32_t* __restrict__ gmask,
                                                         const int64_t* __restrict__ gid, int64_t n,
                                                         uint32_t* __restrict__ lmask) {
    const int64_t w = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (w >= (n + 31) / 32) return;
    uint32_t bits = 0;
    for (int b = 0; b < 32; ++b) {
        const int64_t l = w * 32 + b;
        if (l < n) {
            const int64_t g = gid[l];
            bits |= ((gmask[g >> 5] >> (g & 31)) & 1u) << b;
        }
    }
    lmask[w] = bits;
}

// The search of every shard, queued without a host wait: queries, mask and outputs on
// devices[0], ordered after the work queued on `st` (a stream of devices[0]) so far; the
// outputs are ready once `st` reaches the merge.  Each shard: peer copy of the queries (and
// of the global mask, then its local bitmap built on its device) on the shard's stream, the
// shard's device search (candidate pass + exact rerank, global ids, fp64 keys), peer copy of
// its [B, k] lists into slot g of the root's gather buffers; the root waits for every shard
// on `st` and merges there.  Scratch is stream-ordered (hipMallocAsync / hipFreeAsync).
int shards_search_dev(vdb_shards* s, const float* q_root, int32_t B, int32_t k, const uint32_t* mask_root,
                      float* out_scores, int64_t* out_indices, double* out_keys, hipStream_t st) {
    const int G = (int)s->sh.size();
    const int D = s->dim;
    const size_t qb = (size_t)B * D * 4, lb = (size_t)B * k;
    const int root = s->sh[0].device;
    const int64_t gmw = (s->count + 31) / 32;
    SH_TRY(hipSetDevice(root));
    const int KP = std::max(32, next_pow2(k));
    const size_t r_keys = (size_t)G * lb * 8, r_ids = r_keys, m_bytes = (size_t)B * KP * 16;
    char* rb = nullptr;
    SH_TRY(hipMallocAsync((void**)&rb, r_keys + r_ids + m_bytes + 1024, st));
    double* g_keys = (double*)rb;
    int64_t* g_ids = (int64_t*)(rb + r_keys);
    double* m_keys = (double*)(rb + r_keys + r_ids);
    int64_t* m_ids = (int64_t*)(rb + r_keys + r_ids + (size_t)B * KP * 8);
    hipEvent_t go = nullptr;
    SH_TRY(hipEventCreateWithFlags(&go, hipEventDisableTiming));
    hipError_t e = hipEventRecord(go, st);  // queries / mask written, gather buffers allocated
    int rc = VDB_OK;
    int queued = 0;  // shards whose work (and done event) is queued
    for (int g = 0; g < G && e == hipSuccess && rc == VDB_OK; ++g) {
        Shard& sd = s->sh[g];
        e = hipSetDevice(sd.device);
        if (e == hipSuccess) e = hipStreamWaitEvent(sd.st, go, 0);
        const int64_t mw = (sd.count + 31) / 32;
        const bool masked = mask_root && sd.count > 0;
        const size_t off_m = (qb + 255) & ~size_t(255);
        const size_t off_gm = off_m + (((size_t)(mw + 1) * 4 + 255) & ~size_t(255));
        const size_t off_o = off_gm + (masked && sd.device != root ? (((size_t)gmw * 4 + 255) & ~size_t(255)) : 0);
        char* b = nullptr;
        if (e == hipSuccess) e = hipMallocAsync((void**)&b, off_o + lb * 20 + 1024, sd.st);
        if (e != hipSuccess) break;
        float* q = (float*)b;
        uint32_t* lm = (uint32_t*)(b + off_m);
        float* ls = (float*)(b + off_o);
        int64_t* li = (int64_t*)(b + off_o + lb * 4);
        double* lk = (double*)(b + off_o + lb * 12);
        e = hipMemcpyPeerAsync(q, sd.device, q_root, root, qb, sd.st);
        const uint32_t* md = nullptr;
        if (e == hipSuccess && masked) {
            const uint32_t* gm = mask_root;
            if (sd.device != root) {
                uint32_t* gcopy = (uint32_t*)(b + off_gm);
                e = hipMemcpyPeerAsync(gcopy, sd.device, mask_root, root, (size_t)gmw * 4, sd.st);
                gm = gcopy;
            }
            if (e == hipSuccess) {
                hipLaunchKernelGGL(shard_mask_kernel, dim3((unsigned)((mw + 255) / 256)), dim3(256), 0, sd.st, gm, sd.gid,
                                   sd.count, lm);
                e = hipGetLastError();
            }
            md = lm;
        }
        if (e == hipSuccess) rc = index_search_rows(sd.ix, q, B, k, md, ls, li, lk, sd.st, sd.gid);
        // gather this shard's (key, global id) lists into slot g of the root buffers
        if (e == hipSuccess && rc == VDB_OK) {
            e = hipMemcpyPeerAsync(g_keys + (size_t)g * lb, root, lk, sd.device, lb * 8, sd.st);
            if (e == hipSuccess) e = hipMemcpyPeerAsync(g_ids + (size_t)g * lb, root, li, sd.device, lb * 8, sd.st);
        }
        (void)hipFreeAsync(b, sd.st);  // after this shard's copies (stream order)
        if (e == hipSuccess && rc == VDB_OK) e = hipEventRecord(sd.done, sd.st);
        if (e == hipSuccess && rc == VDB_OK) ++queued;
    }
    (void)hipSetDevice(root);
    // the root waits for every shard that queued work (also on failure, so the gather buffers
    // are freed after the last peer copy into them)
    for (int g = 0; g < queued; ++g) (void)hipStreamWaitEvent(st, s->sh[g].done, 0);
    if (queued < G) {  // a shard failed part-way: its stream may still copy into the buffers
        for (int g = queued; g < G; ++g) {
            (void)hipSetDevice(s->sh[g].device);
            (void)hipStreamSynchronize(s->sh[g].st);
        }
        (void)hipSetDevice(root);
    }
    if (e == hipSuccess && rc == VDB_OK) {
        // list j of query q at j * B * k + q * k
        e = launch_merge_f64_i64(KP, g_keys, g_ids, G, k, k, (int64_t)lb, B, m_keys, m_ids, st);
        if (e == hipSuccess)
            e = launch_finalize_i64(s->metric, m_keys, m_ids, KP, B, nullptr, k, out_scores, out_indices, out_keys, st);
    }
    (void)hipFreeAsync(rb, st);
    (void)hipEventDestroy(go);
    if (rc != VDB_OK) return rc;
    if (e != hipSuccess)
        return fail(e == hipErrorOutOfMemory ? VDB_ERR_OOM : VDB_ERR_HIP,
                    std::string("shard search: ") + hipGetErrorString(e));
    return VDB_OK;
}

}  // namespace

extern "C" {

int32_t vdb_shards_search_device(vdb_shards* s, const float* queries, int32_t B, int32_t k, const uint32_t* row_mask,
                                 float* out_scores, int64_t* out_indices, double* out_keys, void* stream) {
    if (!s) return fail(VDB_ERR_INVALID, "shard set is NULL");
    if (B <= 0) return fail(VDB_ERR_INVALID, "n_queries must be >= 1");
    if (k <= 0 || k > 1024) return fail(VDB_ERR_INVALID, "k must be in [1, 1024]");
    if (!queries || !out_scores || !out_indices) return fail(VDB_ERR_INVALID, "NULL query/output pointer");
    std::shared_lock<std::shared_mutex> lk(s->mu);
    return shards_search_dev(s, queries, B, k, row_mask, out_scores, out_indices, out_keys, (hipStream_t)stream);
}

int32_t vdb_shards_search(vdb_shards* s, const float* queries, int32_t B, int32_t k, const uint32_t* row_mask,
                          float* out_scores, int64_t* out_indices, double* out_keys) {
    if (!s) return fail(VDB_ERR_INVALID, "shard set is NULL");
    if (B <= 0) return fail(VDB_ERR_INVALID, "n_queries must be >= 1");
    if (k <= 0 || k > 1024) return fail(VDB_ERR_INVALID, "k must be in [1, 1024]");
    if (!queries || !out_scores || !out_indices) return fail(VDB_ERR_INVALID, "NULL query/output pointer");
    for (int64_t i = 0; i < (int64_t)B * s->dim; ++i)
        if (!std::isfinite(queries[i])) return fail(VDB_ERR_NONFINITE, "query contains NaN or Inf");
    std::shared_lock<std::shared_mutex> lk(s->mu);
    // host memory: staged on devices[0] and run through the stream-ordered path on a stream of
    // this call, waited for once at the end
    const int root = s->sh[0].device;
    SH_TRY(hipSetDevice(root));
    hipStream_t st = nullptr;
    SH_TRY(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    const size_t qb = (size_t)B * s->dim * 4, lb = (size_t)B * k, mb = row_mask ? (size_t)((s->count + 31) / 32) * 4 : 0;
    char* buf = nullptr;
    hipError_t e = hipMallocAsync((void**)&buf, qb + mb + lb * 20 + 1024, st);
    int rc = VDB_OK;
    if (e == hipSuccess) {
        float* q = (float*)buf;
        uint32_t* m = row_mask ? (uint32_t*)(buf + ((qb + 255) & ~size_t(255))) : nullptr;
        char* o = buf + ((qb + 255) & ~size_t(255)) + ((mb + 255) & ~size_t(255));
        float* os = (float*)o;
        int64_t* oi = (int64_t*)(o + lb * 4);
        double* ok = (double*)(o + lb * 12);
        e = hipMemcpyAsync(q, queries, qb, hipMemcpyHostToDevice, st);
        if (e == hipSuccess && m && mb) e = hipMemcpyAsync(m, row_mask, mb, hipMemcpyHostToDevice, st);
        if (e == hipSuccess) rc = shards_search_dev(s, q, B, k, m, os, oi, ok, st);
        if (e == hipSuccess && rc == VDB_OK) e = hipMemcpyAsync(out_scores, os, lb * 4, hipMemcpyDeviceToHost, st);
        if (e == hipSuccess && rc == VDB_OK) e = hipMemcpyAsync(out_indices, oi, lb * 8, hipMemcpyDeviceToHost, st);
        if (e == hipSuccess && rc == VDB_OK && out_keys)
            e = hipMemcpyAsync(out_keys, ok, lb * 8, hipMemcpyDeviceToHost, st);
        (void)hipFreeAsync(buf, st);
    }
    const hipError_t e2 = hipStreamSynchronize(st);
    (void)hipStreamDestroy(st);
    if (rc != VDB_OK) return rc;
    if (e == hipSuccess) e = e2;
    if (e != hipSuccess)
        return fail(e == hipErrorOutOfMemory ? VDB_ERR_OOM : VDB_ERR_HIP, std::string("shard search: ") + hipGetErrorString(e));
    return VDB_OK;
}

int32_t vdb_shards_get_vectors(vdb_shards* s, int64_t start, int64_t n, float* out_host) {
    if (!s || (!out_host && n > 0)) return fail(VDB_ERR_INVALID, "NULL argument");
    std::shared_lock<std::shared_mutex> lk(s->mu);
    if (start < 0 || n < 0 || start + n > s->count) return fail(VDB_ERR_INVALID, "rows out of range");
    for (Shard& sd : s->sh)
        for (const Piece& pc : sd.pieces) {
            const int64_t a = std::max(start, pc.g0), b = std::min(start + n, pc.g0 + pc.n);
            if (a >= b) continue;
            const int rc = vdb_index_get_vectors(sd.ix, pc.l0 + (a - pc.g0), b - a, out_host + (a - start) * s->dim);
            if (rc != VDB_OK) return rc;
        }
    return VDB_OK;
}

int32_t vdb_shards_clear(vdb_shards* s) {
    if (!s) return fail(VDB_ERR_INVALID, "shard set is NULL");
    std::unique_lock<std::shared_mutex> lk(s->mu);
    for (Shard& sd : s->sh) {
        const int rc = vdb_index_clear(sd.ix);
        if (rc != VDB_OK) return rc;
        sd.pieces.clear();
        sd.count = 0;
    }
    s->count = 0;
    return VDB_OK;
}

int32_t vdb_shards_reserve(vdb_shards* s, int64_t rows) {
    if (!s || rows < 0) return fail(VDB_ERR_INVALID, "bad argument");
    std::unique_lock<std::shared_mutex> lk(s->mu);
    const int64_t per = (rows + (int64_t)s->sh.size() - 1) / (int64_t)s->sh.size();
    for (Shard& sd : s->sh) {
        const int rc = vdb_index_reserve(sd.ix, per);
        if (rc != VDB_OK) return rc;
    }
    return VDB_OK;
}

int32_t vdb_shards_set_param(vdb_shards* s, const char* name, int64_t value) {
    if (!s || !name) return fail(VDB_ERR_INVALID, "NULL argument");
    for (Shard& sd : s->sh) {
        const int rc = vdb_index_set_param(sd.ix, name, value);
        if (rc != VDB_OK) return rc;
    }
    return VDB_OK;
}

int32_t vdb_shards_get_stat(const vdb_shards* s, const char* name, int64_t* value) {
    if (!s || !name || !value) return fail(VDB_ERR_INVALID, "NULL argument");
    const std::string n(name);
    if (n == "count") {
        *value = s->count;
        return VDB_OK;
    }
    if (n == "shards") {
        *value = (int64_t)s->sh.size();
        return VDB_OK;
    }
    int64_t sum = 0;
    for (const Shard& sd : s->sh) {
        int64_t v = 0;
        const int rc = vdb_index_get_stat(sd.ix, name, &v);
        if (rc != VDB_OK) return rc;
        if (n == "precision") {
            *value = v;
            return VDB_OK;
        }
        sum += v;
    }
    *value = sum;  // summed over the shards (searches / queries count once per shard)
    return VDB_OK;
}

int32_t vdb_shards_shard_count(const vdb_shards* s, int32_t shard, int64_t* n) {
    if (!s || !n || shard < 0 || shard >= (int)s->sh.size()) return fail(VDB_ERR_INVALID, "bad argument");
    *n = s->sh[shard].count;
    return VDB_OK;
}

}  // extern "C"
