// vdb_merge.hip: merging sorted per-workgroup / per-shard top-k lists and the
// final result write-out (part of the gfx950 search pipeline, see vdb_scan.hip).
// Built with -ffp-contract=off.
#include "vdb_common.h"
#include "vdb_internal.h"

namespace vdb {

// One workgroup (256 threads) per query.  Inputs: n_lists sorted lists of Lk
// (key, row) entries, element (q, j, e) at q*sq + j*sj + e.  Output: the best KP
// of their union, sorted (key desc, row asc), sentinel padded.
//
// Select path (the common one): T = the KP-th best list HEAD is a lower bound
// on the KP-th best entry overall (those KP heads are distinct rows), so only
// entries not worse than T can be in the result.  Each thread walks its lists
// from the head until an entry is worse than T and appends survivors to LDS;
// one wave sorts them.  Survivors are typically ~KP.  Stream path (heavy ties overflow the buffer, or
// more than 512 lists): one wave streams every entry through WaveTopK.
constexpr int MERGE_BUF = 1024;
constexpr int MERGE_HEADS = 512;

// KP-th best head (key, row) of up to 512 list heads; (-inf, sentinel) if fewer
// than KP lists.
template <typename K, typename I>
__device__ __attribute__((noinline)) void head_threshold(const K* Lq, const I* Iq, int n_lists, int64_t sj, int KP,
                                                         K* tk, I* ti) {
    constexpr int EH = MERGE_HEADS / 64;
    const int lane = threadIdx.x & 63;
    K hv[EH];
    I hx[EH];
#pragma unroll
    for (int i = 0; i < EH; ++i) {
        const int j = i * 64 + lane;
        hv[i] = j < n_lists ? Lq[j * sj] : (K)-INFINITY;
        hx[i] = j < n_lists ? Iq[j * sj] : sentinel_idx<I>();
    }
    wave_sort_desc<K, I, EH>(hv, hx);
    K sel = (K)-INFINITY;
    I seli = sentinel_idx<I>();
#pragma unroll
    for (int i = 0; i < EH; ++i)
        if (i == ((KP - 1) >> 6)) {
            sel = hv[i];
            seli = hx[i];
        }
    sel = shfl_t(sel, (KP - 1) & 63);
    seli = shfl_t(seli, (KP - 1) & 63);
    if (n_lists >= KP && KP <= MERGE_HEADS) {
        *tk = sel;
        *ti = seli;
    } else {
        *tk = (K)-INFINITY;
        *ti = sentinel_idx<I>();
    }
}

// Sort c (<= 64 E) LDS entries with a register network, store the first n_out.
template <typename K, typename I, int E>
__device__ __attribute__((noinline)) void sort_store_prefix(const K* bk, const I* bi, int c, int n_out, K* ok,
                                                            I* oi) {
    const int lane = threadIdx.x & 63;
    K v[E];
    I x[E];
#pragma unroll
    for (int i = 0; i < E; ++i) {
        const int e = i * 64 + lane;
        v[i] = e < c ? bk[e] : (K)-INFINITY;
        x[i] = e < c ? bi[e] : sentinel_idx<I>();
    }
    wave_sort_desc<K, I, E>(v, x);
#pragma unroll
    for (int i = 0; i < E; ++i) {
        const int e = i * 64 + lane;
        if (e < n_out) {
            ok[e] = v[i];
            oi[e] = x[i];
        }
    }
}

template <typename K, typename I>
__global__ void __launch_bounds__(256)
merge_lists_kernel(const K* __restrict__ ls, const I* __restrict__ li, int n_lists, int Lk, int64_t sq, int64_t sj,
                   int KP, K* __restrict__ out_k, I* __restrict__ out_i, const int* __restrict__ qcount) {
    if (qcount && (int)blockIdx.x >= *qcount) return;  // device-gated launch: only the flagged queries
    extern __shared__ __attribute__((aligned(16))) char smem[];
    // LDS: MERGE_BUF survivors (select path) or the WaveTopK buffer (stream path)
    K* s_k = reinterpret_cast<K*>(smem);
    const int buf_entries = WaveTopK<K, I>::capacity(KP) > MERGE_BUF ? WaveTopK<K, I>::capacity(KP) : MERGE_BUF;
    I* s_i = reinterpret_cast<I*>(smem + (size_t)buf_entries * sizeof(K));
    __shared__ K s_tk;
    __shared__ I s_ti;
    __shared__ int s_cnt;
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    const int q = blockIdx.x;
    const K* Lq = ls + q * sq;
    const I* Iq = li + q * sq;
    K* okq = out_k + (size_t)q * KP;
    I* oiq = out_i + (size_t)q * KP;
    const int total = n_lists * Lk;

    if (n_lists <= MERGE_HEADS) {
        if (wv == 0) {
            K tk;
            I ti;
            head_threshold<K, I>(Lq, Iq, n_lists, sj, KP, &tk, &ti);
            if (lane == 0) {
                s_tk = tk;
                s_ti = ti;
                s_cnt = 0;
            }
        }
        __syncthreads();
        const K tk = s_tk;
        const I ti = s_ti;
        // Lists are sorted, so thread t walks lists t, t + 256 from the head and stops
        // at the first entry worse than T: typically one 4-entry batch per list (one
        // round trip), instead of streaming all n_lists * Lk entries.
        for (int j = threadIdx.x; j < n_lists; j += 256) {
            const K* Lj = Lq + j * sj;
            const I* Ij = Iq + j * sj;
            for (int e0 = 0; e0 < Lk; e0 += 4) {
                K kv[4];
                I iv[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const bool in = e0 + u < Lk;
                    kv[u] = in ? Lj[e0 + u] : (K)-INFINITY;
                    iv[u] = in ? Ij[e0 + u] : sentinel_idx<I>();
                }
                bool more = true;
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const bool keep = more && iv[u] != sentinel_idx<I>() && !better(tk, ti, kv[u], iv[u]);
                    if (keep) {
                        const int pos = atomicAdd(&s_cnt, 1);
                        if (pos < MERGE_BUF) {
                            s_k[pos] = kv[u];
                            s_i[pos] = iv[u];
                        }
                    }
                    more = keep;
                }
                if (!more) break;
            }
        }
        __syncthreads();
        const int c = s_cnt;
        if (c <= MERGE_BUF) {
            if (wv == 0) {
                if (c <= 64) {
                    sort_store_prefix<K, I, 1>(s_k, s_i, c, KP, okq, oiq);
                } else if (c <= 128) {
                    sort_store_prefix<K, I, 2>(s_k, s_i, c, KP, okq, oiq);
                } else if (c <= 256) {
                    sort_store_prefix<K, I, 4>(s_k, s_i, c, KP, okq, oiq);
                } else {
                    const int n = pow2_at_least(c);
                    for (int e = c + lane; e < n; e += 64) {
                        s_k[e] = (K)-INFINITY;
                        s_i[e] = sentinel_idx<I>();
                    }
                    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                    wave_lds_sort_desc<K, I>(s_k, s_i, n);
                    for (int e = lane; e < KP; e += 64) {
                        okq[e] = e < c ? s_k[e] : (K)-INFINITY;
                        oiq[e] = e < c ? s_i[e] : sentinel_idx<I>();
                    }
                }
            }
            return;
        }
        __syncthreads();
    }
    // stream path
    if (wv != 0) return;
    WaveTopK<K, I> tk;
    tk.init(s_k, s_i, KP);
    for (int f0 = 0; f0 < total; f0 += 64) {
        const int f = f0 + lane;
        const bool in = f < total;
        const int j = in ? f / Lk : 0, e = in ? f - j * Lk : 0;
        const K kv = in ? Lq[j * sj + e] : (K)-INFINITY;
        const I iv = in ? Iq[j * sj + e] : sentinel_idx<I>();
        tk.offer(in && iv != sentinel_idx<I>(), kv, iv);
    }
    tk.finish();
    for (int e = lane; e < KP; e += 64) {
        okq[e] = s_k[e];
        oiq[e] = s_i[e];
    }
}

template <typename K, typename I>
static hipError_t merge_launch(int KP, const K* lk, const I* li, int n_lists, int Lk, int64_t sq, int64_t sj, int nq,
                               K* ok, I* oi, hipStream_t st, const int* qcount = nullptr) {
    if (KP < 32 || KP > 4096 || (KP & (KP - 1))) return hipErrorInvalidValue;
    const int cap = std::max(WaveTopK<K, I>::capacity(KP), MERGE_BUF);
    const size_t lds = (size_t)cap * (sizeof(K) + sizeof(I));
    hipLaunchKernelGGL((merge_lists_kernel<K, I>), dim3(nq), dim3(256), lds, st, lk, li, n_lists, Lk, sq, sj, KP, ok,
                       oi, qcount);
    return hipGetLastError();
}

hipError_t launch_merge_f32(int KP, const float* ls, const uint32_t* li, int n_lists, int B, float* out_s,
                            uint32_t* out_i, hipStream_t st) {
    return merge_launch<float, uint32_t>(KP, ls, li, n_lists, KP, (int64_t)n_lists * KP, KP, B, out_s, out_i, st);
}

hipError_t launch_merge_f64_u32(int KP, const double* lk, const uint32_t* li, int n_lists, int Lk, int64_t sq,
                                int64_t sj, int nq, double* out_k, uint32_t* out_i, hipStream_t st, const int* qcount) {
    return merge_launch<double, uint32_t>(KP, lk, li, n_lists, Lk, sq, sj, nq, out_k, out_i, st, qcount);
}

hipError_t launch_merge_f64_i64(int KP, const double* lk, const int64_t* li, int n_lists, int Lk, int64_t sq,
                                int64_t sj, int nq, double* out_k, int64_t* out_i, hipStream_t st) {
    return merge_launch<double, int64_t>(KP, lk, li, n_lists, Lk, sq, sj, nq, out_k, out_i, st);
}

// Final results for query rows qmap[q] (or q) from sorted [nq][KP] lists.
template <typename I>
__global__ void __launch_bounds__(256) finalize_kernel(int metric, const double* __restrict__ sk,
                                                       const I* __restrict__ si, int KP, int nq,
                                                       const int* __restrict__ qmap, int k, int64_t index_offset,
                                                       float* __restrict__ out_s, int64_t* __restrict__ out_i,
                                                       double* __restrict__ out_k, const int* __restrict__ qcount,
                                                       const int64_t* __restrict__ row_ids) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= (int64_t)nq * k) return;
    const int qi = (int)(t / k);
    if (qcount && qi >= *qcount) return;  // device-gated launch
    const int e = (int)(t % k);
    const int b = qmap ? qmap[qi] : qi;
    const double key = sk[(size_t)qi * KP + e];
    const I ix = si[(size_t)qi * KP + e];
    const bool valid = sizeof(I) == 8 ? (int64_t)ix >= 0 : (uint32_t)ix != 0xFFFFFFFFu;
    const size_t o = (size_t)b * k + e;
    write_result(metric, key, valid ? global_row(row_ids, (uint64_t)ix, index_offset) : 0, valid && key != -INFINITY,
                 out_s + o, out_i + o, out_k ? out_k + o : nullptr);
}

hipError_t launch_finalize_u32(int metric, const double* sk, const uint32_t* si, int KP, int nq, const int* qmap,
                               int k, int64_t index_offset, float* out_s, int64_t* out_i, double* out_k,
                               hipStream_t st, const int* qcount, const int64_t* row_ids) {
    const int64_t n = (int64_t)nq * k;
    hipLaunchKernelGGL(finalize_kernel<uint32_t>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, metric, sk, si,
                       KP, nq, qmap, k, index_offset, out_s, out_i, out_k, qcount, row_ids);
    return hipGetLastError();
}

hipError_t launch_finalize_i64(int metric, const double* sk, const int64_t* si, int KP, int nq, const int* qmap,
                               int k, float* out_s, int64_t* out_i, double* out_k, hipStream_t st) {
    const int64_t n = (int64_t)nq * k;
    hipLaunchKernelGGL(finalize_kernel<int64_t>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, metric, sk, si,
                       KP, nq, qmap, k, (int64_t)0, out_s, out_i, out_k, (const int*)nullptr, (const int64_t*)nullptr);
    return hipGetLastError();
}

}  // namespace vdb
