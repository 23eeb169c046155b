// vdb_merge_block.h: the block-level merge of sorted per-workgroup top-k lists, shared by
// the merge kernel (vdb_merge.hip) and the device-gated exact fallback (vdb_exact.hip),
// which merges a query's lists in the workgroup that finishes its scan last.
#pragma once
#include "vdb_common.h"

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

// LDS bytes merge_block needs (dynamic; the caller's buffer at smem).
template <typename K, typename I>
__host__ __device__ inline size_t merge_block_lds(int KP) {
    const int cap = WaveTopK<K, I>::capacity(KP) > MERGE_BUF ? WaveTopK<K, I>::capacity(KP) : MERGE_BUF;
    return (size_t)cap * (sizeof(K) + sizeof(I));
}

// The merge of one query's lists (Lq / Iq: list j at j * sj) by one 256-thread workgroup
// into okq / oiq (KP entries); all 256 threads call it.
template <typename K, typename I>
__device__ void merge_block(const K* __restrict__ Lq, const I* __restrict__ Iq, int n_lists, int Lk, int64_t sj,
                            int KP, K* __restrict__ okq, I* __restrict__ oiq, char* smem) {
    // LDS: MERGE_BUF survivors (select path) or the WaveTopK buffer (stream path)
    K* s_k = reinterpret_cast<K*>(smem);
    const int buf_entries = WaveTopK<K, I>::capacity(KP) > MERGE_BUF ? WaveTopK<K, I>::capacity(KP) : MERGE_BUF;
    I* s_i = reinterpret_cast<I*>(smem + (size_t)buf_entries * sizeof(K));
    __shared__ K s_tk;
    __shared__ I s_ti;
    __shared__ int s_cnt;
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
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

}  // namespace vdb
