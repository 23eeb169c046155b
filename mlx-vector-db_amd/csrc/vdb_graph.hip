// vdb_graph.hip — the graph path (HNSW replacement) on gfx950: beam search over a
// flat neighbour graph, one workgroup per query.
//
// Reference: performance/hnsw_index.py:23-129 (hnswlib; M=16, efC=200, search ef;
// knn_query returns hnswlib distances: cosine -> 1 - cos, l2 -> squared L2) as used
// by service/optimized_vector_store.py:110-145.  Re-laid out MI355X-first
// (DESIGN.md §10): one level of out-degree R (= 2M, hnswlib's level-0 degree) as a
// row-major [N][R] int32 array, so an expansion is one coalesced 128-byte load; the
// upper levels' job (a good start) is done by scoring a spread entry set; the beam
// (sorted), the per-wave expansion results and a visited hash live in LDS.  Each
// iteration expands the best 4 unexpanded beam nodes at once (one per wave): 4x
// fewer dependent hops than one-at-a-time best-first search.
#include "vdb_common.h"
#include "vdb_internal.h"

namespace vdb {

constexpr int GS_WAVES = 4;
constexpr int GS_EF_MAX = 256;
constexpr int GS_R_MAX = 64;
constexpr int GS_VIS = 16384;       // visited hash slots (row + 1; 0 = empty)
constexpr int GS_PROBE = 64;        // linear probes before a node is treated as visited
constexpr int GS_ENT_MAX = 256;
constexpr int GS_MAX_ITERS = 8192;  // hard stop: every wave leaves the loop
constexpr int GS_NR = 4;            // rows scored together by one wave

// Scores of up to NR rows against the query in LDS (fp32; higher = better):
// cosine q_hat . x * inv|x| (q_hat normalised), L2 2 q . x - |x|^2.
template <int METRIC>
__device__ __forceinline__ void wave_scores(const float* __restrict__ qs, const float* __restrict__ X, int G, int D,
                                            const float* __restrict__ rowscale, const int32_t* rows, int nr,
                                            float* out) {
    const int lane = threadIdx.x & 63;
    const int npieces = (D + 3) / 4;
    float acc[GS_NR];
#pragma unroll
    for (int u = 0; u < GS_NR; ++u) acc[u] = 0.0f;
    for (int p = lane; p < npieces; p += 64) {
        f32x4 xv[GS_NR];
#pragma unroll
        for (int u = 0; u < GS_NR; ++u)
            xv[u] = u < nr ? *(const f32x4*)(X + tiled_piece_offset((uint64_t)rows[u], p, G)) : f32x4{0.f, 0.f, 0.f, 0.f};
        const f32x4 qv = *(const f32x4*)(qs + 4 * p);
#pragma unroll
        for (int u = 0; u < GS_NR; ++u)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[u] = fmaf(qv[j], xv[u][j], acc[u]);
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1)
#pragma unroll
        for (int u = 0; u < GS_NR; ++u) acc[u] += __shfl_xor(acc[u], off, 64);
#pragma unroll
    for (int u = 0; u < GS_NR; ++u) {
        if (u < nr) {
            const float rs = rowscale[rows[u]];
            out[u] = METRIC == 0 ? acc[u] * rs : fmaf(2.0f, acc[u], -rs);
        }
    }
}

// visited-set insert: true if `row` was not in the set (and is now)
__device__ __forceinline__ bool visit(uint32_t* vis, int32_t row) {
    const uint32_t key = (uint32_t)row + 1u;
    uint32_t h = ((uint32_t)row * 2654435761u) & (GS_VIS - 1);
    for (int i = 0; i < GS_PROBE; ++i) {
        const uint32_t prev = atomicCAS(&vis[h], 0u, key);
        if (prev == 0u) return true;
        if (prev == key) return false;
        h = (h + 1) & (GS_VIS - 1);
    }
    return false;  // table crowded: treat as visited (never a duplicate in the beam)
}

template <int METRIC>
__global__ void __launch_bounds__(64 * GS_WAVES) graph_search_kernel(GraphSearchArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wv = tid >> 6;
    const int b = blockIdx.x;
    const int Dp4 = (a.D + 3) / 4 * 4;
    float* qs = reinterpret_cast<float*>(smem);                                  // [Dp4]
    uint32_t* vis = reinterpret_cast<uint32_t*>(smem + (size_t)Dp4 * 4);         // [GS_VIS]
    __shared__ float s_bs[2][GS_EF_MAX];
    __shared__ int32_t s_bi[2][GS_EF_MAX];
    __shared__ int s_bx[2][GS_EF_MAX];  // expanded flag
    __shared__ float s_cs[GS_WAVES][GS_R_MAX];
    __shared__ int32_t s_ci[GS_WAVES][GS_R_MAX];
    __shared__ int s_cc[GS_WAVES];
    __shared__ int s_pick[GS_WAVES];
    __shared__ int s_npick, s_bn, s_cur;
    __shared__ float s_qn2;

    // query -> LDS (cosine: normalised in fp32), |q|^2 for the L2 distance
    const float* q = a.Q + (int64_t)b * a.D;
    for (int d = tid; d < Dp4; d += 64 * GS_WAVES) qs[d] = d < a.D ? q[d] : 0.0f;
    for (int i = tid; i < GS_VIS; i += 64 * GS_WAVES) vis[i] = 0u;
    __syncthreads();
    if (wv == 0) {
        float ss = 0.0f;
        for (int d = lane; d < a.D; d += 64) ss = fmaf(qs[d], qs[d], ss);
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) ss += __shfl_xor(ss, off, 64);
        if (lane == 0) s_qn2 = ss;
    }
    __syncthreads();
    if (METRIC == 0) {
        const float inv = 1.0f / fmaxf(sqrtf(s_qn2), 1e-8f);
        for (int d = tid; d < a.D; d += 64 * GS_WAVES) qs[d] *= inv;
    }
    __syncthreads();

    // entry set: scored by all waves, the best min(ef, E) start the beam
    const int E = a.n_entries < GS_ENT_MAX ? a.n_entries : GS_ENT_MAX;
    __shared__ float s_es[GS_ENT_MAX];
    __shared__ int32_t s_ei[GS_ENT_MAX];
    for (int e0 = wv * GS_NR; e0 < E; e0 += GS_WAVES * GS_NR) {
        int32_t rows[GS_NR];
        float sc[GS_NR];
        const int nr = min(GS_NR, E - e0);
#pragma unroll
        for (int u = 0; u < GS_NR; ++u) rows[u] = u < nr ? a.entries[e0 + u] : 0;
        wave_scores<METRIC>(qs, a.X, a.G, a.D, a.rowscale, rows, nr, sc);
        if (lane == 0) {
#pragma unroll
            for (int u = 0; u < GS_NR; ++u)
                if (u < nr) {
                    s_es[e0 + u] = sc[u];
                    s_ei[e0 + u] = rows[u];
                }
        }
    }
    __syncthreads();
    const int ef = a.ef;
    for (int e = tid; e < E; e += 64 * GS_WAVES) {
        const float sv = s_es[e];
        const int32_t iv = s_ei[e];
        int rank = 0;
        for (int j = 0; j < E; ++j) rank += better(s_es[j], (uint32_t)s_ei[j], sv, (uint32_t)iv) ? 1 : 0;
        if (rank < ef) {
            s_bs[0][rank] = sv;
            s_bi[0][rank] = iv;
            s_bx[0][rank] = 0;
        }
        visit(vis, iv);
    }
    if (tid == 0) {
        s_bn = E < ef ? E : ef;
        s_cur = 0;
    }
    __syncthreads();

    int iters = 0;
    while (true) {
        const int cur = s_cur;
        const int bn = s_bn;
        // ---- pick the best GS_WAVES unexpanded beam nodes (beam sorted best first)
        if (wv == 0) {
            int found = 0;
            for (int e0 = 0; e0 < bn && found < GS_WAVES; e0 += 64) {
                const int e = e0 + lane;
                const bool un = e < bn && s_bx[cur][e] == 0;
                const unsigned long long m = __ballot(un);
                const int before = __popcll(m & ((1ull << lane) - 1ull));
                if (un && found + before < GS_WAVES) {
                    s_pick[found + before] = e;
                    s_bx[cur][e] = 1;
                }
                found += __popcll(m);
            }
            if (lane == 0) s_npick = found < GS_WAVES ? found : GS_WAVES;
        }
        __syncthreads();
        const int npick = s_npick;
        if (npick == 0 || ++iters > GS_MAX_ITERS) break;
        // ---- expand: wave w takes pick w
        if (wv < npick) {
            const int32_t node = s_bi[cur][s_pick[wv]];
            const int32_t nb = lane < a.R ? a.nbr[(int64_t)node * a.R + lane] : -1;
            const bool fresh = nb >= 0 && nb < a.n_rows && visit(vis, nb);
            const unsigned long long m = __ballot(fresh);
            const int pos = __popcll(m & ((1ull << lane) - 1ull));
            const int cnt = __popcll(m);
            if (fresh) s_ci[wv][pos] = nb;
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            __builtin_amdgcn_wave_barrier();
            for (int j0 = 0; j0 < cnt; j0 += GS_NR) {
                int32_t rows[GS_NR];
                float sc[GS_NR];
                const int nr = min(GS_NR, cnt - j0);
#pragma unroll
                for (int u = 0; u < GS_NR; ++u) rows[u] = u < nr ? s_ci[wv][j0 + u] : 0;
                wave_scores<METRIC>(qs, a.X, a.G, a.D, a.rowscale, rows, nr, sc);
                if (lane == 0) {
#pragma unroll
                    for (int u = 0; u < GS_NR; ++u)
                        if (u < nr) s_cs[wv][j0 + u] = sc[u];
                }
            }
            if (lane == 0) s_cc[wv] = cnt;
        } else if (lane == 0) {
            s_cc[wv] = 0;
        }
        __syncthreads();
        // ---- merge beam (sorted, bn) + new candidates -> top ef, by rank counting
        const int nxt = cur ^ 1;
        int nnew = 0;
#pragma unroll
        for (int w = 0; w < GS_WAVES; ++w) nnew += s_cc[w];
        const float worst = bn >= ef ? s_bs[cur][bn - 1] : -INFINITY;
        // beam entries: rank = own position + new candidates that beat it
        for (int e = tid; e < bn; e += 64 * GS_WAVES) {
            const float sv = s_bs[cur][e];
            const int32_t iv = s_bi[cur][e];
            int r = e;
            for (int w = 0; w < GS_WAVES; ++w)
                for (int j = 0; j < s_cc[w]; ++j) r += better(s_cs[w][j], (uint32_t)s_ci[w][j], sv, (uint32_t)iv) ? 1 : 0;
            if (r < ef) {
                s_bs[nxt][r] = sv;
                s_bi[nxt][r] = iv;
                s_bx[nxt][r] = s_bx[cur][e];
            }
        }
        // new candidates: rank = beam entries that beat it (binary search) + new ones that beat it
        for (int t = tid; t < GS_WAVES * GS_R_MAX; t += 64 * GS_WAVES) {
            const int w = t / GS_R_MAX, j = t % GS_R_MAX;
            if (j >= s_cc[w]) continue;
            const float sv = s_cs[w][j];
            const int32_t iv = s_ci[w][j];
            if (bn >= ef && !(sv > worst)) continue;  // cannot enter
            int lo = 0, hi = bn;  // first beam position not better than (sv, iv)
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (better(s_bs[cur][mid], (uint32_t)s_bi[cur][mid], sv, (uint32_t)iv)) lo = mid + 1;
                else hi = mid;
            }
            int r = lo;
            for (int w2 = 0; w2 < GS_WAVES; ++w2)
                for (int j2 = 0; j2 < s_cc[w2]; ++j2)
                    r += better(s_cs[w2][j2], (uint32_t)s_ci[w2][j2], sv, (uint32_t)iv) ? 1 : 0;
            if (r < ef) {
                s_bs[nxt][r] = sv;
                s_bi[nxt][r] = iv;
                s_bx[nxt][r] = 0;
            }
        }
        __syncthreads();
        if (tid == 0) {
            s_bn = bn + nnew < ef ? bn + nnew : ef;
            s_cur = nxt;
        }
        __syncthreads();
    }
    // ---- results: top k of the beam, hnswlib distance conventions
    const int cur = s_cur;
    const int bn = s_bn;
    for (int e = tid; e < a.k; e += 64 * GS_WAVES) {
        const size_t o = (size_t)b * a.k + e;
        if (e < bn) {
            const float sv = s_bs[cur][e];
            a.out_lab[o] = (int64_t)s_bi[cur][e];
            a.out_dist[o] = METRIC == 0 ? 1.0f - sv : fmaxf(s_qn2 - sv, 0.0f);
        } else {
            a.out_lab[o] = -1;
            a.out_dist[o] = INFINITY;
        }
    }
    if (tid == 0 && a.stats) atomicAdd(a.stats, (unsigned long long)iters);
}

hipError_t launch_graph_search(int metric, const GraphSearchArgs& a, int nq, hipStream_t st) {
    if (a.R > GS_R_MAX || a.ef > GS_EF_MAX || a.ef < 1 || a.k > a.ef) return hipErrorInvalidValue;
    const size_t lds = (size_t)((a.D + 3) / 4 * 4) * 4 + (size_t)GS_VIS * 4;
    if (metric == 0)
        hipLaunchKernelGGL(graph_search_kernel<0>, dim3(nq), dim3(64 * GS_WAVES), lds, st, a);
    else
        hipLaunchKernelGGL(graph_search_kernel<1>, dim3(nq), dim3(64 * GS_WAVES), lds, st, a);
    return hipGetLastError();
}

}  // namespace vdb
