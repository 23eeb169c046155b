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
constexpr int GS_RG = 4;            // groups of 8 rows a wave scores per call (32 rows)
constexpr int GS_PC = 12;           // 16-byte pieces per lane and row in flight (12 x 8 lanes = 384 dims)

// Scores of n <= 32 rows (ids[0..n)) of the row-major copy Xr [rows][Dp] against
// the query in LDS (fp32; higher = better): cosine q_hat . x * inv|x| (q_hat
// normalised), L2 2 q . x - |x|^2; written to out[0..n).  Eight lanes per row, so
// every load instruction reads eight whole 128-byte lines; all pieces of all 32
// rows (and their row scales) are requested before the first FMA: one dependent
// HBM round trip per call for D <= 384.
template <int METRIC>
__device__ __forceinline__ void wave_score_rows(const float* __restrict__ qs, const float* __restrict__ Xr, int Dp,
                                                const float* __restrict__ rowscale, const int32_t* ids, int n,
                                                float* out, int lane) {
    const int sub = lane & 7, u0 = lane >> 3;
    int32_t row[GS_RG];
    float rs[GS_RG], acc[GS_RG];
    bool ok[GS_RG];
#pragma unroll
    for (int g = 0; g < GS_RG; ++g) {
        ok[g] = u0 + 8 * g < n;
        row[g] = ok[g] ? ids[u0 + 8 * g] : 0;
        rs[g] = ok[g] ? rowscale[row[g]] : 0.0f;
        acc[g] = 0.0f;
    }
    const int nper = Dp >> 5;
    for (int i0 = 0; i0 < nper; i0 += GS_PC) {
        f32x4 xv[GS_RG][GS_PC];
#pragma unroll
        for (int g = 0; g < GS_RG; ++g)
#pragma unroll
            for (int c = 0; c < GS_PC; ++c)
                xv[g][c] = ok[g] && i0 + c < nper ? *(const f32x4*)(Xr + (size_t)row[g] * Dp + 4 * (sub + 8 * (i0 + c)))
                                                  : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int c = 0; c < GS_PC; ++c) {
            if (i0 + c < nper) {
                const f32x4 qv = *(const f32x4*)(qs + 4 * (sub + 8 * (i0 + c)));
#pragma unroll
                for (int g = 0; g < GS_RG; ++g)
#pragma unroll
                    for (int j = 0; j < 4; ++j) acc[g] = fmaf(qv[j], xv[g][c][j], acc[g]);
            }
        }
    }
#pragma unroll
    for (int off = 4; off >= 1; off >>= 1)
#pragma unroll
        for (int g = 0; g < GS_RG; ++g) acc[g] += __shfl_xor(acc[g], off, 64);
    if (sub == 0) {
#pragma unroll
        for (int g = 0; g < GS_RG; ++g)
            if (ok[g]) out[u0 + 8 * g] = METRIC == 0 ? acc[g] * rs[g] : fmaf(2.0f, acc[g], -rs[g]);
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
    // teams > 1: a.teams workgroups search one query from disjoint entry slices
    // (entry rank r goes to team r mod teams), each with its own beam and visited
    // set; their top-k lists are merged by graph_merge_kernel.  At batch 1 this
    // puts a.teams CUs on the query instead of one.
    const int T = a.teams;
    const int b = blockIdx.x / T;
    const int team = blockIdx.x % T;
    const int Dp = a.Dp;
    float* qs = reinterpret_cast<float*>(smem);                                  // [Dp]
    uint32_t* vis = reinterpret_cast<uint32_t*>(smem + (size_t)Dp * 4);          // [GS_VIS]
    __shared__ float s_bs[2][GS_EF_MAX];
    __shared__ int32_t s_bi[2][GS_EF_MAX];
    __shared__ int s_bx[2][GS_EF_MAX];  // expanded flag
    __shared__ float s_cs[GS_WAVES][GS_R_MAX];
    __shared__ int32_t s_ci[GS_WAVES][GS_R_MAX];
    __shared__ int s_cc[GS_WAVES];
    __shared__ int s_pick[GS_WAVES];
    __shared__ int s_npick, s_bn, s_cur;
    __shared__ float s_qn2;
    __shared__ unsigned s_scored;  // rows scored (entries + fresh neighbours): the "visited" statistic

    // query -> LDS (cosine: normalised in fp32), |q|^2 for the L2 distance
    const float* q = a.Q + (int64_t)b * a.D;
    for (int d = tid; d < Dp; d += 64 * GS_WAVES) qs[d] = d < a.D ? q[d] : 0.0f;
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

    // Entry set.  Up to GS_ENT_MAX entries: every team scores all of them and takes the ranks
    // r with r mod T == team (the teams start from interleaved ranks).  A larger set (round 5):
    // each team scores its own spread, disjoint slice of at most GS_ENT_MAX entries (entry
    // (j T + team) step) and starts from its best -- with T teams the query meets T x 256
    // entries, so on clustered data (a kNN graph has no edges between clusters) some team
    // starts inside the query's cluster.
    const bool sliced = a.n_entries > GS_ENT_MAX;
    const int E = !sliced ? a.n_entries : min(GS_ENT_MAX, (a.n_entries + T - 1) / T);
    const int64_t step = sliced ? max<int64_t>(1, (int64_t)a.n_entries / ((int64_t)T * E)) : 1;
    __shared__ float s_es[GS_ENT_MAX];
    __shared__ int32_t s_ei[GS_ENT_MAX];
    for (int e = tid; e < E; e += 64 * GS_WAVES) {
        const int64_t src = sliced ? ((int64_t)e * T + team) * step : e;
        s_ei[e] = src < a.n_entries ? a.entries[src] : -1;
    }
    __syncthreads();
    const int Ev = sliced ? (int)min<int64_t>(E, ((int64_t)a.n_entries / step - team + T - 1) / T) : E;  // valid slots
    for (int e0 = wv * 32; e0 < Ev; e0 += GS_WAVES * 32) {
        const int n = min(32, Ev - e0);
        wave_score_rows<METRIC>(qs, a.rows, Dp, a.rowscale, s_ei + e0, n, s_es + e0, lane);
    }
    __syncthreads();
    const int ef = a.ef;
    for (int e = tid; e < Ev; e += 64 * GS_WAVES) {
        const float sv = s_es[e];
        const int32_t iv = s_ei[e];
        int rank = 0;
        for (int j = 0; j < Ev; ++j) rank += better(s_es[j], (uint32_t)s_ei[j], sv, (uint32_t)iv) ? 1 : 0;
        if (sliced || rank % T == team) {
            const int pos = sliced ? rank : rank / T;
            if (pos < ef) {
                s_bs[0][pos] = sv;
                s_bi[0][pos] = iv;
                s_bx[0][pos] = 0;
            }
            visit(vis, iv);
        }
    }
    if (tid == 0) {
        const int mine = sliced ? Ev : (E - team + T - 1) / T;
        s_bn = mine < ef ? mine : ef;
        s_cur = 0;
        s_scored = (unsigned)(sliced ? Ev : E);
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
            for (int j0 = 0; j0 < cnt; j0 += 32) {
                const int n = min(32, cnt - j0);
                wave_score_rows<METRIC>(qs, a.rows, Dp, a.rowscale, s_ci[wv] + j0, n, s_cs[wv] + j0, lane);
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            __builtin_amdgcn_wave_barrier();
            // keep only candidates that can enter a full beam (better than its worst)
            const float cs = lane < cnt ? s_cs[wv][lane] : 0.0f;
            const int32_t ci = lane < cnt ? s_ci[wv][lane] : 0;
            const bool enter = lane < cnt && (bn < ef || better(cs, (uint32_t)ci, s_bs[cur][bn - 1], (uint32_t)s_bi[cur][bn - 1]));
            const unsigned long long km = __ballot(enter);
            __builtin_amdgcn_wave_barrier();
            if (enter) {
                const int kp = __popcll(km & ((1ull << lane) - 1ull));
                s_cs[wv][kp] = cs;
                s_ci[wv][kp] = ci;
            }
            const int kept = __popcll(km);
            if (lane == 0) {
                s_cc[wv] = kept;
                atomicAdd(&s_scored, (unsigned)cnt);
            }
        } else if (lane == 0) {
            s_cc[wv] = 0;
        }
        __syncthreads();
        // ---- merge beam (sorted, bn) + new candidates -> top ef, by rank counting
        const int nxt = cur ^ 1;
        int nnew = 0;
#pragma unroll
        for (int w = 0; w < GS_WAVES; ++w) nnew += s_cc[w];
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
    int64_t* out_lab = T > 1 ? a.tmp_lab + (size_t)team * a.k : a.out_lab;  // teams: [b][team][k]
    float* out_dist = T > 1 ? a.tmp_dist + (size_t)team * a.k : a.out_dist;
    for (int e = tid; e < a.k; e += 64 * GS_WAVES) {
        const size_t o = (size_t)b * T * a.k + e;
        if (e < bn) {
            const float sv = s_bs[cur][e];
            out_lab[o] = (int64_t)s_bi[cur][e];
            out_dist[o] = METRIC == 0 ? 1.0f - sv : fmaxf(s_qn2 - sv, 0.0f);
        } else {
            out_lab[o] = -1;
            out_dist[o] = INFINITY;
        }
    }
    if (tid == 0 && a.stats) {
        atomicAdd(a.stats, (unsigned long long)iters);
        atomicAdd(a.stats + 1, (unsigned long long)s_scored);
    }
}

// ---------------------------------------------------------------------------------
// Build: neighbour selection by hnswlib's heuristic (getNeighborsByHeuristic2, the
// selection hnsw_index.py:63-70's add_items runs for every insertion): walk the
// candidates nearest first and keep c unless an already kept r is closer to c than
// the node is (dist(c, r) < dist(c, node)).  One wave per node; the Gram matrix of
// [node, c_1 .. c_63] comes from v_mfma_f32_32x32x2_f32 over the tiled rows (three
// 32x32 tiles, the fourth is the transpose), so every distance the heuristic
// compares is derived from the same fp32 dot products: deterministic, and
// independent of how the candidates were found.
// ---------------------------------------------------------------------------------
constexpr int GP_WAVES = 4;
constexpr int GP_LD = 65;  // Gram row stride in LDS (floats)

template <int METRIC>
__global__ void __launch_bounds__(64 * GP_WAVES) graph_prune_kernel(GraphPruneArgs a) {
    __shared__ float s_gram[GP_WAVES][64 * GP_LD];
    __shared__ int s_ord[GP_WAVES][64];
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    const int64_t it = (int64_t)blockIdx.x * GP_WAVES + wv;  // work item: candidates / output row
    if (it >= a.n_nodes) return;  // wave-uniform; no block barrier below
    const int64_t v = a.nodes ? (int64_t)a.nodes[it] : it;  // the node
    float* gram = s_gram[wv];
    const int32_t* cand = a.cand + it * a.cw;
    // Gram index i: 0 = the node, i >= 1 = candidate i-1 (-1 padded at the tail)
    const int h = lane >> 5, r = lane & 31;
    const int32_t c0 = r == 0 ? -1 : (r - 1 < a.cw ? cand[r - 1] : -1);
    const int32_t c1 = r + 31 < a.cw ? cand[r + 31] : -1;
    const int32_t row0 = r == 0 ? (int32_t)v : (c0 >= 0 ? c0 : (int32_t)v);
    const int32_t row1 = c1 >= 0 ? c1 : (int32_t)v;
    f32x16 t00, t01, t11;
#pragma unroll
    for (int i = 0; i < 16; ++i) t00[i] = t01[i] = t11[i] = 0.0f;
    f32x4 n0 = *(const f32x4*)(a.X + row_piece_offset((uint64_t)row0, h, a.G));
    f32x4 n1 = *(const f32x4*)(a.X + row_piece_offset((uint64_t)row1, h, a.G));
    for (int j = 0; j < a.G; ++j) {
        const f32x4 x0 = n0, x1 = n1;
        if (j + 1 < a.G) {  // next pieces in flight during this step's MFMAs
            n0 = *(const f32x4*)(a.X + row_piece_offset((uint64_t)row0, 2 * j + 2 + h, a.G));
            n1 = *(const f32x4*)(a.X + row_piece_offset((uint64_t)row1, 2 * j + 2 + h, a.G));
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            t00 = __builtin_amdgcn_mfma_f32_32x32x2f32(x0[s], x0[s], t00, 0, 0, 0);
            t01 = __builtin_amdgcn_mfma_f32_32x32x2f32(x0[s], x1[s], t01, 0, 0, 0);
            t11 = __builtin_amdgcn_mfma_f32_32x32x2f32(x1[s], x1[s], t11, 0, 0, 0);
        }
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int m = (i & 3) + 8 * (i >> 2) + 4 * h;  // C/D layout: row m, column r
        gram[m * GP_LD + r] = t00[i];
        gram[m * GP_LD + 32 + r] = t01[i];
        gram[(32 + r) * GP_LD + m] = t01[i];
        gram[(32 + m) * GP_LD + 32 + r] = t11[i];
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    // this lane's Gram index is `lane`
    const int32_t my_row = lane == 0 ? (int32_t)v : (lane < 32 ? c0 : c1);
    const float sc = a.rowscale[my_row >= 0 ? my_row : (int32_t)v];
    const float sc0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sc), 0));  // the node's
    const unsigned long long valid = __ballot(my_row >= 0);
    uint64_t kept = 0, kept_r = 0;  // by lane / by visiting rank
    int nk = 0;
    const float my_d0 = METRIC == 0 ? 1.0f - gram[lane] * sc * sc0 : fmaf(-2.0f, gram[lane], sc + sc0);
    // visiting order: lane order (candidates arrive nearest first, -1 padded at the tail) or,
    // with a.sort, by (distance to the node, lane) computed here (candidate pools of unknown
    // order: incremental insertion, vdb_graph_add)
    int* ord = s_ord[wv];
    int nvalid = 0, my_rank = lane - 1;
    if (a.sort) {
        nvalid = __popcll(valid & ~1ull);
        int rank = 0;
        for (int c2 = 1; c2 < 64; ++c2) {
            const float d2 = __shfl(my_d0, c2, 64);
            rank += (((valid >> c2) & 1ull) && (d2 < my_d0 || (d2 == my_d0 && c2 < lane))) ? 1 : 0;
        }
        my_rank = rank;
        if (lane >= 1 && ((valid >> lane) & 1ull)) ord[rank] = lane;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
    } else {
        while (nvalid < 63 && ((valid >> (nvalid + 1)) & 1ull)) ++nvalid;
    }
    for (int j = 0; j < nvalid && nk < a.limit; ++j) {
        const int c = a.sort ? ord[j] : j + 1;
        const float g = gram[c * GP_LD + lane];
        const float scc = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sc), c));
        const float d0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(my_d0), c));
        const float dcr = METRIC == 0 ? 1.0f - g * scc * sc : fmaf(-2.0f, g, scc + sc);
        const bool bad = ((kept >> lane) & 1ull) && dcr < d0;
        if (__ballot(bad) == 0ull) {
            kept |= 1ull << c;
            kept_r |= 1ull << j;
            ++nk;
        }
    }
    if (a.fill) {  // hnswlib keepPrunedConnections: top up with the nearest pruned ones
        for (int j = 0; j < nvalid && nk < a.limit; ++j) {
            const int c = a.sort ? ord[j] : j + 1;
            if (!((kept >> c) & 1ull)) {
                kept |= 1ull << c;
                kept_r |= 1ull << j;
                ++nk;
            }
        }
    }
    const bool mine = lane >= 1 && ((kept >> lane) & 1ull);
    const int pos = __popcll(kept_r & ((1ull << (my_rank < 0 ? 0 : my_rank)) - 1ull));  // nearest first
    int32_t* on = a.out_nbr + it * a.rw;
    float* od = a.out_dist + it * a.rw;
    if (mine) {
        on[pos] = my_row;
        od[pos] = my_d0;
    }
    for (int i = nk + lane; i < a.rw; i += 64) {
        on[i] = -1;
        od[i] = INFINITY;
    }
}

hipError_t launch_graph_prune(int metric, const GraphPruneArgs& a, hipStream_t st) {
    if (a.cw < 1 || a.cw > 63 || a.limit < 1 || a.limit > a.rw || a.rw > 64) return hipErrorInvalidValue;
    if (a.n_nodes <= 0) return hipSuccess;
    const dim3 grid((unsigned)((a.n_nodes + GP_WAVES - 1) / GP_WAVES));
    if (metric == 0)
        hipLaunchKernelGGL(graph_prune_kernel<0>, grid, dim3(64 * GP_WAVES), 0, st, a);
    else
        hipLaunchKernelGGL(graph_prune_kernel<1>, grid, dim3(64 * GP_WAVES), 0, st, a);
    return hipGetLastError();
}

// nbr[ids[i]][*] = rows[i][*]: one thread per entry.
__global__ void graph_scatter_kernel(int32_t* __restrict__ nbr, int R, const int32_t* __restrict__ ids,
                                     const int32_t* __restrict__ rows, int64_t n) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n * R) return;
    const int64_t i = t / R;
    nbr[(int64_t)ids[i] * R + (t - i * R)] = rows[t];
}

hipError_t launch_graph_scatter(int32_t* nbr, int R, const int32_t* ids, const int32_t* rows, int64_t n,
                                hipStream_t st) {
    if (n <= 0) return hipSuccess;
    const int64_t total = n * R;
    hipLaunchKernelGGL(graph_scatter_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, nbr, R, ids, rows,
                       n);
    return hipGetLastError();
}

// Teams' lists [b][T][k] (distance ascending) -> top k distinct rows by (distance,
// row).  A row found by several teams carries the same distance in each (same
// arithmetic), so "the next pair strictly after the last one taken" skips copies.
constexpr int64_t kNoLabel = 0x7FFFFFFFFFFFFFFFll;

__global__ void __launch_bounds__(64) graph_merge_kernel(const int64_t* __restrict__ tl, const float* __restrict__ td,
                                                         int T, int k, int64_t* __restrict__ out_lab,
                                                         float* __restrict__ out_dist) {
    const int b = blockIdx.x;
    const int lane = threadIdx.x;
    const int n = T * k;
    const int64_t* L = tl + (size_t)b * n;
    const float* Dd = td + (size_t)b * n;
    float last_d = -INFINITY;
    int64_t last_l = -1;  // labels are >= 0
    for (int e = 0; e < k; ++e) {
        float bd = INFINITY;
        int64_t bl = kNoLabel;
        for (int i = lane; i < n; i += 64) {
            const float d = Dd[i];
            const int64_t l = L[i];
            if (l < 0) continue;
            const bool after = d > last_d || (d == last_d && l > last_l);
            const bool before = d < bd || (d == bd && l < bl);
            if (after && before) {
                bd = d;
                bl = l;
            }
        }
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            const float od = __shfl_xor(bd, off, 64);
            const int64_t ol = __shfl_xor(bl, off, 64);
            if (od < bd || (od == bd && ol < bl)) {
                bd = od;
                bl = ol;
            }
        }
        if (lane == 0) {
            out_lab[(size_t)b * k + e] = bl == kNoLabel ? -1 : bl;
            out_dist[(size_t)b * k + e] = bl == kNoLabel ? INFINITY : bd;
        }
        last_d = bd;
        last_l = bl;
    }
}

hipError_t launch_graph_search(int metric, const GraphSearchArgs& a, int nq, hipStream_t st) {
    if (a.R > GS_R_MAX || a.ef > GS_EF_MAX || a.ef < 1 || a.k > a.ef) return hipErrorInvalidValue;
    if (a.teams < 1 || a.teams > GS_ENT_MAX || (a.teams > 1 && (!a.tmp_lab || !a.tmp_dist))) return hipErrorInvalidValue;
    if (a.Dp % 32 || a.Dp < a.D) return hipErrorInvalidValue;
    const size_t lds = (size_t)a.Dp * 4 + (size_t)GS_VIS * 4;
    const dim3 grid((unsigned)nq * a.teams);
    if (metric == 0)
        hipLaunchKernelGGL(graph_search_kernel<0>, grid, dim3(64 * GS_WAVES), lds, st, a);
    else
        hipLaunchKernelGGL(graph_search_kernel<1>, grid, dim3(64 * GS_WAVES), lds, st, a);
    if (a.teams > 1) {
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(graph_merge_kernel, dim3(nq), dim3(64), 0, st, a.tmp_lab, a.tmp_dist, a.teams, a.k,
                           a.out_lab, a.out_dist);
    }
    return hipGetLastError();
}

}  // namespace vdb
