// hnsw_cpu.cpp: a CPU HNSW (hnswlib's published algorithm: exponential levels with
// mult = 1/ln(M), greedy descent through the upper levels, best-first search of width
// ef_construction per level, the getNeighborsByHeuristic2 selection, M links per upper
// level and 2M on level 0, re-pruning a neighbour whose list overflows), used only as an
// experiment: is the C5 recall gap (5M x 384 uniform, ef 128) a property of the device
// graph or of the data?  It builds the hnswlib-style graph over the same synthetic rows
// as bench.py (numpy PCG64 is not reproduced here: rows come from a file bench.py writes),
// searches it with hnswlib's own search (searchBaseLayerST at ef after the greedy
// descent), and reports recall@k against exact results read from the same file.
//
//   g++ -O3 -march=native -fopenmp -o hnsw_cpu hnsw_cpu.cpp
//   ./hnsw_cpu data.bin M ef_construction ef_search[,ef2,...] [out_graph.bin]
// data.bin: int64 N, D, B, k; float X[N][D]; float Q[B][D]; int64 gt[B][k] (cosine)
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <queue>
#include <random>
#include <string>
#include <vector>
#include <chrono>
#include <omp.h>

struct Graph {
    int64_t N = 0;
    int D = 0, M = 16, M0 = 32, efc = 200;
    double mult = 0;
    std::vector<float> X;                       // normalised rows
    std::vector<int> level;                     // per node
    std::vector<std::vector<int32_t>> links0;   // level 0
    std::vector<std::vector<std::vector<int32_t>>> upper;  // [node][level-1]
    std::vector<std::mutex> locks;
    std::mutex glock;
    int32_t entry = -1;
    int maxlevel = -1;

    float dist(const float* a, const float* b) const {  // 1 - cos on normalised rows
        float s = 0.f;
        for (int i = 0; i < D; ++i) s += a[i] * b[i];
        return 1.0f - s;
    }
    const float* row(int32_t i) const { return X.data() + (size_t)i * D; }
    std::vector<int32_t>& nbrs(int32_t i, int l) { return l == 0 ? links0[i] : upper[i][l - 1]; }

    using P = std::pair<float, int32_t>;
    // best-first search on level l from the entry set: up to ef nearest (max-heap by dist)
    std::vector<P> search_layer(const float* q, const std::vector<int32_t>& eps, int ef, int l,
                                std::vector<uint32_t>& visited, uint32_t& tag) {
        ++tag;
        std::priority_queue<P, std::vector<P>, std::greater<P>> cand;  // min-heap
        std::priority_queue<P> res;                                     // max-heap
        for (int32_t e : eps) {
            const float d = dist(q, row(e));
            visited[e] = tag;
            cand.push({d, e});
            res.push({d, e});
        }
        while (!cand.empty()) {
            const P c = cand.top();
            if (c.first > res.top().first && (int)res.size() >= ef) break;
            cand.pop();
            std::vector<int32_t> nb;
            {
                std::lock_guard<std::mutex> g(locks[c.second]);
                nb = nbrs(c.second, l);
            }
            for (int32_t n : nb) {
                if (visited[n] == tag) continue;
                visited[n] = tag;
                const float d = dist(q, row(n));
                if ((int)res.size() < ef || d < res.top().first) {
                    cand.push({d, n});
                    res.push({d, n});
                    if ((int)res.size() > ef) res.pop();
                }
            }
        }
        std::vector<P> out;
        while (!res.empty()) {
            out.push_back(res.top());
            res.pop();
        }
        std::reverse(out.begin(), out.end());  // nearest first
        return out;
    }
    // getNeighborsByHeuristic2 over candidates sorted nearest first
    std::vector<int32_t> heuristic(const std::vector<P>& sorted, int m) const {
        std::vector<int32_t> keep;
        for (const P& c : sorted) {
            if ((int)keep.size() >= m) break;
            bool good = true;
            for (int32_t r : keep)
                if (dist(row(c.second), row(r)) < c.first) {
                    good = false;
                    break;
                }
            if (good) keep.push_back(c.second);
        }
        return keep;
    }
    void insert(int32_t i, std::vector<uint32_t>& visited, uint32_t& tag) {
        const int l = level[i];
        int32_t ep;
        int top;
        {
            std::lock_guard<std::mutex> g(glock);
            ep = entry;
            top = maxlevel;
            if (ep < 0) {
                entry = i;
                maxlevel = l;
                return;
            }
        }
        const float* q = row(i);
        float dcur = dist(q, row(ep));
        for (int lc = top; lc > l; --lc) {  // greedy descent
            bool changed = true;
            while (changed) {
                changed = false;
                std::vector<int32_t> nb;
                {
                    std::lock_guard<std::mutex> g(locks[ep]);
                    nb = nbrs(ep, lc);
                }
                for (int32_t n : nb) {
                    const float d = dist(q, row(n));
                    if (d < dcur) {
                        dcur = d;
                        ep = n;
                        changed = true;
                    }
                }
            }
        }
        std::vector<int32_t> eps{ep};
        for (int lc = std::min(l, top); lc >= 0; --lc) {
            std::vector<P> W = search_layer(q, eps, efc, lc, visited, tag);
            const int mmax = lc == 0 ? M0 : M;
            std::vector<int32_t> sel = heuristic(W, M);
            {
                std::lock_guard<std::mutex> g(locks[i]);
                nbrs(i, lc) = sel;
            }
            for (int32_t n : sel) {
                std::lock_guard<std::mutex> g(locks[n]);
                std::vector<int32_t>& nl = nbrs(n, lc);
                if ((int)nl.size() < mmax) {
                    nl.push_back(i);
                } else {  // re-prune n's list with i added
                    std::vector<P> c;
                    c.push_back({dist(row(n), q), i});
                    for (int32_t x : nl) c.push_back({dist(row(n), row(x)), x});
                    std::sort(c.begin(), c.end());
                    nl = heuristic(c, mmax);
                }
            }
            eps.clear();
            for (const P& w : W) eps.push_back(w.second);
        }
        if (l > top) {
            std::lock_guard<std::mutex> g(glock);
            if (l > maxlevel) {
                maxlevel = l;
                entry = i;
            }
        }
    }
    std::vector<P> knn(const float* q, int k, int ef, std::vector<uint32_t>& visited, uint32_t& tag) {
        int32_t ep = entry;
        float dcur = dist(q, row(ep));
        for (int lc = maxlevel; lc > 0; --lc) {
            bool changed = true;
            while (changed) {
                changed = false;
                for (int32_t n : nbrs(ep, lc)) {
                    const float d = dist(q, row(n));
                    if (d < dcur) {
                        dcur = d;
                        ep = n;
                        changed = true;
                    }
                }
            }
        }
        std::vector<P> W = search_layer(q, {ep}, std::max(ef, k), 0, visited, tag);
        if ((int)W.size() > k) W.resize(k);
        return W;
    }
};

static void normalise(float* v, int D) {
    double s = 0;
    for (int i = 0; i < D; ++i) s += (double)v[i] * v[i];
    const float iv = (float)(1.0 / std::max(std::sqrt(s), 1e-8));
    for (int i = 0; i < D; ++i) v[i] *= iv;
}

int main(int argc, char** argv) {
    if (argc < 5) {
        std::fprintf(stderr, "usage: %s data.bin M ef_construction ef_search[,..] [graph_out.bin]\n", argv[0]);
        return 2;
    }
    FILE* f = std::fopen(argv[1], "rb");
    if (!f) return 3;
    int64_t hdr[4];
    if (std::fread(hdr, 8, 4, f) != 4) return 4;
    Graph g;
    g.N = hdr[0];
    g.D = (int)hdr[1];
    const int64_t B = hdr[2], K = hdr[3];
    g.M = std::atoi(argv[2]);
    g.M0 = 2 * g.M;
    g.efc = std::atoi(argv[3]);
    g.mult = 1.0 / std::log((double)g.M);
    g.X.resize((size_t)g.N * g.D);
    std::vector<float> Q((size_t)B * g.D);
    std::vector<int64_t> gt((size_t)B * K);
    if (std::fread(g.X.data(), 4, g.X.size(), f) != g.X.size()) return 5;
    if (std::fread(Q.data(), 4, Q.size(), f) != Q.size()) return 6;
    if (std::fread(gt.data(), 8, gt.size(), f) != gt.size()) return 7;
    std::fclose(f);
    for (int64_t i = 0; i < g.N; ++i) normalise(g.X.data() + (size_t)i * g.D, g.D);
    for (int64_t i = 0; i < B; ++i) normalise(Q.data() + (size_t)i * g.D, g.D);
    g.level.resize(g.N);
    std::mt19937_64 rng(100);  // hnswlib's default level seed
    std::uniform_real_distribution<double> U(0.0, 1.0);
    for (int64_t i = 0; i < g.N; ++i) g.level[i] = (int)(-std::log(std::max(U(rng), 1e-300)) * g.mult);
    g.links0.resize(g.N);
    g.upper.resize(g.N);
    for (int64_t i = 0; i < g.N; ++i) g.upper[i].resize(g.level[i]);
    g.locks = std::vector<std::mutex>(g.N);
    auto t0 = std::chrono::steady_clock::now();
    // the first node alone, then parallel insertion (hnswlib's add_items with num_threads)
    {
        std::vector<uint32_t> vis(g.N, 0);
        uint32_t tag = 0;
        g.insert(0, vis, tag);
    }
    std::atomic<int64_t> done{1};
#pragma omp parallel
    {
        std::vector<uint32_t> vis(g.N, 0);
        uint32_t tag = 0;
#pragma omp for schedule(dynamic, 256)
        for (int64_t i = 1; i < g.N; ++i) {
            g.insert((int32_t)i, vis, tag);
            const int64_t d = ++done;
            if (d % 200000 == 0) {
                const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
                std::fprintf(stderr, "  %lld inserted, %.1f s\n", (long long)d, s);
            }
        }
    }
    const double build_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::printf("{\"N\": %lld, \"D\": %d, \"M\": %d, \"ef_construction\": %d, \"build_s\": %.2f, \"max_level\": %d, "
                "\"threads\": %d",
                (long long)g.N, g.D, g.M, g.efc, build_s, g.maxlevel, omp_get_max_threads());
    std::string efs = argv[4];
    size_t pos = 0;
    std::printf(", \"search\": [");
    bool first = true;
    while (pos < efs.size()) {
        size_t c = efs.find(',', pos);
        if (c == std::string::npos) c = efs.size();
        const int ef = std::atoi(efs.substr(pos, c - pos).c_str());
        pos = c + 1;
        std::vector<uint32_t> vis(g.N, 0);
        uint32_t tag = 0;
        int64_t hit = 0;
        auto s0 = std::chrono::steady_clock::now();
        for (int64_t b = 0; b < B; ++b) {
            std::vector<Graph::P> r = g.knn(Q.data() + (size_t)b * g.D, (int)K, ef, vis, tag);
            for (const auto& p : r)
                for (int64_t j = 0; j < K; ++j)
                    if (gt[(size_t)b * K + j] == p.second) {
                        ++hit;
                        break;
                    }
        }
        const double ss = std::chrono::duration<double>(std::chrono::steady_clock::now() - s0).count();
        std::printf("%s{\"ef\": %d, \"recall\": %.4f, \"ms_per_query_1thread\": %.3f}", first ? "" : ", ", ef,
                    (double)hit / (double)(B * K), ss * 1e3 / B);
        first = false;
    }
    std::printf("]}\n");
    if (argc > 5) {  // level-0 lists [N][M0] (-1 padded) + the upper-level nodes as entries
        FILE* o = std::fopen(argv[5], "wb");
        std::vector<int32_t> nb((size_t)g.N * g.M0, -1);
        for (int64_t i = 0; i < g.N; ++i)
            for (size_t j = 0; j < g.links0[i].size() && (int)j < g.M0; ++j) nb[(size_t)i * g.M0 + j] = g.links0[i][j];
        std::vector<int32_t> ent;
        for (int lv = g.maxlevel; lv >= 1 && ent.size() < 256; --lv)
            for (int64_t i = 0; i < g.N && ent.size() < 256; ++i)
                if (g.level[i] == lv) ent.push_back((int32_t)i);
        const int64_t h[3] = {g.N, g.M0, (int64_t)ent.size()};
        std::fwrite(h, 8, 3, o);
        std::fwrite(nb.data(), 4, nb.size(), o);
        std::fwrite(ent.data(), 4, ent.size(), o);
        std::fclose(o);
    }
    return 0;
}
