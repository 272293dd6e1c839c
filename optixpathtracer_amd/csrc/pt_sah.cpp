// pt_sah.cpp — host-side binned-SAH binary BVH over the scene triangles (pt_options.bvh_builder =
// PT_BVH_SAH), handed to the same GPU SAH-optimal BVH4 collapse as the PLOC and LBVH trees
// (pt_build.hip lbvh_build).  Replaces optixAccelBuild (OptixRenderer.cpp:306-456) like the
// other builders: the scene is static, so a slower, top-down build that splits every node at the
// surface-area-heuristic minimum over 64 bins per axis trades pt_create time for fewer node
// visits per ray.  Which tree is traversed never changes an image (the closest hit is the
// (t, index) minimum over acceptable hits for any BVH).
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <vector>

#include "pt_internal.h"

namespace pt {

namespace {

struct Box {
    float lo[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, hi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    // bounds take -0 as +0 (x + 0 under round-to-nearest), as the GPU builder's ordered-int
    // atomics do (pt_sah_gpu.hip f2o): the two builders' boxes agree in the sign of zero
    void grow(const Box& b) {
        for (int a = 0; a < 3; ++a) {
            lo[a] = std::min(lo[a], b.lo[a] + 0.0f);
            hi[a] = std::max(hi[a], b.hi[a] + 0.0f);
        }
    }
    void grow(const float p[3]) {
        for (int a = 0; a < 3; ++a) {
            lo[a] = std::min(lo[a], p[a] + 0.0f);
            hi[a] = std::max(hi[a], p[a] + 0.0f);
        }
    }
    float half_area() const {
        if (lo[0] > hi[0]) return 0.0f;
        const float x = hi[0] - lo[0], y = hi[1] - lo[1], z = hi[2] - lo[2];
        return x * y + y * z + z * x;
    }
};

#ifndef PT_SAH_BINS
#define PT_SAH_BINS 64
#endif
constexpr int kBins = PT_SAH_BINS;  // bins per axis of the split search

// Bin of a centroid coordinate; NaN, below-range and infinite coordinates land in the end bins
// (a float -> int conversion of NaN or of a value past INT_MAX is undefined).
inline int bin_of(float c, float lo, float scale) {
    const float f = (c - lo) * scale;
    if (!(f > 0.0f)) return 0;
    return f < (float)(kBins - 1) ? (int)f : kBins - 1;
}

}  // namespace

// Binary tree over n >= 2 triangles: every internal node splits its range at the binned SAH
// minimum (or, when all centroids coincide, in the middle).  Outputs in the layout of the GPU
// builders: order[k] = original triangle of DFS leaf k, child codes >= 0 internal / ~k leaf k,
// range = the node's DFS leaf range, box = its plain (unpadded) triangle box; root = 0.
void sah_binary_tree(const float4* tri, int n, std::vector<uint32_t>& order, std::vector<int2>& child,
                     std::vector<int2>& range, std::vector<float4>& box) {
    std::vector<Box> tb(n);
    std::vector<float> cen(3 * (size_t)n);
    for (int i = 0; i < n; ++i) {
        for (int v = 0; v < 3; ++v) {
            const float4 p = tri[3 * (size_t)i + v];
            const float q[3] = {p.x, p.y, p.z};
            tb[i].grow(q);
        }
        for (int a = 0; a < 3; ++a) cen[3 * (size_t)i + a] = 0.5f * (tb[i].lo[a] + tb[i].hi[a]);
    }
    order.resize(n);
    for (int i = 0; i < n; ++i) order[i] = (uint32_t)i;
    child.assign(n - 1, make_int2(0, 0));
    range.assign(n - 1, make_int2(0, 0));
    box.assign(2 * (size_t)(n - 1), make_float4(0, 0, 0, 0));
    struct Item {
        int node, begin, end;  // [begin, end) of order, >= 2 triangles
    };
    std::vector<Item> stack;
    stack.push_back({0, 0, n});
    int next_node = 1;
    Box bin_box[3][kBins];
    int bin_cnt[3][kBins];
    float right_area[kBins];
    int right_cnt[kBins];
    while (!stack.empty()) {
        const Item it = stack.back();
        stack.pop_back();
        Box nb, cb;
        for (int k = it.begin; k < it.end; ++k) {
            nb.grow(tb[order[k]]);
            cb.grow(&cen[3 * (size_t)order[k]]);
        }
        box[2 * (size_t)it.node] = make_float4(nb.lo[0], nb.lo[1], nb.lo[2], 0.0f);
        box[2 * (size_t)it.node + 1] = make_float4(nb.hi[0], nb.hi[1], nb.hi[2], 0.0f);
        range[it.node] = make_int2(it.begin, it.end - 1);
        // binned SAH over the three axes
        int best_axis = -1, best_split = 0;
        float best_cost = FLT_MAX;
        for (int a = 0; a < 3; ++a) {
            const float ext = cb.hi[a] - cb.lo[a];
            if (!(ext > 0.0f) || !std::isfinite(ext)) continue;
            const float scale = (float)kBins / ext;
            for (int b = 0; b < kBins; ++b) {
                bin_box[a][b] = Box();
                bin_cnt[a][b] = 0;
            }
            for (int k = it.begin; k < it.end; ++k) {
                const uint32_t t = order[k];
                const int b = bin_of(cen[3 * (size_t)t + a], cb.lo[a], scale);
                bin_box[a][b].grow(tb[t]);
                bin_cnt[a][b]++;
            }
            Box acc;
            int cnt = 0;
            for (int b = kBins - 1; b > 0; --b) {
                acc.grow(bin_box[a][b]);
                cnt += bin_cnt[a][b];
                right_area[b] = acc.half_area();
                right_cnt[b] = cnt;
            }
            acc = Box();
            cnt = 0;
            for (int b = 0; b < kBins - 1; ++b) {  // split between bin b and b + 1
                acc.grow(bin_box[a][b]);
                cnt += bin_cnt[a][b];
                if (cnt == 0 || right_cnt[b + 1] == 0) continue;
                const float cost = acc.half_area() * (float)cnt + right_area[b + 1] * (float)right_cnt[b + 1];
                if (cost < best_cost) {
                    best_cost = cost;
                    best_axis = a;
                    best_split = b;
                }
            }
        }
        int mid;
        if (best_axis < 0) {  // coincident centroids: split the range in the middle
            mid = it.begin + (it.end - it.begin) / 2;
        } else {
            const float scale = (float)kBins / (cb.hi[best_axis] - cb.lo[best_axis]);
            const float lo = cb.lo[best_axis];
            auto left = [&](uint32_t t) {
                return bin_of(cen[3 * (size_t)t + best_axis], lo, scale) <= best_split;
            };
            mid = (int)(std::stable_partition(order.begin() + it.begin, order.begin() + it.end, left) - order.begin());
            if (mid == it.begin || mid == it.end) mid = it.begin + (it.end - it.begin) / 2;
        }
        int codes[2];
        const int b0[2] = {it.begin, mid}, e0[2] = {mid, it.end};
        for (int s = 0; s < 2; ++s) {
            if (e0[s] - b0[s] == 1) {
                codes[s] = ~b0[s];  // a leaf: its DFS position
            } else {
                codes[s] = next_node++;
                stack.push_back({codes[s], b0[s], e0[s]});
            }
        }
        child[it.node] = make_int2(codes[0], codes[1]);
    }
}

// Insertion-based optimisation of a binary tree (after Bittner, Hapala and Havran 2013, "Fast
// insertion-based optimization of bounding volume hierarchies"): the nodes with the largest
// area(node)^2 / (area(child 0) + area(child 1)) are taken out with their parent one at a time,
// and their two children put back where the summed area of the internal nodes -- the part of the
// surface-area cost a move can change, every leaf being one triangle -- grows least
// (branch-and-bound search from the root).  Rounds of 1 % of the nodes repeat while a round
// saves at least 0.1 % of the cost, at most `rounds` times; a move that does not lower the
// cost (a child's place is chosen before its sibling's) is undone.  In and out: the layout of
// sah_binary_tree.  Returns the relative cost reduction (Sponza-class: 8.9 % in 0.13 s).
double sah_reinsert(std::vector<uint32_t>& order, std::vector<int2>& child, std::vector<int2>& range,
                    std::vector<float4>& box, const float4* tri, int rounds) {
    const int n = (int)order.size();
    if (n < 3) return 0.0;
    const int ni = n - 1, nt = 2 * n - 1;  // ids [0, ni) internal, [ni, nt) leaves (DFS position)
    std::vector<int> c0(ni), c1(ni), par(nt, -1);
    std::vector<Box> bx(nt);
    auto uid = [&](int code) { return code >= 0 ? code : ni + ~code; };
    for (int i = 0; i < ni; ++i) {
        c0[i] = uid(child[i].x);
        c1[i] = uid(child[i].y);
        par[c0[i]] = i;
        par[c1[i]] = i;
        bx[i].lo[0] = box[2 * i].x; bx[i].lo[1] = box[2 * i].y; bx[i].lo[2] = box[2 * i].z;
        bx[i].hi[0] = box[2 * i + 1].x; bx[i].hi[1] = box[2 * i + 1].y; bx[i].hi[2] = box[2 * i + 1].z;
    }
    for (int k = 0; k < n; ++k) {
        for (int v = 0; v < 3; ++v) {
            const float4 p = tri[3 * (size_t)order[k] + v];
            const float q[3] = {p.x, p.y, p.z};
            bx[ni + k].grow(q);
        }
    }
    int root = 0;
    auto unite = [](const Box& a, const Box& b) {
        Box u = a;
        u.grow(b);
        return u;
    };
    // every write of a move goes through set() / set_box(), which journal the old value, so a
    // move that does not pay is undone; `total` follows the summed internal-node area
    double total = 0.0;
    std::vector<std::pair<int*, int>> jr_int;
    std::vector<std::pair<int, Box>> jr_box;
    auto set = [&](int& slot, int v) {
        jr_int.push_back({&slot, slot});
        slot = v;
    };
    auto set_box = [&](int x, const Box& b) {
        jr_box.push_back({x, bx[x]});
        if (x < ni) total += (double)b.half_area() - (double)bx[x].half_area();
        bx[x] = b;
    };
    auto refit = [&](int x) {
        for (; x >= 0; x = par[x]) set_box(x, unite(bx[c0[x]], bx[c1[x]]));
    };
    auto cost = [&]() {
        double c = 0.0;
        for (int i = 0; i < ni; ++i) c += bx[i].half_area();
        return c;
    };
    const double c_start = cost();
    if (!std::isfinite(c_start)) return 0.0;  // infinite vertices: no cost to compare, tree as built
    double c_prev = c_start;
    std::vector<std::pair<float, int>> cand;
    std::vector<std::pair<float, int>> heap;  // (induced cost, node), a min-heap
    auto cmp = [](const std::pair<float, int>& a, const std::pair<float, int>& b) { return a.first > b.first; };
    for (int r = 0; r < rounds; ++r) {
        cand.clear();
        for (int i = 0; i < ni; ++i) {
            if (i == root || par[i] == root) continue;
            const float s = bx[c0[i]].half_area() + bx[c1[i]].half_area();
            cand.push_back({s > 0.0f ? bx[i].half_area() / s * bx[i].half_area() : 0.0f, i});
        }
        const size_t k = std::max<size_t>(1, cand.size() / 100);
        if (cand.empty()) break;
        std::partial_sort(cand.begin(), cand.begin() + (long)k, cand.end(),
                          [](const std::pair<float, int>& a, const std::pair<float, int>& b) { return a.first > b.first; });
        for (size_t j = 0; j < k; ++j) {
            const int N = cand[j].second;
            const int P = par[N];
            if (P < 0 || P == root) continue;
            jr_int.clear();
            jr_box.clear();
            total = 0.0;  // the move's change of the summed area
            const int root0 = root;
            // take N and its parent out (the sibling replaces P), then put N's children back one
            // by one, the larger first, with N and P as their new parents
            const int S = c0[P] == N ? c1[P] : c0[P];
            const int G = par[P];
            set(c0[G] == P ? c0[G] : c1[G], S);
            set(par[S], G);
            total -= (double)bx[P].half_area() + (double)bx[N].half_area();
            refit(G);
            int L = c0[N], R = c1[N];
            if (bx[L].half_area() < bx[R].half_area()) std::swap(L, R);
            const int movers[2] = {L, R}, spare[2] = {N, P};
            for (int m = 0; m < 2; ++m) {
                const int M = movers[m], F = spare[m];
                const float aM = bx[M].half_area();
                float best = FLT_MAX;
                int bestX = root;
                heap.clear();
                heap.push_back({0.0f, root});
                while (!heap.empty()) {
                    std::pop_heap(heap.begin(), heap.end(), cmp);
                    const auto [ci, X] = heap.back();
                    heap.pop_back();
                    if (ci + aM >= best) break;
                    const float ax = unite(bx[X], bx[M]).half_area();
                    if (ci + ax < best) {
                        best = ci + ax;
                        bestX = X;
                    }
                    if (X < ni) {
                        const float cc = ci + ax - bx[X].half_area();
                        if (cc + aM < best) {
                            heap.push_back({cc, c0[X]});
                            std::push_heap(heap.begin(), heap.end(), cmp);
                            heap.push_back({cc, c1[X]});
                            std::push_heap(heap.begin(), heap.end(), cmp);
                        }
                    }
                }
                // M becomes bestX's sibling under F (F's box counts again from here)
                const int Q = par[bestX];
                if (Q < 0) root = F;
                else set(c0[Q] == bestX ? c0[Q] : c1[Q], F);
                set(par[F], Q);
                set(c0[F], bestX);
                set(c1[F], M);
                set(par[bestX], F);
                set(par[M], F);
                total += (double)bx[F].half_area();  // set_box below counts the change from here
                refit(F);
            }
            if (total >= 0.0) {  // no gain: undo the move
                for (size_t q = jr_box.size(); q-- > 0;) bx[jr_box[q].first] = jr_box[q].second;
                for (size_t q = jr_int.size(); q-- > 0;) *jr_int[q].first = jr_int[q].second;
                root = root0;
            }
        }
        const double c_now = cost();
        if (c_prev - c_now < 0.001 * c_prev) break;
        c_prev = c_now;
    }
    // re-emit in the builders' layout: internal nodes numbered in DFS pre-order (root 0), leaves in
    // DFS order
    std::vector<uint32_t> order2(n);
    std::vector<int> newid(ni, -1);
    child.assign(ni, make_int2(0, 0));
    range.assign(ni, make_int2(0, 0));
    box.assign(2 * (size_t)ni, make_float4(0, 0, 0, 0));
    int next_id = 0, next_leaf = 0;
    struct Frame {
        int node, stage;
    };
    std::vector<Frame> st;
    newid[root] = next_id++;
    st.push_back({root, 0});
    std::vector<int> first(ni, 0);
    while (!st.empty()) {
        Frame& f = st.back();
        const int x = f.node, id = newid[x];
        if (f.stage == 0) first[x] = next_leaf;
        if (f.stage < 2) {
            const int slot = f.stage++;  // f dangles once a child frame is pushed
            const int c = slot == 0 ? c0[x] : c1[x];
            int code;
            if (c >= ni) {
                order2[next_leaf] = order[c - ni];
                code = ~next_leaf++;
            } else {
                newid[c] = next_id++;
                code = newid[c];
                st.push_back({c, 0});
            }
            if (slot == 0) child[id].x = code; else child[id].y = code;
            continue;
        }
        range[id] = make_int2(first[x], next_leaf - 1);
        box[2 * (size_t)id] = make_float4(bx[x].lo[0], bx[x].lo[1], bx[x].lo[2], 0.0f);
        box[2 * (size_t)id + 1] = make_float4(bx[x].hi[0], bx[x].hi[1], bx[x].hi[2], 0.0f);
        st.pop_back();
    }
    order.swap(order2);
    return c_start > 0.0 ? 1.0 - cost() / c_start : 0.0;
}

}  // namespace pt
