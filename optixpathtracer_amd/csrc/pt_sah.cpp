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
    void grow(const Box& b) {
        for (int a = 0; a < 3; ++a) {
            lo[a] = std::min(lo[a], b.lo[a]);
            hi[a] = std::max(hi[a], b.hi[a]);
        }
    }
    void grow(const float p[3]) {
        for (int a = 0; a < 3; ++a) {
            lo[a] = std::min(lo[a], p[a]);
            hi[a] = std::max(hi[a], p[a]);
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

}  // namespace pt
