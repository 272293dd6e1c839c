// Host check of the binned-SAH builder and its insertion-based refinement (pt_sah.cpp), built by
// tests/test_sah_host.py with hipcc --cuda-host-only (no GPU).  Reads float4 triangles (three
// vertices each, w ignored) from argv[1], builds the binary tree, refines it with argv[2] rounds
// and checks both trees against the layout lbvh_build consumes:
//   - order is a permutation of the triangles;
//   - every internal node but the root and every leaf is some node's child exactly once;
//   - a node's leaf range is its first child's followed directly by its second child's;
//   - a node's box is the union of its children's (leaf: its triangle's vertex box).
// Prints one JSON line: n, the summed internal half-areas before / after, the reported cut.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "pt_internal.h"

namespace {

struct B {
    float lo[3], hi[3];
};

// the builder's Box::grow semantics: std::min / std::max keep the left operand on NaN
B leaf_box(const float4* tri, uint32_t t) {
    B b{{3.402823466e38f, 3.402823466e38f, 3.402823466e38f}, {-3.402823466e38f, -3.402823466e38f, -3.402823466e38f}};
    for (int v = 0; v < 3; ++v) {
        const float4 p = tri[3 * (size_t)t + v];
        const float q[3] = {p.x, p.y, p.z};
        for (int a = 0; a < 3; ++a) {
            b.lo[a] = std::min(b.lo[a], q[a]);
            b.hi[a] = std::max(b.hi[a], q[a]);
        }
    }
    return b;
}

double cost(const std::vector<float4>& box, int ni) {
    double c = 0.0;
    for (int i = 0; i < ni; ++i) {
        const float4 a = box[2 * (size_t)i], b = box[2 * (size_t)i + 1];
        if (a.x > b.x) continue;
        const float x = b.x - a.x, y = b.y - a.y, z = b.z - a.z;
        c += (double)(x * y + y * z + z * x);  // float, as Box::half_area
    }
    return c;
}

int check(const char* what, const float4* tri, int n, const std::vector<uint32_t>& order,
          const std::vector<int2>& child, const std::vector<int2>& range, const std::vector<float4>& box) {
    int bad = 0;
    auto fail = [&](const char* m, long i) {
        if (bad++ < 8) std::fprintf(stderr, "%s: %s at %ld\n", what, m, i);
    };
    const int ni = n - 1;
    if ((int)order.size() != n || (int)child.size() != ni || (int)range.size() != ni || (int)box.size() != 2 * ni) {
        fail("array sizes", 0);
        return bad;
    }
    std::vector<int> seen(n, 0), ref_int(ni, 0), ref_leaf(n, 0);
    for (int k = 0; k < n; ++k) {
        if (order[k] >= (uint32_t)n) fail("order out of range", k);
        else seen[order[k]]++;
    }
    for (int t = 0; t < n; ++t)
        if (seen[t] != 1) fail("triangle not exactly once in order", t);
    auto lo_of = [&](int c) { return c >= 0 ? range[c].x : ~c; };
    auto hi_of = [&](int c) { return c >= 0 ? range[c].y : ~c; };
    auto box_of = [&](int c) {
        if (c < 0) return leaf_box(tri, order[~c]);
        const float4 a = box[2 * (size_t)c], b = box[2 * (size_t)c + 1];
        return B{{a.x, a.y, a.z}, {b.x, b.y, b.z}};
    };
    for (int i = 0; i < ni; ++i) {
        const int cs[2] = {child[i].x, child[i].y};
        for (int c : cs) {
            if (c >= ni || c < -n || c == 0) {
                fail("child code out of range", i);
                return bad;
            }
            if (c > 0) ref_int[c]++;
            else ref_leaf[~c]++;
        }
        if (lo_of(cs[0]) != range[i].x || hi_of(cs[1]) != range[i].y || hi_of(cs[0]) + 1 != lo_of(cs[1]))
            fail("leaf ranges not contiguous", i);
        const B b0 = box_of(cs[0]), b1 = box_of(cs[1]), me = box_of(i);
        for (int a = 0; a < 3; ++a)
            if (me.lo[a] != std::min(b0.lo[a], b1.lo[a]) || me.hi[a] != std::max(b0.hi[a], b1.hi[a]))
                fail("box is not the union of its children", i);
    }
    for (int i = 1; i < ni; ++i)
        if (ref_int[i] != 1) fail("internal node not exactly one node's child", i);
    for (int k = 0; k < n; ++k)
        if (ref_leaf[k] != 1) fail("leaf not exactly one node's child", k);
    return bad;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    FILE* f = std::fopen(argv[1], "rb");
    if (!f) return 2;
    std::fseek(f, 0, SEEK_END);
    const long sz = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    std::vector<float4> tri((size_t)sz / sizeof(float4));
    if (std::fread(tri.data(), sizeof(float4), tri.size(), f) != tri.size()) return 2;
    std::fclose(f);
    const int n = (int)(tri.size() / 3), rounds = std::atoi(argv[2]);
    if (n < 2) return 2;  // lbvh_build takes the SAH branch for n > 1 only
    std::vector<uint32_t> order;
    std::vector<int2> child, range;
    std::vector<float4> box;
    pt::sah_binary_tree(tri.data(), n, order, child, range, box);
    int bad = check("sah", tri.data(), n, order, child, range, box);
    const double c0 = cost(box, n - 1);
    const double cut = pt::sah_reinsert(order, child, range, box, tri.data(), rounds);
    bad += check("reinsert", tri.data(), n, order, child, range, box);
    const double c1 = cost(box, n - 1);
    auto num = [](double v, char* buf) {  // JSON has no inf / nan
        if (std::isfinite(v)) std::snprintf(buf, 32, "%.17g", v);
        else std::snprintf(buf, 32, "null");
        return buf;
    };
    char b0[32], b1[32], b2[32];
    std::printf("{\"n\": %d, \"cost_sah\": %s, \"cost_reinsert\": %s, \"cut\": %s, \"bad\": %d}\n", n,
                num(c0, b0), num(c1, b1), num(cut, b2), bad);
    return bad ? 1 : 0;
}
