// bvh.cpp -- per-mesh BLAS for the ACCEL_BVH intersect path.
//
// Binned-SAH 2-wide BVH in model space.  Boxes bound the region the
// reference's triangle test (Renderer.cpp:174-215) can accept -- the
// triangle grown by its u/v tolerances (EPSILON = 0.005 in barycentric
// units) plus a float-rounding pad -- so traversal never prunes a triangle
// the brute-force closest-hit oracle would pick.  Depth is capped at
// kMaxDepth (balanced splits once the budget gets tight, a larger leaf at the
// cap) so the kernels' fixed LDS traversal stack cannot overflow.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "scene.h"

namespace pt {

namespace {

// Leaf size; PT_BVH_LEAF overrides it for build experiments (1..16).
int leaf_max() {
    static const int v = [] {
        const char* e = std::getenv("PT_BVH_LEAF");
        const int x = e ? std::atoi(e) : 2;
        return x >= 1 && x <= 16 ? x : 2;
    }();
    return v;
}
#ifndef PT_BVH_BINS
#define PT_BVH_BINS 16
#endif
constexpr int kBins = PT_BVH_BINS;   // binned-SAH buckets per axis
constexpr int kMaxDepth = kMaxBvhDepth;   // pt_types.h: the kernels' LDS stacks are sized (and asserted) for it

struct Box {
    double lo[3] = {1e300, 1e300, 1e300};
    double hi[3] = {-1e300, -1e300, -1e300};
    void grow(const double* p) {
        for (int k = 0; k < 3; k++) { lo[k] = std::min(lo[k], p[k]); hi[k] = std::max(hi[k], p[k]); }
    }
    void grow(const Box& b) {
        for (int k = 0; k < 3; k++) { lo[k] = std::min(lo[k], b.lo[k]); hi[k] = std::max(hi[k], b.hi[k]); }
    }
    double area() const {
        double d[3];
        for (int k = 0; k < 3; k++) d[k] = std::max(0.0, hi[k] - lo[k]);
        return 2.0 * (d[0] * d[1] + d[1] * d[2] + d[2] * d[0]);
    }
    bool valid() const { return lo[0] <= hi[0]; }
};

struct Ref { int tri; Box box; double c[3]; };

struct Child { Box box; int link; int count; };   // count 0 = inner node, -1 = empty

struct Builder {
    Scene& s;
    std::vector<Ref>& refs;
    double pad;
    Builder(Scene& sc, std::vector<Ref>& r, double p) : s(sc), refs(r), pad(p) {}

    static int ceil_log2(long long v) { int d = 0; while ((1LL << d) < v) d++; return d; }

    Child leaf(int b, int e, const Box& box) {
        Child c;
        c.box = box;
        c.link = (int)s.bvh_tri_order.size();
        c.count = e - b;
        for (int i = b; i < e; i++) s.bvh_tri_order.push_back(refs[i].tri);
        return c;
    }

    Child build(int b, int e, int depth) {
        Box box, cbox;
        for (int i = b; i < e; i++) { box.grow(refs[i].box); cbox.grow(refs[i].c); }
        const int n = e - b;
        const int kLeafMax = leaf_max();
        if (n <= kLeafMax || depth >= kMaxDepth) return leaf(b, e, box);   // depth cap: a (rare) larger leaf
        // Force balanced splits when the remaining depth budget is tight.
        const bool force_median = depth + ceil_log2((n + kLeafMax - 1) / kLeafMax) >= kMaxDepth - 1;
        int axis = 0;
        double ext = -1;
        for (int k = 0; k < 3; k++)
            if (cbox.hi[k] - cbox.lo[k] > ext) { ext = cbox.hi[k] - cbox.lo[k]; axis = k; }
        int mid = -1;
        if (!force_median && ext > 0) {
            double best = 1e300;
            int best_axis = -1, best_bin = -1;
            for (int k = 0; k < 3; k++) {
                double lo = cbox.lo[k], w = cbox.hi[k] - cbox.lo[k];
                if (!(w > 0)) continue;
                Box bins[kBins];
                int cnt[kBins] = {0};
                for (int i = b; i < e; i++) {
                    int bi = (int)((refs[i].c[k] - lo) / w * kBins);
                    bi = std::min(kBins - 1, std::max(0, bi));
                    cnt[bi]++;
                    bins[bi].grow(refs[i].box);
                }
                double la[kBins], ra[kBins];
                int lc[kBins], rc[kBins];
                Box acc; int c = 0;
                for (int i = 0; i < kBins; i++) { acc.grow(bins[i]); c += cnt[i]; la[i] = acc.valid() ? acc.area() : 0; lc[i] = c; }
                acc = Box(); c = 0;
                for (int i = kBins - 1; i >= 0; i--) { acc.grow(bins[i]); c += cnt[i]; ra[i] = acc.valid() ? acc.area() : 0; rc[i] = c; }
                for (int i = 0; i < kBins - 1; i++) {
                    if (lc[i] == 0 || rc[i + 1] == 0) continue;
                    double cost = la[i] * lc[i] + ra[i + 1] * rc[i + 1];
                    if (cost < best) { best = cost; best_axis = k; best_bin = i; }
                }
            }
            if (best_axis >= 0) {
                double lo = cbox.lo[best_axis], w = cbox.hi[best_axis] - cbox.lo[best_axis];
                Ref* p = std::partition(refs.data() + b, refs.data() + e, [&](const Ref& r) {
                    int bi = (int)((r.c[best_axis] - lo) / w * kBins);
                    bi = std::min(kBins - 1, std::max(0, bi));
                    return bi <= best_bin;
                });
                mid = (int)(p - refs.data());
                if (mid == b || mid == e) mid = -1;
            }
        }
        if (mid < 0) {
            mid = b + n / 2;
            std::nth_element(refs.begin() + b, refs.begin() + mid, refs.begin() + e,
                             [&](const Ref& x, const Ref& y) {
                                 if (x.c[axis] != y.c[axis]) return x.c[axis] < y.c[axis];
                                 return x.tri < y.tri;
                             });
        }
        int node = (int)s.bvh_nodes.size();
        s.bvh_nodes.push_back(BvhNode());
        Child L = build(b, mid, depth + 1);
        Child R = build(mid, e, depth + 1);
        store(node, L, R);
        Child c;
        c.box = box;
        c.link = node;
        c.count = 0;
        return c;
    }

    void put(const Box& bx, float* lo, float* hi) {
        for (int k = 0; k < 3; k++) {
            // round outward to float and pad
            float l = (float)(bx.lo[k] - pad), h = (float)(bx.hi[k] + pad);
            if ((double)l > bx.lo[k] - pad) l = std::nextafter(l, -INFINITY);
            if ((double)h < bx.hi[k] + pad) h = std::nextafter(h, INFINITY);
            lo[k] = l; hi[k] = h;
        }
    }

    void store(int node, const Child& L, const Child& R) {
        BvhNode& nd = s.bvh_nodes[node];
        std::memset(&nd, 0, sizeof nd);
        if (L.count >= 0) put(L.box, nd.lo0, nd.hi0);
        if (R.count >= 0) put(R.box, nd.lo1, nd.hi1);
        nd.link0 = L.link; nd.count0 = L.count;
        nd.link1 = R.link; nd.count1 = R.count;
        if (L.count < 0) { for (int k = 0; k < 3; k++) { nd.lo0[k] = 1.0f; nd.hi0[k] = -1.0f; } }
        if (R.count < 0) { for (int k = 0; k < 3; k++) { nd.lo1[k] = 1.0f; nd.hi1[k] = -1.0f; } }
    }
};

}  // namespace

void Scene::buildBvh(int mesh) {
    const Mesh& m = meshes[mesh];
    const int ts = m.triangle_indices.start_index, te = m.triangle_indices.end_index;
    const int n0 = (int)bvh_nodes.size();     // this mesh's nodes are [n0, end)
    std::vector<Ref> refs;
    refs.reserve(te - ts);
    const double e = (double)kEps;
    double diag = 0;
    {
        const BoundingBox& bb = m.bounding_box;
        if (te > ts) {
            double dx = (double)bb.max.x - bb.min.x, dy = (double)bb.max.y - bb.min.y, dz = (double)bb.max.z - bb.min.z;
            diag = std::sqrt(dx * dx + dy * dy + dz * dz);
        }
    }
    for (int t = ts; t < te; t++) {
        const f3 a = vertices[triangles[t].vertex_indices[0]].position;
        const f3 b = vertices[triangles[t].vertex_indices[1]].position;
        const f3 c = vertices[triangles[t].vertex_indices[2]].position;
        const double v0[3] = {a.x, a.y, a.z};
        const double e1[3] = {(double)b.x - a.x, (double)b.y - a.y, (double)b.z - a.z};
        const double e2[3] = {(double)c.x - a.x, (double)c.y - a.y, (double)c.z - a.z};
        // accepted region: u >= -e, v >= -e, u + v <= 1 + e  -> corners
        const double uv[3][2] = {{-e, -e}, {1 + 2 * e, -e}, {-e, 1 + 2 * e}};
        Ref r;
        r.tri = t;
        double cen[3] = {0, 0, 0};
        for (int q = 0; q < 3; q++) {
            double p[3];
            for (int k = 0; k < 3; k++) p[k] = v0[k] + uv[q][0] * e1[k] + uv[q][1] * e2[k];
            r.box.grow(p);
        }
        const double tri_v[3][3] = {{a.x, a.y, a.z}, {b.x, b.y, b.z}, {c.x, c.y, c.z}};
        for (int q = 0; q < 3; q++)
            for (int k = 0; k < 3; k++) cen[k] += tri_v[q][k] / 3.0;
        for (int k = 0; k < 3; k++) r.c[k] = cen[k];
        // non-finite geometry: make the box cover everything
        bool finite = true;
        for (int k = 0; k < 3; k++) finite &= std::isfinite(r.box.lo[k]) && std::isfinite(r.box.hi[k]);
        if (!finite) {
            for (int k = 0; k < 3; k++) { r.box.lo[k] = -3e38; r.box.hi[k] = 3e38; r.c[k] = 0; }
        }
        refs.push_back(r);
    }
    // Rounding pad: 1e-4 of the mesh diagonal (the triangle test's float error
    // is ~1e-7 relative to the ray-to-triangle distance) plus an absolute floor.
    const double pad = 1e-4 * diag + 1e-3;
    Builder B(*this, refs, pad);
    int root;
    if (refs.empty()) {
        root = (int)bvh_nodes.size();
        bvh_nodes.push_back(BvhNode());
        Child E; E.link = -1; E.count = -1;
        B.store(root, E, E);
    } else {
        Child c = B.build(0, (int)refs.size(), 1);
        if (c.count > 0) {
            root = (int)bvh_nodes.size();
            bvh_nodes.push_back(BvhNode());
            Child E; E.link = -1; E.count = -1;
            B.store(root, c, E);
        } else {
            root = c.link;
        }
    }
    mesh_bvh_root[mesh] = relayoutPairs(n0, root);
}

// Node order for the traversal's memory system: the two inner children of a
// node are stored side by side in one 128-byte line (an even node index; a
// padding node keeps the pairing), pairs in depth-first order.  A visit that
// fetches one child's record brings its sibling's, usually visited next, into
// L2 with it.  Only addresses change: boxes, links' targets, traversal order
// and results do not.  PT_BVH_PAIRS=0 keeps the plain pre-order.
int Scene::relayoutPairs(int n0, int root) {
    static const bool on = [] {
        const char* e = std::getenv("PT_BVH_PAIRS");
        return !(e && std::atoi(e) == 0);
    }();
    const int n1 = (int)bvh_nodes.size();
    if (!on || n1 - n0 <= 1) return root;
    std::vector<BvhNode> out;
    out.reserve((size_t)(n1 - n0) * 5 / 4 + 2);
    std::vector<int> nid(n1 - n0, -1);
    auto place = [&](int old) { nid[old - n0] = n0 + (int)out.size(); out.push_back(bvh_nodes[old]); };
    BvhNode pad_node;
    std::memset(&pad_node, 0, sizeof pad_node);
    pad_node.count0 = pad_node.count1 = -1;
    pad_node.link0 = pad_node.link1 = -1;
    for (int k = 0; k < 3; k++) { pad_node.lo0[k] = pad_node.lo1[k] = 1.0f; pad_node.hi0[k] = pad_node.hi1[k] = -1.0f; }
    place(root);
    std::vector<int> st{root};
    while (!st.empty()) {
        const BvhNode nd = bvh_nodes[st.back()];
        st.pop_back();
        const bool in0 = nd.count0 == 0, in1 = nd.count1 == 0;
        if (in0 && in1 && ((n0 + (int)out.size()) & 1)) out.push_back(pad_node);
        if (in0) place(nd.link0);
        if (in1) place(nd.link1);
        if (in1) st.push_back(nd.link1);
        if (in0) st.push_back(nd.link0);
    }
    for (BvhNode& nd : out) {
        if (nd.count0 == 0) nd.link0 = nid[nd.link0 - n0];
        if (nd.count1 == 0) nd.link1 = nid[nd.link1 - n0];
    }
    bvh_nodes.resize(n0);
    bvh_nodes.insert(bvh_nodes.end(), out.begin(), out.end());
    return nid[root - n0];
}

// 4-wide collapse (Bvh4Node): each 4-wide node takes a binary node's children,
// replacing every inner child by that child's own two children, so it holds
// 2..4 slots; inner slots become 4-wide nodes in turn, breadth-first (a node's
// inner children next to each other; a mesh's top levels are its first nodes).
// PT_BVH4_ORDER=1 renumbers each mesh's nodes depth-first instead (pre-order,
// children in slot order: a subtree is one contiguous range; layout experiments).
// Boxes are copied bit for bit.  A leaf's
// stack entry holds its first record relative to the mesh's first leaf record
// (mesh_leaf_base, ModelRec::leaf_base, added back by the traces), so the
// encoding's 2^kLeafCountShift limit is per mesh, not per scene.  A mesh whose
// leaves still do not fit it (a leaf of more than kMaxLeafCount4 triangles, or
// 2^kLeafCountShift leaf records or more in one mesh), or whose nodes would pass
// 2^27 in the scene, gets no 4-wide BLAS (root -1): every BLAS path walks the
// 4-wide nodes and there is no binary fallback, so Renderer::allocateOnGPU then
// refuses the scene for them (grid mode, which needs no BLAS, still runs).
void Scene::buildBvh4() {
    // PT_BVH4_OPEN=0: open the first inner slot instead of the largest (build experiments)
    const char* eo = std::getenv("PT_BVH4_OPEN");
    const bool kOpenLargest = !(eo && std::atoi(eo) == 0);
    const char* ed = std::getenv("PT_BVH4_ORDER");
    const bool kDepthFirst = ed && std::atoi(ed) == 1;
    bvh4_nodes.clear();
    mesh_bvh4_root.assign(meshes.size(), -1);
    mesh_leaf_base.assign(meshes.size(), 0);
    if (bvh_nodes.empty()) return;
    struct Slot { float lo[3], hi[3]; int link, count; };
    auto child = [&](const BvhNode& nd, int c) {
        Slot s;
        for (int k = 0; k < 3; k++) {
            s.lo[k] = c ? nd.lo1[k] : nd.lo0[k];
            s.hi[k] = c ? nd.hi1[k] : nd.hi0[k];
        }
        s.link = c ? nd.link1 : nd.link0;
        s.count = c ? nd.count1 : nd.count0;
        return s;
    };
    for (size_t m = 0; m < meshes.size(); m++) {
        const int root = mesh_bvh_root[m];
        if (root < 0) continue;
        const size_t n0 = bvh4_nodes.size();
        bool fits = true;
        // the mesh's first leaf record: its leaf entries are stored relative to it
        long long base = -1;
        {
            std::vector<int> st{root};
            while (!st.empty()) {
                const BvhNode nd = bvh_nodes[st.back()];
                st.pop_back();
                for (int c = 0; c < 2; c++) {
                    const int cnt = c ? nd.count1 : nd.count0, lk = c ? nd.link1 : nd.link0;
                    if (cnt == 0) st.push_back(lk);
                    else if (cnt > 0 && (base < 0 || lk < base)) base = lk;
                }
            }
        }
        if (base < 0) base = 0;
#if defined(PT_LEAF_REL) && PT_LEAF_REL == 0
        base = 0;                        // absolute leaf links (timing experiments)
#endif
        // make(b): the 4-wide node for binary node b; returns its index
        std::vector<std::pair<int, int>> work;   // (binary node, 4-wide index) still to fill
        auto alloc = [&](int b) {
            const int id = (int)bvh4_nodes.size();
            bvh4_nodes.push_back(Bvh4Node());
            work.push_back({b, id});
            return id;
        };
        const int r4 = alloc(root);
        for (size_t w = 0; w < work.size(); w++) {
            const int b = work[w].first, id = work[w].second;
            // open inner slots, largest surface area first, until four slots are filled
            // (a leaf child leaves room to open a grandchild as well)
            Slot slots[4];
            int ns = 0;
            const BvhNode nd = bvh_nodes[b];
            slots[ns++] = child(nd, 0);
            slots[ns++] = child(nd, 1);
            auto area = [](const Slot& s) {
                const double dx = (double)s.hi[0] - s.lo[0], dy = (double)s.hi[1] - s.lo[1], dz = (double)s.hi[2] - s.lo[2];
                return dx * dy + dy * dz + dz * dx;
            };
            while (ns < 4) {
                int best = -1;
                for (int c = 0; c < ns; c++)
                    if (slots[c].count == 0 && (best < 0 || (kOpenLargest && area(slots[c]) > area(slots[best])))) best = c;
                if (best < 0) break;
                const BvhNode g = bvh_nodes[slots[best].link];
                for (int c = best; c + 1 < ns; c++) slots[c] = slots[c + 1];   // keep the children's order
                ns--;
                slots[ns++] = child(g, 0);
                slots[ns++] = child(g, 1);
            }
            Bvh4Node out;
            std::memset(&out, 0, sizeof out);
            for (int c = 0; c < 4; c++) {
                Slot s;
                if (c < ns) s = slots[c];
                else s.count = -1;
                if (s.count < 0) {   // an empty slot (past the children, or an empty binary child, as in a
                                     // 1-triangle mesh): an inverted infinite box, which every slab test misses
                    for (int k = 0; k < 3; k++) { s.lo[k] = INFINITY; s.hi[k] = -INFINITY; }
                    s.link = -1; s.count = -1;
                }
                if (s.count > 0) {
                    s.link -= (int)base;   // mesh-relative (ModelRec::leaf_base)
                    if (s.count > kMaxLeafCount4 || s.link < 0 || s.link >= (1 << kLeafCountShift)) fits = false;
                }
                out.lox[c] = s.lo[0]; out.loy[c] = s.lo[1]; out.loz[c] = s.lo[2];
                out.hix[c] = s.hi[0]; out.hiy[c] = s.hi[1]; out.hiz[c] = s.hi[2];
                out.count[c] = s.count;
                // inner: binary index -> 4-wide index; leaf: the stack's leaf entry
                out.link[c] = s.count == 0 ? alloc(s.link)
                            : s.count > 0 ? (int)(0x80000000u | ((unsigned)s.count << kLeafCountShift) | (unsigned)s.link)
                                          : s.link;
            }
            bvh4_nodes[id] = out;
        }
        // node << 4 | slot mask: the one-lane traversal's stack entries (bvh4_traverse)
        if (bvh4_nodes.size() >= (size_t)1 << 27) fits = false;
        if (fits && kDepthFirst) {   // renumber [n0, end) in depth-first pre-order
            const size_t n1 = bvh4_nodes.size();
            std::vector<int> nid(n1 - n0, -1);
            std::vector<int> st{r4};
            int next = (int)n0;
            while (!st.empty()) {
                const int b = st.back();
                st.pop_back();
                nid[b - n0] = next++;
                for (int c = 3; c >= 0; c--)
                    if (bvh4_nodes[b].count[c] == 0) st.push_back(bvh4_nodes[b].link[c]);
            }
            std::vector<Bvh4Node> out(n1 - n0);
            for (size_t i = n0; i < n1; i++) {
                Bvh4Node nd = bvh4_nodes[i];
                for (int c = 0; c < 4; c++)
                    if (nd.count[c] == 0) nd.link[c] = nid[nd.link[c] - n0];
                out[nid[i - n0] - n0] = nd;
            }
            std::copy(out.begin(), out.end(), bvh4_nodes.begin() + n0);
        }
        if (fits) {
            mesh_bvh4_root[m] = r4;
            mesh_leaf_base[m] = (int)base;
        } else {
            bvh4_nodes.resize(n0);
        }
    }
}

}  // namespace pt
