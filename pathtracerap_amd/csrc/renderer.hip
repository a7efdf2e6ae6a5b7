// renderer.hip -- gfx950 kernels + Renderer host code.
//
// Per iteration (one sample per pixel, Renderer.cpp:582-644):
//   bounce 0 : k_bounce<first>  -- camera ray + cached primary hit -> shade ->
//              compact survivors (block-local, stable) / accumulate the dead
//   scan     : k_scan           -- one workgroup: exclusive scan of the block
//              survivor counts -> dense slot numbering for the next bounce
//   bounce b : k_sort_hist / k_sort_prefix / k_sort_scatter (grid_fast) -- claim
//              order of the live rays by a (origin, direction) key;
//              k_trace_gf / k_trace_bvh -- persistent trace of every live slot
//              into the hit buffer (k_trace_deferred: overflowed hit sets);
//              k_bounce<rest, hitbuf> -- gather ray + hit (slot j -> source via
//              the scan), shade, compact / accumulate
//              (PT_GF_SPLIT=0 / PT_TRACE_SPLIT=0: the fused k_bounce<rest, accel>)
// Iterations run `pipelines` at a time on their own streams (Renderer::renderLoop);
// with more than one, terminated rays write a per-pipeline contribution buffer
// that k_merge adds to the image in iteration order.
// The dense slot j of a ray at bounce b equals its index in the reference's
// thrust::stable_partition'ed ray pool, so the RNG seed
// makeSeededRandomEngine(iter, j, remaining_bounces) -- and hence every
// sample -- is identical to the reference algorithm's.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>

#include "renderer.h"

#pragma clang fp contract(off)

namespace pt {

constexpr int kBlock = 256;
#ifndef PT_STACK
#define PT_STACK 24
#endif
#ifndef PT_HITCAP
#define PT_HITCAP 6
#endif
#ifndef PT_CERT_MODE
#define PT_CERT_MODE 1        // k_trace_gf main launch's walk decision: 0 walk_certify only, 1 walk_certify_fast
                              // first, 2 walk_certify_fast only (the rest goes to the tail launch's exact walk)
#endif
#ifndef PT_TRACE_STATS
#define PT_TRACE_STATS 0      // 1: diagnostic counters / timing ablations (PT_DEBUG_ABLATE); cost registers
#endif
#ifndef PT_MINWAVES
#define PT_MINWAVES 5
#endif
#ifndef PT_SEL_MASK
#define PT_SEL_MASK 1         // k_trace_gf main launch: select steps jump over models a fresh ray's mask rules out
#endif
#ifndef PT_NODE_MINLANES
#define PT_NODE_MINLANES 8    // k_trace_gf: the wave leaves a node step once fewer lanes than this are still at a node
#endif
#ifndef PT_NODE_STEP_1P
#define PT_NODE_STEP_1P 4     // k_trace_gf in-place variant (one pipeline, F & 16): node visits per node step
#endif
#ifndef PT_NODE_STEP
#define PT_NODE_STEP 8        // k_trace_gf: node visits per node step (lanes still at an inner node go on)
#endif
constexpr int kAccelHitBuffer = 3;   // k_bounce template value: hits come from k_trace_bvh
constexpr int kStack = PT_STACK;   // BVH traversal stack entries per lane (LDS)
// k_trace_bvh, k_trace_deferred and the one-lane paths push at most one sibling per
// BLAS level and have no spill path: a smaller stack would overwrite other lanes' LDS
static_assert(kStack >= kMaxBvhDepth + 1, "PT_STACK must hold a full BLAS path (pt_types.h kMaxBvhDepth + 1)");
constexpr int kSortBits = 12, kSortBins = 1 << kSortBits;   // ray sort key (k_sort_hist / k_sort_scatter)
#ifndef PT_SORT_WG
#define PT_SORT_WG 512
#endif
#ifndef PT_SCAN_WG
#define PT_SCAN_WG 512
#endif
#ifndef PT_DEFER_WGS
#define PT_DEFER_WGS 64
#endif
// Sort / scan workgroups stay small: at 16 pipelines the persistent traces hold
// nearly every wave slot, and a workgroup only starts once a CU has room for all
// of its waves and LDS at once (1024-lane ones starved for hundreds of us).
constexpr int kSortWG = PT_SORT_WG, kSortPer = 4096 / PT_SORT_WG;   // source indices per sort workgroup: 4096
constexpr int kScanWG = PT_SCAN_WG, kScanPer = 8;                   // k_scan: one workgroup, tiles of 2048 counts

// ---------------------------------------------------------------------------
// Device helpers
// ---------------------------------------------------------------------------
struct Hit { float dist; f3 n; int model; };

// computeRayBoundingBoxIntersection (Renderer.cpp:150-170)
__device__ __forceinline__ bool slab_ref(const float* bb, f3 o, f3 d, f3 inv, float& t) {
    float t1 = d.x == 0.0f ? kFMin : (bb[0] - o.x) * inv.x;
    float t2 = d.x == 0.0f ? kFMax : (bb[3] - o.x) * inv.x;
    float t3 = d.y == 0.0f ? kFMin : (bb[1] - o.y) * inv.y;
    float t4 = d.y == 0.0f ? kFMax : (bb[4] - o.y) * inv.y;
    float t5 = d.z == 0.0f ? kFMin : (bb[2] - o.z) * inv.z;
    float t6 = d.z == 0.0f ? kFMax : (bb[5] - o.z) * inv.z;
    float tmin = fmaxf(fmaxf(fminf(t1, t2), fminf(t3, t4)), fminf(t5, t6));
    float tmax = fminf(fminf(fmaxf(t1, t2), fmaxf(t3, t4)), fmaxf(t5, t6));
    if (tmax < 0 || tmin > tmax) return false;
    t = tmin;
    return true;
}

// computeRayTriangleIntersection (Renderer.cpp:174-215) on a precomputed
// record (v0, e1 = v1 - v0, e2 = v2 - v0).  Returns true when the reference
// test passes; *t_out is the hit distance.  Before paying for the IEEE
// division, u, v, u+v and t are screened against the tolerances widened from
// 0.005 to 0.0052 using numerators scaled by |det| (no division): a test that
// fails the screen fails the exact test too (the screen's rounding error is
// ~1e-7 relative against a 4e-5 margin), so the exact float sequence below
// decides every remaining case exactly as the reference does.
__device__ __forceinline__ bool tri_test_rec(const float4 A, const float4 B, const float4 C, f3 o, f3 d, float& t_out) {
    // Conditions combined with `&` (same comparisons, same NaN behaviour as the
    // early returns): one branch into the exact test instead of one per
    // condition -- the traces are issue-bound, and every divergent early return
    // cost a handful of scalar exec-mask instructions.
    const f3 v0 = mk3(A.x, A.y, A.z), e1 = mk3(B.x, B.y, B.z), e2 = mk3(C.x, C.y, C.z);
    f3 pvec = cross(d, e2);
    float det = dot(e1, pvec);
    f3 tvec = o - v0;
    const float a = dot(tvec, pvec);
    const float sg = det > 0.0f ? 1.0f : -1.0f;
    const float D = det * sg;
    const float as = a * sg;
    f3 qvec = cross(tvec, e1);
    const float b = dot(d, qvec);
    const float bs = b * sg;
    const float c = dot(e2, qvec);
    const bool screen = !(absr(det - 0.0f) < kEps) &
                        !(as < -0.0052f * D) & !(as > 1.0052f * D) &            // u certainly out
                        !(bs < -0.0052f * D) & !((as + bs) > 1.0052f * D) &     // v or u+v certainly out
                        !(c * sg < -0.0052f * D);                               // t certainly < -eps
    if (!screen) return false;
    float inv_det = 1 / det;
    float u = a * inv_det;
    float v = b * inv_det;
    float t = c * inv_det;
    const bool hit = !(u < 0.0f - kEps) & !(u > 1.0f + kEps) & !(v < 0.0f - kEps) & !(u + v > 1.0f + kEps) &
                     !(t < 0.0f - kEps);
    if (hit) t_out = t;
    return hit;
}

__device__ __forceinline__ bool tri_test(const float4* __restrict__ tg, int it, f3 o, f3 d, float& t_out) {
    return tri_test_rec(tg[3 * it + 0], tg[3 * it + 1], tg[3 * it + 2], o, d, t_out);
}

// computeRayGridIntersection (Renderer.cpp:238-360): 3D-DDA over the model's
// uniform grid, stop 3 voxels past the last voxel that produced a hit.
__device__ bool grid_closest(const KParams& p, const ModelRec& M, f3 o, f3 d, f3 inv, float& best, int& best_tri) {
    const int GX = p.gdim[0], GY = p.gdim[1], GZ = p.gdim[2];
    float t_box;
    if (!slab_ref(M.bbox, o, d, inv, t_box)) return false;
    f3 pt = o + d * t_box;
    if ((pt.x - M.bbox[0]) < -kEps || (pt.y - M.bbox[1]) < -kEps || (pt.z - M.bbox[2]) < -kEps) return false;
    int ix = f2i_sat(absr(pt.x - M.bbox[0] + kEps) / M.vw[0]);
    int iy = f2i_sat(absr(pt.y - M.bbox[1] + kEps) / M.vw[1]);
    int iz = f2i_sat(absr(pt.z - M.bbox[2] + kEps) / M.vw[2]);
    ix = ix < 0 ? 0 : (ix > GX - 1 ? GX - 1 : ix);
    iy = iy < 0 ? 0 : (iy > GY - 1 ? GY - 1 : iy);
    iz = iz < 0 ? 0 : (iz > GZ - 1 ? GZ - 1 : iz);
    f3 tmax = mk3(kFMax, kFMax, kFMax), delta = mk3(kFMax, kFMax, kFMax);
    const int sx = d.x > 0.0f ? 1 : -1, sy = d.y > 0.0f ? 1 : -1, sz = d.z > 0.0f ? 1 : -1;
    const int ox = d.x > 0.0f ? GX : -1, oy = d.y > 0.0f ? GY : -1, oz = d.z > 0.0f ? GZ : -1;
    const int nx = d.x > 0.0f ? ix + 1 : ix, ny = d.y > 0.0f ? iy + 1 : iy, nz = d.z > 0.0f ? iz + 1 : iz;
    const float px = M.bbox[0] + (float)nx * M.vw[0];
    const float py = M.bbox[1] + (float)ny * M.vw[1];
    const float pz = M.bbox[2] + (float)nz * M.vw[2];
    if (d.x != 0) { delta.x = absr(M.vw[0] * inv.x); tmax.x = (px - pt.x) * inv.x; }
    if (d.y != 0) { delta.y = absr(M.vw[1] * inv.y); tmax.y = (py - pt.y) * inv.y; }
    if (d.z != 0) { delta.z = absr(M.vw[2] * inv.z); tmax.z = (pz - pt.z) * inv.z; }
    int cx = 0, cy = 0, cz = 0;
    bool hit = false;
    const int plane = GX * GY;
    for (;;) {
        const int2 vr = p.voxels[M.vox_start + ix + iy * GX + iz * plane];
        bool vhit = false;
        for (int i = vr.x; i < vr.y; i++) {
            const int it = p.per_voxel[i];
            float t;
            if (tri_test(p.tri_geom, it, o, d, t)) {
                vhit = true;
                if (best > t) { best = t; best_tri = it; }
            }
        }
        if (vhit) { cx = ix; cy = iy; cz = iz; hit = true; }
        if (hit && (iabs(cx - ix) > 2 || iabs(cy - iy) > 2 || iabs(cz - iz) > 2)) return true;
        if (tmax.x < tmax.y && tmax.x < tmax.z) {
            ix += sx;
            if (ix == ox || tmax.x >= kFMax) return hit;
            tmax.x += delta.x;
        } else if (tmax.y < tmax.z) {
            iy += sy;
            if (iy == oy || tmax.y >= kFMax) return hit;
            tmax.y += delta.y;
        } else {
            iz += sz;
            if (iz == oz || tmax.z >= kFMax) return hit;
            tmax.z += delta.z;
        }
    }
}

// Inverse direction for node tests: clamped to +-1e30 so the FMA form never
// meets inf * 0 or inf - inf (a zero direction component stays a huge slope).
// Slopes for the instance culling are correctly rounded divisions (hardware
// reciprocals measured neutral in round 3; DESIGN.md "Pruned variants").
__device__ __forceinline__ f3 cull_inv(f3 d) {
    return mk3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
}
__device__ __forceinline__ f3 node_inv(f3 inv) {
    return mk3(fminf(fmaxf(inv.x, -1e30f), 1e30f), fminf(fmaxf(inv.y, -1e30f), 1e30f), fminf(fmaxf(inv.z, -1e30f), 1e30f));
}

// Conservative slab test for BVH node boxes (boxes are padded at build time,
// so the test need not follow the reference's rounding: the FMA form
// lo * inv - o * inv is used, with o * inv hoisted per traversal).
__device__ __forceinline__ void node_slab(const float* lo, const float* hi, f3 o, f3 inv, float& tn, float& tf) {
    const f3 oi = o * inv;   // recomputed per call; the compiler hoists it out of the traversal loop
    float a0 = __builtin_fmaf(lo[0], inv.x, -oi.x), b0 = __builtin_fmaf(hi[0], inv.x, -oi.x);
    float a1 = __builtin_fmaf(lo[1], inv.y, -oi.y), b1 = __builtin_fmaf(hi[1], inv.y, -oi.y);
    float a2 = __builtin_fmaf(lo[2], inv.z, -oi.z), b2 = __builtin_fmaf(hi[2], inv.z, -oi.z);
    tn = fmaxf(fmaxf(fminf(a0, b0), fminf(a1, b1)), fminf(a2, b2));
    tf = fminf(fminf(fmaxf(a0, b0), fmaxf(a1, b1)), fmaxf(a2, b2));
}

// One-lane traversal of a mesh's 4-wide BLAS (Bvh4Node), for the per-ray paths:
// k_primary, k_trace_deferred, the fused bounce, k_intersect_rays and
// k_certify_check (the persistent traces have their own phase-scheduled node
// steps).  A visit tests the slots of `todo` with node_slab's values against
// bound() (the same fma entries / exits as every other node test), runs the
// triangles of hit leaf children at once (leaf(first, count), first absolute:
// ModelRec::leaf_base + the link's mesh-relative first), and descends into the
// nearest hit inner child.  Its other hit inner children stay on the stack as
// ONE entry, node << 4 | their slot mask, re-tested against the bound when
// popped, so the stack holds at most one entry per level of the path (<= the
// binary depth cap, kMaxBvhDepth + 1 nodes, < kStack) and needs no spill area.
// Empty slots (count -1) are skipped; the traversal visits every node a binary
// traversal with the same pruning rule visits, so the triangles tested are a
// superset of those the bound requires.  leaf() returns false to abort (hit-set
// overflow); the function then returns false.
template <int STRIDE, typename Leaf, typename Bound>
__device__ __forceinline__ bool bvh4_traverse(const KParams& p, const ModelRec& M, f3 o, f3 ninv,
                                              int* __restrict__ stack, Leaf&& leaf, Bound&& bound, unsigned& nvis) {
    const float4* __restrict__ nodes = reinterpret_cast<const float4*>(p.bvh4);
    const f3 oi = o * ninv;
    int cur = M.bvh4_root, sp = 0;
    if (cur < 0) return true;                        // a mesh without triangles: nothing to traverse
    unsigned todo = 0xFu;
    for (;;) {
        nvis++;
        const float4* n4 = nodes + 8 * (size_t)cur;
        const float4 LX = n4[0], LY = n4[1], LZ = n4[2], HX = n4[3], HY = n4[4], HZ = n4[5], LK = n4[6], CN = n4[7];
        const float lx[4] = {LX.x, LX.y, LX.z, LX.w}, ly[4] = {LY.x, LY.y, LY.z, LY.w}, lz[4] = {LZ.x, LZ.y, LZ.z, LZ.w};
        const float hx[4] = {HX.x, HX.y, HX.z, HX.w}, hy[4] = {HY.x, HY.y, HY.z, HY.w}, hz[4] = {HZ.x, HZ.y, HZ.z, HZ.w};
        const int lk[4] = {__float_as_int(LK.x), __float_as_int(LK.y), __float_as_int(LK.z), __float_as_int(LK.w)};
        const int cn[4] = {__float_as_int(CN.x), __float_as_int(CN.y), __float_as_int(CN.z), __float_as_int(CN.w)};
        const float bd = bound();
        int next = -1;
        float next_t = 0.0f;
        unsigned rest = 0;
#pragma unroll
        for (int c = 0; c < 4; c++) {
            if (!((todo >> c) & 1u) || cn[c] < 0) continue;
            const float a0 = __builtin_fmaf(lx[c], ninv.x, -oi.x), b0 = __builtin_fmaf(hx[c], ninv.x, -oi.x);
            const float a1 = __builtin_fmaf(ly[c], ninv.y, -oi.y), b1 = __builtin_fmaf(hy[c], ninv.y, -oi.y);
            const float a2 = __builtin_fmaf(lz[c], ninv.z, -oi.z), b2 = __builtin_fmaf(hz[c], ninv.z, -oi.z);
            const float tn = fmaxf(fmaxf(fminf(a0, b0), fminf(a1, b1)), fminf(a2, b2));
            const float tf = fminf(fminf(fmaxf(a0, b0), fmaxf(a1, b1)), fmaxf(a2, b2));
            if (!((tn <= tf) & (tf >= -kEps) & (tn <= bd))) continue;
            if (cn[c] > 0) {                         // a leaf: its link is the stack's leaf entry
                if (!leaf(M.leaf_base + (lk[c] & ((1 << kLeafCountShift) - 1)), cn[c])) return false;
                continue;
            }
            if (next < 0 || tn < next_t) {
                if (next >= 0) rest |= 1u << next;
                next = c;
                next_t = tn;
            } else {
                rest |= 1u << c;
            }
        }
        if (rest) {
            if (sp >= kStack) {                      // cannot happen (one entry per level); reported as a fault
                atomicAdd(p.segments + kTraceFaultCounter, 1ull);
                return true;
            }
            stack[sp * STRIDE] = (cur << 4) | (int)rest;
            sp++;
        }
        if (next >= 0) {
            cur = lk[next];
            todo = 0xFu;
            continue;
        }
        if (sp == 0) return true;
        sp--;
        const int e = stack[sp * STRIDE];
        cur = e >> 4;
        todo = (unsigned)e & 0xFu;
    }
}

// Exact closest hit over the mesh's triangles via its BLAS.  Matches the
// brute-force scan in triangle-index order: (t, index) lexicographic minimum
// (a node is pruned only when entered beyond the best t, so a tie with a
// smaller index is still reached).
template <int STRIDE>
__device__ bool bvh_closest(const KParams& p, const ModelRec& M, f3 o, f3 d, f3 ninv, float& best, int& best_tri,
                            int* __restrict__ stack) {
    bool any = false;
    unsigned n_nodes = 0, n_tris = 0;   // PT_DEBUG_ABLATE & 8 statistics
    auto leaf = [&](int first, int count) {
        for (int i = first; i < first + count; i++) {
            const float4 A = p.bvh_tri_geom[3 * i], B = p.bvh_tri_geom[3 * i + 1], C = p.bvh_tri_geom[3 * i + 2];
            const int it = __float_as_int(A.w);
            float t;
            n_tris++;
            if (tri_test_rec(A, B, C, o, d, t)) {
                any = true;
                if (t < best || (t == best && it < best_tri)) { best = t; best_tri = it; }
            }
        }
        return true;
    };
    bvh4_traverse<STRIDE>(p, M, o, ninv, stack, leaf, [&] { return best; }, n_nodes);
    if (PT_TRACE_STATS && (p.debug & 8)) {
        atomicAdd(p.segments + 4 + kMaxBounceCounters, (unsigned long long)n_nodes);
        atomicAdd(p.segments + 5 + kMaxBounceCounters, (unsigned long long)n_tris);
        atomicAdd(p.segments + 6 + kMaxBounceCounters, 1ull);
    }
    return any;
}

constexpr int kHitCap = PT_HITCAP;   // hit-set capacity per lane (LDS); overflow -> global pool block
constexpr int kHitCapPool = 64;      // global pool block (members); overflow -> exact list-walking DDA

// BLAS traversal collecting hit-set members: triangles the reference test
// accepts, as (t bits, index, packed voxel box lo, hi) in the lane's LDS slots
// hs[i * STRIDE].  BOUNDED: only members with t <= t_min + margin are required
// (nodes entered beyond that are pruned; extra members are harmless: t_min only
// falls, so a required member's node is never pruned, in any visit order).
// Returns the count (-1 on overflow); *tmin_out = smallest t accepted.
template <int STRIDE, bool BOUNDED, int HSTRIDE = STRIDE, int CAP = kHitCap>
__device__ int bvh_collect(const KParams& p, const ModelRec& M, f3 o, f3 d, f3 ninv, int* __restrict__ stack,
                           int4* __restrict__ hs, float* tmin_out, float margin) {
    int nh = 0;
    float tmin = kFMax;
    unsigned nvis = 0;
    auto leaf = [&](int first, int count) {
        for (int i = first; i < first + count; i++) {
            const float4 A = p.bvh_tri_geom[3 * i], B = p.bvh_tri_geom[3 * i + 1], C = p.bvh_tri_geom[3 * i + 2];
            float t;
            if (!tri_test_rec(A, B, C, o, d, t)) continue;
            if (BOUNDED) {
                if (t < tmin) tmin = t;
                if (t > tmin + margin) continue;          // not required (NaN is kept)
                if (nh == CAP) {                           // drop members now beyond the bound
                    int w = 0;
                    for (int q = 0; q < nh; q++) {
                        const int4 e = hs[q * HSTRIDE];
                        if (!(__int_as_float(e.x) > tmin + margin)) hs[(w++) * HSTRIDE] = e;
                    }
                    nh = w;
                }
            } else if (t < tmin) {
                tmin = t;
            }
            if (nh == CAP) return false;
            hs[nh * HSTRIDE] = make_int4(__float_as_int(t), __float_as_int(A.w), __float_as_int(B.w),
                                         __float_as_int(C.w));
            nh++;
        }
        return true;
    };
    const bool ok = bvh4_traverse<STRIDE>(p, M, o, ninv, stack, leaf,
                                          [&] { return BOUNDED ? tmin + margin : 3.0e38f; }, nvis);
    if (PT_TRACE_STATS && (p.debug & 4)) {          // collection statistics: node visits, collections
        atomicAdd(p.segments + 22 + kMaxBounceCounters, (unsigned long long)nvis);
        atomicAdd(p.segments + 23 + kMaxBounceCounters, 1ull);
    }
    if (!ok) return -1;
    *tmin_out = tmin;
    return nh;
}

__device__ __forceinline__ bool vbox_has(int lo, int hi, int ix, int iy, int iz) {
    return ix >= (lo & 1023) && ix <= (hi & 1023) && iy >= ((lo >> 10) & 1023) && iy <= ((hi >> 10) & 1023) &&
           iz >= ((lo >> 20) & 1023) && iz <= ((hi >> 20) & 1023);
}

struct WalkResult {
    bool hit;        // computeRayGridIntersection's return value
    float t;         // winning member's t (valid when has_best)
    int tri;
    bool has_best;
    bool final_min;  // a member with t == tmin was tested in a voxel entered before tmin + wdelta: final
    float tw;        // ray parameter (from the model-space origin) where the walk stopped
};

// The reference's DDA walk (Renderer.cpp:263-358) over M's grid, with voxel
// triangle lists replaced by the hit set: voxel V holds triangle h in its list
// iff V lies in h's voxel box (Scene.cpp:364-374), and h's test outcome does not
// depend on V, so V is a hit voxel iff some member's box contains V.  The
// reference keeps the first strict minimum in test order (voxel order, then
// ascending index inside a list): the lexicographic minimum of (t, step, index).
// Split into init + one voxel per step so the persistent trace kernel can
// interleave walks with other lanes' traversal steps.
struct Walk {
    int ix, iy, iz, k;
    f3 tmax, delta;
    int ul, uh;                    // union of the members' voxel boxes (packed 10 bits/axis)
    int c;                         // last hit voxel (packed)
    unsigned long long tested;
    float bt;
    int bk, bi;
    bool hit;
    float te;                      // entry parameter (from pt) of the current voxel
    float tbe;                     // entry parameter of the voxel where the current best was tested
    bool passed;                   // stopped because the walk left the union box (not a reference stop)
};

__device__ __forceinline__ void walk_init(const KParams& p, const ModelRec& M, f3 d, f3 inv, f3 pt, Walk& w) {
    const int GX = p.gdim[0], GY = p.gdim[1], GZ = p.gdim[2];
    int ix = f2i_sat(absr(pt.x - M.bbox[0] + kEps) / M.vw[0]);
    int iy = f2i_sat(absr(pt.y - M.bbox[1] + kEps) / M.vw[1]);
    int iz = f2i_sat(absr(pt.z - M.bbox[2] + kEps) / M.vw[2]);
    w.ix = ix < 0 ? 0 : (ix > GX - 1 ? GX - 1 : ix);
    w.iy = iy < 0 ? 0 : (iy > GY - 1 ? GY - 1 : iy);
    w.iz = iz < 0 ? 0 : (iz > GZ - 1 ? GZ - 1 : iz);
    w.tmax = mk3(kFMax, kFMax, kFMax);
    w.delta = mk3(kFMax, kFMax, kFMax);
    const int nx = d.x > 0.0f ? w.ix + 1 : w.ix, ny = d.y > 0.0f ? w.iy + 1 : w.iy, nz = d.z > 0.0f ? w.iz + 1 : w.iz;
    const float px = M.bbox[0] + (float)nx * M.vw[0];
    const float py = M.bbox[1] + (float)ny * M.vw[1];
    const float pz = M.bbox[2] + (float)nz * M.vw[2];
    if (d.x != 0) { w.delta.x = absr(M.vw[0] * inv.x); w.tmax.x = (px - pt.x) * inv.x; }
    if (d.y != 0) { w.delta.y = absr(M.vw[1] * inv.y); w.tmax.y = (py - pt.y) * inv.y; }
    if (d.z != 0) { w.delta.z = absr(M.vw[2] * inv.z); w.tmax.z = (pz - pt.z) * inv.z; }
    w.k = 0;
    w.c = 0;
    w.tested = 0;
    w.bt = kFMax;
    w.bk = -1;
    w.bi = -1;
    w.hit = false;
    w.te = 0.0f;
    w.tbe = 0.0f;
    w.passed = false;
}

// Union of the members' voxel boxes.  CAP > 0: members come from a
// register array through `get` (fully unrolled, constant indices).
template <int CAP, class GetM>
__device__ __forceinline__ void walk_union_g(GetM get, int nh, Walk& w) {
    int ulx = 1023, uly = 1023, ulz = 1023, uhx = 0, uhy = 0, uhz = 0;
#pragma unroll
    for (int h = 0; h < (CAP > 0 ? CAP : nh); h++) {
        if (CAP > 0 && h >= nh) break;
        const int4 e = get(h);
        ulx = min(ulx, e.z & 1023); uly = min(uly, (e.z >> 10) & 1023); ulz = min(ulz, (e.z >> 20) & 1023);
        uhx = max(uhx, e.w & 1023); uhy = max(uhy, (e.w >> 10) & 1023); uhz = max(uhz, (e.w >> 20) & 1023);
    }
    w.ul = ulx | (uly << 10) | (ulz << 20);
    w.uh = uhx | (uhy << 10) | (uhz << 20);
}

template <int HSTRIDE>
__device__ __forceinline__ void walk_union(const int4* __restrict__ hs, int nh, Walk& w) {
    walk_union_g<0>([&](int h) { return hs[h * HSTRIDE]; }, nh, w);
}

// Fast-forward of the walk to its first voxel inside the members' union box.
// Before that voxel nothing can happen: no voxel outside the union box is a hit
// voxel, and the reference walk cannot stop before its first hit voxel.  The
// DDA's voxel order is the merge of the three per-axis crossing sequences
// tmax_a, tmax_a + delta_a, ... (each sum rounded as the walk rounds it) by
// (value, axis priority z < y < x) -- exactly the walk's
// "x if tmax.x < tmax.y && tmax.x < tmax.z, else y if tmax.y < tmax.z, else z"
// choice -- so the state at entry (indices, tmax, step count k, entry
// parameter te) follows from per-axis running sums, one add per skipped step
// instead of one full walk_step.  Leaves the walk untouched when it is already
// in range on every axis, when an axis leaves its range before the entry
// (the plain walk then stops there), or for zero / huge direction slopes.
__device__ __forceinline__ void walk_skip(f3 d, Walk& w) {
    const float dd[3] = {d.x, d.y, d.z};
    const float t0[3] = {w.tmax.x, w.tmax.y, w.tmax.z};
    const float dl[3] = {w.delta.x, w.delta.y, w.delta.z};
    const int ii[3] = {w.ix, w.iy, w.iz};
    int need[3], over[3];
    bool go = false;
#pragma unroll
    for (int a = 0; a < 3; a++) {
        const int lo = (w.ul >> (10 * a)) & 1023, hi = (w.uh >> (10 * a)) & 1023;
        if (dd[a] == 0.0f || !(absr(t0[a]) < 1e30f) || !(dl[a] < 1e30f)) return;
        need[a] = dd[a] > 0.0f ? max(0, lo - ii[a]) : max(0, ii[a] - hi);
        over[a] = dd[a] > 0.0f ? hi - ii[a] + 1 : ii[a] - lo + 1;
        if (over[a] <= 0) return;                       // already past the range: the walk stops at once
        go = go || need[a] > 0;
    }
    if (!go) return;
    // crossing value of the last step each axis needs; the entry step is their
    // maximum by (value, priority), priority z = 0 < y = 1 < x = 2
    float kn[3];
    int A = -1;
    float T = 0.0f;
#pragma unroll
    for (int a = 2; a >= 0; a--) {                      // z first, so a later axis wins only when strictly greater
        float K = t0[a];
        for (int c = 1; c < need[a]; c++) K += dl[a];
        kn[a] = K;
        const int pa = 2 - a;
        if (need[a] > 0 && (A < 0 || K > T || (K == T && pa > 2 - A))) { A = a; T = K; }
    }
    const int pA = 2 - A;
    int cnt[3];
    float nxt[3];
#pragma unroll
    for (int b = 0; b < 3; b++) {
        if (b == A) { cnt[b] = need[b]; nxt[b] = kn[b] + dl[b]; continue; }
        int c = 0;
        float K = t0[b];
        if (need[b] > 0) { c = need[b] - 1; K = kn[b]; }
        const int pb = 2 - b;
        // count b's steps before the entry step
        while (K < T || (K == T && pb < pA)) {
            c++;
            if (c >= over[b]) return;                   // b leaves its range first: plain walk
            K += dl[b];
        }
        cnt[b] = c;
        nxt[b] = K;
    }
    w.ix = ii[0] + (dd[0] > 0.0f ? cnt[0] : -cnt[0]);
    w.iy = ii[1] + (dd[1] > 0.0f ? cnt[1] : -cnt[1]);
    w.iz = ii[2] + (dd[2] > 0.0f ? cnt[2] : -cnt[2]);
    w.tmax = mk3(nxt[0], nxt[1], nxt[2]);
    w.k = cnt[0] + cnt[1] + cnt[2];
    w.te = T;
}

// One voxel of the walk; returns true when the walk has stopped.  Members
// through `get`; CAP > 0: a register array of CAP entries (unrolled).
// STRICT (the k_trace_gf collection, whose uncollected members may have any t):
// only the minimum-t shortcut ends the walk early, and leaving the union box
// after a hit voxel does not -- the walk steps on to the reference's own stop.
template <int CAP, class GetM, bool STRICT = false>
__device__ __forceinline__ bool walk_step_g(const KParams& p, f3 d, GetM get, int nh, float tmin, Walk& w) {
    const int ulx = w.ul & 1023, uly = (w.ul >> 10) & 1023, ulz = (w.ul >> 20) & 1023;
    const int uhx = w.uh & 1023, uhy = (w.uh >> 10) & 1023, uhz = (w.uh >> 20) & 1023;
    const int ix = w.ix, iy = w.iy, iz = w.iz, k = w.k;
    bool vhit = false;
    if (ix >= ulx && ix <= uhx && iy >= uly && iy <= uhy && iz >= ulz && iz <= uhz) {
#pragma unroll
        for (int h = 0; h < (CAP > 0 ? CAP : nh); h++) {
            if (CAP > 0 && h >= nh) break;
            const int4 e = get(h);
            if (vbox_has(e.z, e.w, ix, iy, iz)) {
                vhit = true;
                if (!((w.tested >> h) & 1ull)) {
                    w.tested |= 1ull << h;
                    const float t = __int_as_float(e.x);
                    if (t < w.bt || (t == w.bt && (k < w.bk || (k == w.bk && e.y < w.bi)))) {
                        w.bt = t; w.bk = k; w.bi = e.y; w.tbe = w.te;
                    }
                }
            }
        }
    }
    if (vhit) { w.c = ix | (iy << 10) | (iz << 20); w.hit = true; }
    // Exact shortcuts: once a minimum-t member (or every member) is tested the
    // result and the return value are final; once the monotone walk has passed
    // the union box along an axis it enters no member's box again.
    const unsigned long long all = nh >= 64 ? ~0ull : ((1ull << nh) - 1ull);
    if ((!STRICT && w.tested == all) || (w.bk >= 0 && w.bt == tmin)) return true;
    const int sx = d.x > 0.0f ? 1 : -1, sy = d.y > 0.0f ? 1 : -1, sz = d.z > 0.0f ? 1 : -1;
    if ((!STRICT || !w.hit) &&
        ((sx > 0 ? ix > uhx : ix < ulx) || (sy > 0 ? iy > uhy : iy < uly) || (sz > 0 ? iz > uhz : iz < ulz))) {
        w.passed = true;
        return true;
    }
    if (w.hit) {
        const int cx = w.c & 1023, cy = (w.c >> 10) & 1023, cz = (w.c >> 20) & 1023;
        if (iabs(cx - ix) > 2 || iabs(cy - iy) > 2 || iabs(cz - iz) > 2) return true;
    }
    w.k = k + 1;
    if (w.tmax.x < w.tmax.y && w.tmax.x < w.tmax.z) {
        w.ix = ix + sx;
        if (w.ix == (d.x > 0.0f ? p.gdim[0] : -1) || w.tmax.x >= kFMax) return true;
        w.te = w.tmax.x;
        w.tmax.x += w.delta.x;
    } else if (w.tmax.y < w.tmax.z) {
        w.iy = iy + sy;
        if (w.iy == (d.y > 0.0f ? p.gdim[1] : -1) || w.tmax.y >= kFMax) return true;
        w.te = w.tmax.y;
        w.tmax.y += w.delta.y;
    } else {
        w.iz = iz + sz;
        if (w.iz == (d.z > 0.0f ? p.gdim[2] : -1) || w.tmax.z >= kFMax) return true;
        w.te = w.tmax.z;
        w.tmax.z += w.delta.z;
    }
    return false;
}

template <int HSTRIDE>
__device__ __forceinline__ bool walk_step(const KParams& p, f3 d, const int4* __restrict__ hs, int nh, float tmin,
                                          Walk& w) {
    return walk_step_g<0>(p, d, [&](int h) { return hs[h * HSTRIDE]; }, nh, tmin, w);
}

// Walk certificate: decides from the ray's continuous geometry, without
// stepping the DDA, the common case where the walk's first voxel inside the
// members' union box U lies in the voxel box of the unique minimum-t member m*.
// Before that voxel no voxel is a hit voxel (nothing outside U is), so the
// walk cannot stop; in it m* is tested and the walk ends on its exact
// "minimum-t member tested" shortcut with result (t_min, m*).  The entry voxel
// is where the ray crosses U's face on the entering axis A; the other axes'
// indices there are read off the ray's position, accepted only when that
// position is farther from every voxel boundary than the DDA's own deviation
// from the exact ray (its +EPSILON initial shift and the rounding of its
// crossing parameters: ModelRec::cslack, plus the A-crossing's parameter error
// times the slope).  Any doubt (zero slopes, ties at t_min, an entry at the
// walk's start, a start within the shift of an interior boundary) -> false,
// and the exact walk runs.
template <int CAP, class GetM>
__device__ __forceinline__ bool walk_certify(const KParams& p, const ModelRec& M, f3 d, f3 inv, f3 pt, float t_box,
                                             GetM get, int nh, float tmin, float win, int& tri) {
    int cnt = 0;
    int ulx = 1023, uly = 1023, ulz = 1023, uhx = 0, uhy = 0, uhz = 0;
    // A failed condition clears `ok` instead of returning: the computation after it is
    // harmless, and one exit saves the scalar exec-mask work of eight divergent returns.
    bool ok = true;
#define PT_CERT_FAIL(r) { if (PT_TRACE_STATS && (p.debug & 4) && ok) atomicAdd(p.segments + 32 + (r) + kMaxBounceCounters, 1ull); ok = false; }
    // U is the union over the members the walk might enter no later than B*
    // (the minimum-t members' union box); members whose box it provably enters
    // only after B* cannot make a voxel before B*'s first one a hit voxel, so
    // they stay out of U (see below).  First pass: B*.
    int blx = 1023, bly = 1023, blz = 1023, bhx = 0, bhy = 0, bhz = 0;
#pragma unroll
    for (int h = 0; h < (CAP > 0 ? CAP : nh); h++) {
        if (CAP > 0 && h >= nh) break;
        const int4 e = get(h);
        if (__int_as_float(e.x) != tmin) continue;
        cnt++;
        blx = min(blx, e.z & 1023); bly = min(bly, (e.z >> 10) & 1023); blz = min(blz, (e.z >> 20) & 1023);
        bhx = max(bhx, e.w & 1023); bhy = max(bhy, (e.w >> 10) & 1023); bhz = max(bhz, (e.w >> 20) & 1023);
    }
    if (cnt == 0) PT_CERT_FAIL(0)
    if (d.x == 0.0f || d.y == 0.0f || d.z == 0.0f) PT_CERT_FAIL(1)
    {
        // sB: exact-ray entry parameter (from pt) of B*.  The walk enters its first
        // voxel of B* at a computed parameter <= sB + errm (errm: the largest
        // crossing-parameter error of any axis up to there), so every walk voxel
        // before it is entered at a parameter <= sB + errm.  A walk voxel W of
        // member h's box, entered at parameter s, puts the exact ray at s within
        // cslack + |d| errm of W, i.e. inside h's box grown by that: the grown
        // box's exact entry g_h <= s.  So g_h > sB + errm (+ rounding slack)
        // proves h's box holds no walk voxel before B*'s first one.
        const float pp[3] = {pt.x, pt.y, pt.z}, dv[3] = {d.x, d.y, d.z}, iv[3] = {inv.x, inv.y, inv.z};
        const int bl[3] = {blx, bly, blz}, bh[3] = {bhx, bhy, bhz};
        float sB = -3.0e38f, sBo = 3.0e38f;
#pragma unroll
        for (int a = 0; a < 3; a++) {
            const float lo = M.bbox[a] + (float)bl[a] * M.vw[a], hi = M.bbox[a] + (float)(bh[a] + 1) * M.vw[a];
            const float s0 = (lo - pp[a]) * iv[a], s1 = (hi - pp[a]) * iv[a];
            sB = fmaxf(sB, fminf(s0, s1));
            sBo = fminf(sBo, fmaxf(s0, s1));
        }
        float errm = 0.0f;
#pragma unroll
        for (int a = 0; a < 3; a++) {
            const float span = M.vw[a] * (float)p.gdim[a];
            errm = fmaxf(errm, 4.8e-7f * (float)(p.gdim[a] + 4) * (absr(sB) + 1.0f) +
                                   1e-6f * (absr(M.bbox[a]) + span + absr(pp[a])) * absr(iv[a]));
        }
        // a ray that misses B* exactly, or bounds out of range: every member stays in U
        const bool use = sB <= sBo && absr(sB) < 1e30f && errm < 1e30f;
        const float lim = sB + 2.0f * errm + 1e-5f * (absr(sB) + 1.0f);
#pragma unroll
        for (int h = 0; h < (CAP > 0 ? CAP : nh); h++) {
            if (CAP > 0 && h >= nh) break;
            const int4 e = get(h);
            bool in = true;
            if (use && __int_as_float(e.x) != tmin) {
                float g = -3.0e38f, go = 3.0e38f;
#pragma unroll
                for (int a = 0; a < 3; a++) {
                    const float dl = M.cslack[a] + absr(dv[a]) * errm;
                    const float lo = M.bbox[a] + (float)((e.z >> (10 * a)) & 1023) * M.vw[a] - dl;
                    const float hi = M.bbox[a] + (float)(((e.w >> (10 * a)) & 1023) + 1) * M.vw[a] + dl;
                    const float s0 = (lo - pp[a]) * iv[a], s1 = (hi - pp[a]) * iv[a];
                    g = fmaxf(g, fminf(s0, s1));
                    go = fminf(go, fmaxf(s0, s1));
                }
                // entered only after B* (a grown box the ray misses is never entered)
                if ((g > go + 1e-5f * (absr(go) + 1.0f) || g - 1e-5f * (absr(g) + 1.0f) > lim) && absr(g) < 1e30f)
                    in = false;
            }
            if (!in) continue;
            ulx = min(ulx, e.z & 1023); uly = min(uly, (e.z >> 10) & 1023); ulz = min(ulz, (e.z >> 20) & 1023);
            uhx = max(uhx, e.w & 1023); uhy = max(uhy, (e.w >> 10) & 1023); uhz = max(uhz, (e.w >> 20) & 1023);
        }
    }
    const float dd[3] = {d.x, d.y, d.z}, iv[3] = {inv.x, inv.y, inv.z}, pp[3] = {pt.x, pt.y, pt.z};
    const int ul[3] = {ulx, uly, ulz}, uh[3] = {uhx, uhy, uhz};
    float sin = -3.0e38f, sout = 3.0e38f;
    int A = 0;
    int v0[3];
    bool in0 = true;
#pragma unroll
    for (int a = 0; a < 3; a++) {
        // the walk's start index is the exact one unless pt lies within the shift of an interior boundary
        const float q = (pp[a] - M.bbox[a]) * M.ivw[a];
        const float n = rintf(q);
        if (n >= 1.0f && n <= (float)(p.gdim[a] - 1) && absr(q - n) * M.vw[a] <= M.cslack[a]) PT_CERT_FAIL(2)
        v0[a] = min(max((int)floorf(q), 0), p.gdim[a] - 1);
        in0 = in0 && v0[a] >= ul[a] && v0[a] <= uh[a];
        const float lo = M.bbox[a] + (float)ul[a] * M.vw[a], hi = M.bbox[a] + (float)(uh[a] + 1) * M.vw[a];
        const float s0 = (lo - pp[a]) * iv[a], s1 = (hi - pp[a]) * iv[a];
        const float en = fminf(s0, s1), ex = fmaxf(s0, s1);
        if (en > sin) { sin = en; A = a; }
        sout = fminf(sout, ex);
    }
    int va[3];
    float te;
    if (in0) {                                   // the walk starts inside U: its first voxel is the entry
        va[0] = v0[0]; va[1] = v0[1]; va[2] = v0[2];
        te = 0.0f;
    } else {
        const float span = M.vw[A] * (float)p.gdim[A];
        const float err = 4.8e-7f * (float)(p.gdim[A] + 4) * (absr(sin) + 1.0f) +
                          1e-6f * (absr(M.bbox[A]) + span + absr(pp[A])) * absr(iv[A]);
        if (!(sin > 2.0f * err)) PT_CERT_FAIL(3)
        if (!(sout - sin > 2.0f * err)) PT_CERT_FAIL(4)
#pragma unroll
        for (int b = 0; b < 3; b++) {
            if (b == A) {
                va[b] = dd[b] > 0.0f ? ul[b] : uh[b];
            } else {
                const float q = (pp[b] + dd[b] * sin - M.bbox[b]) * M.ivw[b];
                const float f = floorf(q);
                if (!(fminf(q - f, f + 1.0f - q) * M.vw[b] > M.cslack[b] + absr(dd[b]) * err)) PT_CERT_FAIL(5)
                // clamped: after a failed condition (no early return any more) f may be
                // huge or NaN; indices outside 0..1023 match no member either way
                va[b] = (int)fminf(fmaxf(f, -1.0f), 1024.0f);
            }
        }
        te = sin + err;
    }
    // the walk tests every member whose box holds the entry voxel there, in index
    // order: the minimum-t member with the lowest index among them wins
    int bi = 0x7fffffff;
#pragma unroll
    for (int h = 0; h < (CAP > 0 ? CAP : nh); h++) {
        if (CAP > 0 && h >= nh) break;
        const int4 e = get(h);
        if (__int_as_float(e.x) == tmin && vbox_has(e.z, e.w, va[0], va[1], va[2]) && e.y < bi) bi = e.y;
    }
    if (bi == 0x7fffffff) PT_CERT_FAIL(6)
    if (!(t_box + te < tmin + win)) PT_CERT_FAIL(7)
#undef PT_CERT_FAIL
    tri = bi;
    return ok;
}

// Fast walk certificate: a cheaper sufficient condition for the common case,
// tried before walk_certify.  It decides the walk's result as (t_min, m*) when
// m* is the unique minimum-t member (or every minimum-t member has m*'s voxel
// box, index = their lowest) and the walk provably tests it before it can stop.  The lemma both certificates rest on: at every walk parameter s
// (from pt) the walk's voxel holds, per axis a, a point within
// delta_a = cslack_a + |d_a| errm of the exact ray point ray(s) (the DDA's
// +EPSILON start shift and its crossing-parameter rounding, errm bounding the
// latter up to s).
//  (i) B*, m*'s voxel box shrunk by delta, holds ray(s*) at s* = max(e, 0) + sl
//      (e: B*'s exact entry, sl a rounding slack, s* + sl < B*'s exit): the
//      walk's voxel at s* lies in m*'s box, so m* is tested no later than s* --
//      unless the walk stopped before, which needs an earlier hit voxel.
// (ii) A voxel of member h visited at s' puts ray(s') inside h's box grown by
//      delta, so s' >= g_h, that grown box's entry.  Only h's voxels outside
//      m*'s box matter (m*'s own voxels test m* too): when h's box leaves m*'s
//      along one side of one axis only, that part is itself a box, else the
//      whole box stands in for it.  g_h > s* (or a grown box the ray misses, or
//      a start inside B*, whose start voxel then is m*'s) means no voxel before
//      the walk reaches m*'s box is a hit voxel: the walk cannot stop before
//      testing m*, and m*'s minimum t makes the result (t_min, m*) (tied members
//      of m*'s box are tested in the same voxel: the lowest index wins).
// (iii) The voxel holding s* was entered at a parameter <= s*: within the
//      window when t_box + s* < t_min + win (plus rounding slack).
// Any doubt (ties at t_min among different boxes, zero slopes, boxes too thin
// to shrink, rays that only graze B*) returns false and walk_certify / the
// exact walk decide.
template <int CAP, class GetM>
__device__ __forceinline__ bool walk_certify_fast(const KParams& p, const ModelRec& M, f3 d, f3 inv, f3 pt, float t_box,
                                                  GetM get, int nh, float tmin, float win, int& tri) {
    // m*: the minimum-t member, or several tied at t_min whose voxel boxes are identical (the two
    // triangles of a quad split along its diagonal share their box: 72 % of the fast certificate's
    // failures at configs[1] were such ties).  Tied members with one box B* are all tested in the
    // walk's first voxel of B*, where the lowest index among them wins (walk_step_g's (t, step,
    // index) order), so they act as one member with that index.
    int cnt = 0;
    bool same = true;                               // every minimum-t member has m*'s box
    int ms_y = 0x7fffffff, ms_z = 0, ms_w = 0;      // m*'s index and packed voxel box (per component:
#pragma unroll                                      // a select of whole int4s went through scratch memory)
    for (int h = 0; h < (CAP > 0 ? CAP : nh); h++) {
        if (CAP > 0 && h >= nh) break;
        const int4 e = get(h);
        const bool mn = __int_as_float(e.x) == tmin;
        same = same & (!mn | (cnt == 0) | ((e.z == ms_z) & (e.w == ms_w)));
        ms_z = (mn & (cnt == 0)) ? e.z : ms_z;
        ms_w = (mn & (cnt == 0)) ? e.w : ms_w;
        ms_y = mn ? min(ms_y, e.y) : ms_y;
        cnt += mn ? 1 : 0;
    }
    const float pp[3] = {pt.x, pt.y, pt.z}, dv[3] = {d.x, d.y, d.z}, iv[3] = {inv.x, inv.y, inv.z};
    int bl[3], bh[3];
    float lo[3], hi[3];
    float sB = -3.0e38f, xB = 3.0e38f;
#pragma unroll
    for (int a = 0; a < 3; a++) {
        bl[a] = (ms_z >> (10 * a)) & 1023;
        bh[a] = (ms_w >> (10 * a)) & 1023;
        lo[a] = M.bbox[a] + (float)bl[a] * M.vw[a];
        hi[a] = M.bbox[a] + (float)(bh[a] + 1) * M.vw[a];
        const float s0 = (lo[a] - pp[a]) * iv[a], s1 = (hi[a] - pp[a]) * iv[a];
        sB = fmaxf(sB, fminf(s0, s1));
        xB = fminf(xB, fmaxf(s0, s1));
    }
    // crossing-parameter error bound for every parameter up to B*'s exit (walk_certify's formula)
    float errm = 0.0f;
#pragma unroll
    for (int a = 0; a < 3; a++) {
        const float span = M.vw[a] * (float)p.gdim[a];
        errm = fmaxf(errm, 4.8e-7f * (float)(p.gdim[a] + 4) * (absr(xB) + 1.0f) +
                               1e-6f * (absr(M.bbox[a]) + span + absr(pp[a])) * absr(iv[a]));
    }
    float dl[3];
    float e = -3.0e38f, x = 3.0e38f;
    bool thick = true;
#pragma unroll
    for (int a = 0; a < 3; a++) {
        dl[a] = M.cslack[a] + absr(dv[a]) * errm;
        const float L = lo[a] + dl[a], H = hi[a] - dl[a];
        thick = thick & (L < H);
        const float s0 = (L - pp[a]) * iv[a], s1 = (H - pp[a]) * iv[a];
        e = fmaxf(e, fminf(s0, s1));
        x = fminf(x, fmaxf(s0, s1));
    }
    const float sl = 1e-5f * (absr(x) + 1.0f);
    const float ss = fmaxf(e, 0.0f) + sl;
    bool ok = (cnt >= 1) & same & (dv[0] != 0.0f) & (dv[1] != 0.0f) & (dv[2] != 0.0f) & thick & (sB <= xB) &
              (ss + sl < x) & (absr(x) < 1e30f) & (errm < 1e30f);
    const float tw = t_box + ss;
    ok = ok & (tw + 1e-5f * (absr(tw) + 1.0f) < tmin + win);
    const bool start_in = e < 0.0f;               // the walk's start voxel is m*'s
    bool mfail1 = false, mfailn = false;          // stats build: a member failed with one / several extensions
#pragma unroll
    for (int h = 0; h < (CAP > 0 ? CAP : nh); h++) {
        if (CAP > 0 && h >= nh) break;
        const int4 m = get(h);
        int ml[3], mh[3];
        int ext = 0, ax = 0;
        bool below = false;
#pragma unroll
        for (int a = 0; a < 3; a++) {
            ml[a] = (m.z >> (10 * a)) & 1023;
            mh[a] = (m.w >> (10 * a)) & 1023;
            const bool lb = ml[a] < bl[a], ha = mh[a] > bh[a];
            ext += (lb ? 1 : 0) + (ha ? 1 : 0);
            ax = (lb | ha) ? a : ax;
            below = (lb | ha) ? lb : below;
        }
        // m* itself, a member inside m*'s box, or a start inside B*: nothing to test
        // (a branch, not a select: the common single-member hit set skips the float work)
        const bool mn = __int_as_float(m.x) == tmin;
        if (!(mn | (ext == 0) | start_in)) {
            // one extension: only the part of h's box outside m*'s along axis ax can hold a
            // voxel the walk visits before m*'s box
#pragma unroll
            for (int a = 0; a < 3; a++) {
                const bool cut = (ext == 1) & (a == ax);
                mh[a] = (cut & below) ? bl[a] - 1 : mh[a];
                ml[a] = (cut & !below) ? bh[a] + 1 : ml[a];
            }
            float g = -3.0e38f, go = 3.0e38f;
#pragma unroll
            for (int a = 0; a < 3; a++) {
                const float L = M.bbox[a] + (float)ml[a] * M.vw[a] - dl[a];
                const float H = M.bbox[a] + (float)(mh[a] + 1) * M.vw[a] + dl[a];
                const float s0 = (L - pp[a]) * iv[a], s1 = (H - pp[a]) * iv[a];
                g = fmaxf(g, fminf(s0, s1));
                go = fminf(go, fmaxf(s0, s1));
            }
            const bool missed = (g > go + 1e-5f * (absr(go) + 1.0f)) & (absr(g) < 1e30f);
            const bool after = (g - 1e-5f * (absr(g) + 1.0f) > ss) & (absr(g) < 1e30f);
            ok = ok & (missed | after);
            if (PT_TRACE_STATS) {
                mfail1 = mfail1 | (!(missed | after) & (ext == 1));
                mfailn = mfailn | (!(missed | after) & (ext > 1));
            }
        }
    }
    if (PT_TRACE_STATS && (p.debug & 4) && !ok) {   // the first failed condition (slots 80..87)
        const int r = !((cnt >= 1) & same) ? 0
                    : !((dv[0] != 0.0f) & (dv[1] != 0.0f) & (dv[2] != 0.0f)) ? 1
                    : !thick ? 2
                    : !(sB <= xB) ? 3
                    : !((ss + sl < x) & (absr(x) < 1e30f) & (errm < 1e30f)) ? 4
                    : !(tw + 1e-5f * (absr(tw) + 1.0f) < tmin + win) ? 5
                    : mfail1 ? 6 : mfailn ? 7 : 5;
        atomicAdd(p.segments + 80 + r + kMaxBounceCounters, 1ull);
    }
    tri = ms_y;
    return ok;
}

template <int CAP, class GetM, bool CERT = true, bool STRICT = false>
__device__ __forceinline__ WalkResult hitset_walk_g(const KParams& p, const ModelRec& M, f3 d, f3 inv, f3 pt, float t_box,
                                                    GetM get, int nh, float tmin, float win, bool try_cert = true) {
    if (CERT && try_cert) {
        int tri;
        if (walk_certify<CAP>(p, M, d, inv, pt, t_box, get, nh, tmin, win, tri)) {
            if (PT_TRACE_STATS && (p.debug & 4)) atomicAdd(p.segments + 13 + kMaxBounceCounters, 1ull);
            WalkResult r;
            r.hit = true; r.t = tmin; r.tri = tri; r.has_best = true; r.final_min = true; r.tw = 0.0f;
            return r;
        }
    }
    const bool stamps = PT_TRACE_STATS && (p.debug & 64);     // wave cycles: init+union, skip, steps
    unsigned long long c0 = stamps ? clock64() : 0;
    Walk w;
    walk_init(p, M, d, inv, pt, w);
    walk_union_g<CAP>(get, nh, w);
    unsigned long long c1 = stamps ? clock64() : 0;
    walk_skip(d, w);
    unsigned long long c2 = stamps ? clock64() : 0;
    unsigned steps = 1;
    while (!walk_step_g<CAP, GetM, STRICT>(p, d, get, nh, tmin, w)) steps++;
    if (stamps) {
        const unsigned long long c3 = clock64();
        if ((int)(threadIdx.x & 63) == __ffsll((long long)__ballot(1)) - 1) {
            atomicAdd(p.segments + 29 + kMaxBounceCounters, c1 - c0);
            atomicAdd(p.segments + 30 + kMaxBounceCounters, c2 - c1);
            atomicAdd(p.segments + 31 + kMaxBounceCounters, c3 - c2);
        }
    }
    if (PT_TRACE_STATS && (p.debug & 4)) {          // walk statistics: steps, walks, members; steps per model
        atomicAdd(p.segments + 20 + kMaxBounceCounters, (unsigned long long)steps);
        atomicAdd(p.segments + 21 + kMaxBounceCounters, 1ull);
        atomicAdd(p.segments + 24 + kMaxBounceCounters, (unsigned long long)nh);
        const int mi = (int)(&M - p.models);
        if (mi >= 0 && mi < 4) atomicAdd(p.segments + 25 + mi + kMaxBounceCounters, (unsigned long long)steps);
    }
    WalkResult r;
    r.hit = w.hit;
    r.t = w.bt;
    r.tri = w.bi;
    r.has_best = w.bk >= 0;
    r.final_min = w.bk >= 0 && w.bt == tmin && t_box + w.tbe < tmin + win;
    // A walk that left the union box before any hit voxel has not stopped in the
    // reference sense: the reference walk goes on (it cannot stop before a hit
    // voxel) and may still enter the box of a member beyond the collection
    // window, so that outcome is final only for an unbounded collection.
    r.tw = (w.passed && !w.hit) ? 3.0e38f : t_box + fminf(fminf(w.tmax.x, w.tmax.y), w.tmax.z);
    return r;
}

template <int HSTRIDE, bool STRICT = false>
__device__ WalkResult hitset_walk(const KParams& p, const ModelRec& M, f3 d, f3 inv, f3 pt, float t_box,
                                  const int4* __restrict__ hs, int nh, float tmin, float win) {
    auto get = [&](int h) { return hs[h * HSTRIDE]; };
    return hitset_walk_g<0, decltype(get), true, STRICT>(p, M, d, inv, pt, t_box, get, nh, tmin, win);
}

// The same walk over at most CAP members copied to registers first: the walk's
// per-voxel membership tests then wait on no LDS reads.
template <int CAP, int HSTRIDE, bool CERT = true, bool STRICT = false>
__device__ __forceinline__ WalkResult hitset_walk_regs(const KParams& p, const ModelRec& M, f3 d, f3 inv, f3 pt,
                                                       float t_box, const int4* __restrict__ hs, int nh, float tmin,
                                                       float win, bool try_cert = true) {
    int4 mem[CAP];
#pragma unroll
    for (int h = 0; h < CAP; h++) mem[h] = h < nh ? hs[h * HSTRIDE] : make_int4(0, 0, 0, 0);
    auto get = [&](int h) { return mem[h]; };
    return hitset_walk_g<CAP, decltype(get), CERT, STRICT>(p, M, d, inv, pt, t_box, get, nh, tmin, win, try_cert);
}

// Overflow tiers of grid_hitset: bounded, then unbounded collection into a
// kHitCapPool-member block bump-allocated from the global pool (k_scan resets
// the pool every bounce).  Returns false when the pool is exhausted or the
// block overflows too (the caller then runs the list-walking DDA).
template <int STRIDE>
__device__ bool grid_hitset_pool(const KParams& p, const ModelRec& M, f3 o, f3 d, f3 inv, f3 ninv,
                                 f3 pt, float t_box, int* __restrict__ stack, WalkResult& w) {
    const int blk = atomicAdd(p.hs_pool_next, 1);
    if (blk >= p.hs_pool_blocks) return false;
    int4* g = p.hs_pool + (size_t)blk * kHitCapPool;
#pragma unroll 1
    for (int tier = 0; tier < 3; tier++) {
        const float win = tier == 0 ? M.wdelta : (tier == 1 ? 2.0f * M.reach : 3.0e38f);
        float tmin;
        const int ng = tier < 2 ? bvh_collect<STRIDE, true, 1, kHitCapPool>(p, M, o, d, ninv, stack, g, &tmin, win + M.reach)
                                : bvh_collect<STRIDE, false, 1, kHitCapPool>(p, M, o, d, ninv, stack, g, &tmin, 3.0e38f);
        if (ng < 0) return false;
        w = hitset_walk<1>(p, M, d, inv, pt, t_box, g, ng, tmin, win);
        if (tier == 2 || w.final_min || w.tw < tmin + win) return true;
    }
    return false;
}

// computeRayGridIntersection (Renderer.cpp:238-360), result-identical, via the
// BLAS hit set and hitset_walk.
// Tier 1 collects members with t <= t_min + W + R only (R = ModelRec::reach: a
// member whose voxel box the walk enters at parameter tau has t <= tau + R;
// W = ModelRec::wdelta), so the simulated walk equals the reference walk up to
// parameter X = t_min + W.  It is exact when the walk tests a minimum-t member
// in a voxel entered before X, or stops before X.  Otherwise tier 2 collects
// the whole set; on hit-set overflow the global pool, then the list-walking DDA.
template <int STRIDE>
__device__ bool grid_hitset(const KParams& p, const ModelRec& M, f3 o, f3 d, f3 inv, float& best, int& best_tri,
                            int* __restrict__ stack, int4* __restrict__ hs) {
    float t_box;
    if (!slab_ref(M.bbox, o, d, inv, t_box)) return false;
    const f3 pt = o + d * t_box;
    if ((pt.x - M.bbox[0]) < -kEps || (pt.y - M.bbox[1]) < -kEps || (pt.z - M.bbox[2]) < -kEps) return false;
    const f3 ninv = node_inv(inv);
    if (PT_TRACE_STATS && (p.debug & 2)) return bvh_closest<STRIDE>(p, M, o, d, ninv, best, best_tri, stack);   // timing-only ablation
    // Tiers: window W (ModelRec::wdelta), then 2R, then unbounded; each collects
    // the members a walk exact up to t_min + window needs (margin window + R).
    WalkResult w;
    bool done = false;
#pragma unroll 1
    for (int tier = 0; tier < 3; tier++) {
        const float win = tier == 0 ? M.wdelta : (tier == 1 ? 2.0f * M.reach : 3.0e38f);
        float tmin;
        const int nh = tier < 2 ? bvh_collect<STRIDE, true>(p, M, o, d, ninv, stack, hs, &tmin, win + M.reach)
                                : bvh_collect<STRIDE, false>(p, M, o, d, ninv, stack, hs, &tmin, 3.0e38f);
        if (nh == 0) return false;       // no accepted triangle anywhere on the ray: no hit voxel
        if (nh < 0) break;               // LDS hit set overflowed
        if (PT_TRACE_STATS && (p.debug & 1)) {   // timing-only ablation: no walk
            for (int h = 0; h < nh; h++) {
                const float t = __int_as_float(hs[h * STRIDE].x);
                if (t < best) { best = t; best_tri = hs[h * STRIDE].y; }
            }
            return true;
        }
        w = hitset_walk<STRIDE>(p, M, d, inv, pt, t_box, hs, nh, tmin, win);
        if (tier == 2 || w.final_min || w.tw < tmin + win) { done = true; break; }
        if (PT_TRACE_STATS && (p.debug & 4)) atomicAdd(p.segments + 1 + kMaxBounceCounters, 1ull);
    }
    if (!done) {
        // LDS hit set overflowed: the same tiers in a 64-entry block of the global pool.
        if (PT_TRACE_STATS && (p.debug & 4)) atomicAdd(p.segments + 2 + kMaxBounceCounters, 1ull);
        done = grid_hitset_pool<STRIDE>(p, M, o, d, inv, ninv, pt, t_box, stack, w);
        if (!done) {
            if (PT_TRACE_STATS && (p.debug & 4)) atomicAdd(p.segments + 3 + kMaxBounceCounters, 1ull);
            return grid_closest(p, M, o, d, inv, best, best_tri);   // exact list-walking DDA
        }
    }
    if (w.hit && w.has_best) { best = w.t; best_tri = w.tri; }
    return w.hit;
}

// Instance culling against a model's conservative world box.  Exact: a
// culled instance either cannot pass the reference's slab test / hit a
// triangle, or can only hit at a world distance > gdist (and `gdist > dd`
// is strict).  Grid mode keeps the slab test's zero-direction quirk by never
// miss-culling when a model-space direction component is 0.
template <int ACCEL>
__device__ __forceinline__ bool model_culled(const ModelRec& M, f3 orig, f3 dir, f3 winv, float dlen, float gdist) {
    float wtn, wtf;
    node_slab(M.wbox, M.wbox + 3, orig, winv, wtn, wtf);
    // both tests in one block (`|`, not `||`: a branch between them re-canonicalised the slab operands)
    const bool beyond = wtn * dlen > gdist * 1.0001f + 0.01f;        // cannot beat the current hit
    const bool miss = (wtn > wtf) | (wtf * dlen < -1.0f);             // misses the instance box
    if (ACCEL == ACCEL_BVH) return beyond | miss;
    if (beyond | miss) {
        if (beyond) return true;
        const f3 dm = xform12(M.w2m, dir, 0.0f);
        if (dm.x != 0.0f && dm.y != 0.0f && dm.z != 0.0f) return true;
    }
    return false;
}

// World distance of a model-space hit (computeRaySceneIntersectionKernel, Renderer.cpp:386-397).
__device__ __forceinline__ float model_hit_dist(const ModelRec& M, f3 o, f3 d, float best, f3 orig) {
    const f3 nd = normalize(d);
    const f3 pm = o + nd * best;
    const f3 pw = xform12(M.m2w, pm, 1.0f);
    return length(pw - orig);
}

__device__ __forceinline__ Hit make_hit(const KParams& p, float gdist, int gmodel, int gtri) {
    Hit h;
    h.dist = kFMax;
    h.n = mk3(0, 0, 0);
    h.model = -1;
    if (gdist < kFMax) {
        const float4 tn = gtri >= 0 ? p.tri_normal[gtri] : make_float4(0, 0, 0, 0);
        h.dist = gdist;
        h.model = gmodel;
        h.n = normalize(xform_normal9(p.models[gmodel].nm, mk3(tn.x, tn.y, tn.z)));
    }
    return h;
}

// Hit record of the split trace -> shade path (p.hit4 / p.hitm, slot j):
// (dist, triangle) + model.  The shading pass fetches the triangle normal and
// transforms it with make_hit's float operations (the same values): the
// latency-bound trace does no dependent normal gather (round 3, +1-2 %).
__device__ __forceinline__ void put_hit(const KParams& p, int j, float gdist, int gmodel, int gtri) {
    const bool any = gdist < kFMax;
    p.hit4[j] = make_float4(any ? gdist : kFMax, __int_as_float(gtri), 0.0f, 0.0f);
    p.hitm[j] = any ? gmodel : -1;
}
__device__ __forceinline__ Hit get_hit(const KParams& p, int hj) {
    const float4 hh = p.hit4[hj];
    Hit h;
    h.dist = hh.x;
    h.model = p.hitm[hj];
    h.n = mk3(0, 0, 0);
    if (h.model >= 0) {
        const int tri = __float_as_int(hh.y);
        const float4 tn = tri >= 0 ? p.tri_normal[tri] : make_float4(0, 0, 0, 0);
        h.n = normalize(xform_normal9(p.models[h.model].nm, mk3(tn.x, tn.y, tn.z)));
    }
    return h;
}

template <int ACCEL, int STRIDE>
__device__ void intersect_scene_g(const KParams& p, f3 orig, f3 dir, int* stack, int4* hs, float& gdist, int& gmodel,
                                  int& gtri) {
    gdist = kFMax;
    gmodel = -1; gtri = -1;
    const f3 winv = node_inv(cull_inv(dir));
    const float dlen = sqrtf(dot(dir, dir));
    for (int im = 0; im < p.nmodels; im++) {
        const ModelRec& M = p.models[im];
        if (model_culled<ACCEL>(M, orig, dir, winv, dlen, gdist)) continue;
        const f3 o = xform12(M.w2m, orig, 1.0f);
        const f3 d = normalize(xform12(M.w2m, dir, 0.0f));
        const f3 inv = mk3(1 / d.x, 1 / d.y, 1 / d.z);
        float best = kFMax;
        int best_tri = -1;
        bool ok;
        if (ACCEL == ACCEL_GRID) ok = grid_closest(p, M, o, d, inv, best, best_tri);
        else if (ACCEL == ACCEL_GRID_FAST) ok = grid_hitset<STRIDE>(p, M, o, d, inv, best, best_tri, stack, hs);
        else ok = bvh_closest<STRIDE>(p, M, o, d, node_inv(inv), best, best_tri, stack);
        if (ok) {
            const float dd = model_hit_dist(M, o, d, best, orig);
            if (gdist > dd) { gdist = dd; gmodel = im; gtri = best_tri; }
        }
    }
}

template <int ACCEL, int STRIDE>
__device__ Hit intersect_scene(const KParams& p, f3 orig, f3 dir, int* stack, int4* hs) {
    float gdist;
    int gmodel, gtri;
    intersect_scene_g<ACCEL, STRIDE>(p, orig, dir, stack, hs, gdist, gmodel, gtri);
    return make_hit(p, gdist, gmodel, gtri);
}

// generateRaysKernel (Renderer.cpp:521-555)
__device__ __forceinline__ void camera_ray(const KParams& p, int i, f3& o, f3& d) {
    const int y = i / p.width, x = i % p.width;
    const float wx = (float)(p.plane_x0 + (double)((float)x * p.step_x));
    const float wy = (float)(p.plane_y0 + (double)((float)y * p.step_y));
    o = mk3(p.cam_x, p.cam_y, p.cam_z);
    d = mk3(wx, wy, p.plane_z) - o;
}

struct RayState { f3 o, d, c; int pixel, bounces; };

// shadeRayKernel (Renderer.cpp:411-479) for one ray; slot = iray.
__device__ __forceinline__ void shade(const KParams& p, RayState& r, const Hit& h, int iter, int slot) {
    if (r.bounces <= 0) r.c = r.c * mk3(0.01f, 0.01f, 0.01f);
    if (h.dist < kFMax) {
        const f3 dir = normalize(r.d);
        const f3 ip = r.o + dir * h.dist;
        if (r.bounces > 0) {
            const ModelShade& S = p.shade[h.model];
            const int mt = S.mat_type;
            const f3 mc = mk3(S.color[0], S.color[1], S.color[2]);
            if (mt == MAT_DIFFUSE || mt == MAT_METAL || mt == MAT_COAT) {
                Rng rng = Rng::make(iter, slot, r.bounces);
                if (mt == MAT_DIFFUSE) r.d = scatter_hemisphere(h.n, rng);
                else if (mt == MAT_METAL) r.d = scatter_metal(h.n, dir, rng);
                else r.d = scatter_coat(h.n, dir, rng);
                r.o = ip + h.n * 0.1f;
                r.c = r.c * mc;
            } else if (mt == MAT_EMISSIVE) {
                r.bounces = 0;
                r.c = r.c * mc;
                return;
            } else if (mt == MAT_REFLECTIVE) {
                r.c = r.c * mc;
                const f3 rr = reflect_ref(dir, h.n);
                r.o = ip + h.n * 0.1f;
                r.d = rr;
            }
        }
    } else {
        r.bounces = 0;
        r.c = r.c * mk3(0.01f, 0.01f, 0.01f);
        return;
    }
    r.bounces--;
}

// ---------------------------------------------------------------------------
// Kernels
// ---------------------------------------------------------------------------

// Primary intersections, cached once per renderer (Renderer.cpp:596-613).
template <int ACCEL>
__global__ __launch_bounds__(kBlock) void k_primary(KParams p) {
    __shared__ int s_stack[ACCEL != ACCEL_GRID ? kStack * kBlock : 1];
    __shared__ int4 s_hs[ACCEL == ACCEL_GRID_FAST ? kHitCap * kBlock : 1];
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= p.npix) return;
    f3 o, d;
    camera_ray(p, i, o, d);
    const Hit h = intersect_scene<ACCEL, kBlock>(p, o, d, s_stack + threadIdx.x, s_hs + threadIdx.x);
    p.cache_hit[i] = make_float4(h.dist, h.n.x, h.n.y, h.n.z);
    p.cache_model[i] = h.model;
}

// Test hook: intersect an arbitrary batch of world-space rays.
template <int ACCEL>
__global__ __launch_bounds__(kBlock) void k_intersect_rays(KParams p, int n, const float* orig, const float* dir,
                                                           float* dist, float* nrm, int* model) {
    __shared__ int s_stack[ACCEL != ACCEL_GRID ? kStack * kBlock : 1];
    __shared__ int4 s_hs[ACCEL == ACCEL_GRID_FAST ? kHitCap * kBlock : 1];
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const Hit h = intersect_scene<ACCEL, kBlock>(p, mk3(orig[3 * i], orig[3 * i + 1], orig[3 * i + 2]),
                                         mk3(dir[3 * i], dir[3 * i + 1], dir[3 * i + 2]), s_stack + threadIdx.x,
                                         s_hs + threadIdx.x);
    dist[i] = h.dist;
    nrm[3 * i] = h.n.x; nrm[3 * i + 1] = h.n.y; nrm[3 * i + 2] = h.n.z;
    model[i] = h.model;
}

// Dense slot j of bounce `bounce` -> its index in the ray pool written by the
// previous bounce (block-local compaction + k_scan offsets).
__device__ __forceinline__ int slot_source(const KParams& p, int j) {
    const int chunk = j / p.chunk;
    int lo = p.dst_start[chunk], hi = p.dst_start[chunk + 1];
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (p.blk_off[mid] <= j) lo = mid; else hi = mid - 1;
    }
    return lo * p.chunk + (j - p.blk_off[lo]);
}

// Persistent BLAS trace for one bounce (ACCEL_BVH): computeRaySceneIntersectionKernel
// (Renderer.cpp:363-409) for every live slot, result-identical to
// intersect_scene<ACCEL_BVH>, written to the hit buffer the shading pass reads.
// Each lane runs its own ray through (model select -> node visits -> leaf
// triangles) one step per loop iteration and takes a new ray when its ray is
// done, so a wave's lanes stay busy instead of idling behind the wave's
// longest ray (secondary rays are incoherent).  Work is claimed per source
// block of the previous bounce (one atomic per <= chunk rays): block b's
// survivors sit at [b*chunk, b*chunk + cnt_b) and own dense slots
// [blk_off[b], blk_off[b] + cnt_b), so no slot->source search is needed.
// Every wave exits once all blocks are claimed and its lanes are idle.
// Per-lane traversal stack: kStack entries in LDS (lane-contiguous), deeper
// entries in a global spill area laid out lane-minor (p.spill_stride lanes).
// The seven float4 loads of a 4-wide node visit (Bvh4Node: planes lo x/y/z, hi x/y/z,
// links; count is never read): each axis' near and far planes by the slope sign's
// offset o* (0 or 3).  PT_NODE_OFF32: 32-bit byte offsets from the node array's base,
// so the loads take the SGPR base + 32-bit VGPR offset form (one 32-bit add per
// plane instead of a 64-bit address each; the BLAS is < 4 GB: leaf entries cap a
// mesh at 2^26 triangles).
#ifndef PT_NODE_OFF32
#define PT_NODE_OFF32 1
#endif
#if PT_NODE_OFF32
#define PT_NODE_LOADS(cur, ox, oy, oz)                                                                   \
    const char* __restrict__ nb_ = reinterpret_cast<const char*>(p.bvh4);                                \
    const unsigned nbo_ = (unsigned)(cur) << 7;                                                          \
    auto ld4_ = [&](int q) { return *reinterpret_cast<const float4*>(nb_ + (nbo_ + 16u * (unsigned)q)); }; \
    const float4 NX = ld4_(ox), NY = ld4_(1 + (oy)), NZ = ld4_(2 + (oz));                                \
    const float4 FX = ld4_(3 - (ox)), FY = ld4_(4 - (oy)), FZ = ld4_(5 - (oz));                          \
    const float4 LKf = ld4_(6);
#else
#define PT_NODE_LOADS(cur, ox, oy, oz)                                                                   \
    const float4* __restrict__ n4 = reinterpret_cast<const float4*>(p.bvh4) + 8 * (size_t)(cur);         \
    const float4 NX = n4[ox], NY = n4[1 + (oy)], NZ = n4[2 + (oz)];                                      \
    const float4 FX = n4[3 - (ox)], FY = n4[4 - (oy)], FZ = n4[5 - (oz)];                                \
    const float4 LKf = n4[6];
#endif

template <int BS, int SCAP = kStack>
__device__ __forceinline__ void spush_t(int* stack, int* spill, int stride, int sp, int e) {
    if (sp < SCAP) stack[sp * BS] = e;
    else spill[(sp - SCAP) * stride] = e;     // 32-bit: allocPipe keeps the spill area under 2^31 entries
}
// Pop for the lanes with `take`, without a branch around the LDS read: every lane
// reads its (clamped) LDS entry; only a spilled entry is read under a branch.
template <int BS, int SCAP = kStack>
__device__ __forceinline__ int spop_if(bool take, const int* stack, const int* spill, int stride, int sp) {
    typedef __attribute__((address_space(3))) const int lds_int;
    typedef __attribute__((address_space(1))) const int glb_int;
    int v = ((lds_int*)stack)[min(max(sp, 0), SCAP - 1) * BS];
    if (take & (sp >= SCAP)) v = ((glb_int*)spill)[(sp - SCAP) * stride];
    return v;
}

#ifndef PT_LEAF_REL
#define PT_LEAF_REL 1         // 4-wide leaf links relative to ModelRec::leaf_base (0: absolute; timing experiments)
#endif
#ifndef PT_EMPTY_SKIP
#define PT_EMPTY_SKIP 1       // the traces' select steps skip models whose mesh has no triangles
#endif
#ifndef PT_LEAF_STEP
#define PT_LEAF_STEP 2        // leaf triangles tested per leaf step of k_trace_bvh (1..4; k_trace_gf: 1 or 2)
#endif
#ifndef PT_BVH_NODE_STEP
#define PT_BVH_NODE_STEP 4    // k_trace_bvh: node visits per node step (as PT_NODE_STEP)
#endif
#ifndef PT_BVH_SEL_MASK
#define PT_BVH_SEL_MASK 1     // k_trace_bvh: PT_SEL_MASK's candidate mask for the main launch's select steps
#endif
#ifndef PT_BVH_LEAF_W
#define PT_BVH_LEAF_W 4       // k_trace_bvh phase weights (x/4) of leaf and select lane counts against node's
#endif
#ifndef PT_BVH_SEL_W
#define PT_BVH_SEL_W 4
#endif
#ifndef PT_BVH_MINWAVES
#define PT_BVH_MINWAVES 4     // waves per SIMD the k_trace_bvh register allocation must allow (4-wide nodes: 4 waves, no spills, +7 % over 5 with 7 spilled)
#endif
// Model records staged in LDS when the scene has at most this many: k_trace_gf
// 8 (7168 B of lane state + 8 x 248 B = 9152 B per 64-lane workgroup), or 12 for
// scenes of 9..12 instances (variant F | 32: 10144 B, still 16 per CU; the
// smaller table leaves LDS room beside 16 trace workgroups for the other
// pipelines' small kernels: 1 % at configs[1]); k_trace_bvh 8 (6144 + 8 x 248
// = 8128 B, 20 per CU), 12 with F | 32 (9120 B, 17 per CU).
#ifndef PT_LDS_MODELS_GF
#define PT_LDS_MODELS_GF 8
#endif
#ifndef PT_LDS_MODELS_BVH
#define PT_LDS_MODELS_BVH 8
#endif
constexpr int kLdsModels = PT_LDS_MODELS_BVH;
constexpr int kLdsModelsWide = 12;
constexpr int kLdsModelsGf = PT_LDS_MODELS_GF;
constexpr int kSpillEntries = 64;  // traversal-stack entries per lane beyond the LDS part (global spill)
// a leaf child pushed on a 4-wide traversal stack (negative: told apart from node indices)
__device__ __forceinline__ int leaf_entry4(int first, int count) {
    return (int)(0x80000000u | ((unsigned)count << kLeafCountShift) | (unsigned)first);
}

// Drain continuations.  Once a persistent trace's pool is exhausted its waves
// empty out: every lane whose ray is done idles until the wave's longest ray
// finishes, and at 16 pipelines those half-empty waves hold the wave slots the
// other pipelines' kernels wait for (35 % of trace wave-iterations ran after
// exhaustion with 8.5 of 64 lanes busy).  So a wave that has at most
// drain_dump busy lanes left writes each busy lane's exact traversal state to
// a continuation record and exits; a second, "tail" launch of the same kernel
// resumes the records packed 64 to a wave.  Only which lane runs a ray and
// when changes, so every result is unchanged.  Records are SoA: field f of
// record r at cont[f * cont_cap + r] (coalesced per wave).  Model-space values
// (o, d, 1/d, node slopes) are recomputed on resume with the same operations.
enum {
    kCJ = 0, kCState, kCIm, kCGdist, kCGmodel, kCGtri, kCOw, kCDw = kCOw + 3, kCCur = kCDw + 3, kCSp, kCLfI, kCLfE,
    kCLf2I, kCLf2E, kCLfNext, kCSpill, kCX      // kernel-specific fields from kCX on
};
constexpr int kContFields = 57;

// F (compile-time variant): 1 = model records in LDS, 32 = room for 12 of them
// (bits 2 and 8 -- leaf triangles as their own steps, phase scheduling -- are
// always set: the variants without them measured slower and were removed).
// TAIL: the tail launch, which resumes drain continuations instead of claiming rays.
template <int BS, int F, bool TAIL = false>
__global__ __launch_bounds__(BS, PT_BVH_MINWAVES) void k_trace_bvh(KParams p, int bounce, int level) {
    static_assert(kCX + 3 + kStack <= kContFields, "continuation record too small");
    __shared__ int s_stack[kStack * BS];
    // F & 32: room for kLdsModelsWide records (scenes of 9..12 models: 17 resident waves per CU
    // instead of 20, but no model reads from global memory: README scene +6 %)
    constexpr int kModelsHere = (F & 1) ? ((F & 32) ? kLdsModelsWide : kLdsModels) : 1;
    __shared__ ModelRec s_models[kModelsHere];
    int* stack = s_stack + threadIdx.x;
    // the 4-wide traversal (up to three pushes per node) spills past kStack entries to this
    // lane's global area
    static_assert(3 * (kMaxBvhDepth + 1) + 1 <= kStack + kSpillEntries,
                  "k_trace_bvh's 4-wide traversal stack (LDS + spill) too small");
    int sbase = (int)(blockIdx.x * BS + threadIdx.x);   // this lane's spill area (a resumed ray brings its own)
    int* spill = p.spill + sbase;
    // level 0: the main launch; level l >= 1: the tail launch resuming level l - 1's records
    const size_t cfield = (size_t)p.cont_cap * kContFields;        // one record buffer
    const int* cin = p.cont + (size_t)((level - 1) & 1) * cfield;   // records this (tail) launch resumes
    int* cout = p.cont + (size_t)(level & 1) * cfield;              // records it hands on
    const bool may_dump = level < p.drain_levels;
    const int ncont = TAIL ? p.cont_count[level - 1] : 0;
    if (TAIL && (int)blockIdx.x * BS >= ncont) return;  // more waves than records (uniform per block)
    if (TAIL && p.tail_rpl > 1 && (int)blockIdx.x >= (ncont + BS * p.tail_rpl - 1) / (BS * p.tail_rpl)) return;
    // Sparse bounces: a main launch whose rays come to fewer than trace_rpl per lane runs only
    // as many waves as give each lane that many (the rest exit at once), so fewer waves pay
    // the drain -- the wait on each wave's slowest rays once the claim counter runs out.
    if (!TAIL && p.trace_rpl > 0) {
        const int n_b = p.n_live[bounce];
        if ((int)blockIdx.x >= max(p.trace_min_blocks, (n_b + BS * p.trace_rpl - 1) / (BS * p.trace_rpl))) return;
    }
    // F & 1 is launched only when the scene has at most kLdsModels models: the
    // choice is compile-time, so model reads are ds_read (LDS) or global loads,
    // never flat loads through a generic pointer.
    constexpr bool lds_models = (F & 1) != 0;
    if (lds_models) {
        const int* src = reinterpret_cast<const int*>(p.models);
        int* dst = reinterpret_cast<int*>(s_models);
        const int nw = min(p.nmodels, kModelsHere) * (int)(sizeof(ModelRec) / 4);
        for (int i = threadIdx.x; i < nw; i += BS) dst[i] = src[i];
        __syncthreads();
    }
    const ModelRec* models = lds_models ? s_models : p.models;
    const int in_buf = (bounce + 1) & 1;
    const int lane = threadIdx.x & 63;
    const int n = p.n_live[bounce];
    // lane state: 0 = needs a ray, 1 = select next model, 2 = node visits, 4 = leaf triangles, 3 = no more rays
    int state = 0;
    int j = -1;
    f3 ow = mk3(0, 0, 0), dw = mk3(0, 0, 0), winv = mk3(0, 0, 0);
    float dlen = 0.0f, gdist = kFMax;
    int gmodel = -1, gtri = -1, im = -1;
    f3 o = mk3(0, 0, 0), d = mk3(0, 0, 0), ninv = mk3(0, 0, 0);
    int cur = 0, sp = 0, best_tri = -1;
    int lf_i = 0, lf_e = 0, lf2_i = 0, lf2_e = 0;    // pending leaves: [lf_i, lf_e) then [lf2_i, lf2_e)
    int lbase = 0;                                  // ModelRec::leaf_base of the model being traced
    int lf_next = -1;                               // then node lf_next (-1: pop the stack)
    float best = kFMax;
    bool any = false, exhausted = false;
    // PT_BVH_SEL_MASK: the main launch's select steps jump to the next model a ray can reach
    // (k_trace_gf's PT_SEL_MASK; the miss test once per ray, the gdist test per candidate)
    constexpr bool kSelMask = PT_BVH_SEL_MASK && !TAIL && (F & 1);
    unsigned cmask = ~0u;
    unsigned long long st_iter = 0, st_node = 0, st_leaf = 0, st_sel = 0;   // PT_DEBUG_ABLATE & 16
    unsigned long long st_busy = 0, st_drain = 0, st_drain_busy = 0;       // busy lanes; iterations after exhaustion
    unsigned long long it_node = 0, it_leaf = 0, it_sel = 0;
    for (unsigned iters = 0;; iters++) {
        unsigned long long idle = __ballot(state == 0);
        const unsigned long long busy = __ballot(state != 0 && state != 3);
        if (idle && !exhausted && (busy == 0 || __popcll(idle) >= (TAIL ? p.tail_refill : p.trace_refill))) {
            if (TAIL) {                                     // resume continuation records
                const int cnt = __popcll(idle);
                const int leader = __ffsll((long long)idle) - 1;
                int base = 0;
                if (lane == leader) base = atomicAdd(p.cont_next + level - 1, cnt);
                base = __builtin_amdgcn_readlane(base, leader);   // uniform: SGPR
                if (base + cnt >= ncont) exhausted = true;
                if (state == 0) {
                    const int r = base + __popcll(idle & ((1ull << lane) - 1ull));
                    if (r < ncont) {
                        const int* C = cin + r;
                        const size_t cs = (size_t)p.cont_cap;
                        j = C[kCJ * cs]; state = C[kCState * cs]; im = C[kCIm * cs];
                        gdist = __int_as_float(C[kCGdist * cs]); gmodel = C[kCGmodel * cs]; gtri = C[kCGtri * cs];
                        ow = mk3(__int_as_float(C[kCOw * cs]), __int_as_float(C[(kCOw + 1) * cs]),
                                 __int_as_float(C[(kCOw + 2) * cs]));
                        dw = mk3(__int_as_float(C[kCDw * cs]), __int_as_float(C[(kCDw + 1) * cs]),
                                 __int_as_float(C[(kCDw + 2) * cs]));
                        cur = C[kCCur * cs]; sp = C[kCSp * cs];
                        lf_i = C[kCLfI * cs]; lf_e = C[kCLfE * cs]; lf2_i = C[kCLf2I * cs]; lf2_e = C[kCLf2E * cs];
                        lf_next = C[kCLfNext * cs];
                        sbase = C[kCSpill * cs]; spill = p.spill + sbase;
                        best = __int_as_float(C[kCX * cs]); best_tri = C[(kCX + 1) * cs]; any = C[(kCX + 2) * cs] != 0;
                        // the live stack entries only, four loads in flight at a time (one wait per four)
#pragma unroll 1
                        for (int q0 = 0; q0 < min(sp, kStack); q0 += 4) {
                            int v[4];
#pragma unroll
                            for (int k = 0; k < 4; k++) v[k] = C[(kCX + 3 + min(q0 + k, kStack - 1)) * cs];
#pragma unroll
                            for (int k = 0; k < 4; k++) if (q0 + k < kStack) stack[(q0 + k) * BS] = v[k];
                        }
                        winv = node_inv(cull_inv(dw));
                        dlen = sqrtf(dot(dw, dw));
                        if (state != 1) {                   // inside model im: its model-space ray, as selected
                            const ModelRec& M = models[im];
                            lbase = M.leaf_base;
                            o = xform12(M.w2m, ow, 1.0f);
                            d = normalize(xform12(M.w2m, dw, 0.0f));
                            const f3 inv = mk3(1 / d.x, 1 / d.y, 1 / d.z);
                            ninv = node_inv(inv);
                        }
                    } else {
                        state = 3;
                    }
                }
            } else {
                const int cnt = __popcll(idle);
                const int leader = __ffsll((long long)idle) - 1;
                int base = 0;
                if (lane == leader) base = atomicAdd(p.trace_next, cnt);
                base = __builtin_amdgcn_readlane(base, leader);   // uniform: SGPR
                if (base + cnt >= n) exhausted = true;
                if (state == 0) {
                    j = base + __popcll(idle & ((1ull << lane) - 1ull));
                    if (j < n) {
                        int src;
                        if (p.order) { const int2 e = p.order[j]; j = e.x; src = e.y; }   // sorted claim order
                        else src = slot_source(p, j);
                        const float4 a = p.ray[in_buf][0][src];
                        const float4 b = p.ray[in_buf][1][src];
                        ow = mk3(a.x, a.y, a.z);
                        dw = mk3(b.x, b.y, b.z);
                        winv = node_inv(cull_inv(dw));
                        dlen = sqrtf(dot(dw, dw));
                        gdist = kFMax; gmodel = -1; gtri = -1; im = -1;
                        cmask = ~0u;
                        state = 1;
                    } else {
                        state = 3;
                    }
                }
            }
        }
        if (exhausted && state == 0) state = 3;
        if (__ballot(state != 3) == 0) break;
        // safety net: never spin forever (reported as a fault); checked every 16th iteration, so
        // the cap's kernel-argument load stays out of the loop's common path
        if ((iters & 15u) == 0 && iters > p.trace_iter_cap) {
            if (lane == 0) atomicAdd(p.segments + kTraceFaultCounter, 1ull);
            break;
        }
        // Phase scheduling: one step kind per iteration -- the one most lanes are
        // waiting in -- so the wave never pays for three partly used blocks.
        int phase = 2;
        {
            const int c1 = __popcll(__ballot(state == 1)), c2 = __popcll(__ballot(state == 2)),
                      c4 = __popcll(__ballot(state == 4));
            int cm = c2;
            if (c4 * 4 > cm * PT_BVH_LEAF_W) { phase = 4; cm = c4; }
            if (c1 * 4 > cm * PT_BVH_SEL_W) phase = 1;
        }
        // drain: at most drain_dump lanes still trace once the pool is exhausted
        {
            const int dd = TAIL ? p.drain_dump_tail : p.drain_dump;
            if (may_dump && exhausted && dd > 0 && __popcll(__ballot(state != 3)) <= dd) phase = 16;
        }
        phase = __builtin_amdgcn_readfirstlane(phase);   // wave-uniform: scalar branches on it
        if (PT_TRACE_STATS && (p.debug & 16)) {       // lane-steps executed per phase, and phase iterations
            st_iter++;
            {
                const unsigned long long nb_ = __popcll(__ballot(state != 0 && state != 3));
                st_busy += nb_;
                if (exhausted) { st_drain++; st_drain_busy += nb_; }
            }
            if (phase & 2) { st_node += __popcll(__ballot(state == 2)); it_node++; }
            if (phase & 4) { st_leaf += __popcll(__ballot(state == 4)); it_leaf++; }
            if (phase & 1) { st_sel += __popcll(__ballot(state == 1)); it_sel++; }
        }
        if (phase & 16) {
            // drain continuation: every busy lane's exact state, then the wave is done
            const unsigned long long bm = __ballot(state != 3);
            const int nbusy = __popcll(bm);
            const int leader = __ffsll((long long)bm) - 1;
            int base = 0;
            if (lane == leader) base = atomicAdd(p.cont_count + level, nbusy);
            base = __builtin_amdgcn_readlane(base, leader);   // uniform: SGPR
            if (state != 3) {
                int* C = cout + base + __popcll(bm & ((1ull << lane) - 1ull));
                const size_t cs = (size_t)p.cont_cap;
                C[kCJ * cs] = j; C[kCState * cs] = state; C[kCIm * cs] = im;
                C[kCGdist * cs] = __float_as_int(gdist); C[kCGmodel * cs] = gmodel; C[kCGtri * cs] = gtri;
                C[kCOw * cs] = __float_as_int(ow.x); C[(kCOw + 1) * cs] = __float_as_int(ow.y);
                C[(kCOw + 2) * cs] = __float_as_int(ow.z);
                C[kCDw * cs] = __float_as_int(dw.x); C[(kCDw + 1) * cs] = __float_as_int(dw.y);
                C[(kCDw + 2) * cs] = __float_as_int(dw.z);
                C[kCCur * cs] = cur; C[kCSp * cs] = sp;
                C[kCLfI * cs] = lf_i; C[kCLfE * cs] = lf_e; C[kCLf2I * cs] = lf2_i; C[kCLf2E * cs] = lf2_e;
                C[kCLfNext * cs] = lf_next; C[kCSpill * cs] = sbase;
                C[kCX * cs] = __float_as_int(best); C[(kCX + 1) * cs] = best_tri; C[(kCX + 2) * cs] = any ? 1 : 0;
#pragma unroll 1
                for (int q = 0; q < min(sp, kStack); q++) C[(kCX + 3 + q) * cs] = stack[q * BS];
            }
            state = 3;
        }
        if ((phase & 1) && state == 1) {                // advance to the next model that survives culling
            if (kSelMask && cmask == ~0u) {
                cmask = 0;
                for (int m = 0; m < p.nmodels; m++) {
                    float wtn, wtf;
                    node_slab(models[m].wbox, models[m].wbox + 3, ow, winv, wtn, wtf);
                    cmask |= ((wtn > wtf) | (wtf * dlen < -1.0f)) ? 0u : 1u << m;
                }
            }
            for (;;) {
                if (kSelMask) {
                    const unsigned rest = cmask >> (im + 1);
                    im = rest ? im + __ffs(rest) : p.nmodels;
                } else {
                    im++;
                }
                if (im >= p.nmodels) {
                    put_hit(p, j, gdist, gmodel, gtri);
                    state = 0;
                    break;
                }
                const ModelRec& M = models[im];
                if (kSelMask) {
                    float wtn, wtf;
                    node_slab(M.wbox, M.wbox + 3, ow, winv, wtn, wtf);
                    if (wtn * dlen > gdist * 1.0001f + 0.01f) continue;
                } else if (model_culled<ACCEL_BVH>(M, ow, dw, winv, dlen, gdist)) continue;
                if (PT_EMPTY_SKIP && M.bvh4_root < 0) continue;   // a mesh without triangles: no hit, no BLAS
                o = xform12(M.w2m, ow, 1.0f);
                d = normalize(xform12(M.w2m, dw, 0.0f));
                const f3 inv = mk3(1 / d.x, 1 / d.y, 1 / d.z);
                ninv = node_inv(inv);
                cur = M.bvh4_root;
                lbase = M.leaf_base;
                sp = 0;
                best = kFMax;
                best_tri = -1;
                any = false;
                state = 2;
                break;
            }
        }
        bool model_done = false;
        if ((phase & 4) && state == 4) {                // leaf triangles: up to PT_LEAF_STEP per iteration
            // the step's triangle loads are issued together (one memory round trip);
            // the (t, index) minimum does not depend on the order of the tests
            float4 TA[PT_LEAF_STEP], TB[PT_LEAF_STEP], TC[PT_LEAF_STEP];
#pragma unroll
            for (int q = 0; q < PT_LEAF_STEP; q++) {
                const int iq = lf_i + q < lf_e ? lf_i + q : lf_i;
                TA[q] = p.bvh_tri_geom[3 * iq]; TB[q] = p.bvh_tri_geom[3 * iq + 1]; TC[q] = p.bvh_tri_geom[3 * iq + 2];
            }
#pragma unroll
            for (int q = 0; q < PT_LEAF_STEP; q++) {
                if (lf_i + q >= lf_e) break;
                const int it = __float_as_int(TA[q].w);
                float t;
                if (tri_test_rec(TA[q], TB[q], TC[q], o, d, t)) {
                    any = true;
                    if (t < best || (t == best && it < best_tri)) { best = t; best_tri = it; }
                }
            }
            lf_i = min(lf_i + PT_LEAF_STEP, lf_e);
            {
            // end of the leaf: the next stack entry, a leaf (encoded, < 0) or a node
            const bool end = lf_i == lf_e;
            const bool pop = end & (sp > 0);
            model_done = end & (sp == 0);
            const int top = spop_if<BS, kStack>(pop, stack, spill, p.spill_stride, sp - 1);
            sp -= pop ? 1 : 0;
            const bool tleaf = pop & (top < 0);
            const int first = (PT_LEAF_REL ? lbase : 0) + (top & ((1 << kLeafCountShift) - 1));   // mesh-relative entry
            lf_e = tleaf ? first + ((top >> kLeafCountShift) & kMaxLeafCount4) : lf_e;
            lf_i = tleaf ? first : lf_i;
            cur = (pop & !tleaf) ? top : cur;
            state = (pop & !tleaf) ? 2 : state;
            }
        } else if ((phase & 2) && state == 2) {   // 4-wide node steps
#pragma unroll 1
            for (int ks = 0; ks < PT_BVH_NODE_STEP; ks++) {
                // 4-wide node visits: every hit child in order of entry, nearest first
                // each axis' near / far planes by the slope's sign (as k_trace_gf): the same entry /
                // exit values as node_slab's min / max, without them; empty slots (inverted
                // infinite boxes) miss by themselves
                const int ox = ninv.x < 0.0f ? 3 : 0, oy = ninv.y < 0.0f ? 3 : 0, oz = ninv.z < 0.0f ? 3 : 0;
                PT_NODE_LOADS(cur, ox, oy, oz)
                const float pnx[4] = {NX.x, NX.y, NX.z, NX.w}, pny[4] = {NY.x, NY.y, NY.z, NY.w};
                const float pnz[4] = {NZ.x, NZ.y, NZ.z, NZ.w}, pfx[4] = {FX.x, FX.y, FX.z, FX.w};
                const float pfy[4] = {FY.x, FY.y, FY.z, FY.w}, pfz[4] = {FZ.x, FZ.y, FZ.z, FZ.w};
                const int lk[4] = {__float_as_int(LKf.x), __float_as_int(LKf.y), __float_as_int(LKf.z),
                                   __float_as_int(LKf.w)};
                const f3 oi = o * ninv;
                float key[4];
                int ent[4];
                int nhit = 0;
#pragma unroll
                for (int c = 0; c < 4; c++) {
                    // node_slab on each of the four boxes, bvh_step's hit rule
                    const float tn = fmaxf(fmaxf(__builtin_fmaf(pnx[c], ninv.x, -oi.x), __builtin_fmaf(pny[c], ninv.y, -oi.y)),
                                           __builtin_fmaf(pnz[c], ninv.z, -oi.z));
                    const float tf = fminf(fminf(__builtin_fmaf(pfx[c], ninv.x, -oi.x), __builtin_fmaf(pfy[c], ninv.y, -oi.y)),
                                           __builtin_fmaf(pfz[c], ninv.z, -oi.z));
                    const bool h = (tn <= tf) & (tf >= -kEps) & (tn <= best);
                    key[c] = h ? tn : __int_as_float(0x7f800000);
                    ent[c] = lk[c];                          // leaves come encoded (Bvh4Node)
                    nhit += h ? 1 : 0;
                }
                auto cas = [&](int a, int b) {
                    const bool sw = key[b] < key[a];
                    const float ka = key[a], kb = key[b];
                    const int ea = ent[a], eb = ent[b];
                    key[a] = sw ? kb : ka; key[b] = sw ? ka : kb;
                    ent[a] = sw ? eb : ea; ent[b] = sw ? ea : eb;
                };
                cas(0, 1); cas(2, 3); cas(0, 2); cas(1, 3); cas(1, 2);
                if (nhit > 3) { spush_t<BS, kStack>(stack, spill, p.spill_stride, sp, ent[3]); sp++; }
                if (nhit > 2) { spush_t<BS, kStack>(stack, spill, p.spill_stride, sp, ent[2]); sp++; }
                if (nhit > 1) { spush_t<BS, kStack>(stack, spill, p.spill_stride, sp, ent[1]); sp++; }
                const bool pop = (nhit == 0) & (sp > 0);
                const int top = spop_if<BS, kStack>(pop, stack, spill, p.spill_stride, sp - 1);
                model_done = (nhit == 0) & (sp == 0);
                sp -= pop ? 1 : 0;
                const int nx = nhit > 0 ? ent[0] : top;
                const bool leaf = !model_done & (nx < 0);
                const int first = (PT_LEAF_REL ? lbase : 0) + (nx & ((1 << kLeafCountShift) - 1));
                lf_i = leaf ? first : lf_i;
                lf_e = leaf ? first + ((nx >> kLeafCountShift) & kMaxLeafCount4) : lf_e;
                cur = (!model_done & !leaf) ? nx : cur;
                state = leaf ? 4 : state;
                if (state != 2 || model_done) break;
            }
        }
        if (model_done) {
            state = 1;
            if (any) {
                const float dd = model_hit_dist(models[im], o, d, best, ow);
                if (gdist > dd) { gdist = dd; gmodel = im; gtri = best_tri; }
            }
        }
    }
    if ((PT_TRACE_STATS && (p.debug & 16)) && lane == 0) {
        atomicAdd(p.segments + 8 + kMaxBounceCounters, st_iter);
        if (TAIL) {                                 // the tail launches' share (slots 15, 43)
            atomicAdd(p.segments + 15 + kMaxBounceCounters, st_iter);
            atomicAdd(p.segments + 43 + kMaxBounceCounters, st_busy);
        }
        atomicAdd(p.segments + 44 + kMaxBounceCounters, st_drain);
        atomicAdd(p.segments + 45 + kMaxBounceCounters, st_drain_busy);
        atomicAdd(p.segments + 46 + kMaxBounceCounters, st_busy);
        atomicAdd(p.segments + 9 + kMaxBounceCounters, st_node);
        atomicAdd(p.segments + 10 + kMaxBounceCounters, st_leaf);
        atomicAdd(p.segments + 12 + kMaxBounceCounters, st_sel);
        atomicAdd(p.segments + 16 + kMaxBounceCounters, it_node);
        atomicAdd(p.segments + 17 + kMaxBounceCounters, it_leaf);
        atomicAdd(p.segments + 19 + kMaxBounceCounters, it_sel);
    }
}

// Persistent grid_fast trace for one bounce: the results of
// computeRayGridIntersection (Renderer.cpp:238-360) computed as grid_hitset
// does, for every live slot, written to the hit buffer the shading pass reads.
// Same skeleton as k_trace_bvh: each lane advances its own ray one step per
// loop iteration -- select the next model (instance culling, model-space
// transform, the grid's bounding-box entry test), visit one BLAS node of the
// bounded hit-set collection, test one leaf triangle, or run the whole DDA walk
// of a collected hit set (fast-forwarded to the members' union box, so a walk
// is a few voxels) -- and the wave runs only the step kind most lanes wait in.
// A walk that is not provably exact restarts the collection with the next
// tier's window (W, 2R, unbounded), in place.  A hit set that overflows the
// kGfHitCap LDS entries defers the whole ray to k_trace_deferred (the fused
// path's tiers with the global pool).  LDS per lane: kGfStack stack entries
// (deeper entries spill to global memory) + kGfHitCap hit-set members.
#ifndef PT_GF_STACK
#define PT_GF_STACK 12
#endif
#ifndef PT_GF_HITCAP
#define PT_GF_HITCAP 4
#endif
#ifndef PT_WALK_W
#define PT_WALK_W 8           // k_trace_gf: the walk phase runs when its lanes outnumber the largest other phase's x W/4
#endif
#ifndef PT_LEAF_W
#define PT_LEAF_W 3           // ... and the leaf phase when they exceed node's x 3/4 (select: x PT_SEL_W/4)
#endif
#ifndef PT_SEL_W
#define PT_SEL_W 4
#endif
#ifndef PT_GF_MINWAVES
#define PT_GF_MINWAVES 4      // waves per SIMD the register allocation must allow
#endif
#ifndef PT_GF_TAIL_MINWAVES
#define PT_GF_TAIL_MINWAVES 4 // the same for the tail launches (k_trace_gf<..., TAIL = true>)
#endif
#ifndef PT_LDS_TOP
#define PT_LDS_TOP 0          // k_trace_gf: top 4-wide nodes per mesh staged in LDS (experiment; 0 = off)
#endif
#ifndef PT_LDS_TOP_MESHES
#define PT_LDS_TOP_MESHES 2   // ... of the largest one or two meshes
#endif
constexpr int kGfStack = PT_GF_STACK, kGfHitCap = PT_GF_HITCAP, kLdsTop = PT_LDS_TOP, kLdsTopMeshes = PT_LDS_TOP_MESHES;
// 4-wide traversal: at most 3 pushes per node on a path of at most kMaxBvhDepth + 1 nodes (an unopened
// slot keeps its binary level, so a 4-wide path can be as long as a binary one)
static_assert(3 * (kMaxBvhDepth + 1) + 1 <= kGfStack + kSpillEntries,
              "k_trace_gf's 4-wide traversal stack (LDS + spill) too small");

// Test hook: the walk certificates against the exact walk on the same hit set.
// k_trace_gf's main launch decides most walks by walk_certify_fast (and, where it
// declines, walk_certify) without stepping the DDA; this kernel runs both on the
// hit set of every model an arbitrary world-space ray enters (grid_hitset's entry
// test), collected as the bounded first tier (window wdelta) and as the unbounded
// last tier, with the members in registers exactly as k_trace_gf holds them, and
// compares every certificate that accepts with hitset_walk_g's stepped result
// (no certificate, STRICT as in k_trace_gf): hit, minimum t, triangle and
// finality must all agree.  out[i] = (fast tried, fast accepted, fast accepted but
// wrong, full accepted but wrong), summed over the ray's models and both tiers.
__global__ __launch_bounds__(kBlock) void k_certify_check(KParams p, int n, const float* orig, const float* dir,
                                                         int4* out) {
    __shared__ int s_stack[kStack * kBlock];
    __shared__ int4 s_hs[kHitCap * kBlock];
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    int* stack = s_stack + threadIdx.x;
    int4* hs = s_hs + threadIdx.x;
    const f3 ow = mk3(orig[3 * i], orig[3 * i + 1], orig[3 * i + 2]);
    const f3 dw = mk3(dir[3 * i], dir[3 * i + 1], dir[3 * i + 2]);
    int tried = 0, fast_ok = 0, fast_bad = 0, full_bad = 0;
    for (int im = 0; im < p.nmodels; im++) {
        const ModelRec& M = p.models[im];
        const f3 o = xform12(M.w2m, ow, 1.0f);
        const f3 d = normalize(xform12(M.w2m, dw, 0.0f));
        const f3 inv = mk3(1 / d.x, 1 / d.y, 1 / d.z);
        float t_box;
        if (!slab_ref(M.bbox, o, d, inv, t_box)) continue;
        const f3 pt = o + d * t_box;
        if ((pt.x - M.bbox[0]) < -kEps || (pt.y - M.bbox[1]) < -kEps || (pt.z - M.bbox[2]) < -kEps) continue;
        const f3 ninv = node_inv(inv);
        const bool exact_inv = (absr(ninv.x) < 1e30f) & (absr(ninv.y) < 1e30f) & (absr(ninv.z) < 1e30f);
        for (int tier = 0; tier < 2; tier++) {
            const float win = tier == 0 ? M.wdelta : 3.0e38f;
            float tmin;
            const int nh = tier == 0 ? bvh_collect<kBlock, true>(p, M, o, d, ninv, stack, hs, &tmin, win + M.reach)
                                     : bvh_collect<kBlock, false>(p, M, o, d, ninv, stack, hs, &tmin, 3.0e38f);
            if (nh <= 0 || nh > kGfHitCap) continue;     // k_trace_gf certifies LDS-held sets only
            int4 mem[kGfHitCap];
#pragma unroll
            for (int h = 0; h < kGfHitCap; h++) mem[h] = h < nh ? hs[h * kBlock] : make_int4(0, 0, 0, 0);
            auto get = [&](int h) { return mem[h]; };
            const WalkResult w = hitset_walk_g<kGfHitCap, decltype(get), false, true>(p, M, d, inv, pt, t_box,
                                                                                         get, nh, tmin, win);
            auto agrees = [&](int tri) {
                const bool final_ = tier == 1 || w.final_min || w.tw < tmin + win;
                return w.hit && w.has_best && w.t == tmin && w.tri == tri && final_;
            };
            int tri = -1;
            if (exact_inv) {
                tried++;
                if (walk_certify_fast<kGfHitCap>(p, M, d, ninv, pt, t_box, get, nh, tmin, win, tri)) {
                    fast_ok++;
                    if (!agrees(tri)) fast_bad++;
                }
            }
            tri = -1;
            if (walk_certify<kGfHitCap>(p, M, d, inv, pt, t_box, get, nh, tmin, win, tri) && !agrees(tri))
                full_bad++;
        }
    }
    out[i] = make_int4(tried, fast_ok, fast_bad, full_bad);
}

// Collection window of k_trace_gf, on voxel boxes instead of the reach R: the
// walk can enter member h's voxel box before X = t_min + window only if the
// exact ray enters that box grown by ModelRec::cslack (the DDA's deviation from
// the ray) before X (+ a parameter slack).  A BLAS node can hold such a member
// only if the ray enters its box grown by one voxel + cslack per axis before X
// (a member's voxel box lies in the node box rounded out to voxels); that entry
// is the node box's per-axis entries minus (vw + cslack) * |1/d| (the G terms).
__device__ __forceinline__ float gf_slack(float x, float t_box) {
    return 1e-5f * (absr(x) + absr(t_box) + 1.0f);
}
__device__ __forceinline__ float vbox_entry(const ModelRec& M, int lo, int hi, f3 o, f3 ninv) {
    float tn = -3.0e38f;
#pragma unroll
    for (int a = 0; a < 3; a++) {
        const float oa = a == 0 ? o.x : (a == 1 ? o.y : o.z), ia = a == 0 ? ninv.x : (a == 1 ? ninv.y : ninv.z);
        const float l = M.bbox[a] + (float)((lo >> (10 * a)) & 1023) * M.vw[a] - M.cslack[a];
        const float h = M.bbox[a] + (float)(((hi >> (10 * a)) & 1023) + 1) * M.vw[a] + M.cslack[a];
        tn = fmaxf(tn, fminf((l - oa) * ia, (h - oa) * ia));
    }
    return tn;
}
__device__ __forceinline__ void node_slab_g(const float* lo, const float* hi, f3 o, f3 inv, f3 G, float& tn, float& tf,
                                            float& tnx) {
    const f3 oi = o * inv;   // hoisted out of the traversal loop by the compiler
    const float a0 = __builtin_fmaf(lo[0], inv.x, -oi.x), b0 = __builtin_fmaf(hi[0], inv.x, -oi.x);
    const float a1 = __builtin_fmaf(lo[1], inv.y, -oi.y), b1 = __builtin_fmaf(hi[1], inv.y, -oi.y);
    const float a2 = __builtin_fmaf(lo[2], inv.z, -oi.z), b2 = __builtin_fmaf(hi[2], inv.z, -oi.z);
    const float e0 = fminf(a0, b0), e1 = fminf(a1, b1), e2 = fminf(a2, b2);
    tn = fmaxf(fmaxf(e0, e1), e2);
    tf = fminf(fminf(fmaxf(a0, b0), fmaxf(a1, b1)), fmaxf(a2, b2));
    tnx = fmaxf(fmaxf(e0 - G.x, e1 - G.y), e2 - G.z);
}

template <int BS, int F, bool TAIL = false>
__global__ __launch_bounds__(BS, TAIL ? PT_GF_TAIL_MINWAVES : PT_GF_MINWAVES) void k_trace_gf(KParams p, int bounce, int level) {
    static_assert(kCX + 9 + kGfStack + 4 * kGfHitCap <= kContFields, "continuation record too small");
    __shared__ int s_stack[kGfStack * BS];
    __shared__ int4 s_hs[kGfHitCap * BS];
    constexpr int kModelsHere = (F & 1) ? ((F & 32) ? kLdsModelsWide : kLdsModelsGf) : 1;
    __shared__ ModelRec s_models[kModelsHere];
    // PT_LDS_TOP (experiment, default 0): the first kLdsTop 4-wide nodes (breadth-first: the
    // root, then level 1, ...) of the two largest meshes (KParams::top_root / top_n) in LDS
    __shared__ float4 s_top[kLdsTop > 0 ? kLdsTopMeshes * kLdsTop * 8 : 1];
    // PT_SEL_MASK: per lane, the models whose world box the ray can reach (gdist aside),
    // found once per ray so later select steps jump to the next candidate
    constexpr bool kSelMask = PT_SEL_MASK && !TAIL && (F & 1);
    // node steps: the in-place variant (F & 16: one pipeline, one launch alone on the chip)
    // measured best at 4 visits (4-wide nodes) without the minimum; the
    // hand-on variants of several pipelines at PT_NODE_STEP / PT_NODE_MINLANES
    constexpr int kNodeSteps = (F & 16) ? PT_NODE_STEP_1P : PT_NODE_STEP;
    constexpr int kNodeMinLanes = (F & 16) ? 0 : PT_NODE_MINLANES;
    int* stack = s_stack + threadIdx.x;
    int4* hs = s_hs + threadIdx.x;
    int sbase = (int)(blockIdx.x * BS + threadIdx.x);   // this lane's spill area (a resumed ray brings its own)
    int* spill = p.spill + sbase;
    // level 0: the main launch; level l >= 1: the tail launch resuming level l - 1's records
    const size_t cfield = (size_t)p.cont_cap * kContFields;        // one record buffer
    const int* cin = p.cont + (size_t)((level - 1) & 1) * cfield;   // records this (tail) launch resumes
    int* cout = p.cont + (size_t)(level & 1) * cfield;              // records it hands on
    const bool may_dump = level < p.drain_levels;
    // records: drain hand-ons at [0, nd), walk hand-ons (level 1 only) at [cont_cap - nw, cont_cap)
    const int nd = TAIL ? p.cont_count[level - 1] : 0;
    const int ncont = nd + (TAIL && level == 1 ? min(p.cont_count[kDrainLevels], p.cont_wcap) : 0);
    if (TAIL && (int)blockIdx.x * BS >= ncont) return;  // more waves than records (uniform per block)
    // a tail launch sized to its records: each lane resumes about tail_rpl of them, refilling as
    // its rays finish, so fewer waves pay the wait on their slowest resumed ray
    if (TAIL && p.tail_rpl > 1 && (int)blockIdx.x >= (ncont + BS * p.tail_rpl - 1) / (BS * p.tail_rpl)) return;
    // Sparse bounces: a main launch whose rays come to fewer than trace_rpl per lane runs only
    // as many waves as give each lane that many (the rest exit at once), so fewer waves pay
    // the drain -- the wait on each wave's slowest rays once the claim counter runs out.
    if (!TAIL && p.trace_rpl > 0) {
        const int n_b = p.n_live[bounce];
        if ((int)blockIdx.x >= max(p.trace_min_blocks, (n_b + BS * p.trace_rpl - 1) / (BS * p.trace_rpl))) return;
    }
    // F & 1 is launched only when the scene has at most kLdsModelsGf models: the
    // choice is compile-time, so model reads are ds_read (LDS) or global loads,
    // never flat loads through a generic pointer.
    constexpr bool lds_models = (F & 1) != 0;
    if (lds_models) {
        const int* src = reinterpret_cast<const int*>(p.models);
        int* dst = reinterpret_cast<int*>(s_models);
        const int nw = min(p.nmodels, kModelsHere) * (int)(sizeof(ModelRec) / 4);
        for (int i = threadIdx.x; i < nw; i += BS) dst[i] = src[i];
        __syncthreads();
    }
    if (kLdsTop > 0) {
        const float4* nodes4 = reinterpret_cast<const float4*>(p.bvh4);
        for (int i = threadIdx.x; i < kLdsTopMeshes * kLdsTop * 8; i += BS) {
            constexpr int kT = kLdsTop > 0 ? kLdsTop : 1;
            const int m = i / (kT * 8), k = (i / 8) % kT;
            s_top[i] = k < p.top_n[m] ? nodes4[8 * (size_t)(p.top_root[m] + k) + (i & 7)] : make_float4(0, 0, 0, 0);
        }
        __syncthreads();
    }
    const ModelRec* models = lds_models ? s_models : p.models;
    const int n = p.n_live[bounce];
    const int in_buf = (bounce + 1) & 1;
    const int lane = threadIdx.x & 63;
    // lane state: 0 needs a ray, 1 select model, 2 node visit, 4 leaf triangle, 5 walk, 3 no more rays,
    // 6 walk handed on (main launch), 7 walk of a resumed hand-on (certificates already declined)
    int state = 0;
    int j = -1;
    f3 ow = mk3(0, 0, 0), dw = mk3(0, 0, 0);
    float gdist = kFMax;
    int gmodel = -1, gtri = -1, im = -1;
    f3 o = mk3(0, 0, 0), d = mk3(0, 0, 0), ninv = mk3(0, 0, 0), G = mk3(0, 0, 0);
    float t_box = 0.0f, tmin = kFMax, win = 0.0f;
    int cur = 0, sp = 0, nh = 0, tier = 0;
    int pblk = -1;                                  // global pool block holding the hit set (-1: LDS)
    int lf_i = 0, lf_e = 0, lf2_i = 0, lf2_e = 0, lf_next = -1;
    int lbase = 0;                                  // ModelRec::leaf_base of the model being traced
    bool exhausted = false;
    unsigned cmask = 0;                            // PT_SEL_MASK: candidate models of the lane's ray
    unsigned long long st_iter = 0, st_node = 0, st_leaf = 0, st_walk = 0, st_sel = 0;   // PT_DEBUG_ABLATE & 16
    unsigned long long st_busy = 0, st_drain = 0, st_drain_busy = 0;       // busy lanes; iterations after exhaustion
    unsigned long long it_node = 0, it_leaf = 0, it_walk = 0, it_sel = 0;
    unsigned long long cy[6] = {0, 0, 0, 0, 0, 0};  // PT_DEBUG_ABLATE & 32: cycles in refill, select, leaf, node,
                                                    // walk (certificates), hand-on / drain records
    const bool stamps = PT_TRACE_STATS && (p.debug & 32);
    unsigned long long cyr[4] = {0, 0, 0, 0};      // refill: claim, -, order entry + ray gather, stores drained before
    unsigned long long ts = stamps ? clock64() : 0;
    for (unsigned iters = 0;; iters++) {
        unsigned long long idle = __ballot(state == 0);
        const unsigned long long busy = __ballot(state != 0 && state != 3);
        if (TAIL && idle && !exhausted && (busy == 0 || __popcll(idle) >= p.tail_refill)) {
            // resume continuation records
            const int cnt = __popcll(idle);
            const int leader = __ffsll((long long)idle) - 1;
            int base = 0;
            if (lane == leader) base = atomicAdd(p.cont_next + level - 1, cnt);
            base = __builtin_amdgcn_readlane(base, leader);   // uniform: SGPR
            if (base + cnt >= ncont) exhausted = true;
            if (state == 0) {
                const int r = base + __popcll(idle & ((1ull << lane) - 1ull));
                if (r < ncont) {
                    const int* C = cin + (r < nd ? r : p.cont_cap - 1 - (r - nd));
                    const size_t cs = (size_t)p.cont_cap;
                    j = C[kCJ * cs]; state = C[kCState * cs]; im = C[kCIm * cs];
                    gdist = __int_as_float(C[kCGdist * cs]); gmodel = C[kCGmodel * cs]; gtri = C[kCGtri * cs];
                    ow = mk3(__int_as_float(C[kCOw * cs]), __int_as_float(C[(kCOw + 1) * cs]),
                             __int_as_float(C[(kCOw + 2) * cs]));
                    dw = mk3(__int_as_float(C[kCDw * cs]), __int_as_float(C[(kCDw + 1) * cs]),
                             __int_as_float(C[(kCDw + 2) * cs]));
                    cur = C[kCCur * cs]; sp = C[kCSp * cs];
                    lf_i = C[kCLfI * cs]; lf_e = C[kCLfE * cs]; lf2_i = C[kCLf2I * cs]; lf2_e = C[kCLf2E * cs];
                    lf_next = C[kCLfNext * cs];
                    sbase = C[kCSpill * cs];
                    // a walk hand-on's traversal stack is empty: this lane's own tail area
                    if (sbase < 0) sbase = p.spill_stride / 2 + (int)(blockIdx.x * BS + threadIdx.x);
                    spill = p.spill + sbase;
                    tmin = __int_as_float(C[kCX * cs]); nh = C[(kCX + 1) * cs]; tier = C[(kCX + 2) * cs];
                    pblk = C[(kCX + 3) * cs]; win = __int_as_float(C[(kCX + 4) * cs]);
                    t_box = __int_as_float(C[(kCX + 5) * cs]);
                    G = mk3(__int_as_float(C[(kCX + 6) * cs]), __int_as_float(C[(kCX + 7) * cs]),
                            __int_as_float(C[(kCX + 8) * cs]));
                    // the live stack entries and hit-set members only (a walk hand-on has no stack; a
                    // pool-held hit set lives in its pool block), four loads in flight at a time
#pragma unroll 1
                    for (int q0 = 0; q0 < min(sp, kGfStack); q0 += 4) {
                        int v[4];
#pragma unroll
                        for (int k = 0; k < 4; k++) v[k] = C[(kCX + 9 + min(q0 + k, kGfStack - 1)) * cs];
#pragma unroll
                        for (int k = 0; k < 4; k++) if (q0 + k < kGfStack) stack[(q0 + k) * BS] = v[k];
                    }
#pragma unroll 1
                    for (int q = 0; q < (pblk < 0 ? nh : 0); q++)
                        hs[q * BS] = make_int4(C[(kCX + 9 + kGfStack + 4 * q) * cs], C[(kCX + 10 + kGfStack + 4 * q) * cs],
                                               C[(kCX + 11 + kGfStack + 4 * q) * cs], C[(kCX + 12 + kGfStack + 4 * q) * cs]);
                    if (state > 1) {                        // inside model im: its model-space ray, as selected
                        const ModelRec& M = models[im];
                        lbase = M.leaf_base;
                        o = xform12(M.w2m, ow, 1.0f);
                        d = normalize(xform12(M.w2m, dw, 0.0f));
                        const f3 inv = mk3(1 / d.x, 1 / d.y, 1 / d.z);
                        ninv = node_inv(inv);
                    }
                } else {
                    state = 3;
                }
            }
        } else if (!TAIL && idle && !exhausted && (busy == 0 || __popcll(idle) >= p.trace_refill)) {
            // refill sub-stamps (stats build, PT_DEBUG_ABLATE & 32): every wait forced where it is
            // stamped, so the claim, the claim-order entry and the ray gather are timed apart
            auto rstamp = [&](int q) {
                if (stamps) {
                    __builtin_amdgcn_s_waitcnt(0);
                    const unsigned long long t = clock64();
                    cyr[q] += t - ts;
                    cy[0] += t - ts;
                    ts = t;
                }
            };
            rstamp(3);
            const int cnt = __popcll(idle);
            const int leader = __ffsll((long long)idle) - 1;
            int base = 0;
            if (lane == leader) base = atomicAdd(p.trace_next, cnt);
            base = __builtin_amdgcn_readlane(base, leader);   // uniform: SGPR
            rstamp(0);
            if (base + cnt >= n) exhausted = true;
            if (state == 0) {
                j = base + __popcll(idle & ((1ull << lane) - 1ull));
                if (j < n) {
                    int src;
                    if (p.order) { const int2 e = p.order[j]; j = e.x; src = e.y; }   // sorted claim order
                    else src = slot_source(p, j);
                    const float4 a = p.ray[in_buf][0][src];
                    const float4 b = p.ray[in_buf][1][src];
                    gdist = kFMax; gmodel = -1; gtri = -1; im = -1;
                    ow = mk3(a.x, a.y, a.z);
                    dw = mk3(b.x, b.y, b.z);
                    state = 1;
                } else {
                    state = 3;
                }
            }
            rstamp(2);
        }
        if (exhausted && state == 0) state = 3;
        if (__ballot(state != 3) == 0) break;
        // safety net: never spin forever (reported as a fault); checked every 16th iteration, so
        // the cap's kernel-argument load stays out of the loop's common path
        if ((iters & 15u) == 0 && iters > p.trace_iter_cap) {
            // the faulting wave's lanes (slots 59..63: idle, done, select, node/leaf/walk; exhausted
            // waves) -- slots no PT_DEBUG_ABLATE statistic uses
            const int f0 = __popcll(__ballot(state == 0)), f3 = __popcll(__ballot(state == 3)),
                      f1 = __popcll(__ballot(state == 1));
            if (lane == 0) {
                atomicAdd(p.segments + kTraceFaultCounter, 1ull);
                atomicAdd(p.segments + 59 + kMaxBounceCounters, (unsigned long long)f0);
                atomicAdd(p.segments + 60 + kMaxBounceCounters, (unsigned long long)f3);
                atomicAdd(p.segments + 61 + kMaxBounceCounters, (unsigned long long)f1);
                atomicAdd(p.segments + 62 + kMaxBounceCounters, (unsigned long long)(64 - f0 - f3 - f1));
                atomicAdd(p.segments + 63 + kMaxBounceCounters, exhausted ? 1ull : 0ull);
            }
            break;
        }
        // Phase scheduling: one step kind per iteration -- the one most lanes are
        // waiting in (weighted) -- so the wave never pays for several partly used blocks.
        int phase = 2;
        {
            const int c1 = __popcll(__ballot(state == 1)), c2 = __popcll(__ballot(state == 2)),
                      c4 = __popcll(__ballot(state == 4)), c5 = __popcll(__ballot(state == 5 || state == 7));
            int cm = c2;
            if (c4 * 4 > cm * PT_LEAF_W) { phase = 4; cm = c4; }
            if (c5 * 4 > cm * PT_WALK_W) { phase = 8; cm = c5; }
            if (c1 * 4 > cm * PT_SEL_W) { phase = 1; cm = c1; }
        }
        // once the rays are claimed and few lanes still trace (PT_ALLPHASE_LANES; experiment, 0 = off),
        // every step kind runs every iteration: no lane waits for the other lanes' phases
        if (exhausted && p.allphase_lanes > 0 && __popcll(__ballot(state != 3)) <= p.allphase_lanes) phase = 1 | 2 | 4 | 8;
        // drain: at most drain_dump lanes still trace once the pool is exhausted
        {
            const int dd = TAIL ? p.drain_dump_tail : p.drain_dump;
            if (may_dump && exhausted && dd > 0 && __popcll(__ballot(state != 3)) <= dd) phase = 16;
        }
        phase = __builtin_amdgcn_readfirstlane(phase);   // wave-uniform: scalar branches on it
        if (PT_TRACE_STATS && (p.debug & 16)) {       // lane-steps executed per phase, and phase iterations
            st_iter++;
            {
                const unsigned long long nb_ = __popcll(__ballot(state != 0 && state != 3));
                st_busy += nb_;
                if (exhausted) { st_drain++; st_drain_busy += nb_; }
            }
            if (phase & 2) { st_node += __popcll(__ballot(state == 2)); it_node++; }
            if (phase & 4) { st_leaf += __popcll(__ballot(state == 4)); it_leaf++; }
            if (phase & 8) { st_walk += __popcll(__ballot(state == 5 || state == 7)); it_walk++; }
            if (phase & 1) { st_sel += __popcll(__ballot(state == 1)); it_sel++; }
        }
        if (stamps) { const unsigned long long t = clock64(); cy[0] += t - ts; ts = t; }
        if ((phase & 1) && state == 1) {                // next model that survives culling and the grid entry test
            // world-space slopes for the instance culling: recomputed here (select steps are
            // rare) instead of living in registers through the traversal
            const f3 winv = node_inv(cull_inv(dw));
            const float dlen = sqrtf(dot(dw, dw));
            if (kSelMask) {
                if (im < 0) {                               // a fresh ray: every model's miss test, once
                    cmask = 0;
                    for (int m = 0; m < p.nmodels; m++) {
                        const ModelRec& M = models[m];
                        float wtn, wtf;
                        node_slab(M.wbox, M.wbox + 3, ow, winv, wtn, wtf);
                        bool cand = !((wtn > wtf) | (wtf * dlen < -1.0f));
                        if (!cand) {                        // model_culled's zero-slope exception
                            const f3 dm = xform12(M.w2m, dw, 0.0f);
                            cand = !(dm.x != 0.0f && dm.y != 0.0f && dm.z != 0.0f);
                        }
                        cmask |= cand ? 1u << m : 0u;
                    }
                }
            }
            for (;;) {
                if (kSelMask) {                             // the next candidate model
                    const unsigned rest = cmask >> (im + 1);
                    im = rest ? im + __ffs(rest) : p.nmodels;
                } else {
                    im++;
                }
                if (im >= p.nmodels) {
                    put_hit(p, j, gdist, gmodel, gtri);
                    state = 0;
                    break;
                }
                const ModelRec& M = models[im];
                if (kSelMask) {                             // model_culled's gdist test for a candidate
                    float wtn, wtf;
                    node_slab(M.wbox, M.wbox + 3, ow, winv, wtn, wtf);
                    if (wtn * dlen > gdist * 1.0001f + 0.01f) continue;
                } else if (model_culled<ACCEL_GRID_FAST>(M, ow, dw, winv, dlen, gdist)) continue;
                if (PT_EMPTY_SKIP && M.bvh4_root < 0) continue;   // a mesh without triangles: no hit, no BLAS
                o = xform12(M.w2m, ow, 1.0f);
                d = normalize(xform12(M.w2m, dw, 0.0f));
                const f3 inv = mk3(1 / d.x, 1 / d.y, 1 / d.z);
                // the grid's box test and entry check as one condition (one divergent `continue`)
                float tb = 0.0f;
                const bool boxhit = slab_ref(M.bbox, o, d, inv, tb);
                const f3 pt = o + d * tb;
                if (!(boxhit & !((pt.x - M.bbox[0]) < -kEps) & !((pt.y - M.bbox[1]) < -kEps) &
                      !((pt.z - M.bbox[2]) < -kEps))) continue;
                t_box = tb;
                ninv = node_inv(inv);
                G = mk3((M.vw[0] + M.cslack[0]) * absr(ninv.x), (M.vw[1] + M.cslack[1]) * absr(ninv.y),
                        (M.vw[2] + M.cslack[2]) * absr(ninv.z));
                if (PT_TRACE_STATS && (p.debug & 512)) G = G * 0.5f;   // timing-only ablation: half-voxel growth
                if (PT_TRACE_STATS && (p.debug & 1024)) G = mk3(0, 0, 0);   // timing-only ablation: no growth
                tier = 0;
                win = (PT_TRACE_STATS && (p.debug & 256)) ? 0.0f : M.wdelta;   // 256: timing-only ablation
                cur = M.bvh4_root;
                lbase = M.leaf_base;
                sp = 0; nh = 0; tmin = kFMax; pblk = -1;
                state = 2;
                break;
            }
        }
        if (stamps) { const unsigned long long t = clock64(); cy[1] += t - ts; ts = t; }
        bool collected = false;
        if ((phase & 4) && state == 4) {                // leaf triangles of the collection: up to PT_LEAF_STEP
            // per step, their loads issued together; tested in leaf order, as one per step would
            // (k_trace_gf: at most two -- selecting from a longer array spilled 33+ VGPRs)
            const int i1 = (PT_LEAF_STEP > 1 && lf_i + 1 < lf_e) ? lf_i + 1 : lf_i;
            const float4 A0 = p.bvh_tri_geom[3 * lf_i], B0 = p.bvh_tri_geom[3 * lf_i + 1], C0 = p.bvh_tri_geom[3 * lf_i + 2];
            const float4 A1 = p.bvh_tri_geom[3 * i1], B1 = p.bvh_tri_geom[3 * i1 + 1], C1 = p.bvh_tri_geom[3 * i1 + 2];
            const int n_step = i1 != lf_i ? 2 : 1;
            if (PT_TRACE_STATS && (p.debug & 16)) atomicAdd(p.segments + 68 + kMaxBounceCounters, (unsigned long long)n_step);
            // Both tests first (pure), then the hits' insertions in leaf order: the loop
            // below runs only for lanes with a hit, and carries 4 values instead of 12.
            float t0 = 0.0f, t1 = 0.0f;
            const bool hit0 = tri_test_rec(A0, B0, C0, o, d, t0);
            const bool hit1 = tri_test_rec(A1, B1, C1, o, d, t1) & (n_step == 2);
            if (hit0 | hit1) {
#pragma unroll 1
                for (int k = 0; k < n_step && state == 4; k++) {
                    const float t = k ? t1 : t0;
                    const int aw = __float_as_int(k ? A1.w : A0.w), bw = __float_as_int(k ? B1.w : B0.w),
                              cw = __float_as_int(k ? C1.w : C0.w);
                    if (k ? hit1 : hit0) {
                        if (t < tmin) tmin = t;
                        const ModelRec& M = models[im];
                        const float X = tmin + win;
                        const float Xs = X + gf_slack(X, t_box);
                        if (!(vbox_entry(M, bw, cw, o, ninv) > Xs)) {   // required member
                            const int4 e = make_int4(__float_as_int(t), aw, bw, cw);
                            if (pblk < 0) {
                                if (nh == kGfHitCap) {          // drop members now beyond the bound
                                    int wn = 0;
                                    for (int q = 0; q < nh; q++) {
                                        const int4 x = hs[q * BS];
                                        if (!(vbox_entry(M, x.z, x.w, o, ninv) > Xs)) hs[(wn++) * BS] = x;
                                    }
                                    nh = wn;
                                }
                                if (nh == kGfHitCap) {          // LDS full: continue in a 64-member global pool block
                                    const int blk = atomicAdd(p.hs_pool_next, 1);
                                    if (blk < p.hs_pool_blocks) {
                                        pblk = blk;
                                        int4* g = p.hs_pool + (size_t)pblk * kHitCapPool;
                                        for (int q = 0; q < nh; q++) g[q] = hs[q * BS];
                                    }
                                }
                            }
                            if (pblk >= 0) {
                                int4* g = p.hs_pool + (size_t)pblk * kHitCapPool;
                                if (nh == kHitCapPool) {
                                    int wn = 0;
                                    for (int q = 0; q < nh; q++) {
                                        const int4 x = g[q];
                                        if (!(vbox_entry(M, x.z, x.w, o, ninv) > Xs)) g[wn++] = x;
                                    }
                                    nh = wn;
                                }
                                if (nh < kHitCapPool) g[nh++] = e;
                                else { p.defer_slots[atomicAdd(p.defer_count, 1)] = j; state = 0; }   // pool block full too
                            } else if (nh < kGfHitCap) {
                                hs[nh * BS] = e;
                                nh++;
                            } else {                            // pool exhausted: the whole ray goes to k_trace_deferred
                                p.defer_slots[atomicAdd(p.defer_count, 1)] = j;
                                state = 0;
                            }
                        }
                    }
                }
            }
            if (state == 4) {
                lf_i += n_step;
                // end of the leaf: the next stack entry, a leaf (encoded, < 0) or a node
                const bool end = lf_i == lf_e;
                const bool pop = end & (sp > 0);
                collected = end & (sp == 0);
                const int top = spop_if<BS, kGfStack>(pop, stack, spill, p.spill_stride, sp - 1);
                sp -= pop ? 1 : 0;
                const bool tleaf = pop & (top < 0);
                const int first = (PT_LEAF_REL ? lbase : 0) + (top & ((1 << kLeafCountShift) - 1));   // mesh-relative entry
                lf_e = tleaf ? first + ((top >> kLeafCountShift) & kMaxLeafCount4) : lf_e;
                lf_i = tleaf ? first : lf_i;
                cur = (pop & !tleaf) ? top : cur;
                state = (pop & !tleaf) ? 2 : state;
            }
        } else if ((phase & 2) && state == 2) {   // 4-wide node steps of the collection
#pragma unroll 1
            for (int ks = 0; ks < kNodeSteps; ks++) {
                // per axis, the slab a child is entered through is fixed by the sign of the slope:
                // load each axis' near and far planes directly (lo for a positive slope), so the
                // entries and exits come without min / max, and the voxel-grown entry is one fma
                const int ox = ninv.x < 0.0f ? 3 : 0, oy = ninv.y < 0.0f ? 3 : 0, oz = ninv.z < 0.0f ? 3 : 0;
#if PT_LDS_TOP
                const int rel0_ = cur - p.top_root[0], rel1_ = cur - p.top_root[1];
                const bool in0_ = (unsigned)rel0_ < (unsigned)p.top_n[0];
                const bool in1_ = kLdsTopMeshes > 1 && (unsigned)rel1_ < (unsigned)p.top_n[1];
                float4 NX, NY, NZ, FX, FY, FZ, LKf;
                if (in0_ | in1_) {
                    const float4* q_ = s_top + 8 * (in0_ ? rel0_ : kLdsTop + rel1_);
                    NX = q_[ox]; NY = q_[1 + oy]; NZ = q_[2 + oz];
                    FX = q_[3 - ox]; FY = q_[4 - oy]; FZ = q_[5 - oz];
                    LKf = q_[6];
                } else {
                    const char* __restrict__ nb_ = reinterpret_cast<const char*>(p.bvh4);
                    const unsigned nbo_ = (unsigned)cur << 7;
                    auto ld4_ = [&](int q) { return *reinterpret_cast<const float4*>(nb_ + (nbo_ + 16u * (unsigned)q)); };
                    NX = ld4_(ox); NY = ld4_(1 + oy); NZ = ld4_(2 + oz);
                    FX = ld4_(3 - ox); FY = ld4_(4 - oy); FZ = ld4_(5 - oz);
                    LKf = ld4_(6);
                }
#else
                PT_NODE_LOADS(cur, ox, oy, oz)
#endif
                const float pnx[4] = {NX.x, NX.y, NX.z, NX.w}, pny[4] = {NY.x, NY.y, NY.z, NY.w};
                const float pnz[4] = {NZ.x, NZ.y, NZ.z, NZ.w}, pfx[4] = {FX.x, FX.y, FX.z, FX.w};
                const float pfy[4] = {FY.x, FY.y, FY.z, FY.w}, pfz[4] = {FZ.x, FZ.y, FZ.z, FZ.w};
                const int lk[4] = {__float_as_int(LKf.x), __float_as_int(LKf.y), __float_as_int(LKf.z),
                                   __float_as_int(LKf.w)};
                const float X = tmin + win;
                const float bound = X + gf_slack(X, t_box);
                const f3 oi = o * ninv;
                float key[4];
                int ent[4];
                int nhit = 0;
#pragma unroll
                for (int c = 0; c < 4; c++) {
                    // tn / tf: the same fma values as node_slab_g's min / max pick; tx: the grown
                    // entry with the growth folded into the offset (within gf_slack of e - G).  An
                    // empty slot's inverted infinite box gives tn = +inf, tf = -inf: a miss, so
                    // Bvh4Node.count is never loaded
                    const float e0 = __builtin_fmaf(pnx[c], ninv.x, -oi.x), e1 = __builtin_fmaf(pny[c], ninv.y, -oi.y);
                    const float e2 = __builtin_fmaf(pnz[c], ninv.z, -oi.z);
                    const float tn = fmaxf(fmaxf(e0, e1), e2);
                    const float tf = fminf(fminf(__builtin_fmaf(pfx[c], ninv.x, -oi.x), __builtin_fmaf(pfy[c], ninv.y, -oi.y)),
                                           __builtin_fmaf(pfz[c], ninv.z, -oi.z));
                    const float tx = fmaxf(fmaxf(__builtin_fmaf(pnx[c], ninv.x, -(oi.x + G.x)),
                                                 __builtin_fmaf(pny[c], ninv.y, -(oi.y + G.y))),
                                           __builtin_fmaf(pnz[c], ninv.z, -(oi.z + G.z)));
                    const bool h = (tn <= tf) & (tf >= -kEps) & (tx <= bound);
                    key[c] = h ? tn : __int_as_float(0x7f800000);
                    ent[c] = lk[c];                          // leaves come encoded (Bvh4Node)
                    nhit += h ? 1 : 0;
                }
                // nearest first: sort the four (entry, key) pairs by key (misses last, at +inf)
                auto cas = [&](int a, int b) {
                    const bool sw = key[b] < key[a];
                    const float ka = key[a], kb = key[b];
                    const int ea = ent[a], eb = ent[b];
                    key[a] = sw ? kb : ka; key[b] = sw ? ka : kb;
                    ent[a] = sw ? eb : ea; ent[b] = sw ? ea : eb;
                };
                cas(0, 1); cas(2, 3); cas(0, 2); cas(1, 3); cas(1, 2);
                // the farther hits go on the stack, farthest first (the nearer pop first)
                if (PT_TRACE_STATS && (p.debug & 16)) {   // slots 64..67: pushes, spilled pushes, node visits, hits
                    const int np = max(nhit - 1, 0);
                    const int ns = max(0, sp + np - kGfStack) - max(0, sp - kGfStack);
                    atomicAdd(p.segments + 64 + kMaxBounceCounters, (unsigned long long)np);
                    if (ns > 0) atomicAdd(p.segments + 65 + kMaxBounceCounters, (unsigned long long)ns);
                    atomicAdd(p.segments + 66 + kMaxBounceCounters, 1ull);
                    atomicAdd(p.segments + 67 + kMaxBounceCounters, (unsigned long long)nhit);
                }
                if (nhit > 3) { spush_t<BS, kGfStack>(stack, spill, p.spill_stride, sp, ent[3]); sp++; }
                if (nhit > 2) { spush_t<BS, kGfStack>(stack, spill, p.spill_stride, sp, ent[2]); sp++; }
                if (nhit > 1) { spush_t<BS, kGfStack>(stack, spill, p.spill_stride, sp, ent[1]); sp++; }
                const bool pop = (nhit == 0) & (sp > 0);
                const int top = spop_if<BS, kGfStack>(pop, stack, spill, p.spill_stride, sp - 1);
                collected = (nhit == 0) & (sp == 0);
                sp -= pop ? 1 : 0;
                const int nx = nhit > 0 ? ent[0] : top;       // the entry to go on with (when not collected)
                const bool leaf = !collected & (nx < 0);
                const int first = (PT_LEAF_REL ? lbase : 0) + (nx & ((1 << kLeafCountShift) - 1));
                lf_i = leaf ? first : lf_i;
                lf_e = leaf ? first + ((nx >> kLeafCountShift) & kMaxLeafCount4) : lf_e;
                cur = (!collected & !leaf) ? nx : cur;
                state = leaf ? 4 : state;
                if (state != 2 || collected) break;    // a leaf reached, or the collection done
                if (kNodeMinLanes > 0 && __popcll(__ballot(state == 2 && !collected)) < kNodeMinLanes) break;
            }
        }
        if (stamps) { const unsigned long long t = clock64(); cy[(phase & 4) ? 2 : 3] += t - ts; ts = t; }
        if (collected) {
            if (nh > 0) {
                state = 5;
            } else if (!(tmin < kFMax)) {
                state = 1;          // no accepted triangle anywhere on the ray: no hit voxel, the model is missed
            } else {
                // accepted triangles exist, but none whose voxel box the walk can enter
                // before t_min + window: the walk is not decided here, next tier
                const ModelRec& M = models[im];
                tier++;
                win = tier == 1 ? 2.0f * M.reach : 3.0e38f;
                cur = M.bvh4_root;
                sp = 0; nh = 0; tmin = kFMax;
                state = 2;
            }
        } else if ((phase & 8) && (state == 5 || state == 7)) {   // the walk: certificate, else the exact walk
            if (PT_TRACE_STATS && (p.debug & 2048))       // walks by hit-set size: 1, 2, 3, >= 4 (pool: >= 4)
                atomicAdd(p.segments + 51 + (pblk >= 0 ? 3 : min(nh, 4) - 1) + kMaxBounceCounters, 1ull);
            const ModelRec& M = models[im];
            const f3 pt = o + d * t_box;
            WalkResult w;
            if (PT_TRACE_STATS && (p.debug & 128) && pblk < 0) {      // timing-only ablation: no walk at all
                w.hit = true; w.has_best = true; w.final_min = true; w.t = tmin; w.tri = -1; w.tw = 0.0f;
                for (int h = 0; h < nh; h++) if (__int_as_float(hs[h * BS].x) == tmin) w.tri = hs[h * BS].y;
            } else if (!TAIL && !(F & 16)) {
                // the certificate only; a ray it cannot decide is handed on to the tail launch
                // (which walks it exactly) or, past the records' room, to k_trace_deferred
                // (hit sets in a global pool block -- more than kGfHitCap members, rare -- are
                // handed on undecided: the pool's runtime-length loops would cost registers here)
                // members copied to registers first: four LDS reads issued together, one wait
                // (read member by member inside the certificates' loops, every read waited
                // on its own)
                int tri = -1;
                int4 mem[kGfHitCap];
#pragma unroll
                for (int h = 0; h < kGfHitCap; h++) mem[h] = hs[h * BS];
                auto lds_get = [&](int h) { return mem[h]; };
                bool ok = false;
                // ninv (1/d clamped to +-1e30, set at select) is the exact 1/d when no slope is clamped
                const bool exact_inv = (absr(ninv.x) < 1e30f) & (absr(ninv.y) < 1e30f) & (absr(ninv.z) < 1e30f);
                if (PT_CERT_MODE >= 1 && pblk < 0 && exact_inv)
                    ok = walk_certify_fast<kGfHitCap>(p, M, d, ninv, pt, t_box, lds_get, nh, tmin, win, tri);
                if (PT_TRACE_STATS && (p.debug & 4)) {
                    atomicAdd(p.segments + 42 + kMaxBounceCounters, 1ull);
                    if (ok) atomicAdd(p.segments + 40 + kMaxBounceCounters, 1ull);
                }
                if (PT_CERT_MODE <= 1 && !ok && pblk < 0) {
                    const f3 inv = mk3(1 / d.x, 1 / d.y, 1 / d.z);
                    ok = walk_certify<kGfHitCap>(p, M, d, inv, pt, t_box, lds_get, nh, tmin, win, tri);
                    if (PT_TRACE_STATS && (p.debug & 4) && ok) atomicAdd(p.segments + 41 + kMaxBounceCounters, 1ull);
                }
                w.hit = ok; w.has_best = ok; w.final_min = ok; w.t = tmin; w.tri = tri; w.tw = 0.0f;
                if (!ok) state = 6;
            } else {
                const f3 inv = mk3(1 / d.x, 1 / d.y, 1 / d.z);
                // state 7: a walk hand-on whose LDS hit set both certificates already declined in
                // the main launch (deterministically: they would decline again): the exact walk only
                w = pblk < 0 ? hitset_walk_regs<kGfHitCap, BS, true, true>(p, M, d, inv, pt, t_box, hs, nh, tmin, win,
                                                                            state != 7)
                             : hitset_walk<1, true>(p, M, d, inv, pt, t_box, p.hs_pool + (size_t)pblk * kHitCapPool, nh,
                                                    tmin, win);
            }
            if (state == 6) {
                // handed on below
            } else if (tier == 2 || w.final_min || w.tw < tmin + win) {
                if (w.hit && w.has_best) {
                    const float dd = model_hit_dist(M, o, d, w.t, ow);
                    if (gdist > dd) { gdist = dd; gmodel = im; gtri = w.tri; }
                }
                state = 1;
            } else {                                    // not provably exact: next tier's collection
                tier++;
                win = tier == 1 ? 2.0f * M.reach : 3.0e38f;
                cur = M.bvh4_root;
                sp = 0; nh = 0; tmin = kFMax;
                state = 2;
            }
        }
        if (stamps) { const unsigned long long t = clock64(); cy[4] += t - ts; ts = t; }
        if ((phase & 16) || (!TAIL && (phase & 8) && __ballot(state == 6))) {
            if (PT_TRACE_STATS && (p.debug & 32) && lane == 0)     // walk iterations with hand-ons, drains
                atomicAdd(p.segments + ((phase & 16) ? 27 : 26) + kMaxBounceCounters, 1ull);
            // hand-on records: the drain (phase 16: every busy lane's exact state, then
            // the wave is done) or walk hand-ons (state 6: a collected hit set the
            // certificate left undecided; the tail launch walks it exactly)
            const bool drain = (phase & 16) != 0;
            bool mine = drain ? state != 3 : state == 6;
            const unsigned long long bm = __ballot(mine);
            const int nbusy = __popcll(bm);
            const int leader = __ffsll((long long)bm) - 1;
            int base = 0;
            if (lane == leader) base = atomicAdd(p.cont_count + (drain ? level : kDrainLevels + level), nbusy);
            base = __builtin_amdgcn_readlane(base, leader);   // uniform: SGPR
            const int r = base + __popcll(bm & ((1ull << lane) - 1ull));
            if (!drain && mine && r >= p.cont_wcap) {  // no room left: the whole ray goes to k_trace_deferred
                p.defer_slots[atomicAdd(p.defer_count, 1)] = j;
                mine = false;
            }
            if (mine) {
                int* C = cout + (drain ? r : p.cont_cap - 1 - r);
                const size_t cs = (size_t)p.cont_cap;
                // a walk hand-on resumes in state 7 (walk, certificates already declined) unless its hit
                // set is in a pool block, where the main launch tries no certificate
                C[kCJ * cs] = j; C[kCState * cs] = drain ? state : (pblk < 0 ? 7 : 5); C[kCIm * cs] = im;
                C[kCGdist * cs] = __float_as_int(gdist); C[kCGmodel * cs] = gmodel; C[kCGtri * cs] = gtri;
                C[kCOw * cs] = __float_as_int(ow.x); C[(kCOw + 1) * cs] = __float_as_int(ow.y);
                C[(kCOw + 2) * cs] = __float_as_int(ow.z);
                C[kCDw * cs] = __float_as_int(dw.x); C[(kCDw + 1) * cs] = __float_as_int(dw.y);
                C[(kCDw + 2) * cs] = __float_as_int(dw.z);
                C[kCCur * cs] = cur; C[kCSp * cs] = sp;
                C[kCLfI * cs] = lf_i; C[kCLfE * cs] = lf_e; C[kCLf2I * cs] = lf2_i; C[kCLf2E * cs] = lf2_e;
                C[kCLfNext * cs] = lf_next; C[kCSpill * cs] = drain ? sbase : -1;
                C[kCX * cs] = __float_as_int(tmin); C[(kCX + 1) * cs] = nh; C[(kCX + 2) * cs] = tier;
                C[(kCX + 3) * cs] = pblk; C[(kCX + 4) * cs] = __float_as_int(win);
                C[(kCX + 5) * cs] = __float_as_int(t_box);
                C[(kCX + 6) * cs] = __float_as_int(G.x); C[(kCX + 7) * cs] = __float_as_int(G.y);
                C[(kCX + 8) * cs] = __float_as_int(G.z);
#pragma unroll 1
                for (int q = 0; q < (drain ? min(sp, kGfStack) : 0); q++) C[(kCX + 9 + q) * cs] = stack[q * BS];
#pragma unroll 1
                for (int q = 0; q < (pblk < 0 ? nh : 0); q++) {
                    const int4 e = hs[q * BS];
                    C[(kCX + 9 + kGfStack + 4 * q) * cs] = e.x; C[(kCX + 10 + kGfStack + 4 * q) * cs] = e.y;
                    C[(kCX + 11 + kGfStack + 4 * q) * cs] = e.z; C[(kCX + 12 + kGfStack + 4 * q) * cs] = e.w;
                }
            }
            state = drain ? 3 : (state == 6 ? 0 : state);
        }
        if (stamps) { const unsigned long long t = clock64(); cy[5] += t - ts; ts = t; }
    }
    if (stamps && lane == 0) {
        for (int q = 0; q < 6; q++) atomicAdd(p.segments + 20 + q + kMaxBounceCounters, cy[q]);
        for (int q = 0; q < 4; q++) atomicAdd(p.segments + 55 + q + kMaxBounceCounters, cyr[q]);
        if (TAIL)                                   // the tail launches' own cycle split (slots 70..75)
            for (int q = 0; q < 6; q++) atomicAdd(p.segments + 70 + q + kMaxBounceCounters, cy[q]);
    }
    if ((PT_TRACE_STATS && (p.debug & 16)) && lane == 0) {
        atomicAdd(p.segments + 8 + kMaxBounceCounters, st_iter);
        if (TAIL) {                                 // the tail launches' share (slots 15, 43)
            atomicAdd(p.segments + 15 + kMaxBounceCounters, st_iter);
            atomicAdd(p.segments + 43 + kMaxBounceCounters, st_busy);
        }
        atomicAdd(p.segments + 44 + kMaxBounceCounters, st_drain);
        atomicAdd(p.segments + 45 + kMaxBounceCounters, st_drain_busy);
        atomicAdd(p.segments + 46 + kMaxBounceCounters, st_busy);
        atomicAdd(p.segments + 9 + kMaxBounceCounters, st_node);
        atomicAdd(p.segments + 10 + kMaxBounceCounters, st_leaf);
        atomicAdd(p.segments + 11 + kMaxBounceCounters, st_walk);
        atomicAdd(p.segments + 12 + kMaxBounceCounters, st_sel);
        atomicAdd(p.segments + 16 + kMaxBounceCounters, it_node);
        atomicAdd(p.segments + 17 + kMaxBounceCounters, it_leaf);
        atomicAdd(p.segments + 18 + kMaxBounceCounters, it_walk);
        atomicAdd(p.segments + 19 + kMaxBounceCounters, it_sel);
    }
}

// Rays k_trace_gf deferred (LDS hit-set overflow): the fused path's
// intersect_scene<ACCEL_GRID_FAST> (LDS tiers, global pool, list-walking DDA),
// one lane per ray.
template <int BS>
__global__ __launch_bounds__(BS) void k_trace_deferred(KParams p, int bounce) {
    __shared__ int s_stack[kStack * BS];
    __shared__ int4 s_hs[kHitCap * BS];
    const int in_buf = (bounce + 1) & 1;
    const int cnt = *p.defer_count;
    if ((PT_TRACE_STATS && (p.debug & 16)) && blockIdx.x == 0 && threadIdx.x == 0)
        atomicAdd(p.segments + 14 + kMaxBounceCounters, (unsigned long long)cnt);
    if (blockIdx.x == 0 && threadIdx.x == 0 && cnt > 0)      // every build: which route the rays took
        atomicAdd(p.segments + kDeferredRayCounter, (unsigned long long)cnt);
    for (int q = blockIdx.x * BS + threadIdx.x; q < cnt; q += gridDim.x * BS) {
        const int j = p.defer_slots[q];
        const int src = slot_source(p, j);
        const float4 a = p.ray[in_buf][0][src];
        const float4 b = p.ray[in_buf][1][src];
        float gdist;
        int gmodel, gtri;
        intersect_scene_g<ACCEL_GRID_FAST, BS>(p, mk3(a.x, a.y, a.z), mk3(b.x, b.y, b.z), s_stack + threadIdx.x,
                                               s_hs + threadIdx.x, gdist, gmodel, gtri);
        put_hit(p, j, gdist, gmodel, gtri);
    }
}

// One bounce for every live ray: gather -> intersect -> shade -> compact / accumulate.
template <bool FIRST, int ACCEL, int BS>
__global__ __launch_bounds__(BS, (ACCEL == ACCEL_GRID_FAST && !FIRST) ? 3 : PT_MINWAVES) void k_bounce(KParams p, int iter, int bounce) {
    __shared__ int s_stack[(!FIRST && ACCEL != ACCEL_GRID && ACCEL != kAccelHitBuffer) ? kStack * BS : 1];
    __shared__ int4 s_hs[(!FIRST && ACCEL == ACCEL_GRID_FAST) ? kHitCap * BS : 1];
    __shared__ int s_wave[BS / 64];
    const int n = FIRST ? p.npix : p.n_live[bounce];
    // Workgroups are dealt round-robin over the 8 XCDs (MI355X_MICROARCH.md); map
    // them so XCD x processes the contiguous chunk range [x q, (x+1) q) of the live
    // pool -- neighbouring rays (neighbouring pixels' paths) share one L2.  The grid
    // has nblocks + 8 workgroups so the permutation covers every live chunk.
    const int chunk = blockIdx.x;
    const int j0 = chunk >= (n + BS - 1) / BS ? n : chunk * BS;
    if (j0 >= n) return;                       // whole block idle (uniform)
    const int j = j0 + threadIdx.x;
    const bool active = j < n;
    const int in_buf = (bounce + 1) & 1, out_buf = bounce & 1;

    RayState r;
    Hit h;
    if (active) {
        if (FIRST) {
            camera_ray(p, j, r.o, r.d);
            r.c = mk3(1.0f, 1.0f, 1.0f);
            r.pixel = j;
            r.bounces = p.max_bounces;
            const float4 ch = p.cache_hit[j];
            h.dist = ch.x;
            h.n = mk3(ch.y, ch.z, ch.w);
            h.model = p.cache_model[j];
        } else {
            // dense slot j -> (source block b, rank) via the scan of the previous bounce
            int lo = p.dst_start[chunk], hi = p.dst_start[chunk + 1];
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (p.blk_off[mid] <= j) lo = mid; else hi = mid - 1;
            }
            const int src = lo * BS + (j - p.blk_off[lo]);
            const float4 a = p.ray[in_buf][0][src];
            const float4 b = p.ray[in_buf][1][src];
            const float4 c = p.ray[in_buf][2][src];
            r.o = mk3(a.x, a.y, a.z); r.pixel = __float_as_int(a.w);
            r.d = mk3(b.x, b.y, b.z); r.bounces = __float_as_int(b.w);
            r.c = mk3(c.x, c.y, c.z);
            if (ACCEL == kAccelHitBuffer) {       // traced by k_trace_bvh / k_trace_gf
                h = get_hit(p, j);
            } else {
                h = intersect_scene<ACCEL, BS>(p, r.o, r.d, s_stack + threadIdx.x, s_hs + threadIdx.x);
            }
        }
        shade(p, r, h, iter >= 0 ? iter : *p.iter_dev, j);   // -1: hipGraph replay reads the id
    }
    const bool alive = active && r.bounces > 0;
    if (active && !alive) {
        // gatherImageDataKernel (Renderer.cpp:481-496): pixel += 1.0f * sqrt(color).
        // Each pixel has exactly one ray per iteration: no atomics needed.
        // With several pipelines in flight the value goes to the pipeline's
        // per-iteration contribution buffer and k_merge adds the buffers to the
        // image in iteration order: the same one add per pixel per iteration.
        if (p.contrib) {
            float* cp = p.contrib + 3 * (size_t)r.pixel;
            cp[0] = 1.0f * sqrtf(r.c.x);
            cp[1] = 1.0f * sqrtf(r.c.y);
            cp[2] = 1.0f * sqrtf(r.c.z);
        } else {
            float* px = p.image + 3 * (size_t)r.pixel;
            px[0] += 1.0f * sqrtf(r.c.x);
            px[1] += 1.0f * sqrtf(r.c.y);
            px[2] += 1.0f * sqrtf(r.c.z);
        }
    }
    // Block-local stable compaction (ballot + wave prefix), order == slot order.
    const unsigned long long m = __ballot(alive);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int rank = __popcll(m & ((1ull << lane) - 1ull));
    int base = 0, total = 0;
    if (BS > 64) {
        if (lane == 0) s_wave[wid] = __popcll(m);
        __syncthreads();
    } else {
        total = __popcll(m);
    }
#pragma unroll
    for (int w = 0; w < (BS > 64 ? BS / 64 : 0); w++) {
        const int c = s_wave[w];
        base += (w < wid) ? c : 0;
        total += c;
    }
    if (alive) {
        const int dst = j0 + base + rank;
        p.ray[out_buf][0][dst] = make_float4(r.o.x, r.o.y, r.o.z, __int_as_float(r.pixel));
        p.ray[out_buf][1][dst] = make_float4(r.d.x, r.d.y, r.d.z, __int_as_float(r.bounces));
        p.ray[out_buf][2][dst] = make_float4(r.c.x, r.c.y, r.c.z, 0.0f);
    }
    if (threadIdx.x == 0) p.blk_cnt[chunk] = total;
}

// One workgroup: exclusive scan of survivor counts of bounce `bounce`,
// live count for bounce+1, and the first source block of every
// destination block (dst_start).  A small workgroup with almost no LDS: it
// must find room on a CU while persistent traces of other pipelines hold
// nearly every wave slot (a 1024-lane, 130 KB-LDS version waited ~300 us per
// launch for a drained CU at 16 pipelines; 256 / 512 lanes measured within
// 1.3 %, 512 kept).  Tiles of kScanWG x kScanPer
// counts, each thread a contiguous run of kScanPer, carried across tiles.
__global__ __launch_bounds__(kScanWG) void k_scan(KParams p, int bounce) {
    __shared__ int s_part[kScanWG];
    __shared__ int s_carry;
    const int tid = threadIdx.x;
    const int n = bounce == 0 ? p.npix : p.n_live[bounce];
    const int CH = p.chunk;
    const int nb = (n + CH - 1) / CH;
    if (tid == 0) s_carry = 0;
    __syncthreads();
    for (int base = 0; base < nb; base += kScanWG * kScanPer) {
        const int i0 = base + tid * kScanPer;
        int c[kScanPer], sum = 0;
#pragma unroll
        for (int q = 0; q < kScanPer; q++) {
            c[q] = i0 + q < nb ? p.blk_cnt[i0 + q] : 0;
            sum += c[q];
        }
        s_part[tid] = sum;
        __syncthreads();
        for (int off = 1; off < kScanWG; off <<= 1) {
            const int v = tid >= off ? s_part[tid - off] : 0;
            __syncthreads();
            s_part[tid] += v;
            __syncthreads();
        }
        const int carry = s_carry;
        const int tile_total = s_part[kScanWG - 1];
        int acc = carry + s_part[tid] - sum;        // exclusive
#pragma unroll
        for (int q = 0; q < kScanPer; q++) {
            if (i0 + q >= nb) break;
            const int o0 = acc, o1 = acc + c[q];
            p.blk_off[i0 + q] = o0;
            for (int bd = (o0 + CH - 1) / CH; bd * CH < o1; bd++) p.dst_start[bd] = i0 + q;
            acc = o1;
        }
        __syncthreads();                            // every thread has read s_carry / s_part
        if (tid == 0) s_carry = carry + tile_total;
        __syncthreads();
    }
    if (tid == 0) {
        const int total = s_carry;
        p.blk_off[nb] = total;
        p.n_live[bounce + 1] = total;
        atomicAdd(p.segments, (unsigned long long)n);           // shared by concurrent pipelines
        if (bounce < kMaxBounceCounters) atomicAdd(p.segments + 1 + bounce, (unsigned long long)n);
        p.dst_start[(total + CH - 1) / CH] = nb > 0 ? nb - 1 : 0;
        if (PT_TRACE_STATS && bounce > 0) {    // hand-on volume of the bounce's trace (slots 47..50)
            atomicAdd(p.segments + 47 + kMaxBounceCounters, (unsigned long long)p.cont_count[0]);   // drained at level 0
            atomicAdd(p.segments + 48 + kMaxBounceCounters,                                        // walk hand-ons
                      (unsigned long long)min(p.cont_count[kDrainLevels], p.cont_wcap));
            atomicAdd(p.segments + 49 + kMaxBounceCounters, (unsigned long long)*p.defer_count);    // deferred rays
            atomicAdd(p.segments + 50 + kMaxBounceCounters, (unsigned long long)p.cont_count[1]);   // drained at level 1
        }
        *p.hs_pool_next = 0;       // the next bounce starts with an empty hit-set pool
        *p.trace_next = 0;         // and an unclaimed persistent-trace counter
        // (a skipped k_trace_deferred launch left deferred rays untraced: their hit records are stale)
        if (!p.defer_launch && bounce > 0 && *p.defer_count > 0) atomicAdd(p.segments + kTraceFaultCounter, 1ull);
        *p.defer_count = 0;        // and no deferred grid_fast rays
        for (int l = 0; l < kDrainLevels; l++) {   // and no drain continuations or walk hand-ons
            p.cont_count[l] = 0;
            p.cont_count[kDrainLevels + l] = 0;
            p.cont_next[l] = 0;
        }
    }
    if (p.order)                   // empty key histogram and cursors for the next bounce's ray sort
        for (int i = tid; i < 2 * kSortBins; i += kScanWG) p.sort_bins[i] = 0;
}

// ---------------------------------------------------------------------------
// Ray sort before a persistent trace (bounce >= 1).  The trace result of a ray
// does not depend on which lane traces it or when, so the claim order is free:
// a counting sort on a 12-bit (direction, origin) key hands each wave rays that
// walk the same BLAS nodes (coherent SIMD steps, shared L2 lines).  The dense
// slot j -- the RNG seed and the hit-buffer index -- is carried, not changed.
// ---------------------------------------------------------------------------

__device__ __forceinline__ int sort_key(const KParams& p, f3 o, f3 d) {
    // octahedral direction map (u, v in [-1, 1]) quantized to 64 x 64, origin cell 16^3
    const float s = fabsf(d.x) + fabsf(d.y) + fabsf(d.z);
    float u = d.x / s, v = d.y / s;
    if (d.z < 0.0f) {
        const float uu = (1.0f - fabsf(v)) * (u < 0.0f ? -1.0f : 1.0f);
        const float vv = (1.0f - fabsf(u)) * (v < 0.0f ? -1.0f : 1.0f);
        u = uu; v = vv;
    }
    const int iu = min(63, max(0, (int)((u * 0.5f + 0.5f) * 64.0f)));
    const int iv = min(63, max(0, (int)((v * 0.5f + 0.5f) * 64.0f)));
    const int ix = min(15, max(0, (int)((o.x - p.sort_lo[0]) * p.sort_sc[0])));
    const int iy = min(15, max(0, (int)((o.y - p.sort_lo[1]) * p.sort_sc[1])));
    const int iz = min(15, max(0, (int)((o.z - p.sort_lo[2]) * p.sort_sc[2])));
    switch (p.sort_mode) {
        case 1:   // direction major (8 x 8 cells), origin 4^3 minor
            return ((iu >> 3) << 9) | ((iv >> 3) << 6) | ((ix >> 2) << 4) | ((iy >> 2) << 2) | (iz >> 2);
        case 2:   // origin 4^3 major, direction 8 x 8 minor
            return ((ix >> 2) << 10) | ((iy >> 2) << 8) | ((iz >> 2) << 6) | ((iu >> 3) << 3) | (iv >> 3);
        case 4:   // direction only, 64 x 64
            return (iu << 6) | iv;
        case 5:   // origin only, 16^3
            return (ix << 8) | (iy << 4) | iz;
        case 6: { // origin 8^3 (interleaved) major, direction octant minor
            const int x = ix >> 1, y = iy >> 1, z = iz >> 1;
            int m = 0;
            for (int q = 2; q >= 0; q--) m = (m << 3) | (((x >> q) & 1) << 2) | (((y >> q) & 1) << 1) | ((z >> q) & 1);
            return (m << 3) | ((d.x < 0.0f) << 2) | ((d.y < 0.0f) << 1) | (d.z < 0.0f);
        }
        case 7: { // interleaved, origin first: x1 y1 z1 u2 v2 x0 y0 z0 u1 v1 u0 v0
            const int a = iu >> 3, b = iv >> 3, x = ix >> 2, y = iy >> 2, z = iz >> 2;
            return (((x >> 1) & 1) << 11) | (((y >> 1) & 1) << 10) | (((z >> 1) & 1) << 9) | (((a >> 2) & 1) << 8) |
                   (((b >> 2) & 1) << 7) | ((x & 1) << 6) | ((y & 1) << 5) | ((z & 1) << 4) | (((a >> 1) & 1) << 3) |
                   (((b >> 1) & 1) << 2) | ((a & 1) << 1) | (b & 1);
        }
        case 8: { // interleaved, direction 16 x 16 and origin 2^3... : u3 v3 x0 y0 z0 u2 v2 u1 v1 u0 v0 + pad
            const int a = iu >> 2, b = iv >> 2, x = ix >> 3, y = iy >> 3, z = iz >> 3;
            return (((a >> 3) & 1) << 10) | (((b >> 3) & 1) << 9) | (x << 8) | (y << 7) | (z << 6) |
                   (((a >> 2) & 1) << 5) | (((b >> 2) & 1) << 4) | (((a >> 1) & 1) << 3) | (((b >> 1) & 1) << 2) |
                   ((a & 1) << 1) | (b & 1);
        }
        default: { // interleaved: u2 v2 x1 y1 z1 u1 v1 x0 y0 z0 u0 v0 (u, v: 3 bits, x, y, z: 2 bits)
            const int a = iu >> 3, b = iv >> 3, x = ix >> 2, y = iy >> 2, z = iz >> 2;
            return (((a >> 2) & 1) << 11) | (((b >> 2) & 1) << 10) | (((x >> 1) & 1) << 9) | (((y >> 1) & 1) << 8) |
                   (((z >> 1) & 1) << 7) | (((a >> 1) & 1) << 6) | (((b >> 1) & 1) << 5) | ((x & 1) << 4) |
                   ((y & 1) << 3) | ((z & 1) << 2) | ((a & 1) << 1) | (b & 1);
        }
    }
}

// Rays entering bounce `bounce` sit at source index i = c*chunk + r (r < blk_cnt[c]) of
// the previous bounce's pool; dense slot j = blk_off[c] + r.
__global__ __launch_bounds__(kSortWG) void k_sort_hist(KParams p, int bounce) {
    __shared__ int s_h[kSortBins];
    const int nprev = bounce == 1 ? p.npix : p.n_live[bounce - 1];
    const int lim = ((nprev + p.chunk - 1) / p.chunk) * p.chunk;
    const int i0 = blockIdx.x * (kSortWG * kSortPer);
    if (i0 >= lim) return;                               // uniform
    for (int b = threadIdx.x; b < kSortBins; b += kSortWG) s_h[b] = 0;
    __syncthreads();
    const int in_buf = (bounce + 1) & 1;
#pragma unroll
    for (int t = 0; t < kSortPer; t++) {
        const int i = i0 + t * kSortWG + threadIdx.x;
        if (i < lim) {
            const int c = i / p.chunk, r = i - c * p.chunk;
            if (r < p.blk_cnt[c]) {
                const float4 a = p.ray[in_buf][0][i];
                const float4 b = p.ray[in_buf][1][i];
                const int key = sort_key(p, mk3(a.x, a.y, a.z), mk3(b.x, b.y, b.z));
                p.sort_key[i] = (unsigned short)key;
                atomicAdd(&s_h[key], 1);
            }
        }
    }
    __syncthreads();
    for (int b = threadIdx.x; b < kSortBins; b += kSortWG)
        if (s_h[b]) atomicAdd(&p.sort_bins[b], s_h[b]);
}

// One workgroup: cursor[b] = exclusive prefix of the key counts (the first claim
// position of key b); k_sort_scatter's workgroups reserve their ranges from it.
__global__ __launch_bounds__(kSortWG) void k_sort_prefix(KParams p) {
    __shared__ int s_part[kSortWG];
    constexpr int kPerT = kSortBins / kSortWG;           // bins per thread
    const int tid = threadIdx.x;
    int v[kPerT], sum = 0;
#pragma unroll
    for (int q = 0; q < kPerT; q++) { v[q] = p.sort_bins[tid * kPerT + q]; sum += v[q]; }
    s_part[tid] = sum;
    __syncthreads();
    for (int off = 1; off < kSortWG; off <<= 1) {
        const int x = tid >= off ? s_part[tid - off] : 0;
        __syncthreads();
        s_part[tid] += x;
        __syncthreads();
    }
    int acc = s_part[tid] - sum;
#pragma unroll
    for (int q = 0; q < kPerT; q++) { p.sort_bins[kSortBins + tid * kPerT + q] = acc; acc += v[q]; }
}

__global__ __launch_bounds__(kSortWG) void k_sort_scatter(KParams p, int bounce) {
    __shared__ int s_h[kSortBins];                       // local counts, then this workgroup's base per key
    const int nprev = bounce == 1 ? p.npix : p.n_live[bounce - 1];
    const int lim = ((nprev + p.chunk - 1) / p.chunk) * p.chunk;
    const int i0 = blockIdx.x * (kSortWG * kSortPer);
    if (i0 >= lim) return;
    const int tid = threadIdx.x;
    for (int b = tid; b < kSortBins; b += kSortWG) s_h[b] = 0;
    __syncthreads();
    int key[kSortPer], rank[kSortPer], jj[kSortPer];
#pragma unroll
    for (int t = 0; t < kSortPer; t++) {
        const int i = i0 + t * kSortWG + tid;
        key[t] = -1; rank[t] = 0; jj[t] = 0;
        if (i < lim) {
            const int c = i / p.chunk, r = i - c * p.chunk;
            if (r < p.blk_cnt[c]) {
                key[t] = p.sort_key[i];
                jj[t] = p.blk_off[c] + r;
                rank[t] = atomicAdd(&s_h[key[t]], 1);
            }
        }
    }
    __syncthreads();
    for (int b = tid; b < kSortBins; b += kSortWG) {
        const int c = s_h[b];
        if (c) s_h[b] = atomicAdd(&p.sort_bins[kSortBins + b], c);   // cursor starts at the key's prefix
    }
    __syncthreads();
#pragma unroll
    for (int t = 0; t < kSortPer; t++)
        if (key[t] >= 0) {
            const int pos = s_h[key[t]] + rank[t];
            p.order[pos] = make_int2(jj[t], i0 + t * kSortWG + tid);
        }
}

__global__ void k_selftest_math(int n, const float* x, const float* y, float* out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float sv, cv;
    sincos_ref(x[i], &sv, &cv);
    out[5 * i + 0] = sv;
    out[5 * i + 1] = cv;
    out[5 * i + 2] = powf_ref(x[i], y[i]);
    out[5 * i + 3] = sqrtf(x[i]);
    out[5 * i + 4] = x[i] / y[i];
}

// image += contribution of one iteration: one add per element, n = W*H*3 floats
// (scalar: the image may be a caller-bound buffer with only 4-byte alignment).
__global__ __launch_bounds__(256) void k_merge(float* __restrict__ image, const float* __restrict__ contrib, size_t n) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) image[i] += contrib[i];
}

// hipGraph replay: the iteration id the captured k_bounce launches read
__global__ void k_set_iter(int* dst, int iter) {
    if (threadIdx.x == 0) *dst = iter;
}

__global__ void k_zero(float* a, size_t n) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) a[i] = 0.0f;
}

// ---------------------------------------------------------------------------
// Host side
// ---------------------------------------------------------------------------
Renderer::Renderer(const RenderConfig& c) : cfg(c) {}
Renderer::~Renderer() { free(); }

int Renderer::fail(hipError_t e, const char* what) {
    last_error = std::string(what) + ": " + hipGetErrorString(e);
    return -1;
}

#define PT_HIP(call)                                   \
    do {                                               \
        hipError_t _e = (call);                        \
        if (_e != hipSuccess) return fail(_e, #call);  \
    } while (0)

int Renderer::setStream(hipStream_t s) {
    if (own_stream && stream) {
        hipStreamSynchronize(stream);
        hipStreamDestroy(stream);
    }
    stream = s;               // may be the null (default) stream
    stream_set = true;
    own_stream = false;
    return 0;
}

int Renderer::bindImage(float* device_rgb) {
    if (allocated && !external_image && kp.image) { last_error = "bind_image must precede allocateOnGPU"; return -1; }
    ext_image = device_rgb;
    external_image = device_rgb != nullptr;
    if (allocated) {
        // captured launches hold the old image pointer: let every launch already
        // enqueued (graphs included) finish before their executables are destroyed
        PT_HIP(hipStreamSynchronize(stream));
        for (int i = 1; i < npipes; i++) PT_HIP(hipStreamSynchronize(pstream[i]));
        dropGraphs();
        kp.image = device_rgb;
        for (int i = 0; i < kMaxPipes; i++) pk[i].image = device_rgb;
    }
    return 0;
}

template <typename T>
static hipError_t upload(std::vector<void*>& allocs, T** dst, const void* src, size_t bytes, hipStream_t s) {
    void* d = nullptr;
    hipError_t e = hipMalloc(&d, bytes ? bytes : 16);
    if (e != hipSuccess) return e;
    allocs.push_back(d);
    if (bytes && src) e = hipMemcpyAsync(d, src, bytes, hipMemcpyHostToDevice, s);
    *dst = (T*)d;
    return e;
}

int Renderer::allocateOnGPU(const Scene& scene) {
    if (!scene.built) { last_error = "scene not built (call build first)"; return -1; }
    if (cfg.width <= 0 || cfg.height <= 0) { last_error = "bad resolution"; return -1; }
    if ((long long)cfg.width * cfg.height > (1LL << 30)) { last_error = "resolution too large"; return -1; }
    for (int k = 0; k < 3; k++)
        if (cfg.grid[k] != scene.grid_dim[k]) { last_error = "config grid dims differ from the scene build"; return -1; }
    if (cfg.accel != ACCEL_GRID && scene.bvh_nodes.empty()) { last_error = "scene built without BVH"; return -1; }
    if (cfg.accel != ACCEL_GRID)     // every BLAS path walks the 4-wide BLAS: there is no binary fallback
        for (const ModelRec& m : scene.model_recs)
            if (m.bvh_root >= 0 && (m.bvh4_root < 0 || scene.bvh4_nodes.empty())) {
                last_error = "a mesh has no 4-wide BLAS (a leaf of more than 31 triangles, 2^26 leaf records or more "
                             "in one mesh, or 2^27 4-wide nodes in the scene: beyond the traversal stacks' "
                             "encodings); use accel grid";
                return -1;
            }
    for (const Voxel& v : scene.voxels)
        if (v.entity_type != ENTITY_TRIANGLE) { last_error = "unsupported voxel entity type"; return -1; }
    freeBuffers();
    if (!stream_set && !stream) {
        PT_HIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
        own_stream = true;
    }
    {
        const char* pe = std::getenv("PT_PIPES");
        npipes = std::max(1, std::min(kMaxPipes, pe ? std::atoi(pe) : cfg.pipelines));
    }
    kp = KParams{};
    kp.defer_launch = 1;
    kp.nmodels = (int)scene.model_recs.size();
    for (int k = 0; k < 3; k++) kp.gdim[k] = scene.grid_dim[k];
    PT_HIP(upload(allocs, &kp.models, scene.model_recs.data(), scene.model_recs.size() * sizeof(ModelRec), stream));
    PT_HIP(upload(allocs, &kp.shade, scene.model_shade.data(), scene.model_shade.size() * sizeof(ModelShade), stream));
    PT_HIP(upload(allocs, &kp.tri_geom, scene.tri_geom.data(), scene.tri_geom.size() * sizeof(float), stream));
    PT_HIP(upload(allocs, &kp.tri_normal, scene.tri_normal.data(), scene.tri_normal.size() * sizeof(float), stream));
    std::vector<int2> vox(scene.voxels.size());
    for (size_t i = 0; i < vox.size(); i++)
        vox[i] = make_int2(scene.voxels[i].entity_index_range.start_index, scene.voxels[i].entity_index_range.end_index);
    PT_HIP(upload(allocs, &kp.voxels, vox.data(), vox.size() * sizeof(int2), stream));
    PT_HIP(upload(allocs, &kp.per_voxel, scene.per_voxel_data_pool.data(), scene.per_voxel_data_pool.size() * sizeof(int), stream));
    // one BLAS on the device: the 4-wide nodes every BLAS path walks (the binary build stays on the
    // host, where the collapse reads it); leaf triangles inline in leaf order
    kp.bvh4 = nullptr;
    if (!scene.bvh4_nodes.empty())
        PT_HIP(upload(allocs, &kp.bvh4, scene.bvh4_nodes.data(), scene.bvh4_nodes.size() * sizeof(Bvh4Node), stream));
    {   // PT_LDS_TOP: the two meshes with the most 4-wide nodes (the one after a root's range bounds it)
        std::vector<std::pair<int, int>> ms;   // (node count, root)
        std::vector<int> roots;
        for (int r : scene.mesh_bvh4_root) if (r >= 0) roots.push_back(r);
        std::sort(roots.begin(), roots.end());
        roots.erase(std::unique(roots.begin(), roots.end()), roots.end());
        for (size_t i = 0; i < roots.size(); i++) {
            const int end = i + 1 < roots.size() ? roots[i + 1] : (int)scene.bvh4_nodes.size();
            ms.push_back({end - roots[i], roots[i]});
        }
        std::sort(ms.rbegin(), ms.rend());
        for (int m = 0; m < 2; m++) {
            kp.top_root[m] = m < (int)ms.size() ? ms[m].second : 0;
            kp.top_n[m] = m < (int)ms.size() ? std::min(ms[m].first, kLdsTop) : 0;
        }
    }
    PT_HIP(upload(allocs, &kp.bvh_tri_geom, scene.bvh_tri_geom.data(), scene.bvh_tri_geom.size() * sizeof(float), stream));

    kp.width = cfg.width;
    kp.height = cfg.height;
    const int npix_all = cfg.width * cfg.height;
    kp.npix = cfg.tail_drop ? (npix_all / 32) * 32 : npix_all;
    kp.max_bounces = cfg.max_bounces;
    {
        const char* dbg = std::getenv("PT_DEBUG_ABLATE");   // timing-only ablations; results become wrong
        kp.debug = dbg ? std::atoi(dbg) : 0;
        // bits 4 (walk / certificate statistics, slots 20..28 and 32..39) and 32 (cycle stamps,
        // slots 20..27) count into the same diagnostic slots: one at a time
        if ((kp.debug & 4) && (kp.debug & 32)) {
            last_error = "PT_DEBUG_ABLATE: bits 4 and 32 share diagnostic slots; set one at a time";
            return -1;
        }
        // persistent-trace safety net; tests lower it to exercise the fault report
        const char* cap = std::getenv("PT_TRACE_ITER_CAP");
        kp.trace_iter_cap = cap ? (unsigned)std::strtoul(cap, nullptr, 10) : (1u << 26);
    }
    kp.chunk = (cfg.block == 64 || cfg.block == 128 || cfg.block == 256) ? cfg.block : 256;
    kp.nblocks = (npix_all + kp.chunk - 1) / kp.chunk;
    kp.step_x = (float)(cfg.plane_w / cfg.width);
    kp.step_y = (float)(cfg.plane_h / cfg.height);
    kp.cam_x = (float)cfg.cam[0]; kp.cam_y = (float)cfg.cam[1]; kp.cam_z = (float)cfg.cam[2];
    kp.plane_z = (float)cfg.plane_z;
    kp.plane_x0 = cfg.plane_x0;
    kp.plane_y0 = cfg.plane_y0;
    const size_t cap = (size_t)kp.nblocks * kp.chunk;
    PT_HIP(upload(allocs, &kp.cache_hit, nullptr, cap * sizeof(float4), stream));
    PT_HIP(upload(allocs, &kp.cache_model, nullptr, cap * sizeof(int), stream));
    if (external_image) kp.image = ext_image;
    else PT_HIP(upload(allocs, &kp.image, nullptr, (size_t)npix_all * 3 * sizeof(float), stream));
    {
        const char* hpb = std::getenv("PT_HS_POOL_BLOCKS");          // 64-member blocks per pipeline
        kp.hs_pool_blocks = cfg.accel == ACCEL_GRID_FAST ? (hpb ? std::max(1, std::atoi(hpb)) : 65536) : 1;   // 64 MiB
    }
    {
        // Persistent trace + shading pass; PT_TRACE_SPLIT=0 / PT_GF_SPLIT=0 keep the fused kernel.
        const char* e = std::getenv("PT_TRACE_SPLIT");
        split_trace = cfg.accel == ACCEL_BVH && !(e && std::atoi(e) == 0);
        const char* eg = std::getenv("PT_GF_SPLIT");
        if (cfg.accel == ACCEL_GRID_FAST) split_trace = eg ? std::atoi(eg) != 0 : true;
        // trace variants: 9 / 11 model records in LDS (the default), 8 / 10 from global memory
        const char* gff = std::getenv("PT_GF_FLAGS");
        // each flag is checked only where it applies (split grid_fast / split bvh): a leftover
        // value does not fail a render whose trace never reads it
        const bool gf_split = split_trace && cfg.accel == ACCEL_GRID_FAST;
        const bool bvh_split = split_trace && cfg.accel == ACCEL_BVH;
        gf_flags = gff && gf_split ? std::atoi(gff) : 9;
        if (gf_flags != 8 && gf_flags != 9) { last_error = "PT_GF_FLAGS must be 8 or 9"; return -1; }
        // 9..12 instances: the default variants with room for 12 LDS model records (F | 32)
        gf_wide_lds = (gf_flags & ~1) == 8 && (gf_flags & 1) && scene.model_recs.size() > (size_t)kLdsModelsGf &&
                      scene.model_recs.size() <= (size_t)kLdsModelsWide;
        if (scene.model_recs.size() > (size_t)kLdsModelsGf && !gf_wide_lds) gf_flags &= ~1;   // records stay global
        const char* rf = std::getenv("PT_TRACE_REFILL");
        // refill a wave once 32 lanes are idle (48 with one pipeline: +2.5 % at configs[1], where a
        // launch has the chip to itself and fewer refills keep more lanes on rays in flight)
        kp.trace_refill = rf ? std::max(1, std::min(64, std::atoi(rf))) : (npipes > 1 ? 32 : 48);
        const char* rpl = std::getenv("PT_TRACE_RPL");
        // 4 rays per lane: +2.4 % at configs[4] (16 bounces, sparse late bounces), neutral at configs[1];
        // off with one pipeline, where a launch has the chip to itself (its idle waves cost nothing).
        // Round 6: 8 for a BLAS beyond the aggregate L2 measured +2..3 % in-process but within noise as
        // separate processes in steady state (1M +0.5 %, 10M 0; profiles/r06/ab_pipes_steady.txt): 4 stays
        kp.trace_rpl = rpl ? std::max(0, std::atoi(rpl)) : (npipes > 1 ? 4 : 0);
        const char* tf = std::getenv("PT_TRACE_FLAGS");
        kp.trace_flags = tf && bvh_split ? std::atoi(tf) : 11;
        if (kp.trace_flags != 10 && kp.trace_flags != 11) { last_error = "PT_TRACE_FLAGS must be 10 or 11"; return -1; }
        // the default variant with 9..12 models: model records in LDS with room for 12 (F | 32)
        bvh_wide_lds = kp.trace_flags == 11 && scene.model_recs.size() > (size_t)kLdsModels &&
                       scene.model_recs.size() <= (size_t)kLdsModelsWide;
        if (scene.model_recs.size() > (size_t)kLdsModels) kp.trace_flags &= ~1;
        int dev = 0, cus = 256;
        if (hipGetDevice(&dev) == hipSuccess) hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        // Waves per CU of a persistent trace launch: with one pipeline the launch
        // fills the chip alone (20; k_trace_gf keeps 16 resident); with several,
        // 8 per launch lets 2-3 pipelines' traces share the CUs, so one launch's
        // drain overlaps another's full waves (measured at 16 pipelines: 20 ->
        // 8 waves 2141 -> 2256 Mrays/s grid_fast, 3211 -> 3393 bvh; 4 / 6 / 10 /
        // 12 / 16 / 32: 2180 / 2232 / 2245 / 2190 / 2188 / 2034).
        const char* wpc = std::getenv("PT_TRACE_WAVES_PER_CU");
        const int w = wpc ? std::max(1, std::atoi(wpc)) : (npipes > 1 ? 8 : 20);
        trace_blocks = std::max(1, cus) * w;
        const char* tb = std::getenv("PT_TAIL_BLOCKS");
        tail_blocks = tb ? std::max(1, std::min(trace_blocks, std::atoi(tb))) : trace_blocks;
        const char* mb = std::getenv("PT_TRACE_MIN_WAVES_PER_CU");
        kp.trace_min_blocks = std::max(1, cus) * (mb ? std::max(1, std::atoi(mb)) : 2);
        // k_trace_gf's 12-entry LDS stack; k_trace_bvh's 4-wide traversal (up to three pushes per node)
        const bool spills = split_trace && (cfg.accel == ACCEL_GRID_FAST || cfg.accel == ACCEL_BVH);
        // drain continuations
        const char* dd = std::getenv("PT_DRAIN_DUMP");
        kp.drain_dump = split_trace ? std::max(0, std::min(64, dd ? std::atoi(dd) : 16)) : 0;
        const char* ddt = std::getenv("PT_DRAIN_DUMP_TAIL");  // a tail that hands on again (PT_DRAIN_LEVELS > 1)
        kp.drain_dump_tail = ddt ? std::max(0, std::min(64, std::atoi(ddt))) : kp.drain_dump;
        const char* trp = std::getenv("PT_TAIL_RPL");
        kp.tail_rpl = trp ? std::max(1, std::atoi(trp)) : 1;
        const char* apl = std::getenv("PT_ALLPHASE_LANES");
        kp.allphase_lanes = apl ? std::max(0, std::min(64, std::atoi(apl))) : 0;
        const char* dfl = std::getenv("PT_DEFER_LAUNCH");
        kp.defer_launch = dfl ? std::atoi(dfl) != 0 : 1;
        const char* trf = std::getenv("PT_TAIL_REFILL");
        kp.tail_refill = trf ? std::max(1, std::min(64, std::atoi(trf))) : kp.trace_refill;
        kp.cont_cap = kp.drain_dump > 0 ? trace_blocks * 64 : 1;
        // walk hand-ons (k_trace_gf main launch -> its level-1 tail): room for one per lane
        // (PT_WALK_WCAP overrides; beyond it a ray goes whole to k_trace_deferred).  With one
        // pipeline the serial tail costs more than the in-place walk saves (measured 927 vs
        // 1306 Mrays/s at configs[1]; 16 pipelines: +2 %), so the main launch walks in place
        // there (variant F | 16) unless PT_WALK_HANDON=1 asks for hand-ons.
        const char* wh = std::getenv("PT_WALK_HANDON");
        const char* wc = std::getenv("PT_WALK_WCAP");
        const bool handon = wh ? std::atoi(wh) != 0 : npipes > 1;
        // Room: one record per lane of the launch, and at least one per 16 pixels -- a large frame
        // hands on more walks per bounce than a launch has lanes (configs[2], 2800x2240: ~145k per
        // bounce against 131k lanes sent 55k rays per sample to k_trace_deferred; -2.4 %).
        kp.cont_wcap = split_trace && cfg.accel == ACCEL_GRID_FAST && handon
                           ? (wc ? std::max(0, std::atoi(wc)) : std::max(trace_blocks * 64, npix_all / 16)) : 0;
        const char* dl = std::getenv("PT_DRAIN_LEVELS");     // tail launches; the last one runs to the end
        kp.drain_levels = std::max(1, std::min(kDrainLevels, dl ? std::atoi(dl) : 1));
        kp.spill_stride = spills ? 2 * trace_blocks * 64 : 1;   // main lanes, then tail lanes' own areas
        // Ray sort before each persistent trace (claim order only; results unchanged).
        const char* so = std::getenv("PT_SORT");
        // auto: key 7 for both persistent traces (bvh: 3421 -> 3571 Mrays/s at 8 waves per CU, 16 pipelines)
        const int want = so ? std::atoi(so) : cfg.ray_sort >= 0 ? cfg.ray_sort : 7;
        kp.sort_mode = split_trace ? std::max(0, std::min(8, want)) : 0;
        float lo[3] = {3e38f, 3e38f, 3e38f}, hi[3] = {-3e38f, -3e38f, -3e38f};
        for (const ModelRec& m : scene.model_recs)
            for (int a = 0; a < 3; a++) { lo[a] = std::min(lo[a], m.wbox[a]); hi[a] = std::max(hi[a], m.wbox[3 + a]); }
        for (int a = 0; a < 3; a++) {
            const float ext = hi[a] - lo[a];
            kp.sort_lo[a] = ext > 0.0f && ext < 1e30f ? lo[a] : 0.0f;
            kp.sort_sc[a] = ext > 0.0f && ext < 1e30f ? 16.0f / ext : 0.0f;
        }
    }
    kp.order = nullptr; kp.sort_bins = nullptr; kp.sort_key = nullptr;
    PT_HIP(upload(allocs, &kp.segments, nullptr, (kDiagCounters + kMaxBounceCounters) * sizeof(unsigned long long), stream));
    PT_HIP(hipMemsetAsync(kp.segments, 0, (kDiagCounters + kMaxBounceCounters) * sizeof(unsigned long long), stream));
    // Pipelines: iterations in flight on their own streams, each with its own
    // ray pools, scan state, hit buffer and work counters (npipes: set above).
    // Drain continuations pay off only when other pipelines' kernels take the
    // wave slots a draining trace frees: with one pipeline they only add the
    // hand-on and the tail launch (measured 0.76 -> 0.91 ms per trace), so
    // they stay off there unless PT_DRAIN_DUMP asks for them.
    if (npipes == 1 && !std::getenv("PT_DRAIN_DUMP")) {
        kp.drain_dump = 0;
        kp.cont_cap = 1;
    }
    kp.cont_cap += kp.cont_wcap;
    kp.contrib = nullptr;
    pstream[0] = stream;
    for (int i = 1; i < npipes; i++) {
        if (!pstream[i]) PT_HIP(hipStreamCreateWithFlags(&pstream[i], hipStreamNonBlocking));
    }
    for (int i = 0; i < npipes; i++) {
        pk[i] = kp;
        if (allocPipe(pk[i], cap, stream) != 0) return -1;
        if (npipes > 1) {
            PT_HIP(upload(allocs, &pk[i].contrib, nullptr, (size_t)npix_all * 3 * sizeof(float), stream));
            PT_HIP(hipMemsetAsync(pk[i].contrib, 0, (size_t)npix_all * 3 * sizeof(float), stream));
        }
        if (!merge_ev[i]) PT_HIP(hipEventCreateWithFlags(&merge_ev[i], hipEventDisableTiming));
    }
    if (!fork_ev) PT_HIP(hipEventCreateWithFlags(&fork_ev, hipEventDisableTiming));
    kp = pk[0];
    PT_HIP(hipStreamSynchronize(stream));
    const char* gr = std::getenv("PT_GRAPH");
    use_graph = gr && std::atoi(gr) != 0;
    allocated = true;
    cache_valid = false;
    return clearImage();
}

// One pipeline's buffers: ray pools, scan state, overflow pool, traversal
// spill, hit buffer and work counters.
int Renderer::allocPipe(KParams& k, size_t cap, hipStream_t st) {
    for (int b = 0; b < 2; b++)
        for (int q = 0; q < 3; q++) PT_HIP(upload(allocs, &k.ray[b][q], nullptr, cap * sizeof(float4), st));
    PT_HIP(upload(allocs, &k.blk_cnt, nullptr, (k.nblocks + 1) * sizeof(int), st));
    PT_HIP(upload(allocs, &k.blk_off, nullptr, (k.nblocks + 2) * sizeof(int), st));
    PT_HIP(upload(allocs, &k.dst_start, nullptr, (k.nblocks + 2) * sizeof(int), st));
    PT_HIP(upload(allocs, &k.n_live, nullptr, (size_t)(cfg.max_bounces + 4) * sizeof(int), st));
    PT_HIP(hipMemsetAsync(k.n_live, 0, (size_t)(cfg.max_bounces + 4) * sizeof(int), st));
    PT_HIP(upload(allocs, &k.hs_pool, nullptr, (size_t)k.hs_pool_blocks * kHitCapPool * sizeof(int4), st));
    PT_HIP(upload(allocs, &k.hs_pool_next, nullptr, sizeof(int), st));
    PT_HIP(hipMemsetAsync(k.hs_pool_next, 0, sizeof(int), st));
    if ((size_t)k.spill_stride * kSpillEntries >= (1ull << 31)) {   // spush_t / spop_if index it in 32 bits
        last_error = "traversal spill area too large";
        return -1;
    }
    PT_HIP(upload(allocs, &k.spill, nullptr, (size_t)k.spill_stride * kSpillEntries * sizeof(int), st));
    const size_t dcap = split_trace && cfg.accel == ACCEL_GRID_FAST ? cap : 1;
    PT_HIP(upload(allocs, &k.defer_slots, nullptr, dcap * sizeof(int), st));
    PT_HIP(upload(allocs, &k.defer_count, nullptr, sizeof(int), st));
    PT_HIP(hipMemsetAsync(k.defer_count, 0, sizeof(int), st));
    if (k.sort_mode) {
        PT_HIP(upload(allocs, &k.order, nullptr, cap * sizeof(int2), st));
        PT_HIP(upload(allocs, &k.sort_key, nullptr, cap * sizeof(unsigned short), st));
        PT_HIP(upload(allocs, &k.sort_bins, nullptr, 2 * kSortBins * sizeof(int), st));
        PT_HIP(hipMemsetAsync(k.sort_bins, 0, 2 * kSortBins * sizeof(int), st));
    }
    const size_t hcap = split_trace ? cap : 1;
    PT_HIP(upload(allocs, &k.hit4, nullptr, hcap * sizeof(float4), st));
    PT_HIP(upload(allocs, &k.hitm, nullptr, hcap * sizeof(int), st));
    // NaN distances / model -1: a record no trace ever wrote (only after a trace
    // fault, which is reported) shades as a miss instead of indexing the models
    PT_HIP(hipMemsetAsync(k.hit4, 0xFF, hcap * sizeof(float4), st));
    PT_HIP(hipMemsetAsync(k.hitm, 0xFF, hcap * sizeof(int), st));
    PT_HIP(upload(allocs, &k.trace_next, nullptr, sizeof(int), st));
    PT_HIP(hipMemsetAsync(k.trace_next, 0, sizeof(int), st));
    PT_HIP(upload(allocs, &k.iter_dev, nullptr, sizeof(int), st));
    PT_HIP(upload(allocs, &k.cont, nullptr, 2 * (size_t)k.cont_cap * kContFields * sizeof(int), st));
    PT_HIP(upload(allocs, &k.cont_count, nullptr, 2 * kDrainLevels * sizeof(int), st));
    PT_HIP(upload(allocs, &k.cont_next, nullptr, kDrainLevels * sizeof(int), st));
    PT_HIP(hipMemsetAsync(k.cont_count, 0, 2 * kDrainLevels * sizeof(int), st));
    PT_HIP(hipMemsetAsync(k.cont_next, 0, kDrainLevels * sizeof(int), st));
    return 0;
}

int Renderer::clearImage() {
    if (!allocated) { last_error = "not allocated"; return -1; }
    const size_t n = (size_t)cfg.width * cfg.height * 3;
    hipLaunchKernelGGL(k_zero, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, kp.image, n);
    PT_HIP(hipGetLastError());
    // a fault invalidated the image it was counted against; the cleared image starts
    // a new render, so later checks report only faults of renders after this point
    PT_HIP(hipMemsetAsync(kp.segments + kTraceFaultCounter, 0, sizeof(unsigned long long), stream));
    return 0;
}

int Renderer::launchPrimary() {
    PT_HIP(hipMemsetAsync(kp.hs_pool_next, 0, sizeof(int), stream));
    const dim3 grid((unsigned)((kp.npix + kBlock - 1) / kBlock));
    if (cfg.accel == ACCEL_BVH) hipLaunchKernelGGL(k_primary<ACCEL_BVH>, grid, dim3(kBlock), 0, stream, kp);
    else if (cfg.accel == ACCEL_GRID_FAST) hipLaunchKernelGGL(k_primary<ACCEL_GRID_FAST>, grid, dim3(kBlock), 0, stream, kp);
    else hipLaunchKernelGGL(k_primary<ACCEL_GRID>, grid, dim3(kBlock), 0, stream, kp);
    PT_HIP(hipGetLastError());
    cache_valid = true;
    return 0;
}

void Renderer::launchTrace(const KParams& k, hipStream_t st, int b) {
    const dim3 g((unsigned)trace_blocks), t(64);
    if (cfg.accel == ACCEL_GRID_FAST) {
        // model records in LDS (gf_flags & 1, cleared by allocateOnGPU when the scene has
        // more models than the tables hold); 9..12 models: the 12-record variants (F | 32).
        // With walk hand-ons the main launch only certifies (F = 9 / 41 / 8), else (F | 16)
        // it walks in place.
        const bool lds = (gf_flags & 1) && k.nmodels <= kLdsModelsGf;
        const bool wide = gf_wide_lds;
        if (k.cont_wcap > 0) {
            if (lds) hipLaunchKernelGGL((k_trace_gf<64, 9>), g, t, 0, st, k, b, 0);
            else if (wide) hipLaunchKernelGGL((k_trace_gf<64, 41>), g, t, 0, st, k, b, 0);
            else hipLaunchKernelGGL((k_trace_gf<64, 8>), g, t, 0, st, k, b, 0);
        } else {
            if (lds) hipLaunchKernelGGL((k_trace_gf<64, 25>), g, t, 0, st, k, b, 0);
            else if (wide) hipLaunchKernelGGL((k_trace_gf<64, 57>), g, t, 0, st, k, b, 0);
            else hipLaunchKernelGGL((k_trace_gf<64, 24>), g, t, 0, st, k, b, 0);
        }
        // tail launches: PT_TAIL_BLOCKS workgroups (experiment; default the main launch's), each lane
        // claiming records until they run out, so any grid traces every record
        const dim3 gt((unsigned)tail_blocks);
        for (int l = 1; (k.drain_dump > 0 && l <= k.drain_levels) || (k.cont_wcap > 0 && l == 1); l++) {
            // the rays handed on (drain continuations; walk hand-ons go to level 1), packed
            if (lds) hipLaunchKernelGGL((k_trace_gf<64, 9, true>), gt, t, 0, st, k, b, l);
            else if (wide) hipLaunchKernelGGL((k_trace_gf<64, 41, true>), gt, t, 0, st, k, b, l);
            else hipLaunchKernelGGL((k_trace_gf<64, 8, true>), gt, t, 0, st, k, b, l);
        }
        // normally empty (grid-stride over the deferred slots): a small grid keeps the empty launch short
        if (k.defer_launch)
            hipLaunchKernelGGL(k_trace_deferred<64>, dim3((unsigned)std::min(trace_blocks, PT_DEFER_WGS)), t, 0, st, k, b);
        return;
    }
    // k_trace_bvh: 11 (LDS records), 43 (11 with room for 12), 10 (records in global memory)
    const bool lds = k.trace_flags == 11 && k.nmodels <= kLdsModels;
    for (int l = 0; l == 0 || (k.drain_dump > 0 && l <= k.drain_levels); l++) {   // main launch, then the tails
        if (bvh_wide_lds) {
            if (l == 0) hipLaunchKernelGGL((k_trace_bvh<64, 43>), g, t, 0, st, k, b, 0);
            else hipLaunchKernelGGL((k_trace_bvh<64, 43, true>), g, t, 0, st, k, b, l);
        } else if (lds) {
            if (l == 0) hipLaunchKernelGGL((k_trace_bvh<64, 11>), g, t, 0, st, k, b, 0);
            else hipLaunchKernelGGL((k_trace_bvh<64, 11, true>), g, t, 0, st, k, b, l);
        } else {
            if (l == 0) hipLaunchKernelGGL((k_trace_bvh<64, 10>), g, t, 0, st, k, b, 0);
            else hipLaunchKernelGGL((k_trace_bvh<64, 10, true>), g, t, 0, st, k, b, l);
        }
    }
}

template <bool FIRST, int BS>
static void launch_bounce_bs(int accel, dim3 grid, hipStream_t st, const KParams& kp, int iter, int b) {
    if (accel == kAccelHitBuffer)
        hipLaunchKernelGGL((k_bounce<FIRST, kAccelHitBuffer, BS>), grid, dim3(BS), 0, st, kp, iter, b);
    else if (accel == ACCEL_BVH) hipLaunchKernelGGL((k_bounce<FIRST, ACCEL_BVH, BS>), grid, dim3(BS), 0, st, kp, iter, b);
    else if (accel == ACCEL_GRID_FAST)
        hipLaunchKernelGGL((k_bounce<FIRST, ACCEL_GRID_FAST, BS>), grid, dim3(BS), 0, st, kp, iter, b);
    else hipLaunchKernelGGL((k_bounce<FIRST, ACCEL_GRID, BS>), grid, dim3(BS), 0, st, kp, iter, b);
}

void Renderer::launchBounce(const KParams& k, hipStream_t st, bool first, dim3 grid, int iter, int b, int accel) {
    switch (k.chunk) {
        case 64:
            if (first) launch_bounce_bs<true, 64>(accel, grid, st, k, iter, b);
            else launch_bounce_bs<false, 64>(accel, grid, st, k, iter, b);
            break;
        case 128:
            if (first) launch_bounce_bs<true, 128>(accel, grid, st, k, iter, b);
            else launch_bounce_bs<false, 128>(accel, grid, st, k, iter, b);
            break;
        default:
            if (first) launch_bounce_bs<true, 256>(accel, grid, st, k, iter, b);
            else launch_bounce_bs<false, 256>(accel, grid, st, k, iter, b);
            break;
    }
}

// One iteration's bounce loop on pipeline q (stream st): sort / trace / shade /
// scan per bounce.  iter = -1: k_bounce reads the id from k.iter_dev (capture).
int Renderer::enqueueIteration(int q, hipStream_t st, int iter, int passes) {
    const KParams& k = pk[q];
    const dim3 grid((unsigned)kp.nblocks + 8u);
    // profiling 1: an event pair around every kernel group on every pipeline; 2: around the
    // trace phases of pipeline 0 only (cheap enough for a timed region: 1/16 of the pairs)
    const bool pall = profiling == 1, ptrace = pall || (profiling == 2 && q == 0);
    for (int b = 0; b < passes; b++) {
        hipEvent_t e0 = nullptr, e1 = nullptr;
        if (b > 0 && split_trace) {
            if (k.order) {
                if (pall) { hipEventCreate(&e0); hipEventCreate(&e1); hipEventRecord(e0, st); }
                const dim3 sg((unsigned)((k.nblocks * (size_t)k.chunk + kSortWG * kSortPer - 1) / (kSortWG * kSortPer)));
                hipLaunchKernelGGL(k_sort_hist, sg, dim3(kSortWG), 0, st, k, b);
                hipLaunchKernelGGL(k_sort_prefix, dim3(1), dim3(kSortWG), 0, st, k);
                hipLaunchKernelGGL(k_sort_scatter, sg, dim3(kSortWG), 0, st, k, b);
                if (pall) { hipEventRecord(e1, st); sort_events.push_back({e0, e1}); e0 = e1 = nullptr; }
            }
            // the trace pair brackets the trace launches only (not the sort kernels)
            if (ptrace) { hipEventCreate(&e0); hipEventCreate(&e1); hipEventRecord(e0, st); }
            launchTrace(k, st, b);
            PT_HIP(hipGetLastError());
            if (ptrace) {
                hipEventRecord(e1, st);
                trace_events.push_back({e0, e1});
                e0 = e1 = nullptr;
            }
            if (pall) { hipEventCreate(&e0); hipEventCreate(&e1); hipEventRecord(e0, st); }
            launchBounce(k, st, false, grid, iter, b, kAccelHitBuffer);
        } else {
            if (pall) { hipEventCreate(&e0); hipEventCreate(&e1); hipEventRecord(e0, st); }
            launchBounce(k, st, b == 0, grid, iter, b, cfg.accel);
        }
        PT_HIP(hipGetLastError());
        if (pall) {
            hipEventRecord(e1, st);
            (b == 0 ? first_events : bounce_events).push_back({e0, e1});
            e0 = e1 = nullptr;
        }
        if (pall) { hipEventCreate(&e0); hipEventCreate(&e1); hipEventRecord(e0, st); }
        hipLaunchKernelGGL(k_scan, dim3(1), dim3(kScanWG), 0, st, k, b);
        PT_HIP(hipGetLastError());
        if (pall) { hipEventRecord(e1, st); scan_events.push_back({e0, e1}); }
    }
    return 0;
}

void Renderer::dropGraphs() {
    for (int i = 0; i < kMaxPipes; i++) {
        if (gexec[i]) hipGraphExecDestroy(gexec[i]);
        gexec[i] = nullptr;
    }
}

int Renderer::renderLoop(int first_iter, int n_iters) {
    if (!allocated) { last_error = "renderLoop before allocateOnGPU"; return -1; }
    if (n_iters < 0 || first_iter < 0) { last_error = "bad iteration range"; return -1; }
    if (kp.npix == 0) return 0;
    if (!kp.image || !kp.cache_hit || !kp.models) { last_error = "renderLoop: device buffers missing"; return -1; }
    if (!cache_valid) {
        hipEvent_t e0 = nullptr, e1 = nullptr;
        if (profiling == 1) { hipEventCreate(&e0); hipEventCreate(&e1); hipEventRecord(e0, stream); }
        if (launchPrimary() != 0) return -1;
        if (profiling == 1) {
            hipEventRecord(e1, stream);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            stats.primary_ms += ms;
            hipEventDestroy(e0); hipEventDestroy(e1);
        }
    }
    const int passes = cfg.max_bounces > 1 ? cfg.max_bounces : 1;
    const int np = npipes;
    if (np > 1) {                                   // fork the pipeline streams off the caller's stream
        PT_HIP(hipEventRecord(fork_ev, stream));
        for (int q = 1; q < np; q++) PT_HIP(hipStreamWaitEvent(pstream[q], fork_ev, 0));
    }
    const size_t n3 = (size_t)cfg.width * cfg.height * 3;
    // Every exit after the fork goes through joinPipes, so a later clearImage /
    // readImage on the caller's stream is ordered after everything enqueued here,
    // also when an iteration fails to enqueue part way through.
    auto body = [&](int it) -> int {
        const int iter = first_iter + it;
        const int q = it % np;
        const KParams& k = pk[q];
        hipStream_t st = q == 0 ? stream : pstream[q];
        if (use_graph && !profiling && st) {   // (no capture on the legacy null stream)
            // The bounce loop's launches are identical every iteration but for the
            // iteration id: capture them once per pipeline (k_bounce reads the id from
            // k.iter_dev) and replay the graph after one k_set_iter.
            hipLaunchKernelGGL(k_set_iter, dim3(1), dim3(64), 0, st, k.iter_dev, iter);
            PT_HIP(hipGetLastError());
            if (!gexec[q]) {
                PT_HIP(hipStreamBeginCapture(st, hipStreamCaptureModeRelaxed));
                const int rc = enqueueIteration(q, st, -1, passes);
                hipGraph_t g = nullptr;
                const hipError_t ec = hipStreamEndCapture(st, &g);
                if (rc != 0) { if (g) hipGraphDestroy(g); return -1; }
                PT_HIP(ec);
                const hipError_t ei = hipGraphInstantiate(&gexec[q], g, nullptr, nullptr, 0);
                hipGraphDestroy(g);
                PT_HIP(ei);
            }
            PT_HIP(hipGraphLaunch(gexec[q], st));
        } else if (enqueueIteration(q, st, iter, passes) != 0) {
            return -1;
        }
        if (np > 1) {
            // image += this iteration's contributions, after the previous iteration's merge
            if (it > 0) PT_HIP(hipStreamWaitEvent(st, merge_ev[(it - 1) % np], 0));
            hipLaunchKernelGGL(k_merge, dim3((unsigned)((n3 + 255) / 256)), dim3(256), 0, st, k.image, k.contrib, n3);
            PT_HIP(hipGetLastError());
            PT_HIP(hipEventRecord(merge_ev[q], st));
        }
        return 0;
    };
    int done = 0;
    int rc = 0;
    for (; done < n_iters; done++) {
        if ((rc = body(done)) != 0) break;
    }
    const std::string err = last_error;
    const int jrc = joinPipes(np);
    if (rc != 0) { last_error = err; return -1; }     // the first failure is the one reported
    return jrc;
}

// Join the forked pipeline streams back into the caller's stream: the caller's
// stream waits for the last merge (which follows every earlier one) and for
// everything else enqueued on each pipeline stream since the fork.
int Renderer::joinPipes(int np) {
    if (np <= 1) return 0;
    for (int q2 = 1; q2 < np; q2++) {
        PT_HIP(hipEventRecord(merge_ev[q2], pstream[q2]));
        PT_HIP(hipStreamWaitEvent(stream, merge_ev[q2], 0));
    }
    return 0;
}

int Renderer::synchronize() {
    if (!allocated && !stream) return 0;
    PT_HIP(hipStreamSynchronize(stream));
    return allocated ? checkFaults() : 0;
}

long long Renderer::traceFaults() {
    if (!allocated) return 0;
    unsigned long long v = 0;
    if (hipMemcpyAsync(&v, kp.segments + kTraceFaultCounter, sizeof v, hipMemcpyDeviceToHost, stream) != hipSuccess)
        return -1;
    if (hipStreamSynchronize(stream) != hipSuccess) return -1;
    return (long long)v;
}

// A persistent trace that hit its iteration cap left rays with stale hit
// records, so the accumulated image is wrong: report it as an error.
int Renderer::checkFaults() {
    const long long f = traceFaults();
    if (f < 0) { last_error = "reading the trace fault counter failed"; return -1; }
    if (f > 0) {
        last_error = "persistent trace gave up on " + std::to_string(f) +
                     " wave(s) (iteration cap): image invalid";
        return -1;
    }
    return 0;
}

int Renderer::setProfiling(int on) {
    if (on < 0 || on > 2) { last_error = "profiling level must be 0, 1 or 2"; return -1; }
    profiling = on;
    return 0;
}

int Renderer::kernelStats(KernelStats* out) {
    PT_HIP(hipStreamSynchronize(stream));
    for (auto& ev : bounce_events) {
        float ms = 0;
        hipEventElapsedTime(&ms, ev.first, ev.second);
        stats.bounce_ms += ms;
        stats.bounce_launches++;
        hipEventDestroy(ev.first); hipEventDestroy(ev.second);
    }
    for (auto& ev : first_events) {
        float ms = 0;
        hipEventElapsedTime(&ms, ev.first, ev.second);
        stats.first_ms += ms;
        stats.first_launches++;
        hipEventDestroy(ev.first); hipEventDestroy(ev.second);
    }
    first_events.clear();
    for (auto& ev : trace_events) {
        float ms = 0;
        hipEventElapsedTime(&ms, ev.first, ev.second);
        stats.trace_ms += ms;
        stats.trace_launches++;
        hipEventDestroy(ev.first); hipEventDestroy(ev.second);
    }
    trace_events.clear();
    for (auto& ev : sort_events) {
        float ms = 0;
        hipEventElapsedTime(&ms, ev.first, ev.second);
        stats.sort_ms += ms;
        stats.sort_launches++;
        hipEventDestroy(ev.first); hipEventDestroy(ev.second);
    }
    sort_events.clear();
    for (auto& ev : scan_events) {
        float ms = 0;
        hipEventElapsedTime(&ms, ev.first, ev.second);
        stats.scan_ms += ms;
        stats.scan_launches++;
        hipEventDestroy(ev.first); hipEventDestroy(ev.second);
    }
    bounce_events.clear();
    scan_events.clear();
    *out = stats;
    stats = KernelStats();
    return 0;
}

long long Renderer::segments() {
    if (!allocated) return 0;
    unsigned long long v = 0;
    if (hipMemcpyAsync(&v, kp.segments, sizeof v, hipMemcpyDeviceToHost, stream) != hipSuccess) return -1;
    if (hipStreamSynchronize(stream) != hipSuccess) return -1;
    return (long long)v;
}

int Renderer::segmentsPerBounce(long long* out, int n) {
    if (!allocated) { last_error = "not allocated"; return -1; }
    unsigned long long v[kDiagCounters + kMaxBounceCounters];
    PT_HIP(hipMemcpyAsync(v, kp.segments, sizeof v, hipMemcpyDeviceToHost, stream));
    PT_HIP(hipStreamSynchronize(stream));
    for (int i = 0; i < n && i < kMaxBounceCounters + kDiagCounters - 1; i++) out[i] = (long long)v[1 + i];
    for (int i = kMaxBounceCounters + kDiagCounters - 1; i < n; i++) out[i] = 0;
    return 0;
}

int Renderer::readImage(float* host_rgb) {
    if (!allocated) { last_error = "not allocated"; return -1; }
    PT_HIP(hipMemcpyAsync(host_rgb, kp.image, (size_t)cfg.width * cfg.height * 3 * sizeof(float), hipMemcpyDeviceToHost, stream));
    PT_HIP(hipStreamSynchronize(stream));
    return checkFaults();
}

// Renderer::renderImage (Renderer.cpp:15-63): 54-byte BMP header, rows written
// y = 0 (bottom) first, bytes (x, y, z) of (sum * (1/ITER)) * 255 cast to char.
int Renderer::renderImage(const std::string& path, int iterations_total) {
    std::vector<float> img((size_t)cfg.width * cfg.height * 3);
    if (readImage(img.data()) != 0) return -1;
    const int W = cfg.width, H = cfg.height;
    unsigned char hdr[54] = {'B', 'M', 0, 0, 0, 0, 0, 0, 0, 0, 54, 0, 0, 0, 40, 0, 0, 0};
    std::memcpy(hdr + 18, &W, 4);
    std::memcpy(hdr + 22, &H, 4);
    hdr[26] = 1; hdr[28] = 24;
    const int file_size = 54 + 3 * W * H, image_size = 3 * W * H;
    std::memcpy(hdr + 2, &file_size, 4);
    std::memcpy(hdr + 34, &image_size, 4);
    std::ofstream out(path, std::ios::binary);
    if (!out) { last_error = "cannot open " + path; return -1; }
    out.write((const char*)hdr, 54);
    std::vector<unsigned char> row((size_t)W * 3);
    const float div = 1 / (float)iterations_total;
    for (int y = 0; y < H; y++) {
        for (int x = 0; x < W; x++)
            for (int k = 0; k < 3; k++) {
                const float v = (img[3 * ((size_t)x + (size_t)y * W) + k] * div) * 255.0f;
                row[3 * x + k] = (unsigned char)(f2i_x86(v) & 0xFF);
            }
        out.write((const char*)row.data(), (std::streamsize)row.size());
    }
    return out ? 0 : -1;
}

int Renderer::primaryHits(float* dist, float* normal, int* model) {
    if (!allocated) { last_error = "not allocated"; return -1; }
    if (!cache_valid && launchPrimary() != 0) return -1;
    std::vector<float4> hit(kp.npix);
    PT_HIP(hipMemcpyAsync(hit.data(), kp.cache_hit, kp.npix * sizeof(float4), hipMemcpyDeviceToHost, stream));
    PT_HIP(hipMemcpyAsync(model, kp.cache_model, kp.npix * sizeof(int), hipMemcpyDeviceToHost, stream));
    PT_HIP(hipStreamSynchronize(stream));
    for (int i = 0; i < kp.npix; i++) {
        dist[i] = hit[i].x;
        normal[3 * i] = hit[i].y; normal[3 * i + 1] = hit[i].z; normal[3 * i + 2] = hit[i].w;
    }
    return 0;
}

int Renderer::intersectRays(int n, const float* orig, const float* dir, float* dist, float* normal, int* model) {
    if (!allocated) { last_error = "not allocated"; return -1; }
    if (n <= 0) return 0;
    float *d_o, *d_d, *d_t, *d_n;
    int* d_m;
    PT_HIP(hipMalloc(&d_o, n * 12));
    PT_HIP(hipMalloc(&d_d, n * 12));
    PT_HIP(hipMalloc(&d_t, n * 4));
    PT_HIP(hipMalloc(&d_n, n * 12));
    PT_HIP(hipMalloc(&d_m, n * 4));
    PT_HIP(hipMemcpyAsync(d_o, orig, n * 12, hipMemcpyHostToDevice, stream));
    PT_HIP(hipMemcpyAsync(d_d, dir, n * 12, hipMemcpyHostToDevice, stream));
    PT_HIP(hipMemsetAsync(kp.hs_pool_next, 0, sizeof(int), stream));
    const dim3 grid((unsigned)((n + kBlock - 1) / kBlock));
    if (cfg.accel == ACCEL_BVH) hipLaunchKernelGGL(k_intersect_rays<ACCEL_BVH>, grid, dim3(kBlock), 0, stream, kp, n, d_o, d_d, d_t, d_n, d_m);
    else if (cfg.accel == ACCEL_GRID_FAST)
        hipLaunchKernelGGL(k_intersect_rays<ACCEL_GRID_FAST>, grid, dim3(kBlock), 0, stream, kp, n, d_o, d_d, d_t, d_n, d_m);
    else hipLaunchKernelGGL(k_intersect_rays<ACCEL_GRID>, grid, dim3(kBlock), 0, stream, kp, n, d_o, d_d, d_t, d_n, d_m);
    PT_HIP(hipGetLastError());
    PT_HIP(hipMemcpyAsync(dist, d_t, n * 4, hipMemcpyDeviceToHost, stream));
    PT_HIP(hipMemcpyAsync(normal, d_n, n * 12, hipMemcpyDeviceToHost, stream));
    PT_HIP(hipMemcpyAsync(model, d_m, n * 4, hipMemcpyDeviceToHost, stream));
    PT_HIP(hipStreamSynchronize(stream));
    hipFree(d_o); hipFree(d_d); hipFree(d_t); hipFree(d_n); hipFree(d_m);
    return 0;
}

int Renderer::certifyCheck(int n, const float* orig, const float* dir, int* out4) {
    if (!allocated) { last_error = "not allocated"; return -1; }
    if (cfg.accel != ACCEL_GRID_FAST) { last_error = "certify_check needs accel grid_fast (the BLAS hit sets)"; return -1; }
    if (n <= 0) return 0;
    float *d_o, *d_d;
    int4* d_out;
    PT_HIP(hipMalloc(&d_o, n * 12));
    PT_HIP(hipMalloc(&d_d, n * 12));
    PT_HIP(hipMalloc(&d_out, n * sizeof(int4)));
    PT_HIP(hipMemcpyAsync(d_o, orig, n * 12, hipMemcpyHostToDevice, stream));
    PT_HIP(hipMemcpyAsync(d_d, dir, n * 12, hipMemcpyHostToDevice, stream));
    const dim3 grid((unsigned)((n + kBlock - 1) / kBlock));
    hipLaunchKernelGGL(k_certify_check, grid, dim3(kBlock), 0, stream, kp, n, d_o, d_d, d_out);
    PT_HIP(hipGetLastError());
    PT_HIP(hipMemcpyAsync(out4, d_out, n * sizeof(int4), hipMemcpyDeviceToHost, stream));
    PT_HIP(hipStreamSynchronize(stream));
    hipFree(d_o); hipFree(d_d); hipFree(d_out);
    return 0;
}

int selftest_math(int n, const float* x, const float* y, float* out, std::string* err) {
    if (n == 0) return 0;
    float *dx = nullptr, *dy = nullptr, *dout = nullptr;
    hipError_t e = hipMalloc(&dx, n * 4);
    if (e == hipSuccess) e = hipMalloc(&dy, n * 4);
    if (e == hipSuccess) e = hipMalloc(&dout, (size_t)n * 20);
    if (e == hipSuccess) e = hipMemcpy(dx, x, n * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(dy, y, n * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_selftest_math, dim3((n + 255) / 256), dim3(256), 0, 0, n, dx, dy, dout);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpy(out, dout, (size_t)n * 20, hipMemcpyDeviceToHost);
    hipFree(dx); hipFree(dy); hipFree(dout);
    if (e != hipSuccess) { *err = std::string("selftest_math: ") + hipGetErrorString(e); return -1; }
    return 0;
}

void Renderer::freeBuffers() {
    if (allocated || stream) hipStreamSynchronize(stream);
    for (int i = 1; i < kMaxPipes; i++)
        if (pstream[i]) hipStreamSynchronize(pstream[i]);
    dropGraphs();
    for (void* p : allocs) hipFree(p);
    allocs.clear();
    kp.image = nullptr;
    allocated = false;
    cache_valid = false;
}

void Renderer::free() {
    freeBuffers();
    for (auto& ev : bounce_events) { hipEventDestroy(ev.first); hipEventDestroy(ev.second); }
    for (auto& ev : first_events) { hipEventDestroy(ev.first); hipEventDestroy(ev.second); }
    for (auto& ev : scan_events) { hipEventDestroy(ev.first); hipEventDestroy(ev.second); }
    for (auto& ev : trace_events) { hipEventDestroy(ev.first); hipEventDestroy(ev.second); }
    for (auto& ev : sort_events) { hipEventDestroy(ev.first); hipEventDestroy(ev.second); }
    trace_events.clear();
    sort_events.clear();
    bounce_events.clear();
    first_events.clear();
    scan_events.clear();
    for (int i = 1; i < kMaxPipes; i++) {
        if (pstream[i]) hipStreamDestroy(pstream[i]);
        pstream[i] = nullptr;
    }
    for (int i = 0; i < kMaxPipes; i++) {
        if (merge_ev[i]) hipEventDestroy(merge_ev[i]);
        merge_ev[i] = nullptr;
    }
    if (fork_ev) hipEventDestroy(fork_ev);
    fork_ev = nullptr;
    if (own_stream && stream) hipStreamDestroy(stream);
    stream = nullptr;
    own_stream = false;
    stream_set = false;
}

}  // namespace pt
