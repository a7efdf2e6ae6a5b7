// pt_types.h -- POD records shared by the host scene builder and the kernels.
#pragma once

#include "pt_math.h"

namespace pt {

// Primitive.h:109-114 SpatialAcceleration::EntityType
enum EntityType : int { ENTITY_MODEL = 0, ENTITY_SCENE = 1, ENTITY_TRIANGLE = 2, ENTITY_SPHERE = 3 };

// Acceleration structure used by the intersect stage.
//  ACCEL_GRID: the reference's per-mesh uniform grid + 3D-DDA with its
//              "2 voxels past the last hit" early exit (Renderer.cpp:238-360);
//              bit-exact with the reference algorithm.
//  ACCEL_BVH : MI355X BLAS per mesh (binned SAH, 2-wide nodes, LDS stacks),
//              exact closest hit with the reference's triangle test; equals
//              the grid result except where the grid's early exit misses a
//              nearer triangle.
//  ACCEL_GRID_FAST: the ACCEL_GRID result computed without voxel triangle
//              lists: the BLAS collects the ray's hit set H (every triangle the
//              reference test accepts), then the reference DDA walks the grid
//              testing only voxel-box membership of H.  Bit-identical to
//              ACCEL_GRID; needs the BVH.
enum Accel : int { ACCEL_GRID = 0, ACCEL_BVH = 1, ACCEL_GRID_FAST = 2 };

// Deepest BLAS inner-node level below a root (bvh.cpp's builder caps the depth
// here).  A traversal holds at most one deferred sibling per level, so a lane's
// stack needs kMaxBvhDepth entries; renderer.hip asserts its LDS stacks (kStack)
// hold that many, since k_trace_bvh and the one-lane paths have no spill path.
constexpr int kMaxBvhDepth = 23;

// One instance (Model, Primitive.h:94-101) flattened for the traces: 62
// dwords (the material, which only the shading pass reads, is ModelShade), so
// k_trace_gf stages up to 12 of them in LDS at 16 resident waves per CU.
struct ModelRec {
    float w2m[12];        // world_to_model columns 0..3, rows 0..2 (m[c*3+k])
    float m2w[12];        // model_to_world, same packing
    float nm[9];          // inverse(mat3(model_to_world)): nm[r*3+c] = Inverse[r][c]
    float bbox[6];        // mesh bounding box (model space) min3 max3
    float vw[3];          // grid voxel widths
    int vox_start;        // grid->voxelIndices.start_index
    int leaf_base;        // the mesh's first leaf record (bvh_tri_order entry): 4-wide leaf entries are relative to it
    int tri_start, tri_end;
    int bvh_root;         // index of the mesh's BLAS root node
    float wbox[6];        // conservative world-space AABB of everything the instance can hit
    float reach;          // R: max over triangles of the (tolerance-grown) voxel-box diameter, model units
    int bvh4_root;        // index of the mesh's 4-wide BLAS root (Bvh4Node), -1: none (the 4-wide traces refuse it)
    float wdelta;         // tier-1 window: the walk is exact up to t_min + wdelta
    float ivw[3];         // 1 / vw (rounded; walk certificate only, used with margins)
    float cslack[3];      // walk certificate: position slack per axis (DDA +EPSILON shift + rounding)
};
static_assert(sizeof(ModelRec) == 62 * 4, "ModelRec layout");

// The instance's material (Primitive.h:68-84), read by the shading pass.
struct ModelShade {
    float color[3];       // Material::color
    int mat_type;         // Material::MaterialType
};

// 2-wide BVH node: both children's boxes in one 64-byte line.
// link/count: count == 0 -> link is a child node index; count > 0 -> link is
// the first entry of bvh_tri_order and count the number of triangles.
struct BvhNode {
    float lo0[3]; int link0;
    float hi0[3]; int link1;
    float lo1[3]; int count0;
    float hi1[3]; int count1;
};
static_assert(sizeof(BvhNode) == 64, "BvhNode layout");

// 4-wide BLAS node for the traces' node steps: a binary node and its children
// collapsed, so one 128-byte fetch (one dependent round trip) tests what the
// binary layout tests in two.  Child c's box is (lo*[c], hi*[c]); count[c] -1 =
// empty (box lo = +inf, hi = -inf: the node steps' near / far slab test misses
// it by itself, so they never load count), 0 = inner (link = Bvh4Node index), > 0 = leaf, whose link is already
// the traversal stack's leaf entry (1 << 31) | count << kLeafCountShift | first
// (first = its first bvh_tri_order entry minus the mesh's ModelRec::leaf_base),
// so a node step pushes links as they are.  The same boxes as the binary nodes: only the number of fetches per
// traversal changes, never the set of triangles tested.
struct Bvh4Node {
    float lox[4], loy[4], loz[4];
    float hix[4], hiy[4], hiz[4];
    int link[4];
    int count[4];
};
static_assert(sizeof(Bvh4Node) == 128, "Bvh4Node layout");
// Leaf children pushed on k_trace_gf's 4-wide traversal stack are encoded as
// (1 << 31) | (count << kLeafCountShift) | first: count <= kMaxLeafCount4,
// first (mesh-relative) < 2^kLeafCountShift (Scene::buildBvh4 checks both).
constexpr int kLeafCountShift = 26;
constexpr int kMaxLeafCount4 = 31;


}  // namespace pt
