// scene.h -- host-side scene for the MI355X path tracer.
//
// Mirrors the reference's Scene (Scene.h:21-40): the same member vectors
// (models, meshes, vertices, triangles, grids, voxels, per_voxel_data_pool)
// built with the same rules (Scene.cpp:226-396), plus the device-ready
// tables the gfx950 kernels read (precomputed triangle edges/normals,
// per-model transform records, BVH nodes).
#pragma once

#include <string>
#include <vector>

#include "pt_types.h"

namespace pt {

struct Vertex { f3 position; f3 normal; };            // Primitive.h:23-28 (uv unused)
struct Triangle { int vertex_indices[3]; };            // Primitive.h:30-33
struct BoundingBox {                                   // Primitive.h:35-60
    f3 min = {kFMax, kFMax, kFMax};
    f3 max = {kFMin, kFMin, kFMin};
    void update(f3 v) {
        min.x = min.x > v.x ? v.x : min.x;
        min.y = min.y > v.y ? v.y : min.y;
        min.z = min.z > v.z ? v.z : min.z;
        max.x = max.x < v.x ? v.x : max.x;
        max.y = max.y < v.y ? v.y : max.y;
        max.z = max.z < v.z ? v.z : max.z;
    }
};
struct IndexRange { int start_index = 0, end_index = 0; };    // Primitive.h:14-18
struct Mesh { IndexRange vertex_indices, triangle_indices; BoundingBox bounding_box; };  // Primitive.h:86-91
struct Material { int material_type = MAT_DIFFUSE; float color[3] = {1, 1, 1}; };       // Primitive.h:68-84
struct Model {                                          // Primitive.h:94-101
    int grid_index = -1;
    int mesh_index = 0;
    float model_to_world[16];                           // column-major glm::mat4
    float world_to_model[16];
    Material mat;
};
struct Voxel { IndexRange entity_index_range; int entity_type = ENTITY_TRIANGLE; };  // Primitive.h:123-127
struct Grid {                                           // Primitive.h:129-139
    IndexRange voxelIndices;
    float voxel_width[3];
    int entity_type = ENTITY_MODEL;
    int entity_index = 0;
};

struct RenderSettings {                                 // Config.h constants, runtime
    int width = 1000, height = 800, iterations = 500, max_bounces = 5;
    int grid[3] = {25, 25, 25};
    int accel = ACCEL_GRID_FAST;
    bool has_width = false, has_iterations = false, has_bounces = false, has_accel = false;
};

class Scene {
public:
    Scene() = default;
    // Scene::Scene(string config) (Scene.cpp:3): parse a Config.txt-grammar file.
    // Returns 0 or a negative error (message in last_error()).
    int loadConfig(const std::string& path);

    // Scene::loadAndProcessMeshFile (Scene.cpp:226-238) -> mesh index or -1.
    int loadObj(const std::string& path);
    // Scene::processMesh (Scene.cpp:264-291) on raw (unscaled) arrays -> mesh index.
    int addMesh(const float* pos, const float* nrm, int nv, const int* tris, int nt);
    // Scene.cpp:32-42 pattern; returns model index.
    int addModel(int mesh_index, const float scale[3], const float rot_deg[3],
                 const float translate[3], int material_type, const float color[3]);
    // addMeshesToGrid (Scene.cpp:318-396) + device tables.  `grid_dim` = GRID_X/Y/Z.
    int build(const int grid_dim[3], bool with_bvh);
    // The BLAS on demand: Renderer::allocateOnGPU calls this for the accels that
    // traverse it (grid_fast, bvh) when the scene was built grid-only.
    int ensureBvh();

    // Scene.h:26-32
    std::vector<Model> models;
    std::vector<Mesh> meshes;
    std::vector<Vertex> vertices;
    std::vector<Triangle> triangles;
    std::vector<Grid> grids;
    std::vector<Voxel> voxels;
    std::vector<int> per_voxel_data_pool;

    // Device-ready tables (filled by build()).
    int grid_dim[3] = {25, 25, 25};
    bool built = false;
    std::vector<float> tri_geom;      // 12 floats / triangle: v0.xyz,_, e1.xyz,_, e2.xyz,_
    std::vector<float> tri_normal;    // 4 floats / triangle: normalize((n0+n1+n2)*(1/3))
    std::vector<ModelRec> model_recs;
    std::vector<ModelShade> model_shade;  // per model: material (shading pass)
    std::vector<BvhNode> bvh_nodes;   // all meshes' BLAS, concatenated
    std::vector<int> bvh_tri_order;   // leaf triangle references (global triangle index)
    std::vector<float> bvh_tri_geom;  // 12 floats / leaf reference: tri_geom in leaf order; w lanes carry
                                      // the triangle index and its packed grid voxel box (mn, mx; 10 bits/axis)
    std::vector<int> tri_vbox;        // 2 ints / triangle: packed computeVoxelIndex min / max
    std::vector<int> mesh_bvh_root;
    std::vector<Bvh4Node> bvh4_nodes; // the same BLAS collapsed 4-wide (k_trace_gf), all meshes
    std::vector<int> mesh_bvh4_root;  // -1: no 4-wide BLAS (empty mesh, or a leaf the encoding cannot hold)
    std::vector<int> mesh_leaf_base;  // the mesh's first bvh_tri_order entry (4-wide leaf entries are relative)

    RenderSettings settings;          // optional RENDER block of the config
    std::string last_error;

private:
    int addVertexRun(const std::vector<f3>& pos, const std::vector<f3>& nrm,
                     const std::vector<int>& tri_local);
    void addMeshesToGrid();
    void buildDeviceTables();
    void buildBvh(int mesh);
    int relayoutPairs(int n0, int root);       // sibling inner nodes side by side (bvh.cpp)
    void buildBvh4();                          // 4-wide collapse of every mesh's binary BLAS (bvh.cpp)
    void world_box(const Model& m, const Mesh& mesh, int root, float* out) const;
};

// glm restatements (Scene.cpp:30-39): M = T * R * S, W = inverse(M).
void model_matrices(const float scale[3], const float rot_deg[3], const float translate[3],
                    float m2w[16], float w2m[16]);

}  // namespace pt
