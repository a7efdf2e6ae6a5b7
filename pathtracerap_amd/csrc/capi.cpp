// capi.cpp -- extern "C" boundary (include/pathtracer_amd.h).
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>

#include "../../include/pathtracer_amd.h"
#include "renderer.h"
#include "scene.h"

// bvh_mu: pt_renderer_allocate_on_gpu may add the BLAS to a scene built grid-only;
// renderers allocating from one shared scene on several threads (ctypes drops the
// GIL) take turns there, and only the first one builds
struct pt_scene { pt::Scene s; std::mutex bvh_mu; };
struct pt_renderer { pt::Renderer* r; };

static thread_local std::string g_err;

// Iterations in flight run on their own HIP streams (pt_render_config.pipelines,
// default 16); HIP maps streams onto GPU_MAX_HW_QUEUES hardware queues (default
// 4), so with the default several pipelines share a queue and serialise
// (DESIGN.md "Results": 8 pipelines on 4 queues ran 1570 Mrays/s at configs[1]).  The variable is read once, when
// the HIP runtime initialises: set it at load time unless the process already
// chose a value.  (A process whose HIP runtime started before this library was
// loaded keeps its own setting.)
// What the process had chosen is recorded (pt_hw_queue_info), so a host can
// report the queue count in effect or warn when it differs from the default.
static int g_queues_at_load = -1;        // GPU_MAX_HW_QUEUES when the library loaded (-1: unset)
static int g_queues_set_by_lib = 0;      // 1: the library set it (the process had not)
__attribute__((constructor)) static void pt_default_hw_queues() {
    const char* e = std::getenv("GPU_MAX_HW_QUEUES");
    if (e) {
        g_queues_at_load = std::atoi(e);
    } else {
        setenv("GPU_MAX_HW_QUEUES", "16", /*overwrite=*/0);
        g_queues_set_by_lib = 1;
    }
}

static int set_err(const std::string& m) { g_err = m; return -1; }

extern "C" {

int pt_abi_version(void) { return PT_ABI_VERSION; }

int pt_hw_queue_info(int* at_load, int* set_by_library) {
    if (at_load) *at_load = g_queues_at_load;
    if (set_by_library) *set_by_library = g_queues_set_by_lib;
    return 0;
}
const char* pt_last_error(void) { return g_err.c_str(); }

void pt_default_config(pt_render_config* c) {
    pt::RenderConfig d;
    c->width = d.width; c->height = d.height; c->iterations = d.iterations; c->max_bounces = d.max_bounces;
    c->accel = d.accel;
    for (int k = 0; k < 3; k++) { c->grid[k] = d.grid[k]; c->cam[k] = d.cam[k]; }
    c->tail_drop = d.tail_drop;
    c->plane_z = d.plane_z; c->plane_x0 = d.plane_x0; c->plane_y0 = d.plane_y0;
    c->plane_w = d.plane_w; c->plane_h = d.plane_h;
    c->block = d.block;
    c->pipelines = d.pipelines;
    c->ray_sort = d.ray_sort;
}

static pt::RenderConfig to_cfg(const pt_render_config* c) {
    pt::RenderConfig d;
    d.width = c->width; d.height = c->height; d.iterations = c->iterations; d.max_bounces = c->max_bounces;
    d.accel = c->accel;
    for (int k = 0; k < 3; k++) { d.grid[k] = c->grid[k]; d.cam[k] = c->cam[k]; }
    d.tail_drop = c->tail_drop;
    d.plane_z = c->plane_z; d.plane_x0 = c->plane_x0; d.plane_y0 = c->plane_y0;
    d.plane_w = c->plane_w; d.plane_h = c->plane_h;
    d.block = c->block;
    d.pipelines = c->pipelines;
    d.ray_sort = c->ray_sort;
    return d;
}

pt_scene* pt_scene_create(void) {
    try { return new pt_scene(); } catch (...) { set_err("out of memory"); return nullptr; }
}
void pt_scene_destroy(pt_scene* s) { delete s; }

#define SCENE_CALL(expr)                                  \
    do {                                                  \
        if (!s) return set_err("null scene");             \
        try {                                             \
            int _rc = (expr);                             \
            if (_rc < 0) return set_err(s->s.last_error); \
            return _rc;                                   \
        } catch (const std::exception& e) {               \
            return set_err(e.what());                     \
        }                                                 \
    } while (0)

int pt_scene_load_config(pt_scene* s, const char* path) { SCENE_CALL(s->s.loadConfig(path ? path : "")); }

int pt_scene_apply_settings(const pt_scene* s, pt_render_config* c) {
    if (!s || !c) return set_err("null argument");
    const pt::RenderSettings& st = s->s.settings;
    if (st.has_width) { c->width = st.width; c->height = st.height; }
    if (st.has_iterations) c->iterations = st.iterations;
    if (st.has_bounces) c->max_bounces = st.max_bounces;
    if (st.has_accel) c->accel = st.accel;
    for (int k = 0; k < 3; k++) c->grid[k] = st.grid[k];
    return 0;
}

int pt_scene_load_obj(pt_scene* s, const char* path) { SCENE_CALL(s->s.loadObj(path ? path : "")); }

int pt_scene_add_mesh(pt_scene* s, const float* pos, const float* nrm, int nv, const int* tris, int nt) {
    if (!pos || !nrm || !tris || nv < 0 || nt < 0) return set_err("pt_scene_add_mesh: bad arguments");
    SCENE_CALL(s->s.addMesh(pos, nrm, nv, tris, nt));
}

int pt_scene_add_model(pt_scene* s, int mesh, const float scale[3], const float rot[3], const float tr[3],
                       int material, const float color[3]) {
    if (!scale || !rot || !tr || !color) return set_err("pt_scene_add_model: null argument");
    SCENE_CALL(s->s.addModel(mesh, scale, rot, tr, material, color));
}

int pt_scene_build(pt_scene* s, const int grid[3], int with_bvh) {
    const int def[3] = {25, 25, 25};
    SCENE_CALL(s->s.build(grid ? grid : def, with_bvh != 0));
}

int pt_scene_counts(const pt_scene* s, int c[9]) {
    if (!s || !c) return set_err("null argument");
    const pt::Scene& S = s->s;
    c[0] = (int)S.vertices.size(); c[1] = (int)S.triangles.size(); c[2] = (int)S.meshes.size();
    c[3] = (int)S.models.size(); c[4] = (int)S.grids.size(); c[5] = (int)S.voxels.size();
    c[6] = (int)S.per_voxel_data_pool.size(); c[7] = (int)S.bvh_nodes.size(); c[8] = (int)S.bvh_tri_order.size();
    return 0;
}

int pt_scene_export(const pt_scene* s, float* vpos, float* vnrm, int* tris, int* mesh_ranges, float* mesh_bbox,
                    int* model_ints, float* m2w, float* w2m, float* color, int* grid_ints, float* grid_vw,
                    int* vox, int* per_voxel) {
    if (!s) return set_err("null scene");
    const pt::Scene& S = s->s;
    for (size_t i = 0; i < S.vertices.size(); i++) {
        const pt::Vertex& v = S.vertices[i];
        if (vpos) { vpos[3 * i] = v.position.x; vpos[3 * i + 1] = v.position.y; vpos[3 * i + 2] = v.position.z; }
        if (vnrm) { vnrm[3 * i] = v.normal.x; vnrm[3 * i + 1] = v.normal.y; vnrm[3 * i + 2] = v.normal.z; }
    }
    if (tris) for (size_t i = 0; i < S.triangles.size(); i++) std::memcpy(tris + 3 * i, S.triangles[i].vertex_indices, 12);
    for (size_t i = 0; i < S.meshes.size(); i++) {
        const pt::Mesh& m = S.meshes[i];
        if (mesh_ranges) {
            mesh_ranges[4 * i] = m.vertex_indices.start_index; mesh_ranges[4 * i + 1] = m.vertex_indices.end_index;
            mesh_ranges[4 * i + 2] = m.triangle_indices.start_index; mesh_ranges[4 * i + 3] = m.triangle_indices.end_index;
        }
        if (mesh_bbox) {
            const pt::BoundingBox& b = m.bounding_box;
            const float v[6] = {b.min.x, b.min.y, b.min.z, b.max.x, b.max.y, b.max.z};
            std::memcpy(mesh_bbox + 6 * i, v, 24);
        }
    }
    for (size_t i = 0; i < S.models.size(); i++) {
        const pt::Model& m = S.models[i];
        if (model_ints) { model_ints[3 * i] = m.mesh_index; model_ints[3 * i + 1] = m.grid_index; model_ints[3 * i + 2] = m.mat.material_type; }
        if (m2w) std::memcpy(m2w + 16 * i, m.model_to_world, 64);
        if (w2m) std::memcpy(w2m + 16 * i, m.world_to_model, 64);
        if (color) std::memcpy(color + 3 * i, m.mat.color, 12);
    }
    for (size_t i = 0; i < S.grids.size(); i++) {
        const pt::Grid& g = S.grids[i];
        if (grid_ints) {
            grid_ints[4 * i] = g.voxelIndices.start_index; grid_ints[4 * i + 1] = g.voxelIndices.end_index;
            grid_ints[4 * i + 2] = g.entity_type; grid_ints[4 * i + 3] = g.entity_index;
        }
        if (grid_vw) std::memcpy(grid_vw + 3 * i, g.voxel_width, 12);
    }
    if (vox)
        for (size_t i = 0; i < S.voxels.size(); i++) {
            vox[3 * i] = S.voxels[i].entity_index_range.start_index;
            vox[3 * i + 1] = S.voxels[i].entity_index_range.end_index;
            vox[3 * i + 2] = S.voxels[i].entity_type;
        }
    if (per_voxel && !S.per_voxel_data_pool.empty())
        std::memcpy(per_voxel, S.per_voxel_data_pool.data(), S.per_voxel_data_pool.size() * sizeof(int));
    return 0;
}

int pt_scene_export_bvh(const pt_scene* s, float* nodes, int* refs, int* roots) {
    if (!s) return set_err("null scene");
    const pt::Scene& S = s->s;
    if (nodes && !S.bvh_nodes.empty()) std::memcpy(nodes, S.bvh_nodes.data(), S.bvh_nodes.size() * sizeof(pt::BvhNode));
    if (refs && !S.bvh_tri_order.empty()) std::memcpy(refs, S.bvh_tri_order.data(), S.bvh_tri_order.size() * sizeof(int));
    if (roots)
        for (size_t i = 0; i < S.meshes.size(); i++) roots[i] = S.mesh_bvh_root.empty() ? -1 : S.mesh_bvh_root[i];
    return 0;
}

int pt_scene_export_bvh4(const pt_scene* s, float* nodes, int* roots) {
    if (!s) return set_err("null scene");
    const pt::Scene& S = s->s;
    if (nodes && !S.bvh4_nodes.empty()) std::memcpy(nodes, S.bvh4_nodes.data(), S.bvh4_nodes.size() * sizeof(pt::Bvh4Node));
    if (roots)
        for (size_t i = 0; i < S.meshes.size(); i++) roots[i] = S.mesh_bvh4_root.empty() ? -1 : S.mesh_bvh4_root[i];
    return (int)S.bvh4_nodes.size();
}

int pt_scene_export_bvh4_leaf_base(const pt_scene* s, int* bases) {
    if (!s) return set_err("null scene");
    const pt::Scene& S = s->s;
    if (bases)
        for (size_t i = 0; i < S.meshes.size(); i++) bases[i] = S.mesh_leaf_base.empty() ? 0 : S.mesh_leaf_base[i];
    return (int)S.meshes.size();
}

pt_renderer* pt_renderer_create(const pt_render_config* c) {
    if (!c) { set_err("null config"); return nullptr; }
    if (c->accel != PT_ACCEL_GRID && c->accel != PT_ACCEL_BVH && c->accel != PT_ACCEL_GRID_FAST) {
        set_err("bad accel");
        return nullptr;
    }
    if (c->block != 64 && c->block != 128 && c->block != 256) { set_err("block must be 64, 128 or 256"); return nullptr; }
    try {
        pt_renderer* r = new pt_renderer();
        r->r = new pt::Renderer(to_cfg(c));
        return r;
    } catch (...) {
        set_err("out of memory");
        return nullptr;
    }
}

#define R_CALL(expr)                                     \
    do {                                                 \
        if (!r || !r->r) return set_err("null renderer"); \
        int _rc = (expr);                                \
        if (_rc < 0) return set_err(r->r->last_error);   \
        return _rc;                                      \
    } while (0)

int pt_renderer_set_stream(pt_renderer* r, void* st) { R_CALL(r->r->setStream((hipStream_t)st)); }
int pt_renderer_bind_image(pt_renderer* r, float* d) { R_CALL(r->r->bindImage(d)); }
int pt_renderer_allocate_on_gpu(pt_renderer* r, const pt_scene* s) {
    if (!s) return set_err("null scene");
    if (!r || !r->r) return set_err("null renderer");
    // grid_fast / bvh traverse the per-mesh BLAS: a scene built grid-only gets it here,
    // once (the scene's grid tables are rebuilt identically alongside); the lock also
    // keeps other renderers from reading the scene while that happens
    pt_scene* ms = const_cast<pt_scene*>(s);
    std::lock_guard<std::mutex> lock(ms->bvh_mu);
    if (r->r->cfg.accel != PT_ACCEL_GRID && ms->s.built && ms->s.bvh_nodes.empty() && ms->s.ensureBvh() < 0)
        return set_err(ms->s.last_error);
    R_CALL(r->r->allocateOnGPU(s->s));
}
int pt_renderer_clear_image(pt_renderer* r) { R_CALL(r->r->clearImage()); }
int pt_renderer_render_loop(pt_renderer* r, int first, int n) { R_CALL(r->r->renderLoop(first, n)); }
int pt_renderer_synchronize(pt_renderer* r) { R_CALL(r->r->synchronize()); }
int pt_renderer_read_image(pt_renderer* r, float* h) {
    if (!h) return set_err("null buffer");
    R_CALL(r->r->readImage(h));
}
int pt_renderer_render_image(pt_renderer* r, const char* path, int iters) {
    if (!path || iters <= 0) return set_err("bad arguments");
    R_CALL(r->r->renderImage(path, iters));
}
long long pt_renderer_segments(pt_renderer* r) {
    if (!r || !r->r) { set_err("null renderer"); return -1; }
    return r->r->segments();
}
long long pt_renderer_trace_faults(pt_renderer* r) {
    if (!r || !r->r) { set_err("null renderer"); return -1; }
    const long long f = r->r->traceFaults();
    if (f < 0) set_err("reading the trace fault counter failed");
    return f;
}
int pt_renderer_segments_per_bounce(pt_renderer* r, long long* out, int n) {
    if (!out || n < 0) return set_err("bad arguments");
    R_CALL(r->r->segmentsPerBounce(out, n));
}
int pt_renderer_pipelines(pt_renderer* r) {
    if (!r || !r->r) return set_err("null renderer");
    return r->r->pipelines();
}
int pt_renderer_set_profiling(pt_renderer* r, int on) { R_CALL(r->r->setProfiling(on)); }
int pt_renderer_kernel_stats(pt_renderer* r, double st[7]) {
    if (!r || !r->r || !st) return set_err("null argument");
    pt::KernelStats k;
    if (r->r->kernelStats(&k) < 0) return set_err(r->r->last_error);
    st[0] = k.bounce_ms; st[1] = k.scan_ms; st[2] = k.primary_ms;
    st[3] = (double)k.bounce_launches; st[4] = (double)k.scan_launches;
    st[5] = k.first_ms; st[6] = (double)k.first_launches;
    return 0;
}
int pt_renderer_kernel_stats_ex(pt_renderer* r, double* st, int n) {
    if (!r || !r->r || !st || n < 0) return set_err("bad arguments");
    pt::KernelStats k;
    if (r->r->kernelStats(&k) < 0) return set_err(r->r->last_error);
    const double v[11] = {k.bounce_ms, k.scan_ms, k.primary_ms, (double)k.bounce_launches, (double)k.scan_launches,
                          k.first_ms, (double)k.first_launches, k.trace_ms, (double)k.trace_launches,
                          k.sort_ms, (double)k.sort_launches};
    for (int i = 0; i < n; i++) st[i] = i < 11 ? v[i] : 0.0;
    return 0;
}
int pt_renderer_primary_hits(pt_renderer* r, float* d, float* n, int* m) {
    if (!d || !n || !m) return set_err("null buffer");
    R_CALL(r->r->primaryHits(d, n, m));
}
int pt_renderer_intersect_rays(pt_renderer* r, int n, const float* o, const float* d, float* t, float* nn, int* m) {
    if (n < 0 || (n > 0 && (!o || !d || !t || !nn || !m))) return set_err("bad arguments");
    R_CALL(r->r->intersectRays(n, o, d, t, nn, m));
}
int pt_renderer_certify_check(pt_renderer* r, int n, const float* o, const float* d, int* out4) {
    if (n < 0 || (n > 0 && (!o || !d || !out4))) return set_err("bad arguments");
    R_CALL(r->r->certifyCheck(n, o, d, out4));
}
void pt_renderer_free(pt_renderer* r) {
    if (!r) return;
    delete r->r;
    delete r;
}

int pt_selftest_math(int n, const float* x, const float* y, float* out) {
    if (n < 0 || (n > 0 && (!x || !y || !out))) return set_err("bad arguments");
    std::string e;
    if (pt::selftest_math(n, x, y, out, &e) < 0) return set_err(e);
    return 0;
}

int pt_render(const char* scene_config, const pt_render_config* cfg, const char* bmp_out) {
    pt_render_config c;
    if (cfg) c = *cfg; else pt_default_config(&c);
    pt_scene* s = pt_scene_create();
    if (!s) return -1;
    int rc = pt_scene_load_config(s, scene_config);
    if (rc >= 0) rc = pt_scene_apply_settings(s, &c);
    if (rc >= 0) rc = pt_scene_build(s, c.grid, c.accel != PT_ACCEL_GRID ? 1 : 0);
    pt_renderer* r = rc >= 0 ? pt_renderer_create(&c) : nullptr;
    if (rc >= 0 && !r) rc = -1;
    if (rc >= 0) rc = pt_renderer_allocate_on_gpu(r, s);
    if (rc >= 0) rc = pt_renderer_render_loop(r, 0, c.iterations);
    if (rc >= 0) rc = pt_renderer_synchronize(r);
    if (rc >= 0 && bmp_out) rc = pt_renderer_render_image(r, bmp_out, c.iterations);
    pt_renderer_free(r);
    pt_scene_destroy(s);
    return rc < 0 ? -1 : 0;
}

}  // extern "C"
