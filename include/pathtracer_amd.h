/*
 * pathtracer_amd.h -- C ABI of the MI355X-native PathTracerAP hot path.
 *
 * Drop-in boundary for the reference's render path
 * (purvakulkarni15/PathTracerAP).  Plain pointers and sizes only; the
 * implementation is libpathtracer_amd.so (C++ host + gfx950 HIP kernels).
 * Each entry point names the reference interface it replaces:
 *
 *   pt_scene_load_config     <- Scene::Scene(string config)          Scene.cpp:3, Scene.h:24
 *   pt_scene_load_obj        <- Scene::loadAndProcessMeshFile        Scene.cpp:226-238
 *   pt_scene_add_mesh        <- Scene::processMesh                   Scene.cpp:264-291
 *   pt_scene_add_model       <- Model setup in Scene::Scene          Scene.cpp:32-42 (x11)
 *   pt_scene_build           <- Scene::addMeshesToGrid               Scene.cpp:318-396 (+ the per-mesh BLAS)
 *   pt_renderer_allocate_on_gpu <- Renderer::allocateOnGPU           Renderer.cpp:65-130, Renderer.h:49
 *   pt_renderer_clear_image  <- initImageKernel                      Renderer.cpp:557-565
 *   pt_renderer_render_loop  <- Renderer::renderLoop                 Renderer.cpp:567-648, Renderer.h:50
 *   pt_renderer_render_image <- Renderer::renderImage                Renderer.cpp:15-63, Renderer.h:51
 *   pt_renderer_free         <- Renderer::free                       Renderer.cpp:132-148, Renderer.h:52
 *   pt_render                <- main()                               main.cpp:11-27
 *
 * Compile-time constants of Config.h (RESOLUTION_X/Y, ITER, GRID_X/Y/Z) and
 * the hard-coded camera/bounce count of generateRaysKernel
 * (Renderer.cpp:521-555) are fields of pt_render_config.
 *
 * Error behaviour: functions returning int return 0 on success and a
 * negative value on failure; pointer-returning functions return NULL.  The
 * message is available from pt_last_error() (per thread).  There is no CPU
 * fallback: without a usable gfx950 device, pt_renderer_allocate_on_gpu
 * fails.
 */
#ifndef PATHTRACER_AMD_H
#define PATHTRACER_AMD_H

#ifdef __cplusplus
extern "C" {
#endif

#define PT_ABI_VERSION 8

/* Primitive.h:70-79 Material::MaterialType */
enum {
    PT_MAT_DIFFUSE = 0, PT_MAT_SPECULAR = 1, PT_MAT_REFLECTIVE = 2, PT_MAT_REFRACTIVE = 3,
    PT_MAT_EMISSIVE = 4, PT_MAT_COAT = 5, PT_MAT_METAL = 6
};

/* Intersect-stage acceleration structure. */
enum {
    PT_ACCEL_GRID = 0,      /* reference uniform grid + DDA (Renderer.cpp:238-360), bit-exact */
    PT_ACCEL_BVH = 1,       /* MI355X BVH, exact closest hit with the reference triangle test */
    PT_ACCEL_GRID_FAST = 2  /* PT_ACCEL_GRID's result via BVH hit set + voxel-box DDA walk (needs BVH) */
};

typedef struct pt_scene pt_scene;
typedef struct pt_renderer pt_renderer;

typedef struct pt_render_config {
    int width, height;        /* RESOLUTION_X/Y (Config.h:12-13), default 1000 x 800 */
    int iterations;           /* ITER (Config.h:19), default 500: used by render_image / pt_render */
    int max_bounces;          /* remaining_bounces (Renderer.cpp:550), default 5 */
    int accel;                /* PT_ACCEL_*, default PT_ACCEL_GRID_FAST (the reference grid's results, bit for bit) */
    int grid[3];              /* GRID_X/Y/Z (Config.h:8-10), default 25^3 */
    int tail_drop;            /* 1: replicate the reference's ceil(n/32) launch truncation */
    double cam[3];            /* camera origin (Renderer.cpp:528), default (0,0,920) */
    double plane_z;           /* image plane z (Renderer.cpp:543), default 900 */
    double plane_x0, plane_y0, plane_w, plane_h;  /* Renderer.cpp:538-542: -10,-4,20,16 */
    int block;                /* bounce-kernel workgroup = compaction chunk: 64 (default), 128 or 256 */
    int pipelines;            /* iterations in flight on their own HIP streams, 1..32 (default 16); results
                                 are identical for every value (contributions merge in iteration order).
                                 Loading the library sets GPU_MAX_HW_QUEUES=16 (one hardware queue per
                                 pipeline stream) unless the process already set it */
    int ray_sort;             /* ray sort before each persistent trace: -1 auto (key 7 for grid_fast and bvh),
                                 0 off, 1..8 key layout; claim order only, results identical */
} pt_render_config;

int pt_abi_version(void);
const char *pt_last_error(void);
/* GPU_MAX_HW_QUEUES as the library found it when it was loaded (*at_load = -1: unset)
 * and whether the library then set it to 16 (*set_by_library = 1).  HIP reads the
 * variable once, when its runtime starts: a process whose HIP runtime started before
 * the library loaded runs with its own value (HIP's default is 4). */
int pt_hw_queue_info(int *at_load, int *set_by_library);
void pt_default_config(pt_render_config *cfg);

/* ---- Scene ---- */
pt_scene *pt_scene_create(void);
void pt_scene_destroy(pt_scene *s);
int pt_scene_load_config(pt_scene *s, const char *path);
/* Copies the config file's optional RENDER block over *cfg (only fields it sets). */
int pt_scene_apply_settings(const pt_scene *s, pt_render_config *cfg);
int pt_scene_load_obj(pt_scene *s, const char *path);                 /* -> mesh index */
int pt_scene_add_mesh(pt_scene *s, const float *pos, const float *nrm, int nv,
                      const int *tris, int nt);                        /* -> mesh index */
int pt_scene_add_model(pt_scene *s, int mesh, const float scale[3], const float rot_deg[3],
                       const float translate[3], int material, const float color[3]); /* -> model index */
/* with_bvh: also build the per-mesh BLAS (needed by PT_ACCEL_GRID_FAST and PT_ACCEL_BVH;
 * pt_renderer_allocate_on_gpu adds it on demand to a scene built without it). */
int pt_scene_build(pt_scene *s, const int grid[3], int with_bvh);
/* counts[9] = nv nt nmesh nmodel ngrid nvox npv nbvh_nodes nbvh_refs */
int pt_scene_counts(const pt_scene *s, int counts[9]);
/* Flat export of Scene.h's vectors (any pointer may be NULL):
 * vpos/vnrm nv*3, tris nt*3, mesh_ranges nmesh*4 (vs ve ts te), mesh_bbox nmesh*6,
 * model_ints nmodel*3 (mesh grid material), m2w/w2m nmodel*16 column-major,
 * color nmodel*3, grid_ints ngrid*4 (vox_start vox_end entity_type entity_index),
 * grid_vw ngrid*3, vox nvox*3 (start end entity_type), per_voxel npv. */
int pt_scene_export(const pt_scene *s, float *vpos, float *vnrm, int *tris, int *mesh_ranges,
                    float *mesh_bbox, int *model_ints, float *m2w, float *w2m, float *color,
                    int *grid_ints, float *grid_vw, int *vox, int *per_voxel);

/* BVH export (ACCEL_BVH builds): nodes nbvh_nodes*16 (the 64-byte BvhNode as
 * 16 floats; int fields bit-cast), refs nbvh_refs, roots nmesh. */
int pt_scene_export_bvh(const pt_scene *s, float *nodes, int *refs, int *roots);
/* The same BLAS collapsed 4-wide (k_trace_gf's node steps): Bvh4Node records,
 * 32 words each (lo x/y/z[4], hi x/y/z[4], link[4], count[4]), and each mesh's
 * 4-wide root (-1: none).  Returns the node count (call with nodes = NULL to
 * size the buffer), < 0 on error. */
int pt_scene_export_bvh4(const pt_scene *s, float *nodes, int *roots);
/* Each mesh's first leaf record (bvh_tri_order entry), nmesh ints: a 4-wide
 * leaf link (1 << 31 | count << 26 | first) holds first relative to it, so
 * the 2^26 limit of the encoding is per mesh (ABI 8).  Returns nmesh. */
int pt_scene_export_bvh4_leaf_base(const pt_scene *s, int *bases);

/* ---- Renderer ---- */
pt_renderer *pt_renderer_create(const pt_render_config *cfg);
/* Use an existing hipStream_t (e.g. torch.cuda.current_stream().cuda_stream). */
int pt_renderer_set_stream(pt_renderer *r, void *hip_stream);
/* Accumulate into caller-owned device memory (W*H*3 floats) instead of an internal buffer. */
int pt_renderer_bind_image(pt_renderer *r, float *device_rgb);
/* For PT_ACCEL_GRID_FAST / PT_ACCEL_BVH a scene built without the BLAS gets it here (once). */
int pt_renderer_allocate_on_gpu(pt_renderer *r, const pt_scene *s);
/* Zeroes the accumulator and the trace-fault counter (a new render starts). */
int pt_renderer_clear_image(pt_renderer *r);
/* Enqueue iterations [first_iter, first_iter + n_iters) (asynchronous). */
int pt_renderer_render_loop(pt_renderer *r, int first_iter, int n_iters);
int pt_renderer_synchronize(pt_renderer *r);
int pt_renderer_read_image(pt_renderer *r, float *host_rgb);
int pt_renderer_render_image(pt_renderer *r, const char *bmp_path, int iterations_total);
/* Ray segments shaded so far (sum over bounces of live rays). */
long long pt_renderer_segments(pt_renderer *r);
/* Persistent-trace waves that hit their iteration cap and left rays untraced since
 * allocate_on_gpu or the last clear_image (0 in a correct run; -1 on error).  Non-zero
 * makes pt_renderer_synchronize / read_image / render_image fail: the image is invalid. */
long long pt_renderer_trace_faults(pt_renderer *r);
/* out[b] = live rays entering bounce b, summed over the iterations rendered (b < n, n <= 64 useful). */
int pt_renderer_segments_per_bounce(pt_renderer *r, long long *out, int n);
/* HIP-event timing read by kernel_stats: 0 off, 1 around every kernel group on every
 * pipeline, 2 around pipeline 0's trace phases only (light enough for a timed run). */
int pt_renderer_set_profiling(pt_renderer *r, int on);
/* Iterations in flight after allocate_on_gpu (config.pipelines clamped to 1..32, PT_PIPES overrides). */
int pt_renderer_pipelines(pt_renderer *r);
/* stats[0..6] = secondary-bounce ms, scan ms, primary ms, secondary-bounce launches,
 * scan launches, first-bounce ms, first-bounce launches (HIP events; resets). */
int pt_renderer_kernel_stats(pt_renderer *r, double stats[7]);
/* Same, n values: stats[7..8] = persistent-trace ms, launches (grid_fast / bvh split each
 * secondary bounce into a persistent trace + a shading pass; stats[0] is then the shading
 * pass); stats[9..10] = ray-sort ms, sort passes (k_sort_hist + prefix + scatter). */
int pt_renderer_kernel_stats_ex(pt_renderer *r, double *stats, int n);
/* Test hooks: primary-hit cache and batch intersection (host arrays). */
int pt_renderer_primary_hits(pt_renderer *r, float *dist, float *normal, int *model);
int pt_renderer_intersect_rays(pt_renderer *r, int n, const float *orig, const float *dir,
                               float *dist, float *normal, int *model);
/* Test hook (grid_fast): k_trace_gf's walk certificates (walk_certify_fast,
 * walk_certify) against the exact stepped walk on the same hit sets of each ray;
 * out4[4i..4i+3] = fast certificates tried, accepted, accepted-but-wrong,
 * full certificates accepted-but-wrong (no counterpart in the reference: it
 * checks the exactness of Renderer.cpp:238-360's replacement). */
int pt_renderer_certify_check(pt_renderer *r, int n, const float *orig, const float *dir, int *out4);
void pt_renderer_free(pt_renderer *r);

/* Device math conformance hook: evaluates the kernels' sinf/cosf/powf/sqrtf/div
 * replacements on n inputs (x, y) -> out[n*5] = sin(x) cos(x) pow(x,y) sqrt(x) x/y. */
int pt_selftest_math(int n, const float *x, const float *y, float *out);

/* main.cpp: load scene config, render cfg->iterations, write BMP. */
int pt_render(const char *scene_config, const pt_render_config *cfg, const char *bmp_out);

#ifdef __cplusplus
}
#endif
#endif
