/*
 * ptoracle.h -- CPU ORACLE for the PathTracerAP bounce loop.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in pathtracerap_amd/ may include, link
 * or call this; only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg use it, and only as the checker.
 *
 * This is a plain-C restatement of the reference's algorithm
 * (purvakulkarni15/PathTracerAP, CUDA + glm 0.9.6 + thrust), written from
 * a reading of its sources.  Every function cites the reference file:line
 * it follows.  The reference itself is unbuildable in this image (needs the
 * CUDA toolkit, thrust and Assimp), so the oracle is pinned against the
 * reference's own golden output (PathTracerAP/Render.bmp, 1000x800, 500
 * iterations, the Scene.cpp scene) -- see tests/test_oracle_golden.py.
 *
 * Data layout deliberately mirrors the reference (Primitive.h structs,
 * array-of-structs ray pool, stable partition of the ray pool after every
 * bounce) so that it stays an independent check of the wavefront/SoA
 * HIP implementation.
 */
#ifndef PTORACLE_H
#define PTORACLE_H

#ifdef __cplusplus
extern "C" {
#endif

/* Flat scene description (Scene.h:21-40 member vectors, flattened). */
typedef struct {
    int nv;            const float *vpos;  const float *vnrm;   /* nv*3 each            */
    int nt;            const int   *tris;                      /* nt*3 vertex indices  */
    int nmesh;         const int   *mesh_ranges;               /* nmesh*4: vs ve ts te */
                       const float *mesh_bbox;                 /* nmesh*6: min3 max3   */
    int nmodel;        const int   *model_ints;                /* nmodel*3: mesh grid mattype */
                       const float *model_m2w;                 /* nmodel*16 column-major */
                       const float *model_w2m;                 /* nmodel*16 column-major */
                       const float *model_color;               /* nmodel*3 */
    int ngrid;         const int   *grid_ints;                 /* ngrid*4: vox_s vox_e etype eidx */
                       const float *grid_vw;                   /* ngrid*3 voxel widths */
    int nvox;          const int   *vox;                       /* nvox*3: start end etype */
    int npv;           const int   *per_voxel;                 /* npv triangle indices */
    int gdim[3];                                               /* GRID_X/Y/Z (Config.h:8-10) */
} ptor_scene;

typedef struct {
    int width, height;        /* RESOLUTION_X/Y (Config.h:12-13)             */
    int first_iter;           /* iteration index of the first rendered pass  */
    int iterations;           /* number of passes (ITER, Config.h:19)        */
    int max_bounces;          /* remaining_bounces init (Renderer.cpp:550)   */
    int accel;                /* 0 = reference uniform grid, 1 = exact closest hit */
    int threads;              /* OpenMP threads (<=0: default)               */
    int tail_drop;            /* 1: replicate ceil(n/32) launch truncation   */
    double cam[3];            /* camera origin (Renderer.cpp:528)            */
    double plane_z;           /* image plane z (Renderer.cpp:543)            */
    double plane_x0, plane_y0, plane_w, plane_h; /* Renderer.cpp:538-542      */
} ptor_config;

/* Renders `iterations` passes and ADDS them into image[w*h*3] (the
 * dev_image_data accumulator, Renderer.cpp:495).  Returns the number of ray
 * segments shaded (sum over bounces of live rays) in *segments. */
int ptor_render(const ptor_scene *s, const ptor_config *c, float *image,
                long long *segments);

/* Primary-ray intersection only (computeRaySceneIntersectionKernel on the
 * camera rays, Renderer.cpp:364-409): per pixel dist, normal[3], model id
 * (-1 = miss).  Used by the unit parity tests. */
int ptor_intersect_primary(const ptor_scene *s, const ptor_config *c,
                           float *dist, float *normal, int *model);

/* Generic ray batch intersection (world-space rays, unnormalised dirs). */
int ptor_intersect_rays(const ptor_scene *s, int accel, int n,
                        const float *orig, const float *dir,
                        float *dist, float *normal, int *model, int threads);

/* Shade a single bounce for a batch of rays given their hits (shadeRayKernel,
 * Renderer.cpp:412-479).  state arrays are updated in place. */
int ptor_shade(int n, int iter, const int *slot, float *orig, float *dir,
               float *color, int *bounces, const float *hit_dist,
               const float *hit_normal, const int *hit_type,
               const float *hit_color);

/* ---- scene construction (Scene.cpp) ---- */

/* glm 0.9.6 restatements used by Scene.cpp:30-221 (column-major mat4). */
void ptor_model_matrix(const float scale[3], const float rot_deg[3],
                       const float translate[3], float m2w[16], float w2m[16]);

/* addMeshesToGrid (Scene.cpp:318-396).  Outputs are caller-allocated:
 * grid_ints[ngrid_max*4], grid_vw[ngrid_max*3], vox[ngrid_max*G*3],
 * per_voxel capacity pv_cap (returns -needed if too small).  model_ints'
 * grid column is written. */
int ptor_build_grids(int nmesh, const int *mesh_ranges, const float *mesh_bbox,
                     const float *vpos, const int *tris,
                     int nmodel, int *model_ints, const int gdim[3],
                     int *ngrid, int *grid_ints, float *grid_vw,
                     int *nvox, int *vox, int pv_cap, int *npv, int *per_voxel);

/* Self-contained math used by the oracle (exposed for the conformance test). */
float ptor_sinf(float x);
float ptor_cosf(float x);
float ptor_powf(float x, float y);
unsigned ptor_hash(unsigned a);
float ptor_u01_first(int iter, int index, int depth);

#ifdef __cplusplus
}
#endif
#endif
