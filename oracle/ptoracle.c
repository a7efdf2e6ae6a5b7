/*
 * ptoracle.c -- CPU ORACLE (test infrastructure, see ptoracle.h).
 *
 * Plain-C restatement of purvakulkarni15/PathTracerAP's render path:
 *   Renderer.cpp  : generateRaysKernel, computeRaySceneIntersectionKernel,
 *                   computeRayGridIntersection (DDA), computeRayVoxelIntersection,
 *                   computeRayTriangleIntersection, computeRayBoundingBoxIntersection,
 *                   shadeRayKernel, compactStencilKernel + thrust::stable_partition,
 *                   gatherImageDataKernel, renderLoop
 *   utility.h     : utilHash, makeSeededRandomEngine, reflectRay, transform*,
 *                   calculateRandomDirectionInHemisphere / Metal / Coat
 *   Scene.cpp     : computeVoxelIndex, addMeshesToGrid, model matrices
 *   glm 0.9.6     : dot/cross/normalize/length, mat4*vec4, inverse (generic paths)
 *   thrust        : minstd_rand (linear_congruential_engine<uint32,48271,0,2^31-1>)
 *                   and uniform_real_distribution<float>
 *
 * Floating-point policy: every expression keeps the reference's operand order
 * with no contraction (build with -ffp-contract=off).  sinf/cosf/powf are
 * replaced by the self-contained double-precision evaluations below (the
 * GPU implementation evaluates the identical sequence), so GPU vs oracle is
 * bit-exact; vs the CUDA reference they differ by <= 1 ulp per call.
 */
#include "ptoracle.h"

#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* Config.h:4-6 */
#define OR_EPS 0.005f
#define OR_FMAX 9999999.0f
#define OR_FMIN -9999990.0f
/* utility.h:20-22 */
#define OR_TWO_PI 6.2831853071795864769252867665590057683943f
#define OR_SQRT13 0.5773502691896257645091487805019574556476f

/* Primitive.h:70-79 MaterialType */
enum { M_DIFFUSE = 0, M_SPECULAR, M_REFLECTIVE, M_REFRACTIVE, M_EMISSIVE, M_COAT, M_METAL };

typedef struct { float x, y, z; } v3;

static inline v3 mk(float x, float y, float z) { v3 r; r.x = x; r.y = y; r.z = z; return r; }
static inline v3 vadd(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 vsub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 vmul(v3 a, v3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 vs(v3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
/* glm compute_dot<tvec3>: tmp = x*y; tmp.x + tmp.y + tmp.z (func_geometric.inl:67-71) */
static inline float vdot(v3 a, v3 b) { v3 t = vmul(a, b); return t.x + t.y + t.z; }
/* glm cross (func_geometric.inl:134-142) */
static inline v3 vcross(v3 x, v3 y) {
    return mk(x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y);
}
/* glm normalize = x * inversesqrt(dot(x,x)), inversesqrt = 1/sqrt (func_exponential.inl:150) */
static inline v3 vnorm(v3 a) { float s = 1.0f / sqrtf(vdot(a, a)); return vs(a, s); }
static inline float vlen(v3 a) { return sqrtf(vdot(a, a)); }
/* utility.h:14 ABS */
static inline float fabs_ref(float x) { return x < 0 ? -x : x; }
static inline int iabs(int x) { return x < 0 ? -x : x; }

/* float -> int as the GPU converts (cvt.rzi.s32.f32 / v_cvt_i32_f32):
 * NaN -> 0, saturate at the int range. */
static inline int f2i_sat(float f) {
    if (f != f) return 0;
    if (f >= 2147483648.0f) return 2147483647;
    if (f <= -2147483648.0f) return (-2147483647 - 1);
    return (int)f;
}
/* float -> int as the x86 host converts (cvttss2si): NaN / out of range -> INT_MIN. */
static inline int f2i_x86(float f) {
    if (f != f || f >= 2147483648.0f || f < -2147483648.0f) return (-2147483647 - 1);
    return (int)f;
}

/* glm mat4 * vec4 (type_mat4x4.inl:591-628): (m0*x + m1*y) + (m2*z + m3*w), column-major. */
static inline v3 xform(const float *m, v3 p, float w) {
    float r[3];
    for (int k = 0; k < 3; k++) {
        float a0 = m[0 * 4 + k] * p.x;
        float a1 = m[1 * 4 + k] * p.y;
        float a2 = m[2 * 4 + k] * p.z;
        float a3 = m[3 * 4 + k] * w;
        r[k] = (a0 + a1) + (a2 + a3);
    }
    return mk(r[0], r[1], r[2]);
}

/* ---------------------------------------------------------------------- */
/* Self-contained transcendental functions (double-precision polynomials)  */
/* ---------------------------------------------------------------------- */

static inline double or_floor(double q) {
    double t = (double)(long long)q;
    return (t > q) ? t - 1.0 : t;
}

static void or_sincos(float xf, float *so, float *co) {
    double x = (double)xf;
    if (!(x - x == 0.0)) { *so = NAN; *co = NAN; return; }
    double k = or_floor(x * 0.63661977236758134308 + 0.5);
    const double pio2_1 = 1.57079632673412561417e+00;
    const double pio2_1t = 6.07710050650619224932e-11;
    double r = (x - k * pio2_1) - k * pio2_1t;
    double r2 = r * r;
    /* sin(r) Taylor to r^17 (|r| <= pi/4: truncation < 1e-19) */
    double sp = 1.0 / 355687428096000.0;                /* +1/17! */
    sp = sp * r2 + (-1.0 / 1307674368000.0);            /* -1/15! */
    sp = sp * r2 + (1.0 / 6227020800.0);                /* +1/13! */
    sp = sp * r2 + (-1.0 / 39916800.0);                 /* -1/11! */
    sp = sp * r2 + (1.0 / 362880.0);                    /* +1/9!  */
    sp = sp * r2 + (-1.0 / 5040.0);                     /* -1/7!  */
    sp = sp * r2 + (1.0 / 120.0);                       /* +1/5!  */
    sp = sp * r2 + (-1.0 / 6.0);                        /* -1/3!  */
    double s = r + (r * r2) * sp;
    double cp = 1.0 / 6402373705728000.0;               /* +1/18! */
    cp = cp * r2 + (-1.0 / 20922789888000.0);           /* -1/16! */
    cp = cp * r2 + (1.0 / 87178291200.0);               /* +1/14! */
    cp = cp * r2 + (-1.0 / 479001600.0);                /* -1/12! */
    cp = cp * r2 + (1.0 / 3628800.0);                   /* +1/10! */
    cp = cp * r2 + (-1.0 / 40320.0);                    /* -1/8!  */
    cp = cp * r2 + (1.0 / 720.0);                       /* +1/6!  */
    cp = cp * r2 + (-1.0 / 24.0);                       /* -1/4!  */
    cp = cp * r2 + 0.5;                                 /* cp = 1/2 - r2/4! + r2^2/6! - ... */
    double c = 1.0 - r2 * cp;                           /* cos(r) Taylor to r^18 */
    long long n = (long long)k;
    int q = (int)(n & 3);
    double sv, cv;
    switch (q) {
        case 0: sv = s; cv = c; break;
        case 1: sv = c; cv = -s; break;
        case 2: sv = -s; cv = -c; break;
        default: sv = -c; cv = s; break;
    }
    *so = (float)sv;
    *co = (float)cv;
}

float ptor_sinf(float x) { float s, c; or_sincos(x, &s, &c); return s; }
float ptor_cosf(float x) { float s, c; or_sincos(x, &s, &c); return c; }

static double or_log(double x) {
    uint64_t b; memcpy(&b, &x, 8);
    int e = (int)((b >> 52) & 0x7ff) - 1023;
    b = (b & 0x000fffffffffffffULL) | 0x3ff0000000000000ULL;
    double m; memcpy(&m, &b, 8);
    if (m > 1.41421356237309504880) { m = m * 0.5; e = e + 1; }
    double s = (m - 1.0) / (m + 1.0);
    double s2 = s * s;
    double p = 1.0 / 23.0;
    p = p * s2 + 1.0 / 21.0;
    p = p * s2 + 1.0 / 19.0;
    p = p * s2 + 1.0 / 17.0;
    p = p * s2 + 1.0 / 15.0;
    p = p * s2 + 1.0 / 13.0;
    p = p * s2 + 1.0 / 11.0;
    p = p * s2 + 1.0 / 9.0;
    p = p * s2 + 1.0 / 7.0;
    p = p * s2 + 1.0 / 5.0;
    p = p * s2 + 1.0 / 3.0;
    double lm = 2.0 * (s + (s * s2) * p);
    const double ln2_hi = 6.93147180369123816490e-01;
    const double ln2_lo = 1.90821492927058770002e-10;
    double ed = (double)e;
    return ed * ln2_hi + (lm + ed * ln2_lo);
}

static double or_exp(double z) {
    if (z < -745.0) return 0.0;
    if (z > 709.0) return INFINITY;
    double k = or_floor(z * 1.44269504088896338700 + 0.5);
    const double ln2_hi = 6.93147180369123816490e-01;
    const double ln2_lo = 1.90821492927058770002e-10;
    double r = (z - k * ln2_hi) - k * ln2_lo;
    double p = 1.0 / 87178291200.0;                     /* 1/14! */
    p = p * r + 1.0 / 6227020800.0;
    p = p * r + 1.0 / 479001600.0;
    p = p * r + 1.0 / 39916800.0;
    p = p * r + 1.0 / 3628800.0;
    p = p * r + 1.0 / 362880.0;
    p = p * r + 1.0 / 40320.0;
    p = p * r + 1.0 / 5040.0;
    p = p * r + 1.0 / 720.0;
    p = p * r + 1.0 / 120.0;
    p = p * r + 1.0 / 24.0;
    p = p * r + 1.0 / 6.0;
    p = p * r + 0.5;
    p = p * r + 1.0;
    p = p * r + 1.0;
    int ki = (int)k;
    /* scale by 2^ki in two exact steps to stay in the normal range */
    int k1 = ki / 2, k2 = ki - k1;
    uint64_t b1 = (uint64_t)(k1 + 1023) << 52, b2 = (uint64_t)(k2 + 1023) << 52;
    double s1, s2; memcpy(&s1, &b1, 8); memcpy(&s2, &b2, 8);
    return (p * s1) * s2;
}

float ptor_powf(float xf, float yf) {
    if (xf != xf || yf != yf) return NAN;
    if (yf == 0.0f) return 1.0f;
    if (xf == 1.0f) return 1.0f;
    if (xf == 0.0f) return yf > 0.0f ? 0.0f : INFINITY;
    if (xf < 0.0f) return NAN;
    double l = or_log((double)xf);
    return (float)or_exp((double)yf * l);
}

/* ---------------------------------------------------------------------- */
/* RNG: utility.h:43-62 + thrust minstd_rand + uniform_real_distribution   */
/* ---------------------------------------------------------------------- */

unsigned ptor_hash(unsigned a) {
    a = (a + 0x7ed55d16u) + (a << 12);
    a = (a ^ 0xc761c23cu) ^ (a >> 19);
    a = (a + 0x165667b1u) + (a << 5);
    a = (a + 0xd3a2646cu) ^ (a << 9);
    a = (a + 0xfd7046c5u) + (a << 3);
    a = (a ^ 0xb55a4f09u) ^ (a >> 16);
    return a;
}

typedef struct { uint32_t x; } or_rng;

/* makeSeededRandomEngine (utility.h:57-62): h = hash((1<<31)|(depth<<22)|iter) ^ hash(index);
 * linear_congruential_engine::seed: x = s mod m, 0 -> 1. */
static inline or_rng rng_make(int iter, int index, int depth) {
    unsigned h = ptor_hash(0x80000000u | ((unsigned)depth << 22) | (unsigned)iter) ^ ptor_hash((unsigned)index);
    or_rng r;
    r.x = h % 2147483647u;
    if (r.x == 0) r.x = 1;
    return r;
}
/* minstd_rand step + uniform_real_distribution<float>(0,1):
 * (float)(x - min) / (1 + (float)(max - min)) * (b - a) + a */
static inline float rng_u01(or_rng *r) {
    r->x = (uint32_t)(((uint64_t)r->x * 48271u) % 2147483647u);
    float res = (float)(uint32_t)(r->x - 1u);
    res = res / (1.0f + (float)(2147483646u - 1u));
    return res * (1.0f - 0.0f) + 0.0f;
}

float ptor_u01_first(int iter, int index, int depth) {
    or_rng r = rng_make(iter, index, depth);
    return rng_u01(&r);
}

/* ---------------------------------------------------------------------- */
/* Scattering (utility.h:64-170)                                            */
/* ---------------------------------------------------------------------- */

/* reflectRay (utility.h:64-69): n - (2*dot(i,n))*n  (sic: reference formula) */
static inline v3 reflect_ref(v3 i, v3 n) { return vsub(n, vs(n, 2.0f * vdot(i, n))); }

/* calculateRandomDirectionInHemisphere (utility.h:91-123) */
static v3 hemisphere(v3 n, or_rng *rng) {
    float up = sqrtf(rng_u01(rng));
    float over = sqrtf(1.0f - up * up);
    float around = rng_u01(rng) * OR_TWO_PI;
    v3 dnn;
    if (fabs_ref(n.x) < OR_SQRT13) dnn = mk(1, 0, 0);
    else if (fabs_ref(n.y) < OR_SQRT13) dnn = mk(0, 1, 0);
    else dnn = mk(0, 0, 1);
    v3 p1 = vnorm(vcross(n, dnn));
    v3 p2 = vnorm(vcross(n, p1));
    float sa, ca; or_sincos(around, &sa, &ca);
    return vadd(vadd(vs(n, up), vs(p1, ca * over)), vs(p2, sa * over));
}

/* calculateCoatScattering (utility.h:125-143) */
static v3 coat(v3 n, v3 d, or_rng *rng) {
    float roulette = rng_u01(rng);
    if (roulette < 0.5f) return reflect_ref(d, n);
    return hemisphere(n, rng);
}

/* calculateMetalScattering (utility.h:145-170) */
static v3 metal(v3 n, v3 d, or_rng *rng) {
    float up = sqrtf(rng_u01(rng));
    float over = sqrtf(1.0f - up * up);
    float around = rng_u01(rng) * OR_TWO_PI;
    (void)over; (void)around;
    float phi = OR_TWO_PI * rng_u01(rng);
    float r2 = rng_u01(rng);
    float phong = 30.0f;
    float cos_t = ptor_powf(1.0f - r2, 1.0f / (phong + 1.0f));
    float sin_t = sqrtf(1.0f - cos_t * cos_t);
    v3 w = vnorm(vsub(d, vs(vs(n, 2.0f), vdot(n, d))));
    v3 a = ((double)fabs_ref(w.x) > .1) ? mk(0, 1, 0) : mk(1, 0, 0);
    v3 u = vnorm(vcross(a, w));
    v3 v = vcross(w, u);
    float sp, cp; or_sincos(phi, &sp, &cp);
    return vadd(vadd(vs(vs(u, cp), sin_t), vs(vs(v, sp), sin_t)), vs(w, cos_t));
}

/* ---------------------------------------------------------------------- */
/* Intersection (Renderer.cpp:150-409)                                      */
/* ---------------------------------------------------------------------- */

typedef struct {
    v3 orig, dir, inv;                   /* Ray::transformed + Ray::cache */
} or_tray;

typedef struct {
    float dist;
    v3 normal;
} or_hit;

/* computeRayBoundingBoxIntersection (Renderer.cpp:150-170) */
static int slab(const or_tray *r, const float *bb, float *t) {
    float t1 = r->dir.x == 0.0f ? OR_FMIN : (bb[0] - r->orig.x) * r->inv.x;
    float t2 = r->dir.x == 0.0f ? OR_FMAX : (bb[3] - r->orig.x) * r->inv.x;
    float t3 = r->dir.y == 0.0f ? OR_FMIN : (bb[1] - r->orig.y) * r->inv.y;
    float t4 = r->dir.y == 0.0f ? OR_FMAX : (bb[4] - r->orig.y) * r->inv.y;
    float t5 = r->dir.z == 0.0f ? OR_FMIN : (bb[2] - r->orig.z) * r->inv.z;
    float t6 = r->dir.z == 0.0f ? OR_FMAX : (bb[5] - r->orig.z) * r->inv.z;
    float tmin = fmaxf(fmaxf(fminf(t1, t2), fminf(t3, t4)), fminf(t5, t6));
    float tmax = fminf(fminf(fmaxf(t1, t2), fmaxf(t3, t4)), fmaxf(t5, t6));
    if (tmax < 0 || tmin > tmax) return 0;
    *t = tmin;
    return 1;
}

static inline v3 vpos(const ptor_scene *s, int i) { return mk(s->vpos[3 * i], s->vpos[3 * i + 1], s->vpos[3 * i + 2]); }
static inline v3 vnrm(const ptor_scene *s, int i) { return mk(s->vnrm[3 * i], s->vnrm[3 * i + 1], s->vnrm[3 * i + 2]); }

/* computeRayTriangleIntersection (Renderer.cpp:174-215).  *tri_out records
 * the triangle that produced the stored hit (tie: first tested wins). */
static int tri_test(const ptor_scene *s, const or_tray *r, or_hit *h, int it) {
    const int *tv = s->tris + 3 * it;
    v3 p0 = vpos(s, tv[0]), p1 = vpos(s, tv[1]), p2 = vpos(s, tv[2]);
    v3 e1 = vsub(p1, p0);
    v3 e2 = vsub(p2, p0);
    v3 pvec = vcross(r->dir, e2);
    float det = vdot(e1, pvec);
    if (fabs_ref(det - 0.0f) < OR_EPS) return 0;                 /* IS_EQUAL */
    float inv_det = 1 / det;
    v3 tvec = vsub(r->orig, p0);
    float u = vdot(tvec, pvec) * inv_det;
    if (u < 0.0f - OR_EPS || u > 1.0f + OR_EPS) return 0;        /* IS_LESS_THAN / IS_MORE_THAN */
    v3 qvec = vcross(tvec, e1);
    float v = vdot(r->dir, qvec) * inv_det;
    if (v < 0.0f - OR_EPS || u + v > 1.0f + OR_EPS) return 0;
    float t = vdot(e2, qvec) * inv_det;
    if (t < 0.0f - OR_EPS) return 0;
    v3 nsum = vadd(vadd(vnrm(s, tv[0]), vnrm(s, tv[1])), vnrm(s, tv[2]));
    v3 n = vnorm(vs(nsum, 1 / 3.0f));
    if (h->dist > t) { h->dist = t; h->normal = n; }
    return 1;
}

/* computeRayVoxelIntersection (Renderer.cpp:217-236) */
static int voxel_test(const ptor_scene *s, const or_tray *r, or_hit *h, int iv) {
    const int *vx = s->vox + 3 * iv;
    int any = 0;
    if (vx[2] == 2 /* EntityType::TRIANGLE */) {
        for (int i = vx[0]; i < vx[1]; i++)
            if (tri_test(s, r, h, s->per_voxel[i])) any = 1;
    }
    return any;
}

/* computeRayGridIntersection (Renderer.cpp:238-360) */
static int grid_test(const ptor_scene *s, const or_tray *r, or_hit *h, int igrid) {
    const int *g = s->grid_ints + 4 * igrid;
    const float *vw = s->grid_vw + 3 * igrid;
    const int GX = s->gdim[0], GY = s->gdim[1], GZ = s->gdim[2];
    /* grid->entity_type == MODEL: bbox of models[entity_index].mesh */
    int model = g[3];
    int mesh = s->model_ints[3 * model + 0];
    const float *bb = s->mesh_bbox + 6 * mesh;
    float t_box;
    if (!slab(r, bb, &t_box)) return 0;
    v3 p = vadd(r->orig, vs(r->dir, t_box));
    if ((p.x - bb[0]) < -OR_EPS || (p.y - bb[1]) < -OR_EPS || (p.z - bb[2]) < -OR_EPS) return 0;
    int ix = f2i_sat(fabs_ref(p.x - bb[0] + OR_EPS) / vw[0]);
    int iy = f2i_sat(fabs_ref(p.y - bb[1] + OR_EPS) / vw[1]);
    int iz = f2i_sat(fabs_ref(p.z - bb[2] + OR_EPS) / vw[2]);
    ix = ix < 0 ? 0 : (ix > GX - 1 ? GX - 1 : ix);
    iy = iy < 0 ? 0 : (iy > GY - 1 ? GY - 1 : iy);
    iz = iz < 0 ? 0 : (iz > GZ - 1 ? GZ - 1 : iz);
    v3 tmax = mk(OR_FMAX, OR_FMAX, OR_FMAX);
    v3 delta = mk(OR_FMAX, OR_FMAX, OR_FMAX);
    int sx = r->dir.x > 0.0f ? 1 : -1, sy = r->dir.y > 0.0f ? 1 : -1, sz = r->dir.z > 0.0f ? 1 : -1;
    int ox = r->dir.x > 0.0f ? GX : -1, oy = r->dir.y > 0.0f ? GY : -1, oz = r->dir.z > 0.0f ? GZ : -1;
    int nx = r->dir.x > 0.0f ? ix + 1 : ix;
    float px = bb[0] + (float)nx * vw[0];
    int ny = r->dir.y > 0.0f ? iy + 1 : iy;
    float py = bb[1] + (float)ny * vw[1];
    int nz = r->dir.z > 0.0f ? iz + 1 : iz;
    float pz = bb[2] + (float)nz * vw[2];
    if (r->dir.x != 0) { delta.x = fabs_ref(vw[0] * r->inv.x); tmax.x = (px - p.x) * r->inv.x; }
    if (r->dir.y != 0) { delta.y = fabs_ref(vw[1] * r->inv.y); tmax.y = (py - p.y) * r->inv.y; }
    if (r->dir.z != 0) { delta.z = fabs_ref(vw[2] * r->inv.z); tmax.z = (pz - p.z) * r->inv.z; }
    int cx = 0, cy = 0, cz = 0;
    int hit = 0;
    for (;;) {
        int iv = g[0] + ix + iy * GX + iz * GX * GY;
        if (voxel_test(s, r, h, iv)) { cx = ix; cy = iy; cz = iz; hit = 1; }
        if (hit && (iabs(cx - ix) > 2 || iabs(cy - iy) > 2 || iabs(cz - iz) > 2)) return 1;
        if (tmax.x < tmax.y && tmax.x < tmax.z) {
            ix += sx;
            if (ix == ox || tmax.x >= OR_FMAX) return hit;
            tmax.x += delta.x;
        } else if (tmax.y < tmax.z) {
            iy += sy;
            if (iy == oy || tmax.y >= OR_FMAX) return hit;
            tmax.y += delta.y;
        } else {
            iz += sz;
            if (iz == oz || tmax.z >= OR_FMAX) return hit;
            tmax.z += delta.z;
        }
    }
}

/* Exact closest hit over every triangle of the mesh (accel = 1): the
 * semantic the BVH implements.  Same triangle test; ties -> lowest index. */
static int brute_test(const ptor_scene *s, const or_tray *r, or_hit *h, int mesh) {
    const int *mr = s->mesh_ranges + 4 * mesh;
    int any = 0;
    for (int it = mr[2]; it < mr[3]; it++)
        if (tri_test(s, r, h, it)) any = 1;
    return any;
}

/* transformNormal (utility.h:82-88): transpose(inverse(mat3(m))) * n */
static v3 xform_normal(const float *m, v3 n) {
    /* glm compute_inverse<tmat3x3> (type_mat3x3.inl:37-56), m[c][r] = m[c*4+r] */
#define M(c, r) m[(c)*4 + (r)]
    float det = +M(0, 0) * (M(1, 1) * M(2, 2) - M(2, 1) * M(1, 2))
                - M(1, 0) * (M(0, 1) * M(2, 2) - M(2, 1) * M(0, 2))
                + M(2, 0) * (M(0, 1) * M(1, 2) - M(1, 1) * M(0, 2));
    float od = 1.0f / det;
    float inv[3][3];
    inv[0][0] = +(M(1, 1) * M(2, 2) - M(2, 1) * M(1, 2)) * od;
    inv[1][0] = -(M(1, 0) * M(2, 2) - M(2, 0) * M(1, 2)) * od;
    inv[2][0] = +(M(1, 0) * M(2, 1) - M(2, 0) * M(1, 1)) * od;
    inv[0][1] = -(M(0, 1) * M(2, 2) - M(2, 1) * M(0, 2)) * od;
    inv[1][1] = +(M(0, 0) * M(2, 2) - M(2, 0) * M(0, 2)) * od;
    inv[2][1] = -(M(0, 0) * M(2, 1) - M(2, 0) * M(0, 1)) * od;
    inv[0][2] = +(M(0, 1) * M(1, 2) - M(1, 1) * M(0, 2)) * od;
    inv[1][2] = -(M(0, 0) * M(1, 2) - M(1, 0) * M(0, 2)) * od;
    inv[2][2] = +(M(0, 0) * M(1, 1) - M(1, 0) * M(0, 1)) * od;
#undef M
    /* it = transpose(inv): it[c][r] = inv[r][c]; glm mat3*vec3 (type_mat3x3.inl:487-493):
     * out.r = it[0][r]*n.x + it[1][r]*n.y + it[2][r]*n.z = inv[r][0]*n.x + inv[r][1]*n.y + inv[r][2]*n.z */
    float o[3];
    for (int r = 0; r < 3; r++) o[r] = inv[r][0] * n.x + inv[r][1] * n.y + inv[r][2] * n.z;
    return mk(o[0], o[1], o[2]);
}

/* computeRaySceneIntersectionKernel body (Renderer.cpp:364-409) for one ray.
 * Returns the model index hit (or -1) and fills dist/normal. */
static int scene_intersect(const ptor_scene *s, int accel, v3 orig, v3 dir, float *dist_out, v3 *n_out) {
    float gdist = OR_FMAX;
    v3 gn = mk(0, 0, 0);
    int gmodel = -1;
    for (int im = 0; im < s->nmodel; im++) {
        const float *w2m = s->model_w2m + 16 * im;
        const float *m2w = s->model_m2w + 16 * im;
        or_tray tr;
        tr.orig = xform(w2m, orig, 1.0f);
        tr.dir = vnorm(xform(w2m, dir, 0.0f));
        tr.inv = mk(1 / tr.dir.x, 1 / tr.dir.y, 1 / tr.dir.z);
        or_hit h; h.dist = OR_FMAX; h.normal = mk(0, 0, 0);
        int ok = accel == 0 ? grid_test(s, &tr, &h, s->model_ints[3 * im + 1])
                            : brute_test(s, &tr, &h, s->model_ints[3 * im + 0]);
        if (ok) {
            v3 nd = vnorm(tr.dir);
            v3 pm = vadd(tr.orig, vs(nd, h.dist));
            v3 pw = xform(m2w, pm, 1.0f);
            float d = vlen(vsub(pw, orig));
            if (gdist > d) {
                gdist = d;
                gmodel = im;
                gn = vnorm(xform_normal(m2w, h.normal));
            }
        }
    }
    if (gdist < OR_FMAX) { *dist_out = gdist; *n_out = gn; return gmodel; }
    *dist_out = OR_FMAX; *n_out = gn;
    return -1;
}

/* ---------------------------------------------------------------------- */
/* Render loop (Renderer.cpp:521-648)                                      */
/* ---------------------------------------------------------------------- */

typedef struct {
    v3 orig, dir;            /* Ray::base */
    v3 color;
    int ipixel, bounces;     /* Ray::MetaData */
} or_ray;

typedef struct {
    float dist;
    v3 normal;
    int model;               /* carries IntersectionData::impact_mat */
} or_isect;

/* generateRaysKernel (Renderer.cpp:521-555) */
static void gen_ray(const ptor_config *c, int iray, or_ray *r) {
    int W = c->width, H = c->height;
    v3 cam = mk((float)c->cam[0], (float)c->cam[1], (float)c->cam[2]);
    int y = iray / W, x = iray % W;
    float step_x = (float)(c->plane_w / W);
    float step_y = (float)(c->plane_h / H);
    float wx = (float)(c->plane_x0 + (double)((float)x * step_x));
    float wy = (float)(c->plane_y0 + (double)((float)y * step_y));
    float wz = (float)c->plane_z;
    r->orig = cam;
    r->dir = vsub(mk(wx, wy, wz), cam);
    r->color = mk(1.0f, 1.0f, 1.0f);
    r->bounces = c->max_bounces;
    r->ipixel = iray;
}

/* shadeRayKernel (Renderer.cpp:411-479) for one ray. */
static void shade_one(or_ray *ray, or_isect *hit, int iter, int iray, const ptor_scene *s) {
    if (ray->bounces <= 0) ray->color = vmul(ray->color, mk(0.01f, 0.01f, 0.01f));
    if (hit->dist < OR_FMAX) {
        v3 dir = vnorm(ray->dir);
        v3 p = vadd(ray->orig, vs(dir, hit->dist));
        if (ray->bounces > 0) {
            int mt = s->model_ints[3 * hit->model + 2];
            v3 mc = mk(s->model_color[3 * hit->model], s->model_color[3 * hit->model + 1], s->model_color[3 * hit->model + 2]);
            v3 n = hit->normal;
            if (mt == M_DIFFUSE) {
                or_rng rng = rng_make(iter, iray, ray->bounces);
                ray->dir = hemisphere(n, &rng);
                ray->orig = vadd(p, vs(n, 0.1f));
                ray->color = vmul(ray->color, mc);
            } else if (mt == M_METAL) {
                or_rng rng = rng_make(iter, iray, ray->bounces);
                ray->dir = metal(n, dir, &rng);
                ray->orig = vadd(p, vs(n, 0.1f));
                ray->color = vmul(ray->color, mc);
            } else if (mt == M_COAT) {
                or_rng rng = rng_make(iter, iray, ray->bounces);
                ray->dir = coat(n, dir, &rng);
                ray->orig = vadd(p, vs(n, 0.1f));
                ray->color = vmul(ray->color, mc);
            } else if (mt == M_EMISSIVE) {
                ray->bounces = 0;
                ray->color = vmul(ray->color, mc);
                hit->dist = OR_FMAX;
                return;
            } else if (mt == M_REFLECTIVE) {
                ray->color = vmul(ray->color, mc);
                v3 rr = reflect_ref(dir, n);
                ray->orig = vadd(p, vs(n, 0.1f));
                ray->dir = rr;
            }
        }
        hit->dist = OR_FMAX;
    } else {
        ray->bounces = 0;
        ray->color = vmul(ray->color, mk(0.01f, 0.01f, 0.01f));
        hit->dist = OR_FMAX;
        return;
    }
    ray->bounces--;
}

static void set_threads(int t) {
#ifdef _OPENMP
    if (t > 0) omp_set_num_threads(t);
#else
    (void)t;
#endif
}

int ptor_intersect_primary(const ptor_scene *s, const ptor_config *c, float *dist, float *normal, int *model) {
    int n = c->width * c->height;
    set_threads(c->threads);
#pragma omp parallel for schedule(dynamic, 256)
    for (int i = 0; i < n; i++) {
        or_ray r; gen_ray(c, i, &r);
        v3 nn; float d;
        int m = scene_intersect(s, c->accel, r.orig, r.dir, &d, &nn);
        dist[i] = d; normal[3 * i] = nn.x; normal[3 * i + 1] = nn.y; normal[3 * i + 2] = nn.z; model[i] = m;
    }
    return 0;
}

int ptor_intersect_rays(const ptor_scene *s, int accel, int n, const float *orig, const float *dir,
                        float *dist, float *normal, int *model, int threads) {
    set_threads(threads);
#pragma omp parallel for schedule(dynamic, 256)
    for (int i = 0; i < n; i++) {
        v3 nn; float d;
        int m = scene_intersect(s, accel, mk(orig[3 * i], orig[3 * i + 1], orig[3 * i + 2]),
                                mk(dir[3 * i], dir[3 * i + 1], dir[3 * i + 2]), &d, &nn);
        dist[i] = d; normal[3 * i] = nn.x; normal[3 * i + 1] = nn.y; normal[3 * i + 2] = nn.z; model[i] = m;
    }
    return 0;
}

int ptor_shade(int n, int iter, const int *slot, float *orig, float *dir, float *color, int *bounces,
               const float *hit_dist, const float *hit_normal, const int *hit_type, const float *hit_color) {
    for (int i = 0; i < n; i++) {
        /* build a one-model scene carrying the hit material */
        int mi[3] = {0, 0, hit_type[i]};
        ptor_scene s; memset(&s, 0, sizeof s);
        s.model_ints = mi; s.model_color = hit_color + 3 * i; s.nmodel = 1;
        or_ray r;
        r.orig = mk(orig[3 * i], orig[3 * i + 1], orig[3 * i + 2]);
        r.dir = mk(dir[3 * i], dir[3 * i + 1], dir[3 * i + 2]);
        r.color = mk(color[3 * i], color[3 * i + 1], color[3 * i + 2]);
        r.bounces = bounces[i]; r.ipixel = 0;
        or_isect h; h.dist = hit_dist[i];
        h.normal = mk(hit_normal[3 * i], hit_normal[3 * i + 1], hit_normal[3 * i + 2]); h.model = 0;
        shade_one(&r, &h, iter, slot[i], &s);
        orig[3 * i] = r.orig.x; orig[3 * i + 1] = r.orig.y; orig[3 * i + 2] = r.orig.z;
        dir[3 * i] = r.dir.x; dir[3 * i + 1] = r.dir.y; dir[3 * i + 2] = r.dir.z;
        color[3 * i] = r.color.x; color[3 * i + 1] = r.color.y; color[3 * i + 2] = r.color.z;
        bounces[i] = r.bounces;
    }
    return 0;
}

/* renderLoop (Renderer.cpp:567-648) */
int ptor_render(const ptor_scene *s, const ptor_config *c, float *image, long long *segments) {
    int n_total = c->width * c->height;
    /* dim3 blocks = ceil(nrays / 32) with integer division (Renderer.cpp:573):
     * the trailing nrays % 32 rays are never launched.  Optional. */
    int n_launch = c->tail_drop ? (n_total / 32) * 32 : n_total;
    or_ray *rays = (or_ray *)calloc((size_t)n_total, sizeof(or_ray));
    or_ray *tmp = (or_ray *)calloc((size_t)n_total, sizeof(or_ray));
    or_isect *isect = (or_isect *)calloc((size_t)n_total, sizeof(or_isect));
    or_isect *cache = (or_isect *)calloc((size_t)n_total, sizeof(or_isect));
    unsigned char *alive = (unsigned char *)calloc((size_t)n_total, 1);
    if (!rays || !tmp || !isect || !cache || !alive) { free(rays); free(tmp); free(isect); free(cache); free(alive); return -1; }
    set_threads(c->threads);
    long long seg = 0;
    /* dev_ray_data starts zero-filled (vector<Ray>): never-launched rays gather 0. */
    for (int it = 0; it < c->iterations; it++) {
        int iter = c->first_iter + it;
        int nrays = n_launch;
        for (int i = 0; i < nrays; i++) {
            gen_ray(c, i, &rays[i]);
            isect[i].dist = OR_FMAX;
        }
        int ib = 0;
        for (;;) {
            seg += nrays;
            if (ib == 0) {
                if (it == 0) {
                    /* computeRaySceneIntersectionKernel then cache (Renderer.cpp:603-612) */
#pragma omp parallel for schedule(dynamic, 256)
                    for (int i = 0; i < nrays; i++) {
                        v3 nn; float d;
                        int m = scene_intersect(s, c->accel, rays[i].orig, rays[i].dir, &d, &nn);
                        isect[i].dist = d;
                        if (m >= 0) { isect[i].normal = nn; isect[i].model = m; }
                        cache[i] = isect[i];
                    }
                } else {
                    memcpy(isect, cache, sizeof(or_isect) * (size_t)nrays);
                }
            } else {
#pragma omp parallel for schedule(dynamic, 256)
                for (int i = 0; i < nrays; i++) {
                    v3 nn; float d;
                    int m = scene_intersect(s, c->accel, rays[i].orig, rays[i].dir, &d, &nn);
                    isect[i].dist = d;
                    if (m >= 0) { isect[i].normal = nn; isect[i].model = m; }
                }
            }
            /* shadeRayKernel + compactStencilKernel */
#pragma omp parallel for schedule(static)
            for (int i = 0; i < nrays; i++) {
                shade_one(&rays[i], &isect[i], iter, i, s);
                alive[i] = rays[i].bounces <= 0 ? 0 : 1;
            }
            /* thrust::stable_partition(rays, rays + nrays, stencil, x == 1) */
            int na = 0;
            for (int i = 0; i < nrays; i++) if (alive[i]) tmp[na++] = rays[i];
            int nd = na;
            for (int i = 0; i < nrays; i++) if (!alive[i]) tmp[nd++] = rays[i];
            memcpy(rays, tmp, sizeof(or_ray) * (size_t)nrays);
            nrays = na;
            ib++;
            if (nrays == 0) break;
        }
        /* gatherImageDataKernel (Renderer.cpp:481-496) over the launched rays */
        for (int i = 0; i < n_launch; i++) {
            or_ray *r = &rays[i];
            v3 col = mk(sqrtf(r->color.x), sqrtf(r->color.y), sqrtf(r->color.z));
            float avg = (float)(1 / (1 * 1));
            float *px = image + 3 * (size_t)r->ipixel;
            px[0] += avg * col.x; px[1] += avg * col.y; px[2] += avg * col.z;
        }
    }
    if (segments) *segments = seg;
    free(rays); free(tmp); free(isect); free(cache); free(alive);
    return 0;
}

/* ---------------------------------------------------------------------- */
/* Scene construction                                                       */
/* ---------------------------------------------------------------------- */

static void m4_identity(float *m) { memset(m, 0, 64); m[0] = m[5] = m[10] = m[15] = 1.0f; }

/* glm mat4*mat4 (type_mat4x4.inl:686-704): R[i] = A0*B[i][0] + A1*B[i][1] + A2*B[i][2] + A3*B[i][3] */
static void m4_mul(const float *a, const float *b, float *out) {
    float r[16];
    for (int i = 0; i < 4; i++)
        for (int k = 0; k < 4; k++)
            r[i * 4 + k] = a[0 * 4 + k] * b[i * 4 + 0] + a[1 * 4 + k] * b[i * 4 + 1]
                         + a[2 * 4 + k] * b[i * 4 + 2] + a[3 * 4 + k] * b[i * 4 + 3];
    memcpy(out, r, 64);
}

/* glm::scale (matrix_transform.inl:122-134) */
static void m4_scale(const float *m, const float *v, float *out) {
    float r[16];
    for (int k = 0; k < 4; k++) {
        r[0 * 4 + k] = m[0 * 4 + k] * v[0];
        r[1 * 4 + k] = m[1 * 4 + k] * v[1];
        r[2 * 4 + k] = m[2 * 4 + k] * v[2];
        r[3 * 4 + k] = m[3 * 4 + k];
    }
    memcpy(out, r, 64);
}

/* glm::translate (matrix_transform.inl:39-48) */
static void m4_translate(const float *m, const float *v, float *out) {
    float r[16];
    memcpy(r, m, 64);
    for (int k = 0; k < 4; k++)
        r[3 * 4 + k] = m[0 * 4 + k] * v[0] + m[1 * 4 + k] * v[1] + m[2 * 4 + k] * v[2] + m[3 * 4 + k];
    memcpy(out, r, 64);
}

/* glm::rotate (matrix_transform.inl:51-85), angle in radians (float) */
static void m4_rotate(const float *m, float angle, v3 axis_in, float *out) {
    float c = cosf(angle), s = sinf(angle);
    v3 axis = vnorm(axis_in);
    v3 temp = vs(axis, 1.0f - c);
    float R[3][3];
    R[0][0] = c + temp.x * axis.x;
    R[0][1] = 0 + temp.x * axis.y + s * axis.z;
    R[0][2] = 0 + temp.x * axis.z - s * axis.y;
    R[1][0] = 0 + temp.y * axis.x - s * axis.z;
    R[1][1] = c + temp.y * axis.y;
    R[1][2] = 0 + temp.y * axis.z + s * axis.x;
    R[2][0] = 0 + temp.z * axis.x + s * axis.y;
    R[2][1] = 0 + temp.z * axis.y - s * axis.x;
    R[2][2] = c + temp.z * axis.z;
    float r[16];
    for (int i = 0; i < 3; i++)
        for (int k = 0; k < 4; k++)
            r[i * 4 + k] = m[0 * 4 + k] * R[i][0] + m[1 * 4 + k] * R[i][1] + m[2 * 4 + k] * R[i][2];
    for (int k = 0; k < 4; k++) r[3 * 4 + k] = m[3 * 4 + k];
    memcpy(out, r, 64);
}

/* glm compute_inverse<tmat4x4> (type_mat4x4.inl:37-92) */
static void m4_inverse(const float *mm, float *out) {
#define M(c, r) mm[(c)*4 + (r)]
    float C00 = M(2, 2) * M(3, 3) - M(3, 2) * M(2, 3);
    float C02 = M(1, 2) * M(3, 3) - M(3, 2) * M(1, 3);
    float C03 = M(1, 2) * M(2, 3) - M(2, 2) * M(1, 3);
    float C04 = M(2, 1) * M(3, 3) - M(3, 1) * M(2, 3);
    float C06 = M(1, 1) * M(3, 3) - M(3, 1) * M(1, 3);
    float C07 = M(1, 1) * M(2, 3) - M(2, 1) * M(1, 3);
    float C08 = M(2, 1) * M(3, 2) - M(3, 1) * M(2, 2);
    float C10 = M(1, 1) * M(3, 2) - M(3, 1) * M(1, 2);
    float C11 = M(1, 1) * M(2, 2) - M(2, 1) * M(1, 2);
    float C12 = M(2, 0) * M(3, 3) - M(3, 0) * M(2, 3);
    float C14 = M(1, 0) * M(3, 3) - M(3, 0) * M(1, 3);
    float C15 = M(1, 0) * M(2, 3) - M(2, 0) * M(1, 3);
    float C16 = M(2, 0) * M(3, 2) - M(3, 0) * M(2, 2);
    float C18 = M(1, 0) * M(3, 2) - M(3, 0) * M(1, 2);
    float C19 = M(1, 0) * M(2, 2) - M(2, 0) * M(1, 2);
    float C20 = M(2, 0) * M(3, 1) - M(3, 0) * M(2, 1);
    float C22 = M(1, 0) * M(3, 1) - M(3, 0) * M(1, 1);
    float C23 = M(1, 0) * M(2, 1) - M(2, 0) * M(1, 1);
    float F0[4] = {C00, C00, C02, C03}, F1[4] = {C04, C04, C06, C07}, F2[4] = {C08, C08, C10, C11};
    float F3[4] = {C12, C12, C14, C15}, F4[4] = {C16, C16, C18, C19}, F5[4] = {C20, C20, C22, C23};
    float V0[4] = {M(1, 0), M(0, 0), M(0, 0), M(0, 0)};
    float V1[4] = {M(1, 1), M(0, 1), M(0, 1), M(0, 1)};
    float V2[4] = {M(1, 2), M(0, 2), M(0, 2), M(0, 2)};
    float V3[4] = {M(1, 3), M(0, 3), M(0, 3), M(0, 3)};
    float I0[4], I1[4], I2[4], I3[4];
    for (int k = 0; k < 4; k++) {
        I0[k] = V1[k] * F0[k] - V2[k] * F1[k] + V3[k] * F2[k];
        I1[k] = V0[k] * F0[k] - V2[k] * F3[k] + V3[k] * F4[k];
        I2[k] = V0[k] * F1[k] - V1[k] * F3[k] + V3[k] * F5[k];
        I3[k] = V0[k] * F2[k] - V1[k] * F4[k] + V2[k] * F5[k];
    }
    float SA[4] = {+1, -1, +1, -1}, SB[4] = {-1, +1, -1, +1};
    float inv[16];
    for (int k = 0; k < 4; k++) {
        inv[0 * 4 + k] = I0[k] * SA[k];
        inv[1 * 4 + k] = I1[k] * SB[k];
        inv[2 * 4 + k] = I2[k] * SA[k];
        inv[3 * 4 + k] = I3[k] * SB[k];
    }
    float row0[4] = {inv[0], inv[4], inv[8], inv[12]};
    float d0[4];
    for (int k = 0; k < 4; k++) d0[k] = M(0, k) * row0[k];
    float d1 = (d0[0] + d0[1]) + (d0[2] + d0[3]);
    float od = 1.0f / d1;
    for (int i = 0; i < 16; i++) out[i] = inv[i] * od;
#undef M
}

/* Scene.cpp:34-39 pattern: M = translate * rotate * scale, W = inverse(M).
 * rotate = rotate(rotate(rotate(I, rx, X), ry, Y), rz, Z) with glm::radians. */
void ptor_model_matrix(const float scale[3], const float rot_deg[3], const float translate[3], float m2w[16], float w2m[16]) {
    float I[16], S[16], R[16], T[16], TR[16];
    m4_identity(I);
    m4_scale(I, scale, S);
    const float deg2rad = (float)0.01745329251994329576923690768489; /* glm::radians */
    m4_rotate(I, rot_deg[0] * deg2rad, mk(1.0f, 0.0f, 0.0f), R);
    m4_rotate(R, rot_deg[1] * deg2rad, mk(0.0f, 1.0f, 0.0f), R);
    m4_rotate(R, rot_deg[2] * deg2rad, mk(0.0f, 0.0f, 1.0f), R);
    m4_translate(I, translate, T);
    m4_mul(T, R, TR);
    m4_mul(TR, S, m2w);
    m4_inverse(m2w, w2m);
}

/* computeVoxelIndex (Scene.cpp:293-316), host (x86) float->int semantics */
static void voxel_range(const float *bb, const float *vw, const v3 *tri, const int gd[3], int mn[3], int mx[3]) {
    float tmin[3] = {OR_FMAX, OR_FMAX, OR_FMAX}, tmax[3] = {OR_FMIN, OR_FMIN, OR_FMIN};
    for (int j = 0; j < 3; j++) {
        float p[3] = {tri[j].x, tri[j].y, tri[j].z};
        for (int a = 0; a < 3; a++) {
            tmin[a] = tmin[a] > p[a] ? p[a] : tmin[a];
            tmax[a] = tmax[a] < p[a] ? p[a] : tmax[a];
        }
    }
    for (int a = 0; a < 3; a++) {
        mn[a] = f2i_x86(floorf(fabsf(bb[a] - tmin[a]) / vw[a]));
        mx[a] = f2i_x86(floorf(fabsf(bb[a] - tmax[a]) / vw[a]));
        mn[a] = mn[a] < 0 ? 0 : (mn[a] > gd[a] - 1 ? gd[a] - 1 : mn[a]);
        mx[a] = mx[a] < 0 ? 0 : (mx[a] > gd[a] - 1 ? gd[a] - 1 : mx[a]);
    }
}

/* addMeshesToGrid (Scene.cpp:318-396) */
int ptor_build_grids(int nmesh, const int *mesh_ranges, const float *mesh_bbox, const float *vpos, const int *tris,
                     int nmodel, int *model_ints, const int gdim[3], int *ngrid, int *grid_ints, float *grid_vw,
                     int *nvox, int *vox, int pv_cap, int *npv, int *per_voxel) {
    const int G = gdim[0] * gdim[1] * gdim[2];
    int *done = (int *)calloc((size_t)(nmesh > 0 ? nmesh : 1), sizeof(int));
    int *cache = (int *)calloc((size_t)(nmesh > 0 ? nmesh : 1), sizeof(int));
    int *cnt = (int *)malloc(sizeof(int) * (size_t)G);
    int *off = (int *)malloc(sizeof(int) * (size_t)G);
    int ng = 0, nv = 0, np = 0, rc = 0;
    for (int i = 0; i < nmodel; i++) {
        int mesh = model_ints[3 * i + 0];
        if (done[mesh]) { model_ints[3 * i + 1] = cache[mesh]; continue; }
        done[mesh] = 1;
        cache[mesh] = ng;
        model_ints[3 * i + 1] = ng;
        const float *bb = mesh_bbox + 6 * mesh;
        float vw[3];
        vw[0] = (bb[3] - bb[0]) / (float)gdim[0];
        vw[1] = (bb[4] - bb[1]) / (float)gdim[1];
        vw[2] = (bb[5] - bb[2]) / (float)gdim[2];
        const int *mr = mesh_ranges + 4 * mesh;
        /* two passes: count, then fill in triangle order (== vector push_back order) */
        memset(cnt, 0, sizeof(int) * (size_t)G);
        for (int pass = 0; pass < 2; pass++) {
            if (pass == 1) {
                int acc = 0;
                for (int v = 0; v < G; v++) { off[v] = acc; acc += cnt[v]; }
                if (np + acc > pv_cap) rc = -(np + acc);
                memset(cnt, 0, sizeof(int) * (size_t)G);
            }
            for (int t = mr[2]; t < mr[3]; t++) {
                v3 tri[3];
                for (int j = 0; j < 3; j++) {
                    int vi = tris[3 * t + j];
                    tri[j] = mk(vpos[3 * vi], vpos[3 * vi + 1], vpos[3 * vi + 2]);
                }
                int mn[3], mx[3];
                voxel_range(bb, vw, tri, gdim, mn, mx);
                for (int z = mn[2]; z <= mx[2]; z++)
                    for (int y = mn[1]; y <= mx[1]; y++)
                        for (int x = mn[0]; x <= mx[0]; x++) {
                            int idx = x + y * gdim[0] + gdim[0] * gdim[1] * z;
                            if (pass == 1 && rc == 0) per_voxel[np + off[idx] + cnt[idx]] = t;
                            cnt[idx]++;
                        }
            }
        }
        int *g = grid_ints + 4 * ng;
        g[0] = nv;
        for (int v = 0; v < G; v++) {
            vox[3 * nv + 0] = np + off[v];
            vox[3 * nv + 1] = np + off[v] + cnt[v];
            vox[3 * nv + 2] = 2; /* EntityType::TRIANGLE */
            nv++;
        }
        np += (G > 0) ? off[G - 1] + cnt[G - 1] : 0;
        g[1] = nv;
        g[2] = 0; /* EntityType::MODEL */
        g[3] = i;
        grid_vw[3 * ng + 0] = vw[0]; grid_vw[3 * ng + 1] = vw[1]; grid_vw[3 * ng + 2] = vw[2];
        ng++;
    }
    *ngrid = ng; *nvox = nv; *npv = np;
    free(done); free(cache); free(cnt); free(off);
    return rc;
}
