// pt_math.h -- float/double arithmetic shared by the host scene builder and
// the gfx950 kernels.  Every helper keeps the operand order of the
// reference's glm 0.9.6 / thrust / utility.h code (cited per function) so the
// HIP path is bit-reproducible; the translation units are compiled with
// -ffp-contract=off (and the pragma below) so no a*b+c is fused.
#pragma once
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>
#include <stdint.h>

#define PT_HD __host__ __device__ __forceinline__

namespace pt {

// Config.h:4-6
constexpr float kEps = 0.005f;
constexpr float kFMax = 9999999.0f;
constexpr float kFMin = -9999990.0f;
// utility.h:20-22
constexpr float kTwoPi = 6.2831853071795864769252867665590057683943f;
constexpr float kSqrtOneThird = 0.5773502691896257645091487805019574556476f;

// Primitive.h:70-79 Material::MaterialType
enum MaterialType : int {
    MAT_DIFFUSE = 0, MAT_SPECULAR = 1, MAT_REFLECTIVE = 2, MAT_REFRACTIVE = 3,
    MAT_EMISSIVE = 4, MAT_COAT = 5, MAT_METAL = 6
};

struct f3 { float x, y, z; };

PT_HD f3 mk3(float x, float y, float z) { f3 r; r.x = x; r.y = y; r.z = z; return r; }
PT_HD f3 operator+(f3 a, f3 b) { return mk3(a.x + b.x, a.y + b.y, a.z + b.z); }
PT_HD f3 operator-(f3 a, f3 b) { return mk3(a.x - b.x, a.y - b.y, a.z - b.z); }
PT_HD f3 operator*(f3 a, f3 b) { return mk3(a.x * b.x, a.y * b.y, a.z * b.z); }
PT_HD f3 operator*(f3 a, float s) { return mk3(a.x * s, a.y * s, a.z * s); }
// glm compute_dot<tvec3> (func_geometric.inl:67-71): (x*x' + y*y') + z*z'
PT_HD float dot(f3 a, f3 b) { f3 t = a * b; return t.x + t.y + t.z; }
// glm cross (func_geometric.inl:134-142)
PT_HD f3 cross(f3 x, f3 y) {
    return mk3(x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y);
}
// glm normalize: x * (1 / sqrt(dot(x, x))) (func_geometric.inl:153-159, func_exponential.inl:150)
PT_HD f3 normalize(f3 a) { float s = 1.0f / sqrtf(dot(a, a)); return a * s; }
PT_HD float length(f3 a) { return sqrtf(dot(a, a)); }
// utility.h:14 ABS
PT_HD float absr(float x) { return x < 0 ? -x : x; }
PT_HD int iabs(int x) { return x < 0 ? -x : x; }

// GPU float->int (v_cvt_i32_f32, the reference's cvt.rzi.s32.f32): NaN -> 0, saturating.
PT_HD int f2i_sat(float f) {
    if (f != f) return 0;
    if (f >= 2147483648.0f) return 2147483647;
    if (f <= -2147483648.0f) return (-2147483647 - 1);
    return (int)f;
}
// x86 host float->int (cvttss2si, the reference's Scene.cpp on MSVC): NaN/overflow -> INT_MIN.
PT_HD int f2i_x86(float f) {
    if (f != f || f >= 2147483648.0f || f < -2147483648.0f) return (-2147483647 - 1);
    return (int)f;
}

// glm mat4 * vec4 (type_mat4x4.inl:591-628) keeping rows 0..2:
// (m0*x + m1*y) + (m2*z + m3*w).  `m` holds 12 floats: column c, row k at m[c*3+k].
PT_HD f3 xform12(const float* m, f3 p, float w) {
    float r[3];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        float a0 = m[0 * 3 + k] * p.x;
        float a1 = m[1 * 3 + k] * p.y;
        float a2 = m[2 * 3 + k] * p.z;
        float a3 = m[3 * 3 + k] * w;
        r[k] = (a0 + a1) + (a2 + a3);
    }
    return mk3(r[0], r[1], r[2]);
}

// transformNormal (utility.h:82-88) with the inverse-transpose precomputed as
// nm[r*3+c] = inverse(mat3(m))[r][c]: out.r = nm[r][0]*n.x + nm[r][1]*n.y + nm[r][2]*n.z
PT_HD f3 xform_normal9(const float* nm, f3 n) {
    float o[3];
#pragma unroll
    for (int r = 0; r < 3; r++) o[r] = nm[r * 3 + 0] * n.x + nm[r * 3 + 1] * n.y + nm[r * 3 + 2] * n.z;
    return mk3(o[0], o[1], o[2]);
}

// ---------------------------------------------------------------------------
// Transcendentals.  CUDA's sinf/cosf/powf are replaced by double-precision
// polynomial evaluations rounded once to float (correctly rounded in all
// sampled cases, so within 1 ulp of the reference's device functions).
// ---------------------------------------------------------------------------
PT_HD double dfloor(double q) {
    double t = (double)(long long)q;
    return (t > q) ? t - 1.0 : t;
}

PT_HD void sincos_ref(float xf, float* so, float* co) {
    double x = (double)xf;
    if (!(x - x == 0.0)) { *so = __builtin_nanf(""); *co = __builtin_nanf(""); return; }
    double k = dfloor(x * 0.63661977236758134308 + 0.5);
    const double pio2_1 = 1.57079632673412561417e+00;
    const double pio2_1t = 6.07710050650619224932e-11;
    double r = (x - k * pio2_1) - k * pio2_1t;
    double r2 = r * r;
    double sp = 1.0 / 355687428096000.0;
    sp = sp * r2 + (-1.0 / 1307674368000.0);
    sp = sp * r2 + (1.0 / 6227020800.0);
    sp = sp * r2 + (-1.0 / 39916800.0);
    sp = sp * r2 + (1.0 / 362880.0);
    sp = sp * r2 + (-1.0 / 5040.0);
    sp = sp * r2 + (1.0 / 120.0);
    sp = sp * r2 + (-1.0 / 6.0);
    double s = r + (r * r2) * sp;
    double cp = 1.0 / 6402373705728000.0;
    cp = cp * r2 + (-1.0 / 20922789888000.0);
    cp = cp * r2 + (1.0 / 87178291200.0);
    cp = cp * r2 + (-1.0 / 479001600.0);
    cp = cp * r2 + (1.0 / 3628800.0);
    cp = cp * r2 + (-1.0 / 40320.0);
    cp = cp * r2 + (1.0 / 720.0);
    cp = cp * r2 + (-1.0 / 24.0);
    cp = cp * r2 + 0.5;
    double c = 1.0 - r2 * cp;
    int q = (int)(((long long)k) & 3);
    double sv, cv;
    if (q == 0) { sv = s; cv = c; }
    else if (q == 1) { sv = c; cv = -s; }
    else if (q == 2) { sv = -s; cv = -c; }
    else { sv = -c; cv = s; }
    *so = (float)sv;
    *co = (float)cv;
}

PT_HD double dlog_ref(double x) {
    uint64_t b = __builtin_bit_cast(uint64_t, x);
    int e = (int)((b >> 52) & 0x7ff) - 1023;
    b = (b & 0x000fffffffffffffULL) | 0x3ff0000000000000ULL;
    double m = __builtin_bit_cast(double, b);
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

PT_HD double dexp_ref(double z) {
    if (z < -745.0) return 0.0;
    if (z > 709.0) return __builtin_inf();
    double k = dfloor(z * 1.44269504088896338700 + 0.5);
    const double ln2_hi = 6.93147180369123816490e-01;
    const double ln2_lo = 1.90821492927058770002e-10;
    double r = (z - k * ln2_hi) - k * ln2_lo;
    double p = 1.0 / 87178291200.0;
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
    int k1 = ki / 2, k2 = ki - k1;
    double s1 = __builtin_bit_cast(double, (uint64_t)(k1 + 1023) << 52);
    double s2 = __builtin_bit_cast(double, (uint64_t)(k2 + 1023) << 52);
    return (p * s1) * s2;
}

PT_HD float powf_ref(float xf, float yf) {
    if (xf != xf || yf != yf) return __builtin_nanf("");
    if (yf == 0.0f) return 1.0f;
    if (xf == 1.0f) return 1.0f;
    if (xf == 0.0f) return yf > 0.0f ? 0.0f : __builtin_inff();
    if (xf < 0.0f) return __builtin_nanf("");
    return (float)dexp_ref((double)yf * dlog_ref((double)xf));
}

// ---------------------------------------------------------------------------
// RNG: utility.h:43-62 (utilHash, makeSeededRandomEngine) over thrust's
// default_random_engine = minstd_rand (x <- 48271 x mod 2^31-1, min 1) and
// uniform_real_distribution<float>(0,1).
// ---------------------------------------------------------------------------
PT_HD uint32_t util_hash(uint32_t a) {
    a = (a + 0x7ed55d16u) + (a << 12);
    a = (a ^ 0xc761c23cu) ^ (a >> 19);
    a = (a + 0x165667b1u) + (a << 5);
    a = (a + 0xd3a2646cu) ^ (a << 9);
    a = (a + 0xfd7046c5u) + (a << 3);
    a = (a ^ 0xb55a4f09u) ^ (a >> 16);
    return a;
}

struct Rng {
    uint32_t x;
    PT_HD static Rng make(int iter, int index, int depth) {
        uint32_t h = util_hash(0x80000000u | ((uint32_t)depth << 22) | (uint32_t)iter) ^ util_hash((uint32_t)index);
        Rng r;
        r.x = h % 2147483647u;
        if (r.x == 0) r.x = 1;
        return r;
    }
    PT_HD float u01() {
        x = (uint32_t)(((uint64_t)x * 48271u) % 2147483647u);
        float res = (float)(uint32_t)(x - 1u);
        res = res / (1.0f + (float)(2147483646u - 1u));
        return res * (1.0f - 0.0f) + 0.0f;
    }
};

// ---------------------------------------------------------------------------
// Scattering (utility.h:64-170)
// ---------------------------------------------------------------------------
// reflectRay (utility.h:64-69): n - (2 dot(i,n)) n   (the reference's formula)
PT_HD f3 reflect_ref(f3 i, f3 n) { return n - n * (2.0f * dot(i, n)); }

// calculateRandomDirectionInHemisphere (utility.h:91-123)
PT_HD f3 scatter_hemisphere(f3 n, Rng& rng) {
    float up = sqrtf(rng.u01());
    float over = sqrtf(1.0f - up * up);
    float around = rng.u01() * kTwoPi;
    f3 dnn;
    if (absr(n.x) < kSqrtOneThird) dnn = mk3(1, 0, 0);
    else if (absr(n.y) < kSqrtOneThird) dnn = mk3(0, 1, 0);
    else dnn = mk3(0, 0, 1);
    f3 p1 = normalize(cross(n, dnn));
    f3 p2 = normalize(cross(n, p1));
    float sa, ca;
    sincos_ref(around, &sa, &ca);
    return (n * up + p1 * (ca * over)) + p2 * (sa * over);
}

// calculateCoatScattering (utility.h:125-143)
PT_HD f3 scatter_coat(f3 n, f3 d, Rng& rng) {
    float roulette = rng.u01();
    if (roulette < 0.5f) return reflect_ref(d, n);
    return scatter_hemisphere(n, rng);
}

// calculateMetalScattering (utility.h:145-170)
PT_HD f3 scatter_metal(f3 n, f3 d, Rng& rng) {
    (void)rng.u01();              // up     (drawn, unused)
    (void)rng.u01();              // around (drawn, unused)
    float phi = kTwoPi * rng.u01();
    float r2 = rng.u01();
    float phong = 30.0f;
    float cos_t = powf_ref(1.0f - r2, 1.0f / (phong + 1.0f));
    float sin_t = sqrtf(1.0f - cos_t * cos_t);
    f3 w = normalize(d - (n * 2.0f) * dot(n, d));
    f3 a = ((double)absr(w.x) > .1) ? mk3(0, 1, 0) : mk3(1, 0, 0);
    f3 u = normalize(cross(a, w));
    f3 v = cross(w, u);
    float sp, cp;
    sincos_ref(phi, &sp, &cp);
    return ((u * cp) * sin_t + (v * sp) * sin_t) + w * cos_t;
}

}  // namespace pt
