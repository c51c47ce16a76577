// device_math.hpp -- CDNA4 device-side arithmetic of the render loop.
//
// Every helper reproduces, operation for operation, the evaluation order of the
// reference's glm 0.9.8.5 / libstdc++ code (cited per function), so that with
// -ffp-contract=off and IEEE div/sqrt the kernels are bit-identical to the CPU
// restatement in oracle/oracle.c.  Nothing here may be "simplified": a fused
// multiply-add, an rsq instead of 1/sqrt, or fminf instead of the ternary changes
// results in the last ulp and, through hit/miss flips, whole paths.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cr {

struct f3 {
    float x, y, z;
};
__device__ __forceinline__ f3 mk(float x, float y, float z) { return f3{x, y, z}; }
__device__ __forceinline__ f3 add(f3 a, f3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ f3 sub(f3 a, f3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ f3 mul(f3 a, f3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ f3 muls(f3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ f3 divs(f3 a, float s) { return mk(a.x / s, a.y / s, a.z / s); } // type_vec3.inl:672
__device__ __forceinline__ f3 neg(f3 a) { return mk(-a.x, -a.y, -a.z); }
// func_geometric.inl:53-59
__device__ __forceinline__ float dot(f3 a, f3 b) {
    f3 t = mul(a, b);
    return t.x + t.y + t.z;
}
// func_geometric.inl:77-83
__device__ __forceinline__ f3 cross(f3 x, f3 y) {
    return mk(x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y);
}
// func_geometric.inl:94, func_exponential.inl:130-133
__device__ __forceinline__ f3 normalize(f3 v) { return muls(v, 1.0f / sqrtf(dot(v, v))); }
__device__ __forceinline__ float length3(f3 v) { return sqrtf(dot(v, v)); }
__device__ __forceinline__ float distance3(f3 p0, f3 p1) { return length3(sub(p1, p0)); }
// libstdc++ std::min/std::max and glm::max semantics (NaN / signed-zero exact)
__device__ __forceinline__ float std_min(float a, float b) { return (b < a) ? b : a; }
__device__ __forceinline__ float std_max(float a, float b) { return (a < b) ? b : a; }
__device__ __forceinline__ float glm_max(float x, float y) { return x > y ? x : y; }
__device__ __forceinline__ float comp(f3 a, uint32_t i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }
__device__ __forceinline__ f3 ld3(const float4 v) { return mk(v.x, v.y, v.z); }

// ---------------------------------------------------- exact fast division --
// Both return exactly the correctly rounded IEEE result the reference's float
// division gives; the short sequences are only taken inside the ranges where
// they are proven/checked exact, anything else takes the full division.
//
// RN(a/b) given y = rcp_for_div(b) (once per ray and axis): Markstein's
// correction q0 = RN(a*y), r = a - b*q0 (exact by fma), q = RN(q0 + r*y).
// Exact when y = RN(1/b) and nothing under/overflows, which the ranges
// 2^-40 <= |b| <= 2^40 and 2^-60 <= |q0| <= 2^60 guarantee (checked:
// scripts/markstein_check.c, 1.7e10 pairs half of them next to rounding
// midpoints; tests/test_gpu_numerics.py on the GPU).
__device__ __forceinline__ float rcp_for_div(float b) {
    const float ab = fabsf(b);
    return (ab >= 0x1p-40f && ab <= 0x1p40f) ? 1.f / b : __builtin_nanf(""); // NaN: always the slow path
}
__device__ __forceinline__ float div_by_rcp(float a, float b, float y) {
    const float q0 = a * y;
    if (fabsf(q0) >= 0x1p-60f && fabsf(q0) <= 0x1p60f) return __builtin_fmaf(__builtin_fmaf(-q0, b, a), y, q0);
    return a / b;
}
// div_by_rcp for wave-wide use (the packet camera trace): the range test is one wave-uniform
// branch, the full division runs for the whole wave only when some lane is out of range.
__device__ __forceinline__ float div_by_rcp_wave(float a, float b, float y) {
    const float q0 = a * y;
    float q = __builtin_fmaf(__builtin_fmaf(-q0, b, a), y, q0);
    const bool in = fabsf(q0) >= 0x1p-60f && fabsf(q0) <= 0x1p60f;
    if (__ballot(!in)) q = in ? q : a / b;
    return q;
}
// RN(1/a): hardware reciprocal (1 ulp) + one Newton step with fma.  Checked
// exhaustively over every float with 2^-100 <= |a| <= 2^100 on gfx950
// (tests/test_gpu_numerics.py).
__device__ __forceinline__ float rcp_rn(float a) {
    const float aa = fabsf(a);
    if (aa >= 0x1p-100f && aa <= 0x1p100f) {
        const float y0 = __builtin_amdgcn_rcpf(a);
        return __builtin_fmaf(__builtin_fmaf(-a, y0, 1.f), y0, y0);
    }
    return 1.f / a;
}

// rcp_rn for wave-wide use: the range test is one wave-uniform branch (the full
// division runs for the whole wave only when some lane is out of range) instead
// of a divergent if/else, which costs the scalar unit ~6 exec-mask instructions.
__device__ __forceinline__ float rcp_rn_wave(float a) {
    const float aa = fabsf(a);
    const float y0 = __builtin_amdgcn_rcpf(a);
    float r = __builtin_fmaf(__builtin_fmaf(-a, y0, 1.f), y0, y0);
    const bool in = aa >= 0x1p-100f && aa <= 0x1p100f;
    if (__ballot(!in)) r = in ? r : 1.f / a;
    return r;
}

// ---------------------------------------------------------------- RNG --
// Counter-based URBG (DESIGN.md "RNG"); identical to oracle/oracle.c rng_*.
__device__ __forceinline__ uint32_t mix32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}
struct Rng {
    uint32_t key, ctr;
};
__device__ __forceinline__ Rng rng_make(uint32_t seed, uint32_t layer, uint32_t pixel, uint32_t sample) {
    return Rng{mix32(mix32(mix32(mix32(seed) ^ layer) ^ pixel) ^ sample), 0u};
}
__device__ __forceinline__ uint32_t rng_u32(Rng &r) {
    uint32_t u = mix32(r.key + r.ctr * 0x9E3779B9U);
    r.ctr++;
    return u;
}
// uniform_real_distribution<float>(a, b): generate_canonical (random.tcc:3348-3377)
__device__ __forceinline__ float rng_uniform(Rng &r, float a, float b) {
    float c = (float)rng_u32(r) / 4294967296.0f;
    if (c >= 1.0f) c = 0x1.fffffep-1f;
    return c * (b - a) + a;
}
// uniform_int_distribution<int>(0, n-1), Lemire (uniform_int_dist.h:245-269)
__device__ __forceinline__ uint32_t rng_index(Rng &r, uint32_t n) {
    uint64_t prod = (uint64_t)rng_u32(r) * (uint64_t)n;
    uint32_t low = (uint32_t)prod;
    if (low < n) {
        uint32_t thr = (uint32_t)(0u - n) % n;
        while (low < thr) {
            prod = (uint64_t)rng_u32(r) * (uint64_t)n;
            low = (uint32_t)prod;
        }
    }
    return (uint32_t)(prod >> 32);
}

// ------------------------------------------------------------ sincos --
// glibc's sinf / cosf, the functions src/brdf.cpp:52-53 calls (glibc 2.35,
// x86-64 FMA ifunc; sysdeps/ieee754/flt-32 s_sinf.c / s_cosf.c / sincosf.h):
// double-precision polynomials on the argument reduced by a 2^24-scaled 2/pi,
// every a*b+c of the C source contracted to one fma as the -mfma build does.
// The same op sequence is oracle/oracle.c glibc_sincosf, checked equal to the
// host's libm sinf / cosf on every float with |x| < 120 (tests/test_oracle_golden.py
// samples it; scripts/glibc_trig_check.c sweeps all 2.25e9) and run against libm on
// the GPU over all of [0, 2pi] (tests/native/numerics_check.hip).
// The coefficients are glibc's __sincosf_table[0] as libm holds it; table [1]
// (quadrants 2, 3) is [0] with the cosine coefficients negated, which negates the
// cosine polynomial exactly (round-to-nearest is sign-symmetric), so it is
// applied as a sign on the result.
namespace glibc_sincos {
constexpr double HPI_INV = 0x1.45f306dc9c883p+23, HPI = 0x1.921fb54442d18p+0;
constexpr double C0 = 0x1p0, C1 = -0x1.ffffffd0c621cp-2, C2 = 0x1.55553e1068f19p-5, C3 = -0x1.6c087e89a359dp-10,
                 C4 = 0x1.99343027bf8c3p-16;
constexpr double S1 = -0x1.555545995a603p-3, S2 = 0x1.1107605230bc4p-7, S3 = -0x1.994eb3774cf24p-13;
} // namespace glibc_sincos
__device__ __forceinline__ uint32_t abstop12(float x) { return (__float_as_uint(x) >> 20) & 0x7ffu; }
// sincosf.h sinf_poly, n even (sine) and odd (cosine)
__device__ __forceinline__ double glibc_sin_poly(double x, double x2) {
    using namespace glibc_sincos;
    const double x3 = x * x2;
    const double s1 = __fma_rn(x2, S3, S2);
    const double x7 = x3 * x2;
    const double s = __fma_rn(x3, S1, x);
    return __fma_rn(x7, s1, s);
}
__device__ __forceinline__ double glibc_cos_poly(double x2) {
    using namespace glibc_sincos;
    const double x4 = x2 * x2;
    const double c2 = __fma_rn(x2, C4, C3);
    const double c1 = __fma_rn(x2, C1, C0);
    const double x6 = x4 * x2;
    const double c = __fma_rn(x4, C2, c1);
    return __fma_rn(x6, c2, c);
}
// s_sinf.c / s_cosf.c for |y| < 120 (theta of concentric() lies in [0, 2pi])
__device__ __forceinline__ void cr_sincosf(float y, float &sn, float &cs) {
    double x = (double)y;
    if (abstop12(y) < abstop12(0x1.921FB6p-1f)) { // |y| < ~pi/4
        if (abstop12(y) < abstop12(0x1p-12f)) {
            sn = y;
            cs = 1.0f;
            return;
        }
        const double x2 = x * x;
        sn = (float)glibc_sin_poly(x, x2);
        cs = (float)glibc_cos_poly(x2);
        return;
    }
    // reduce_fast, !TOINT_INTRINSICS: the quadrant from the 2^24-scaled product
    const double r = x * glibc_sincos::HPI_INV;
    const int n = ((int32_t)r + 0x800000) >> 24;
    x = __fma_rn(-(double)n, glibc_sincos::HPI, x);
    const double xs = ((n & 3) == 1 || (n & 3) == 2) ? -x : x; // sign[n & 3] = {1, -1, -1, 1}
    const double x2 = x * x;
    const double ps = glibc_sin_poly(xs, x2), pc = (n & 2) ? -glibc_cos_poly(x2) : glibc_cos_poly(x2);
    // odd quadrants swap the polynomials (sinf_poly(.., n) / (.., n ^ 1))
    sn = (float)((n & 1) ? pc : ps);
    cs = (float)((n & 1) ? ps : pc);
}

// --------------------------------------------------------------- BRDF --
// src/brdf.cpp:10-15
__device__ __forceinline__ f3 perpendicular(f3 v) {
    if (fabsf(v.x) < fabsf(v.y)) return mk(0.0f, -v.z, v.y);
    return mk(-v.z, 0.0f, v.x);
}
// src/brdf.cpp:18-54 (draws supplied by the caller in the reference's order)
__device__ __forceinline__ void concentric(float sx, float sy, float &dx, float &dy) {
    if (sx == 0.0f && sy == 0.0f) {
        dx = 0.0f;
        dy = 0.0f;
        return;
    }
    float r, theta;
    if (sx >= -sy) {
        if (sx > sy) {
            r = sx;
            theta = (sy > 0.0f) ? sy / r : 8.0f + sy / r;
        } else {
            r = sy;
            theta = 2.0f - sx / r;
        }
    } else {
        if (sx <= sy) {
            r = -sx;
            theta = 4.0f - sy / r;
        } else {
            r = -sy;
            theta = 6.0f + sx / r;
        }
    }
    theta = (float)((double)theta * (3.14159265358979323846 / 4.0)); // theta *= M_PI / 4.f (double)
    float sn, cs;
    cr_sincosf(theta, sn, cs);
    dx = r * cs;
    dy = r * sn;
}
// src/brdf.cpp:57-62, 72-79 Diffuse::sample_wi
__device__ __forceinline__ void sample_wi(f3 n, float sx, float sy, f3 &wi, float &pdf) {
    const f3 tangent = normalize(perpendicular(n));
    const f3 bitangent = normalize(cross(tangent, n));
    float hx, hy;
    concentric(sx, sy, hx, hy);
    const float hz = sqrtf(std_max(0.f, 1.f - hx * hx - hy * hy));
    wi = normalize(add(add(muls(tangent, hx), muls(bitangent, hy)), muls(n, hz)));
    pdf = (float)((double)glm_max(0.0f, dot(n, wi)) * 0.31830988618379067154);
}

} // namespace cr
