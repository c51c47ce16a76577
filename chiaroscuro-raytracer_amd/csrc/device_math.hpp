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
// Same double-precision evaluation as oracle/oracle.c cr_sincosf.
__device__ __forceinline__ void cr_sincosf(float xf, float &s, float &c) {
    const double PIO2_1 = 1.57079632673412561417e+00, PIO2_1T = 6.07710050650619224932e-11;
    const double TWO_OVER_PI = 6.36619772367581382433e-01;
    double x = (double)xf;
    double k = floor(x * TWO_OVER_PI + 0.5);
    int q = (int)k;
    double r = (x - k * PIO2_1) - k * PIO2_1T;
    double r2 = r * r;
    double ps = 1.0 / 355687428096000.0;
    ps = -1.0 / 1307674368000.0 + r2 * ps;
    ps = 1.0 / 6227020800.0 + r2 * ps;
    ps = -1.0 / 39916800.0 + r2 * ps;
    ps = 1.0 / 362880.0 + r2 * ps;
    ps = -1.0 / 5040.0 + r2 * ps;
    ps = 1.0 / 120.0 + r2 * ps;
    ps = -1.0 / 6.0 + r2 * ps;
    double sv = r + r * (r2 * ps);
    double pc = 1.0 / 6402373705728000.0;
    pc = -1.0 / 20922789888000.0 + r2 * pc;
    pc = 1.0 / 87178291200.0 + r2 * pc;
    pc = -1.0 / 479001600.0 + r2 * pc;
    pc = 1.0 / 3628800.0 + r2 * pc;
    pc = -1.0 / 40320.0 + r2 * pc;
    pc = 1.0 / 720.0 + r2 * pc;
    pc = -1.0 / 24.0 + r2 * pc;
    pc = 1.0 / 2.0 + r2 * pc;
    double cv = 1.0 - r2 * pc;
    double S, C;
    switch (q & 3) {
    case 0: S = sv; C = cv; break;
    case 1: S = cv; C = -sv; break;
    case 2: S = -sv; C = -cv; break;
    default: S = -cv; C = sv; break;
    }
    s = (float)S;
    c = (float)C;
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
