// render_common.hpp -- device pieces shared by every render / query kernel.
#pragma once
#include "device_math.hpp"
#include "kernels.hpp"

namespace cr {

// Query counters (cr_counters order).  Per-lane by default; the persistent kernel
// keeps the per-query ones as wave-uniform tallies taken with __ballot at
// converged points (flush_counters' `uniform` bit i set -> field i is a wave total).
struct Ctr {
    uint32_t closest = 0, shadow = 0, inner = 0, leaf = 0, tritest = 0, hit = 0, texhit = 0, paths = 0, pixels = 0;
    uint32_t wave_desc = 0, wave_tri = 0, wave_round = 0, wave_query = 0; // diagnostics, see chiaro_hip.h
    uint32_t wave_desc_uniform = 0, wave_tri_uniform = 0;
    uint32_t wave_desc_lines = 0, wave_tri_lines = 0;
    uint32_t leaf_rounds = 0, leaf_distinct = 0, leaf_records = 0, leaf_fit21 = 0, leaf_fit56 = 0;
};
__device__ __forceinline__ uint32_t wave_count(bool pred) { return (uint32_t)__popcll(__ballot(pred)); }
// The lane's index in its wave, recomputed at every use (two VALU; volatile: never hoisted or shared),
// so the trace kernels' persistent loops hold no register with threadIdx.x (at 64 VGPRs it was spilled).
__device__ __forceinline__ uint32_t lane_id() {
    uint32_t l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}
// True in exactly one active lane (the lowest): `if (wave_leader()) n++` counts
// iterations of the enclosing (possibly divergent) loop as the WAVE executes them.
__device__ __forceinline__ bool wave_leader() {
    return lane_id() == (uint32_t)(__ffsll((long long)__ballot(1)) - 1);
}

// Call with the whole wave converged.
__device__ __forceinline__ void flush_counters(unsigned long long *ctrs, const Ctr &c, uint32_t uniform = 0u) {
    const uint32_t ln = lane_id();
    const uint32_t v[CTR_N] = {c.closest,   c.shadow,    c.inner,      c.leaf,       c.tritest,
                               c.hit,       c.texhit,    c.paths,      c.pixels,     c.wave_desc,
                               c.wave_tri,  c.wave_round, c.wave_query, c.wave_desc_uniform, c.wave_tri_uniform,
                               c.wave_desc_lines, c.wave_tri_lines, c.leaf_rounds, c.leaf_distinct,
                               c.leaf_records,    c.leaf_fit21,     c.leaf_fit56};
#pragma unroll
    for (int i = 0; i < CTR_N; i++) {
        unsigned long long s = v[i];
        if (!(uniform & (1u << i))) {
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1) s += __shfl_xor(s, off, 64);
        }
        if (ln == 0 && s) atomicAdd(&ctrs[i], s);
    }
}

// kdtree.cpp:196-208 slab test against the padded root box
// inv = the correctly rounded 1/d per axis (what the reference's 1.f/d gives).
__device__ __forceinline__ void ray_box_inv(const DevScene &S, f3 o, f3 inv, float &first, float &second) {
    const float dix = inv.x, diy = inv.y, diz = inv.z;
    const float txmin = (S.bmin.x - o.x) * dix, txmax = (S.bmax.x - o.x) * dix;
    const float tymin = (S.bmin.y - o.y) * diy, tymax = (S.bmax.y - o.y) * diy;
    const float tzmin = (S.bmin.z - o.z) * diz, tzmax = (S.bmax.z - o.z) * diz;
    first = std_max(std_max(std_min(txmin, txmax), std_min(tymin, tymax)), std_min(tzmin, tzmax));
    second = std_min(std_min(std_max(txmin, txmax), std_max(tymin, tymax)), std_max(tzmin, tzmax));
}
__device__ __forceinline__ void ray_box(const DevScene &S, f3 o, f3 d, float &first, float &second) {
    const float diy = 1.f / d.y, dix = 1.f / d.x, diz = 1.f / d.z;
    const float txmin = (S.bmin.x - o.x) * dix, txmax = (S.bmax.x - o.x) * dix;
    const float tymin = (S.bmin.y - o.y) * diy, tymax = (S.bmax.y - o.y) * diy;
    const float tzmin = (S.bmin.z - o.z) * diz, tzmax = (S.bmax.z - o.z) * diz;
    first = std_max(std_max(std_min(txmin, txmax), std_min(tymin, tymax)), std_min(tzmin, tzmax));
    second = std_min(std_min(std_max(txmin, txmax), std_max(tymin, tymax)), std_max(tzmin, tzmax));
}

// Moller-Trumbore, kdtree.cpp:219-246 / 293-320.  True when the reference would
// accept the triangle for a segment ending at tmax (0 <= t < tmax); ux, uy, t set then.
// The early returns are kept: neighbouring lanes often test the same triangle
// (coherent camera rays), and a wave-uniform rejection skips the rest (measured:
// a branch-free form was 10% slower on the sponza stand-in).  f = RN(1/aa) as
// the reference's 1.f/a, by rcp_rn (exact, checked over every float in range).
struct TriRec {
    float4 a; // A, tri id bits
    float4 b; // e1
    float4 c; // e2
};
// 32-bit byte offset from the SGPR base (global_load saddr + voffset: one VGPR
// of address per lane, not two); cr_upload_scene keeps the records under 4 GiB.
__device__ __forceinline__ TriRec load_rec(const DevScene &S, uint32_t ref) {
    const float4 *p = (const float4 *)((const char *)S.recs + (ref * (uint32_t)(16 * REC_STRIDE)));
    return TriRec{p[0], p[1], p[2]};
}
__device__ __forceinline__ uint32_t rec_id(const TriRec &r) { return __float_as_uint(r.a.w); }
__device__ __forceinline__ bool tri_test(f3 o, f3 d, const TriRec &r, float tmax, float &ux, float &uy, float &t) {
    const f3 v0 = ld3(r.a), e1 = ld3(r.b), e2 = ld3(r.c);
    const f3 p = cross(d, e2);
    const float aa = dot(e1, p);
    if (aa < 1.19209290e-7F && aa > -1.19209290e-7F) return false;
    const float f = rcp_rn(aa);
    const f3 sv = sub(o, v0);
    ux = f * dot(sv, p);
    if (ux < 0.f || ux > 1.f) return false;
    const f3 q = cross(sv, e1);
    uy = f * dot(d, q);
    if (uy < 0.f || uy + ux > 1.f) return false;
    t = f * dot(e2, q);
    return t >= 0.f && t < tmax;
}

// tri_test with the scalar unit in mind (BF trace builds): the early exits are
// wave-uniform (taken when no active lane can still accept) and the lanes that
// already failed compute on, masked by `ok`, so no exec-mask bookkeeping runs per
// test.  Same values, same acceptance.  live: false for a lane with no test (it never accepts).
__device__ __forceinline__ bool tri_test_wave(f3 o, f3 d, const TriRec &r, float tmax, float &ux, float &uy,
                                              float &t, bool live = true) {
    const f3 v0 = ld3(r.a), e1 = ld3(r.b), e2 = ld3(r.c);
    const f3 p = cross(d, e2);
    const float aa = dot(e1, p);
    // (bitwise logic on the lane masks: no short-circuit exec branches)
    bool ok = live & !((aa < 1.19209290e-7F) & (aa > -1.19209290e-7F));
    if (!__ballot(ok)) return false;
    const float f = rcp_rn_wave(aa);
    const f3 sv = sub(o, v0);
    ux = f * dot(sv, p);
    ok = ok & !((ux < 0.f) | (ux > 1.f));
    if (!__ballot(ok)) return false;
    const f3 q = cross(sv, e1);
    uy = f * dot(d, q);
    ok = ok & !((uy < 0.f) | (uy + ux > 1.f));
    if (!__ballot(ok)) return false;
    t = f * dot(e2, q);
    return ok & (t >= 0.f) & (t < tmax);
}

// tsplit = (split - oa) / da of a kd node (kdtree.cpp:266), correctly rounded.
__device__ __forceinline__ float split_distance(float split, float oa, float da) { return (split - oa) / da; }

// src/mesh.cpp:21-35 Texture::getColorAt (texture padded with zeros past its end)
__device__ __forceinline__ f3 tex_lookup(const DevScene &S, int ti, float u, float v) {
    const uint4 t = S.texs[ti];
    const int w = (int)t.x, h = (int)t.y, nc = (int)t.z;
    // The reference loops forever on +-inf; bound the loops so a bad uv cannot hang the GPU.
    for (int i = 0; u > 1.f && i < (1 << 24); i++) u -= 1.f;
    for (int i = 0; u < 0.f && i < (1 << 24); i++) u += 1.f;
    for (int i = 0; v > 1.f && i < (1 << 24); i++) v -= 1.f;
    for (int i = 0; v < 0.f && i < (1 << 24); i++) v += 1.f;
    int x = (int)(u * (float)w);
    int y = (int)(v * (float)h);
    long idx = ((long)y * w + x) * nc;
    const long lim = (long)w * h * nc + (long)tex_pad(w, nc); // bytes incl. zero pad
    if (idx < 0 || idx + 3 > lim) idx = lim - 3 - nc;         // unreachable for finite uv
    const uint8_t *px = S.texels + t.w + idx;
    return mk((float)px[0] * 0.00392156862f, (float)px[1] * 0.00392156862f, (float)px[2] * 0.00392156862f);
}

// sxy: the sample's screen position (sx, sy), which the direction is affine in (camcull.hpp)
__device__ __forceinline__ f3 camera_dir(const RenderArgs &A, uint32_t x, uint32_t y, Rng &rng,
                                         float2 *sxy = nullptr) {
    const f3 lu = mk(A.cam[3], A.cam[4], A.cam[5]), dx = mk(A.cam[6], A.cam[7], A.cam[8]),
             dy = mk(A.cam[9], A.cam[10], A.cam[11]);
    // rayTracer.cpp:61 -- the y-jitter draw is evaluated first (g++ order)
    const float uy = rng_uniform(rng, 0.f, 1.f);
    const float ux = rng_uniform(rng, 0.f, 1.f);
    const float sx = (float)x + ux, sy = (float)y + uy;
    if (sxy) *sxy = make_float2(sx, sy);
    return add(add(lu, muls(dx, sx)), muls(dy, sy));
}

// Work item -> pixel: this rank's tiles (slot s -> rank s % nranks), row-major in a tile.
__device__ __forceinline__ bool item_pixel(const RenderArgs &A, uint32_t item, uint32_t &x, uint32_t &y) {
    const uint32_t T = A.tile, TT = A.tile * A.tile;
    const uint32_t lt = item / TT, o = item - lt * TT;
    const uint32_t s = A.rank + lt * A.nranks;
    const uint32_t gy = s / A.tiles_x, gx = tile_slot_column(s, A.tiles_x, A.nranks);
    x = gx * T + (o % T);
    y = gy * T + (o / T);
    return x < A.xres && y < A.yres;
}

// The RNG stream of a path: pixel and sample s of this pass, which holds A.nl layers' samples as
// one run per item (s / spp = the layer's offset from A.layer); A.nl = 1: the layer itself.
__device__ __forceinline__ Rng path_rng(const RenderArgs &A, uint32_t pixel, uint32_t s) {
    const uint32_t j = A.nl > 1 ? s / A.spp : 0u;
    return rng_make(A.seed, A.layer + j, pixel, s - j * A.spp);
}

// lj: the layer's offset in this pass (layer A.layer + lj)
__device__ __forceinline__ void write_pixel(const RenderArgs &A, uint32_t x, uint32_t y, uint32_t item, f3 temp,
                                            uint32_t lj = 0) {
    const float inv = 1.f / (float)A.spp;
    const uint32_t layer = A.layer + lj;
    if (A.mode == MODE_TILES) {
        const f3 m = muls(temp, inv);
        size_t slot = item;
        if (A.piece_m > 1) {
            const uint32_t TT = A.tile * A.tile, lt = item / TT;
            slot = (size_t)(A.piece_k + lt * A.piece_m) * TT + (item - lt * TT);
        }
        float *o = A.out + (size_t)lj * A.layer_stride + 3 * slot;
        o[0] = m.x;
        o[1] = m.y;
        o[2] = m.z;
    } else {
        float *o = A.out + 3 * ((size_t)y * A.xres + x);
        // rayTracer.cpp:64  (old * (L-1) + temp * invSamples) / L
        const f3 old = (layer > 1) ? mk(o[0], o[1], o[2]) : mk(0.f, 0.f, 0.f);
        const f3 nw = divs(add(muls(old, (float)(layer - 1)), muls(temp, inv)), (float)layer);
        o[0] = nw.x;
        o[1] = nw.y;
        o[2] = nw.z;
    }
}

// Hit reconstruction + emission + NEE set-up of one bounce: the part of
// RayTracer::sendRay (rayTracer.cpp:80-99) and intersectRayKDTree (137-169)
// before the shadow query.  Returns false when the scene has no light.
struct HitShade {
    f3 p, normal, fcol, direct;
    bool textured;
};
__device__ __forceinline__ HitShade shade_hit(const DevScene &S, f3 origin, uint32_t t, float bx, float by, int k) {
    HitShade h;
    const float4 nrm4 = S.mat_n[t];
    h.normal = ld3(nrm4);
    const float bz = (1.f - bx - by);
    h.p = add(add(muls(ld3(S.tri[3 * t]), bz), muls(ld3(S.tri[3 * t + 1]), bx)), muls(ld3(S.tri[3 * t + 2]), by));
    const float4 kd4 = S.mat_kd[t];
    f3 Kd = ld3(kd4);
    const int ti = __float_as_int(kd4.w);
    h.textured = ti >= 0;
    if (h.textured) {
        const float2 ua = S.mat_uv[3 * t], ub = S.mat_uv[3 * t + 1], uc = S.mat_uv[3 * t + 2];
        Kd = tex_lookup(S, ti, (ua.x * bz + ub.x * bx) + uc.x * by, (ua.y * bz + ub.y * bx) + uc.y * by);
    }
    h.fcol = muls(Kd, (float)0.31830988618379067154); // Diffuse::f = float(M_1_PI) * color, brdf.cpp:70
    const f3 wo = normalize(sub(origin, h.p));
    if (k > 1) {
        h.direct = mk(0.f, 0.f, 0.f);
    } else {
        const bool emissive = __float_as_uint(nrm4.w) != 0u;
        const f3 rad = emissive ? ld3(S.mat_ke[t]) : mk(0.f, 0.f, 0.f);
        h.direct = muls(rad, std_max(0.f, dot(wo, h.normal)));
    }
    return h;
}

// NEE light sample (rayTracer.cpp:91-109): picks the light, the point on it, and
// returns the shadow ray + the contribution added when it is not occluded.
struct Nee {
    f3 origin, dir, contrib;
    float distance;
    uint32_t light;
};
__device__ __forceinline__ Nee sample_light(const DevScene &S, f3 p, f3 normal, f3 fcol, Rng &rng) {
    Nee n;
    const uint32_t li = rng_index(rng, S.nlights);
    const uint2 L = S.lights[li];
    n.light = L.x;
    const float v0 = rng_uniform(rng, 0.f, 1.f);
    const float v1 = rng_uniform(rng, 0.f, 1.f - v0);
    const f3 lp = add(add(muls(ld3(S.tri[3 * n.light]), v0), muls(ld3(S.tri[3 * n.light + 1]), v1)),
                      muls(ld3(S.tri[3 * n.light + 2]), 1.f - v0 - v1));
    n.distance = distance3(p, lp);
    n.dir = normalize(sub(lp, p));
    n.origin = add(p, muls(normal, 0.001f));
    // the term does not depend on the shadow result; the reference evaluates it only when unoccluded
    const float geometric =
        std_max(0.f, dot(normal, n.dir) * dot(neg(n.dir), ld3(S.mat_n[n.light])) / (1.f + n.distance * n.distance));
    n.contrib = mul(muls(ld3(S.mat_ke[n.light]), geometric * __uint_as_float(L.y) * (float)S.nlights), fcol);
    return n;
}

} // namespace cr
