// kernels.hip -- CDNA4 (gfx950) kernels of the Chiaroscuro render loop.
//
// Hot path as one megakernel family:
//   camera sample (src/rayTracer.cpp:58-62) -> closest-hit kd traversal
//   (src/kdtree.cpp:210-281) -> hit reconstruction (src/rayTracer.cpp:137-169)
//   -> NEE light pick + shadow traversal (src/rayTracer.cpp:89-111,
//   src/kdtree.cpp:283-344) -> Diffuse::sample_wi + Russian roulette
//   (src/rayTracer.cpp:113-132, src/brdf.cpp:57-79) -> next bounce.
// The reference's recursion `direct + w * sendRay(...)` is evaluated back to
// front from per-bounce (direct, w) registers so the float result is identical.
//
// Layout in HBM (built by cabi.cpp):
//   nodes  : uint2 per kd node {split bits | first ref, axis | child<<2 (axis 3 = leaf, count<<2)}
//   recs   : 3 x float4 per leaf reference, leaf-ordered: {A, id}, {B-A}, {C-A}
//   tri    : 3 x float4 per triangle {A, B, C} (hit reconstruction only)
//   mat    : float4 normal (w: emissive flag), float4 Kd (w: texture index), float4 Ke, 3 x float2 uv
//   lights : uint2 {triangle id, surface bits}
// Traversal stack: LDS, [depth][thread] so every lane's push/pop hits its own bank.
#include "device_math.hpp"
#include "kernels.hpp"

namespace cr {

// Query counters (cr_counters order).  Per-lane by default; the persistent kernel
// keeps the per-query ones as wave-uniform tallies taken with __ballot at
// converged points (flag `uniform` bit i set -> field i is already a wave total).
struct Ctr {
    uint32_t closest = 0, shadow = 0, inner = 0, leaf = 0, tritest = 0, hit = 0, texhit = 0, paths = 0, pixels = 0;
};
__device__ __forceinline__ uint32_t wave_count(bool pred) { return (uint32_t)__popcll(__ballot(pred)); }

struct Stack {
    uint32_t *node;
    float *tmin;
    float *tmax;
    uint32_t stride; // = blockDim.x
};

// kdtree.cpp:196-208 slab test against the padded root box
__device__ __forceinline__ void ray_box(const DevScene &S, f3 o, f3 d, float &first, float &second) {
    const float diy = 1.f / d.y, dix = 1.f / d.x, diz = 1.f / d.z;
    const float txmin = (S.bmin.x - o.x) * dix, txmax = (S.bmax.x - o.x) * dix;
    const float tymin = (S.bmin.y - o.y) * diy, tymax = (S.bmax.y - o.y) * diy;
    const float tzmin = (S.bmin.z - o.z) * diz, tzmax = (S.bmax.z - o.z) * diz;
    first = std_max(std_max(std_min(txmin, txmax), std_min(tymin, tymax)), std_min(tzmin, tzmax));
    second = std_min(std_min(std_max(txmin, txmax), std_max(tymin, tymax)), std_max(tzmin, tzmax));
}

// Unified kd traversal.
//   closest (shadow=false): KDTree::intersectRay, src/kdtree.cpp:210-281 -- first
//     leaf (near-to-far, stack-emulated recursion) holding an accepted hit ends it.
//   shadow  (shadow=true):  KDTree::intersectShadowRay, src/kdtree.cpp:283-344 --
//     any accepted triangle other than `exclude` ends it.
// Both accept 0 <= t < segment tmax (kdtree.cpp:255, 319).
template <bool SHADOW>
__device__ __forceinline__ bool traverse(const DevScene &S, const Stack &stk, f3 o, f3 d, float limit,
                                         uint32_t exclude, uint32_t &tri, float &bx, float &by, float &dist,
                                         Ctr &c) {
    float tmin, tmax;
    ray_box(S, o, d, tmin, tmax);
    if (SHADOW) {
        if (tmax < 0 || tmax < tmin || tmin > limit) return false;
        tmax = std_min(tmax, limit);
    } else {
        if (tmax < 0 || tmax < tmin) return false;
    }
    const uint32_t tid = threadIdx.x;
    uint32_t sp = 0;
    uint32_t node = 0;
    for (;;) {
        uint2 nd = S.nodes[node];
        while ((nd.y & 3u) != 3u) {
            c.inner++;
            const uint32_t a = nd.y & 3u;
            const float split = __uint_as_float(nd.x);
            const float oa = comp(o, a), da = comp(d, a);
            const float tsplit = (split - oa) / da;
            const uint32_t below = (oa < split) || (oa == split && da <= 0);
            const uint32_t child = nd.y >> 2;
            if (tsplit >= tmax || tsplit < 0) {
                node = child + (1u - below);
            } else if (tsplit <= tmin) {
                node = child + below;
            } else {
                stk.node[sp * stk.stride + tid] = child + below;
                stk.tmin[sp * stk.stride + tid] = tsplit;
                stk.tmax[sp * stk.stride + tid] = tmax;
                sp++;
                node = child + (1u - below);
                tmax = tsplit;
            }
            nd = S.nodes[node];
        }
        // leaf
        c.leaf++;
        const uint32_t first = nd.x, count = nd.y >> 2;
        bool found = false;
        for (uint32_t j = 0; j < count; j++) {
            const float4 r0 = S.recs[3 * (first + j)];
            const uint32_t id = __float_as_uint(r0.w);
            if (SHADOW && id == exclude) continue;
            c.tritest++;
            // kdtree.cpp:219-246 Moller-Trumbore
            const f3 v0 = ld3(r0);
            const f3 e1 = ld3(S.recs[3 * (first + j) + 1]);
            const f3 e2 = ld3(S.recs[3 * (first + j) + 2]);
            const f3 p = cross(d, e2);
            const float aa = dot(e1, p);
            if (aa < 1.19209290e-7F && aa > -1.19209290e-7F) continue;
            const float f = 1.f / aa;
            const f3 sv = sub(o, v0);
            const float ux = f * dot(sv, p);
            if (ux < 0.f || ux > 1.f) continue;
            const f3 q = cross(sv, e1);
            const float uy = f * dot(d, q);
            if (uy < 0.f || uy + ux > 1.f) continue;
            const float t = f * dot(e2, q);
            if (t >= 0.f && t < tmax) {
                if (SHADOW) return true;
                bx = ux;
                by = uy;
                tmax = t;
                tri = id;
                found = true;
            }
        }
        if (!SHADOW && found) {
            dist = tmax;
            return true;
        }
        if (sp == 0) return false;
        sp--;
        node = stk.node[sp * stk.stride + tid];
        tmin = stk.tmin[sp * stk.stride + tid];
        tmax = stk.tmax[sp * stk.stride + tid];
    }
}

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
    const long lim = (long)w * h * nc + (long)(w + 1) * nc + 4; // bytes incl. zero pad (TEX_PAD)
    if (idx < 0 || idx + 3 > lim) idx = lim - 3 - nc;        // unreachable for finite in-range uv
    const uint8_t *px = S.texels + t.w + idx;
    return mk((float)px[0] * 0.00392156862f, (float)px[1] * 0.00392156862f, (float)px[2] * 0.00392156862f);
}

__device__ __forceinline__ f3 camera_dir(const RenderArgs &A, uint32_t x, uint32_t y, Rng &rng) {
    const f3 lu = mk(A.cam[3], A.cam[4], A.cam[5]), dx = mk(A.cam[6], A.cam[7], A.cam[8]),
             dy = mk(A.cam[9], A.cam[10], A.cam[11]);
    // rayTracer.cpp:61 -- the y-jitter draw is evaluated first (g++ order)
    const float uy = rng_uniform(rng, 0.f, 1.f);
    const float ux = rng_uniform(rng, 0.f, 1.f);
    return add(add(lu, muls(dx, (float)x + ux)), muls(dy, (float)y + uy));
}

// One camera path; RayTracer::sendRay (src/rayTracer.cpp:76-135) unrolled.
template <int MAXK>
__device__ f3 trace_path(const RenderArgs &A, const Stack &stk, uint32_t x, uint32_t y, uint32_t sample, Ctr &c) {
    const DevScene &S = A.S;
    Rng rng = rng_make(A.seed, A.layer, y * A.xres + x, sample);
    f3 origin = mk(A.cam[0], A.cam[1], A.cam[2]);
    f3 dir = camera_dir(A, x, y, rng);
    f3 D[MAXK], W[MAXK];
    int k = 1;
    f3 tail;
    c.paths++;
    for (;;) {
        uint32_t t = 0;
        float bx = 0.f, by = 0.f, dist = 0.f;
        c.closest++;
        if (!traverse<false>(S, stk, origin, dir, 0.f, 0xffffffffu, t, bx, by, dist, c)) {
            tail = mk(A.bg[0], A.bg[1], A.bg[2]);
            break;
        }
        c.hit++;
        // intersectRayKDTree, rayTracer.cpp:145-166
        const float4 nrm4 = S.mat_n[t];
        const f3 normal = ld3(nrm4);
        const float bz = (1.f - bx - by);
        const f3 p = add(add(muls(ld3(S.tri[3 * t]), bz), muls(ld3(S.tri[3 * t + 1]), bx)),
                         muls(ld3(S.tri[3 * t + 2]), by));
        const float4 kd4 = S.mat_kd[t];
        f3 Kd = ld3(kd4);
        const int ti = __float_as_int(kd4.w);
        if (ti >= 0) {
            const float2 ua = S.mat_uv[3 * t], ub = S.mat_uv[3 * t + 1], uc = S.mat_uv[3 * t + 2];
            Kd = tex_lookup(S, ti, (ua.x * bz + ub.x * bx) + uc.x * by, (ua.y * bz + ub.y * bx) + uc.y * by);
            c.texhit++;
        }
        const bool emissive = __float_as_uint(nrm4.w) != 0u;
        const f3 fcol = muls(Kd, (float)0.31830988618379067154); // Diffuse::f, brdf.cpp:70
        const f3 wo = normalize(sub(origin, p));
        f3 direct;
        if (k > 1) {
            direct = mk(0.f, 0.f, 0.f);
        } else {
            const f3 rad = emissive ? ld3(S.mat_ke[t]) : mk(0.f, 0.f, 0.f);
            direct = muls(rad, std_max(0.f, dot(wo, normal)));
        }
        if (S.nlights) {
            const uint32_t li = rng_index(rng, S.nlights);
            const uint2 L = S.lights[li];
            const uint32_t lid = L.x;
            const float v0 = rng_uniform(rng, 0.f, 1.f);
            const float v1 = rng_uniform(rng, 0.f, 1.f - v0);
            const f3 lp = add(add(muls(ld3(S.tri[3 * lid]), v0), muls(ld3(S.tri[3 * lid + 1]), v1)),
                              muls(ld3(S.tri[3 * lid + 2]), 1.f - v0 - v1));
            const float distance = distance3(p, lp);
            const f3 wl = normalize(sub(lp, p));
            c.shadow++;
            uint32_t dt;
            float d0, d1, d2;
            if (!traverse<true>(S, stk, add(p, muls(normal, 0.001f)), wl, distance, lid, dt, d0, d1, d2, c)) {
                const float geometric = std_max(
                    0.f, dot(normal, wl) * dot(neg(wl), ld3(S.mat_n[lid])) / (1.f + distance * distance));
                direct = add(direct,
                             mul(muls(ld3(S.mat_ke[lid]), geometric * __uint_as_float(L.y) * (float)S.nlights), fcol));
            }
        }
        if (k == A.K) {
            tail = direct;
            break;
        }
        const float sx = rng_uniform(rng, -1.f, 1.f);
        const float sy = rng_uniform(rng, -1.f, 1.f);
        f3 wi;
        float pdf;
        sample_wi(normal, sx, sy, wi, pdf);
        const float Kmax = std_max(std_max(fcol.x, fcol.y), fcol.z);
        if (pdf == 0.f || rng_uniform(rng, 0.f, 1.f) > Kmax) {
            tail = direct;
            break;
        }
        const float cosine = fabsf(dot(normal, wi));
        const f3 w = divs(muls(fcol, cosine), pdf * Kmax);
#pragma unroll
        for (int j = 0; j < MAXK; j++)
            if (j == k - 1) {
                D[j] = direct;
                W[j] = w;
            }
        origin = add(p, muls(normal, 0.001f));
        dir = wi;
        k++;
    }
    // back-to-front fold: r_j = D_j + W_j * r_{j+1}
    f3 acc = tail;
#pragma unroll
    for (int j = MAXK - 1; j >= 0; j--)
        if (j < k - 1) acc = add(D[j], mul(W[j], acc));
    return acc;
}

__device__ __forceinline__ bool item_pixel(const RenderArgs &A, uint32_t item, uint32_t &x, uint32_t &y,
                                           uint32_t &tile_slot) {
    const uint32_t T = A.tile, TT = A.tile * A.tile;
    const uint32_t lt = item / TT, o = item - lt * TT;
    const uint32_t gt = A.rank + lt * A.nranks;
    const uint32_t gy = gt / A.tiles_x, gx = gt - gy * A.tiles_x;
    x = gx * T + (o % T);
    y = gy * T + (o / T);
    tile_slot = item;
    return x < A.xres && y < A.yres;
}

__device__ __forceinline__ void write_pixel(const RenderArgs &A, uint32_t x, uint32_t y, uint32_t slot, f3 temp) {
    const float inv = 1.f / (float)A.spp;
    if (A.mode == MODE_TILES) {
        const f3 m = muls(temp, inv);
        float *o = A.out + 3 * (size_t)slot;
        o[0] = m.x;
        o[1] = m.y;
        o[2] = m.z;
    } else {
        float *o = A.out + 3 * ((size_t)y * A.xres + x);
        // rayTracer.cpp:64  (old * (L-1) + temp * invSamples) / L
        const f3 old = (A.layer > 1) ? mk(o[0], o[1], o[2]) : mk(0.f, 0.f, 0.f);
        const f3 nw = divs(add(muls(old, (float)(A.layer - 1)), muls(temp, inv)), (float)A.layer);
        o[0] = nw.x;
        o[1] = nw.y;
        o[2] = nw.z;
    }
}

// Call with the whole wave converged.  Fields whose bit is set in `uniform` are
// wave totals already; the others are summed over the 64 lanes.
__device__ __forceinline__ void flush_counters(unsigned long long *ctrs, const Ctr &c, uint32_t uniform = 0u) {
    const uint32_t v[9] = {c.closest, c.shadow, c.inner, c.leaf, c.tritest, c.hit, c.texhit, c.paths, c.pixels};
#pragma unroll
    for (int i = 0; i < 9; i++) {
        unsigned long long s = v[i];
        if (!(uniform & (1u << i))) {
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1) s += __shfl_xor(s, off, 64);
        }
        if ((threadIdx.x & 63) == 0 && s) atomicAdd(&ctrs[i], s);
    }
}

// ---------------------------------------------------------------------------
// Kernel 1: one thread per pixel, sample loop in the thread (the reference's
// loop nest, rayTracer.cpp:56-62).  Baseline for the persistent kernel.
template <int MAXK>
__global__ void __launch_bounds__(128) render_simple(RenderArgs A) {
    extern __shared__ uint32_t lds[];
    const uint32_t depth = A.stack_depth;
    Stack stk{lds, (float *)(lds + depth * blockDim.x), (float *)(lds + 2 * depth * blockDim.x), blockDim.x};
    Ctr c = {};
    const uint32_t item = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t x, y, slot;
    if (item < A.n_items && item_pixel(A, item, x, y, slot)) {
        f3 temp = mk(0.f, 0.f, 0.f);
        for (uint32_t s = 0; s < A.spp; s++) temp = add(temp, trace_path<MAXK>(A, stk, x, y, s, c));
        write_pixel(A, x, y, slot, temp);
        c.pixels++;
    }
    flush_counters(A.counters, c);
}

// ---------------------------------------------------------------------------
// Kernel 0: persistent waves with per-lane path regeneration.
//
// Every lane owns one pixel at a time and runs its samples one after another
// (so the per-pixel sum keeps the reference's sample order), but a lane never
// waits for the rest of its wave between queries: each outer iteration every live
// lane runs exactly one kd query -- a camera/bounce ray (closest hit) or a NEE
// shadow ray (any hit) -- in ONE traversal loop, then advances its own path state
// machine (shade / start shadow ray / bounce / finish sample / next pixel).
// Pixels are handed out wave-wide: one atomicAdd per refill, lanes ranked by
// __ballot + mbcnt.
//
// Traversal stack: 8-byte entries {far node, tmax}.  The far child's tmin is the
// current tmax at pop time (it always equals the split distance stored implicitly
// -- see DESIGN.md "stack invariant"), so the reference's (node, tmin, tmax)
// recursion state fits in half the bytes.  The top R entries live in an LDS ring
// laid out [slot][thread] (each lane on its own bank pair); deeper entries spill
// to a per-lane global overflow area.
// Per-bounce (direct, w) pairs for the back-to-front fold go to a per-lane global
// buffer instead of registers, keeping the VGPR budget for occupancy.
enum : uint32_t { ST_NEED_PIXEL = 0, ST_NEW_SAMPLE = 1, ST_CLOSEST = 2, ST_SHADOW = 3, ST_DONE = 4 };

template <int R, bool FULL>
__device__ __forceinline__ bool traverse_ring(const DevScene &S, uint2 *ring, uint2 *gstk, uint32_t gstride,
                                              uint32_t gid, f3 o, f3 d, bool shadow, float limit, uint32_t exclude,
                                              uint32_t &tri, float &bx, float &by, Ctr &c) {
    float tmin, tmax;
    ray_box(S, o, d, tmin, tmax);
    if (shadow) {
        if (tmax < 0 || tmax < tmin || tmin > limit) return false;
        tmax = std_min(tmax, limit);
    } else {
        if (tmax < 0 || tmax < tmin) return false;
    }
    const uint32_t bdim = blockDim.x, tid = threadIdx.x;
    uint32_t sp = 0, nl = 0, node = 0;
    for (;;) {
        uint2 nd = S.nodes[node];
        while ((nd.y & 3u) != 3u) {
            if (FULL) c.inner++;
            const uint32_t a = nd.y & 3u;
            const float split = __uint_as_float(nd.x);
            const float oa = comp(o, a), da = comp(d, a);
            const float tsplit = (split - oa) / da;
            const uint32_t below = (oa < split) || (oa == split && da <= 0);
            const uint32_t child = nd.y >> 2;
            if (tsplit >= tmax || tsplit < 0) {
                node = child + (1u - below);
            } else if (tsplit <= tmin) {
                node = child + below;
            } else {
                const uint2 e = make_uint2(child + below, __float_as_uint(tmax));
                const uint32_t slot = (sp & (R - 1)) * bdim + tid;
                if (nl == R) gstk[(size_t)(sp - R) * gstride + gid] = ring[slot]; // spill the oldest
                else nl++;
                ring[slot] = e;
                sp++;
                node = child + (1u - below);
                tmax = tsplit;
            }
            nd = S.nodes[node];
        }
        if (FULL) c.leaf++;
        const uint32_t first = nd.x, count = nd.y >> 2;
        bool found = false;
        for (uint32_t j = 0; j < count; j++) {
            const float4 r0 = S.recs[3 * (first + j)];
            const float4 r1 = S.recs[3 * (first + j) + 1];
            const float4 r2 = S.recs[3 * (first + j) + 2];
            const uint32_t id = __float_as_uint(r0.w);
            if (shadow && id == exclude) continue;
            if (FULL) c.tritest++;
            const f3 v0 = ld3(r0), e1 = ld3(r1), e2 = ld3(r2);
            const f3 p = cross(d, e2);
            const float aa = dot(e1, p);
            if (aa < 1.19209290e-7F && aa > -1.19209290e-7F) continue;
            const float f = 1.f / aa;
            const f3 sv = sub(o, v0);
            const float ux = f * dot(sv, p);
            if (ux < 0.f || ux > 1.f) continue;
            const f3 q = cross(sv, e1);
            const float uy = f * dot(d, q);
            if (uy < 0.f || uy + ux > 1.f) continue;
            const float t = f * dot(e2, q);
            if (t >= 0.f && t < tmax) {
                if (shadow) return true;
                bx = ux;
                by = uy;
                tmax = t;
                tri = id;
                found = true;
            }
        }
        if (found) return true;
        if (sp == 0) return false;
        sp--;
        uint2 e;
        if (nl) {
            e = ring[(sp & (R - 1)) * bdim + tid];
            nl--;
        } else {
            e = gstk[(size_t)sp * gstride + gid];
        }
        node = e.x;
        tmin = tmax; // == split distance of the popped entry (stack invariant)
        tmax = __uint_as_float(e.y);
    }
}

template <int R, bool FULL>
__global__ void __launch_bounds__(256) render_persistent(RenderArgs A) {
    extern __shared__ uint2 ring_lds[];
    const DevScene &S = A.S;
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t lane = threadIdx.x & 63u;
    const f3 eye = mk(A.cam[0], A.cam[1], A.cam[2]);
    Ctr c = {};

    uint32_t state = ST_NEED_PIXEL;
    uint32_t px = 0, py = 0, slot = 0, s = 0;
    f3 temp = mk(0.f, 0.f, 0.f);
    Rng rng{0u, 0u};
    int k = 1;
    f3 o = eye, d = mk(0.f, 0.f, 1.f);
    float limit = 0.f;
    uint32_t exclude = 0xffffffffu;
    f3 p = mk(0.f, 0.f, 0.f), normal = p, fcol = p, direct = p, contrib = p;

    for (;;) {
        // ---- wave-wide pixel refill (ballot + mbcnt ranks, one atomic per refill)
        for (;;) {
            const uint64_t need = __ballot(state == ST_NEED_PIXEL);
            if (!need) break;
            const uint32_t n = (uint32_t)__popcll(need);
            const uint32_t leader = (uint32_t)__ffsll((long long)need) - 1u;
            uint32_t base = 0;
            if (lane == leader) base = atomicAdd(A.work, n);
            base = __shfl(base, (int)leader, 64);
            if (state == ST_NEED_PIXEL) {
                const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(need >> 32),
                                                                __builtin_amdgcn_mbcnt_lo((uint32_t)need, 0u));
                const uint32_t item = base + rank;
                if (item >= A.n_items) {
                    state = ST_DONE;
                } else if (item_pixel(A, item, px, py, slot)) {
                    state = ST_NEW_SAMPLE;
                    s = 0;
                    temp = mk(0.f, 0.f, 0.f);
                } // else: partial-tile pixel outside the image, fetch again
            }
        }
        c.paths += wave_count(state == ST_NEW_SAMPLE);
        if (state == ST_NEW_SAMPLE) {
            rng = rng_make(A.seed, A.layer, py * A.xres + px, s);
            o = eye;
            d = camera_dir(A, px, py, rng);
            k = 1;
            state = ST_CLOSEST;
        }
        if (!__any(state != ST_DONE)) break;

        // ---- one kd query per live lane
        const bool shadow = state == ST_SHADOW;
        c.shadow += wave_count(shadow);
        c.closest += wave_count(state == ST_CLOSEST);
        uint32_t t = 0;
        float bx = 0.f, by = 0.f;
        bool h = false;
        if (state == ST_CLOSEST || state == ST_SHADOW)
            h = traverse_ring<R, FULL>(S, ring_lds, A.gstack, A.gstride, gid, o, d, shadow, limit, exclude, t, bx, by, c);
        c.hit += wave_count(state == ST_CLOSEST && h);

        // ---- advance the path state machine (RayTracer::sendRay, rayTracer.cpp:76-135)
        bool bounce = false, finish = false, textured = false, pixel_done = false;
        f3 tail = mk(0.f, 0.f, 0.f);
        if (state == ST_SHADOW) {
            if (!h) direct = add(direct, contrib);
            bounce = true;
        } else if (state == ST_CLOSEST) {
            if (!h) {
                tail = mk(A.bg[0], A.bg[1], A.bg[2]);
                finish = true;
            } else {
                const float4 nrm4 = S.mat_n[t];
                normal = ld3(nrm4);
                const float bz = (1.f - bx - by);
                p = add(add(muls(ld3(S.tri[3 * t]), bz), muls(ld3(S.tri[3 * t + 1]), bx)),
                        muls(ld3(S.tri[3 * t + 2]), by));
                const float4 kd4 = S.mat_kd[t];
                f3 Kd = ld3(kd4);
                const int ti = __float_as_int(kd4.w);
                if (ti >= 0) {
                    const float2 ua = S.mat_uv[3 * t], ub = S.mat_uv[3 * t + 1], uc = S.mat_uv[3 * t + 2];
                    Kd = tex_lookup(S, ti, (ua.x * bz + ub.x * bx) + uc.x * by, (ua.y * bz + ub.y * bx) + uc.y * by);
                    textured = true;
                }
                fcol = muls(Kd, (float)0.31830988618379067154);
                const f3 wo = normalize(sub(o, p));
                if (k > 1) {
                    direct = mk(0.f, 0.f, 0.f);
                } else {
                    const bool emissive = __float_as_uint(nrm4.w) != 0u;
                    const f3 rad = emissive ? ld3(S.mat_ke[t]) : mk(0.f, 0.f, 0.f);
                    direct = muls(rad, std_max(0.f, dot(wo, normal)));
                }
                if (S.nlights) {
                    const uint32_t li = rng_index(rng, S.nlights);
                    const uint2 L = S.lights[li];
                    const uint32_t lid = L.x;
                    const float v0 = rng_uniform(rng, 0.f, 1.f);
                    const float v1 = rng_uniform(rng, 0.f, 1.f - v0);
                    const f3 lp = add(add(muls(ld3(S.tri[3 * lid]), v0), muls(ld3(S.tri[3 * lid + 1]), v1)),
                                      muls(ld3(S.tri[3 * lid + 2]), 1.f - v0 - v1));
                    const float distance = distance3(p, lp);
                    const f3 wl = normalize(sub(lp, p));
                    // the NEE term does not depend on the shadow result: evaluate it now
                    const float geometric = std_max(
                        0.f, dot(normal, wl) * dot(neg(wl), ld3(S.mat_n[lid])) / (1.f + distance * distance));
                    contrib = mul(muls(ld3(S.mat_ke[lid]), geometric * __uint_as_float(L.y) * (float)S.nlights), fcol);
                    o = add(p, muls(normal, 0.001f));
                    d = wl;
                    limit = distance;
                    exclude = lid;
                    state = ST_SHADOW;
                } else {
                    bounce = true;
                }
            }
        }
        if (bounce) {
            if (k == A.K) {
                tail = direct;
                finish = true;
            } else {
                const float sx = rng_uniform(rng, -1.f, 1.f);
                const float sy = rng_uniform(rng, -1.f, 1.f);
                f3 wi;
                float pdf;
                sample_wi(normal, sx, sy, wi, pdf);
                const float Kmax = std_max(std_max(fcol.x, fcol.y), fcol.z);
                if (pdf == 0.f || rng_uniform(rng, 0.f, 1.f) > Kmax) {
                    tail = direct;
                    finish = true;
                } else {
                    const float cosine = fabsf(dot(normal, wi));
                    const f3 w = divs(muls(fcol, cosine), pdf * Kmax);
                    A.pathbuf[(size_t)(2 * (k - 1)) * A.gstride + gid] = make_float4(direct.x, direct.y, direct.z, 0.f);
                    A.pathbuf[(size_t)(2 * (k - 1) + 1) * A.gstride + gid] = make_float4(w.x, w.y, w.z, 0.f);
                    o = add(p, muls(normal, 0.001f));
                    d = wi;
                    k++;
                    state = ST_CLOSEST;
                }
            }
        }
        if (finish) {
            f3 acc = tail; // back-to-front fold r_j = D_j + W_j * r_{j+1}
            for (int j = k - 2; j >= 0; j--) {
                const float4 Dj = A.pathbuf[(size_t)(2 * j) * A.gstride + gid];
                const float4 Wj = A.pathbuf[(size_t)(2 * j + 1) * A.gstride + gid];
                acc = add(ld3(Dj), mul(ld3(Wj), acc));
            }
            temp = add(temp, acc);
            s++;
            if (s == A.spp) {
                write_pixel(A, px, py, slot, temp);
                pixel_done = true;
                state = ST_NEED_PIXEL;
            } else {
                state = ST_NEW_SAMPLE;
            }
        }
        c.texhit += wave_count(textured);
        c.pixels += wave_count(pixel_done);
    }
    // closest, shadow, hit, texhit, paths, pixels are wave tallies
    flush_counters(A.counters, c, (1u << 0) | (1u << 1) | (1u << 5) | (1u << 6) | (1u << 7) | (1u << 8));
}

// ---------------------------------------------------------------------------
// Ray-query kernels (cr_intersect / cr_intersect_shadow)
__global__ void __launch_bounds__(128) intersect_kernel(QueryArgs Q) {
    extern __shared__ uint32_t lds[];
    const uint32_t depth = Q.stack_depth;
    Stack stk{lds, (float *)(lds + depth * blockDim.x), (float *)(lds + 2 * depth * blockDim.x), blockDim.x};
    Ctr c = {};
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < Q.n) {
        const f3 o = mk(Q.orig[3 * i], Q.orig[3 * i + 1], Q.orig[3 * i + 2]);
        const f3 d = mk(Q.dir[3 * i], Q.dir[3 * i + 1], Q.dir[3 * i + 2]);
        uint32_t t = 0;
        float bx = 0.f, by = 0.f, ds = 0.f;
        if (Q.shadow) {
            c.shadow++;
            Q.hit[i] = traverse<true>(Q.S, stk, o, d, Q.dist[i], Q.light[i], t, bx, by, ds, c) ? 1u : 0u;
        } else {
            c.closest++;
            const bool h = traverse<false>(Q.S, stk, o, d, 0.f, 0xffffffffu, t, bx, by, ds, c);
            Q.hit[i] = h ? 1u : 0u;
            if (h) {
                c.hit++;
                Q.tri[i] = t;
                Q.bary[2 * i] = bx;
                Q.bary[2 * i + 1] = by;
                Q.dist_out[i] = ds;
            }
        }
    }
    flush_counters(Q.counters, c);
}

// Root-side unpermute + progressive blend of gathered tile buffers.
__global__ void __launch_bounds__(256) blend_tiles_kernel(BlendArgs B) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; // pixel in frame
    if (i >= B.xres * B.yres) return;
    const uint32_t y = i / B.xres, x = i - y * B.xres;
    const uint32_t T = B.tile;
    const uint32_t gt = (y / T) * B.tiles_x + (x / T);
    const uint32_t r = gt % B.nranks, lt = gt / B.nranks;
    const size_t src = ((size_t)r * B.max_tiles + lt) * T * T + (y % T) * T + (x % T);
    const f3 m = mk(B.gathered[3 * src], B.gathered[3 * src + 1], B.gathered[3 * src + 2]);
    float *o = B.frame + 3 * (size_t)i;
    const f3 old = (B.layer > 1) ? mk(o[0], o[1], o[2]) : mk(0.f, 0.f, 0.f);
    // rayTracer.cpp:64 with mean = temp * invSamples already applied by the rank
    const f3 nw = divs(add(muls(old, (float)(B.layer - 1)), m), (float)B.layer);
    o[0] = nw.x;
    o[1] = nw.y;
    o[2] = nw.z;
}

// ---------------------------------------------------------------- launch --
static const int RING = 8; // LDS ring entries per lane (8 B each)

void persistent_geometry(int num_cus, uint32_t waves_per_cu, uint32_t &block, uint32_t &blocks) {
    block = 256;
    if (waves_per_cu == 0) waves_per_cu = 24;
    blocks = (uint32_t)(num_cus > 0 ? num_cus : 256) * ((waves_per_cu * 64 + block - 1) / block);
}

int launch_render(const RenderArgs &A, int kernel, uint32_t block, uint32_t waves_per_cu, int num_cus,
                  hipStream_t st) {
    if (kernel == 0) {
        uint32_t blk, blocks;
        persistent_geometry(num_cus, waves_per_cu, blk, blocks);
        if (A.gstride < blk * blocks) return (int)hipErrorInvalidValue;
        const size_t lds = (size_t)RING * blk * sizeof(uint2);
        if (A.full_counters)
            hipLaunchKernelGGL(HIP_KERNEL_NAME(render_persistent<RING, true>), dim3(blocks), dim3(blk), lds, st, A);
        else
            hipLaunchKernelGGL(HIP_KERNEL_NAME(render_persistent<RING, false>), dim3(blocks), dim3(blk), lds, st, A);
        return (int)hipGetLastError();
    }
    block = 128;
    const size_t lds = (size_t)3 * A.stack_depth * block * sizeof(uint32_t);
    const uint32_t grid = (A.n_items + block - 1) / block;
    if (grid == 0) return 0;
    if (A.K <= 8)
        hipLaunchKernelGGL(render_simple<8>, dim3(grid), dim3(block), lds, st, A);
    else
        hipLaunchKernelGGL(render_simple<64>, dim3(grid), dim3(block), lds, st, A);
    return (int)hipGetLastError();
}

int launch_intersect(const QueryArgs &Q, hipStream_t st) {
    const uint32_t block = 128;
    const size_t lds = (size_t)3 * Q.stack_depth * block * sizeof(uint32_t);
    const uint32_t grid = (Q.n + block - 1) / block;
    if (grid == 0) return 0;
    hipLaunchKernelGGL(intersect_kernel, dim3(grid), dim3(block), lds, st, Q);
    return (int)hipGetLastError();
}

int launch_blend(const BlendArgs &B, hipStream_t st) {
    const uint32_t n = B.xres * B.yres;
    if (n == 0) return 0;
    hipLaunchKernelGGL(blend_tiles_kernel, dim3((n + 255) / 256), dim3(256), 0, st, B);
    return (int)hipGetLastError();
}

} // namespace cr
