// persistent.hip -- the production render kernel: persistent waves with per-lane
// path regeneration (cr_set_option "kernel" 0, the default).
//
// Every lane owns one pixel at a time and runs its samples one after another (so
// the per-pixel sum keeps the reference's sample order, src/rayTracer.cpp:59-62),
// but a lane never waits for the rest of its wave between queries: each outer
// iteration every live lane runs exactly ONE kd query -- a camera/bounce ray
// (closest hit) or a NEE shadow ray (any hit) -- through one shared traversal
// loop, then advances its own path state machine (shade and start the shadow ray
// / bounce / finish the sample / take the next pixel).  Pixels are handed out
// wave-wide: one atomicAdd per refill, lanes ranked by __ballot + mbcnt.
//
// Register budget (the kernel is latency bound: occupancy is the lever, see
// DESIGN.md "Kernel"):
//   * traversal stack entries are 8 B {far node, tmax}; the far child's tmin is
//     the CURRENT tmax at pop time (stack invariant), the top R
//     entries live in an LDS ring [slot][thread], deeper ones spill to HBM;
//   * path state not needed by the traversal (running pixel sum, hit shading,
//     NEE term, RNG, counters of the sample) is parked in a per-lane HBM record
//     across each query instead of occupying VGPRs;
//   * per-bounce (direct, w) pairs for the back-to-front fold go to HBM too.
#include "render_common.hpp"

namespace cr {

enum : uint32_t { ST_NEED_PIXEL = 0, ST_NEW_SAMPLE = 1, ST_CLOSEST = 2, ST_SHADOW = 3, ST_DONE = 4 };

template <int R, bool FULL, bool PF>
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
            if (FULL) {
                c.inner++;
                if (wave_leader()) c.wave_desc++;
            }
            const uint32_t a = nd.y & 3u;
            const float split = __uint_as_float(nd.x);
            const float oa = comp(o, a), da = comp(d, a);
            const float tsplit = split_distance(split, oa, da);
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
        if (FULL) {
            c.leaf++;
            if (wave_leader()) c.wave_round++;
        }
        const uint32_t first = nd.x, count = nd.y >> 2;
        bool found = false;
        float4 n0, n1, n2;
        if (PF && count) {
            n0 = S.recs[3 * first];
            n1 = S.recs[3 * first + 1];
            n2 = S.recs[3 * first + 2];
        }
        for (uint32_t j = 0; j < count; j++) {
            if (FULL && wave_leader()) c.wave_tri++;
            float4 r0, r1, r2;
            if (PF) { // software pipeline: issue triangle j+1's loads before testing j
                r0 = n0;
                r1 = n1;
                r2 = n2;
                if (j + 1 < count) {
                    n0 = S.recs[3 * (first + j + 1)];
                    n1 = S.recs[3 * (first + j + 1) + 1];
                    n2 = S.recs[3 * (first + j + 1) + 2];
                }
            } else {
                r0 = S.recs[3 * (first + j)];
                r1 = S.recs[3 * (first + j) + 1];
                r2 = S.recs[3 * (first + j) + 2];
            }
            const uint32_t id = __float_as_uint(r0.w);
            if (shadow && id == exclude) continue;
            if (FULL) c.tritest++;
            float ux, uy, t;
            if (tri_test(o, d, r0, r1, r2, tmax, ux, uy, t)) {
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
        tmin = tmax; // == the popped entry's split distance (stack invariant)
        tmax = __uint_as_float(e.y);
    }
}

// Parked lane state, float4 slots [slot][gstride]:
//   0 temp.xyz | s        1 direct.xyz | k       2 fcol.xyz | item
//   3 normal.xyz | rng.key  4 contrib.xyz | rng.ctr
struct Lane {
    f3 temp, direct, fcol, normal, contrib;
    uint32_t s, k, item;
    Rng rng;
};
__device__ __forceinline__ float4 pk(f3 v, uint32_t w) { return make_float4(v.x, v.y, v.z, __uint_as_float(w)); }
__device__ __forceinline__ void park(float4 *buf, uint32_t gstride, uint32_t gid, const Lane &L) {
    buf[gid] = pk(L.temp, L.s);
    buf[(size_t)gstride + gid] = pk(L.direct, L.k);
    buf[(size_t)2 * gstride + gid] = pk(L.fcol, L.item);
    buf[(size_t)3 * gstride + gid] = pk(L.normal, L.rng.key);
    buf[(size_t)4 * gstride + gid] = pk(L.contrib, L.rng.ctr);
}
__device__ __forceinline__ void unpark(const float4 *buf, uint32_t gstride, uint32_t gid, Lane &L) {
    const float4 a = buf[gid], b = buf[(size_t)gstride + gid], c = buf[(size_t)2 * gstride + gid],
                 d = buf[(size_t)3 * gstride + gid], e = buf[(size_t)4 * gstride + gid];
    L.temp = ld3(a);
    L.s = __float_as_uint(a.w);
    L.direct = ld3(b);
    L.k = __float_as_uint(b.w);
    L.fcol = ld3(c);
    L.item = __float_as_uint(c.w);
    L.normal = ld3(d);
    L.rng.key = __float_as_uint(d.w);
    L.contrib = ld3(e);
    L.rng.ctr = __float_as_uint(e.w);
}

// Pixel refill (wave-wide, converged) + camera ray of a new sample.
__device__ __forceinline__ void regenerate(const RenderArgs &A, Lane &L, uint32_t &state, f3 &o, f3 &d, Ctr &c) {
    const uint32_t lane = threadIdx.x & 63u;
    for (;;) {
        const uint64_t need = __ballot(state == ST_NEED_PIXEL);
        if (!need) break;
        const uint32_t n = (uint32_t)__popcll(need);
        const uint32_t leader = (uint32_t)__ffsll((long long)need) - 1u;
        uint32_t base = 0;
        if (lane == leader) base = atomicAdd(A.work, n);
        base = __shfl(base, (int)leader, 64);
        if (state == ST_NEED_PIXEL) {
            const uint32_t rank =
                __builtin_amdgcn_mbcnt_hi((uint32_t)(need >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)need, 0u));
            const uint32_t item = base + rank;
            uint32_t px, py;
            if (item >= A.n_items) {
                state = ST_DONE;
            } else if (item_pixel(A, item, px, py)) {
                state = ST_NEW_SAMPLE;
                L.item = item;
                L.s = 0;
                L.temp = mk(0.f, 0.f, 0.f);
            } // else: a partial-tile pixel outside the image: fetch again
        }
    }
    c.paths += wave_count(state == ST_NEW_SAMPLE);
    if (state == ST_NEW_SAMPLE) {
        uint32_t px, py;
        item_pixel(A, L.item, px, py);
        L.rng = rng_make(A.seed, A.layer, py * A.xres + px, L.s);
        o = mk(A.cam[0], A.cam[1], A.cam[2]);
        d = camera_dir(A, px, py, L.rng);
        L.k = 1;
        state = ST_CLOSEST;
    }
}

template <int R, bool FULL, bool PF, int MINW>
__global__ void __launch_bounds__(256, MINW) render_persistent(RenderArgs A) {
    extern __shared__ uint2 ring_lds[];
    const DevScene &S = A.S;
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t gstride = A.gstride;
    float4 *lbuf = A.pathbuf;
    float4 *dw = A.pathbuf + (size_t)PARK_SLOTS * gstride;
    Ctr c = {};

    uint32_t state = ST_NEED_PIXEL;
    f3 o = mk(0.f, 0.f, 0.f), d = mk(0.f, 0.f, 1.f);
    float limit = 0.f;
    uint32_t exclude = 0xffffffffu;
    {
        Lane L;
        L.temp = L.direct = L.fcol = L.normal = L.contrib = mk(0.f, 0.f, 0.f);
        L.s = L.k = L.item = 0;
        L.rng = Rng{0u, 0u};
        regenerate(A, L, state, o, d, c);
        park(lbuf, gstride, gid, L);
    }

    for (;;) {
        if (!__any(state != ST_DONE)) break;
        if (FULL && wave_leader()) c.wave_query++;
        // ---- one kd query per live lane
        const bool shadow = state == ST_SHADOW;
        c.shadow += wave_count(shadow);
        c.closest += wave_count(state == ST_CLOSEST);
        uint32_t t = 0;
        float bx = 0.f, by = 0.f;
        bool h = false;
        if (state == ST_CLOSEST || state == ST_SHADOW)
            h = traverse_ring<R, FULL, PF>(S, ring_lds, A.gstack, gstride, gid, o, d, shadow, limit, exclude, t, bx,
                                           by, c);
        c.hit += wave_count(state == ST_CLOSEST && h);

        // ---- advance the path state machine (RayTracer::sendRay, rayTracer.cpp:76-135)
        Lane L;
        unpark(lbuf, gstride, gid, L);
        bool bounce = false, finish = false, textured = false, pixel_done = false;
        f3 tail = mk(0.f, 0.f, 0.f);
        if (state == ST_SHADOW) {
            if (!h) L.direct = add(L.direct, L.contrib);
            bounce = true;
        } else if (state == ST_CLOSEST) {
            if (!h) {
                tail = mk(A.bg[0], A.bg[1], A.bg[2]);
                finish = true;
            } else {
                const HitShade hs = shade_hit(S, o, t, bx, by, (int)L.k);
                textured = hs.textured;
                L.normal = hs.normal;
                L.fcol = hs.fcol;
                L.direct = hs.direct;
                if (S.nlights) {
                    const Nee n = sample_light(S, hs.p, hs.normal, hs.fcol, L.rng);
                    L.contrib = n.contrib;
                    o = n.origin; // == p + 0.001 n, also the origin of the next bounce
                    d = n.dir;
                    limit = n.distance;
                    exclude = n.light;
                    state = ST_SHADOW;
                } else {
                    o = add(hs.p, muls(hs.normal, 0.001f));
                    bounce = true;
                }
            }
        }
        if (bounce) {
            if ((int)L.k == A.K) {
                tail = L.direct;
                finish = true;
            } else {
                const float sx = rng_uniform(L.rng, -1.f, 1.f);
                const float sy = rng_uniform(L.rng, -1.f, 1.f);
                f3 wi;
                float pdf;
                sample_wi(L.normal, sx, sy, wi, pdf);
                const float Kmax = std_max(std_max(L.fcol.x, L.fcol.y), L.fcol.z);
                if (pdf == 0.f || rng_uniform(L.rng, 0.f, 1.f) > Kmax) {
                    tail = L.direct;
                    finish = true;
                } else {
                    const float cosine = fabsf(dot(L.normal, wi));
                    const f3 w = divs(muls(L.fcol, cosine), pdf * Kmax);
                    dw[(size_t)(2 * (L.k - 1)) * gstride + gid] = pk(L.direct, 0u);
                    dw[(size_t)(2 * (L.k - 1) + 1) * gstride + gid] = pk(w, 0u);
                    d = wi; // o already = p + 0.001 n
                    L.k++;
                    state = ST_CLOSEST;
                }
            }
        }
        if (finish) {
            f3 acc = tail; // back-to-front fold r_j = D_j + W_j * r_{j+1}
            for (int j = (int)L.k - 2; j >= 0; j--) {
                const float4 Dj = dw[(size_t)(2 * j) * gstride + gid];
                const float4 Wj = dw[(size_t)(2 * j + 1) * gstride + gid];
                acc = add(ld3(Dj), mul(ld3(Wj), acc));
            }
            L.temp = add(L.temp, acc);
            L.s++;
            if (L.s == A.spp) {
                uint32_t px, py;
                item_pixel(A, L.item, px, py);
                write_pixel(A, px, py, L.item, L.temp);
                pixel_done = true;
                state = ST_NEED_PIXEL;
            } else {
                state = ST_NEW_SAMPLE;
            }
        }
        c.texhit += wave_count(textured);
        c.pixels += wave_count(pixel_done);
        regenerate(A, L, state, o, d, c);
        park(lbuf, gstride, gid, L);
    }
    // closest, shadow, hit, texhit, paths, pixels are wave tallies
    flush_counters(A.counters, c, (1u << 0) | (1u << 1) | (1u << 5) | (1u << 6) | (1u << 7) | (1u << 8));
}

// Variants (cr_set_option "variant"): LDS ring depth R, software-pipelined leaf
// loads PF, minimum waves per SIMD MINW (caps VGPRs).  The counting build (full
// counters) is one fixed variant: the counts do not depend on the variant.
struct Variant {
    void (*fn)(RenderArgs);
    int ring;
};
#define CR_VARIANT(R, PF, W) {render_persistent<R, false, PF, W>, R}
// Measured on MI355X, sponza stand-in 1080p x 8 spp (profiles/r01_sweep_*.txt):
// (8, PF, 8 waves) 275 Mray/s > (4, PF, 8) 274 > (8, -, 8) 258 > (8, PF, 6) 246 > (8, PF, 4) 196.
static const Variant kVariants[] = {
    CR_VARIANT(8, true, 8), CR_VARIANT(4, true, 8), CR_VARIANT(8, false, 8), CR_VARIANT(8, true, 6),
    CR_VARIANT(8, true, 1),
};
static const int kNumVariants = (int)(sizeof(kVariants) / sizeof(kVariants[0]));
int num_persistent_variants() { return kNumVariants; }

void persistent_geometry(int num_cus, uint32_t waves_per_cu, uint32_t &block, uint32_t &blocks) {
    block = 256;
    if (waves_per_cu == 0) waves_per_cu = 32;
    blocks = (uint32_t)(num_cus > 0 ? num_cus : 256) * ((waves_per_cu * 64 + block - 1) / block);
}

int launch_persistent(const RenderArgs &A, uint32_t waves_per_cu, int num_cus, hipStream_t st) {
    uint32_t blk, blocks;
    persistent_geometry(num_cus, waves_per_cu, blk, blocks);
    if (A.gstride < blk * blocks) return (int)hipErrorInvalidValue;
    if (A.full_counters) {
        const size_t lds = (size_t)8 * blk * sizeof(uint2);
        hipLaunchKernelGGL(HIP_KERNEL_NAME(render_persistent<8, true, true, 1>), dim3(blocks), dim3(blk), lds, st, A);
    } else {
        const Variant &v = kVariants[(A.variant >= 0 && A.variant < kNumVariants) ? A.variant : 0];
        const size_t lds = (size_t)v.ring * blk * sizeof(uint2);
        hipLaunchKernelGGL(v.fn, dim3(blocks), dim3(blk), lds, st, A);
    }
    return (int)hipGetLastError();
}

} // namespace cr
