// persistent.hip -- the production render kernel (cr_set_option "kernel" 0, the
// default): persistent waves, one PATH per lane at a time, resumable kd
// traversal with dynamic path fetch.
//
// Work items are (pixel, sample) pairs in pixel-major order, so the 64 lanes of
// a wave trace samples of the same few pixels: the camera rays (about 80% of
// the closest-hit queries on the sponza stand-in) and their NEE rays are close
// to coherent, which is what the SIMD lanes need.  Each lane writes its path's
// radiance to a per-sample buffer; a second kernel sums every pixel's samples
// in sample order (the reference's order, src/rayTracer.cpp:59-62) and blends
// the layer, so the result is bit-identical to the sequential loop whatever
// order the paths were traced in.
//
// Traversal: one ROUND (descend to a leaf, test it, pop) per outer iteration.
// A lane whose query ended waits in a result state until `A.refill` lanes of
// its wave are waiting (or none is traversing); those lanes then run the path
// state machine (RayTracer::sendRay) up to their next query while the rest of
// the wave keeps its traversal state in registers.
//
// Register budget (the kernel is latency bound: occupancy is the lever, see
// DESIGN.md "Kernel"):
//   * traversal stack entries are 8 B {far node, tmax}; the far child's tmin is
//     the CURRENT tmax at pop time (stack invariant), the top R
//     entries live in an LDS ring [slot][thread], deeper ones spill to HBM;
//   * path state not needed by the traversal (hit shading, NEE term, RNG,
//     bounce count, work item) is parked in a per-lane HBM record across the
//     traversal rounds instead of occupying VGPRs;
//   * per-bounce (direct, w) pairs for the back-to-front fold go to HBM too.
#include "traverse.hpp"

namespace cr {

// Parked lane state, float4 slots [slot][gstride]:
//   0 direct.xyz | k     1 fcol.xyz | work item
//   2 normal.xyz | rng.key   3 contrib.xyz | rng.ctr
struct Lane {
    f3 direct, fcol, normal, contrib;
    uint32_t k, w;
    Rng rng;
};
__device__ __forceinline__ void park(float4 *buf, uint32_t gstride, uint32_t gid, const Lane &L) {
    buf[gid] = pk(L.direct, L.k);
    buf[(size_t)gstride + gid] = pk(L.fcol, L.w);
    buf[(size_t)2 * gstride + gid] = pk(L.normal, L.rng.key);
    buf[(size_t)3 * gstride + gid] = pk(L.contrib, L.rng.ctr);
}
__device__ __forceinline__ void unpark(const float4 *buf, uint32_t gstride, uint32_t gid, Lane &L) {
    const float4 a = buf[gid], b = buf[(size_t)gstride + gid], c = buf[(size_t)2 * gstride + gid],
                 d = buf[(size_t)3 * gstride + gid];
    L.direct = ld3(a);
    L.k = __float_as_uint(a.w);
    L.fcol = ld3(b);
    L.w = __float_as_uint(b.w);
    L.normal = ld3(c);
    L.rng.key = __float_as_uint(c.w);
    L.contrib = ld3(d);
    L.rng.ctr = __float_as_uint(d.w);
}

// Work item w of this launch -> (rank-local pixel item, sample index).
__device__ __forceinline__ void work_item(const RenderArgs &A, uint32_t w, uint32_t &item, uint32_t &s) {
    item = w / A.s_count;
    s = A.s0 + (w - item * A.s_count);
}

// Path state machine of one lane (RayTracer::sendRay, rayTracer.cpp:76-135):
// consume the finished query's result, then shade / start the shadow ray /
// bounce / finish the path / take the next item, until the lane has a new
// query in flight (ST_CLOSEST / ST_SHADOW, traversal set up) or is ST_DONE.
__device__ __forceinline__ void path_advance(const RenderArgs &A, Lane &L, uint32_t &state, f3 &o, f3 &d,
                                             float &limit, uint32_t &exclude, Trav &T, float4 *dw, uint32_t gstride,
                                             uint32_t gid, unsigned long long *tl) {
    const DevScene &S = A.S;
    const uint32_t lane = threadIdx.x & 63u;
    do {
        bool bounce = false, finish = false, textured = false;
        f3 tail = mk(0.f, 0.f, 0.f);
        tally(tl, T_HIT, state == ST_HIT);
        if (state == ST_VISIBLE) {
            L.direct = add(L.direct, L.contrib);
            bounce = true;
        } else if (state == ST_OCCLUDED) {
            bounce = true;
        } else if (state == ST_MISS) {
            tail = mk(A.bg[0], A.bg[1], A.bg[2]);
            finish = true;
        } else if (state == ST_HIT) {
            const HitShade hs = shade_hit(S, o, __float_as_uint(d.z), d.x, d.y, (int)L.k);
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
        tally(tl, T_TEXHIT, textured);
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
            float *out = A.samples + 3 * (size_t)L.w; // [item][sample] == work-item order
            out[0] = acc.x;
            out[1] = acc.y;
            out[2] = acc.z;
            state = ST_NEED_WORK;
        }
        // item fetch: one atomicAdd per group of lanes that need work, lanes
        // ranked by __ballot + mbcnt (consecutive lanes get consecutive samples)
        bool fresh = false;
        for (;;) {
            const uint64_t need = __ballot(state == ST_NEED_WORK);
            if (!need) break;
            const uint32_t n = (uint32_t)__popcll(need);
            const uint32_t leader = (uint32_t)__ffsll((long long)need) - 1u;
            uint32_t base = 0;
            if (lane == leader) base = atomicAdd(A.work, n);
            base = __shfl(base, (int)leader, 64);
            if (state == ST_NEED_WORK) {
                const uint32_t rank =
                    __builtin_amdgcn_mbcnt_hi((uint32_t)(need >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)need, 0u));
                const uint32_t w = base + rank;
                uint32_t item, s, px, py;
                work_item(A, w, item, s);
                if (w >= A.n_work) {
                    state = ST_DONE;
                } else if (item_pixel(A, item, px, py)) {
                    // new path: camera ray (rayTracer.cpp:61)
                    L.w = w;
                    L.rng = rng_make(A.seed, A.layer, py * A.xres + px, s);
                    o = mk(A.cam[0], A.cam[1], A.cam[2]);
                    d = camera_dir(A, px, py, L.rng);
                    L.k = 1;
                    state = ST_CLOSEST;
                    fresh = true;
                } // else: a partial-tile pixel outside the image: fetch again
            }
        }
        tally(tl, T_PATHS, fresh);
        // issue the query
        tally(tl, T_CLOSEST, state == ST_CLOSEST);
        tally(tl, T_SHADOW, state == ST_SHADOW);
        if (state == ST_CLOSEST || state == ST_SHADOW) {
            const bool shadow = state == ST_SHADOW;
            if (!trav_begin(S, o, d, shadow, limit, T)) state = shadow ? ST_VISIBLE : ST_MISS;
        }
    } while (state != ST_CLOSEST && state != ST_SHADOW && state != ST_DONE);
}

// the megakernel's traversal configuration (traverse.hpp TraceDefaults)
template <int R_, bool FULL_, bool PF_, bool FD_> struct MegaCfg : TraceDefaults {
    static constexpr int R = R_, PF = PF_ ? 1 : 0;
    static constexpr bool FULL = FULL_, FD = FD_;
};

template <int R, bool FULL, bool PF, int MINW, bool FD>
__global__ void __launch_bounds__(256, MINW) render_dynamic(RenderArgs A) {
    extern __shared__ uint2 ring_lds[];
    __shared__ unsigned long long tl[T_N];
    if (threadIdx.x < T_N) tl[threadIdx.x] = 0;
    __syncthreads();
    const DevScene &S = A.S;
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t gstride = A.gstride;
    float4 *lbuf = A.pathbuf;
    float4 *dw = A.pathbuf + (size_t)PARK_SLOTS * gstride;
    Ctr c = {};

    uint32_t state = ST_NEED_WORK;
    f3 o = mk(0.f, 0.f, 0.f), d = mk(0.f, 0.f, 1.f);
    float limit = 0.f;
    uint32_t exclude = 0xffffffffu;
    Trav T = {0u, 0u, 0u, 0.f, 0.f, mk(0.f, 0.f, 0.f)};
    {
        Lane L;
        L.direct = L.fcol = L.normal = L.contrib = mk(0.f, 0.f, 0.f);
        L.k = L.w = 0;
        L.rng = Rng{0u, 0u};
        park(lbuf, gstride, gid, L);
    }
    for (;;) {
        const bool busy = state == ST_CLOSEST || state == ST_SHADOW;
        const bool idle = !busy && state != ST_DONE;
        const uint64_t idle_m = __ballot(idle), busy_m = __ballot(busy);
        if (idle_m && (busy_m == 0 || (uint32_t)__popcll(idle_m) >= A.refill)) {
            if (FULL && wave_leader()) c.wave_query++;
            if (idle) {
                Lane L;
                unpark(lbuf, gstride, gid, L);
                path_advance(A, L, state, o, d, limit, exclude, T, dw, gstride, gid, tl);
                park(lbuf, gstride, gid, L);
            }
        }
        const bool go = state == ST_CLOSEST || state == ST_SHADOW;
        if (!__any(go)) {
            if (!__any(state != ST_DONE)) break;
            continue;
        }
        if (go)
            state = trav_round<MegaCfg<R, FULL, PF, FD>>(A.lc_debug, A.lc_min, S, ring_lds, A.gstack, gstride, gid, o, d, state == ST_SHADOW,
                                                exclude, T, c);
    }
    flush_counters(A.counters, c, 0u);
    __syncthreads();
    if (threadIdx.x < T_N && tl[threadIdx.x]) atomicAdd(&A.counters[tally_slot(threadIdx.x)], tl[threadIdx.x]);
}

// Per pixel: add this launch's samples in sample order onto the running sum
// (A.run, carried across sample chunks), then on the last chunk blend the
// layer into the frame / write the tile mean (write_pixel).
__global__ void __launch_bounds__(256) sum_samples(RenderArgs A, int first, int last) {
    const uint32_t item = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t px = 0, py = 0;
    const bool valid = item < A.n_items && item_pixel(A, item, px, py);
    if (valid) {
        f3 temp = mk(0.f, 0.f, 0.f);
        if (!first) temp = mk(A.run[3 * (size_t)item], A.run[3 * (size_t)item + 1], A.run[3 * (size_t)item + 2]);
        const float *sm = A.samples + 3 * (size_t)item * A.s_count;
        // A.nl layers in one pass (never sample-chunked): each layer's run of A.spp samples is
        // summed in sample order and blended / written as its own layer, in layer order
        for (uint32_t j = 0; j + 1 < A.nl; j++) {
            for (uint32_t s = j * A.spp; s < (j + 1) * A.spp; s++)
                temp = add(temp, mk(sm[3 * s], sm[3 * s + 1], sm[3 * s + 2]));
            write_pixel(A, px, py, item, temp, j);
            temp = mk(0.f, 0.f, 0.f);
        }
        const uint32_t s_first = (A.nl - 1) * A.spp;
        for (uint32_t s = s_first; s < A.s_count; s++) temp = add(temp, mk(sm[3 * s], sm[3 * s + 1], sm[3 * s + 2]));
        if (last) {
            write_pixel(A, px, py, item, temp, A.nl - 1);
        } else {
            A.run[3 * (size_t)item] = temp.x;
            A.run[3 * (size_t)item + 1] = temp.y;
            A.run[3 * (size_t)item + 2] = temp.z;
        }
    }
    const uint64_t b = __ballot(valid && last);
    // (pixels written: one per layer of the pass)
    if (b && (threadIdx.x & 63u) == 0) atomicAdd(&A.counters[T_PIXELS], (unsigned long long)__popcll(b) * A.nl);
}

// sum_samples with the sample runs staged through LDS: a block's 256 pixels read their next SUM_C samples
// together (each pixel's run of SUM_C x 12 B read by consecutive lanes, 16 B each), then each thread adds
// its pixel's from LDS -- the same adds in the same order as sum_samples.  The thread-per-pixel reads of
// sum_samples touch 64 lines per wave-load and re-read each line ~10 loads later, by which time the many
// waves streaming beside it have evicted it from L2 (2-3x the sample bytes at the fabric).  Needs
// s_count % 4 == 0 (16-B aligned runs).
enum : uint32_t { SUM_C = 16, SUM_ROW = 3 * SUM_C + 1 }; // (+1: the rows of consecutive pixels start in other banks)
__global__ void __launch_bounds__(256) sum_samples_lds(RenderArgs A, int first, int last) {
    __shared__ float buf[256 * SUM_ROW];
    const uint32_t item0 = blockIdx.x * blockDim.x, item = item0 + threadIdx.x;
    const uint32_t nitems = min((uint32_t)blockDim.x, A.n_items - item0);
    uint32_t px = 0, py = 0;
    const bool valid = item < A.n_items && item_pixel(A, item, px, py);
    f3 temp = mk(0.f, 0.f, 0.f);
    if (valid && !first) temp = mk(A.run[3 * (size_t)item], A.run[3 * (size_t)item + 1], A.run[3 * (size_t)item + 2]);
    const uint32_t S = A.s_count;
    const float4 *run4 = (const float4 *)(A.samples + 3 * (size_t)item0 * S); // S % 4 == 0: 16-B aligned
    const size_t stride4 = 3 * (size_t)S / 4;                                   // float4 per pixel run
    uint32_t lj = 0;                                                            // the layer of the pass
    for (uint32_t s0 = 0; s0 < S; s0 += SUM_C) {
        const uint32_t cs = min((uint32_t)SUM_C, S - s0), q = 3 * cs / 4; // samples and float4 per pixel this chunk
        __syncthreads(); // (the previous chunk is consumed)
        for (uint32_t k = threadIdx.x; k < nitems * q; k += blockDim.x) {
            const uint32_t pix = k / q, part = k - pix * q;
            const float4 v = run4[pix * stride4 + 3 * (size_t)s0 / 4 + part];
            float *d = buf + pix * SUM_ROW + 4 * part;
            d[0] = v.x;
            d[1] = v.y;
            d[2] = v.z;
            d[3] = v.w;
        }
        __syncthreads();
        if (valid) {
            const float *b = buf + threadIdx.x * SUM_ROW;
            for (uint32_t t = 0; t < cs; t++) {
                temp = add(temp, mk(b[3 * t], b[3 * t + 1], b[3 * t + 2]));
                // A.nl layers in one pass (never sample-chunked): a layer's run ends -> blend / write it
                const uint32_t s = s0 + t + 1;
                if (A.nl > 1 && s < S && s % A.spp == 0) {
                    write_pixel(A, px, py, item, temp, lj);
                    temp = mk(0.f, 0.f, 0.f);
                    lj++;
                }
            }
        }
    }
    if (valid) {
        if (last) {
            write_pixel(A, px, py, item, temp, A.nl - 1);
        } else {
            A.run[3 * (size_t)item] = temp.x;
            A.run[3 * (size_t)item + 1] = temp.y;
            A.run[3 * (size_t)item + 2] = temp.z;
        }
    }
    const uint64_t bl = __ballot(valid && last);
    if (bl && (threadIdx.x & 63u) == 0) atomicAdd(&A.counters[T_PIXELS], (unsigned long long)__popcll(bl) * A.nl);
}

// Variants (cr_set_option "variant"): LDS ring depth R, software-pipelined leaf
// loads PF, minimum waves per SIMD MINW (caps VGPRs), short exact split
// division FD.  The counting build (full counters) is one fixed variant per
// FD: the counts do not depend on the variant.
struct Variant {
    void (*fn)(RenderArgs);
    void (*counting)(RenderArgs);
    int ring;
};
#define CR_DYNAMIC(R, PF, W, FD) {render_dynamic<R, false, PF, W, FD>, render_dynamic<8, true, true, 1, FD>, R}
// History on MI355X, sponza stand-in 1080p x 8 spp (profiles/r01_sweep_*.txt):
//   per-query loop, wave waits for its longest query (8, PF, 8 waves)   287 Mray/s
//   dynamic fetch, one pixel (all its samples) per lane (8, PF, 6)     382
//     + speculative descent 360; + query registers spilled around the state
//     machine 376; + per-XCD pixel bands 340 (the shared front keeps the
//     Infinity-Cache working set small): none kept
static const Variant kVariants[] = {
    CR_DYNAMIC(8, true, 6, false), CR_DYNAMIC(8, true, 6, true), CR_DYNAMIC(8, true, 8, false),
    CR_DYNAMIC(4, true, 6, false), CR_DYNAMIC(8, false, 6, false), CR_DYNAMIC(8, true, 5, false),
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
    if (A.gstride < blk * blocks || !A.samples || A.s_count == 0) return (int)hipErrorInvalidValue;
    const Variant &v = kVariants[(A.variant >= 0 && A.variant < kNumVariants) ? A.variant : 0];
    if (A.full_counters) {
        const size_t lds = (size_t)8 * blk * sizeof(uint2);
        hipLaunchKernelGGL(v.counting, dim3(blocks), dim3(blk), lds, st, A);
    } else {
        const size_t lds = (size_t)v.ring * blk * sizeof(uint2);
        hipLaunchKernelGGL(v.fn, dim3(blocks), dim3(blk), lds, st, A);
    }
    return (int)hipGetLastError();
}

// lds: dynamic LDS reserved per block (unused: it only caps the blocks per CU, so fewer waves share
// each CU's slice of L2 while they stream their pixels' sample runs; option "sum_lds")
// staged: sum_samples_lds when the runs are 16-B aligned (option "sum_staged", default)
int launch_sum_samples(const RenderArgs &A, bool first, bool last, hipStream_t st, uint32_t lds, bool staged) {
    const uint32_t blocks = (A.n_items + 255) / 256;
    if (!blocks) return (int)hipGetLastError();
    if (staged && A.s_count % 4 == 0)
        hipLaunchKernelGGL(sum_samples_lds, dim3(blocks), dim3(256), lds, st, A, first ? 1 : 0, last ? 1 : 0);
    else
        hipLaunchKernelGGL(sum_samples, dim3(blocks), dim3(256), lds, st, A, first ? 1 : 0, last ? 1 : 0);
    return (int)hipGetLastError();
}

} // namespace cr
