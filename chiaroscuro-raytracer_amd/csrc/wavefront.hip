// wavefront.hip -- wavefront path tracer (cr_set_option "kernel" 2).
//
// The megakernel (persistent.hip) keeps every lane's traversal registers live
// while other lanes of its wave shade, so its register peak is traversal +
// shading and it runs at 6 waves/SIMD; occupancy measured as its main lever
// (2 -> 6 waves/SIMD: 260 -> 563 Mray/s).  Here the same per-path arithmetic is
// split by phase into kernels that exchange work through queues in HBM:
//
//   wf_camera                 one closest ray per path of the chunk
//   wf_trace<closest>(1)
//   for g = 1..K:
//     wf_shade(g)             hit reconstruction, emission, NEE light sample
//                             -> shadow queue g, then BRDF sample + RR -> closest
//                             queue g + 1 (rayTracer.cpp:80-134: none of these
//                             draws depends on the shadow result)
//     wf_trace<shadow>(g)  ||  wf_trace<closest>(g + 1)    two streams: each
//                             launch's tail (its longest queries) overlaps the other
//     wf_resolve(g)           NEE result -> the bounce's direct term; paths that
//                             ended at bounce g are folded into samples[w]
//   (a closest queue below wf_tail_min: the rest of the chunk runs in wf_tail)
//
// Paths keep their (pixel, sample) RNG keys and draw order, and every path
// writes its radiance to samples[w]; sum_samples adds them per pixel in sample
// order, so the image is bit-identical to the megakernel's and the oracle's.
// Queue appends are wave-aggregated (one atomic per wave, lane order kept), so
// neighbouring paths -- samples of the same pixel -- stay neighbours in the
// queues and the trace waves stay coherent.
#include "camcull.hpp"
#include "traverse.hpp"

#include <atomic>
#include <thread>

namespace cr {

// DEAD_RAY: the hit record .x of a partial-tile slot's camera ray when the camera is fused (.w = 0: no hit)
enum : uint32_t { NO_SLOT = 0xffffffffu, NO_PATH = 0xffffffffu, DEAD_RAY = 1u };
// sexcl[j]: the light triangle shadow ray j ignores, bit 31 set when the ray's path continues
// (the overlapped tail traces those; triangle ids stay below 2^31)
enum : uint32_t { SEXCL_CONT = 0x80000000u };

// Block-aggregated appends (call with the whole block, uniformly): one global atomicAdd per block and
// queue instead of one per wave -- same-address atomics from every wave of the grid serialise in one L2
// slice.  Slots keep lane order within a wave and wave order within the block.
// (lds: one word per wave of the block, up to 16, then the base)
enum : uint32_t { APP_W = 16 };
// N appends of one block at once (wf_shade's shadow and closest queues): one barrier round and
// the N global atomics in flight together instead of one after another.  lds: [2][4 N + N] words,
// the half `buf` alternating between consecutive calls (so no barrier is needed before the next
// call writes it: the one after that is separated from this one by the next call's barriers).
template <int N>
__device__ __forceinline__ void block_append_n(uint32_t *const (&counter)[N], const bool (&pred)[N], uint32_t *lds,
                                               uint32_t buf, uint32_t (&slot)[N]) {
    uint32_t *L = lds + buf * (APP_W + 1u) * N;
    const uint32_t wave = threadIdx.x >> 6;
    uint64_t m[N];
#pragma unroll
    for (int q = 0; q < N; q++) {
        m[q] = __ballot(pred[q]);
        if ((threadIdx.x & 63u) == 0) L[APP_W * q + wave] = (uint32_t)__popcll(m[q]);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t tot[N];
#pragma unroll
        for (int q = 0; q < N; q++) {
            uint32_t s = 0;
            for (uint32_t w = 0; w < (blockDim.x >> 6); w++) {
                const uint32_t c = L[APP_W * q + w];
                L[APP_W * q + w] = s;
                s += c;
            }
            tot[q] = s;
        }
        uint32_t base[N];
#pragma unroll
        for (int q = 0; q < N; q++) base[q] = tot[q] ? atomicAdd(counter[q], tot[q]) : 0u;
#pragma unroll
        for (int q = 0; q < N; q++) L[APP_W * N + q] = base[q];
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < N; q++)
        slot[q] = L[APP_W * N + q] + L[APP_W * q + wave] +
                  __builtin_amdgcn_mbcnt_hi((uint32_t)(m[q] >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m[q], 0u));
}

// block_append_n with the slots reserved app_chunk at a time (WfArgs::app_chunk): thread 0 keeps each
// queue's current chunk (cb: its first slot, cu: slots used; cu = C and cb anything before the first) in its
// registers and reserves a new chunk only when an iteration's appends do not fit the current one; the
// appends of one call then split at most once, the first `room` of them at the end of the old chunk, the
// rest at the start of the new one.  lds: [2][4 N + 3 N] words, alternating halves as block_append_n's.
template <int N>
__device__ __forceinline__ void block_append_chunk(uint32_t *const (&counter)[N], const bool (&pred)[N], uint32_t *lds,
                                                   uint32_t buf, uint32_t C, uint32_t (&cb)[N], uint32_t (&cu)[N],
                                                   uint32_t (&slot)[N]) {
    uint32_t *L = lds + buf * (APP_W + 3u) * N;
    const uint32_t wave = threadIdx.x >> 6;
    uint64_t m[N];
#pragma unroll
    for (int q = 0; q < N; q++) {
        m[q] = __ballot(pred[q]);
        if ((threadIdx.x & 63u) == 0) L[APP_W * q + wave] = (uint32_t)__popcll(m[q]);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t tot[N], fresh[N];
#pragma unroll
        for (int q = 0; q < N; q++) {
            uint32_t s = 0;
            for (uint32_t w = 0; w < (blockDim.x >> 6); w++) {
                const uint32_t c = L[APP_W * q + w];
                L[APP_W * q + w] = s;
                s += c;
            }
            tot[q] = s;
            fresh[q] = s > C - cu[q] ? atomicAdd(counter[q], C) : 0u; // (all reservations in flight together)
        }
#pragma unroll
        for (int q = 0; q < N; q++) {
            const uint32_t room = C - cu[q];
            L[APP_W * N + 3 * q] = cb[q] + cu[q];
            L[APP_W * N + 3 * q + 1] = tot[q] > room ? room : tot[q];
            L[APP_W * N + 3 * q + 2] = fresh[q];
            if (tot[q] > room) {
                cb[q] = fresh[q];
                cu[q] = tot[q] - room;
            } else {
                cu[q] += tot[q];
            }
        }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < N; q++) {
        const uint32_t i = L[APP_W * q + wave] +
                           __builtin_amdgcn_mbcnt_hi((uint32_t)(m[q] >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m[q], 0u));
        const uint32_t room = L[APP_W * N + 3 * q + 1];
        slot[q] = i < room ? L[APP_W * N + 3 * q] + i : L[APP_W * N + 3 * q + 2] + (i - room);
    }
}

__device__ __forceinline__ uint32_t *cnt_closest(const WfArgs &W, uint32_t g) { return W.cnt + g; }
__device__ __forceinline__ uint32_t *cnt_shadow(const WfArgs &W, uint32_t g) { return W.cnt + WF_G + g; }
__device__ __forceinline__ uint32_t *work_closest(const WfArgs &W, uint32_t g) { return W.cnt + 2 * WF_G + g; }
__device__ __forceinline__ uint32_t *work_shadow(const WfArgs &W, uint32_t g) { return W.cnt + 3 * WF_G + g; }

// Queue sort key (raysort.hip): 8x8-pixel sub-tile of the path's pixel, then an
// 8x8 octahedral direction bin.  Any deterministic key is exact -- it only
// orders the work.
__device__ __forceinline__ uint32_t dir_bin(f3 d, uint32_t res) {
    const float s = fabsf(d.x) + fabsf(d.y) + fabsf(d.z);
    if (!(s > 0.f)) return 0u;
    float u = d.x / s, v = d.z / s;
    if (d.y < 0.f) {
        const float uu = (1.f - fabsf(v)) * (u >= 0.f ? 1.f : -1.f), vv = (1.f - fabsf(u)) * (v >= 0.f ? 1.f : -1.f);
        u = uu;
        v = vv;
    }
    const float h = 0.5f * (float)res;
    const uint32_t bu = (uint32_t)min((int)res - 1, max(0, (int)((u + 1.f) * h)));
    const uint32_t bv = (uint32_t)min((int)res - 1, max(0, (int)((v + 1.f) * h)));
    // Morton order: consecutive keys stay close in direction along both axes
    uint32_t m = 0;
    for (uint32_t b = 0; (1u << b) < res; b++) m |= ((bu >> b) & 1u) << (2 * b + 1) | ((bv >> b) & 1u) << (2 * b);
    return m;
}
// World-space variant for rays whose origins are not tied to their pixel (the
// shadow rays of bounce >= 2 and the closest rays of bounce >= 3): a 3-D Morton
// code of the origin in the scene box (WORLD_BITS per axis), then the direction.
__device__ __forceinline__ uint32_t world_key(const RenderArgs &A, const WfArgs &W, f3 o, f3 dir) {
    const DevScene &S = A.S;
    const uint32_t WORLD_BITS = W.world_bits;
    const float sc = (float)(1u << WORLD_BITS);
    const uint32_t qx = (uint32_t)min((int)sc - 1, max(0, (int)((o.x - S.bmin.x) / (S.bmax.x - S.bmin.x) * sc)));
    const uint32_t qy = (uint32_t)min((int)sc - 1, max(0, (int)((o.y - S.bmin.y) / (S.bmax.y - S.bmin.y) * sc)));
    const uint32_t qz = (uint32_t)min((int)sc - 1, max(0, (int)((o.z - S.bmin.z) / (S.bmax.z - S.bmin.z) * sc)));
    uint32_t m = 0;
    for (uint32_t b = 0; b < WORLD_BITS; b++)
        m |= ((qx >> b) & 1u) << (3 * b + 2) | ((qy >> b) & 1u) << (3 * b + 1) | ((qz >> b) & 1u) << (3 * b);
    return m * (W.dir_res * W.dir_res) + dir_bin(dir, W.dir_res);
}
__device__ __forceinline__ uint32_t sort_key(const RenderArgs &A, const WfArgs &W, uint32_t p, f3 dir) {
    const uint32_t item = (W.w0 + p) / A.s_count;
    const uint32_t T = A.tile, TT = T * T, lt = item / TT, o = item - lt * TT, sh = W.sort_tile;
    const uint32_t S = (T + (1u << sh) - 1) >> sh;
    const uint32_t sub = ((o / T) >> sh) * S + ((o % T) >> sh);
    return (lt * S * S + sub) * (W.dir_res * W.dir_res) + dir_bin(dir, W.dir_res);
}

__device__ __forceinline__ void flush_tallies(const RenderArgs &A, unsigned long long *tl) {
    __syncthreads();
    if (threadIdx.x < T_N && tl[threadIdx.x]) atomicAdd(&A.counters[tally_slot(threadIdx.x)], tl[threadIdx.x]);
}

// Back-to-front fold of a finished path (r_j = D_j + W_j * r_{j+1}) into samples[w].
__device__ __forceinline__ void finish_path(const RenderArgs &A, const WfArgs &W, uint32_t p, uint32_t k, f3 tail) {
    f3 acc = tail;
    for (int j = (int)k - 2; j >= 0; j--) {
        const float4 Dj = W.dw[(size_t)(2 * j) * W.P + p];
        const float4 Wj = W.dw[(size_t)(2 * j + 1) * W.P + p];
        acc = add(ld3(Dj), mul(ld3(Wj), acc));
    }
    float *out = A.samples + 3 * (size_t)(W.w0 + p);
    out[0] = acc.x;
    out[1] = acc.y;
    out[2] = acc.z;
}

// Path state slots [slot][P]: 0 {direct, -}  1 {fcol, -}  2 {normal, -}  (wf_tail's bounce only)
//                             3 {contrib, shadow slot}  4 {next origin, -}
//                             5 {k, rng.key, rng.ctr, -}: the control words, one 16-B slot (the
//                               per-generation kernels write only this one, not slots 0-2)
__device__ __forceinline__ float4 &PS(const WfArgs &W, int slot, uint32_t p) { return W.ps[(size_t)slot * W.P + p]; }
enum { PS_CTL = 5 };
__device__ __forceinline__ void ctl_store(const WfArgs &W, uint32_t p, uint32_t k, const Rng &rng) {
    PS(W, PS_CTL, p) = make_float4(__uint_as_float(k), __uint_as_float(rng.key), __uint_as_float(rng.ctr), 0.f);
}

// Path state (PS above).  When generation 1 runs as wavefront launches (the chunk is not handed to
// wf_tail at once), wf_camera writes only the resolve mark: wf_shade derives generation 1's
// RNG state -- the camera sample's stream after its two jitter draws -- from the path's (pixel, sample)
// instead of reading it.
__host__ __device__ __forceinline__ bool camera_state_lean(const WfArgs &W) { return W.cam_lean && W.P >= W.tail_min; }
// the key of path p's RNG stream: a function of its (pixel, sample) alone
__device__ __forceinline__ uint32_t path_key(const RenderArgs &A, const WfArgs &W, uint32_t p) {
    const uint32_t w = W.w0 + p, item = w / A.s_count, s = A.s0 + (w - item * A.s_count);
    uint32_t px = 0, py = 0;
    item_pixel(A, item, px, py);
    return path_rng(A, py * A.xres + px, s).key;
}
__device__ __forceinline__ Rng camera_rng(const RenderArgs &A, const WfArgs &W, uint32_t p) {
    return Rng{path_key(A, W, p), 2u}; // (camera_dir's y- and x-jitter draws)
}

// ---------------------------------------------------------------- camera --
__global__ void __launch_bounds__(256) wf_camera(RenderArgs A, WfArgs W) {
    __shared__ unsigned long long tl[T_N];
    if (threadIdx.x < T_N) tl[threadIdx.x] = 0;
    __syncthreads();
    for (uint32_t base = blockIdx.x * blockDim.x; base < W.P; base += gridDim.x * blockDim.x) {
        const uint32_t p = base + threadIdx.x;
        const uint32_t w = W.w0 + p;
        uint32_t item = 0, s = 0, px = 0, py = 0;
        bool valid = p < W.P && w < A.n_work;
        if (valid) {
            item = w / A.s_count;
            s = A.s0 + (w - item * A.s_count);
            valid = item_pixel(A, item, px, py); // partial-tile pixels outside the image: no path
        }
        tally(tl, T_PATHS, valid);
        // ray p of generation 1 is path p's camera ray (no compaction: the few
        // partial-tile paths get a dead ray, path = NO_PATH)
        if (valid) { // rayTracer.cpp:58-62: jittered camera ray of sample s
            Rng rng = path_rng(A, py * A.xres + px, s);
            float2 sxy;
            const f3 d = camera_dir(A, px, py, rng, &sxy);
            if (A.cull) W.cxy[p] = sxy;
            if (!camera_state_lean(W)) ctl_store(W, p, 1u, rng); // (wf_tail from generation 1 reads it)
            W.mark[p] = 0; // no resolve mark (wf_resolve)
            W.ray[1][2 * (size_t)p] = make_float4(A.cam[0], A.cam[1], A.cam[2], __uint_as_float(p));
            W.ray[1][2 * (size_t)p + 1] = pk(d, 0u);
        } else if (p < W.P) {
            W.mark[p] = 0;
            W.ray[1][2 * (size_t)p] = make_float4(0.f, 0.f, 0.f, __uint_as_float(NO_PATH));
            W.ray[1][2 * (size_t)p + 1] = make_float4(0.f, 0.f, 1.f, 0.f);
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) *cnt_closest(W, 1) = W.P;
    flush_tallies(A, tl);
}

// The result of shadow query idx of generation g: occ[idx] or, with WfArgs::vis_dw, the w of the path's
// dw record of bounce g (idx is then the path), which held the query's slot (SHADOW_VIS / SHADOW_OCC
// replace it; NO_SLOT -- no NEE ray -- is never written here).
enum : uint32_t { SHADOW_VIS = 0u, SHADOW_OCC = 1u };
// With WfArgs::vis_mark idx is the path | ENDED_BIT when it ends at this bounce: a visible answer sets the
// visible bit of the path's resolve mark (one byte), an occluded one writes nothing.
enum : uint32_t { ENDED_BIT = 0x80000000u };
__device__ __forceinline__ void shadow_store(const WfArgs &W, uint32_t g, uint32_t idx, bool occluded) {
    if (W.vis_mark) {
        if (!occluded) W.mark[idx & ~ENDED_BIT] = (uint8_t)((g << 2) | 2u | (idx >> 31));
    } else if (W.vis_dw) {
        ((uint32_t *)(W.dw + (size_t)(2 * (g - 1)) * W.P + idx))[3] = occluded ? SHADOW_OCC : SHADOW_VIS;
    } else {
        W.occ[idx] = occluded ? 1u : 0u;
    }
}
// WfArgs::nee_skip: an NEE term of exactly (+0, +0, +0) -- the reference's geometric factor max(0, ...)
// is 0 (the surface or the light faces away), or the product underflows -- adds nothing whatever the
// shadow query answers: direct + (+0) == direct bit for bit unless a component of direct is -0 or a NaN
// (rayTracer.cpp:85 makes it +0 or positive; checked anyway), so the query is answered without a
// traversal and counted as the root-box culls are.
__device__ __forceinline__ bool keeps_plus_zero(float v) { // v + (+0) has v's bits
    const uint32_t b = __float_as_uint(v);
    return b != 0x80000000u && (b & 0x7fffffffu) <= 0x7f800000u;
}
__device__ __forceinline__ bool nee_zero(const WfArgs &W, const RenderArgs &A, f3 contrib, f3 direct) {
    return W.nee_skip && !A.full_counters && !A.perf_counters &&
           (__float_as_uint(contrib.x) | __float_as_uint(contrib.y) | __float_as_uint(contrib.z)) == 0u &&
           keeps_plus_zero(direct.x) && keeps_plus_zero(direct.y) && keeps_plus_zero(direct.z);
}
// true: the NEE ray of a bounce whose dw record's w is `slot` found no occluder
__device__ __forceinline__ bool nee_visible(const WfArgs &W, uint32_t slot) {
    return slot != NO_SLOT && (W.vis_dw ? slot == SHADOW_VIS : W.occ[slot] == 0u);
}

// ----------------------------------------------------------------- trace --
// Persistent: every lane runs one query at a time through trav_round; when
// `A.refill` lanes of a wave have finished (or none is busy) they take the
// next rays of the queue (one atomicAdd per wave).
// CAM: the generation-1 closest trace (camera rays) as its own instantiation, the
// same code: it is the largest launch of a pass and never runs beside another
// trace, so profiles and the bench roofline see it separately.
// CULL (camera instantiation only): triangle tests skipped by the screen-space cull
// boxes (camcull.hpp, A.cull); the lane keeps its sample's screen position.
// C: the build's configuration (traverse.hpp TraceDefaults; the builds: namespace tc below)
template <class C>
__global__ void __launch_bounds__(256, C::MINW) wf_trace(RenderArgs A, WfArgs W, uint32_t g) {
    static constexpr bool SHADOW = C::SHADOW, FULL = C::FULL, CAM = C::CAM, PC = C::PC;
    static constexpr int CULL = C::CULL;
    static_assert(!CULL || (CAM && !SHADOW), "the cull applies to camera rays");
    extern __shared__ uint2 ring_lds[];
    const DevScene &S = A.S;
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x, lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t n = SHADOW ? *cnt_shadow(W, g) : *cnt_closest(W, g);
    uint32_t *work = SHADOW ? work_shadow(W, g) : work_closest(W, g);
    const float4 *rays = SHADOW ? W.sray : W.ray[g & 1];
    Ctr c = {};
    Diag dg = {};
    dg.on = FULL && ((A.diag_kinds >> (SHADOW ? TK_SHADOW : (CAM ? TK_CAMERA : TK_CLOSEST))) & 1u);
    uint32_t state = ST_NEED_WORK, idx = 0, exclude = 0;
    uint32_t issued = 0; // the wave's queries (wave-uniform: an SGPR, not a VGPR per lane)
    f3 o = mk(0.f, 0.f, 0.f), d = mk(0.f, 0.f, 1.f);
    float csx = 0.f, csy = 0.f;
    Trav T = {0u, 0u, 0u, 0.f, 0.f, mk(0.f, 0.f, 0.f)};
    const uint32_t busy_st = SHADOW ? ST_SHADOW : ST_CLOSEST;
    const uint32_t refill = SHADOW ? A.refill_shadow : (g == 1 ? A.refill_camera : A.refill);
    // XCD partition (WfArgs::xcd): wave-uniform range part = xs % 256, WF_XCDS ranges tried
    // in turn (xs / 256 of them drained); one register, the rest is derived at refill
    uint32_t xs = blockIdx.x % WF_XCDS;
    Pc pc = {};
    for (;;) {
        const uint64_t need_m = __ballot(state == ST_NEED_WORK), busy_m = __ballot(state == busy_st);
        if (need_m && (busy_m == 0 || (uint32_t)__popcll(need_m) >= refill)) {
            const bool xp = (W.xcd >> (SHADOW ? 0 : (g == 1 ? 2 : 1))) & 1u;
            uint32_t *xwork = W.cnt + WF_XBASE + ((SHADOW ? WF_G : 0u) + g) * WF_XCDS * WF_XSTRIDE;
            for (;;) { // refill; a ray culled by the root box is answered at once and refetched
                const uint64_t m = __ballot(state == ST_NEED_WORK);
                if (!m) break;
                const uint32_t part = xs & 255u;
                if (xp && (xs >> 8) == WF_XCDS) { // every range drained
                    if (state == ST_NEED_WORK) state = ST_DONE;
                    break;
                }
                const uint32_t leader = (uint32_t)__ffsll((long long)m) - 1u;
                bool iss = false;
                const uint32_t lo = xp ? (uint32_t)((uint64_t)n * part / WF_XCDS) : 0u;
                const uint32_t hi = xp ? (uint32_t)((uint64_t)n * (part + 1) / WF_XCDS) : n;
                uint32_t base = 0;
                if (lane == leader)
                    base = atomicAdd(xp ? xwork + part * WF_XSTRIDE : work, (uint32_t)__popcll(m));
                base = lo + __shfl(base, (int)leader, 64);
                if (xp && base + (uint32_t)__popcll(m) > hi) // this range is drained: the next one
                    xs = (xs & ~255u) + 256u + (part + 1) % WF_XCDS;
                if (state == ST_NEED_WORK) {
                    idx = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                           __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                    if (idx >= hi) {
                        if (!xp) state = ST_DONE; // else: stays idle and takes a ray of the next range
                    } else {
                        if (W.order) idx = W.order[idx]; // sorted queue: results still go to slot idx
                        if (PC) pc.vb += (W.order ? 4u : 0u) + 32u + (SHADOW ? 4u : 0u) + (CULL ? 8u : 0u);
                        const float4 r0 = rays[2 * (size_t)idx], r1 = rays[2 * (size_t)idx + 1];
                        // overlapped tail: a path that continues traces this ray in wf_tail (the lane
                        // stays idle and takes another; no `continue`: every lane reaches the count below)
                        if (!(SHADOW && W.ended_only && (W.sexcl[idx] & SEXCL_CONT))) {
                        o = ld3(r0);
                        d = ld3(r1);
                        const uint32_t sx = SHADOW ? W.sexcl[idx] : 0u;
                        if (SHADOW) exclude = sx & ~SEXCL_CONT;
                        // the result goes to path idx's dw record (vis_dw) or resolve mark (vis_mark: its
                        // ended bit rides in idx)
                        if (SHADOW && W.vis_mark) idx = __float_as_uint(r0.w) | ((sx & SEXCL_CONT) ? 0u : ENDED_BIT);
                        else if (SHADOW && W.vis_dw) idx = __float_as_uint(r0.w);
                        if (CULL) { // ray idx of generation 1 is path idx's camera ray
                            const float2 q = W.cxy[idx];
                            csx = q.x;
                            csy = q.y;
                        }
                        // a dead camera ray or a dead queue entry (wf_shade's chunked appends): no query -- for
                        // shadow queues only in the C::DEAD builds (the check costs the others registers)
                        if ((!SHADOW || C::DEAD) && __float_as_uint(r0.w) == NO_PATH) {
                            if (!SHADOW) W.hit[g & 1][idx] = make_uint4(0u, 0u, 0u, 0u);
                        } else if (iss = true, trav_begin(S, o, d, SHADOW, r1.w, T)) {
                            state = busy_st;
                            if (FULL) diag_begin(&dg);
                        } else if (SHADOW) {
                            if (PC) pc.vb += W.vis_mark ? 1u : 4u;
                            shadow_store(W, g, idx, false); // culled: visible (kdtree.cpp:285-287)
                        } else {
                            if (PC) pc.vb += 16;
                            W.hit[g & 1][idx] = make_uint4(0u, 0u, 0u, 0u);
                        }
                        }
                    }
                }
                issued = __builtin_amdgcn_readfirstlane(issued + (uint32_t)__popcll(__ballot(iss)));
            }
        }
        if (!__any(state == busy_st)) {
            if (!__any(state != ST_DONE)) break;
            continue;
        }
        // the query's result: the answer stored, the lane free
        auto answer = [&](uint32_t r) {
            if (PC) pc.vb += SHADOW ? (W.vis_mark ? (r == ST_OCCLUDED ? 0u : 1u) : 4u) : 16u;
            if (SHADOW) shadow_store(W, g, idx, r == ST_OCCLUDED);
            // w: the hit's leaf + 1, the queue sort's key region
            else W.hit[g & 1][idx] = r == ST_HIT ? make_uint4(__float_as_uint(d.z), __float_as_uint(d.x),
                                                       __float_as_uint(d.y), T.node + 1u)
                                          : make_uint4(0u, 0u, 0u, 0u);
            state = ST_NEED_WORK;
        };
        if (!C::LX) {
            if (state == busy_st) {
                const uint32_t r = trav_round<C>(A.lc_debug, A.lc_min, S, ring_lds, W.gstack, W.gstride, gid, o, d, SHADOW, exclude, T,
                                                 c, csx, csy, A.cull, A.cull_node, FULL ? &dg : nullptr,
                                                 PC ? &pc : nullptr, A.desc_quorum);
                if (r != busy_st) answer(r);
            }
            continue;
        }
        LeafX lx = {0u, 0u};
        uint32_t r = busy_st;
        if (state == busy_st)
            r = trav_round<C>(A.lc_debug, A.lc_min,
                S, ring_lds, W.gstack, W.gstride, gid, o, d, SHADOW, exclude, T, c, csx, csy, A.cull,
                A.cull_node, FULL ? &dg : nullptr, PC ? &pc : nullptr, A.desc_quorum, &lx);
        // LX: the deferred leaves' tests by the whole wave (traverse.hpp leaf_exchange), then each deferred
        // lane ends its round as trav_round does after a leaf
        if (C::LX && __ballot(r == ST_LEAFX)) {
            __shared__ uint32_t lx_lds[4][192]; // per wave (blocks of 256 threads: wf_trace_geometry)
            bool occl, fnd;
            float bx = 0.f, by = 0.f, bt = 0.f;
            uint32_t tri = 0u;
            const bool deferred = r == ST_LEAFX;
            leaf_exchange<SHADOW, C::LXD>(S, (volatile lds_u32 *)lx_lds[wave], deferred ? lx.mask : 0u,
                                  lx.first, o, d, T.tmax, exclude, occl, fnd, bx, by, bt, tri, PC ? &pc : nullptr);
            if (deferred) {
                if (occl) {
                    r = ST_OCCLUDED;
                } else if (fnd) {
                    d = mk(bx, by, __uint_as_float(tri));
                    T.tmax = bt;
                    r = ST_HIT;
                } else if (T.sp == 0) {
                    r = SHADOW ? ST_VISIBLE : ST_MISS;
                } else {
                    trav_pop<C::R>(ring_lds, W.gstack, W.gstride, gid, T);
                    r = busy_st;
                }
            }
        }
        if (state == busy_st && r != busy_st) answer(r);
    }
    if (SHADOW) c.shadow = issued; // queries, box-culled ones included
    else c.closest = issued;
    flush_counters(A.counters, c, SHADOW ? 2u : 1u); // (the count is the wave's already)
    if (PC) {
        pc.q = lane == 0 ? issued : 0u;
        pc_flush(A.counters + CTR_PERF + PERF_N * (SHADOW ? TK_SHADOW : (CAM ? TK_CAMERA : TK_CLOSEST)), pc);
    }
    if (FULL) { // per-instantiation split of the §8d work counters (bench roofline)
        unsigned long long *base = A.counters + CTR_TRACE + 3 * (SHADOW ? TK_SHADOW : (CAM ? TK_CAMERA : TK_CLOSEST));
        const uint32_t v[3] = {c.inner, c.leaf, c.tritest};
#pragma unroll
        for (int i = 0; i < 3; i++) {
            unsigned long long x = v[i];
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1) x += __shfl_xor(x, off, 64);
            if (lane == 0 && x) atomicAdd(&base[i], x);
        }
        diag_flush(A.counters, dg);
    }
}

// ------------------------------------------------------ per-path bodies --
// Shared by the per-generation kernels (wf_shade / wf_bounce) and the tail
// kernel (wf_tail), so both execute the same arithmetic on the same state.

// RayTracer::sendRay up to the shadow query (rayTracer.cpp:80-99) for a closest
// hit of path p: hit shading, emission, NEE light sample.  Writes the path state
// (slot 3's w -- the shadow-queue slot -- is left to the caller).  Returns the
// shadow ray in `sh` when the scene has lights.
struct ShadowRay {
    f3 o, d;
    float dist;
    uint32_t light;
};
__device__ __forceinline__ bool shade_path(const RenderArgs &A, const WfArgs &W, uint32_t p, f3 ro, uint4 h,
                                           bool &textured, ShadowRay &sh) {
    const DevScene &S = A.S;
    const float4 ctl = PS(W, PS_CTL, p);
    const uint32_t k = __float_as_uint(ctl.x);
    const HitShade hs = shade_hit(S, ro, h.x, __uint_as_float(h.y), __uint_as_float(h.z), (int)k);
    textured = hs.textured;
    Rng rng{__float_as_uint(ctl.y), __float_as_uint(ctl.z)};
    f3 contrib = mk(0.f, 0.f, 0.f), next = add(hs.p, muls(hs.normal, 0.001f));
    bool nee = false;
    if (S.nlights) {
        const Nee e = sample_light(S, hs.p, hs.normal, hs.fcol, rng);
        contrib = e.contrib;
        next = e.origin;
        sh.o = e.origin;
        sh.d = e.dir;
        sh.dist = e.distance;
        sh.light = e.light;
        nee = !nee_zero(W, A, contrib, hs.direct); // (the caller counts the query either way)
    }
    PS(W, 0, p) = pk(hs.direct, 0u);
    PS(W, 1, p) = pk(hs.fcol, 0u);
    PS(W, 2, p) = pk(hs.normal, 0u);
    ctl_store(W, p, k, rng);
    PS(W, 4, p) = pk(next, 0u);
    PS(W, 3, p) = pk(contrib, NO_SLOT);
    return nee;
}

// NEE result, then the k == K cut, BRDF sample and Russian roulette
// (rayTracer.cpp:100-134) of path p.  visible: the shadow ray found no occluder
// (false when there was no NEE).  Returns true when the path continues with the
// closest ray (org, wi) of its next bounce; otherwise the path is finished.
__device__ __forceinline__ bool bounce_path(const RenderArgs &A, const WfArgs &W, uint32_t p, bool visible, f3 &org,
                                            f3 &wi) {
    const float4 s0 = PS(W, 0, p), s1 = PS(W, 1, p), s2 = PS(W, 2, p), s3 = PS(W, 3, p), ctl = PS(W, PS_CTL, p);
    const uint32_t k = __float_as_uint(ctl.x);
    f3 direct = ld3(s0);
    const f3 fcol = ld3(s1), normal = ld3(s2);
    Rng rng{__float_as_uint(ctl.y), __float_as_uint(ctl.z)};
    if (visible) direct = add(direct, ld3(s3));
    if ((int)k == A.K) {
        finish_path(A, W, p, k, direct);
        return false;
    }
    const float sx = rng_uniform(rng, -1.f, 1.f);
    const float sy = rng_uniform(rng, -1.f, 1.f);
    float pdf;
    sample_wi(normal, sx, sy, wi, pdf);
    const float Kmax = std_max(std_max(fcol.x, fcol.y), fcol.z);
    if (pdf == 0.f || rng_uniform(rng, 0.f, 1.f) > Kmax) {
        finish_path(A, W, p, k, direct);
        return false;
    }
    const float cosine = fabsf(dot(normal, wi));
    const f3 w = divs(muls(fcol, cosine), pdf * Kmax);
    W.dw[(size_t)(2 * (k - 1)) * W.P + p] = pk(direct, 0u);
    W.dw[(size_t)(2 * (k - 1) + 1) * W.P + p] = pk(w, 0u);
    ctl_store(W, p, k + 1, rng);
    org = ld3(PS(W, 4, p));
    return true;
}

// Everything of RayTracer::sendRay at a closest hit of bounce k = g that does not
// need the shadow result (rayTracer.cpp:80-134): hit shading, emission, the NEE
// light sample and -- for k < K -- the BRDF sample and Russian roulette, in the
// reference's draw order.  The NEE term stays pending for wf_resolve:
// dw[2(k-1)] = {direct, shadow slot (set by the caller)}, PS3 = {contrib, -}, mark = 2k | ended:
// the mark 2k tells wf_resolve's path-order sweep which paths hit at bounce k.
// A continuing path gets W_k in dw[2(k-1)+1] and its next closest ray (org, wi).
// ctr: W.ctl_ray -- the RNG counter the closest ray carries (in: this bounce's, out: the next ray's)
// skipped: the NEE query was answered without a trace (nee_zero; the return value is then false)
// direct: the bounce's emission + direct term, for the caller's dw[2(k-1)] = {direct, shadow slot}
__device__ __forceinline__ bool shade_next(const RenderArgs &A, const WfArgs &W, uint32_t p, uint32_t k, f3 ro, uint4 h,
                                           bool &textured, ShadowRay &sh, bool &cont, f3 &org, f3 &wi, uint32_t &ctr,
                                           f3 &direct, bool &skipped) {
    const DevScene &S = A.S;
    const HitShade hs = shade_hit(S, ro, h.x, __uint_as_float(h.y), __uint_as_float(h.z), (int)k);
    textured = hs.textured;
    const bool cam = k == 1u && camera_state_lean(W);
    Rng rng;
    if (cam) {
        rng = camera_rng(A, W, p);
    } else if (W.ctl_ray && k >= 2u) {
        rng = Rng{path_key(A, W, p), ctr};
    } else {
        const float4 ctl = PS(W, PS_CTL, p);
        rng = Rng{__float_as_uint(ctl.y), __float_as_uint(ctl.z)};
    }
    f3 contrib = mk(0.f, 0.f, 0.f), next = add(hs.p, muls(hs.normal, 0.001f));
    bool nee = false;
    if (S.nlights) {
        const Nee e = sample_light(S, hs.p, hs.normal, hs.fcol, rng);
        contrib = e.contrib;
        next = e.origin;
        sh.o = e.origin;
        sh.d = e.dir;
        sh.dist = e.distance;
        sh.light = e.light;
        nee = true;
        skipped = nee_zero(W, A, contrib, hs.direct);
        nee = !skipped;
    }
    cont = false;
    if ((int)k != A.K) {
        const float sx = rng_uniform(rng, -1.f, 1.f);
        const float sy = rng_uniform(rng, -1.f, 1.f);
        float pdf;
        sample_wi(hs.normal, sx, sy, wi, pdf);
        const float Kmax = std_max(std_max(hs.fcol.x, hs.fcol.y), hs.fcol.z);
        if (!(pdf == 0.f || rng_uniform(rng, 0.f, 1.f) > Kmax)) {
            const float cosine = fabsf(dot(hs.normal, wi));
            const f3 w = divs(muls(hs.fcol, cosine), pdf * Kmax);
            W.dw[(size_t)(2 * (k - 1) + 1) * W.P + p] = pk(w, 0u);
            if (W.ctl_ray) ctr = rng.ctr;
            else ctl_store(W, p, k + 1, rng);
            org = next;
            cont = true;
        }
    }
    direct = hs.direct;
    // vis_mark: the visible case's D_k = direct + contrib, the reference's add (rayTracer.cpp:96-99) done here
    PS(W, 3, p) = pk(W.vis_mark ? add(hs.direct, contrib) : contrib, 0u);
    W.mark[p] = (uint8_t)(W.vis_mark ? (k << 2) | (cont ? 0u : 1u) : (k << 1) | (cont ? 0u : 1u));
    return nee;
}

// ----------------------------------------------------------------- shade --
// Every closest ray of generation g: misses finish their path with the
// background; hits run shade_next and append their NEE ray to shadow queue g and
// their next ray to closest queue g + 1.
// MINW: waves per SIMD the build is held to (6: its 75 VGPRs, no spills; 8: 64 VGPRs, the rest spilled)
// CH: the chunked appends (WfArgs::app_chunk) -- a build of its own, so the per-iteration form keeps its
// registers.  BS: threads per block (a block-aggregated append serves BS rays)
template <int MINW, bool CH = false, int BS = 256>
__global__ void __launch_bounds__(BS, MINW) wf_shade(RenderArgs A, WfArgs W, uint32_t g) {
    __shared__ unsigned long long tl[T_N];
    __shared__ uint32_t app2[2 * (APP_W + 3) * 2];
    if (threadIdx.x < T_N) tl[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t n = *cnt_closest(W, g);
    // chunked appends (WfArgs::app_chunk): thread 0's current chunk per queue, none yet
    const uint32_t C = CH ? W.app_chunk : 0u;
    uint32_t cb[2] = {0u, 0u}, cu[2] = {C, C};
    const float4 *rays = W.ray[g & 1];
    const uint4 *hits = W.hit[g & 1];
    float4 *next_rays = W.ray[(g + 1) & 1];
    uint32_t *const queues[2] = {cnt_shadow(W, g), cnt_closest(W, g + 1)};
    uint32_t it = 0;
    // fused camera (WfArgs::cam_fused): ray i of generation 1 is path i's, from the eye; no wf_camera
    // cleared its resolve mark or counted it
    const bool fused = g == 1 && W.cam_fused;
    // chunked appends: each block takes one contiguous range of the queue (a multiple of the block), so a
    // chunk holds the outputs of neighbouring rays -- the queue keeps the input's locality (and a sorted
    // queue its order among equal keys); otherwise the grid-stride sweep
    const uint32_t span = CH ? ((n + gridDim.x - 1) / gridDim.x + blockDim.x - 1) / blockDim.x * blockDim.x : 0u;
    const uint32_t b0 = CH ? blockIdx.x * span : blockIdx.x * blockDim.x;
    const uint32_t b1 = CH ? min(n, b0 + span) : n, bstep = CH ? blockDim.x : gridDim.x * blockDim.x;
    for (uint32_t base = b0; base < b1; base += bstep, it++) {
        const uint32_t i = base + threadIdx.x;
        const bool in = i < n;
        uint4 h = make_uint4(0u, 0u, 0u, 0u);
        float4 r0 = make_float4(0.f, 0.f, 0.f, 0.f);
        uint32_t ctr = 0; // W.ctl_ray: the RNG counter in the closest ray's w (in the cache line of r0)
        if (in) {
            h = hits[i];
            if (fused) r0 = make_float4(A.cam[0], A.cam[1], A.cam[2], __uint_as_float(h.x == DEAD_RAY && !h.w ? NO_PATH : i));
            else r0 = rays[2 * (size_t)i];
            if (W.ctl_ray && g >= 2 && h.w) ctr = __float_as_uint(rays[2 * (size_t)i + 1].w);
        }
        const uint32_t p = __float_as_uint(r0.w);
        const bool hit = in && h.w != 0u;
        if (fused) {
            if (in && !hit) W.mark[i] = 0; // no resolve mark (wf_resolve)
            tally(tl, T_PATHS, in && p != NO_PATH);
        }
        bool textured = false, nee = false, cont = false, skipped = false;
        ShadowRay sh = {mk(0.f, 0.f, 0.f), mk(0.f, 0.f, 0.f), 0.f, 0u};
        f3 org = mk(0.f, 0.f, 0.f), wi = mk(0.f, 0.f, 0.f), direct = mk(0.f, 0.f, 0.f);
        if (in && !hit) {
            if (p != NO_PATH) finish_path(A, W, p, g, mk(A.bg[0], A.bg[1], A.bg[2]));
        } else if (hit) {
            nee = shade_next(A, W, p, g, ld3(r0), h, textured, sh, cont, org, wi, ctr, direct, skipped);
        }
        tally(tl, T_SHADOW, skipped); // (a query, answered here)
        tally(tl, T_NEE, skipped);
        // shadow queue g and closest queue g + 1 in one barrier round (uniform: the whole block)
        const bool want[2] = {nee, cont};
        uint32_t slots[2];
        if (CH) block_append_chunk<2>(queues, want, app2, it & 1u, C, cb, cu, slots);
        else block_append_n<2>(queues, want, app2, it & 1u, slots);
        const uint32_t j = slots[0], jc = slots[1];
        if (hit) W.dw[(size_t)(2 * (g - 1)) * W.P + p] = pk(direct, nee ? j : NO_SLOT);
        if (nee) {
            W.sray[2 * (size_t)j] = pk(sh.o, p);
            W.sray[2 * (size_t)j + 1] = make_float4(sh.d.x, sh.d.y, sh.d.z, sh.dist);
            W.sexcl[j] = sh.light | (cont ? SEXCL_CONT : 0u);
            if (W.sort) {
                W.key[0][0][j] = W.leaf_keys ? ((h.w - 1u) >> W.leaf_shift) * (W.dir_res_s * W.dir_res_s) + dir_bin(sh.d, W.dir_res_s)
                                 : (W.world_keys && g >= (uint32_t)W.world_keys) ? world_key(A, W, sh.o, sh.d)
                                                                                 : sort_key(A, W, p, sh.d);
            }
        }
        if (cont) {
            next_rays[2 * (size_t)jc] = pk(org, p);
            next_rays[2 * (size_t)jc + 1] = pk(wi, W.ctl_ray ? ctr : 0u);
            if (W.sort) {
                W.key[1][0][jc] = W.leaf_keys ? ((h.w - 1u) >> W.leaf_shift) * (W.dir_res * W.dir_res) + dir_bin(wi, W.dir_res)
                                  : (W.world_keys && g >= (uint32_t)W.world_keys) ? world_key(A, W, org, wi)
                                                                                  : sort_key(A, W, p, wi);
            }
        }
        tally(tl, T_HIT, hit);
        tally(tl, T_TEXHIT, textured);
    }
    if (CH) { // the unused end of each queue's last chunk: dead entries (no path; sorted last)
        __syncthreads();
        if (threadIdx.x == 0) {
            app2[0] = cb[0] + cu[0];
            app2[1] = cu[0] < C ? C - cu[0] : 0u;
            app2[2] = cb[1] + cu[1];
            app2[3] = cu[1] < C ? C - cu[1] : 0u;
        }
        __syncthreads();
        for (uint32_t q = 0; q < 2; q++) {
            const uint32_t from = app2[2 * q], len = app2[2 * q + 1];
            float4 *rq = q ? next_rays : W.sray;
            for (uint32_t k = threadIdx.x; k < len; k += blockDim.x) {
                const uint32_t j = from + k;
                rq[2 * (size_t)j] = make_float4(0.f, 0.f, 0.f, __uint_as_float(NO_PATH));
                rq[2 * (size_t)j + 1] = make_float4(0.f, 0.f, 1.f, 0.f);
                if (!q) W.sexcl[j] = 0u;
                if (W.sort) {
                    W.key[q][0][j] = 0xffffffffu;
                }
            }
        }
    }
    flush_tallies(A, tl);
}

// --------------------------------------------------------------- resolve --
// After the shadow trace of generation g: the bounce's direct term
// D_k = direct + (visible ? contrib : 0) (rayTracer.cpp:96-99), and the
// back-to-front fold of every path that ended at this bounce (ended: bit 0 of its mark).
// The contribution (PS3) is read only for a visible NEE ray.
// m: the path's resolve mark (a hit of generation g)
__device__ __forceinline__ void resolve_path(const RenderArgs &A, const WfArgs &W, uint32_t p, uint32_t g, uint32_t m) {
    const bool ended = m & 1u;
    float4 &dk = W.dw[(size_t)(2 * (g - 1)) * W.P + p];
    if (W.vis_mark) { // dw holds direct; PS3 direct + contrib, the D_k of a visible NEE ray
        if (m & 2u) {
            const float4 s3 = PS(W, 3, p);
            if (ended) finish_path(A, W, p, g, ld3(s3));
            else dk = s3;
        } else if (ended) {
            finish_path(A, W, p, g, ld3(dk));
        }
        return;
    }
    const float4 d4 = dk;
    const uint32_t slot = __float_as_uint(d4.w);
    f3 direct = ld3(d4);
    if (nee_visible(W, slot)) direct = add(direct, ld3(PS(W, 3, p)));
    if (ended) finish_path(A, W, p, g, direct);
    else dk = pk(direct, 0u);
}

// A long queue (at least P / resolve_paths rays) is swept in PATH order: the hits of generation g are the
// paths whose byte mark (WfArgs::mark) is 2g | ended (wf_camera / wf_shade(1) clear it, shade_next sets
// it), so the dw and sample accesses are coalesced instead of scattered in the queue's leaf order, and
// the sweep reads one byte per path.  A short queue is swept in queue order (fewer bytes than a pass
// over all P slots).  Each path's arithmetic is the same either way.
__global__ void __launch_bounds__(256) wf_resolve(RenderArgs A, WfArgs W, uint32_t g) {
    const uint32_t n = *cnt_closest(W, g);
    if (W.resolve_paths && (uint64_t)n * W.resolve_paths >= (uint64_t)W.P) {
        const uint32_t sh = W.vis_mark ? 2u : 1u;
        for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < W.P; p += gridDim.x * blockDim.x) {
            const uint32_t m = W.mark[p];
            if ((m >> sh) == g && (!W.ended_only || (m & 1u))) resolve_path(A, W, p, g, m);
        }
        return;
    }
    const float4 *rays = W.ray[g & 1];
    const uint4 *hits = W.hit[g & 1];
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        if (hits[i].w == 0u) continue;
        const uint32_t p = g == 1 && W.cam_fused ? i : __float_as_uint(rays[2 * (size_t)i].w);
        const uint32_t m = W.mark[p]; // (2g | ended: a hit of this queue)
        // (overlapped tail: a continuing path is the tail's, which resolves this bounce itself)
        if (W.ended_only && !(m & 1u)) continue;
        resolve_path(A, W, p, g, m);
    }
}

// ------------------------------------------------------------------ tail --
// The last generations in ONE launch: every path left in the closest queue of
// generation g0 runs to its end on one lane -- closest query, shade, shadow
// query, bounce, next closest query ... -- with the same per-path bodies as
// the per-generation kernels.  Small late generations are bound by their
// longest query (a per-launch latency floor of ~1.3 ms on the sponza stand-in);
// here the paths' chains overlap instead of paying that floor per generation
// and kind.  Lanes refill from the queue (one atomicAdd per wave) when `refill`
// of them are idle or none is busy; a lane with a finished query advances its
// path at once.
// Overlapped (W.tail_shadow_gen = g0 - 1 = gs): launched beside the shadow trace of generation gs,
// which then takes only the paths that ended at gs; a lane first traces its path's generation-gs
// shadow ray (slot in dw[2(gs-1)].w), resolves that bounce as wf_resolve does (same add), then
// starts the path's closest query of g0.
// the tail kernel's traversal configuration (traverse.hpp TraceDefaults): fat records, scalar loads, and
// with leaf cull records the branch-light steps
template <bool FULL_, int R_, int LC_> struct TailCfg : TraceDefaults {
    static constexpr int R = R_, LC = LC_;
    static constexpr bool FULL = FULL_, SC = true, FAT = true, BF = LC_ != 0;
};

template <bool FULL, int R, int MINW, int LC = 0, bool PC = false>
__global__ void __launch_bounds__(256, MINW) wf_tail(RenderArgs A, WfArgs W, uint32_t g0) {
    extern __shared__ uint2 ring_lds[];
    __shared__ unsigned long long tl[T_N];
    if (threadIdx.x < T_N) tl[threadIdx.x] = 0;
    __syncthreads();
    const DevScene &S = A.S;
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x, lane = threadIdx.x & 63u;
    const uint32_t n = *cnt_closest(W, g0);
    uint32_t *work = work_closest(W, g0);
    const float4 *rays = W.ray[g0 & 1];
    Ctr c = {};
    Pc pc = {};
    uint32_t state = ST_NEED_WORK, p = 0, exclude = 0, nclosest = 0, nshadow = 0, qidx = 0;
    const uint32_t gs = W.tail_shadow_gen;
    bool pend = false; // overlapped: the lane's generation-gs shadow query is in flight
    f3 o = mk(0.f, 0.f, 0.f), d = mk(0.f, 0.f, 1.f);
    Trav T = {0u, 0u, 0u, 0.f, 0.f, mk(0.f, 0.f, 0.f)};
    // start the next closest query of path p from (o, d); a root-box miss is a MISS at once
    auto start_closest = [&]() {
        nclosest++;
        state = trav_begin(S, o, d, false, 0.f, T) ? ST_CLOSEST : ST_MISS;
    };
    for (;;) {
        const uint64_t need_m = __ballot(state == ST_NEED_WORK);
        const uint64_t busy_m = __ballot(state == ST_CLOSEST || state == ST_SHADOW);
        if (need_m && (busy_m == 0 || (uint32_t)__popcll(need_m) >= A.refill)) {
            const uint32_t leader = (uint32_t)__ffsll((long long)need_m) - 1u;
            uint32_t base = 0;
            if (lane == leader) base = atomicAdd(work, (uint32_t)__popcll(need_m));
            base = __shfl(base, (int)leader, 64);
            if (state == ST_NEED_WORK) {
                const uint32_t idx = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(need_m >> 32),
                                                                     __builtin_amdgcn_mbcnt_lo((uint32_t)need_m, 0u));
                if (idx >= n) {
                    state = ST_DONE;
                } else {
                    if (PC) pc.vb += 32;
                    const float4 r0 = rays[2 * (size_t)idx], r1 = rays[2 * (size_t)idx + 1];
                    o = ld3(r0);
                    d = ld3(r1);
                    p = __float_as_uint(r0.w);
                    // W.ctl_ray: the path's control words from its ray (bounce g0, the ray's RNG counter)
                    if (W.ctl_ray && g0 >= 2 && p != NO_PATH)
                        ctl_store(W, p, g0, Rng{path_key(A, W, p), __float_as_uint(r1.w)});
                    const uint32_t slot = (gs && p != NO_PATH)
                                              ? __float_as_uint(W.dw[(size_t)(2 * (gs - 1)) * W.P + p].w) : NO_SLOT;
                    if (slot != NO_SLOT) { // overlapped: this path's generation-gs shadow query first
                        const float4 s0 = W.sray[2 * (size_t)slot], s1 = W.sray[2 * (size_t)slot + 1];
                        if (PC) pc.vb += 36;
                        qidx = idx;
                        pend = true;
                        o = ld3(s0);
                        d = ld3(s1);
                        exclude = W.sexcl[slot] & ~SEXCL_CONT;
                        nshadow++;
                        state = trav_begin(S, o, d, true, s1.w, T) ? ST_SHADOW : ST_VISIBLE;
                    } else if (p != NO_PATH) {
                        start_closest(); // (a dead camera ray of a partial tile: no query)
                    }
                }
            }
        }
        // advance every lane whose query has a result, until it has a new query or is idle
        while (state >= ST_HIT) {
            if (pend) { // overlapped: resolve bounce gs (wf_resolve's resolve_path, a path that continues)
                float4 &dk = W.dw[(size_t)(2 * (gs - 1)) * W.P + p];
                f3 direct = ld3(dk);
                if (state == ST_VISIBLE) direct = add(direct, ld3(PS(W, 3, p)));
                dk = pk(direct, 0u);
                pend = false;
                const float4 r0 = rays[2 * (size_t)qidx], r1 = rays[2 * (size_t)qidx + 1];
                o = ld3(r0);
                d = ld3(r1);
                start_closest();
            } else if (state == ST_MISS) {
                finish_path(A, W, p, __float_as_uint(PS(W, PS_CTL, p).x), mk(A.bg[0], A.bg[1], A.bg[2]));
                state = ST_NEED_WORK;
            } else if (state == ST_HIT) {
                bool textured = false;
                ShadowRay sh;
                tally(tl, T_HIT, true);
                const bool nee = shade_path(A, W, p, o, make_uint4(__float_as_uint(d.z), __float_as_uint(d.x),
                                                                 __float_as_uint(d.y), 1u),
                                            textured, sh);
                tally(tl, T_TEXHIT, textured);
                if (nee) {
                    o = sh.o;
                    d = sh.d;
                    exclude = sh.light;
                    nshadow++;
                    state = trav_begin(S, o, d, true, sh.dist, T) ? ST_SHADOW : ST_VISIBLE;
                } else {
                    if (S.nlights) { // (nee_zero: a query answered without a trace)
                        nshadow++;
                        tally(tl, T_NEE, true);
                    }
                    state = ST_OCCLUDED; // no NEE term: bounce without the contribution
                }
            } else { // ST_VISIBLE / ST_OCCLUDED: the bounce
                f3 org, wi;
                if (bounce_path(A, W, p, state == ST_VISIBLE, org, wi)) {
                    o = org;
                    d = wi;
                    start_closest();
                } else {
                    state = ST_NEED_WORK;
                }
            }
        }
        const bool busy = state == ST_CLOSEST || state == ST_SHADOW;
        if (!__any(busy)) {
            if (!__any(state != ST_DONE)) break;
            continue;
        }
        if (busy) {
            const bool shadow = state == ST_SHADOW;
            const uint32_t r = trav_round<TailCfg<FULL, R, LC>>(A.lc_debug, A.lc_min, S, ring_lds, W.gstack, W.gstride, gid, o, d,
                                                                        shadow, exclude, T, c, 0.f, 0.f,
                                                                        nullptr, nullptr, nullptr,
                                                                        PC ? &pc : nullptr, FULL ? 0u : A.desc_quorum);
            if (r != (shadow ? ST_SHADOW : ST_CLOSEST)) state = r;
        }
    }
    c.closest = nclosest;
    c.shadow = nshadow;
    flush_counters(A.counters, c, 0u);
    if (PC) { // the tail's traversal work (its shading is not counted)
        pc.q = nclosest + nshadow;
        pc_flush(A.counters + CTR_PERF + PERF_N * TK_TAIL, pc);
    }
    flush_tallies(A, tl);
}

// ------------------------------------------------- packet camera-ray trace --
// Trace builds 17 / 18's camera-ray trace.  A wave's 64 (S = 1) or 128 (S = 2, two per
// lane) camera rays -- consecutive samples of one pixel, taken in lock-step -- traverse
// the kd tree as ONE packet: the node is
// wave-uniform (scalar loads, uniform control flow), and every lane keeps its own
// interval and an active flag.  All camera rays start at the eye, so a node's near
// child (kdtree.cpp:262, `belowFirst` from the origin's side of the split) is the same
// for every lane; the packet visits nodes depth-first, near child first, and a lane
// is active exactly at the nodes its own traversal (kdtree.cpp:248-281) visits, with
// the same interval and in the same order:
//   near only   (tsplit >= tmax or < 0)  near with [tmin, tmax]
//   far only    (tsplit <= tmin)         far  with [tmin, tmax]
//   both                                 near with [tmin, tsplit], then far with [tsplit, tmax]
// A lane that finds a hit in a leaf is done (the first leaf with a hit ends its query),
// the others go on; cull boxes (camcull.hpp) deactivate a lane for a subtree / leaf /
// triangle exactly as in build 15.  The stack: per entry the node (per wave, LDS) and
// each ray's tmax at push or an inactive mark (the ring [R][thread][S] in LDS, deeper
// entries spilled to gstack as in trav_round; tmin comes back by the stack invariant, see
// below; tests/test_packet_model.py checks the scheme on the CPU).  If the eye lies exactly on a split plane of its
// axis the near child could differ between lanes; the host then uses build 15's camera
// trace for that render (RenderArgs::eye_on_split).
enum : uint32_t { PACKET_DEPTH = 256 }; // >= the deepest tree cr_upload_scene accepts
// S rays per lane (S = 2: a packet of 128 rays -- at 128 spp exactly one pixel's samples --
// so the per-node scalar control work is shared by twice the rays).
// The stack keeps per ray only the tmax at push (or INACTIVE): on pop a reactivated ray's
// tmin is its current tmax (the kd stack invariant).  It holds for every
// ray that pushed the entry: a ray crossing both children went near with tmax = tsplit,
// and a near subtree finished without a hit (or left by a cull) ends at its interval's
// end; a ray going to the far child only is parked with tmax = its tmin.  Only active
// rays' intervals change, so an inactive ray's tmax still holds its value for the next
// entry it owns.
// FD: the split distance by the exact short division from the ray's RN(1/d) per axis, kept in
// VGPRs (div_by_rcp: Markstein's correction, the full division outside its checked range).
template <int R, int S, bool PC = false, bool FD = false>
__global__ void __launch_bounds__(256, 8) wf_trace_packet(RenderArgs A, WfArgs W, uint32_t g) {
    extern __shared__ uint32_t pring_lds[]; // [R][blockDim][S] per-ray tmax bits at push
    __shared__ uint32_t pnode[4][PACKET_DEPTH];
    static_assert(S == 1 || S == 2, "one or two rays per lane");
    const DevScene &Sc = A.S;
    const uint32_t tid = threadIdx.x, wv = tid >> 6, lane = tid & 63u, bdim = blockDim.x;
    const uint32_t gid = blockIdx.x * bdim + tid, gstride = W.gstride;
    uint32_t *ring = pring_lds;
    uint2 *gstk = W.gstack;
    // fused: every path of the chunk has its camera ray here (wf_camera's queue length, set for wf_shade)
    const uint32_t n = W.cam_fused ? W.P : *cnt_closest(W, 1);
    if (W.cam_fused && gid == 0) *cnt_closest(W, 1) = W.P;
    uint32_t *work = work_closest(W, 1);
    const float4 *rays = W.ray[1];
    uint4 *hits = W.hit[1];
    const f3 eye = mk(A.cam[0], A.cam[1], A.cam[2]); // every camera ray's origin (wf_camera)
    const float4 *cnode = A.cull_node, *cref = A.cull;
    // FD: the eye's offsets to the root box (ray_box_inv's first operands), wave-uniform -- kept in
    // SGPRs so the compiler does not hoist them into VGPRs it then spills
    auto rfl = [](float v) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v))); };
    const float box_lo[3] = {rfl(Sc.bmin.x - eye.x), rfl(Sc.bmin.y - eye.y), rfl(Sc.bmin.z - eye.z)};
    const float box_hi[3] = {rfl(Sc.bmax.x - eye.x), rfl(Sc.bmax.y - eye.y), rfl(Sc.bmax.z - eye.z)};
    const float eye_s[3] = {rfl(eye.x), rfl(eye.y), rfl(eye.z)};
    const uint32_t INACTIVE = 0xffffffffu;
    Ctr c = {};
    Pc pc = {};
    uint32_t issued = 0;
    // XCD partition (WfArgs::xcd bit 2), as in wf_trace: own range first, then the others
    const bool xp = (W.xcd >> 2) & 1u;
    uint32_t part = blockIdx.x % WF_XCDS, tried = 0;
    uint32_t *xwork = W.cnt + WF_XBASE + g * WF_XCDS * WF_XSTRIDE;
    for (;;) {
        const uint32_t lo = xp ? (uint32_t)((uint64_t)n * part / WF_XCDS) : 0u;
        const uint32_t hi = xp ? (uint32_t)((uint64_t)n * (part + 1) / WF_XCDS) : n;
        uint32_t base = 0;
        if (lane == 0) base = atomicAdd(xp ? xwork + part * WF_XSTRIDE : work, 64u * S);
        base = __builtin_amdgcn_readfirstlane(lo + __shfl(base, 0, 64));
        if (base >= hi) {
            if (!xp || ++tried == WF_XCDS) break;
            part = (part + 1) % WF_XCDS;
            continue;
        }
        uint32_t idx[S];
        bool live[S], active[S], found[S];
        f3 d[S], y[S];
        float tmin[S], tmax[S], csx[S], csy[S];
#pragma unroll
        for (int s = 0; s < S; s++) {
            idx[s] = base + 64u * s + lane;
            live[s] = idx[s] < hi;
            d[s] = mk(0.f, 0.f, 1.f);
            y[s] = mk(0.f, 0.f, 0.f);
            tmin[s] = tmax[s] = csx[s] = csy[s] = 0.f;
            found[s] = false;
            if (live[s]) {
                bool dead;
                if (W.cam_fused) { // wf_camera's ray, here: rayTracer.cpp:58-62
                    const uint32_t w = W.w0 + idx[s], item = w / A.s_count, sm = A.s0 + (w - item * A.s_count);
                    uint32_t px = 0, py = 0;
                    dead = !(w < A.n_work && item_pixel(A, item, px, py));
                    if (!dead) {
                        Rng rng = path_rng(A, py * A.xres + px, sm);
                        float2 q;
                        d[s] = camera_dir(A, px, py, rng, &q);
                        csx[s] = q.x;
                        csy[s] = q.y;
                    }
                } else {
                    if (PC) pc.vb += 32;
                    const float4 r0 = rays[2 * (size_t)idx[s]], r1 = rays[2 * (size_t)idx[s] + 1];
                    d[s] = ld3(r1);
                    dead = __float_as_uint(r0.w) == NO_PATH;
                    if (!dead) {
                        if (PC) pc.vb += 8;
                        const float2 q = W.cxy[idx[s]];
                        csx[s] = q.x;
                        csy[s] = q.y;
                    }
                }
                if (dead) { // partial-tile slot: no query (fused: the record says so to wf_shade)
                    hits[idx[s]] = make_uint4(W.cam_fused ? DEAD_RAY : 0u, 0u, 0u, 0u);
                    live[s] = false;
                } else {
                    issued++;
                    Trav T;
                    bool in;
                    if (FD) { // trav_begin's root-box clip and T.r with the uniform offsets above
                        // (rcp_rn_wave == 1.f / d bit for bit; the same products, min and max)
                        const f3 inv = mk(rcp_rn_wave(d[s].x), rcp_rn_wave(d[s].y), rcp_rn_wave(d[s].z));
                        const float txmin = box_lo[0] * inv.x, txmax = box_hi[0] * inv.x;
                        const float tymin = box_lo[1] * inv.y, tymax = box_hi[1] * inv.y;
                        const float tzmin = box_lo[2] * inv.z, tzmax = box_hi[2] * inv.z;
                        T.tmin = std_max(std_max(std_min(txmin, txmax), std_min(tymin, tymax)), std_min(tzmin, tzmax));
                        T.tmax = std_min(std_min(std_max(txmin, txmax), std_max(tymin, tymax)), std_max(tzmin, tzmax));
                        in = !(T.tmax < 0 || T.tmax < T.tmin);
                        const float nan = __builtin_nanf("");
                        y[s] = mk(fabsf(d[s].x) >= 0x1p-40f && fabsf(d[s].x) <= 0x1p40f ? inv.x : nan,
                                  fabsf(d[s].y) >= 0x1p-40f && fabsf(d[s].y) <= 0x1p40f ? inv.y : nan,
                                  fabsf(d[s].z) >= 0x1p-40f && fabsf(d[s].z) <= 0x1p40f ? inv.z : nan);
                    } else {
                        in = trav_begin(Sc, eye, d[s], false, 0.f, T);
                    }
                    if (in) {
                        tmin[s] = T.tmin;
                        tmax[s] = T.tmax;
                    } else {
                        hits[idx[s]] = make_uint4(0u, 0u, 0u, 0u);
                        live[s] = false;
                    }
                }
            }
            active[s] = live[s];
        }
        uint32_t cn = 0, sp = 0, nl = 0; // wave-uniform
        auto any_active = [&]() {
            bool a = false;
#pragma unroll
            for (int s = 0; s < S; s++) a = a | active[s];
            return __ballot(a) != 0;
        };
        // (bitwise &: four compares and three mask ands, no short-circuit branches)
        auto inb = [&](int s, float4 b) {
            return (csx[s] >= b.x) & (csx[s] <= b.y) & (csy[s] >= b.z) & (csy[s] <= b.w);
        };
        // push node with, per ray, its tmax (act) or INACTIVE
        auto push = [&](uint32_t node, const bool (&act)[S]) {
            const uint32_t slot = (sp & (R - 1)) * bdim + tid;
            if (nl == (uint32_t)R) { // spill the oldest
                if (PC) pc.vb += 8;
                uint2 e = make_uint2(ring[slot * S], S == 2 ? ring[slot * S + (S - 1)] : 0u);
                gstack_at(gstk, sp - R, gstride, gid) = e;
            } else {
                nl++;
            }
#pragma unroll
            for (int s = 0; s < S; s++) ring[slot * S + s] = act[s] ? __float_as_uint(tmax[s]) : INACTIVE;
            pnode[wv][sp] = node;
            sp++;
        };
        // the next entry with an active ray; false: the packet's traversal is over
        auto pop = [&]() -> bool {
            while (sp) {
                sp--;
                uint32_t e[S];
                if (nl) {
                    const uint32_t slot = (sp & (R - 1)) * bdim + tid;
#pragma unroll
                    for (int s = 0; s < S; s++) e[s] = ring[slot * S + s];
                    nl--;
                } else {
                    if (PC) pc.vb += 8;
                    const uint2 ge = gstack_at(gstk, sp, gstride, gid);
                    e[0] = ge.x;
                    if (S == 2) e[S - 1] = ge.y;
                }
                cn = __builtin_amdgcn_readfirstlane(pnode[wv][sp]);
                bool a = false;
#pragma unroll
                for (int s = 0; s < S; s++) {
                    const bool act = live[s] & !found[s] & (e[s] != INACTIVE);
                    tmin[s] = act ? tmax[s] : tmin[s]; // the stack invariant
                    tmax[s] = act ? __uint_as_float(e[s]) : tmax[s];
                    active[s] = act;
                    a = a | act;
                }
                if (__ballot(a)) return true;
            }
            return false;
        };
        // a leaf reached with record nd; boxed: its box was read with its fat record
        auto leaf = [&](uint2 nd, bool boxed) {
            const uint32_t first = nd.x, count = nd.y >> 2;
            if (PC) {
#pragma unroll
                for (int s = 0; s < S; s++) pc.leaves += active[s] ? 1u : 0u;
            }
            if (!boxed) {
                if (PC && wave_leader()) pc.sb += 16;
                const float4 lb = sload_box(cnode + __builtin_amdgcn_readfirstlane(cn));
#pragma unroll
                for (int s = 0; s < S; s++) active[s] = active[s] & inb(s, lb);
            }
            if (!any_active() || !count) return;
            const float4 *rb = Sc.recs + (size_t)REC_STRIDE * first;
            const uint32_t leafw = __builtin_amdgcn_readfirstlane(cn) + 1u; // hit record w: the leaf + 1
            for (uint32_t j = 0; j < count; j += 4) {
                if (PC && wave_leader()) pc.sb += 64;
                const cr_v16f bb = sload_box4(cref + first + j);
#pragma unroll
                for (uint32_t k = 0; k < 4; k++) {
                    if (j + k >= count) break;
                    const float4 b = make_float4(bb[4 * k], bb[4 * k + 1], bb[4 * k + 2], bb[4 * k + 3]);
                    bool in[S], any = false;
#pragma unroll
                    for (int s = 0; s < S; s++) {
                        in[s] = active[s] & inb(s, b);
                        any = any | in[s];
                    }
                    if (!__ballot(any)) continue;
                    if (PC && wave_leader()) pc.sb += 16u * REC_STRIDE;
                    const TriRec r = sload_rec(rb + (size_t)REC_STRIDE * (j + k));
#pragma unroll
                    for (int s = 0; s < S; s++) {
                        if (!__ballot(in[s])) continue;
                        float ux, uy, t;
                        const bool acc = in[s] & tri_test_wave(eye, d[s], r, tmax[s], ux, uy, t);
                        if (PC) pc.tests += in[s] ? 1u : 0u;
                        if (PC && acc) pc.vb += 16;
                        // the hit record straight to the queue (a later, nearer one in this leaf overwrites it)
                        if (acc) hits[idx[s]] = make_uint4(rec_id(r), __float_as_uint(ux), __float_as_uint(uy), leafw);
                        tmax[s] = acc ? t : tmax[s];
                        found[s] = found[s] | acc;
                    }
                }
            }
        };
        bool go = any_active();
        while (go) {
            // fetch node cn: its record, both children's records and its subtree box
            uint4 f0, f1;
            float4 b;
            cn = __builtin_amdgcn_readfirstlane(cn); // uniform by construction
            if (PC && wave_leader()) {
                pc.sb += 48;
                pc.waves++;
            }
            sload_fat_box_n(Sc.fat, cnode, cn, f0, f1, b);
#pragma unroll
            for (int s = 0; s < S; s++) active[s] = active[s] & inb(s, b);
            uint2 nd = make_uint2(f0.x, f0.y);
            bool popit = true;
            // one fat record serves two levels: the fetched node (lvl 0, its children's
            // records at hand) and the child stepped into (lvl 1, its children fetched next)
            for (uint32_t lvl = 0;; lvl++) {
                if (!any_active()) break;
                if ((nd.y & 3u) == 3u) {
                    leaf(nd, lvl == 0);
                    break;
                }
                const uint32_t a = nd.y & 3u, child = nd.y >> 2;
                const float split = __uint_as_float(nd.x);
                // the split axis is wave-uniform: the lanes' components are picked by scalar branches
                // (one move per value, kept apart by the asm) instead of two v_cndmask per value
                float oa, da[S], ya[S];
                auto pick = [&](float e, const float (&dv)[S], const float (&yv)[S]) {
                    oa = e;
#pragma unroll
                    for (int s = 0; s < S; s++) {
                        asm volatile("v_mov_b32 %0, %1" : "=v"(da[s]) : "v"(dv[s]));
                        asm volatile("v_mov_b32 %0, %1" : "=v"(ya[s]) : "v"(yv[s]));
                    }
                };
                if (a == 0) {
                    float dv[S], yv[S];
#pragma unroll
                    for (int s = 0; s < S; s++) dv[s] = d[s].x, yv[s] = y[s].x;
                    pick(eye_s[0], dv, yv);
                } else if (a == 1) {
                    float dv[S], yv[S];
#pragma unroll
                    for (int s = 0; s < S; s++) dv[s] = d[s].y, yv[s] = y[s].y;
                    pick(eye_s[1], dv, yv);
                } else {
                    float dv[S], yv[S];
#pragma unroll
                    for (int s = 0; s < S; s++) dv[s] = d[s].z, yv[s] = y[s].z;
                    pick(eye_s[2], dv, yv);
                }
                const uint32_t below = oa < split ? 1u : 0u; // uniform: the eye is not on the plane
                const uint32_t nearc = child + (1u - below), farc = child + below;
                // (bitwise logic on the lane masks: no short-circuit branches)
                float tsp[S];
                bool crosses[S], after[S], to_near[S], to_far[S], anyn = false, anyf = false;
#pragma unroll
                for (int s = 0; s < S; s++) {
                    if (PC) pc.steps += active[s] ? 1u : 0u;
                    tsp[s] = FD ? div_by_rcp_wave(split - oa, da[s], ya[s]) : split_distance(split, oa, da[s]);
                    crosses[s] = !(tsp[s] >= tmax[s]) & !(tsp[s] < 0.f); // !near_only
                    after[s] = !(tsp[s] <= tmin[s]);                     // far_only = crosses & !after
                    to_near[s] = active[s] & (!crosses[s] | after[s]);
                    to_far[s] = active[s] & crosses[s];
                    anyn = anyn | to_near[s];
                    anyf = anyf | to_far[s];
                }
                if (!__ballot(anyn)) { // every active ray goes to the far child only
                    cn = farc;
                } else {
                    if (__ballot(anyf)) push(farc, to_far);
#pragma unroll
                    for (int s = 0; s < S; s++) {
                        // both: near with tmax = tsplit; far only: parked with tmax = tmin
                        const float nt = after[s] ? tsp[s] : tmin[s];
                        tmax[s] = to_far[s] ? nt : tmax[s];
                        active[s] = to_near[s];
                    }
                    cn = nearc;
                }
                if (lvl == 1) { // cn's record is not in this fat record: fetch it
                    popit = false;
                    break;
                }
                nd = cn == child ? make_uint2(f0.z, f0.w) : make_uint2(f1.x, f1.y);
            }
            go = popit ? pop() : true;
        }
#pragma unroll
        for (int s = 0; s < S; s++) {
            if (PC && (live[s] & !found[s])) pc.vb += 16;
            if (live[s] & !found[s]) hits[idx[s]] = make_uint4(0u, 0u, 0u, 0u);
        }
    }
    c.closest = issued;
    flush_counters(A.counters, c, 0u);
    if (PC) {
        pc.q = issued;
        pc_flush(A.counters + CTR_PERF + PERF_N * TK_CAMERA, pc);
    }
}

// --------------------------------------------------------------- launch --
struct WfVariant {
    void (*camera)(RenderArgs, WfArgs, uint32_t);
    void (*closest)(RenderArgs, WfArgs, uint32_t);
    void (*shadow)(RenderArgs, WfArgs, uint32_t);
    int ring, waves_per_simd;
    int cull; // the camera trace reads the cull boxes (1: references and leaves, 2: also subtrees)
    int packet; // the camera trace is a packet trace (needs a near child common to all camera rays)
    int lc;     // the tail kernel's leaf cull form (trav_round's LC; 0: none)
    // the shadow trace of a queue wf_shade appended in chunks (its dead entries skipped); null: the build's
    // wf_shade appends per iteration
    void (*shadow_dead)(RenderArgs, WfArgs, uint32_t) = nullptr;
};

// The trace configurations of the builds (traverse.hpp TraceDefaults), by what they restate.
namespace tc {
// build 0: the plain reference build (4-deep ring, vector loads, one level per load)
struct CameraRef : TraceDefaults { static constexpr int R = 4; static constexpr bool CAM = true; };
struct ClosestRef : TraceDefaults { static constexpr int R = 4; };
struct ShadowRef : TraceDefaults { static constexpr int R = 4; static constexpr bool SHADOW = true; };
// fat records, scalar loads of wave-uniform nodes / leaves, branch-light steps (build 9's; 15, 18, 42, 44)
struct Fat : TraceDefaults { static constexpr bool SC = true, FAT = true, BF = true; };
struct ClosestFat : Fat {};
struct ShadowFat : Fat { static constexpr bool SHADOW = true; };
// build 15's camera trace: cull boxes of references, leaves and subtrees
struct CameraCull : Fat { static constexpr bool CAM = true; static constexpr int CULL = 2; };
// + packed fixed-pad leaf cull records (build 26's; 40, 43)
struct ClosestFatLc : Fat { static constexpr int LC = 4; };
struct ShadowFatLc : ClosestFatLc { static constexpr bool SHADOW = true; };
// + the exact short split division by the ray's RN(1/d) in the shadow trace (43; 44 without the leaf cull)
struct ShadowFatLcFd : ShadowFatLc { static constexpr bool FD = true; };
struct ShadowFatFd : ShadowFat { static constexpr bool FD = true; };
struct ShadowFatFdDead : ShadowFatFd { static constexpr bool DEAD = true; };
// the same with the compressed leaf cull records (48 B per leaf instead of 96: three loads, not six)
struct ClosestFatLc5 : Fat { static constexpr int LC = 5; };
struct ShadowFatLc5Fd : ClosestFatLc5 { static constexpr bool SHADOW = true, FD = true; };
struct ShadowFatLc5FdDead : ShadowFatLc5Fd { static constexpr bool DEAD = true; };
// + the leaf exchange (traverse.hpp leaf_exchange: a divergent leaf's masked tests spread over the wave)
struct ClosestFatLc5Lx : ClosestFatLc5 { static constexpr bool LX = true; };
struct ShadowFatLc5FdLx : ShadowFatLc5Fd { static constexpr bool LX = true; };
struct ShadowFatLc5FdDeadLx : ShadowFatLc5FdDead { static constexpr bool LX = true; };
struct ClosestFatLc5LxD : ClosestFatLc5Lx { static constexpr bool LXD = true; };
struct ShadowFatLc5FdLxD : ShadowFatLc5FdLx { static constexpr bool LXD = true; };
struct ShadowFatLc5FdDeadLxD : ShadowFatLc5FdDeadLx { static constexpr bool LXD = true; };
struct ClosestFatLc5LxPerf : ClosestFatLc5Lx { static constexpr bool PC = true; };
struct ShadowFatLc5LxPerf : ClosestFatLc5LxPerf { static constexpr bool SHADOW = true; };
struct ClosestFatLc5Perf : ClosestFatLc5 { static constexpr bool PC = true; };
struct ShadowFatLc5Perf : ClosestFatLc5Perf { static constexpr bool SHADOW = true; };
// the performed-work counting instances (RenderArgs::perf_counters; measurement only)
struct ClosestFatLcPerf : ClosestFatLc { static constexpr bool PC = true; };
struct ShadowFatLcPerf : ShadowFatLc { static constexpr bool PC = true; };
struct ClosestFatPerf : ClosestFat { static constexpr bool PC = true; };
struct ShadowFatPerf : ShadowFat { static constexpr bool PC = true; };
// the counting build (SURVEY §8d work counters, diagnostics: RenderArgs::full_counters), 1 wave per SIMD
struct Count : TraceDefaults { static constexpr bool FULL = true; static constexpr int MINW = 1; };
struct CameraCount : Count { static constexpr bool CAM = true; };
struct ClosestCount : Count {};
struct ShadowCount : Count { static constexpr bool SHADOW = true; };
} // namespace tc

// (macro arguments with commas come parenthesised: CR_UNPAREN strips the parentheses)
#define CR_ID(...) __VA_ARGS__
#define CR_UNPAREN(x) CR_ID x
#define CR_WF3(CAM, CL, SH, ...) {wf_trace<CR_UNPAREN(CAM)>, wf_trace<CR_UNPAREN(CL)>, wf_trace<CR_UNPAREN(SH)>, __VA_ARGS__}
// The trace builds by number (cr_set_option "variant").  The default compile holds the plain reference
// build 0, build 15 (the packet camera trace's fallback for an eye on a split plane), 18 and 26 (round 2's
// and round 3's defaults), 40 / 42 (26 / 18 with the exact short division in the camera packet) and the
// defaults 43 / 44 (40 / 42 with it in the shadow trace too) and 49 (43 with the compressed leaf cull
// records).  The measured and superseded builds 1-14, 16, 17, 19-25, 27-39, 41, 45-48 and 51 are gone;
// DESIGN.md keeps their numbers.
struct WfBuild {
    int id;
    WfVariant v;
};
static const WfBuild kWf[] = {
    {0, CR_WF3((tc::CameraRef), (tc::ClosestRef), (tc::ShadowRef), 4, 8, 0, 0, 0)},
    // 15: fat records, scalar loads, branch-light steps; the camera trace skips the tests, leaves and
    // subtrees whose screen-space cull box excludes the sample
    {15, CR_WF3((tc::CameraCull), (tc::ClosestFat), (tc::ShadowFat), 8, 8, 2, 0, 0)},
    // 18: 15 whose camera rays traverse as one packet of 128 per wave (two per lane; wf_trace_packet)
    {18, {wf_trace_packet<8, 2>, wf_trace<tc::ClosestFat>, wf_trace<tc::ShadowFat>, 8, 8, 2, 1, 0}},
    // 26: 18 whose secondary closest and shadow traces skip the references a leaf's packed cull record
    // (leafcull.hpp: two normal groups, each a box and a normal cone) excludes for the ray; the tail
    // kernel culls the same way
    {26, {wf_trace_packet<8, 2>, wf_trace<tc::ClosestFatLc>, wf_trace<tc::ShadowFatLc>, 8, 8, 2, 1, 4}},
    // 40: 26 whose camera packet divides by the rays' RN(1/d) kept in VGPRs (FD; the packet's spills are
    //     outside its loops): camera trace 41.0 -> 37.7 ms, 363.1 -> 360.0 ms per pass
    {40, {wf_trace_packet<8, 2, false, true>, wf_trace<tc::ClosestFatLc>, wf_trace<tc::ShadowFatLc>, 8, 8, 2, 1, 4}},
    // 42: 18 with 40's camera packet (the default below LEAF_CULL_MIN_TRIS triangles)
    {42, {wf_trace_packet<8, 2, false, true>, wf_trace<tc::ClosestFat>, wf_trace<tc::ShadowFat>, 8, 8, 2, 1, 0}},
    // 43 / 44 (the defaults): 40 / 42 whose shadow trace divides by the ray's RN(1/d) in VGPRs too (FD;
    //     no spills at 8 waves once the stack-overflow pointer and the query count stopped occupying
    //     VGPRs): 357.5 / 355.3 vs 358.4 / 358.1 ms per pass, nanobox 162.4 vs 163.7 ms (shadow 30.7 -> 29.9)
    {43, {wf_trace_packet<8, 2, false, true>, wf_trace<tc::ClosestFatLc>, wf_trace<tc::ShadowFatLcFd>, 8, 8, 2, 1, 4}},
    {44, {wf_trace_packet<8, 2, false, true>, wf_trace<tc::ClosestFat>, wf_trace<tc::ShadowFatFd>, 8, 8, 2, 1, 0,
          wf_trace<tc::ShadowFatFdDead>}},
    // 49: 43 whose secondary closest, shadow and tail traces read the compressed leaf cull records
    //     (leafcull.hpp LC_RECC: boxes on the scene's 16-bit grid, octahedral axes, half constants)
    {49, {wf_trace_packet<8, 2, false, true>, wf_trace<tc::ClosestFatLc5>, wf_trace<tc::ShadowFatLc5Fd>, 8, 8, 2, 1, 5,
          wf_trace<tc::ShadowFatLc5FdDead>}},
    // 53 / 54 (54: the default, round 6): 49 whose shadow trace (53) or shadow and secondary closest traces
    //     (54) test a divergent leaf round's masked references with the whole wave (the leaf exchange,
    //     traverse.hpp leaf_exchange): sponza 2315 -> 2348 (53) / 2362 (54) Mray/s, shadow
    //     trace 39.2 -> 38.3 ms, closest 68.9 -> 67.2 ms per launch beside it.  Measured and removed: the
    //     shadow exchange at 7 waves per SIMD (no spills then; 2305 Mray/s) and the lane index recomputed
    //     per use instead of held in a register (no spills at 8 waves; 2300 / 2330 Mray/s)
    {53, {wf_trace_packet<8, 2, false, true>, wf_trace<tc::ClosestFatLc5>, wf_trace<tc::ShadowFatLc5FdLx>, 8, 8, 2, 1, 5,
          wf_trace<tc::ShadowFatLc5FdDeadLx>}},
    {54, {wf_trace_packet<8, 2, false, true>, wf_trace<tc::ClosestFatLc5Lx>, wf_trace<tc::ShadowFatLc5FdLx>, 8, 8, 2, 1, 5,
          wf_trace<tc::ShadowFatLc5FdDeadLx>}},
    // 59 (the default, round 6): 54 with the exchange's prefix by a DPP scan (LXD: six row-shift / row-broadcast
    //     adds instead of six bit-sliced ballots with their mbcnt pairs): 2348 -> 2395 Mray/s, shadow trace
    //     38.4 -> 37.6 ms, closest 67.3 -> 65.5 ms (three interleaved rounds)
    {59, {wf_trace_packet<8, 2, false, true>, wf_trace<tc::ClosestFatLc5LxD>, wf_trace<tc::ShadowFatLc5FdLxD>, 8, 8, 2, 1, 5,
          wf_trace<tc::ShadowFatLc5FdDeadLxD>}},
};
static const int kNumWf = (int)(sizeof(kWf) / sizeof(kWf[0]));
// the build numbered `variant`, or null when it is not compiled in
static const WfVariant *wf_build(int variant) {
    for (int i = 0; i < kNumWf; i++)
        if (kWf[i].id == variant) return &kWf[i].v;
    return nullptr;
}
static const WfVariant &wf_build_or_ref(int variant) {
    const WfVariant *v = wf_build(variant);
    return v ? *v : kWf[0].v;
}
// Builds 26 and 18 with the performed-work counts (RenderArgs::perf_counters; measurement only)
static const WfVariant kWfPerf26 = {wf_trace_packet<8, 2, true>, wf_trace<tc::ClosestFatLcPerf>,
                                    wf_trace<tc::ShadowFatLcPerf>, 8, 8, 2, 1, 4};
static const WfVariant kWfPerf18 = {wf_trace_packet<8, 2, true>, wf_trace<tc::ClosestFatPerf>,
                                    wf_trace<tc::ShadowFatPerf>, 8, 8, 2, 1, 0};
// ... and builds 40 / 42 (26 / 18 with the FD camera packet: the same work, the division shortened)
static const WfVariant kWfPerf40 = {wf_trace_packet<8, 2, true, true>, wf_trace<tc::ClosestFatLcPerf>,
                                    wf_trace<tc::ShadowFatLcPerf>, 8, 8, 2, 1, 4};
static const WfVariant kWfPerf42 = {wf_trace_packet<8, 2, true, true>, wf_trace<tc::ClosestFatPerf>,
                                    wf_trace<tc::ShadowFatPerf>, 8, 8, 2, 1, 0};
// ... and build 49 (the compressed leaf cull records: the same work, half the mask bytes)
static const WfVariant kWfPerf49 = {wf_trace_packet<8, 2, true, true>, wf_trace<tc::ClosestFatLc5Perf>,
                                    wf_trace<tc::ShadowFatLc5Perf>, 8, 8, 2, 1, 5};
// ... and the leaf-exchange builds 53 / 54 (59 counts through 54's: its DPP prefix does the same work)
static const WfVariant kWfPerf53 = {wf_trace_packet<8, 2, true, true>, wf_trace<tc::ClosestFatLc5Perf>,
                                    wf_trace<tc::ShadowFatLc5LxPerf>, 8, 8, 2, 1, 5};
static const WfVariant kWfPerf54 = {wf_trace_packet<8, 2, true, true>, wf_trace<tc::ClosestFatLc5LxPerf>,
                                    wf_trace<tc::ShadowFatLc5LxPerf>, 8, 8, 2, 1, 5};
// (43 / 44 count through 40 / 42's instances: their shadow trace's short division does the same work)
bool wf_perf_available(int variant) {
    return variant == 18 || variant == 26 || variant == 40 || variant == 42 || variant == 43 || variant == 44 ||
           variant == 49 || variant == 53 || variant == 54 || variant == 59;
}
static const WfVariant &perf_variant(int variant) {
    return variant == 18 ? kWfPerf18
           : variant == 49 ? kWfPerf49
           : variant == 53 ? kWfPerf53
           : (variant == 54 || variant == 59) ? kWfPerf54
           : (variant == 40 || variant == 43) ? kWfPerf40
           : (variant == 42 || variant == 44) ? kWfPerf42
                                              : kWfPerf26;
}
static const WfVariant kWfCount = {wf_trace<tc::CameraCount>, wf_trace<tc::ClosestCount>, wf_trace<tc::ShadowCount>,
                                   8, 4, 0, 0, 0};
// one past the largest build number (option validation)
int num_wf_variants() {
    int m = 0;
    for (int i = 0; i < kNumWf; i++) m = kWf[i].id + 1 > m ? kWf[i].id + 1 : m;
    return m;
}
// The camera-ray trace of a variant; the packet trace (build 17) needs a near child common to all
// camera rays, which an eye lying exactly on a split plane breaks: build 15's then.
static void (*camera_kernel(const WfVariant &v, const RenderArgs &A))(RenderArgs, WfArgs, uint32_t) {
    return (v.packet && A.eye_on_split) ? wf_build(15)->camera : v.camera;
}
// The chunk's camera rays come from the packet trace itself (WfArgs::cam_fused) when the ctx asks for it
// (W.cam_fused on entry), the camera kernel is the packet trace, generation 1 runs as its own launches
// (not handed to wf_tail, which reads wf_camera's rays) and wf_shade derives generation 1's RNG state.
static bool camera_fuses(const WfVariant &v, const RenderArgs &A, const WfArgs &W) {
    return W.cam_fused && v.packet && !A.eye_on_split && camera_state_lean(W);
}
bool wf_variant_culls(int variant) { return wf_build(variant) && wf_build(variant)->cull; }
bool wf_variant_available(int variant) { return wf_build(variant) != nullptr; }

// One thread per leaf reference: its cull box for this render's camera (camcull.hpp),
// from the record's A, e1, e2 -- the floats the triangle test uses.  Boxes
// nrefs..nrefs+3 are empty (the four-box scalar loads of uniform leaves read past a
// leaf's end, also from an empty leaf's `first` == nrefs).  Samples lie in [0, xres] x [0, yres] (global pixel coordinates).
__global__ void __launch_bounds__(256) cam_cull_kernel(RenderArgs A, uint32_t nrefs, float4 *boxes) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nrefs + 4) return;
    if (r >= nrefs) {
        boxes[r] = make_float4(INFINITY, -INFINITY, INFINITY, -INFINITY);
        return;
    }
    CullCam cc;
    for (int i = 0; i < 12; i++) cc.cam[i] = A.cam[i];
    cc.xres = (float)A.xres;
    cc.yres = (float)A.yres;
    const float4 *q = A.S.recs + (size_t)REC_STRIDE * r;
    const float4 a = q[0], e1 = q[1], e2 = q[2];
    const float av[3] = {a.x, a.y, a.z}, e1v[3] = {e1.x, e1.y, e1.z}, e2v[3] = {e2.x, e2.y, e2.z};
    float b[4];
    cam_cull_box(av, e1v, e2v, cc, b);
    boxes[r] = make_float4(b[0], b[1], b[2], b[3]);
}

// One thread per node: a leaf's box is the union of its references' boxes (a sample
// outside it is outside every one of them: the whole leaf loop is skipped).
__global__ void __launch_bounds__(256) cam_cull_leaf_kernel(RenderArgs A, const float4 *boxes, float4 *node_boxes) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= A.S.n_nodes) return;
    const uint2 nd = A.S.nodes[i];
    float4 u = make_float4(-INFINITY, INFINITY, -INFINITY, INFINITY);
    if ((nd.y & 3u) == 3u) {
        u = make_float4(INFINITY, -INFINITY, INFINITY, -INFINITY);
        for (uint32_t j = 0, n = nd.y >> 2; j < n; j++) {
            const float4 b = boxes[nd.x + j];
            u = make_float4(fminf(u.x, b.x), fmaxf(u.y, b.y), fminf(u.z, b.z), fmaxf(u.w, b.w));
        }
    }
    node_boxes[i] = u;
}

// One thread per inner node of one level: the union of its children's boxes.
__global__ void __launch_bounds__(256) cam_cull_inner_kernel(RenderArgs A, const uint32_t *ids, uint32_t n,
                                                             float4 *node_boxes) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t id = ids[i], ch = A.S.nodes[id].y >> 2;
    const float4 a = node_boxes[ch], b = node_boxes[ch + 1];
    node_boxes[id] = make_float4(fminf(a.x, b.x), fmaxf(a.y, b.y), fminf(a.z, b.z), fmaxf(a.w, b.w));
}

int launch_cam_cull(const RenderArgs &A, uint32_t nrefs, float4 *boxes, float4 *node_boxes, const uint32_t *levels,
                    const uint32_t (*level_off)[2], int nlevels, hipStream_t st) {
    const uint32_t n = nrefs + 4;
    hipLaunchKernelGGL(cam_cull_kernel, dim3((n + 255) / 256), dim3(256), 0, st, A, nrefs, boxes);
    hipLaunchKernelGGL(cam_cull_leaf_kernel, dim3((A.S.n_nodes + 255) / 256), dim3(256), 0, st, A, boxes, node_boxes);
    for (int l = 0; l < nlevels; l++)
        if (level_off[l][1])
            hipLaunchKernelGGL(cam_cull_inner_kernel, dim3((level_off[l][1] + 255) / 256), dim3(256), 0, st, A,
                               levels + level_off[l][0], level_off[l][1], node_boxes);
    return (int)hipGetLastError();
}

void wf_trace_geometry(int variant, int num_cus, uint32_t &block, uint32_t &blocks) {
    const WfVariant &v = wf_build_or_ref(variant);
    block = 256;
    blocks = (uint32_t)(num_cus > 0 ? num_cus : 256) * (uint32_t)v.waves_per_simd; // 4 SIMDs, 4 waves/block
}

// Sorts the queue of n rays whose keys wf_shade wrote into key / perm set `set`
// (0 shadow, 1 closest); returns the permutation for the trace kernel (nullptr:
// trace in queue order).
// pixel: the queue's keys are pixel keys (wf_shade of a generation below world_keys), which
// need fewer bits than world keys -- one digit pass fewer for a rank's share of a frame
static const uint32_t *order_queue(const WfArgs &W, int set, uint32_t n, hipStream_t st, int &err, bool pixel) {
    if (!W.sort || err || n < W.sort_min || (W.measure_skip & 2u)) return nullptr;
    uint32_t *keys[2] = {W.key[set][0], W.key[set][1]}, *vals[2] = {W.perm[set][0], W.perm[set][1]};
    size_t tb = W.sort_tmp_bytes;
    const int bits = pixel ? W.key_bits_pixel : (set == 0 ? W.key_bits_s : W.key_bits);
    // (the trace reads the permutation only: the last pass writes no keys)
    const int sel = sort_queue(keys, vals, n, bits, W.sort_tmp, tb, st, false, true, false);
    if (sel < 0) {
        err = (int)hipErrorUnknown;
        return nullptr;
    }
    return vals[sel];
}

// Records a (start, stop) event pair around one trace launch when te is given.
static int trace_event(TraceEvents *te, hipStream_t st, int kind, bool start) {
    if (!te) return 0;
    if (start) {
        if (te->n == te->cap) {
            const int cap = te->cap ? 2 * te->cap : 64;
            hipEvent_t *ev = new hipEvent_t[2 * (size_t)cap];
            int *kd = new int[cap];
            for (int i = 0; i < 2 * te->cap; i++) ev[i] = te->ev[i];
            for (int i = 0; i < te->cap; i++) kd[i] = te->kind[i];
            for (int i = 2 * te->cap; i < 2 * cap; i++)
                if (int e = (int)hipEventCreate(&ev[i])) {
                    for (int j = 2 * te->cap; j < i; j++) hipEventDestroy(ev[j]);
                    delete[] ev;
                    delete[] kd;
                    return e;
                }
            delete[] te->ev;
            delete[] te->kind;
            te->ev = ev;
            te->kind = kd;
            te->cap = cap;
        }
        te->kind[te->n] = kind;
        return (int)hipEventRecord(te->ev[2 * te->n], st);
    }
    return (int)hipEventRecord(te->ev[2 * te->n++ + 1], st);
}

// Tail kernel builds: lean and counting; 4 waves/SIMD (the path bodies need more
// registers than the trace kernels' 64).
enum { TAIL_MINW = 4 };
// lean tail launch at `waves` per SIMD (option "wf_tail_waves"; 4, 5 or 6)
template <int LC> static void launch_tail_lean(int waves, uint32_t blk, int num_cus, size_t lds, hipStream_t s,
                                               const RenderArgs &A, const WfArgs &W, uint32_t g) {
    const uint32_t cus = (uint32_t)(num_cus > 0 ? num_cus : 256);
    if (waves == 5) hipLaunchKernelGGL((wf_tail<false, 8, 5, LC>), dim3(cus * 5), dim3(blk), lds, s, A, W, g);
    else if (waves == 6) hipLaunchKernelGGL((wf_tail<false, 8, 6, LC>), dim3(cus * 6), dim3(blk), lds, s, A, W, g);
    else hipLaunchKernelGGL((wf_tail<false, 8, TAIL_MINW, LC>), dim3(cus * TAIL_MINW), dim3(blk), lds, s, A, W, g);
}
void wf_tail_geometry(int num_cus, uint32_t &block, uint32_t &blocks) {
    block = 256;
    blocks = (uint32_t)(num_cus > 0 ? num_cus : 256) * TAIL_MINW;
}

// Grid of the grid-stride wf_shade: every block resident at once.  wf_shade needs 71 VGPRs,
// so a SIMD holds 7 of its waves, not 8: with 8 blocks per CU the eighth started only when
// another had finished its whole share (the grid-stride loop gives every block the same).
// The occupancy is queried for the instantiation actually launched (CH: the chunked appends, whose extra
// chunk state may need more registers than the per-iteration form), so every block of the grid is resident
// at once -- a chunked block owns one contiguous span of the queue, and a block that started late would
// run its whole span after the others had finished.
template <int MINW, bool CH, int BS> static int shade_occupancy() {
    int b = 0;
    const hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, wf_shade<MINW, CH, BS>, BS, 0);
    return e != hipSuccess || b <= 0 ? 8 * 256 / BS : b;
}
static uint32_t shade_grid(int num_cus, int waves, int bs = 256, bool chunked = false) {
    static std::atomic<int> per_cu[2][3][2] = {};
    const int i = waves == 8 ? 1 : 0, j = bs == 1024 ? 2 : bs == 512 ? 1 : 0, k = chunked ? 1 : 0;
    int b = per_cu[i][j][k].load();
    if (!b) {
        if (k) b = j == 2 ? shade_occupancy<8, true, 1024>() : i ? shade_occupancy<8, true, 256>() : shade_occupancy<1, true, 256>();
        else if (j == 2) b = i ? shade_occupancy<8, false, 1024>() : shade_occupancy<1, false, 1024>();
        else if (j == 1) b = i ? shade_occupancy<8, false, 512>() : shade_occupancy<1, false, 512>();
        else b = i ? shade_occupancy<8, false, 256>() : shade_occupancy<1, false, 256>();
        per_cu[i][j][k].store(b);
    }
    return (uint32_t)(num_cus > 0 ? num_cus : 256) * (uint32_t)std::min(b, 8 * 256 / bs);
}
// Blocks of any chunked wf_shade launch at most (the spare queue slots hold every block's partial last chunk):
// the larger of the 256- and 1024-thread chunked grids
uint32_t wf_shade_blocks(int num_cus, int shade_waves) {
    return std::max(shade_grid(num_cus, shade_waves == 8 ? 8 : 6, 256, true), shade_grid(num_cus, 8, 1024, true));
}
// wf_shade at the ctx's option "wf_shade_waves" (8, the default since round 4; or 6)
// The append chunk of a wf_shade launch over nin rays (WfArgs::app_chunk): a power of two giving each
// block about 16 chunks per queue, so the dead entries stay a few percent of the queue; 0 (one atomic
// per block iteration) for queues that short, and at most what the queues' spare slots hold for every
// block's partial last chunk.  Only for queues traced in append order (W.sort 0: scenes below
// SORT_MIN_TRIS): round 5, two interleaved rounds, cornell_box 13,002 / 13,000 -> 14,331 / 14,298 Mray/s;
// on sorted queues (sponza stand-in) wf_shade gains 9 % but the shadow trace loses 1.7 % -- the chunks
// change the order among equal keys -- 2278.5 / 2278.7 -> 2274.8 / 2270.4
static uint32_t shade_app_chunk(const WfArgs &W, uint32_t nin, int num_cus) {
    if (!W.qspare) return 0u;
    const uint32_t grid = wf_shade_blocks(num_cus, W.shade_waves);
    const uint32_t want = nin / (grid * 16u), cap = W.qspare / grid;
    if (W.app_force) return W.app_force <= cap ? W.app_force : 0u;
    if (W.sort) return 0u;
    uint32_t c = 256u;
    while (c * 2u <= want && c * 2u <= cap && c < 4096u) c *= 2u;
    return c <= want && c <= cap ? c : 0u;
}
static void launch_shade(const RenderArgs &A, const WfArgs &W, uint32_t g, int num_cus, hipStream_t st) {
    // (a chunk holds at least one iteration's appends: 1024-thread blocks need chunks of 1024 or more)
    if (W.app_chunk >= 1024 && W.shade_block == 1024 && W.shade_waves == 8)
        hipLaunchKernelGGL((wf_shade<8, true, 1024>), dim3(shade_grid(num_cus, 8, 1024, true)), dim3(1024), 0, st, A, W, g);
    else if (W.app_chunk && W.shade_waves == 8)
        hipLaunchKernelGGL((wf_shade<8, true>), dim3(shade_grid(num_cus, 8, 256, true)), dim3(256), 0, st, A, W, g);
    else if (W.app_chunk)
        hipLaunchKernelGGL((wf_shade<1, true>), dim3(shade_grid(num_cus, 6, 256, true)), dim3(256), 0, st, A, W, g);
    else if (W.shade_block == 1024 && W.shade_waves == 8)
        hipLaunchKernelGGL((wf_shade<8, false, 1024>), dim3(shade_grid(num_cus, 8, 1024)), dim3(1024), 0, st, A, W, g);
    else if (W.shade_block == 1024)
        hipLaunchKernelGGL((wf_shade<1, false, 1024>), dim3(shade_grid(num_cus, 6, 1024)), dim3(1024), 0, st, A, W, g);
    else if (W.shade_block == 512 && W.shade_waves == 8)
        hipLaunchKernelGGL((wf_shade<8, false, 512>), dim3(shade_grid(num_cus, 8, 512)), dim3(512), 0, st, A, W, g);
    else if (W.shade_block == 512)
        hipLaunchKernelGGL((wf_shade<1, false, 512>), dim3(shade_grid(num_cus, 6, 512)), dim3(512), 0, st, A, W, g);
    else if (W.shade_waves == 8)
        hipLaunchKernelGGL(wf_shade<8>, dim3(shade_grid(num_cus, 8)), dim3(256), 0, st, A, W, g);
    else
        hipLaunchKernelGGL(wf_shade<1>, dim3(shade_grid(num_cus, 6)), dim3(256), 0, st, A, W, g);
}

int launch_wavefront_chunk(const RenderArgs &A, const WfArgs &W0, int num_cus, hipStream_t st, const WfStreams &ss,
                           TraceEvents *te) {
    WfArgs W = W0;
    const WfVariant &v = A.full_counters ? kWfCount
                         : A.perf_counters ? perf_variant(A.variant)
                                           : wf_build_or_ref(A.variant);
    uint32_t blk, blocks, tblk, tblocks;
    wf_trace_geometry(A.full_counters ? -1 : A.variant, num_cus, blk, blocks);
    const uint32_t cblocks = blocks, sblocks = blocks;
    wf_tail_geometry(num_cus, tblk, tblocks);
    if (W.gstride < blk * blocks || W.gstride < tblk * tblocks) return (int)hipErrorInvalidValue;
    if (blk != 256) return (int)hipErrorInvalidConfiguration; // (wf_trace's per-wave LDS of the leaf exchange)
    const size_t lds =
        (size_t)v.ring * blk * sizeof(uint2);
    const uint32_t sgrid = (uint32_t)(num_cus > 0 ? num_cus : 256) * 8; // grid-stride phases
    int err = 0;
    // the rest of the chunk from closest queue g on, in one launch
    auto tail = [&](uint32_t g, hipStream_t s, WfArgs Wt) {
        const size_t tlds = (size_t)8 * tblk * sizeof(uint2);
        Wt.order = nullptr;
        if ((err = trace_event(te, s, TK_TAIL, true))) return;
        if (A.full_counters)
            hipLaunchKernelGGL((wf_tail<true, 8, TAIL_MINW>), dim3(tblocks), dim3(tblk), tlds, s, A, Wt, g);
        else if (A.perf_counters && v.lc == 5)
            hipLaunchKernelGGL((wf_tail<false, 8, TAIL_MINW, 5, true>), dim3(tblocks), dim3(tblk), tlds, s, A, Wt, g);
        else if (A.perf_counters && v.lc == 4)
            hipLaunchKernelGGL((wf_tail<false, 8, TAIL_MINW, 4, true>), dim3(tblocks), dim3(tblk), tlds, s, A, Wt, g);
        else if (A.perf_counters)
            hipLaunchKernelGGL((wf_tail<false, 8, TAIL_MINW, 0, true>), dim3(tblocks), dim3(tblk), tlds, s, A, Wt, g);
        else if (v.lc == 5)
            launch_tail_lean<5>(Wt.tail_waves, tblk, num_cus, tlds, s, A, Wt, g);
        else if (v.lc == 4)
            launch_tail_lean<4>(Wt.tail_waves, tblk, num_cus, tlds, s, A, Wt, g);
        else
            launch_tail_lean<0>(Wt.tail_waves, tblk, num_cus, tlds, s, A, Wt, g);
        err = trace_event(te, s, TK_TAIL, false);
    };
    // closest trace of generation g on stream s; its stack overflow rows are the
    // second half of gstack when it runs beside a shadow trace
    auto closest = [&](uint32_t g, hipStream_t s, const uint32_t *order, uint2 *gstack) {
        WfArgs Wc = W;
        Wc.order = order;
        Wc.gstack = gstack;
        const int kind = g == 1 ? TK_CAMERA : TK_CLOSEST;
        if ((err = trace_event(te, s, kind, true))) return;
        hipLaunchKernelGGL(g == 1 ? camera_kernel(v, A) : v.closest, dim3(g == 1 ? blocks : cblocks), dim3(blk),
                           lds, s, A, Wc, g);
        err = trace_event(te, s, kind, false);
    };
    W.cam_fused = camera_fuses(v, A, W) ? 1 : 0;
    if (!W.cam_fused) hipLaunchKernelGGL(wf_camera, dim3(sgrid), dim3(256), 0, st, A, W);
    if (W.P < W.tail_min) {
        tail(1, st, W);
        return err ? err : (int)hipGetLastError();
    }
    closest(1, st, nullptr, W.gstack); // camera rays: path order is already coherent
    uint32_t nin = W.P; // rays of closest queue g (generation 1: one per path)
    for (uint32_t g = 1; g <= (uint32_t)A.K && !err; g++) {
        W.app_chunk = v.shadow_dead ? shade_app_chunk(W, nin, num_cus) : 0u;
        if (te && W.app_chunk) te->chunked++;
        launch_shade(A, W, g, num_cus, st);
        const bool dead = W.app_chunk != 0u; // shadow queue g may hold dead entries
        W.app_chunk = 0u;
        uint32_t cnt[2] = {0u, 0u}; // shadow queue g, closest queue g + 1
        if ((err = (int)hipMemcpyAsync(&cnt[0], W.cnt + WF_G + g, 4, hipMemcpyDeviceToHost, st)) ||
            (err = (int)hipMemcpyAsync(&cnt[1], W.cnt + g + 1, 4, hipMemcpyDeviceToHost, st)) ||
            (err = (int)hipStreamSynchronize(st)))
            break;
        const uint32_t nc = g < (uint32_t)A.K ? cnt[1] : 0u;
        nin = nc;
        const bool next = nc >= W.tail_min && nc > 0; // closest g + 1 as its own launch, beside shadow g
        const bool pixel = !W.leaf_keys && !(W.world_keys && g >= (uint32_t)W.world_keys); // wf_shade's key choice
        const uint32_t *order_s = (g > 1 || (W.sort_g1 & 1u)) ? order_queue(W, 0, cnt[0], st, err, pixel) : nullptr;
        const uint32_t *order_c = (next && (g > 1 || (W.sort_g1 & 2u))) ? order_queue(W, 1, nc, st, err, pixel) : nullptr;
        if (err) break;
        // overlapped tail: the rest of the chunk starts beside this generation's shadow trace, tracing
        // its own paths' shadow rays of generation g first (the paths that end at g stay with
        // wf_trace / wf_resolve); only for scenes with lights -- a hit whose NEE query was answered
        // without a trace (nee_skip) has no shadow ray, and the tail reads its NO_SLOT as "nothing to trace"
        const bool overlap = !next && nc > 0 && W.tail_overlap && A.S.nlights > 0;
        if (next || overlap) {
            if ((err = (int)hipEventRecord(ss.fork, st)) || (err = (int)hipStreamWaitEvent(ss.side, ss.fork, 0))) break;
            if (next) {
                closest(g + 1, ss.side, order_c, W.gstack2);
            } else {
                WfArgs Wt = W;
                Wt.gstack = W.gstack2;
                Wt.tail_shadow_gen = g;
                tail(g + 1, ss.side, Wt);
            }
            if (err) break;
        }
        W.order = order_s;
        W.ended_only = overlap ? 1u : 0u;
        if ((err = trace_event(te, st, TK_SHADOW, true))) break;
        hipLaunchKernelGGL(dead ? v.shadow_dead : v.shadow, dim3(sblocks), dim3(blk), lds, st, A, W, g);
        if ((err = trace_event(te, st, TK_SHADOW, false))) break;
        if (!(W.measure_skip & 1u)) hipLaunchKernelGGL(wf_resolve, dim3(sgrid), dim3(256), 0, st, A, W, g);
        W.ended_only = 0u;
        if (next || overlap)
            if ((err = (int)hipEventRecord(ss.join, ss.side)) || (err = (int)hipStreamWaitEvent(st, ss.join, 0)))
                break;
        if (!next) {
            if (nc > 0 && !overlap) tail(g + 1, st, W);
            break;
        }
    }
    return err ? err : (int)hipGetLastError();
}

int run_wavefront_lanes(const RenderArgs &A, WfLane *L, int nl, int num_cus, hipStream_t st, TraceEvents *te) {
    const WfVariant &v = A.full_counters ? kWfCount
                         : A.perf_counters ? perf_variant(A.variant)
                                           : wf_build_or_ref(A.variant);
    uint32_t blk, blocks, tblk, tblocks;
    wf_trace_geometry(A.full_counters ? -1 : A.variant, num_cus, blk, blocks);
    const uint32_t cblocks = blocks, sblocks = blocks;
    wf_tail_geometry(num_cus, tblk, tblocks);
    for (int i = 0; i < nl; i++)
        if (L[i].W.gstride < blk * blocks || L[i].W.gstride < tblk * tblocks) return (int)hipErrorInvalidValue;
    if (blk != 256) return (int)hipErrorInvalidConfiguration; // (wf_trace's per-wave LDS of the leaf exchange)
    const size_t lds =
        (size_t)v.ring * blk * sizeof(uint2);
    const uint32_t sgrid = (uint32_t)(num_cus > 0 ? num_cus : 256) * 8;
    int err = 0;
    struct Run {
        WfArgs W;
        uint32_t g = 0;
        int phase = 0; // 0 idle, 1 shade g, 2 wait for queue lengths of g
        bool past_camera = false;
    } run[2];
    auto tail = [&](WfLane &ln, WfArgs &W, uint32_t g) {
        const size_t tlds = (size_t)8 * tblk * sizeof(uint2);
        W.order = nullptr;
        if ((err = trace_event(te, ln.st, TK_TAIL, true))) return;
        if (A.full_counters)
            hipLaunchKernelGGL((wf_tail<true, 8, TAIL_MINW>), dim3(tblocks), dim3(tblk), tlds, ln.st, A, W, g);
        else if (A.perf_counters && v.lc == 5)
            hipLaunchKernelGGL((wf_tail<false, 8, TAIL_MINW, 5, true>), dim3(tblocks), dim3(tblk), tlds, ln.st, A, W, g);
        else if (A.perf_counters && v.lc == 4)
            hipLaunchKernelGGL((wf_tail<false, 8, TAIL_MINW, 4, true>), dim3(tblocks), dim3(tblk), tlds, ln.st, A, W, g);
        else if (A.perf_counters)
            hipLaunchKernelGGL((wf_tail<false, 8, TAIL_MINW, 0, true>), dim3(tblocks), dim3(tblk), tlds, ln.st, A, W, g);
        else if (v.lc == 5)
            hipLaunchKernelGGL((wf_tail<false, 8, TAIL_MINW, 5>), dim3(tblocks), dim3(tblk), tlds, ln.st, A, W, g);
        else if (v.lc == 4)
            hipLaunchKernelGGL((wf_tail<false, 8, TAIL_MINW, 4>), dim3(tblocks), dim3(tblk), tlds, ln.st, A, W, g);
        else
            hipLaunchKernelGGL((wf_tail<false, 8, TAIL_MINW>), dim3(tblocks), dim3(tblk), tlds, ln.st, A, W, g);
        err = trace_event(te, ln.st, TK_TAIL, false);
    };
    auto closest = [&](const WfArgs &W, uint32_t g, hipStream_t s, const uint32_t *order, uint2 *gstack) {
        WfArgs Wc = W;
        Wc.order = order;
        Wc.gstack = gstack;
        const int kind = g == 1 ? TK_CAMERA : TK_CLOSEST;
        if ((err = trace_event(te, s, kind, true))) return;
        hipLaunchKernelGGL(g == 1 ? camera_kernel(v, A) : v.closest, dim3(g == 1 ? blocks : cblocks), dim3(blk),
                           lds, s, A, Wc, g);
        err = trace_event(te, s, kind, false);
    };
    auto shade = [&](WfLane &ln, Run &r) { // wf_shade(g), then the queue lengths to the host, async
        launch_shade(A, r.W, r.g, num_cus, ln.st);
        if ((err = (int)hipMemcpyAsync(&ln.hcnt[0], r.W.cnt + WF_G + r.g, 4, hipMemcpyDeviceToHost, ln.st)) ||
            (err = (int)hipMemcpyAsync(&ln.hcnt[1], r.W.cnt + r.g + 1, 4, hipMemcpyDeviceToHost, ln.st)) ||
            (err = (int)hipEventRecord(ln.ready, ln.st)))
            return;
        r.phase = 2;
    };
    auto start = [&](WfLane &ln, Run &r, uint32_t w0, uint32_t P) {
        r.W = ln.W;
        r.W.w0 = w0;
        r.W.P = P;
        r.g = 1;
        r.past_camera = false;
        if ((err = (int)hipMemsetAsync(r.W.cnt, 0, WF_CNT * sizeof(uint32_t), ln.st))) return;
        r.W.cam_fused = camera_fuses(v, A, r.W) ? 1 : 0;
        if (!r.W.cam_fused) hipLaunchKernelGGL(wf_camera, dim3(sgrid), dim3(256), 0, ln.st, A, r.W);
        if (P < r.W.tail_min) {
            tail(ln, r.W, 1);
            r.phase = 0;
            r.past_camera = true;
            return;
        }
        closest(r.W, 1, ln.st, nullptr, r.W.gstack); // camera rays: path order is already coherent
        if (!err) shade(ln, r);
    };
    // one generation's traces once its queue lengths are on the host; false: not yet
    auto advance = [&](WfLane &ln, Run &r) -> bool {
        const hipError_t q = hipEventQuery(ln.ready);
        if (q == hipErrorNotReady) return false;
        if (q != hipSuccess) {
            err = (int)q;
            return true;
        }
        r.past_camera = true;
        const uint32_t g = r.g, ns = ln.hcnt[0];
        const uint32_t nc = g < (uint32_t)A.K ? ln.hcnt[1] : 0u;
        const bool next = nc >= r.W.tail_min && nc > 0;
        const bool pixel = !r.W.leaf_keys && !(r.W.world_keys && g >= (uint32_t)r.W.world_keys); // wf_shade's key choice
        const uint32_t *order_s = order_queue(r.W, 0, ns, ln.st, err, pixel);
        const uint32_t *order_c = next ? order_queue(r.W, 1, nc, ln.st, err, pixel) : nullptr;
        if (err) return true;
        if (next) {
            if ((err = (int)hipEventRecord(ln.fork, ln.st)) || (err = (int)hipStreamWaitEvent(ln.side, ln.fork, 0)))
                return true;
            closest(r.W, g + 1, ln.side, order_c, r.W.gstack2);
            if (err) return true;
        }
        WfArgs Ws = r.W;
        Ws.order = order_s;
        if ((err = trace_event(te, ln.st, TK_SHADOW, true))) return true;
        hipLaunchKernelGGL(v.shadow, dim3(sblocks), dim3(blk), lds, ln.st, A, Ws, g);
        if ((err = trace_event(te, ln.st, TK_SHADOW, false))) return true;
        hipLaunchKernelGGL(wf_resolve, dim3(sgrid), dim3(256), 0, ln.st, A, r.W, g);
        if (next) {
            if ((err = (int)hipEventRecord(ln.join, ln.side)) || (err = (int)hipStreamWaitEvent(ln.st, ln.join, 0)))
                return true;
            r.g = g + 1;
            shade(ln, r);
        } else {
            if (nc > 0) tail(ln, r.W, g + 1);
            r.phase = 0;
        }
        return true;
    };
    // lanes > 0 start after the work already queued on st
    for (int i = 1; i < nl && !err; i++)
        if (!(err = (int)hipEventRecord(L[i].ready, st))) err = (int)hipStreamWaitEvent(L[i].st, L[i].ready, 0);
    uint32_t next_w0 = 0;
    while (!err) {
        bool progress = false, busy = false;
        for (int i = 0; i < nl && !err; i++) {
            if (run[i].phase == 0) {
                bool others_past = true;
                for (int j = 0; j < nl; j++)
                    if (j != i && run[j].phase != 0 && !run[j].past_camera) others_past = false;
                if (next_w0 < A.n_work && others_past) {
                    const uint32_t P = min(L[i].W.P, A.n_work - next_w0);
                    start(L[i], run[i], next_w0, P);
                    next_w0 += P;
                    progress = true;
                }
            } else {
                progress = advance(L[i], run[i]) || progress;
            }
            busy = busy || run[i].phase != 0;
        }
        if (!busy && next_w0 >= A.n_work) break;
        if (!progress) std::this_thread::yield();
    }
    // st waits for the other lanes' last work
    for (int i = 1; i < nl && !err; i++)
        if (!(err = (int)hipEventRecord(L[i].ready, L[i].st))) err = (int)hipStreamWaitEvent(st, L[i].ready, 0);
    return err ? err : (int)hipGetLastError();
}

// Bytes of sort workspace for queues of up to n rays (temp storage only).
size_t wf_sort_tmp_bytes(uint32_t n, int key_bits) {
    size_t tb = 0;
    uint32_t *k[2] = {nullptr, nullptr}, *v[2] = {nullptr, nullptr};
    sort_queue(k, v, n, key_bits, nullptr, tb, nullptr, false);
    return tb;
}

} // namespace cr
