// traverse.hpp -- the resumable kd traversal of the wavefront trace kernels and the tail kernel
// (wavefront.hip).
#pragma once
#include "leafcull.hpp"
#include "render_common.hpp"

namespace cr {

enum : uint32_t {
    ST_NEED_WORK = 0, // lane has no query: take the next item / ray
    ST_CLOSEST = 2,   // closest-hit query in flight
    ST_SHADOW = 3,    // NEE shadow query in flight
    ST_DONE = 4,      // no work left
    ST_HIT = 5,       // query results
    ST_MISS = 6,
    ST_OCCLUDED = 7,
    ST_VISIBLE = 8,
    ST_LEAFX = 9,     // LX builds: the lane's leaf tests wait for the wave's leaf exchange (leaf_exchange)
};

// True when every active lane holds the same x.
__device__ __forceinline__ bool wave_uniform(uint32_t x) {
    return __ballot(x == (uint32_t)__builtin_amdgcn_readfirstlane(x)) == __ballot(1);
}

// Distinct values of key over the active lanes (FULL-build diagnostics).
__device__ __forceinline__ uint32_t wave_distinct(uint32_t key) {
    uint64_t m = __ballot(1);
    uint32_t n = 0;
    while (m) {
        const uint32_t k = (uint32_t)__shfl((int)key, __ffsll((long long)m) - 1, 64);
        m &= ~__ballot(key == k);
        n++;
    }
    return n;
}

// Traversal registers of a query in flight.  r = per-axis rcp_for_div(d) for
// the exact short split-distance division (FD builds, device_math.hpp).
struct Trav {
    uint32_t node, sp, nl;
    float tmin, tmax;
    f3 r;
};

// Counting-build diagnostics of one lane (DIAG_* in kernels.hpp): the lane's last 8
// triangles that missed for any segment in its current query (a per-lane mailbox, as a
// census: no test is skipped), and its tallies (wave-level ones kept by the leader).
struct Diag {
    bool on;        // the trace kind is in RenderArgs::diag_kinds
    uint32_t n;     // misses recorded in this query (reset at each query start)
    uint32_t mb[8]; // mb[i & 7]: the i-th
    uint32_t v[DIAG_N];
};
__device__ __forceinline__ void diag_begin(Diag *dg) {
    if (dg) dg->n = 0;
}
__device__ __forceinline__ void diag_flush(unsigned long long *ctrs, const Diag &dg) {
    const uint32_t ln = lane_id();
#pragma unroll
    for (int i = 0; i < DIAG_N; i++) {
        unsigned long long s = dg.v[i];
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) s += __shfl_xor(s, off, 64);
        if (ln == 0 && s) atomicAdd(&ctrs[CTR_DIAG + i], s);
    }
}

// Performed work of one lane (perf builds, PERF_* in kernels.hpp): what the kernel executes and
// the bytes its loads and stores move -- vector accesses per lane, scalar loads once per wave
// (counted by the wave's leader).
struct Pc {
    uint32_t q, steps, leaves, masks, tests, waves;
    uint64_t vb, sb;
    uint32_t drounds, diters, dlanes, dtests;
};
__device__ __forceinline__ void pc_load(Pc *pc, bool scalar, uint32_t bytes) {
    if (!pc) return;
    if (!scalar) pc->vb += bytes;
    else if (wave_leader()) pc->sb += bytes;
}
// Call with the whole wave converged: the lane sums go to ctrs[0 .. PERF_N).
__device__ __forceinline__ void pc_flush(unsigned long long *ctrs, const Pc &pc) {
    const uint32_t ln = lane_id();
    const unsigned long long v[PERF_N] = {pc.q,     pc.steps,   pc.leaves, pc.masks,  pc.tests,  pc.vb,
                                          pc.sb,    pc.waves,   pc.drounds, pc.diters, pc.dlanes, pc.dtests};
#pragma unroll
    for (int i = 0; i < PERF_N; i++) {
        unsigned long long x = v[i];
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) x += __shfl_xor(x, off, 64);
        if (ln == 0 && x) atomicAdd(&ctrs[i], x);
    }
}

// A lane's stack-overflow entry at `depth` ([depth][gstride] rows): a 32-bit byte offset from the
// wave-uniform base, so the access uses scalar-base addressing and no 64-bit per-lane pointer is kept
// live (the compiler spilled one); cr_render checks that an area stays below 4 GiB.
__device__ __forceinline__ uint2 &gstack_at(uint2 *gstk, uint32_t depth, uint32_t gstride, uint32_t gid) {
    return *(uint2 *)((char *)gstk + (depth * gstride + gid) * 8u);
}

// Root-box clip (kdtree.cpp:196-208, 276-283); false: the query ends without a hit.
__device__ __forceinline__ bool trav_begin(const DevScene &S, f3 o, f3 d, bool shadow, float limit, Trav &T) {
    const f3 inv = mk(1.f / d.x, 1.f / d.y, 1.f / d.z);
    ray_box_inv(S, o, inv, T.tmin, T.tmax);
    if (T.tmax < 0 || T.tmax < T.tmin) return false;
    if (shadow) {
        if (T.tmin > limit) return false;
        T.tmax = std_min(T.tmax, limit);
    }
    const float nan = __builtin_nanf("");
    T.r = mk(fabsf(d.x) >= 0x1p-40f && fabsf(d.x) <= 0x1p40f ? inv.x : nan,
             fabsf(d.y) >= 0x1p-40f && fabsf(d.y) <= 0x1p40f ? inv.y : nan,
             fabsf(d.z) >= 0x1p-40f && fabsf(d.z) <= 0x1p40f ? inv.z : nan);
    T.node = T.sp = T.nl = 0;
    return true;
}

// One traversal round (kdtree.cpp:250-330 as an explicit stack): descend to the
// next leaf, test it, pop.  Returns the lane's new state: unchanged while the
// query continues, else its result (a closest hit leaves {bx, by, tri} in d:
// the direction is dead by then).
//   Stack: entries {far node, tmax at push}; the top R live in an LDS ring
//   [slot][thread] (blockDim.x threads), deeper ones spill to gstk
//   [depth][gstride].  On pop the interval is [current tmax, entry.tmax]: the
//   current tmax equals the push-time tsplit (stack invariant).
// (A wave-level mailbox -- per wave in LDS, the lanes for which a triangle was
// a geometric miss in their current query, so a uniform leaf skips it when all
// active lanes know it -- is exact too and measured 3% slower: the LDS lookup
// serialises behind every scalar record load.)
// (Speculative descent -- lanes that reached their leaf early descending toward
// the next one, Aila & Laine's postponed leaves -- is exact here too but
// measured slower: the merged descent loop costs more than the idle lanes.)
// Scalar-memory loads for wave-uniform addresses (SC builds): when every active
// lane wants the same node / leaf, one s_load serves the wave and the vector
// memory address path -- the measured bottleneck -- is not used at all.  The
// data is read-only for the whole launch, so the scalar cache is coherent.
// Every block that issues more than one load marks its outputs early-clobber
// ("=&s"): without it the register allocator may give a later load's base the
// registers an earlier load of the same block is filling, and a scalar load
// that returns before the next one issues then rewrites that base (the
// full-size-only illegal address of the grandchild-prefetch builds).
typedef unsigned int cr_v2u __attribute__((ext_vector_type(2)));
typedef float cr_v4f __attribute__((ext_vector_type(4)));
typedef float cr_v8f __attribute__((ext_vector_type(8)));
typedef unsigned int cr_v8u __attribute__((ext_vector_type(8)));
typedef unsigned int cr_v4u __attribute__((ext_vector_type(4)));
typedef float cr_v16f __attribute__((ext_vector_type(16)));
__device__ __forceinline__ uint2 sload_node(const uint2 *p) {
    cr_v2u r;
    asm volatile("s_load_dwordx2 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(r) : "s"(p));
    return make_uint2(r.x, r.y);
}
__device__ __forceinline__ TriRec sload_rec(const float4 *p) {
    cr_v8f a;
    cr_v4f b;
    asm volatile("s_load_dwordx8 %0, %2, 0x0\n\ts_load_dwordx4 %1, %2, 0x20\n\ts_waitcnt lgkmcnt(0)"
                 : "=&s"(a), "=&s"(b)
                 : "s"(p));
    return TriRec{make_float4(a[0], a[1], a[2], a[3]), make_float4(a[4], a[5], a[6], a[7]),
                  make_float4(b[0], b[1], b[2], b[3])};
}
// Four consecutive cull boxes (64 B; cull buffers carry three padding boxes).
__device__ __forceinline__ cr_v16f sload_box4(const float4 *p) {
    cr_v16f r;
    asm volatile("s_load_dwordx16 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(r) : "s"(p));
    return r;
}
__device__ __forceinline__ float4 sload_box(const float4 *p) {
    cr_v4f r;
    asm volatile("s_load_dwordx4 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(r) : "s"(p));
    return make_float4(r[0], r[1], r[2], r[3]);
}
// A fat record and its subtree box (CULL >= 2) under one scalar-load wait.
__device__ __forceinline__ void sload_fat_box(const uint4 *p, const float4 *q, uint4 &a, uint4 &b, float4 &box) {
    cr_v8u r;
    cr_v4f x;
    asm volatile("s_load_dwordx8 %0, %2, 0x0\n\ts_load_dwordx4 %1, %3, 0x0\n\ts_waitcnt lgkmcnt(0)"
                 : "=&s"(r), "=&s"(x)
                 : "s"(p), "s"(q));
    a = make_uint4(r[0], r[1], r[2], r[3]);
    b = make_uint4(r[4], r[5], r[6], r[7]);
    box = make_float4(x[0], x[1], x[2], x[3]);
}
// The same for node n with the byte offsets in SGPRs (s_load's soffset form): no 64-bit
// address arithmetic on the scalar unit, which bounds the packet trace.
__device__ __forceinline__ void sload_fat_box_n(const uint4 *fat, const float4 *boxes, uint32_t n, uint4 &a, uint4 &b,
                                                float4 &box) {
    cr_v8u r;
    cr_v4f x;
    asm volatile("s_load_dwordx8 %0, %2, %4\n\ts_load_dwordx4 %1, %3, %5\n\ts_waitcnt lgkmcnt(0)"
                 : "=&s"(r), "=&s"(x)
                 : "s"(fat), "s"(boxes), "s"(n * 32u), "s"(n * 16u));
    a = make_uint4(r[0], r[1], r[2], r[3]);
    b = make_uint4(r[4], r[5], r[6], r[7]);
    box = make_float4(x[0], x[1], x[2], x[3]);
}
// A packed leaf cull record (LC_RECP float4, 96 B) under one scalar-load wait.
__device__ __forceinline__ void sload_lcullp(const float4 *p, LcFloat4 (&r)[LC_REC]) {
    cr_v16f a;
    cr_v8f b;
    asm volatile("s_load_dwordx16 %0, %2, 0x0\n\ts_load_dwordx8 %1, %2, 0x40\n\ts_waitcnt lgkmcnt(0)"
                 : "=&s"(a), "=&s"(b)
                 : "s"(p));
#pragma unroll
    for (int i = 0; i < 4; i++) r[i] = LcFloat4{a[4 * i], a[4 * i + 1], a[4 * i + 2], a[4 * i + 3]};
    r[4] = LcFloat4{b[0], b[1], b[2], b[3]};
    r[5] = LcFloat4{b[4], b[5], b[6], b[7]};
}
// A compressed leaf cull record (S.lcullc, 48 B: three 16-B loads, or one 48-B scalar load pair)
__device__ __forceinline__ void sload_lcullc(const uint4 *p, uint32_t (&w)[12]) {
    cr_v8u a;
    cr_v4u b;
    asm volatile("s_load_dwordx8 %0, %2, 0x0\n\ts_load_dwordx4 %1, %2, 0x20\n\ts_waitcnt lgkmcnt(0)"
                 : "=&s"(a), "=&s"(b)
                 : "s"(p));
#pragma unroll
    for (int i = 0; i < 8; i++) w[i] = a[i];
#pragma unroll
    for (int i = 0; i < 4; i++) w[8 + i] = b[i];
}
// The references of the leaf at `node` that the lane's ray (o, d: unit, segment [0, tmax]) must test
// (leafcull.hpp); bits < count.  FORM 2: packed fixed-pad records (S.lcullp), 4: compressed (S.lcullc).
template <bool SC, int FORM>
__device__ __forceinline__ uint32_t leaf_mask(const DevScene &S, uint32_t node, uint32_t count, f3 o, f3 d, float tmax) {
    if (FORM == 4) {
        uint32_t w[12];
        if (SC && wave_uniform(node)) {
            sload_lcullc(S.lcullc + (size_t)LC_RECC * __builtin_amdgcn_readfirstlane(node), w);
        } else {
            const uint4 *p = (const uint4 *)((const char *)S.lcullc + node * (uint32_t)(16 * LC_RECC));
#pragma unroll
            for (int i = 0; i < LC_RECC; i++) {
                const uint4 v = p[i];
                w[4 * i] = v.x, w[4 * i + 1] = v.y, w[4 * i + 2] = v.z, w[4 * i + 3] = v.w;
            }
        }
        const float ov[3] = {o.x, o.y, o.z}, dv[3] = {d.x, d.y, d.z};
        const float inv[3] = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y), __builtin_amdgcn_rcpf(d.z)};
        return leaf_cull_mask_c(ov, dv, inv, lc_unit(d.x, d.y, d.z), tmax, w, count, S.lcg);
    }
    static_assert(FORM == 2 || FORM == 4, "leaf cull record forms: 2 (packed) or 4 (compressed)");
    LcFloat4 rec[LC_REC];
    constexpr int NR = LC_RECP;
    const float4 *recs = S.lcullp;
    if (SC && wave_uniform(node)) {
        sload_lcullp(recs + (size_t)NR * __builtin_amdgcn_readfirstlane(node), rec);
    } else {
        const float4 *p = (const float4 *)((const char *)recs + node * (uint32_t)(16 * NR));
#pragma unroll
        for (int i = 0; i < NR; i++) {
            const float4 v = p[i];
            rec[i] = LcFloat4{v.x, v.y, v.z, v.w};
        }
#ifdef CR_PAD_LC // address-path calibration only: CR_PAD_LC extra 16-B loads of the record's own lines
        typedef const __attribute__((address_space(1))) cr_v4f g_f4;
        g_f4 *q = (g_f4 *)p;
        asm volatile("" : "+v"(q));
#pragma unroll
        for (int i = 0; i < CR_PAD_LC; i++) {
            const cr_v4f v = q[i];
            asm volatile("" ::"v"(v));
        }
#endif
    }
    const float ov[3] = {o.x, o.y, o.z}, dv[3] = {d.x, d.y, d.z};
    // v_rcp_f32: within 1 ulp of 1/d (the check allows 2, tests/native/leafcull_check.cpp)
    const float inv[3] = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y), __builtin_amdgcn_rcpf(d.z)};
    return leaf_cull_mask_packed(ov, dv, inv, lc_unit(d.x, d.y, d.z), tmax, rec, count);
}

template <bool SC> __device__ __forceinline__ float4 load_box(const float4 *b, uint32_t i) {
    if (SC && wave_uniform(i)) return sload_box(b + __builtin_amdgcn_readfirstlane(i));
    return b[i];
}
template <bool SC> __device__ __forceinline__ uint2 load_node(const DevScene &S, uint32_t node) {
    if (SC && wave_uniform(node)) return sload_node(S.nodes + __builtin_amdgcn_readfirstlane(node));
    return S.nodes[node];
}

// Fat node records (DevScene::fat): 32 B per node, {self, child 0, child 1}, so
// one dependent load serves two descent levels.
__device__ __forceinline__ void sload_fat(const uint4 *p, uint4 &a, uint4 &b) {
    cr_v8u r;
    asm volatile("s_load_dwordx8 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(r) : "s"(p));
    a = make_uint4(r[0], r[1], r[2], r[3]);
    b = make_uint4(r[4], r[5], r[6], r[7]);
}
template <bool SC> __device__ __forceinline__ void load_fat(const DevScene &S, uint32_t node, uint4 &a, uint4 &b) {
    if (SC && wave_uniform(node)) return sload_fat(S.fat + 2u * __builtin_amdgcn_readfirstlane(node), a, b);
    const uint4 *p = (const uint4 *)((const char *)S.fat + node * 32u);
    a = p[0];
    b = p[1];
#ifdef CR_PAD_FETCH // address-path calibration only: CR_PAD_FETCH extra 16-B loads of the record's line
    typedef const __attribute__((address_space(1))) cr_v4u g_u4;
    g_u4 *q = (g_u4 *)p;
    asm volatile("" : "+v"(q));
#pragma unroll
    for (int i = 0; i < CR_PAD_FETCH; i++) {
        const cr_v4u v = q[i & 1];
        asm volatile("" ::"v"(v));
    }
#endif
}

// The leaf loop is software-pipelined (triangle j+1's loads issued before j is
// tested).  Measured and dropped: the same unrolled by two with unconditional
// loads (no register rotation copies, but count-1 leaves fetch a second record:
// -2.3%), and compiler-scheduled, pipelined scalar loads for uniform leaves
// (address_space(4): -2.5% against the asm s_load + wait below).  The other measured
// and dropped knobs (DESIGN.md keeps their numbers): the top of the tree in LDS, a
// uniform leaf's records two per wait, per-reference plane records, two-level 16-B node
// records, the per-ray, fixed-pad and short leaf cull record forms, the phase clock.
// BF: the decisions as selects instead of divergent branches (the trace kernels
// are bound by the scalar unit's exec-mask bookkeeping, SURVEY §8d / DESIGN §3.3):
// a descent step branches only around its stack push, and a uniform leaf's
// triangle tests keep their result by select (tri_test_wave).
// CULL (camera rays; BF + SC): a triangle test runs only when the lane's sample
// position (csx, csy) lies in the reference's cull box (camcull.hpp) -- outside it the
// test cannot accept, so skipping it changes nothing.  A uniform leaf reads four boxes
// per scalar load and tests a triangle only if some lane is inside its box; a divergent
// lane reads its box (16 B) and, inside, the record (48 B).
// LC (secondary closest / shadow rays, unit directions; BF + SC): a leaf's tests run only
// for the references its cull record (leafcull.hpp) cannot exclude for this ray and segment.
// A trace build's configuration: every knob of trav_round and wf_trace (wavefront.hip), named.  The
// defaults are the plain reference build; a build is a type deriving from this and restating what it
// changes (wavefront.hip namespace tc), so a kernel reads e.g. wf_trace<cr::tc::ShadowLcFd>.
struct TraceDefaults {
    static constexpr bool SHADOW = false; // shadow (any-hit) queries, else closest-hit
    static constexpr bool FULL = false;   // counting build: SURVEY §8d work counters and diagnostics
    static constexpr int R = 8;           // LDS ring entries of the traversal stack per lane
    static constexpr int MINW = 8;        // waves per SIMD the launch bounds ask for
    static constexpr bool SC = false;     // scalar loads of wave-uniform nodes and leaves
    static constexpr bool FD = false;     // exact short split division by the ray's RN(1/d)
    static constexpr bool FAT = false;    // fat node records (a node and its children per load)
    static constexpr bool CAM = false;    // the generation-1 closest (camera-ray) instantiation
    static constexpr bool BF = false;     // branch-light steps and uniform-leaf tests by select
    static constexpr int CULL = 0;        // camera cull boxes: 1 references and leaves, 2 also subtrees
    static constexpr int LC = 0;          // leaf cull records (4 packed, 5 compressed)
    static constexpr bool PC = false;     // performed-work counters (measurement only)
    static constexpr bool DEAD = false;   // shadow queues with dead entries (wf_shade's chunked appends) skipped
    static constexpr bool LX = false;     // a divergent leaf's masked tests spread over the wave (leaf_exchange)
    static constexpr bool LXD = false;    // LX builds: the exchange's prefix by a DPP scan
};

// A lane's deferred leaf (LX builds): the references of the leaf whose first record is `first` that its
// cull mask keeps (bit j: first + j).
struct LeafX {
    uint32_t mask, first;
};

// The stack's top entry becomes the query's node and interval (stack invariant).
// ring: the LDS ring's column of the wave's lane 0 ([slot][blockDim.x]); gstk as gstack_at's.
// ring: the LDS ring [slot][blockDim.x]; gstk / gid: the stack-overflow area and the lane's global index.
template <int R>
__device__ __forceinline__ void trav_pop(uint2 *ring, uint2 *gstk, uint32_t gstride, uint32_t gid, Trav &T,
                                         Pc *pc = nullptr) {
    T.sp--;
    uint2 e;
    if (T.nl) {
        e = ring[(T.sp & (R - 1)) * blockDim.x + threadIdx.x];
        T.nl--;
    } else {
        e = gstack_at(gstk, T.sp, gstride, gid);
        if (pc) pc->vb += 8;
    }
    T.node = e.x;
    T.tmin = T.tmax; // == the popped entry's split distance (stack invariant)
    T.tmax = __uint_as_float(e.y);
}

template <class C>
__device__ __forceinline__ uint32_t trav_round(int lc_debug, uint32_t lc_min, const DevScene &S, uint2 *ring, uint2 *gstk, uint32_t gstride,
                                               uint32_t gid, f3 o, f3 &d, bool shadow, uint32_t exclude, Trav &T,
                                               Ctr &c, float csx = 0.f, float csy = 0.f, const float4 *cull = nullptr,
                                               const float4 *cull_node = nullptr, Diag *dg = nullptr,
                                               Pc *pc = nullptr, uint32_t quorum = 0, LeafX *lx = nullptr) {
    static constexpr int R = C::R, CULL = C::CULL, LC = C::LC;
    static constexpr bool FULL = C::FULL, FD = C::FD, SC = C::SC, FAT = C::FAT, BF = C::BF;
    // quorum (lean FAT builds without the camera cull): the wave's descent stops at a fetch once at most
    // quorum / 64 of the lanes that entered the round still descend; those keep T.node (the node to fetch)
    // and their interval and go on next round -- the same node visits with the same intervals, so the
    // same answers -- while the others test their leaves now instead of idling
    const uint32_t nbusy = quorum ? (uint32_t)__popcll(__ballot(1)) : 0u;
    constexpr uint32_t PENDING_LEAF = 0xfffffffeu;
    bool pending = false;
    if (pc && wave_leader()) pc->waves++;
    // performed-work accounting of record loads (pc: perf builds)
    auto lrec = [&](uint32_t i) -> TriRec {
        if (pc) pc->vb += 16u * REC_STRIDE;
        return load_rec(S, i);
    };
    auto srec = [&](const float4 *q) -> TriRec {
        pc_load(pc, true, 16u * REC_STRIDE);
        return sload_rec(q);
    };
    static_assert(!CULL || (BF && SC && !FULL), "cull: lean BF + SC builds");
    static_assert(CULL < 2 || FAT, "subtree cull: fat-record builds");
    static_assert(!LC || ((LC == 4 || LC == 5) && !CULL && BF && SC && !FULL), "leaf cull: lean BF + SC builds, forms 4 / 5");
    static_assert(!C::LX || LC, "leaf exchange: leaf-cull builds");
    const uint32_t bdim = blockDim.x, tid = threadIdx.x;
    // one kd decision at inner node nd (kdtree.cpp:258-275): T.node = the child to
    // descend into (child + k), the far child pushed when both are crossed
    auto step = [&](uint2 nd) -> uint32_t {
        if (pc) pc->steps++;
#ifdef CR_PAD_STEP // issue-cost calibration only: CR_PAD_STEP extra VALU per shadow descent step
        if (C::SHADOW) {
            uint32_t z = nd.x;
#pragma unroll
            for (int i = 0; i < CR_PAD_STEP; i++) asm volatile("v_mov_b32 %0, %0" : "+v"(z));
        }
#endif
        if (FULL) {
            c.inner++;
            const bool uni = wave_uniform(T.node);
            const uint32_t lines = wave_distinct(T.node >> (FAT ? 2 : 4)); // 32-B / 8-B node records
            if (wave_leader()) {
                c.wave_desc++;
                c.wave_desc_uniform += uni;
                c.wave_desc_lines += lines;
            }
        }
        const uint32_t a = nd.y & 3u;
        const float split = __uint_as_float(nd.x);
        const float oa = comp(o, a), da = comp(d, a);
        const float tsplit = FD ? div_by_rcp_wave(split - oa, da, comp(T.r, a)) : split_distance(split, oa, da);
        const uint32_t below = (oa < split) || (oa == split && da <= 0);
        const uint32_t child = nd.y >> 2;
        uint32_t k;
        if (BF) { // (bitwise logic on the lane masks: no short-circuit exec branches)
            const bool near_only = (tsplit >= T.tmax) | (tsplit < 0);
            const bool far_only = !near_only & (tsplit <= T.tmin);
            const bool push = !near_only & !far_only;
            k = far_only ? below : 1u - below;
            if (push) {
                const uint32_t slot = (T.sp & (R - 1)) * bdim + tid;
                if (pc && T.nl == R) pc->vb += 8;
                if (T.nl == R) gstack_at(gstk, T.sp - R, gstride, gid) = ring[slot]; // spill the oldest
                ring[slot] = make_uint2(child + below, __float_as_uint(T.tmax));
            }
            T.nl = push && T.nl < R ? T.nl + 1 : T.nl;
            T.sp += push ? 1u : 0u;
            T.tmax = push ? tsplit : T.tmax;
        } else if (tsplit >= T.tmax || tsplit < 0) {
            k = 1u - below;
        } else if (tsplit <= T.tmin) {
            k = below;
        } else {
            const uint2 e = make_uint2(child + below, __float_as_uint(T.tmax));
            const uint32_t slot = (T.sp & (R - 1)) * bdim + tid;
            if (T.nl == R) gstack_at(gstk, T.sp - R, gstride, gid) = ring[slot]; // spill the oldest
            else T.nl++;
            ring[slot] = e;
            T.sp++;
            T.tmax = tsplit;
            k = 1u - below;
        }
        T.node = child + k;
        return k;
    };
    uint2 nd;
    // CULL >= 2: a fetched node whose subtree box excludes the sample is treated as an
    // empty leaf -- none of its triangles can accept, so the traversal would leave it
    // without a hit and with tmax = its interval's end, which is exactly this state
    bool culled = false;
    uint32_t first, count, lmask;
    bool lin;
    auto pop_entry = [&]() { trav_pop<R>(ring, gstk, gstride, gid, T, pc); };
    if (FAT) { // two levels per dependent load: a node's record carries its children's
        uint4 f0, f1;
        auto fetch = [&](uint32_t node) {
            if (CULL >= 2) { // the record and the subtree box, loads issued together
                float4 b;
                pc_load(pc, SC && wave_uniform(node), 48);
                if (SC && wave_uniform(node)) {
                    const uint32_t un = __builtin_amdgcn_readfirstlane(node);
                    sload_fat_box(S.fat + 2u * un, cull_node + un, f0, f1, b);
                } else {
                    const uint4 *p = (const uint4 *)((const char *)S.fat + node * 32u);
                    f0 = p[0];
                    f1 = p[1];
                    b = cull_node[node];
                }
                nd = make_uint2(f0.x, f0.y);
                if (!(csx >= b.x && csx <= b.y && csy >= b.z && csy <= b.w)) {
                    culled = true;
                    nd = make_uint2(0xffffffffu, 3u); // an empty leaf no real leaf shares `first` with
                }
                return;
            } else {
                pc_load(pc, SC && wave_uniform(node), 32);
                load_fat<SC>(S, node, f0, f1);
            }
            nd = make_uint2(f0.x, f0.y);
            if (CULL >= 2) {
                const float4 b = load_box<SC>(cull_node, node);
                if (!(csx >= b.x && csx <= b.y && csy >= b.z && csy <= b.w)) {
                    culled = true;
                    nd = make_uint2(0xffffffffu, 3u); // an empty leaf no real leaf shares `first` with
                }
            }
        };
        fetch(T.node);
        // one exit: a lane whose level-1 node is a leaf skips the second step and leaves at the loop test
        // (a second exit would double the exec-mask bookkeeping of this divergent loop on the scalar
        // unit); the quorum leaves the same way
        while ((nd.y & 3u) != 3u) {
            const uint32_t k = step(nd);
            nd = k ? make_uint2(f1.x, f1.y) : make_uint2(f0.z, f0.w);
            if ((nd.y & 3u) != 3u) {
                step(nd);
                if (!FULL && !CULL && quorum && (uint32_t)__popcll(__ballot(1)) * 64u <= nbusy * quorum)
                    nd = make_uint2(PENDING_LEAF, 3u); // (an empty "leaf" no real leaf shares `first` with)
                else
                    fetch(T.node);
            }
        }
        pending = !FULL && !CULL && quorum && nd.x == PENDING_LEAF;
    } else {
        pc_load(pc, SC && wave_uniform(T.node), 8);
        nd = load_node<SC>(S, T.node);
        while ((nd.y & 3u) != 3u) {
            step(nd);
            pc_load(pc, SC && wave_uniform(T.node), 8);
            nd = load_node<SC>(S, T.node);
        }
    }
    if (pending) return shadow ? ST_SHADOW : ST_CLOSEST; // descends on next round from T.node
    if (FULL) {
        c.leaf++;
        if (wave_leader()) c.wave_round++;
    }
    if (pc) pc->leaves++;
    first = nd.x;
    count = nd.y >> 2;
    lin = !culled; // CULL: the sample lies in the leaf's box (the union of its references')
    if (CULL && !culled) {
        pc_load(pc, SC && wave_uniform(T.node), 16);
        const float4 lb = load_box<SC>(cull_node, T.node);
        lin = csx >= lb.x && csx <= lb.y && csy >= lb.z && csy <= lb.w;
    }
    // LC: the references to test (bit j: first + j); count > LC_MAXREFS: every one (lmask unused)
    lmask = 0u;
    if (LC && count && count <= (uint32_t)LC_MAXREFS) {
        // leaves below lc_min: every reference, no check
        const uint32_t lcid = T.node;
        if (pc && count >= lc_min) {
            pc->masks++;
            pc_load(pc, SC && wave_uniform(lcid), 16u * (LC == 5 ? LC_RECC : LC_RECP));
        }
        lmask = count >= lc_min ? leaf_mask<SC, LC == 5 ? 4 : 2>(S, lcid, count, o, d, T.tmax)
                                : (count >= 32 ? 0xffffffffu : (1u << count) - 1u);
        if (lc_debug) lmask = lc_debug == 1 ? (count >= 32 ? 0xffffffffu : (1u << count) - 1u) : 0u;
    }
    bool found = false, occluded = false;
    uint32_t tri = 0;
    float bx = 0.f, by = 0.f;
    // one triangle of the leaf (kdtree.cpp:235-246 / 309-320); false: stop the leaf
    auto test = [&](const TriRec &r) -> bool {
        const uint32_t id = rec_id(r);
        if (shadow && id == exclude) return true;
        if (FULL) c.tritest++;
        if (pc) pc->tests++;
        if (FULL && dg && dg->on) { // repeated-miss census: a miss for any segment is one for every later one
            dg->v[DIAG_TESTS]++;
            float gx, gy, gt;
            if (!tri_test(o, d, r, __builtin_inff(), gx, gy, gt)) {
                dg->v[DIAG_GEOMISS]++;
                const uint32_t n = dg->n;
                bool r1 = false, r4 = false, r8 = false;
#pragma unroll
                for (uint32_t j = 0; j < 8; j++) {
                    const bool m = j < n && dg->mb[(n - 1 - j) & 7u] == id;
                    r1 = r1 | (m & (j < 1));
                    r4 = r4 | (m & (j < 4));
                    r8 = r8 | m;
                }
                dg->v[DIAG_REP1] += r1;
                dg->v[DIAG_REP4] += r4;
                dg->v[DIAG_REP8] += r8;
                dg->mb[n & 7u] = id;
                dg->n = n + 1;
            }
        }
        float ux, uy, t;
        // BF: the lanes that failed an early test compute on (wave-uniform exits, no exec bookkeeping)
        if (BF ? tri_test_wave(o, d, r, T.tmax, ux, uy, t) : tri_test(o, d, r, T.tmax, ux, uy, t)) {
            if (shadow) {
                occluded = true;
                return false;
            }
            bx = ux;
            by = uy;
            T.tmax = t;
            tri = id;
            found = true;
        }
        return true;
    };
    auto tally_tri = [&](uint32_t ref) {
        if (FULL) {
            const bool uni = wave_uniform(ref);
            const uint32_t lines = wave_distinct(ref * (16u * REC_STRIDE) >> 7);
            if (wave_leader()) {
                c.wave_tri++;
                c.wave_tri_uniform += uni;
                c.wave_tri_lines += lines;
            }
        }
    };
    if (FULL && (!dg || dg->on) && !wave_uniform(first)) { // what staging the wave's leaves in LDS would take
        uint64_t m = __ballot(count > 0);
        uint32_t nd = 0, nr = 0, mc = 0, lt = 0;
        const uint32_t lanes = (uint32_t)__popcll(m);
        while (m) {
            const int l = __ffsll((long long)m) - 1;
            const uint32_t f = (uint32_t)__shfl((int)first, l, 64), n = (uint32_t)__shfl((int)count, l, 64);
            const uint64_t same = __ballot(first == f && count > 0);
            m &= ~same;
            nd++;
            nr += n;
            mc = max(mc, n);
            lt += n * (uint32_t)__popcll(same);
        }
        if (wave_leader()) {
            c.leaf_rounds++;
            c.leaf_distinct += nd;
            c.leaf_records += nr;
            c.leaf_fit21 += nr <= 21;
            c.leaf_fit56 += nr <= 56;
            if (dg) {
                dg->v[DIAG_ROUNDS]++;
                dg->v[DIAG_LANES] += lanes;
                dg->v[DIAG_DISTINCT] += nd;
                dg->v[DIAG_RECORDS] += nr;
                dg->v[DIAG_MAXCOUNT] += mc;
                dg->v[DIAG_LANETESTS] += lt;
                dg->v[DIAG_FIT64] += nr <= 64;
                dg->v[DIAG_FIT128] += nr <= 128;
            }
        }
    } else if (FULL && dg && dg->on && wave_leader()) {
        dg->v[DIAG_UROUNDS]++;
    }
    if (BF && SC && wave_uniform(first)) { // uniform leaf, results by select
        const uint32_t uf = __builtin_amdgcn_readfirstlane(first), uc = __builtin_amdgcn_readfirstlane(count);
        const float4 *base = S.recs + (size_t)REC_STRIDE * uf;
        // one triangle of the uniform leaf; false: every active lane occluded (stop)
        // in: the lane tests this triangle (LC: the bit of its own mask)
        auto utest = [&](const TriRec &r, uint32_t j, bool in = true) -> bool {
            tally_tri(uf + j);
            const uint32_t id = rec_id(r);
            const bool live = in & !(shadow & (occluded | (id == exclude)));
            if (FULL) c.tritest += live ? 1u : 0u;
            if (pc) pc->tests += live ? 1u : 0u;
            float ux, uy, t;
            const bool acc = live & tri_test_wave(o, d, r, T.tmax, ux, uy, t);
            if (shadow) {
                occluded = occluded | acc;
                return __ballot(!occluded) != 0;
            }
            bx = acc ? ux : bx;
            by = acc ? uy : by;
            T.tmax = acc ? t : T.tmax;
            tri = acc ? id : tri;
            found = found | acc;
            return true;
        };
        if (CULL) {
            const float4 *cb = cull + uf;
            for (uint32_t j = 0; j < uc && __ballot(lin); j += 4) {
                pc_load(pc, true, 64);
                const cr_v16f bx = sload_box4(cb + j);
#pragma unroll
                for (uint32_t k = 0; k < 4; k++) {
                    if (j + k >= uc) break;
                    const bool in = csx >= bx[4 * k] && csx <= bx[4 * k + 1] && csy >= bx[4 * k + 2] &&
                                    csy <= bx[4 * k + 3];
                    if (__ballot(in)) utest(srec(base + (size_t)REC_STRIDE * (j + k)), j + k);
                }
            }
        } else if (LC && uc <= (uint32_t)LC_MAXREFS) {
            // a triangle runs when some lane's mask holds it (a lane tests only its own
            // references: utest's `in`); per-bit ballots, since a butterfly over the wave
            // would not see the bits of lanes whose partners are inactive
            for (uint32_t j = 0; j < uc; j++) {
                const bool in = (lmask >> j) & 1u;
                if (!__ballot(in)) continue;
                if (!utest(srec(base + (size_t)REC_STRIDE * j), j, in)) break;
            }
        } else {
            for (uint32_t j = 0; j < uc; j++)
                if (!utest(srec(base + (size_t)REC_STRIDE * j), j)) break;
        }
    } else if (SC && wave_uniform(first)) { // every lane at the same leaf: scalar loads
        const float4 *base = S.recs + (size_t)REC_STRIDE * __builtin_amdgcn_readfirstlane(first);
        for (uint32_t j = 0; j < count; j++) {
            tally_tri(first + j);
            if (!test(srec(base + (size_t)REC_STRIDE * j))) break;
        }
    } else if (C::LX && LC && count <= (uint32_t)LC_MAXREFS) { // tests deferred to the wave's leaf exchange
        if (lmask) {
            lx->mask = lmask;
            lx->first = first;
            return ST_LEAFX;
        }
    } else if (LC && count <= (uint32_t)LC_MAXREFS) { // the mask's references, pipelined one ahead
        uint32_t m = lmask;
        if (pc) { // the divergent leaf loop's shape: iterations = the largest lane mask
            const uint32_t pop = (uint32_t)__builtin_popcount(m);
            const uint32_t lanes = (uint32_t)__popcll(__ballot(pop > 0));
            uint32_t mx = 0;
            while (__ballot(pop > mx)) mx++;
            if (lanes && wave_leader()) {
                pc->drounds++;
                pc->diters += mx;
                pc->dlanes += lanes;
            }
            pc->dtests += pop;
        }
        TriRec nx;
        if (m) nx = lrec(first + (uint32_t)__builtin_ctz(m));
        while (m) {
            m &= m - 1u;
            const TriRec r = nx;
            if (m) nx = lrec(first + (uint32_t)__builtin_ctz(m));
            if (!test(r)) break;
        }
    } else if (CULL) { // boxes pipelined one ahead; a record only for a sample inside its box
        if (!lin) count = 0;
        float4 nb = make_float4(0.f, 0.f, 0.f, 0.f);
        if (count) nb = cull[first];
        if (pc && count) pc->vb += 16;
        for (uint32_t j = 0; j < count; j++) {
            const float4 b = nb;
            if (j + 1 < count) nb = cull[first + j + 1];
            if (pc && j + 1 < count) pc->vb += 16;
            if (csx >= b.x && csx <= b.y && csy >= b.z && csy <= b.w)
                if (!test(lrec(first + j))) break;
        }
    } else {
        TriRec nx;
        if (count) nx = lrec(first);
        for (uint32_t j = 0; j < count; j++) { // software pipeline: triangle j+1's loads before j's test
            tally_tri(first + j);
            const TriRec r = nx;
            if (j + 1 < count) nx = lrec(first + j + 1);
            if (!test(r)) break;
        }
    }
    if (occluded) return ST_OCCLUDED;
    if (found) {
        d = mk(bx, by, __uint_as_float(tri));
        return ST_HIT;
    }
    if (T.sp == 0) return shadow ? ST_VISIBLE : ST_MISS;
    pop_entry();
    return shadow ? ST_SHADOW : ST_CLOSEST;
}

// ------------------------------------------------------------ leaf exchange --
// LX builds.  In a divergent leaf round the leaf cull leaves tests in ~16 of a wave's lanes, ~5 each, and
// the per-lane loop runs as long as the longest mask: 6 iterations at 0.2 of the lanes.
// Here the whole wave (every lane, busy or idle) tests the round's (lane, reference) pairs 64 at a time:
// pair i belongs to the lane whose exclusive prefix of mask popcounts is the largest one <= i, and is that
// lane's (i - prefix)-th mask bit.  The answers are the per-lane loop's:
//   shadow: occluded == some masked reference other than the excluded one accepts (0 <= t < tmax) -- an OR,
//           whatever the order (kdtree.cpp:309-320);
//   closest: the loop keeps a hit when t < the current tmax, so it ends with the smallest t over the
//           accepting references and, among equal t (+0 == -0), the first in mask order
//           (kdtree.cpp:235-246); the pairs are reduced in ascending (window, lane) = mask order with a
//           strict <, which selects the same reference, and its own ux, uy, t are taken.
// Every lane of the wave must be active.  lx: 192 words of LDS owned by the wave (the window's start marks,
// every lane's mask and first record).

// the position of the q-th (from 0) set bit of m (q < popcount(m))
__device__ __forceinline__ uint32_t nth_bit(uint32_t m, uint32_t q) {
    uint32_t pos = 0;
#pragma unroll
    for (uint32_t w = 16; w >= 1; w >>= 1) {
        const uint32_t c = (uint32_t)__builtin_popcount(m & ((1u << w) - 1u));
        const bool up = q >= c;
        q = up ? q - c : q;
        m = up ? m >> w : m;
        pos = up ? pos + w : pos;
    }
    return pos;
}
__device__ __forceinline__ uint32_t bperm(uint32_t addr, uint32_t v) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)addr, (int)v);
}
__device__ __forceinline__ float bpermf(uint32_t addr, float v) { return __uint_as_float(bperm(addr, __float_as_uint(v))); }

typedef __attribute__((address_space(3))) uint32_t lds_u32;
// Inclusive prefix sum of x over the 64 lanes of a converged wave: row scans by DPP row shifts (out-of-row
// sources read 0), then rows 1 / 3 add lane 15 of the row below and rows 2 / 3 add lane 31.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, true); // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, true); // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, true); // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, true); // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false); // row_bcast:15
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false); // row_bcast:31
    return x;
}

// DPP: the prefix by wave_incl_scan instead of the six bit-sliced ballots
template <bool SHADOW, bool DPP = false>
__device__ __forceinline__ void leaf_exchange(const DevScene &S, volatile lds_u32 *lx, uint32_t m, uint32_t first,
                                              f3 o, f3 d, float tmax, uint32_t exclude, bool &occluded, bool &found,
                                              float &bx, float &by, float &bt, uint32_t &tri, Pc *pc = nullptr) {
    const uint32_t lane = lane_id();
    const uint32_t c = (uint32_t)__builtin_popcount(m);
    if (pc) { // the exchange's shape: rounds, windows (diters), owner lanes and their pairs
        const uint32_t owners = (uint32_t)__popcll(__ballot(c > 0u));
        if (wave_leader()) {
            pc->drounds++;
            pc->dlanes += owners;
        }
        pc->dtests += c;
    }
    // exclusive prefix P of c over the lanes and the total, bit-sliced (c <= 32)
    uint32_t P = 0, total = 0;
    if (DPP) {
        const uint32_t inc = wave_incl_scan(c);
        P = inc - c;
        total = __builtin_amdgcn_readlane(inc, 63);
    } else {
#pragma unroll
        for (int b = 0; b < 6; b++) {
            const uint64_t bal = __ballot((c >> b) & 1u);
            P += __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u)) << b;
            total += (uint32_t)__popcll(bal) << b;
        }
    }
    // this lane's pairs: [P, E) (packed: one register through the exchange)
    const uint32_t pe = P | ((P + c) << 16);
    occluded = found = false;
    // lx: [0, 64) the window's start marks, [64, 128) every lane's mask, [128, 192) its leaf's first record
    // (read from LDS by the pairs' testers, so they hold no registers during the exchange)
    volatile lds_u32 *const marks = lx;
    lx[64 + lane] = m;
    lx[128 + lane] = first;
    uint32_t carry = 0, carry_q = 0; // the owner of the pair before the window, and its rank + 1
    for (uint32_t base = 0; base < total; base += 64u) {
        // the owner of pair base + lane: the last lane that starts at or before it
        const uint32_t ln = lane_id(); // (re-derived per window: values hoisted out of this loop hold registers)
        marks[ln] = 0u;
        const uint32_t P0 = pe & 0xffffu, E0 = pe >> 16;
        if (E0 > P0 && P0 >= base && P0 < base + 64u) marks[P0 - base] = ln + 1u;
        const uint32_t mv = marks[ln];
        // the last start at or before this lane: s = ln - (its distance below), none when the shifted mask is 0
        const uint64_t upto = __ballot(mv != 0u) << (63u - ln);
        const uint32_t back = upto ? (uint32_t)__builtin_clzll(upto) : 0u;
        const uint32_t sm = bperm((ln - back) << 2, mv);
        const uint32_t owner = upto ? sm - 1u : carry;
        // q: the pair's rank among its owner's (a carried owner started before the window)
        const uint32_t q = upto ? back : ln + carry_q;
        carry = __builtin_amdgcn_readlane(owner, 63);
        carry_q = __builtin_amdgcn_readlane(q, 63) + 1u;
        const bool live = base + ln < total;
        const uint32_t a = owner << 2;
        const uint32_t om = lx[64 + owner], of = lx[128 + owner];
        const uint32_t j = nth_bit(om, q);                    // (any value < 32 for a dead lane)
        const uint32_t ref = live ? of + j : 0u;              // (record 0: a dead lane's harmless load)
        const TriRec r = load_rec(S, ref);
        if (pc) {
            if (wave_leader()) pc->diters++;
            pc->tests += live ? 1u : 0u;
            pc->vb += live ? 16u * REC_STRIDE : 0u;
        }
        // tri_test_wave's arithmetic with the owner's ray fetched in stages (the direction, then the origin,
        // then tmax), each where it is first used: the scheduler keeps them apart (fewer live registers)
        float ux, uy, t;
        bool acc;
        {
            const f3 od = mk(bpermf(a, d.x), bpermf(a, d.y), bpermf(a, d.z));
            const f3 v0 = ld3(r.a), e1 = ld3(r.b), e2 = ld3(r.c);
            const f3 p = cross(od, e2);
            const float aa = dot(e1, p);
            bool ok = live & !((aa < 1.19209290e-7F) & (aa > -1.19209290e-7F));
            acc = false;
            if (__ballot(ok)) {
                __builtin_amdgcn_sched_barrier(0);
                const f3 oo = mk(bpermf(a, o.x), bpermf(a, o.y), bpermf(a, o.z));
                const float f = rcp_rn_wave(aa);
                const f3 sv = sub(oo, v0);
                ux = f * dot(sv, p);
                ok = ok & !((ux < 0.f) | (ux > 1.f));
                if (__ballot(ok)) {
                    const f3 qv = cross(sv, e1);
                    uy = f * dot(od, qv);
                    ok = ok & !((uy < 0.f) | (uy + ux > 1.f));
                    if (__ballot(ok)) {
                        __builtin_amdgcn_sched_barrier(0);
                        const float ot = bpermf(a, tmax);
                        t = f * dot(e2, qv);
                        acc = ok & (t >= 0.f) & (t < ot);
                    }
                }
            }
        }
        if (SHADOW) {
            acc = acc & (rec_id(r) != bperm(a, exclude));
            const uint64_t h = __ballot(acc);
            // this lane's pairs in the window: [lo, hi)
            const uint32_t P1 = pe & 0xffffu, E1 = pe >> 16;
            const int lo = (int)P1 - (int)base, hi = (int)E1 - (int)base;
            const int l = lo < 0 ? 0 : lo, e = hi > 64 ? 64 : hi;
            if (h && l < e) {
                const uint64_t bits = h >> l;
                occluded = occluded | ((e - l == 64 ? bits : bits & ((1ull << (e - l)) - 1ull)) != 0ull);
            }
            // every lane with pairs past the window is occluded already: done
            if (!__ballot(E1 > P1 && !occluded && E1 > base + 64u)) break;
        } else {
            uint64_t h = __ballot(acc);
            while (h) { // ascending lanes = ascending mask order within each owner
                const uint32_t w = (uint32_t)__builtin_ctzll(h);
                h &= h - 1ull;
                const uint32_t ow = __builtin_amdgcn_readlane(owner, w);
                const float tw = __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(t), w));
                const float uxw = __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(ux), w));
                const float uyw = __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(uy), w));
                const uint32_t idw = __builtin_amdgcn_readlane(rec_id(r), w);
                const bool take = lane_id() == ow && (!found || (__float_as_uint(tw) & 0x7fffffffu) <
                                                               (__float_as_uint(bt) & 0x7fffffffu));
                found = found | take;
                bt = take ? tw : bt;
                bx = take ? uxw : bx;
                by = take ? uyw : by;
                tri = take ? idw : tri;
            }
        }
    }
}

// Per-query tallies are wave-aggregated LDS atomics: the callers run in
// divergent code, so a wave total cannot be kept wave-uniform in registers.
enum : int { T_CLOSEST = 0, T_SHADOW = 1, T_HIT = 5, T_TEXHIT = 6, T_PATHS = 7, T_PIXELS = 8, T_NEE = 9, T_N = 10 };
// the device counter slot of tally i (T_NEE: CTR_NEE, past the cr_counters fields of the Ctr order)
__device__ __forceinline__ int tally_slot(int i) { return i == T_NEE ? CTR_NEE : i; }
__device__ __forceinline__ void tally(unsigned long long *tl, int i, bool pred) {
    const uint64_t b = __ballot(pred);
    if (b && wave_leader()) atomicAdd(&tl[i], (unsigned long long)__popcll(b));
}

__device__ __forceinline__ float4 pk(f3 v, uint32_t w) { return make_float4(v.x, v.y, v.z, __uint_as_float(w)); }

// Wave-aggregated append: one atomicAdd per wave, slots in lane order.
__device__ __forceinline__ uint32_t wave_append(uint32_t *counter, bool pred) {
    const uint64_t m = __ballot(pred);
    if (!m) return 0;
    const uint32_t leader = (uint32_t)__ffsll((long long)m) - 1u;
    uint32_t base = 0;
    if ((threadIdx.x & 63u) == leader) base = atomicAdd(counter, (uint32_t)__popcll(m));
    base = __shfl(base, (int)leader, 64);
    return base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

} // namespace cr
