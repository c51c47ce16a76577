// leafcull.hpp -- leaf cull records: an exact skip of the Moller-Trumbore tests
// (kdtree.cpp:219-246 / 293-320) of secondary closest and shadow rays whose test
// segment cannot reach the triangles.
//
// A kd leaf's reference list holds every triangle that has a vertex on the leaf's side
// of each ancestor split, so most of its triangles lie far from the leaf's cell: on the
// sponza stand-in 96% of the tests a shadow ray performs are of triangles whose tight box
// the ray's test segment [0, tmax_leaf] does not even touch (scripts/leafcull_census.py).
// A test accepts only for a segment that reaches the triangle up to rounding, so those
// tests can be skipped -- exactly, if the rounding is bounded.
//
// The bound.  With sv = RN(o - A) and the record's e1, e2, Moller-Trumbore computes
// AA = e1.(d x e2), U = sv.(d x e2), V = d.(sv x e1), T = e2.(sv x e1) with rounding
// errors |dX| <= Ex (camcull.hpp's terms).  Let d be a unit vector (|d|_2 = 1 +- 8u,
// checked per ray), S >= |sv_i| (the origin against the group box), E >= |e1|_1 + |e2|_1
// and g >= E^2 / |e1 x e2| for every triangle of a group.  Then
//     Ea <= 10.04u E^2,  Eu, Ev <= 10.04u S E,  Et <= 10.04u S E^2        (u = 2^-24)
// and for any accepting evaluation with |AA| > Ea (so sign(AA) is the computed one) the
// exact solution o' + t* d = A + u* e1 + v* e2 (o' = A + sv, |o' - o|_i <= u S) has
// barycentric weights >= -m, m <= 10.05u (1 + 2S/E) g / cb + 3.1u, where cb <= |d^.n^|
// bounds the cosine between the ray and the triangle's normal line: |AA| >= |n| cb.
// So the point o + t* d lies within pad = 2 m E + u S of the triangle's box, at
//     t* in [-dt, tmax (1 + 10.05u g / cb)(1 + 2.1u) + dt],  dt = 10.05u S g / cb.
// cb comes from a cone of normal lines per group: every |a^.n^| >= ct (= cos theta), so
// |d^.n^| >= cos(psi + theta) with cos psi = |d^.a^|.  A grazing ray (cb small) gets a
// large pad or none (cb <= 20.2u g: never skipped) -- with |AA| near its rounding error
// the test can accept anywhere along a line close to the triangle's PLANE, so no box
// bound holds there, and a single cone per leaf would be too wide (columns, corners):
// the leaf's triangles are split into two groups by normal direction (k-means on normal
// lines), each with its own box and cone.  Degenerate triangles are always tested.
//
// Record per kd node (LC_REC float4, leaves with 1..32 references; others test all):
//   {lo0, g0} {hi0, E0} {axis0, ct0} {lo1, g1} {hi1, E1} {axis1, ct1}
//   {mask0, mask1, always, 0}   (bit j: reference first + j is in group 0 / 1 / tested always)
// The kernel evaluates the skip in float with every rounding of its own accounted for
// (leaf_cull_mask); tests/native/leafcull_check.cpp checks the whole argument against
// the float test on random and adversarial rays and triangles.
#pragma once
#include <float.h>
#include <math.h>
#include <stdint.h>

#if defined(__HIPCC__)
#define CR_LC_HD __host__ __device__
#else
#define CR_LC_HD
#endif

namespace cr {

enum { LC_REC = 7, LC_MAXREFS = 32 };

struct LcFloat4 {
    float x, y, z, w;
};

// 1 when |d|^2 is within 12u of 1 (so |d| = 1 +- 8u): the bound assumes unit directions
CR_LC_HD inline bool lc_unit(float dx, float dy, float dz) {
    const float dd = (dx * dx + dy * dy) + dz * dz;
    return fabsf(dd - 1.f) <= 12.f * 0x1p-24f;
}

// One group's skip for ray (o, d) (unit, inv = RN(1/d)), segment [0, tmax]; db bounds
// |coordinate| of the scene (origins and vertices).  True: no triangle of the group can
// accept.  Float arithmetic, every rounding covered by a margin.
CR_LC_HD inline bool lc_group_skip(const float o[3], const float d[3], const float inv[3], float tmax, float db,
                                   LcFloat4 lo, LcFloat4 hi, LcFloat4 ax) {
    const float u = 0x1p-24f;
    const float g = lo.w, E = hi.w, ct = ax.w;
    // cos psi >= |d.a| - 16u (rounding of the dot, |d|, |a| = 1 +- 8u); sin psi and sin theta from above
    const float dn = fabsf((d[0] * ax.x + d[1] * ax.y) + d[2] * ax.z);
    const float cpl = fmaxf(dn - 16.f * u, 0.f);
    const float sph = sqrtf(fmaxf(1.f - cpl * cpl, 0.f) + 3.f * u) * (1.f + u);
    const float sth = sqrtf(fmaxf(1.f - ct * ct, 0.f) + 3.f * u) * (1.f + u);
    const float cb = (cpl * ct - sph * sth) - 3.f * u;
    if (!(cb > 20.2f * u * g)) return false; // grazing (or NaN): the test could accept anywhere near the plane
    float S = 0.f;
    for (int i = 0; i < 3; i++) S = fmaxf(S, fmaxf(fabsf(o[i] - (&lo.x)[i]), fabsf(o[i] - (&hi.x)[i])));
    S *= 1.f + 3.f * u;
    const float ic = (1.f / cb) * (1.f + 2.f * u);
    // the slab arithmetic below rounds coordinates up to max(db, |o|): 4u of that on top
    const float mb = fmaxf(db, fmaxf(fabsf(o[0]), fmaxf(fabsf(o[1]), fabsf(o[2]))));
    const float pad = ((20.11f * u) * (E + 2.f * S) * g * ic + (6.21f * u) * E + u * S) * (1.f + 8.f * u) +
                      4.f * u * mb + 1e-20f;
    const float dt = ((10.06f * u) * S * g * ic) * (1.f + 4.f * u) + 1e-20f;
    const float t_hi = (tmax * (1.f + (10.06f * u) * g * ic) * (1.f + 3.f * u)) * (1.f + 2.f * u) + dt;
    const float t_lo = -dt;
    float tn = -INFINITY, tf = INFINITY;
    for (int i = 0; i < 3; i++) {
        const float t0 = (((&lo.x)[i] - pad) - o[i]) * inv[i], t1 = (((&hi.x)[i] + pad) - o[i]) * inv[i];
        const bool nan = !(t0 == t0) || !(t1 == t1); // o on a face with d_i = 0: the whole line
        const float a = nan ? -INFINITY : (t0 < t1 ? t0 : t1), b = nan ? INFINITY : (t0 < t1 ? t1 : t0);
        tn = a > tn ? a : tn;
        tf = b < tf ? b : tf;
    }
    // the slab parameters carry 3u of relative rounding: widen before deciding
    tn -= 4.f * u * fabsf(tn);
    tf += 4.f * u * fabsf(tf);
    return (tn > tf) | (tn > t_hi) | (tf < t_lo);
}

// The same skip with the per-ray terms bounded once per scene (records of
// leaf_cull_record_fixed): every ray whose |d.a| - 16u >= kappa has cb >= C0 on the group,
// and with S <= the scene's extent the pad, dt and the tmax factor are constants of the
// group -- the box comes pre-padded, so a ray does one dot product and a slab test.
//   {lo - pad, kappa} {hi + pad, dt} {axis, tk}:  skip iff |d.a| >= kappa and
//   o + t d misses the box for t in [-dt, tmax tk + dt]
enum { LC_C0_INV = 16 }; // C0 = 1/16: rays within ~86 degrees of every normal of the group
CR_LC_HD inline bool lc_group_skip_fixed(const float o[3], const float d[3], const float inv[3], float tmax, LcFloat4 lo,
                                         LcFloat4 hi, LcFloat4 ax) {
    const float u = 0x1p-24f;
    const float dn = fabsf((d[0] * ax.x + d[1] * ax.y) + d[2] * ax.z);
    if (!(dn >= lo.w)) return false; // possibly grazing (or NaN): never skipped
    const float dt = hi.w, t_hi = (tmax * ax.w) * (1.f + 2.f * u) + dt, t_lo = -dt;
    float tn = -INFINITY, tf = INFINITY;
    for (int i = 0; i < 3; i++) {
        const float t0 = ((&lo.x)[i] - o[i]) * inv[i], t1 = ((&hi.x)[i] - o[i]) * inv[i];
        const bool nan = !(t0 == t0) || !(t1 == t1);
        const float a = nan ? -INFINITY : (t0 < t1 ? t0 : t1), b = nan ? INFINITY : (t0 < t1 ? t1 : t0);
        tn = a > tn ? a : tn;
        tf = b < tf ? b : tf;
    }
    tn -= 4.f * u * fabsf(tn);
    tf += 4.f * u * fabsf(tf);
    return (tn > tf) | (tn > t_hi) | (tf < t_lo);
}
CR_LC_HD inline uint32_t leaf_cull_mask_fixed(const float o[3], const float d[3], const float inv[3], bool unit,
                                              float tmax, const LcFloat4 *rec, uint32_t count) {
    const uint32_t all = count >= 32 ? 0xffffffffu : ((1u << count) - 1u);
    if (!unit || count > (uint32_t)LC_MAXREFS) return all;
    const LcFloat4 m = rec[6];
    uint32_t keep, m0, m1;
    __builtin_memcpy(&keep, &m.z, 4);
    __builtin_memcpy(&m0, &m.x, 4);
    __builtin_memcpy(&m1, &m.y, 4);
    if (m0 && !lc_group_skip_fixed(o, d, inv, tmax, rec[0], rec[1], rec[2])) keep |= m0;
    if (m1 && !lc_group_skip_fixed(o, d, inv, tmax, rec[3], rec[4], rec[5])) keep |= m1;
    return keep & all;
}

// Packed fixed-pad records (LC_RECP float4, leaves of up to 16 references): the three masks
// ride in the low 8 mantissa bits of the six per-group constants kappa, dt, tk -- each
// rounded UP to a multiple of 256 ulps first, so the bits only enlarge a bound that is
// already an upper one.  {lo0, kappa0} {hi0, dt0} {axis0, tk0} {lo1, kappa1} {hi1, dt1} {axis1, tk1};
// mask0 = kappa0 | dt0 << 8, mask1 = tk0 | kappa1 << 8, always = dt1 | tk1 << 8 (low bytes).
enum { LC_RECP = 6, LC_MAXREFS_P = 16 };
CR_LC_HD inline uint32_t lc_lowbyte(float f) {
    uint32_t b;
    __builtin_memcpy(&b, &f, 4);
    return b & 0xffu;
}
CR_LC_HD inline uint32_t leaf_cull_mask_packed(const float o[3], const float d[3], const float inv[3], bool unit,
                                               float tmax, const LcFloat4 *rec, uint32_t count) {
    const uint32_t all = count >= 32 ? 0xffffffffu : ((1u << count) - 1u);
    if (!unit || count > (uint32_t)LC_MAXREFS_P) return all;
    const uint32_t m0 = lc_lowbyte(rec[0].w) | lc_lowbyte(rec[1].w) << 8;
    const uint32_t m1 = lc_lowbyte(rec[2].w) | lc_lowbyte(rec[3].w) << 8;
    uint32_t keep = lc_lowbyte(rec[4].w) | lc_lowbyte(rec[5].w) << 8;
    if (m0 && !lc_group_skip_fixed(o, d, inv, tmax, rec[0], rec[1], rec[2])) keep |= m0;
    if (m1 && !lc_group_skip_fixed(o, d, inv, tmax, rec[3], rec[4], rec[5])) keep |= m1;
    return keep & all;
}

// Compressed fixed-pad records (LC_RECC uint4 = 48 B per node, leaves of up to 16 references):
// the packed record's six 16-B loads per leaf were the secondary and shadow traces' largest
// load-instruction cost.  Twelve words:
//   {box0 x, y, z} {ax0.x | ax0.y << 16} {ax0.z | kappa0 << 16} {dt0 | dt1 << 16}
//   {box1 x, y, z} {ax1.x | ax1.y << 16} {ax1.z | kappa1 << 16} {mask0 | mask1 << 16}
// box word: lo | hi << 16 on the scene's grid (LcGrid: base + q * step), lo rounded down and hi up
// past the fixed-pad box by the rounding of the kernels' fused evaluation (below); the normal
// cone's axis as three IEEE halves (any vector: kappa is recomputed for the decoded one), kappa
// and dt as halves rounded up; tk is one bound for the whole scene (LcGrid::tk).  A reference in
// neither mask is tested always.  Every change against the fixed-pad record only enlarges a bound,
// so the skip stays exact (tests/native/leafcull_check.cpp, form 3).
// The slab parameter of a grid plane q is RN(RN(fma(q, step, RN(base - o))) * inv): the plane
// moves by |RN(base - o) - (base - o)| <= u |base - o| <= u (|base| + db), which the host pads;
// the relative rounding is that of the fixed form's RN(RN(lo - o) * inv).
enum { LC_RECC = 3 };
struct LcGrid {
    float base[3], step[3], tk;
    float pad; // (host: the margin every box got past its fixed-pad bounds)
    float dt0; // the short records' dt unit (LC_RECS: dt = dt0 2^e; lc_grid_dt)
};
// an IEEE half (low 16 bits of h) as float: exact
CR_LC_HD inline float lc_half(uint32_t h) {
#if defined(__HIP_DEVICE_COMPILE__)
    return (float)__builtin_bit_cast(_Float16, (unsigned short)h);
#else
    const uint32_t e = (h >> 10) & 31u, m = h & 1023u;
    const float v = e == 0 ? ldexpf((float)m, -24) : e == 31 ? (m ? NAN : INFINITY) : ldexpf((float)(m | 1024u), (int)e - 25);
    return (h & 0x8000u) ? -v : v;
#endif
}
// lc_group_skip_fixed on a compressed group (bo[i] = RN(base[i] - o[i])).  FINITE: every inv[i] is
// finite, so no slab parameter is NaN (0 * inf) -- entry and exit are then plain min / max, the
// values the NaN-aware selects give (up to the sign of a zero, which no comparison below sees)
template <bool FINITE = false>
CR_LC_HD inline bool lc_group_skip_c(const float d[3], const float inv[3], const float bo[3], float tmax,
                                     const uint32_t box[3], uint32_t axw, uint32_t azk, float dt, const LcGrid &G) {
    const float u = 0x1p-24f;
    const float dn = fabsf((d[0] * lc_half(axw & 0xffffu) + d[1] * lc_half(axw >> 16)) + d[2] * lc_half(azk & 0xffffu));
    if (!(dn >= lc_half(azk >> 16))) return false; // possibly grazing (or NaN): never skipped
    const float t_hi = (tmax * G.tk) * (1.f + 2.f * u) + dt, t_lo = -dt;
    float tn = -INFINITY, tf = INFINITY;
    for (int i = 0; i < 3; i++) {
        const float t0 = fmaf((float)(box[i] & 0xffffu), G.step[i], bo[i]) * inv[i];
        const float t1 = fmaf((float)(box[i] >> 16), G.step[i], bo[i]) * inv[i];
        if (FINITE) {
            tn = i ? fmaxf(tn, fminf(t0, t1)) : fminf(t0, t1);
            tf = i ? fminf(tf, fmaxf(t0, t1)) : fmaxf(t0, t1);
        } else {
            const bool nan = !(t0 == t0) || !(t1 == t1);
            const float a = nan ? -INFINITY : (t0 < t1 ? t0 : t1), b = nan ? INFINITY : (t0 < t1 ? t1 : t0);
            tn = a > tn ? a : tn;
            tf = b < tf ? b : tf;
        }
    }
    // the slab parameters carry 4u of relative rounding (4u |t| is exact: the fma rounds once)
    tn = fmaf(-4.f * u, fabsf(tn), tn);
    tf = fmaf(4.f * u, fabsf(tf), tf);
    return (tn > tf) | (tn > t_hi) | (tf < t_lo);
}
CR_LC_HD inline uint32_t leaf_cull_mask_c(const float o[3], const float d[3], const float inv[3], bool unit, float tmax,
                                          const uint32_t w[12], uint32_t count, const LcGrid &G) {
    const uint32_t all = count >= 32 ? 0xffffffffu : ((1u << count) - 1u);
    if (!unit || count > (uint32_t)LC_MAXREFS_P) return all;
    const uint32_t m0 = w[11] & 0xffffu, m1 = w[11] >> 16;
    const float bo[3] = {G.base[0] - o[0], G.base[1] - o[1], G.base[2] - o[2]};
    const float dt0 = lc_half(w[5] & 0xffffu), dt1 = lc_half(w[5] >> 16);
    uint32_t drop = 0u;
    if (fabsf(inv[0]) < INFINITY && fabsf(inv[1]) < INFINITY && fabsf(inv[2]) < INFINITY) {
        if (m0 && lc_group_skip_c<true>(d, inv, bo, tmax, w, w[3], w[4], dt0, G)) drop |= m0;
        if (m1 && lc_group_skip_c<true>(d, inv, bo, tmax, w + 6, w[9], w[10], dt1, G)) drop |= m1;
    } else {
        if (m0 && lc_group_skip_c(d, inv, bo, tmax, w, w[3], w[4], dt0, G)) drop |= m0;
        if (m1 && lc_group_skip_c(d, inv, bo, tmax, w + 6, w[9], w[10], dt1, G)) drop |= m1;
    }
    return all & ~drop;
}

// Short compressed records (LC_RECS uint4 = 32 B per node, leaves of up to 16 references): the
// compressed record in two 16-B loads, or one 32-B scalar load -- the secondary and shadow traces'
// cost follows their load instructions.  Eight words:
//   {box0 x, y, z} {box1 x, y, z}                        as LC_RECC's (lo | hi << 16 on grid G)
//   {ax0.p | ax0.q << 7 | ax1.p << 14 | ax1.q << 21 | e0 << 28}
//   {mask0 | kappa0 << 16 | kappa1 << 22 | e1 << 28}
// Group 0 is mask0's references, group 1 the leaf's others (a leaf whose references include ones
// tested always puts them in group 1, and never skips it).  Axis k: the normal LINE's octahedral
// coordinates on the upper hemisphere, x = RN(fma(p, RN(1/63), -1)), y the same of q, z =
// RN(RN(1 - |x|) - |y|) -- any vector: kappa is computed for the decoded one; kappa = RN(c RN(1/62))
// (c = 63 with the axis (0, 0, 1) is above any |d.v|: never skipped); dt = G.dt0 2^e.  Every field only enlarges a bound of
// the fixed-pad record, so the skip stays exact (tests/native/leafcull_check.cpp, form 4).
enum { LC_RECS = 2 };
CR_LC_HD inline float lc_axis_s(uint32_t c) { return fmaf((float)c, 1.f / 63.f, -1.f); }
CR_LC_HD inline float lc_kappa_s(uint32_t c) { return (float)c * (1.f / 62.f); }
// the slab part of lc_group_skip_c for the segment [t_lo, t_hi]
template <bool FINITE>
CR_LC_HD inline bool lc_slab_skip(const float inv[3], const float bo[3], const uint32_t box[3], float t_lo, float t_hi,
                                  const LcGrid &G) {
    const float u = 0x1p-24f;
    float tn = -INFINITY, tf = INFINITY;
    for (int i = 0; i < 3; i++) {
        const float t0 = fmaf((float)(box[i] & 0xffffu), G.step[i], bo[i]) * inv[i];
        const float t1 = fmaf((float)(box[i] >> 16), G.step[i], bo[i]) * inv[i];
        if (FINITE) {
            tn = i ? fmaxf(tn, fminf(t0, t1)) : fminf(t0, t1);
            tf = i ? fminf(tf, fmaxf(t0, t1)) : fmaxf(t0, t1);
        } else {
            const bool nan = !(t0 == t0) || !(t1 == t1);
            const float a = nan ? -INFINITY : (t0 < t1 ? t0 : t1), b = nan ? INFINITY : (t0 < t1 ? t1 : t0);
            tn = a > tn ? a : tn;
            tf = b < tf ? b : tf;
        }
    }
    tn = fmaf(-4.f * u, fabsf(tn), tn);
    tf = fmaf(4.f * u, fabsf(tf), tf);
    return (tn > tf) | (tn > t_hi) | (tf < t_lo);
}
template <bool FINITE>
CR_LC_HD inline uint32_t leaf_cull_drop_s(const float d[3], const float inv[3], const float bo[3], float th,
                                          const uint32_t w[8], uint32_t m0, uint32_t m1, const LcGrid &G) {
    uint32_t drop = 0u;
#pragma unroll
    for (int k = 0; k < 2; k++) {
        const uint32_t m = k ? m1 : m0;
        if (!m) continue;
        const uint32_t a = w[6] >> (14 * k);
        const float x = lc_axis_s(a & 127u), y = lc_axis_s((a >> 7) & 127u);
        const float z = (1.f - fabsf(x)) - fabsf(y);
        const float dn = fabsf((d[0] * x + d[1] * y) + d[2] * z);
        if (!(dn >= lc_kappa_s((w[7] >> (16 + 6 * k)) & 63u))) continue; // possibly grazing (or NaN)
        const float dt = ldexpf(G.dt0, (int)(w[6 + k] >> 28));
        if (lc_slab_skip<FINITE>(inv, bo, w + 3 * k, -dt, th + dt, G)) drop |= m;
    }
    return drop;
}
CR_LC_HD inline uint32_t leaf_cull_mask_s(const float o[3], const float d[3], const float inv[3], bool unit, float tmax,
                                          const uint32_t w[8], uint32_t count, const LcGrid &G) {
    const uint32_t all = count >= 32 ? 0xffffffffu : ((1u << count) - 1u);
    if (!unit || count > (uint32_t)LC_MAXREFS_P) return all;
    const uint32_t m0 = w[7] & 0xffffu & all, m1 = all & ~m0;
    const float bo[3] = {G.base[0] - o[0], G.base[1] - o[1], G.base[2] - o[2]};
    const float th = (tmax * G.tk) * (1.f + 2.f * 0x1p-24f);
    const uint32_t drop = fabsf(inv[0]) < INFINITY && fabsf(inv[1]) < INFINITY && fabsf(inv[2]) < INFINITY
                              ? leaf_cull_drop_s<true>(d, inv, bo, th, w, m0, m1, G)
                              : leaf_cull_drop_s<false>(d, inv, bo, th, w, m0, m1, G);
    return all & ~drop;
}

// The references of a leaf (count of them) its tests need for this ray: bit j for
// reference first + j.  rec: the node's LC_REC float4.  Leaves beyond LC_MAXREFS and
// non-unit rays: every reference (the caller tests count references then).
CR_LC_HD inline uint32_t leaf_cull_mask(const float o[3], const float d[3], const float inv[3], bool unit,
                                        float tmax, float db, const LcFloat4 *rec, uint32_t count) {
    const uint32_t all = count >= 32 ? 0xffffffffu : ((1u << count) - 1u);
    if (!unit || count > (uint32_t)LC_MAXREFS) return all;
    const LcFloat4 m = rec[6];
    uint32_t keep;
    __builtin_memcpy(&keep, &m.z, 4);
    uint32_t m0, m1;
    __builtin_memcpy(&m0, &m.x, 4);
    __builtin_memcpy(&m1, &m.y, 4);
    if (m0 && !lc_group_skip(o, d, inv, tmax, db, rec[0], rec[1], rec[2])) keep |= m0;
    if (m1 && !lc_group_skip(o, d, inv, tmax, db, rec[3], rec[4], rec[5])) keep |= m1;
    return keep & all;
}

// Host: the record of a leaf from its references' floats as the test uses them
// (A, e1, e2 per reference, in list order).  count 0 or > LC_MAXREFS: every bit "always".
inline void leaf_cull_record(const float (*A)[3], const float (*e1)[3], const float (*e2)[3], uint32_t count,
                             LcFloat4 out[LC_REC]) {
    for (int i = 0; i < LC_REC; i++) out[i] = LcFloat4{0.f, 0.f, 0.f, 0.f};
    auto put_u = [](float &f, uint32_t v) { __builtin_memcpy(&f, &v, 4); };
    if (count == 0 || count > (uint32_t)LC_MAXREFS) {
        put_u(out[6].z, 0xffffffffu);
        return;
    }
    double N[LC_MAXREFS][3], Ev[LC_MAXREFS], Gv[LC_MAXREFS];
    bool ok[LC_MAXREFS];
    for (uint32_t j = 0; j < count; j++) {
        const double a[3] = {e1[j][0], e1[j][1], e1[j][2]}, b[3] = {e2[j][0], e2[j][1], e2[j][2]};
        const double n[3] = {a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]};
        const double nl = sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
        double mag = 0;
        for (int i = 0; i < 3; i++) mag = fmax(mag, fabs(A[j][i]));
        Ev[j] = (fabs(a[0]) + fabs(a[1]) + fabs(a[2])) + (fabs(b[0]) + fabs(b[1]) + fabs(b[2]));
        ok[j] = nl > 0 && nl < 1e30 && Ev[j] < 1e15 && mag < 1e15;
        Gv[j] = ok[j] ? Ev[j] * Ev[j] / nl * (1 + 1e-12) : 0;
        ok[j] = ok[j] && Gv[j] < 1e20;
        for (int i = 0; i < 3; i++) N[j][i] = ok[j] ? n[i] / nl : 0;
    }
    // two groups of normal LINES (sign-free): farthest-point start, k-means on |cos|
    double C[2][3] = {{0, 0, 0}, {0, 0, 0}};
    int nc = 0;
    for (uint32_t j = 0; j < count && !nc; j++)
        if (ok[j]) {
            for (int i = 0; i < 3; i++) C[0][i] = N[j][i];
            nc = 1;
        }
    if (nc) {
        double worst = 2;
        int wj = -1;
        for (uint32_t j = 0; j < count; j++) {
            if (!ok[j]) continue;
            const double c = fabs(N[j][0] * C[0][0] + N[j][1] * C[0][1] + N[j][2] * C[0][2]);
            if (c < worst) {
                worst = c;
                wj = (int)j;
            }
        }
        if (wj >= 0 && worst < 0.999999) {
            for (int i = 0; i < 3; i++) C[1][i] = N[wj][i];
            nc = 2;
        }
    }
    int lab[LC_MAXREFS];
    for (int it = 0; it < 12 && nc; it++) {
        double M[2][9] = {};
        for (uint32_t j = 0; j < count; j++) {
            if (!ok[j]) continue;
            int q = 0;
            double best = -1;
            for (int k = 0; k < nc; k++) {
                const double c = fabs(N[j][0] * C[k][0] + N[j][1] * C[k][1] + N[j][2] * C[k][2]);
                if (c > best) {
                    best = c;
                    q = k;
                }
            }
            lab[j] = q;
            for (int a = 0; a < 3; a++)
                for (int b = 0; b < 3; b++) M[q][3 * a + b] += N[j][a] * N[j][b];
        }
        for (int k = 0; k < nc; k++) { // principal direction of the group's normal lines
            double v[3] = {C[k][0], C[k][1], C[k][2]};
            for (int r = 0; r < 40; r++) {
                const double w[3] = {M[k][0] * v[0] + M[k][1] * v[1] + M[k][2] * v[2],
                                     M[k][3] * v[0] + M[k][4] * v[1] + M[k][5] * v[2],
                                     M[k][6] * v[0] + M[k][7] * v[1] + M[k][8] * v[2]};
                const double l = sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
                if (!(l > 0)) break;
                for (int i = 0; i < 3; i++) v[i] = w[i] / l;
            }
            for (int i = 0; i < 3; i++) C[k][i] = v[i];
        }
    }
    uint32_t mask[2] = {0u, 0u}, always = 0u;
    double lo[2][3], hi[2][3], g[2] = {0, 0}, E[2] = {0, 0};
    float axf[2][3];
    double ct[2] = {1, 1};
    for (int k = 0; k < 2; k++) {
        // the axis as the kernel reads it (float), normalised; the cone is measured against it
        double l = 0;
        for (int i = 0; i < 3; i++) {
            axf[k][i] = (float)C[k][i];
            l += (double)axf[k][i] * axf[k][i];
        }
        l = sqrt(l);
        for (int i = 0; i < 3; i++) {
            lo[k][i] = INFINITY;
            hi[k][i] = -INFINITY;
        }
        if (!(l > 0)) ct[k] = 0;
        C[k][0] = l > 0 ? axf[k][0] / l : 0;
        C[k][1] = l > 0 ? axf[k][1] / l : 0;
        C[k][2] = l > 0 ? axf[k][2] / l : 0;
    }
    for (uint32_t j = 0; j < count; j++) {
        if (!ok[j] || !nc) {
            always |= 1u << j;
            continue;
        }
        int q = 0;
        double best = -1;
        for (int k = 0; k < nc; k++) {
            const double c = fabs(N[j][0] * C[k][0] + N[j][1] * C[k][1] + N[j][2] * C[k][2]);
            if (c > best) {
                best = c;
                q = k;
            }
        }
        mask[q] |= 1u << j;
        ct[q] = fmin(ct[q], best);
        g[q] = fmax(g[q], Gv[j]);
        E[q] = fmax(E[q], Ev[j]);
        // the triangle the test solves for: A, A + e1, A + e2 (exact, not the model's B, C)
        for (int i = 0; i < 3; i++) {
            const double a = A[j][i], b = a + (double)e1[j][i], c = a + (double)e2[j][i];
            lo[q][i] = fmin(lo[q][i], fmin(a, fmin(b, c)));
            hi[q][i] = fmax(hi[q][i], fmax(a, fmax(b, c)));
        }
    }
    auto down = [](double x) {
        float f = (float)x;
        if ((double)f > x) f = nextafterf(f, -INFINITY);
        return f;
    };
    auto up = [](double x) {
        float f = (float)x;
        if ((double)f < x) f = nextafterf(f, INFINITY);
        return f;
    };
    for (int k = 0; k < 2; k++) {
        if (!mask[k]) continue;
        // 1e-9 below the measured cosine: the double evaluation of the normals and the axis
        const double c = fmax(0.0, ct[k] - 1e-9);
        out[3 * k + 0] = LcFloat4{down(lo[k][0]), down(lo[k][1]), down(lo[k][2]), up(g[k] * (1 + 1e-9))};
        out[3 * k + 1] = LcFloat4{up(hi[k][0]), up(hi[k][1]), up(hi[k][2]), up(E[k] * (1 + 1e-9))};
        out[3 * k + 2] = LcFloat4{axf[k][0], axf[k][1], axf[k][2], down(c)};
    }
    put_u(out[6].x, mask[0]);
    put_u(out[6].y, mask[1]);
    put_u(out[6].z, always);
}

// Host: leaf_cull_record turned into the fixed-pad form (lc_group_skip_fixed) for a scene
// whose origins and vertices have |coordinate| <= db and differ by at most smax per axis.
// The bound of lc_group_skip with cb >= C0 and S = smax, every factor rounded upward.
inline void leaf_cull_fixed(const LcFloat4 in[LC_REC], double db, double smax, LcFloat4 out[LC_REC]) {
    auto up = [](double x) {
        float f = (float)x;
        if ((double)f < x) f = nextafterf(f, INFINITY);
        return f;
    };
    auto down = [](double x) {
        float f = (float)x;
        if ((double)f > x) f = nextafterf(f, -INFINITY);
        return f;
    };
    const double u = 0x1p-24, c0 = 1.0 / LC_C0_INV, S = smax * (1 + 4 * u) + 1e-6;
    for (int k = 0; k < 2; k++) {
        const LcFloat4 lo = in[3 * k], hi = in[3 * k + 1], ax = in[3 * k + 2];
        const double g = lo.w, E = hi.w, ct = ax.w;
        // kappa: |d^.a^| >= kappa  =>  cos(psi + theta) >= c0 (the float dot's 16u margin added here)
        const double th = acos(fmin(1.0, fmax(0.0, ct))), room = acos(c0) - th;
        double kappa = room > 1e-6 ? cos(room) + 1e-12 : 2.0;
        if (!(c0 > 20.2 * u * g) || !(g < 1e20)) kappa = 2.0; // no useful bound: never skip
        kappa += 16 * u;
        const double pad = (20.11 * u * (E + 2 * S) * g / c0 + 6.21 * u * E + u * S) * (1 + 1e-6) + 4 * u * db + 1e-20;
        const double dt = 10.06 * u * S * g / c0 * (1 + 1e-6) + 1e-20;
        const double tk = (1 + 10.06 * u * g / c0) * (1 + 3 * u) * (1 + 1e-6);
        out[3 * k] = LcFloat4{down((double)lo.x - pad), down((double)lo.y - pad), down((double)lo.z - pad), up(kappa)};
        out[3 * k + 1] = LcFloat4{up((double)hi.x + pad), up((double)hi.y + pad), up((double)hi.z + pad), up(dt)};
        out[3 * k + 2] = LcFloat4{ax.x, ax.y, ax.z, up(tk)};
    }
    out[6] = in[6];
}

// Host: the fixed-pad record packed into LC_RECP float4 (leaf_cull_mask_packed); leaves of
// more than 16 references keep every reference (the masks cannot hold them).
inline void leaf_cull_pack(const LcFloat4 fx[LC_REC], uint32_t count, LcFloat4 out[LC_RECP]) {
    uint32_t m[3];
    __builtin_memcpy(&m[0], &fx[6].x, 4);
    __builtin_memcpy(&m[1], &fx[6].y, 4);
    __builtin_memcpy(&m[2], &fx[6].z, 4);
    if (count > (uint32_t)LC_MAXREFS_P) {
        m[0] = m[1] = 0u;
        m[2] = 0xffffu;
    }
    for (int i = 0; i < LC_RECP; i++) out[i] = fx[i];
    // the six constants (kappa, dt, tk per group), each carrying one byte of the masks
    float *w[6] = {&out[0].w, &out[1].w, &out[2].w, &out[3].w, &out[4].w, &out[5].w};
    const uint32_t bytes[6] = {m[0] & 0xffu, (m[0] >> 8) & 0xffu, m[1] & 0xffu, (m[1] >> 8) & 0xffu, m[2] & 0xffu,
                               (m[2] >> 8) & 0xffu};
    for (int i = 0; i < 6; i++) {
        float f = *w[i];
        uint32_t b;
        __builtin_memcpy(&b, &f, 4);
        // positive finite constants: round up to a multiple of 256 ulps, then the byte
        if (!(f > 0.f) || !(f < 1e30f)) b = 0x7f000000u; // (2^127: a group that never passes)
        b = ((b + 0xffu) & ~0xffu) | bytes[i];
        __builtin_memcpy(w[i], &b, 4);
    }
}

// Host: the smallest IEEE half >= x (x >= 0; +inf when none is)
inline uint32_t lc_half_up(double x) {
    if (!(x >= 0.0)) return x < 0.0 ? 0u : 0x7c00u;
    if (!(x <= 65504.0)) return 0x7c00u;
    uint32_t lo = 0u, hi = 0x7bffu;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) / 2u;
        if ((double)lc_half(mid) >= x) hi = mid;
        else lo = mid + 1u;
    }
    return lo;
}
// Host: the nearest IEEE half to x (finite x within the half range)
inline uint32_t lc_half_near(double x) {
    const uint32_t sg = x < 0 ? 0x8000u : 0u;
    const uint32_t h = lc_half_up(fabs(x));
    if (h == 0u || h >= 0x7c00u) return sg | (h >= 0x7c00u ? 0x7bffu : 0u);
    return sg | ((double)lc_half(h) - fabs(x) <= fabs(x) - (double)lc_half(h - 1u) ? h : h - 1u);
}
// Host: the scene's grid from the fixed-pad boxes of every group that has references (fx: LC_REC
// float4 per node, n nodes), for origins with |o_i| <= db.  pad: the fused evaluation moves a plane by
// up to u |base - o| <= u (|base| + db); the boxes get 2.5 times that bound (the rest covers the host's
// double arithmetic); tk = the largest group tk.
inline LcGrid lc_grid_make(const LcFloat4 *fx, size_t n, double db) {
    double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    float tk = 1.f;
    for (size_t i = 0; i < n; i++) {
        const LcFloat4 *r = fx + (size_t)LC_REC * i;
        uint32_t m[2];
        __builtin_memcpy(&m[0], &r[6].x, 4);
        __builtin_memcpy(&m[1], &r[6].y, 4);
        for (int k = 0; k < 2; k++) {
            if (!m[k]) continue;
            const float l[3] = {r[3 * k].x, r[3 * k].y, r[3 * k].z}, h[3] = {r[3 * k + 1].x, r[3 * k + 1].y, r[3 * k + 1].z};
            bool fin = fabs(r[3 * k + 2].w) < 1e30;
            for (int a = 0; a < 3; a++) fin = fin && fabs(l[a]) < 1e30 && fabs(h[a]) < 1e30; // (NaN: false)
            if (!fin) continue;
            for (int a = 0; a < 3; a++) {
                lo[a] = fmin(lo[a], (double)l[a]);
                hi[a] = fmax(hi[a], (double)h[a]);
            }
            tk = fmaxf(tk, r[3 * k + 2].w);
        }
    }
    double M = db;
    for (int a = 0; a < 3; a++)
        if (lo[a] <= hi[a]) M = fmax(M, fmax(fabs(lo[a]), fabs(hi[a])));
    const double pad = 2.5 * 0x1p-24 * (db + M) * (1 + 1e-6) + 1e-30;
    LcGrid G;
    G.pad = (float)pad;
    if ((double)G.pad < pad) G.pad = nextafterf(G.pad, INFINITY);
    for (int a = 0; a < 3; a++) {
        if (lo[a] <= hi[a]) {
            lo[a] -= 2 * (double)G.pad;
            hi[a] += 2 * (double)G.pad;
        }
        if (!(lo[a] <= hi[a])) lo[a] = hi[a] = 0.0;
        G.base[a] = (float)lo[a];
        if ((double)G.base[a] > lo[a]) G.base[a] = nextafterf(G.base[a], -INFINITY);
        float s = (float)((hi[a] - (double)G.base[a]) / 65535.0);
        if (!(s > 0.f)) s = 1e-30f;
        while ((double)G.base[a] + 65535.0 * (double)s < hi[a]) s = nextafterf(s, INFINITY);
        G.step[a] = s;
    }
    G.tk = tk;
    return G;
}
// Host: group k's fixed-pad box (fx) on grid G, outward past `pad` (base + q step exact in double:
// q < 2^16): three words lo | hi << 16; false when it leaves the grid
inline bool lc_grid_box(const LcFloat4 fx[LC_REC], int k, const LcGrid &G, double pad, uint32_t bw[3]) {
    for (int i = 0; i < 3; i++) {
        const double lo = (double)(&fx[3 * k].x)[i] - pad, hi = (double)(&fx[3 * k + 1].x)[i] + pad;
        const double b = G.base[i], st = G.step[i];
        double ql = floor((lo - b) / st), qh = ceil((hi - b) / st);
        if (!(ql >= 0.0) || !(qh <= 65535.0)) return false;
        while (ql > 0.0 && b + ql * st > lo) ql -= 1.0;
        while (qh < 65535.0 && b + qh * st < hi) qh += 1.0;
        if (!(b + ql * st <= lo && b + qh * st >= hi)) return false;
        bw[i] = (uint32_t)ql | (uint32_t)qh << 16;
    }
    return true;
}
// Host: the fixed-pad record of a node (fx, leaf_cull_fixed of `in`) compressed to twelve words on
// grid G (its boxes G.pad past the fixed ones); count: the leaf's references (above LC_MAXREFS_P: every
// one tested always).  A group whose box leaves the grid, or that the fixed record never skips, gets
// kappa = +inf (never skipped).  The planes are the exact reals base + q step (the kernels' fma).
inline void leaf_cull_compress(const LcFloat4 in[LC_REC], const LcFloat4 fx[LC_REC], uint32_t count, const LcGrid &G,
                               uint32_t w[12]) {
    const double pad = G.pad;
    for (int i = 0; i < 12; i++) w[i] = 0u;
    uint32_t m[2];
    __builtin_memcpy(&m[0], &fx[6].x, 4);
    __builtin_memcpy(&m[1], &fx[6].y, 4);
    if (count > (uint32_t)LC_MAXREFS_P) m[0] = m[1] = 0u;
    const double u = 0x1p-24, c0 = 1.0 / LC_C0_INV;
    uint32_t hd[2] = {0u, 0u};
    for (int k = 0; k < 2; k++) {
        uint32_t *box = w + 6 * k;
        box[4] = 0x7c00u << 16; // kappa +inf: never skipped
        if (!m[k]) continue;
        // the axis as three halves, and the cone around the decoded vector: the fixed record's
        // half-angle plus the axis's move
        const double a[3] = {in[3 * k + 2].x, in[3 * k + 2].y, in[3 * k + 2].z};
        const double an = sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
        if (!(an > 0)) continue;
        uint32_t hv[3];
        double v[3];
        for (int i = 0; i < 3; i++) {
            hv[i] = lc_half_near(a[i] / an);
            v[i] = lc_half(hv[i]);
        }
        const double vn = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]) * (1 + 1e-15);
        if (!(vn > 0.5)) continue;
        const double cd = fmin(1.0, fabs(a[0] * v[0] + a[1] * v[1] + a[2] * v[2]) / (an * vn));
        const double th = acos(fmin(1.0, fmax(0.0, (double)in[3 * k + 2].w))) + acos(cd) + 1e-9;
        const double room = acos(c0) - th, g = in[3 * k].w;
        if (!(room > 1e-6 && c0 > 20.2 * u * g && g < 1e20) || !(fx[3 * k + 2].w <= G.tk)) continue;
        uint32_t bw[3];
        if (!lc_grid_box(fx, k, G, pad, bw)) continue;
        // dn >= (K + 3.01u)(1 + 8u)|v|  =>  |d^.v^| >= K (|d| <= 1 + 8u, the float dot's rounding)
        const uint32_t hk = lc_half_up((cos(room) + 1e-12 + 3.01 * u) * (1 + 8 * u) * vn * (1 + 1e-9));
        for (int i = 0; i < 3; i++) box[i] = bw[i];
        box[3] = hv[0] | hv[1] << 16;
        box[4] = hv[2] | hk << 16;
        hd[k] = lc_half_up((double)fx[3 * k + 1].w);
    }
    w[5] = hd[0] | hd[1] << 16;
    w[11] = (m[0] & 0xffffu) | (m[1] & 0xffffu) << 16;
}

// Host: G.dt0 for the short records -- the smallest dt of a group with references (fx: LC_REC float4
// per node, n nodes); 1 when there is none
inline void lc_grid_dt(LcGrid &G, const LcFloat4 *fx, size_t n) {
    float m = INFINITY;
    for (size_t i = 0; i < n; i++) {
        const LcFloat4 *r = fx + (size_t)LC_REC * i;
        uint32_t mk[2];
        __builtin_memcpy(&mk[0], &r[6].x, 4);
        __builtin_memcpy(&mk[1], &r[6].y, 4);
        for (int k = 0; k < 2; k++)
            if (mk[k] && r[3 * k + 1].w > 0.f) m = fminf(m, r[3 * k + 1].w);
    }
    G.dt0 = m < 1e30f ? m : 1.f;
}
// Host: the fixed-pad record of a node compressed to the eight words of LC_RECS on grid G (G.dt0 set
// by lc_grid_dt); count above LC_MAXREFS_P: every reference tested (both groups never skipped).
inline void leaf_cull_compress_s(const LcFloat4 in[LC_REC], const LcFloat4 fx[LC_REC], uint32_t count, const LcGrid &G,
                                 uint32_t w[8]) {
    for (int i = 0; i < 8; i++) w[i] = 0u;
    uint32_t m[3];
    __builtin_memcpy(&m[0], &fx[6].x, 4);
    __builtin_memcpy(&m[1], &fx[6].y, 4);
    __builtin_memcpy(&m[2], &fx[6].z, 4);
    // a group never skipped: kappa code 63 with the axis (0, 0, 1), so |d.v| <= |d| < 63 / 62
    const uint32_t pole = 63u | 63u << 7;
    uint32_t kc[2] = {63u, 63u}, ec[2] = {0u, 0u}, ac[2] = {pole, pole};
    if (count > (uint32_t)LC_MAXREFS_P || count == 0) {
        w[6] = ac[0] | ac[1] << 14;
        w[7] = kc[0] << 16 | kc[1] << 22;
        return;
    }
    const uint32_t all = (1u << count) - 1u;
    // slot 0: a group of the record; slot 1: the rest.  With references tested always, slot 1 holds
    // them and is never skipped, so slot 0 gets the group with more references
    int src[2] = {0, 1};
    const bool always = (m[2] & all) != 0u;
    if (always && __builtin_popcount(m[1]) > __builtin_popcount(m[0])) src[0] = 1, src[1] = 0;
    const uint32_t mask0 = m[src[0]] & all;
    const double u = 0x1p-24, c0 = 1.0 / LC_C0_INV;
    for (int s = 0; s < 2; s++) {
        const int k = src[s];
        if (s == 1 && always) break;
        if (!m[k]) continue;
        if (!lc_grid_box(fx, k, G, G.pad, w + 3 * s)) continue;
        // the axis line on the upper hemisphere, octahedral, and the cone around the decoded vector
        double a[3] = {in[3 * k + 2].x, in[3 * k + 2].y, in[3 * k + 2].z};
        const double an = sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
        if (!(an > 0)) continue;
        if (a[2] < 0) a[0] = -a[0], a[1] = -a[1], a[2] = -a[2];
        const double l1 = fabs(a[0]) + fabs(a[1]) + fabs(a[2]);
        const double pq[2] = {fmin(126.0, fmax(0.0, nearbyint((a[0] / l1 + 1.0) * 63.0))),
                              fmin(126.0, fmax(0.0, nearbyint((a[1] / l1 + 1.0) * 63.0)))};
        const uint32_t p = (uint32_t)pq[0], q = (uint32_t)pq[1];
        const float vx = lc_axis_s(p), vy = lc_axis_s(q), vz = (1.f - fabsf(vx)) - fabsf(vy);
        const double v[3] = {vx, vy, vz};
        const double vn = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]) * (1 + 1e-15);
        if (!(vn > 0.5)) continue;
        const double cd = fmin(1.0, fabs(a[0] * v[0] + a[1] * v[1] + a[2] * v[2]) / (an * vn));
        const double th = acos(fmin(1.0, fmax(0.0, (double)in[3 * k + 2].w))) + acos(cd) + 1e-9;
        const double room = acos(c0) - th, g = in[3 * k].w;
        if (!(room > 1e-6 && c0 > 20.2 * u * g && g < 1e20) || !(fx[3 * k + 2].w <= G.tk)) continue;
        // dn >= (K + 3.01u)(1 + 8u)|v|  =>  |d^.v^| >= K (|d| <= 1 + 8u, the float dot's rounding)
        const double K = (cos(room) + 1e-12 + 3.01 * u) * (1 + 8 * u) * vn * (1 + 1e-9);
        uint32_t c = 0;
        while (c < 63u && !((double)lc_kappa_s(c) >= K)) c++;
        uint32_t e = 0;
        while (e < 16u && !((double)ldexpf(G.dt0, (int)e) >= (double)fx[3 * k + 1].w)) e++;
        if (c >= 63u || e >= 16u) continue;
        kc[s] = c;
        ec[s] = e;
        ac[s] = p | q << 7;
    }
    w[6] = ac[0] | ac[1] << 14 | ec[0] << 28;
    w[7] = (mask0 & 0xffffu) | kc[0] << 16 | kc[1] << 22 | ec[1] << 28;
}

} // namespace cr
