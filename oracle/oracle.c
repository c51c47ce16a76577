/*
 * oracle.c -- CPU restatement of Chiaroscuro's per-pixel render loop.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h header for the rules and the parity
 * status: kd build / traversal / BRDF / integrator are parity unpinned by the
 * reference itself; texture lookup and glm arithmetic are pinned by
 * tests/golden/ref_*.json from oracle/ref).
 *
 * Every function cites the reference line it restates.  Arithmetic is written
 * operation-for-operation in the order glm 0.9.8.5 / the reference evaluates it
 * and must be compiled with -ffp-contract=off and without -ffast-math (the
 * reference's Makefile:4-5 builds for plain x86-64, i.e. SSE2 without FMA).
 */
#include "oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------ glm -- */
typedef struct { float x, y, z; } v3;
typedef struct { float x, y; } v2;

static inline v3 V3(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v3 add(v3 a, v3 b) { return V3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 sub(v3 a, v3 b) { return V3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 mul(v3 a, v3 b) { return V3(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 muls(v3 a, float s) { return V3(a.x * s, a.y * s, a.z * s); }   /* v * s and s * v */
static inline v3 divs(v3 a, float s) { return V3(a.x / s, a.y / s, a.z / s); }   /* type_vec3.inl:672 */
static inline v3 neg(v3 a) { return V3(-a.x, -a.y, -a.z); }
static inline float comp(v3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }
/* func_geometric.inl:53-59: tmp = x*y; tmp.x + tmp.y + tmp.z */
static inline float dot(v3 a, v3 b) { v3 t = mul(a, b); return t.x + t.y + t.z; }
/* func_geometric.inl:77-83 */
static inline v3 cross(v3 x, v3 y) {
    return V3(x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y);
}
/* func_geometric.inl:94 + func_exponential.inl:130-133: v * (1 / sqrt(dot(v,v))) */
static inline v3 normalize(v3 v) { return muls(v, 1.0f / sqrtf(dot(v, v))); }
/* func_geometric.inl:14-28: length = sqrt(dot), distance(p0,p1) = length(p1 - p0) */
static inline float length3(v3 v) { return sqrtf(dot(v, v)); }
static inline float distance3(v3 p0, v3 p1) { return length3(sub(p1, p0)); }
/* libstdc++ std::min / std::max: (b < a) ? b : a  /  (a < b) ? b : a */
static inline float std_min(float a, float b) { return (b < a) ? b : a; }
static inline float std_max(float a, float b) { return (a < b) ? b : a; }
/* glm::max(x, y) = x > y ? x : y (func_common.inl:23-28) */
static inline float glm_max(float x, float y) { return x > y ? x : y; }

/* ------------------------------------------------------------------ RNG -- */
/* The reference's PRNG source is missing.  We define the URBG as a
 * counter-based 32-bit stream keyed by (seed, layer, global pixel, sample) and
 * feed it through exactly the libstdc++-11 distributions the reference uses. */
static inline uint32_t mix32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16; return x;
}
typedef struct { uint32_t key, ctr; } rng_t;
static inline rng_t rng_make(uint32_t seed, uint32_t layer, uint32_t pixel, uint32_t sample) {
    rng_t r; r.key = mix32(mix32(mix32(mix32(seed) ^ layer) ^ pixel) ^ sample); r.ctr = 0; return r;
}
static inline uint32_t rng_u32(rng_t *r) { uint32_t u = mix32(r->key + r->ctr * 0x9E3779B9U); r->ctr++; return u; }
/* std::uniform_real_distribution<float>(a,b) over a 32-bit URBG:
 * generate_canonical<float,24> (random.tcc:3348-3377) then * (b - a) + a. */
static inline float rng_uniform(rng_t *r, float a, float b) {
    float c = (float)rng_u32(r) / 4294967296.0f;
    if (c >= 1.0f) c = 0x1.fffffep-1f; /* nextafter(1, 0) */
    return c * (b - a) + a;
}
/* std::uniform_int_distribution<int>(0, n-1): libstdc++-11 Lemire path
 * (uniform_int_dist.h:245-269, 316) -- Scene::randomLight, src/scene.cpp:79-82 */
static inline uint32_t rng_index(rng_t *r, uint32_t n) {
    uint64_t prod = (uint64_t)rng_u32(r) * (uint64_t)n;
    uint32_t low = (uint32_t)prod;
    if (low < n) {
        uint32_t thr = (uint32_t)(-n) % n;
        while (low < thr) { prod = (uint64_t)rng_u32(r) * (uint64_t)n; low = (uint32_t)prod; }
    }
    return (uint32_t)(prod >> 32);
}

/* ------------------------------------------------------------- sincos -- */
/* glibc's sinf / cosf, which src/brdf.cpp:52-53 calls: glibc 2.35 x86-64 (FMA
 * ifunc) sysdeps/ieee754/flt-32/s_sinf.c, s_cosf.c, sincosf.h -- double
 * polynomials after a 2^24-scaled 2/pi reduction, each a*b+c of the source one
 * fma as the -mfma build contracts it; coefficients = __sincosf_table[0] as libm
 * holds it (table [1] = cosine coefficients negated, applied as a sign on the
 * cosine polynomial, which is exact).  The kernels run the same op sequence
 * (csrc/device_math.hpp cr_sincosf).  or_sincos_check sweeps it against the
 * host libm: equal on every float with |x| < 120 (2.25e9 values).
 * or_set_trig_mode(1) calls libm sinf / cosf instead -- what the reference's std::sin / std::cos do
 * (brdf.cpp:53); the restatement's fma() is a software call without -mfma, so the timed CPU baseline
 * (OR_LEAN) starts in mode 1: the same bits (or_sincos_check), 2.70 -> 3.20 Mray/s on one thread (C1). */
#ifdef OR_LEAN
static int g_trig_mode = 1;
#else
static int g_trig_mode = 0;
#endif
void or_set_trig_mode(int mode) { g_trig_mode = mode; }
static uint32_t abstop12(float x) { uint32_t u; memcpy(&u, &x, 4); return (u >> 20) & 0x7ffu; }
static const double GS_HPI_INV = 0x1.45f306dc9c883p+23, GS_HPI = 0x1.921fb54442d18p+0;
static const double GS_C0 = 0x1p0, GS_C1 = -0x1.ffffffd0c621cp-2, GS_C2 = 0x1.55553e1068f19p-5,
                    GS_C3 = -0x1.6c087e89a359dp-10, GS_C4 = 0x1.99343027bf8c3p-16;
static const double GS_S1 = -0x1.555545995a603p-3, GS_S2 = 0x1.1107605230bc4p-7, GS_S3 = -0x1.994eb3774cf24p-13;
static double gs_sin_poly(double x, double x2) {
    double x3 = x * x2, s1 = fma(x2, GS_S3, GS_S2), x7 = x3 * x2, s = fma(x3, GS_S1, x);
    return fma(x7, s1, s);
}
static double gs_cos_poly(double x2) {
    double x4 = x2 * x2, c2 = fma(x2, GS_C4, GS_C3), c1 = fma(x2, GS_C1, GS_C0), x6 = x4 * x2;
    double c = fma(x4, GS_C2, c1);
    return fma(x6, c2, c);
}
static void glibc_sincosf(float y, float *sn, float *cs) {
    double x = (double)y;
    if (abstop12(y) < abstop12(0x1.921FB6p-1f)) {
        if (abstop12(y) < abstop12(0x1p-12f)) { *sn = y; *cs = 1.0f; return; }
        double x2 = x * x;
        *sn = (float)gs_sin_poly(x, x2);
        *cs = (float)gs_cos_poly(x2);
        return;
    }
    double r = x * GS_HPI_INV;
    int n = ((int32_t)r + 0x800000) >> 24;
    x = fma(-(double)n, GS_HPI, x);
    double xs = ((n & 3) == 1 || (n & 3) == 2) ? -x : x, x2 = x * x;
    double ps = gs_sin_poly(xs, x2), pc = (n & 2) ? -gs_cos_poly(x2) : gs_cos_poly(x2);
    *sn = (float)((n & 1) ? pc : ps);
    *cs = (float)((n & 1) ? ps : pc);
}
void or_sincos(float x, float *s, float *c) {
    if (g_trig_mode == 1) { *s = sinf(x); *c = cosf(x); }
    else glibc_sincosf(x, s, c);
}
/* mismatches of glibc_sincosf vs libm sinf / cosf over the float bit patterns
 * lo, lo + stride, ... <= hi (both signs when both_signs) */
uint64_t or_sincos_check(uint32_t lo, uint32_t hi, uint32_t stride, int both_signs, int threads) {
    uint64_t bad = 0;
    const int nt = threads > 0 ? threads : omp_get_max_threads();
    #pragma omp parallel for num_threads(nt) reduction(+ : bad) schedule(static)
    for (int64_t i = lo; i <= (int64_t)hi; i += stride) {
        for (int sg = 0; sg <= both_signs; sg++) {
            uint32_t u = (uint32_t)i | (sg ? 0x80000000u : 0u);
            float x, a, b, c, d;
            memcpy(&x, &u, 4);
            glibc_sincosf(x, &a, &b);
            c = sinf(x);
            d = cosf(x);
            bad += (memcmp(&a, &c, 4) != 0) + (memcmp(&b, &d, 4) != 0);
        }
    }
    return bad;
}

/* -------------------------------------------------------------- scene -- */
typedef struct { int w, h, nc; size_t off; } tex_t;
typedef struct {
    uint32_t is_leaf, axis, child;
    float split;
    uint32_t first, count; /* into refs */
} node_t;

struct or_scene {
    uint32_t ntri;
    v3 *A, *B, *C;          /* Triangle{posFst,posSnd,posTrd} kdtree.hpp:15-18 */
    v3 *nrm, *kd, *ke;      /* Material kdtree.hpp:20-33 */
    v2 *uvA, *uvB, *uvC;
    int32_t *tex;
    uint8_t *is_light;
    uint32_t nlights;
    uint32_t *light_id;
    float *light_surf;
    uint32_t leaf_size;
    v3 minc, maxc;          /* padded root box */
    node_t *nodes; uint32_t nnodes, cap_nodes;
    uint32_t *refs; uint32_t nrefs, cap_refs;
    uint32_t max_depth;
    tex_t *texs; uint32_t ntex;
    uint8_t *texels; size_t ntexels;
    float ratios[128]; int nratios;
};

/* kdtree.cpp:10-20 triMax/triMin */
static inline float tri_max(const or_scene *s, uint32_t t, int ax) {
    float m = comp(s->A[t], ax);
    m = comp(s->B[t], ax) > m ? comp(s->B[t], ax) : m;
    return comp(s->C[t], ax) > m ? comp(s->C[t], ax) : m;
}
static inline float tri_min(const or_scene *s, uint32_t t, int ax) {
    float m = comp(s->A[t], ax);
    m = comp(s->B[t], ax) < m ? comp(s->B[t], ax) : m;
    return comp(s->C[t], ax) < m ? comp(s->C[t], ax) : m;
}
/* kdtree.cpp:22-28 */
static inline int in_left(const or_scene *s, uint32_t t, float mx, int ax) {
    return comp(s->A[t], ax) <= mx || comp(s->B[t], ax) <= mx || comp(s->C[t], ax) <= mx;
}
static inline int in_right(const or_scene *s, uint32_t t, float mn, int ax) {
    return comp(s->A[t], ax) >= mn || comp(s->B[t], ax) >= mn || comp(s->C[t], ax) >= mn;
}

static uint32_t alloc_nodes(or_scene *s, uint32_t n) {
    if (s->nnodes + n > s->cap_nodes) {
        s->cap_nodes = (s->nnodes + n) * 2;
        s->nodes = (node_t *)realloc(s->nodes, sizeof(node_t) * s->cap_nodes);
    }
    uint32_t first = s->nnodes;
    memset(s->nodes + first, 0, sizeof(node_t) * n);
    s->nnodes += n;
    return first;
}
static uint32_t append_refs(or_scene *s, const uint32_t *ids, uint32_t n) {
    if (s->nrefs + n > s->cap_refs) {
        s->cap_refs = (s->nrefs + n) * 2 + 16;
        s->refs = (uint32_t *)realloc(s->refs, sizeof(uint32_t) * s->cap_refs);
    }
    uint32_t first = s->nrefs;
    memcpy(s->refs + first, ids, sizeof(uint32_t) * n);
    s->nrefs += n;
    return first;
}

/* kdtree.cpp:110-141 findSplit.  The 300 candidates are independent; each keeps
 * its own sequential float cost over `tris` in order, so evaluating them in a
 * vectorised / threaded way changes nothing.  The best is then chosen in the
 * reference's (axis, ratio) order with strict `<`. */
static void find_split(const or_scene *s, const uint32_t *tris, uint32_t n, const float mx[3], const float mn[3],
                       uint32_t *best_axis, float *best_split, int threads) {
    const int NR = s->nratios;
    float split[3 * 128], cost[3 * 128];
    size_t lc[3 * 128], rc[3 * 128];
    for (int ax = 0; ax < 3; ax++)
        for (int i = 0; i < NR; i++) split[ax * NR + i] = mn[ax] + s->ratios[i] * (mx[ax] - mn[ax]);
    (void)threads;
#pragma omp parallel for schedule(static) num_threads(threads > 0 ? threads : 1) if (n > 4096 && threads > 1)
    for (int ax = 0; ax < 3; ax++) {
        float c[128]; size_t L[128], R[128];
        const float *sp = split + ax * NR;
        for (int i = 0; i < NR; i++) { c[i] = 0.f; L[i] = 0; R[i] = 0; }
        for (uint32_t j = 0; j < n; j++) {
            uint32_t t = tris[j];
            float a = comp(s->A[t], ax), b = comp(s->B[t], ax), cc = comp(s->C[t], ax);
            for (int i = 0; i < NR; i++) {
                const float sv = sp[i], ratio = s->ratios[i];
                if (a <= sv || b <= sv || cc <= sv) { c[i] += ratio; L[i]++; }
                if (a >= sv || b >= sv || cc >= sv) { c[i] += (1.f - ratio); R[i]++; }
            }
        }
        for (int i = 0; i < NR; i++) { cost[ax * NR + i] = c[i]; lc[ax * NR + i] = L[i]; rc[ax * NR + i] = R[i]; }
    }
    uint32_t bax = 3; float bsp = 0.f, bcost = (float)n;
    for (int ax = 0; ax < 3; ax++)
        for (int i = 0; i < NR; i++) {
            int k = ax * NR + i;
            if (lc[k] < n && rc[k] < n && cost[k] < bcost) { bax = (uint32_t)ax; bsp = split[k]; bcost = cost[k]; }
        }
    *best_axis = bax;
    *best_split = bsp;
}

/* kdtree.cpp:143-194 build.  Child pairs are allocated at nodes.size() before
 * recursing left then right; results are stored through an index (the
 * reference's `nodes[node.child] = build(...)` aliasing hazard). */
static void build(or_scene *s, uint32_t idx, uint32_t *tris, uint32_t n, const float mx[3], const float mn[3],
                  uint32_t depth, int threads) {
    if (depth > s->max_depth) s->max_depth = depth;
    uint32_t ax = 3; float sp = 0.f;
    if (!(n <= s->leaf_size)) find_split(s, tris, n, mx, mn, &ax, &sp, threads);
    if (n <= s->leaf_size || ax == 3) {
        uint32_t first = append_refs(s, tris, n);
        node_t *nd = &s->nodes[idx];
        nd->is_leaf = 1; nd->axis = 3; nd->split = 0.f; nd->child = 0; nd->first = first; nd->count = n;
        return;
    }
    uint32_t child = alloc_nodes(s, 2);
    s->nodes[idx].is_leaf = 0; s->nodes[idx].axis = ax; s->nodes[idx].split = sp; s->nodes[idx].child = child;
    for (int side = 0; side < 2; side++) {
        float cmn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, cmx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
        uint32_t *ct = (uint32_t *)malloc(sizeof(uint32_t) * (n ? n : 1));
        uint32_t cn = 0;
        for (uint32_t j = 0; j < n; j++) {
            uint32_t t = tris[j];
            int in = side == 0 ? in_left(s, t, sp, (int)ax) : in_right(s, t, sp, (int)ax);
            if (!in) continue;
            ct[cn++] = t;
            int a = (int)ax;
            for (int q = 0; q < 3; q++) {
                float tm = tri_min(s, t, a), tM = tri_max(s, t, a);
                cmn[a] = std_min(cmn[a], tm);
                cmx[a] = std_max(cmx[a], tM);
                a = (a + 1) % 3;
            }
        }
        build(s, child + (uint32_t)side, ct, cn, cmx, cmn, depth + 1, threads);
        free(ct);
    }
}

or_scene *or_scene_create(uint32_t ntri, const float *pos, const float *vnrm, const float *uv, const float *kd,
                          const float *ke, const int32_t *tex, uint32_t leaf_size, int build_threads) {
    or_scene *s = (or_scene *)calloc(1, sizeof(or_scene));
    s->ntri = ntri;
    s->leaf_size = leaf_size;
    s->A = (v3 *)malloc(sizeof(v3) * (ntri + 1)); s->B = (v3 *)malloc(sizeof(v3) * (ntri + 1));
    s->C = (v3 *)malloc(sizeof(v3) * (ntri + 1));
    s->nrm = (v3 *)malloc(sizeof(v3) * (ntri + 1)); s->kd = (v3 *)malloc(sizeof(v3) * (ntri + 1));
    s->ke = (v3 *)malloc(sizeof(v3) * (ntri + 1));
    s->uvA = (v2 *)malloc(sizeof(v2) * (ntri + 1)); s->uvB = (v2 *)malloc(sizeof(v2) * (ntri + 1));
    s->uvC = (v2 *)malloc(sizeof(v2) * (ntri + 1));
    s->tex = (int32_t *)malloc(sizeof(int32_t) * (ntri + 1));
    s->is_light = (uint8_t *)malloc(ntri + 1);
    s->light_id = (uint32_t *)malloc(sizeof(uint32_t) * (ntri + 1));
    s->light_surf = (float *)malloc(sizeof(float) * (ntri + 1));
    /* findSplit ratio sequence: float 0.01f, += 0.01f, while < 1.0f (kdtree.cpp:116) */
    s->nratios = 0;
    for (float r = 0.01f; r < 1.0f; r += 0.01f) s->ratios[s->nratios++] = r;

    /* kdtree.cpp:35 -- min starts at FLT_MAX, max at FLT_MIN (tiny positive) */
    v3 minc = V3(FLT_MAX, FLT_MAX, FLT_MAX), maxc = V3(FLT_MIN, FLT_MIN, FLT_MIN);
    for (uint32_t t = 0; t < ntri; t++) {
        const float *p = pos + 9 * (size_t)t, *n = vnrm + 9 * (size_t)t;
        s->A[t] = V3(p[0], p[1], p[2]); s->B[t] = V3(p[3], p[4], p[5]); s->C[t] = V3(p[6], p[7], p[8]);
        /* kdtree.cpp:58-60: (n0 + n1 + n2) / 3.f, not normalised */
        s->nrm[t] = divs(add(add(V3(n[0], n[1], n[2]), V3(n[3], n[4], n[5])), V3(n[6], n[7], n[8])), 3.f);
        s->kd[t] = V3(kd[3 * t], kd[3 * t + 1], kd[3 * t + 2]);
        s->ke[t] = V3(ke[3 * t], ke[3 * t + 1], ke[3 * t + 2]);
        const float *u = uv + 6 * (size_t)t;
        s->uvA[t].x = u[0]; s->uvA[t].y = u[1]; s->uvB[t].x = u[2]; s->uvB[t].y = u[3];
        s->uvC[t].x = u[4]; s->uvC[t].y = u[5];
        s->tex[t] = tex ? tex[t] : -1;
        /* kdtree.cpp:46-47 */
        s->is_light[t] = s->ke[t].x > 0.f || s->ke[t].y > 0.f || s->ke[t].z > 0.f;
        if (s->is_light[t]) {
            /* kdtree.cpp:72-77 */
            float surf = 0.5f * length3(cross(sub(s->B[t], s->A[t]), sub(s->C[t], s->A[t])));
            s->light_id[s->nlights] = t;
            s->light_surf[s->nlights] = surf;
            s->nlights++;
        }
        /* kdtree.cpp:79-84: std::min(P, minCoords) / std::max(P, maxCoords) */
        v3 P[3] = {s->A[t], s->B[t], s->C[t]};
        for (int k = 0; k < 3; k++) {
            minc.x = std_min(P[k].x, minc.x); minc.y = std_min(P[k].y, minc.y); minc.z = std_min(P[k].z, minc.z);
            maxc.x = std_max(P[k].x, maxc.x); maxc.y = std_max(P[k].y, maxc.y); maxc.z = std_max(P[k].z, maxc.z);
        }
    }
    /* kdtree.cpp:89-90: build on the unpadded box */
    uint32_t *ids = (uint32_t *)malloc(sizeof(uint32_t) * (ntri + 1));
    for (uint32_t t = 0; t < ntri; t++) ids[t] = t;
    alloc_nodes(s, 1);
    float mx[3] = {maxc.x, maxc.y, maxc.z}, mn[3] = {minc.x, minc.y, minc.z};
    build(s, 0, ids, ntri, mx, mn, 0, build_threads);
    free(ids);
    /* kdtree.cpp:106-107: pad after the build */
    s->minc = V3(minc.x - 0.0001f, minc.y - 0.0001f, minc.z - 0.0001f);
    s->maxc = V3(maxc.x + 0.0001f, maxc.y + 0.0001f, maxc.z + 0.0001f);
    return s;
}

int or_scene_add_texture(or_scene *s, int w, int h, int nc, const uint8_t *data) {
    size_t bytes = (size_t)w * h * nc;
    size_t pad = (size_t)(w + 1) * nc + 4; /* defined zeros for the reference's 1-texel over-read */
    s->texs = (tex_t *)realloc(s->texs, sizeof(tex_t) * (s->ntex + 1));
    s->texels = (uint8_t *)realloc(s->texels, s->ntexels + bytes + pad);
    memcpy(s->texels + s->ntexels, data, bytes);
    memset(s->texels + s->ntexels + bytes, 0, pad);
    s->texs[s->ntex].w = w; s->texs[s->ntex].h = h; s->texs[s->ntex].nc = nc; s->texs[s->ntex].off = s->ntexels;
    s->ntexels += bytes + pad;
    return (int)s->ntex++;
}

void or_scene_destroy(or_scene *s) {
    if (!s) return;
    free(s->A); free(s->B); free(s->C); free(s->nrm); free(s->kd); free(s->ke);
    free(s->uvA); free(s->uvB); free(s->uvC); free(s->tex); free(s->is_light);
    free(s->light_id); free(s->light_surf); free(s->nodes); free(s->refs); free(s->texs); free(s->texels);
    free(s);
}

uint32_t or_kd_num_nodes(const or_scene *s) { return s->nnodes; }
uint32_t or_kd_num_refs(const or_scene *s) { return s->nrefs; }
uint32_t or_kd_max_depth(const or_scene *s) { return s->max_depth; }
void or_kd_export(const or_scene *s, uint32_t *is_leaf, uint32_t *axis, float *split, uint32_t *child,
                  uint32_t *leaf_first, uint32_t *leaf_count, uint32_t *refs, float *box) {
    for (uint32_t i = 0; i < s->nnodes; i++) {
        is_leaf[i] = s->nodes[i].is_leaf; axis[i] = s->nodes[i].axis; split[i] = s->nodes[i].split;
        child[i] = s->nodes[i].child; leaf_first[i] = s->nodes[i].first; leaf_count[i] = s->nodes[i].count;
    }
    memcpy(refs, s->refs, sizeof(uint32_t) * s->nrefs);
    box[0] = s->minc.x; box[1] = s->minc.y; box[2] = s->minc.z;
    box[3] = s->maxc.x; box[4] = s->maxc.y; box[5] = s->maxc.z;
}
uint32_t or_num_lights(const or_scene *s) { return s->nlights; }
void or_lights(const or_scene *s, uint32_t *ids, float *surface) {
    for (uint32_t i = 0; i < s->nlights; i++) { ids[i] = s->light_id[i]; surface[i] = s->light_surf[i]; }
}

/* ------------------------------------------------------------- camera -- */
void or_camera(const float e[3], const float c[3], const float u_[3], float yview, uint32_t xres, uint32_t yres,
               float out[12]) {
    v3 eye = V3(e[0], e[1], e[2]), center = V3(c[0], c[1], c[2]), up = V3(u_[0], u_[1], u_[2]);
    /* rayTracer.cpp:41-43 */
    float z = 1.f;
    float y = z * 0.5f * yview;
    float x = y * ((float)xres / (float)yres);
    /* gtc/matrix_transform.inl:521-546 lookAtRH, upper 3x3: m[col][row] */
    v3 f = normalize(sub(center, eye));
    v3 s = normalize(cross(f, up));
    v3 u = cross(s, f);
    float m[3][3] = {{s.x, u.x, -f.x}, {s.y, u.y, -f.y}, {s.z, u.z, -f.z}};
    /* func_matrix.inl:272-294 compute_inverse<tmat3x3> */
    float ood = 1.f / (+m[0][0] * (m[1][1] * m[2][2] - m[2][1] * m[1][2])
                       - m[1][0] * (m[0][1] * m[2][2] - m[2][1] * m[0][2])
                       + m[2][0] * (m[0][1] * m[1][2] - m[1][1] * m[0][2]));
    float r[3][3];
    r[0][0] = +(m[1][1] * m[2][2] - m[2][1] * m[1][2]) * ood;
    r[1][0] = -(m[1][0] * m[2][2] - m[2][0] * m[1][2]) * ood;
    r[2][0] = +(m[1][0] * m[2][1] - m[2][0] * m[1][1]) * ood;
    r[0][1] = -(m[0][1] * m[2][2] - m[2][1] * m[0][2]) * ood;
    r[1][1] = +(m[0][0] * m[2][2] - m[2][0] * m[0][2]) * ood;
    r[2][1] = -(m[0][0] * m[2][1] - m[2][0] * m[0][1]) * ood;
    r[0][2] = +(m[0][1] * m[1][2] - m[1][1] * m[0][2]) * ood;
    r[1][2] = -(m[0][0] * m[1][2] - m[1][0] * m[0][2]) * ood;
    r[2][2] = +(m[0][0] * m[1][1] - m[1][0] * m[0][1]) * ood;
    /* rayTracer.cpp:47-49: (scalar * mat3) * vec3, type_mat3x3.inl:419-433 */
    float sy = 1.f / (float)yres, sx = 1.f / (float)xres;
    float a[3][3], b[3][3];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) { a[i][j] = r[i][j] * sy; b[i][j] = r[i][j] * sx; }
    v3 vy = V3(0.f, -2.f * y, 0.f), vx = V3(2.f * x, 0.f, 0.f), vl = V3(-x, y, -z);
    v3 dy = V3(a[0][0] * vy.x + a[1][0] * vy.y + a[2][0] * vy.z, a[0][1] * vy.x + a[1][1] * vy.y + a[2][1] * vy.z,
               a[0][2] * vy.x + a[1][2] * vy.y + a[2][2] * vy.z);
    v3 dx = V3(b[0][0] * vx.x + b[1][0] * vx.y + b[2][0] * vx.z, b[0][1] * vx.x + b[1][1] * vx.y + b[2][1] * vx.z,
               b[0][2] * vx.x + b[1][2] * vx.y + b[2][2] * vx.z);
    v3 lu = V3(r[0][0] * vl.x + r[1][0] * vl.y + r[2][0] * vl.z, r[0][1] * vl.x + r[1][1] * vl.y + r[2][1] * vl.z,
               r[0][2] * vl.x + r[1][2] * vl.y + r[2][2] * vl.z);
    out[0] = eye.x; out[1] = eye.y; out[2] = eye.z;
    out[3] = lu.x; out[4] = lu.y; out[5] = lu.z;
    out[6] = dx.x; out[7] = dx.y; out[8] = dx.z;
    out[9] = dy.x; out[10] = dy.y; out[11] = dy.z;
}

/* ---------------------------------------------------------- traversal -- */
typedef struct { uint64_t c[OR_C_COUNT]; } ctr_t;
/* Work counters inside the hot recursion (inner nodes, leaves, triangle tests, hits, texture hits).
 * OR_LEAN (liboracle_lean.so, the timed CPU baseline only): compiled out, so the baseline runs the
 * reference's arithmetic without the checker's bookkeeping; the query and path counts stay (they
 * are outside the recursion and give the baseline its ray count). */
#ifdef OR_LEAN
#define CT_HOT(ct, i) ((void)(ct))
#else
#define CT_HOT(ct, i) ((ct)->c[(i)]++)
#endif

/* kdtree.cpp:196-208 */
static inline void ray_box(v3 o, v3 d, v3 mx, v3 mn, float *first, float *second) {
    const float diy = 1.f / d.y, dix = 1.f / d.x, diz = 1.f / d.z;
    const float txmin = (mn.x - o.x) * dix, txmax = (mx.x - o.x) * dix;
    const float tymin = (mn.y - o.y) * diy, tymax = (mx.y - o.y) * diy;
    const float tzmin = (mn.z - o.z) * diz, tzmax = (mx.z - o.z) * diz;
    *first = std_max(std_max(std_min(txmin, txmax), std_min(tymin, tymax)), std_min(tzmin, tzmax));
    *second = std_min(std_min(std_max(txmin, txmax), std_max(tymin, tymax)), std_max(tzmin, tzmax));
}

/* kdtree.cpp:219-246 Moller-Trumbore */
static inline int tri_test(const or_scene *s, v3 o, v3 d, uint32_t t, float *bx, float *by, float *dist) {
    const v3 v0 = s->A[t];
    const v3 e1 = sub(s->B[t], v0), e2 = sub(s->C[t], v0);
    const v3 p = cross(d, e2);
    const float a = dot(e1, p);
    if (a < FLT_EPSILON && a > -FLT_EPSILON) return 0;
    const float f = 1.f / a;
    const v3 sv = sub(o, v0);
    *bx = f * dot(sv, p);
    if (*bx < 0.f || *bx > 1.f) return 0;
    const v3 q = cross(sv, e1);
    *by = f * dot(d, q);
    if (*by < 0.f || *by + *bx > 1.f) return 0;
    return (*dist = f * dot(e2, q)) >= 0.f;
}

/* kdtree.cpp:248-281 (recursive, as written) */
static int node_closest(const or_scene *s, v3 o, v3 d, uint32_t *tri, float *bx, float *by, float *dist,
                        uint32_t ni, float tmin, float tmax, ctr_t *ct) {
    const node_t *nd = &s->nodes[ni];
    if (nd->is_leaf) {
        CT_HOT(ct, OR_C_LEAF);
        int ret = 0;
        for (uint32_t j = 0; j < nd->count; j++) {
            uint32_t t = s->refs[nd->first + j];
            float px, py, pd;
            CT_HOT(ct, OR_C_TRITEST);
            if (tri_test(s, o, d, t, &px, &py, &pd) && pd < tmax) {
                *bx = px; *by = py; tmax = pd; *tri = t; ret = 1;
            }
        }
        *dist = tmax;
        return ret;
    }
    CT_HOT(ct, OR_C_INNER);
    const int a = (int)nd->axis;
    const float oa = comp(o, a), da = comp(d, a);
    const float tsplit = (nd->split - oa) / da;
    const uint32_t below = (oa < nd->split) || (oa == nd->split && da <= 0);
    if (tsplit >= tmax || tsplit < 0)
        return node_closest(s, o, d, tri, bx, by, dist, nd->child + (1 - below), tmin, tmax, ct);
    else if (tsplit <= tmin)
        return node_closest(s, o, d, tri, bx, by, dist, nd->child + below, tmin, tmax, ct);
    else
        return node_closest(s, o, d, tri, bx, by, dist, nd->child + (1 - below), tmin, tsplit, ct) ||
               node_closest(s, o, d, tri, bx, by, dist, nd->child + below, tsplit, tmax, ct);
}

/* kdtree.cpp:210-216 */
static int intersect_ray(const or_scene *s, v3 o, v3 d, uint32_t *tri, float *bx, float *by, float *dist,
                         ctr_t *ct) {
    ct->c[OR_C_CLOSEST]++;
    float t0, t1;
    ray_box(o, d, s->maxc, s->minc, &t0, &t1);
    if (t1 < 0 || t1 < t0) return 0;
    return node_closest(s, o, d, tri, bx, by, dist, 0, t0, t1, ct);
}

/* kdtree.cpp:293-320 */
static inline int shadow_tri(const or_scene *s, v3 o, v3 d, uint32_t t, float tmax) {
    const v3 v0 = s->A[t];
    const v3 e1 = sub(s->B[t], v0), e2 = sub(s->C[t], v0);
    const v3 p = cross(d, e2);
    const float a = dot(e1, p);
    if (a < FLT_EPSILON && a > -FLT_EPSILON) return 0;
    const float f = 1.f / a;
    const v3 sv = sub(o, v0);
    const float bx = f * dot(sv, p);
    if (bx < 0.f || bx > 1.f) return 0;
    const v3 q = cross(sv, e1);
    const float by = f * dot(d, q);
    if (by < 0.f || by + bx > 1.f) return 0;
    const float t_ = f * dot(e2, q);
    return t_ >= 0.f && t_ < tmax;
}

/* kdtree.cpp:322-344 */
static int node_shadow(const or_scene *s, v3 o, v3 d, uint32_t light, uint32_t ni, float tmin, float tmax,
                       ctr_t *ct) {
    const node_t *nd = &s->nodes[ni];
    if (nd->is_leaf) {
        CT_HOT(ct, OR_C_LEAF);
        for (uint32_t j = 0; j < nd->count; j++) {
            uint32_t t = s->refs[nd->first + j];
            if (t != light) {
                CT_HOT(ct, OR_C_TRITEST);
                if (shadow_tri(s, o, d, t, tmax)) return 1;
            }
        }
        return 0;
    }
    CT_HOT(ct, OR_C_INNER);
    const int a = (int)nd->axis;
    const float oa = comp(o, a), da = comp(d, a);
    const float tsplit = (nd->split - oa) / da;
    const uint32_t below = (oa < nd->split) || (oa == nd->split && da <= 0);
    if (tsplit >= tmax || tsplit < 0)
        return node_shadow(s, o, d, light, nd->child + (1 - below), tmin, tmax, ct);
    else if (tsplit <= tmin)
        return node_shadow(s, o, d, light, nd->child + below, tmin, tmax, ct);
    else
        return node_shadow(s, o, d, light, nd->child + (1 - below), tmin, tsplit, ct) ||
               node_shadow(s, o, d, light, nd->child + below, tsplit, tmax, ct);
}

/* kdtree.cpp:283-290 */
static int intersect_shadow(const or_scene *s, v3 o, v3 d, float distance, uint32_t light, ctr_t *ct) {
    ct->c[OR_C_SHADOW]++;
    float t0, t1;
    ray_box(o, d, s->maxc, s->minc, &t0, &t1);
    if (t1 < 0 || t1 < t0 || t0 > distance) return 0;
    return node_shadow(s, o, d, light, 0, t0, std_min(t1, distance), ct);
}

void or_intersect(or_scene *s, uint32_t n, const float *orig, const float *dir, uint32_t *hit, uint32_t *tri,
                  float *bary, float *dist) {
    ctr_t ct; memset(&ct, 0, sizeof ct);
    for (uint32_t i = 0; i < n; i++) {
        v3 o = V3(orig[3 * i], orig[3 * i + 1], orig[3 * i + 2]), d = V3(dir[3 * i], dir[3 * i + 1], dir[3 * i + 2]);
        uint32_t t = 0; float bx = 0, by = 0, ds = 0;
        hit[i] = (uint32_t)intersect_ray(s, o, d, &t, &bx, &by, &ds, &ct);
        if (hit[i]) { tri[i] = t; bary[2 * i] = bx; bary[2 * i + 1] = by; dist[i] = ds; }
    }
}
void or_intersect_shadow(or_scene *s, uint32_t n, const float *orig, const float *dir, const float *dist,
                         const uint32_t *light, uint32_t *occluded) {
    ctr_t ct; memset(&ct, 0, sizeof ct);
    for (uint32_t i = 0; i < n; i++) {
        v3 o = V3(orig[3 * i], orig[3 * i + 1], orig[3 * i + 2]), d = V3(dir[3 * i], dir[3 * i + 1], dir[3 * i + 2]);
        occluded[i] = (uint32_t)intersect_shadow(s, o, d, dist[i], light[i], &ct);
    }
}

/* ------------------------------------------------------------ shading -- */
/* src/mesh.cpp:21-35 Texture::getColorAt */
static v3 tex_lookup(const or_scene *s, int ti, v2 c) {
    const tex_t *t = &s->texs[ti];
    while (c.x > 1.f) c.x -= 1.f;
    while (c.x < 0.f) c.x += 1.f;
    while (c.y > 1.f) c.y -= 1.f;
    while (c.y < 0.f) c.y += 1.f;
    const int x = (int)(c.x * (float)t->w);
    const int y = (int)(c.y * (float)t->h);
    const uint8_t *px = s->texels + t->off + (size_t)(y * t->w + x) * (size_t)t->nc;
    return V3((float)px[0] * 0.00392156862f, (float)px[1] * 0.00392156862f, (float)px[2] * 0.00392156862f);
}
void or_tex_lookup(const or_scene *s, int tex, float u, float v, float out[3]) {
    v2 c; c.x = u; c.y = v;
    v3 r = tex_lookup(s, tex, c);
    out[0] = r.x; out[1] = r.y; out[2] = r.z;
}

/* src/brdf.cpp:10-15 */
static inline v3 perpendicular(v3 v) {
    if (fabsf(v.x) < fabsf(v.y)) return V3(0.0f, -v.z, v.y);
    return V3(-v.z, 0.0f, v.x);
}
/* src/brdf.cpp:18-54 with the two draws supplied */
static void concentric(float sx, float sy, float *dx, float *dy) {
    if (sx == 0.0 && sy == 0.0) { *dx = 0.0f; *dy = 0.0f; return; }
    float r, theta;
    if (sx >= -sy) {
        if (sx > sy) { r = sx; if (sy > 0.0) theta = sy / r; else theta = 8.0f + sy / r; }
        else { r = sy; theta = 2.0f - sx / r; }
    } else {
        if (sx <= sy) { r = -sx; theta = 4.0f - sy / r; }
        else { r = -sy; theta = 6.0f + sx / r; }
    }
    theta = (float)((double)theta * (M_PI / 4.0)); /* theta *= M_PI / 4.f : double multiply */
    float sn, cs;
    or_sincos(theta, &sn, &cs);
    *dx = r * cs;
    *dy = r * sn;
}
void or_concentric(float sx, float sy, float *dx, float *dy) { concentric(sx, sy, dx, dy); }

/* src/brdf.cpp:57-62 + 72-79 (Diffuse::sample_wi); returns wi and pdf. */
static void sample_wi(v3 n, float sx, float sy, v3 *wi, float *pdf) {
    v3 tangent = normalize(perpendicular(n));
    v3 bitangent = normalize(cross(tangent, n));
    float hx, hy;
    concentric(sx, sy, &hx, &hy);
    float hz = (float)sqrt((double)std_max(0.f, 1.f - hx * hx - hy * hy));
    *wi = normalize(add(add(muls(tangent, hx), muls(bitangent, hy)), muls(n, hz)));
    *pdf = (float)((double)glm_max(0.0f, dot(n, *wi)) * M_1_PI);
}
void or_sample_wi(const float n[3], float sx, float sy, float wi[3], float *pdf) {
    v3 w; sample_wi(V3(n[0], n[1], n[2]), sx, sy, &w, pdf);
    wi[0] = w.x; wi[1] = w.y; wi[2] = w.z;
}

/* ---------------------------------------------------------- integrator -- */
typedef struct {
    const or_scene *s;
    int K;
    v3 bg;
} itg_t;

/* src/rayTracer.cpp:76-135 sendRay (recursive) + 137-169 intersectRayKDTree */
static v3 send_ray(const itg_t *it, v3 origin, v3 dir, int k, rng_t *rng, ctr_t *ct) {
    const or_scene *s = it->s;
    uint32_t t; float bx, by, dist;
    if (!intersect_ray(s, origin, dir, &t, &bx, &by, &dist, ct)) return it->bg;
    CT_HOT(ct, OR_C_HIT);
    /* intersectRayKDTree */
    const v3 normal = s->nrm[t];
    const float bz = (1.f - bx - by);
    const v3 p = add(add(muls(s->A[t], bz), muls(s->B[t], bx)), muls(s->C[t], by));
    v3 Kd = s->kd[t];
    if (s->tex[t] >= 0) {
        v2 c;
        c.x = (s->uvA[t].x * bz + s->uvB[t].x * bx) + s->uvC[t].x * by;
        c.y = (s->uvA[t].y * bz + s->uvB[t].y * bx) + s->uvC[t].y * by;
        Kd = tex_lookup(s, s->tex[t], c);
        CT_HOT(ct, OR_C_TEXHIT);
    }
    const int emissive = s->is_light[t];
    const v3 fcol = muls(Kd, (float)M_1_PI); /* Diffuse::f = float(M_1_PI) * color, brdf.cpp:70 */

    const v3 wo = normalize(sub(origin, p));
    v3 direct;
    if (k > 1) direct = V3(0.f, 0.f, 0.f);
    else {
        const v3 rad = emissive ? s->ke[t] : V3(0.f, 0.f, 0.f);
        direct = muls(rad, std_max(0.f, dot(wo, normal)));
    }
    if (s->nlights) {
        const uint32_t li = rng_index(rng, s->nlights);
        const uint32_t lid = s->light_id[li];
        const float v0 = rng_uniform(rng, 0.f, 1.f);
        const float v1 = rng_uniform(rng, 0.f, 1.f - v0);
        const v3 lp = add(add(muls(s->A[lid], v0), muls(s->B[lid], v1)), muls(s->C[lid], 1.f - v0 - v1));
        const float distance = distance3(p, lp);
        const v3 wl = normalize(sub(lp, p));
        if (!intersect_shadow(s, add(p, muls(normal, 0.001f)), wl, distance, lid, ct)) {
            const float geometric =
                std_max(0.f, dot(normal, wl) * dot(neg(wl), s->nrm[lid]) / (1.f + distance * distance));
            direct = add(direct, mul(muls(s->ke[lid], geometric * s->light_surf[li] * (float)s->nlights), fcol));
        }
    }
    if (k == it->K) return direct;
    const float sx = rng_uniform(rng, -1.f, 1.f);
    const float sy = rng_uniform(rng, -1.f, 1.f);
    v3 wi; float pdf;
    sample_wi(normal, sx, sy, &wi, &pdf);
    const v3 f = fcol;
    const float Kmax = std_max(std_max(f.x, f.y), f.z);
    if (pdf == 0.f || rng_uniform(rng, 0.f, 1.f) > Kmax) return direct;
    const float cosine = fabsf(dot(normal, wi));
    const v3 w = divs(muls(f, cosine), pdf * Kmax);
    const v3 rec = send_ray(it, add(p, muls(normal, 0.001f)), wi, k + 1, rng, ct);
    return add(direct, mul(w, rec));
}

static inline v3 camera_sample(const float cam[12], uint32_t x, uint32_t y, rng_t *rng, v3 *eye) {
    *eye = V3(cam[0], cam[1], cam[2]);
    const v3 lu = V3(cam[3], cam[4], cam[5]), dx = V3(cam[6], cam[7], cam[8]), dy = V3(cam[9], cam[10], cam[11]);
    /* rayTracer.cpp:61 -- g++ evaluates the y-jitter draw before the x-jitter */
    const float uy = rng_uniform(rng, 0.f, 1.f);
    const float ux = rng_uniform(rng, 0.f, 1.f);
    return add(add(lu, muls(dx, (float)x + ux)), muls(dy, (float)y + uy));
}

void or_path(or_scene *s, const float cam[12], uint32_t xres, uint32_t yres, int k, const float bg[3],
             uint32_t seed, uint32_t layer, uint32_t x, uint32_t y, uint32_t sample, float out[3]) {
    (void)yres;
    itg_t it = {s, k, V3(bg[0], bg[1], bg[2])};
    ctr_t ct; memset(&ct, 0, sizeof ct);
    rng_t rng = rng_make(seed, layer, y * xres + x, sample);
    v3 eye;
    v3 dir = camera_sample(cam, x, y, &rng, &eye);
    v3 r = send_ray(&it, eye, dir, 1, &rng, &ct);
    out[0] = r.x; out[1] = r.y; out[2] = r.z;
}

void or_rng_draws(uint32_t seed, uint32_t layer, uint32_t pixel, uint32_t sample, uint32_t n, uint32_t *out) {
    rng_t r = rng_make(seed, layer, pixel, sample);
    for (uint32_t i = 0; i < n; i++) out[i] = rng_u32(&r);
}

/* src/rayTracer.cpp:52-70 */
void or_render(or_scene *s, const float cam[12], uint32_t xres, uint32_t yres, uint32_t spp, int k,
               const float bg[3], uint32_t seed, uint32_t layer, uint32_t y0, uint32_t y1, uint32_t ystep,
               int threads, float *pix, uint64_t *counters) {
    itg_t it = {s, k, V3(bg[0], bg[1], bg[2])};
    const float inv = 1.f / (float)spp;
    if (y1 > yres) y1 = yres;
    if (ystep == 0) ystep = 1;
    uint64_t tot[OR_C_COUNT];
    memset(tot, 0, sizeof tot);
#ifdef _OPENMP
    int nth = threads > 0 ? threads : omp_get_max_threads();
#else
    int nth = 1;
    (void)threads;
#endif
    int64_t nrows = y0 < y1 ? ((int64_t)(y1 - y0) + ystep - 1) / ystep : 0;
#pragma omp parallel num_threads(nth)
    {
        ctr_t ct; memset(&ct, 0, sizeof ct);
#pragma omp for schedule(static) /* src/rayTracer.cpp:55: the default (static) schedule over rows */
        for (int64_t ri = 0; ri < nrows; ri++) {
            const uint32_t y = y0 + (uint32_t)ri * ystep;
            for (uint32_t x = 0; x < xres; x++) {
                v3 temp = V3(0.f, 0.f, 0.f);
                for (uint32_t smp = 0; smp < spp; smp++) {
                    rng_t rng = rng_make(seed, layer, y * xres + x, smp);
                    v3 eye;
                    v3 dir = camera_sample(cam, x, y, &rng, &eye);
                    ct.c[OR_C_PATHS]++;
                    temp = add(temp, send_ray(&it, eye, dir, 1, &rng, &ct));
                }
                float *P = pix + 3 * ((size_t)y * xres + x);
                v3 old = V3(P[0], P[1], P[2]);
                v3 nw = divs(add(muls(old, (float)(layer - 1)), muls(temp, inv)), (float)layer);
                P[0] = nw.x; P[1] = nw.y; P[2] = nw.z;
            }
        }
#pragma omp critical
        for (int i = 0; i < OR_C_COUNT; i++) tot[i] += ct.c[i];
    }
    if (counters)
        for (int i = 0; i < OR_C_COUNT; i++) counters[i] = tot[i];
}

/* Batch means of a list of pixels (the tile split's per-rank work):
 * mean[i] = (sum over samples in order of sendRay) * (1/spp), counters summed. */
void or_render_pixels(or_scene *s, const float cam[12], uint32_t xres, uint32_t yres, uint32_t spp, int k,
                      const float bg[3], uint32_t seed, uint32_t layer, uint32_t n, const uint32_t *px,
                      const uint32_t *py, int threads, float *mean, uint64_t *counters) {
    itg_t it = {s, k, V3(bg[0], bg[1], bg[2])};
    const float inv = 1.f / (float)spp;
    (void)yres;
    uint64_t tot[OR_C_COUNT];
    memset(tot, 0, sizeof tot);
#ifdef _OPENMP
    int nth = threads > 0 ? threads : omp_get_max_threads();
#else
    int nth = 1;
    (void)threads;
#endif
#pragma omp parallel num_threads(nth)
    {
        ctr_t ct; memset(&ct, 0, sizeof ct);
        /* (a checker, not the timed baseline: dynamic chunks balance pixels of uneven cost) */
#pragma omp for schedule(dynamic, 16)
        for (int64_t i = 0; i < (int64_t)n; i++) {
            v3 temp = V3(0.f, 0.f, 0.f);
            for (uint32_t smp = 0; smp < spp; smp++) {
                rng_t rng = rng_make(seed, layer, py[i] * xres + px[i], smp);
                v3 eye;
                v3 dir = camera_sample(cam, px[i], py[i], &rng, &eye);
                ct.c[OR_C_PATHS]++;
                temp = add(temp, send_ray(&it, eye, dir, 1, &rng, &ct));
            }
            const v3 m = muls(temp, inv);
            mean[3 * i] = m.x; mean[3 * i + 1] = m.y; mean[3 * i + 2] = m.z;
        }
#pragma omp critical
        for (int i = 0; i < OR_C_COUNT; i++) tot[i] += ct.c[i];
    }
    if (counters)
        for (int i = 0; i < OR_C_COUNT; i++) counters[i] = tot[i];
}

/* ------------------------------------------------ glm primitives (KAT) -- */
void or_glm_normalize(const float a[3], float out[3]) {
    v3 r = normalize(V3(a[0], a[1], a[2]));
    out[0] = r.x; out[1] = r.y; out[2] = r.z;
}
void or_glm_cross(const float a[3], const float b[3], float out[3]) {
    v3 r = cross(V3(a[0], a[1], a[2]), V3(b[0], b[1], b[2]));
    out[0] = r.x; out[1] = r.y; out[2] = r.z;
}
float or_glm_dot(const float a[3], const float b[3]) { return dot(V3(a[0], a[1], a[2]), V3(b[0], b[1], b[2])); }
float or_glm_distance(const float a[3], const float b[3]) {
    return distance3(V3(a[0], a[1], a[2]), V3(b[0], b[1], b[2]));
}
/* kdtree.cpp:58-60 and 72-77 */
void or_material_normal(const float n[9], float out[3]) {
    v3 r = divs(add(add(V3(n[0], n[1], n[2]), V3(n[3], n[4], n[5])), V3(n[6], n[7], n[8])), 3.f);
    out[0] = r.x; out[1] = r.y; out[2] = r.z;
}
float or_light_surface(const float p[9]) {
    v3 A = V3(p[0], p[1], p[2]), B = V3(p[3], p[4], p[5]), Cc = V3(p[6], p[7], p[8]);
    return 0.5f * length3(cross(sub(B, A), sub(Cc, A)));
}

/* ---------------------------------------------- tonemap (normalizeImage) -- */
/* rayTracer.cpp:172-194: knee and findKneeF (glibc logf on a float argument:
 * the double x*f + 1 is converted to float at the call, the quotient is double) */
static inline float tm_knee(double x, double f) { return logf((float)(x * f + 1)) / f; }
static float tm_find_knee_f(float x, float y) {
    float f0 = 0, f1 = 1;
    while (tm_knee(x, f1) > y) {
        f0 = f1;
        f1 = f1 * 2;
    }
    for (int i = 0; i < 30; ++i) {
        float f2 = (f0 + f1) / 2;
        if (tm_knee(x, f2) < y) f1 = f2;
        else f0 = f2;
    }
    return (f0 + f1) / 2;
}
/* rayTracer.cpp:196-222: rgb [yres][xres][3] (row 0 = top) -> out with the rows
 * flipped as the reference's data; glibc powf / logf throughout. */
void or_tonemap(const float *rgb, uint32_t xres, uint32_t yres, float exposure, float defog, float kneeLow,
                float kneeHigh, float gamma, uint8_t *out) {
    const float m = powf(2.f, exposure + 2.47393f);
    const float s = 255.f * powf(2.f, -3.5f * gamma);
    const float kl = powf(2.f, kneeLow);
    const float f = tm_find_knee_f(powf(2.f, kneeHigh), powf(2.f, 3.5f) - kl); /* C++ powf(2.f, 3.5) */
    for (uint32_t y = 0; y < yres; y++)
        for (uint32_t x = 0; x < xres; x++)
            for (int ch = 0; ch < 3; ch++) {
                float v = rgb[3 * ((size_t)y * xres + x) + ch];
                v = std_max(0.f, v - defog);
                v *= m;
                if (v > kl) v = kl + tm_knee(v - kl, f);
                const float w = powf(v, gamma) * s;
                const float c = (w > 0.f ? w : 0.f) < 255.f ? (w > 0.f ? w : 0.f) : 255.f; /* glm::clamp */
                out[3 * ((size_t)(yres - y - 1) * xres + x) + ch] = (uint8_t)c;
            }
}
