/* packet_census.c -- CPU census (diagnostic only): shadow queries traced one ray per lane (the reference's
 * kd recursion, kdtree.cpp:322-344, near child first) against a shadow PACKET per 64 consecutive queries of
 * the sorted queue: the wave walks one node at a time, every lane keeps its own interval (the reference's
 * three cases per node), children are visited in the majority's near-first order -- a shadow answer is the
 * OR over the (leaf, interval) pairs the reference visits, which does not depend on the order -- and an
 * occluded lane leaves the packet.  Counts wave steps, active lanes per step, leaves and tests of both.
 * Built by scripts/packet_census.py. */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

enum { C_QUERIES, C_OCC, C_LANE_INNER, C_LANE_LEAVES, C_LANE_TESTS, C_PK_INNER, C_PK_INNER_LANES, C_PK_LEAVES,
       C_PK_LEAF_LANES, C_PK_TESTS, C_PK_TEST_LANES, C_PK_MISMATCH, C_PACKETS, C_PK_LANE_INNER, C_N };

/* kdtree.cpp:293-320 (float, no contraction) */
static int mt(const float o[3], const float d[3], const float *tri, float tmax) {
    float e1[3], e2[3], p[3], s[3], q[3];
    for (int i = 0; i < 3; i++) {
        e1[i] = tri[3 + i] - tri[i];
        e2[i] = tri[6 + i] - tri[i];
    }
    p[0] = d[1] * e2[2] - d[2] * e2[1];
    p[1] = d[2] * e2[0] - d[0] * e2[2];
    p[2] = d[0] * e2[1] - d[1] * e2[0];
    const float a = (e1[0] * p[0] + e1[1] * p[1]) + e1[2] * p[2];
    if (a < FLT_EPSILON && a > -FLT_EPSILON) return 0;
    const float f = 1.f / a;
    for (int i = 0; i < 3; i++) s[i] = o[i] - tri[i];
    const float u = f * ((s[0] * p[0] + s[1] * p[1]) + s[2] * p[2]);
    if (u < 0.f || u > 1.f) return 0;
    q[0] = s[1] * e1[2] - s[2] * e1[1];
    q[1] = s[2] * e1[0] - s[0] * e1[2];
    q[2] = s[0] * e1[1] - s[1] * e1[0];
    const float v = f * ((d[0] * q[0] + d[1] * q[1]) + d[2] * q[2]);
    if (v < 0.f || u + v > 1.f) return 0;
    const float t = f * ((e2[0] * q[0] + e2[1] * q[1]) + e2[2] * q[2]);
    return t >= 0.f && t < tmax;
}

typedef struct {
    const uint32_t *is_leaf, *axis, *child, *first, *count, *refs;
    const float *split, *pos;
} Kd;

/* the reference's recursion (kdtree.cpp:322-344) with work counts */
static int lane_node(const Kd *T, uint32_t n, const float o[3], const float d[3], float tmin, float tmax, uint32_t excl,
                     uint64_t *c) {
    if (T->is_leaf[n]) {
        c[C_LANE_LEAVES]++;
        for (uint32_t j = 0; j < T->count[n]; j++) {
            const uint32_t id = T->refs[T->first[n] + j];
            if (id == excl) continue;
            c[C_LANE_TESTS]++;
            if (mt(o, d, T->pos + 9 * (size_t)id, tmax)) return 1;
        }
        return 0;
    }
    c[C_LANE_INNER]++;
    const uint32_t a = T->axis[n];
    const float sp = T->split[n];
    const float ts = (sp - o[a]) / d[a];
    const uint32_t below = (o[a] < sp) || (o[a] == sp && d[a] <= 0);
    const uint32_t ch = T->child[n];
    if (ts >= tmax || ts < 0) return lane_node(T, ch + (1 - below), o, d, tmin, tmax, excl, c);
    if (ts <= tmin) return lane_node(T, ch + below, o, d, tmin, tmax, excl, c);
    return lane_node(T, ch + (1 - below), o, d, tmin, ts, excl, c) || lane_node(T, ch + below, o, d, ts, tmax, excl, c);
}

typedef struct {
    const float *o, *d;
    const uint32_t *excl;
    float tmin[64], tmax[64];
    int occ[64];
    int n;
} Pk;

/* one packet node visit: `act` the lanes that visit n, with their intervals in lo / hi */
static void pk_node(const Kd *T, Pk *P, uint32_t n, uint64_t act, const float *lo, const float *hi, uint64_t *c) {
    uint64_t live = 0;
    for (int l = 0; l < P->n; l++)
        if (((act >> l) & 1) && !P->occ[l]) live |= 1ull << l;
    if (!live) return;
    if (T->is_leaf[n]) {
        c[C_PK_LEAVES]++;
        c[C_PK_LEAF_LANES] += __builtin_popcountll(live);
        for (uint32_t j = 0; j < T->count[n]; j++) {
            const uint32_t id = T->refs[T->first[n] + j];
            uint64_t tl = 0;
            for (int l = 0; l < P->n; l++)
                if (((live >> l) & 1) && !P->occ[l] && id != P->excl[l]) tl |= 1ull << l;
            if (!tl) continue;
            c[C_PK_TESTS]++;
            c[C_PK_TEST_LANES] += __builtin_popcountll(tl);
            for (int l = 0; l < P->n; l++)
                if ((tl >> l) & 1)
                    if (mt(P->o + 3 * l, P->d + 3 * l, T->pos + 9 * (size_t)id, hi[l])) P->occ[l] = 1;
        }
        return;
    }
    c[C_PK_INNER]++;
    c[C_PK_INNER_LANES] += __builtin_popcountll(live);
    const uint32_t a = T->axis[n];
    const float sp = T->split[n];
    const uint32_t ch = T->child[n];
    float lo0[64], hi0[64], lo1[64], hi1[64];
    uint64_t a0 = 0, a1 = 0;
    int near0 = 0, near1 = 0;
    for (int l = 0; l < P->n; l++) {
        if (!((live >> l) & 1)) continue;
        c[C_PK_LANE_INNER]++;
        const float *o = P->o + 3 * l, *d = P->d + 3 * l;
        const float ts = (sp - o[a]) / d[a];
        const uint32_t below = (o[a] < sp) || (o[a] == sp && d[a] <= 0);
        const uint32_t nearc = 1 - below, farc = below; /* child offsets */
        float nl = lo[l], nh = hi[l], fl = lo[l], fh = hi[l];
        int gn = 0, gf = 0;
        if (ts >= hi[l] || ts < 0) gn = 1;
        else if (ts <= lo[l]) gf = 1;
        else { gn = gf = 1; nh = ts; fl = ts; }
        if (gn) {
            if (nearc == 0) { a0 |= 1ull << l; lo0[l] = nl; hi0[l] = nh; near0++; }
            else { a1 |= 1ull << l; lo1[l] = nl; hi1[l] = nh; near1++; }
        }
        if (gf) {
            if (farc == 0) { a0 |= 1ull << l; lo0[l] = fl; hi0[l] = fh; }
            else { a1 |= 1ull << l; lo1[l] = fl; hi1[l] = fh; }
        }
    }
    if (near0 >= near1) {
        pk_node(T, P, ch, a0, lo0, hi0, c);
        pk_node(T, P, ch + 1, a1, lo1, hi1, c);
    } else {
        pk_node(T, P, ch + 1, a1, lo1, hi1, c);
        pk_node(T, P, ch, a0, lo0, hi0, c);
    }
}

static void ray_box(const float *box, const float o[3], const float d[3], float *t0, float *t1) {
    float inv[3] = {1.f / d[0], 1.f / d[1], 1.f / d[2]};
    float tl[3], th[3];
    for (int i = 0; i < 3; i++) {
        const float a = (box[i] - o[i]) * inv[i], b = (box[3 + i] - o[i]) * inv[i];
        tl[i] = a < b ? a : b;
        th[i] = a < b ? b : a;
    }
    *t0 = fmaxf(fmaxf(tl[0], tl[1]), tl[2]);
    *t1 = fminf(fminf(th[0], th[1]), th[2]);
}

/* queries in queue order; packets of `width` consecutive queries */
void census(const uint32_t *is_leaf, const uint32_t *axis, const float *split, const uint32_t *child,
            const uint32_t *first, const uint32_t *count, const uint32_t *refs, const float *box, const float *pos,
            uint32_t nq, const float *o, const float *d, const float *dist, const uint32_t *excl, int width,
            uint64_t *stats) {
    Kd T = {is_leaf, axis, child, first, count, refs, split, pos};
    memset(stats, 0, sizeof(uint64_t) * C_N);
#pragma omp parallel
    {
        uint64_t c[C_N];
        memset(c, 0, sizeof c);
#pragma omp for schedule(dynamic, 16)
        for (uint32_t b = 0; b < nq; b += (uint32_t)width) {
            Pk P;
            P.n = (int)((nq - b) < (uint32_t)width ? nq - b : (uint32_t)width);
            P.o = o + 3 * (size_t)b;
            P.d = d + 3 * (size_t)b;
            P.excl = excl + b;
            uint64_t act = 0;
            int ref[64];
            for (int l = 0; l < P.n; l++) {
                const size_t q = b + (size_t)l;
                float t0, t1;
                ray_box(box, o + 3 * q, d + 3 * q, &t0, &t1);
                P.occ[l] = 0;
                ref[l] = 0;
                c[C_QUERIES]++;
                if (t1 < 0 || t1 < t0 || t0 > dist[q]) continue;
                P.tmin[l] = t0;
                P.tmax[l] = fminf(t1, dist[q]);
                act |= 1ull << l;
                ref[l] = lane_node(&T, 0, o + 3 * q, d + 3 * q, P.tmin[l], P.tmax[l], excl[q], c);
                c[C_OCC] += ref[l];
            }
            c[C_PACKETS]++;
            pk_node(&T, &P, 0, act, P.tmin, P.tmax, c);
            for (int l = 0; l < P.n; l++) c[C_PK_MISMATCH] += P.occ[l] != ref[l];
        }
#pragma omp critical
        for (int i = 0; i < C_N; i++) stats[i] += c[i];
    }
}

/* the leaf holding each point (below the split: child + 0, kdtree.cpp:262) */
void locate(const uint32_t *is_leaf, const uint32_t *axis, const float *split, const uint32_t *child, uint32_t n,
            const float *p, uint32_t *leaf) {
#pragma omp parallel for
    for (uint32_t i = 0; i < n; i++) {
        uint32_t k = 0;
        while (!is_leaf[k]) k = child[k] + (p[3 * (size_t)i + axis[k]] < split[k] ? 0u : 1u);
        leaf[i] = k;
    }
}
