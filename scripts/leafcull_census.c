/* leafcull_census.c -- CPU census for a per-leaf exact skip of the kd traversal.
 *
 * Traverses rays with the reference's semantics (kdtree.cpp:196-344: root slab
 * test, near/far descent, a leaf tests all its triangles with tmax = the leaf
 * interval's end, a shadow query ends at its first occluder) and asks, for every
 * visited leaf with triangles, whether the ray's test segment [0, tmax_L] misses
 * the leaf's TIGHT triangle box -- unpadded (an upper bound on what a cull could
 * skip) and padded by the Moller-Trumbore rounding bound of the leaf's triangles
 * for this ray (what an exact cull could skip).  Diagnostic only (scripts/).
 *
 *   gcc -O2 -fopenmp -shared -fPIC -o /tmp/leafcull_census.so scripts/leafcull_census.c -lm
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* per-leaf record of the implementable cull: the normal-line cone (axis, cos / sin of its
 * half-angle), g = max E^2 / |n| and E = max |e|_1 over the leaf's triangles */
typedef struct {
    double ax[3], ct, st, g, E;
    int ok;
} Cone;
/* a leaf's triangles split into up to KMAX normal groups, each with its own cone and box
 * (cull per group); 'risky' = degenerate triangles, always tested */
enum { KMAX = 4, KCFG = 4 };
#ifndef SUBMODE
#define SUBMODE 1
#endif
#ifndef SUBK
#define SUBK 4
#endif
typedef struct {
    int ng, risky;
    int size[KMAX];
    double ax[KMAX][3], ct[KMAX], st[KMAX], g[KMAX], E[KMAX], box[KMAX][6];
} Groups;

/* normal groups (k-means on normal lines, k = 1..KCFG) of a list of triangles */
static void make_groups(const float *pos, const uint32_t *ids, uint32_t c, Groups *out) {
        double *N = (double *)malloc(sizeof(double) * 3 * c), *Ev = (double *)malloc(sizeof(double) * c),
               *Gv = (double *)malloc(sizeof(double) * c);
        int *ok = (int *)malloc(sizeof(int) * c), *lab = (int *)malloc(sizeof(int) * c);
        for (uint32_t j = 0; j < c; j++) {
            const float *p = pos + 9 * (size_t)ids[j];
            double e1[3], e2[3];
            for (int i = 0; i < 3; i++) {
                e1[i] = (double)(p[3 + i] - p[i]);
                e2[i] = (double)(p[6 + i] - p[i]);
            }
            double nv[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]};
            double nl = sqrt(nv[0] * nv[0] + nv[1] * nv[1] + nv[2] * nv[2]);
            Ev[j] = fmax(fabs(e1[0]) + fabs(e1[1]) + fabs(e1[2]), fabs(e2[0]) + fabs(e2[1]) + fabs(e2[2]));
            ok[j] = nl > 0;
            Gv[j] = ok[j] ? Ev[j] * Ev[j] / nl : 0;
            for (int i = 0; i < 3; i++) N[3 * j + i] = ok[j] ? nv[i] / nl : 0;
        }
        for (int k = 0; k < KCFG; k++) {
            Groups *G = out + k;
            const int K = k + 1;
            double C[KMAX][3];
            int nc = 0;
            /* farthest-point init on normal lines, then k-means (sign-free) */
            for (uint32_t j = 0; j < c && nc == 0; j++)
                if (ok[j]) {
                    for (int i = 0; i < 3; i++) C[0][i] = N[3 * j + i];
                    nc = 1;
                }
            while (nc && nc < K) {
                double worst = 2;
                int wj = -1;
                for (uint32_t j = 0; j < c; j++) {
                    if (!ok[j]) continue;
                    double best = 0;
                    for (int q = 0; q < nc; q++)
                        best = fmax(best, fabs(N[3 * j] * C[q][0] + N[3 * j + 1] * C[q][1] + N[3 * j + 2] * C[q][2]));
                    if (best < worst) {
                        worst = best;
                        wj = (int)j;
                    }
                }
                if (wj < 0 || worst > 0.999999) break;
                for (int i = 0; i < 3; i++) C[nc][i] = N[3 * wj + i];
                nc++;
            }
            for (int it = 0; it < 10 && nc; it++) {
                double M[KMAX][9];
                memset(M, 0, sizeof(M));
                for (uint32_t j = 0; j < c; j++) {
                    if (!ok[j]) continue;
                    int bq = 0;
                    double best = -1;
                    for (int q = 0; q < nc; q++) {
                        double v = fabs(N[3 * j] * C[q][0] + N[3 * j + 1] * C[q][1] + N[3 * j + 2] * C[q][2]);
                        if (v > best) {
                            best = v;
                            bq = q;
                        }
                    }
                    lab[j] = bq;
                    for (int a = 0; a < 3; a++)
                        for (int b = 0; b < 3; b++) M[bq][3 * a + b] += N[3 * j + a] * N[3 * j + b];
                }
                for (int q = 0; q < nc; q++) {
                    double v[3] = {C[q][0], C[q][1], C[q][2]};
                    for (int r = 0; r < 30; r++) {
                        double w[3] = {M[q][0] * v[0] + M[q][1] * v[1] + M[q][2] * v[2],
                                       M[q][3] * v[0] + M[q][4] * v[1] + M[q][5] * v[2],
                                       M[q][6] * v[0] + M[q][7] * v[1] + M[q][8] * v[2]};
                        double l = sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
                        if (!(l > 0)) break;
                        for (int i = 0; i < 3; i++) v[i] = w[i] / l;
                    }
                    for (int i = 0; i < 3; i++) C[q][i] = v[i];
                }
            }
            G->ng = nc;
            G->risky = 0;
            for (int q = 0; q < nc; q++) {
                G->size[q] = 0;
                G->ct[q] = 1;
                G->g[q] = G->E[q] = 0;
                for (int i = 0; i < 3; i++) {
                    G->ax[q][i] = C[q][i];
                    G->box[q][i] = INFINITY;
                    G->box[q][3 + i] = -INFINITY;
                }
            }
            for (uint32_t j = 0; j < c; j++) {
                if (!ok[j] || !nc) {
                    G->risky++;
                    continue;
                }
                int bq = 0;
                double best = -1;
                for (int q = 0; q < nc; q++) {
                    double v = fabs(N[3 * j] * C[q][0] + N[3 * j + 1] * C[q][1] + N[3 * j + 2] * C[q][2]);
                    if (v > best) {
                        best = v;
                        bq = q;
                    }
                }
                G->size[bq]++;
                G->ct[bq] = fmin(G->ct[bq], fmax(0.0, best - 1e-9));
                G->g[bq] = fmax(G->g[bq], Gv[j]);
                G->E[bq] = fmax(G->E[bq], Ev[j]);
                const float *p = pos + 9 * (size_t)ids[j];
                for (int v = 0; v < 3; v++)
                    for (int i = 0; i < 3; i++) {
                        G->box[bq][i] = fmin(G->box[bq][i], p[3 * v + i]);
                        G->box[bq][3 + i] = fmax(G->box[bq][3 + i], p[3 * v + i]);
                    }
            }
            for (int q = 0; q < nc; q++) G->st[q] = sqrt(1 - G->ct[q] * G->ct[q]);
        }
        free(N);
        free(Ev);
        free(Gv);
        free(ok);
        free(lab);
}


typedef struct {
    const uint32_t *is_leaf, *axis, *child, *first, *count, *refs;
    const float *split, *box, *pos; /* pos: 9 floats per triangle */
    double *lbox;                   /* per node: tight box of the leaf's triangles (min3 max3) */
    double *sbox;                   /* per node: union of the leaf boxes of its subtree */
    double spad;                    /* relative pad of the padded subtree variant (x scene extent) */
    Cone *cone;
    Groups *grp; /* [node][KCFG]: 1..KCFG groups */
    Groups *sgrp; /* [node]: SUBK groups over the subtree's references */
} Tree;

enum { S_QUERIES, S_LEAVES, S_TESTS, S_LEAF_EMPTY, S_CULL0_LEAVES, S_CULL0_TESTS, S_CULLP_LEAVES, S_CULLP_TESTS,
       S_OCCLUDED, S_CONE_LEAVES, S_CONE_TESTS, S_CONE_FAIL, S_G1_TESTS, S_G2_TESTS, S_G3_TESTS, S_G4_TESTS,
       S_INNER, S_SUB_ROOTS, S_SUB_INNER, S_SUB_LEAVES, S_SUB_TESTS, S_SUBP_ROOTS, S_SUBP_INNER, S_SUBP_LEAVES,
       S_SUBP_TESTS, S_SUBG_ROOTS, S_SUBG_INNER, S_SUBG_LEAVES, S_SUBG_TESTS, S_N };


static int mt(const float o[3], const float d[3], const float *tri, float tmax, float *tout) {
    float e1[3], e2[3], p[3], sv[3], q[3];
    for (int i = 0; i < 3; i++) {
        e1[i] = tri[3 + i] - tri[i];
        e2[i] = tri[6 + i] - tri[i];
    }
    p[0] = d[1] * e2[2] - d[2] * e2[1];
    p[1] = d[2] * e2[0] - d[0] * e2[2];
    p[2] = d[0] * e2[1] - d[1] * e2[0];
    float a = (e1[0] * p[0] + e1[1] * p[1]) + e1[2] * p[2];
    if (a < FLT_EPSILON && a > -FLT_EPSILON) return 0;
    float f = 1.f / a;
    for (int i = 0; i < 3; i++) sv[i] = o[i] - tri[i];
    float u = f * ((sv[0] * p[0] + sv[1] * p[1]) + sv[2] * p[2]);
    if (u < 0.f || u > 1.f) return 0;
    q[0] = sv[1] * e1[2] - sv[2] * e1[1];
    q[1] = sv[2] * e1[0] - sv[0] * e1[2];
    q[2] = sv[0] * e1[1] - sv[1] * e1[0];
    float v = f * ((d[0] * q[0] + d[1] * q[1]) + d[2] * q[2]);
    if (v < 0.f || u + v > 1.f) return 0;
    float t = f * ((e2[0] * q[0] + e2[1] * q[1]) + e2[2] * q[2]);
    *tout = t;
    return t >= 0.f && t < tmax;
}

/* The padded skip test of one triangle for one ray: bounds of the exact line-triangle
 * configuration any accepting float evaluation implies (camcull.hpp's error terms with
 * this ray's sv), as a box pad and a t range; returns 0 when no bound exists (|AA| too
 * small against its error: never skip). */
static int tri_pad(const float o[3], const float d[3], const float *tri, float tmax, double *pad, double *tlo,
                   double *thi) {
    const double u = 0x1p-24;
    double e1[3], e2[3], s[3], D[3];
    for (int i = 0; i < 3; i++) {
        e1[i] = (double)(tri[3 + i] - tri[i]);
        e2[i] = (double)(tri[6 + i] - tri[i]);
        s[i] = (double)(o[i] - tri[i]);
        D[i] = fabs((double)d[i]);
    }
    double P[3] = {D[1] * fabs(e2[2]) + D[2] * fabs(e2[1]), D[2] * fabs(e2[0]) + D[0] * fabs(e2[2]),
                   D[0] * fabs(e2[1]) + D[1] * fabs(e2[0])};
    double Q[3] = {fabs(s[1] * e1[2]) + fabs(s[2] * e1[1]), fabs(s[2] * e1[0]) + fabs(s[0] * e1[2]),
                   fabs(s[0] * e1[1]) + fabs(s[1] * e1[0])};
    double Ea = 5.1 * u * (fabs(e1[0]) * P[0] + fabs(e1[1]) * P[1] + fabs(e1[2]) * P[2]);
    double Eu = 5.1 * u * (fabs(s[0]) * P[0] + fabs(s[1]) * P[1] + fabs(s[2]) * P[2]);
    double Ev = 5.1 * u * (D[0] * Q[0] + D[1] * Q[1] + D[2] * Q[2]);
    double Et = 5.1 * u * (fabs(e2[0]) * Q[0] + fabs(e2[1]) * Q[1] + fabs(e2[2]) * Q[2]);
    double p[3] = {d[1] * e2[2] - d[2] * e2[1], d[2] * e2[0] - d[0] * e2[2], d[0] * e2[1] - d[1] * e2[0]};
    double AA = e1[0] * p[0] + e1[1] * p[1] + e1[2] * p[2];
    double aAA = fabs(AA);
    if (aAA <= 2.0 * Ea + 1e-30) return 0;
    double Kw = Ea + Eu + Ev + 3.1 * u * (aAA + Ea);
    double den = aAA - Ea;
    double m = (Eu + Ev + Kw) / den; /* barycentric margin */
    double le = 0;
    for (int i = 0; i < 3; i++) le = fmax(le, fabs(e1[i]) + fabs(e2[i]));
    *pad = m * le + u * (fabs(s[0]) + fabs(s[1]) + fabs(s[2])) + 1e-9;
    *tlo = -Et / den;
    *thi = (double)tmax * (1.0 + Ea / den) * (1.0 + 4 * u) + Et / den;
    return 1;
}

/* does the segment o + t d, t in [t0, t1], meet the box [lo, hi]? (double, exact enough) */
static int seg_box(const float o[3], const float d[3], double t0, double t1, const double lo[3], const double hi[3]) {
    for (int a = 0; a < 3; a++) {
        double oa = o[a], da = d[a];
        if (da == 0.0) {
            if (oa < lo[a] || oa > hi[a]) return 0;
            continue;
        }
        double ta = (lo[a] - oa) / da, tb = (hi[a] - oa) / da;
        if (ta > tb) {
            double x = ta;
            ta = tb;
            tb = x;
        }
        t0 = fmax(t0, ta);
        t1 = fmin(t1, tb);
        if (t0 > t1) return 0;
    }
    return 1;
}

/* the per-group skip: true when no triangle of the group (normal lines within the cone,
 * all inside box, E / g bounds) can accept for this ray's segment [0, tmax] */
static int group_skip(const float o[3], const float d[3], float tmax, const double ax[3], double ct, double st,
                      double g, double E, const double *bx) {
    /* DESIGN: accept => o + t d within pad of the group box for some t in [tlo, thi], with
     *   cb  = cos(psi + theta) <= |d^.n^| for every normal of the group (cone)
     *   pad = 20.12u (E + 2S) g / cb + u (S + 6.2 E),   dt = 10.05u S g / cb
     *   t in [-dt, tmax (1 + 10.05u g / cb)(1 + 2.1u) + dt]   (needs cb > 20.1u g) */
    const double u = 0x1p-24;
    double dn = fabs(d[0] * ax[0] + d[1] * ax[1] + d[2] * ax[2]);
    double sn = sqrt(fmax(0.0, 1.0 - dn * dn));
    double cb = dn * ct - sn * st;
    double S = 0.0;
    for (int i = 0; i < 3; i++) S = fmax(S, fmax(fabs(o[i] - bx[i]), fabs(o[i] - bx[3 + i])));
    if (!(cb > 20.1 * u * g)) return 0;
    double pad = 20.12 * u * (E + 2 * S) * g / cb + u * (S + 6.2 * E);
    double dt = 10.05 * u * S * g / cb;
    double lo[3], hi[3];
    for (int i = 0; i < 3; i++) {
        lo[i] = bx[i] - pad;
        hi[i] = bx[3 + i] + pad;
    }
    return !seg_box(o, d, -dt, (double)tmax * (1 + 10.05 * u * g / cb) * (1 + 2.1 * u) + dt, lo, hi);
}

static void leaf_census(const Tree *T, uint32_t n, const float o[3], const float d[3], float tmax, uint64_t *st) {
    const uint32_t c = T->count[n], f = T->first[n];
    if (!c) {
        st[S_LEAF_EMPTY]++;
        return;
    }
    const double *lb = T->lbox + 6 * (size_t)n;
    if (!seg_box(o, d, 0.0, (double)tmax, lb, lb + 3)) {
        st[S_CULL0_LEAVES]++;
        st[S_CULL0_TESTS] += c;
    }
    /* implementable: the leaf box padded by the bound valid for every ray whose direction
     * line lies within the cone's complement (|d.n| >= cos(psi + theta) |n| for all normals) */
    {
        const Cone *K = T->cone + n;
        int skip = 0;
        if (K->ok) {
            const double u = 0x1p-24;
            double dn = fabs(d[0] * K->ax[0] + d[1] * K->ax[1] + d[2] * K->ax[2]);
            double dl = sqrt((double)d[0] * d[0] + (double)d[1] * d[1] + (double)d[2] * d[2]);
            dn /= dl;
            double sn = sqrt(fmax(0.0, 1.0 - dn * dn));
            double cb = dn * K->ct - sn * K->st; /* cos(psi + theta) */
            double S = 0.0;
            for (int i = 0; i < 3; i++) S = fmax(S, fmax(fabs(o[i] - lb[i]), fabs(o[i] - lb[3 + i])));
            double den = cb - 17.7 * u * K->g;
            if (den > 0) {
                double m = (2 * 17.7 * u * S + 2 * 30.6 * u * S + 2 * 17.7 * u * K->E + 3.1 * u * 3 * K->E) * K->g / den;
                double pad = m * K->E + u * 3 * S + 1e-6 * (S + K->E);
                double dt = 30.6 * u * S * K->g / den;
                double lo[3], hi[3];
                for (int i = 0; i < 3; i++) {
                    lo[i] = lb[i] - pad;
                    hi[i] = lb[3 + i] + pad;
                }
                if (!seg_box(o, d, -dt, (double)tmax * (1 + 17.7 * u * K->g / den) * (1 + 4 * u) + dt, lo, hi))
                    skip = 1;
            } else {
                st[S_CONE_FAIL]++;
            }
        } else {
            st[S_CONE_FAIL]++;
        }
        if (skip) {
            st[S_CONE_LEAVES]++;
            st[S_CONE_TESTS] += c;
        }
    }
    for (int k = 0; k < KCFG; k++) {
        const Groups *G = T->grp + (size_t)n * KCFG + k;
        uint64_t left = G->risky;
        for (int q = 0; q < G->ng; q++)
            if (!group_skip(o, d, tmax, G->ax[q], G->ct[q], G->st[q], G->g[q], G->E[q], G->box[q])) left += G->size[q];
        st[S_G1_TESTS + k] += c - left;
    }
    /* padded: the union over the leaf's triangles of each one's own padded box and t range */
    int skip = 1;
    for (uint32_t j = 0; j < c && skip; j++) {
        const float *tri = T->pos + 9 * (size_t)T->refs[f + j];
        double pad, tlo, thi;
        if (!tri_pad(o, d, tri, tmax, &pad, &tlo, &thi)) {
            skip = 0;
            break;
        }
        double lo[3], hi[3];
        for (int i = 0; i < 3; i++) {
            lo[i] = fmin(fmin(tri[i], tri[3 + i]), tri[6 + i]) - pad;
            hi[i] = fmax(fmax(tri[i], tri[3 + i]), tri[6 + i]) + pad;
        }
        if (seg_box(o, d, tlo, thi, lo, hi)) skip = 0;
    }
    if (skip) {
        st[S_CULLP_LEAVES]++;
        st[S_CULLP_TESTS] += c;
    }
}

/* returns 1 when the shadow query is occluded / the closest query hit */
static int node(const Tree *T, uint32_t n, const float o[3], const float d[3], float tmin, float tmax, int shadow,
                uint32_t excl, float *best, uint64_t *st, int sub, int subp, int subg, int entry) {
    /* subtree census: would a box test of the subtree's triangle union against [0, tmax]
     * skip this node (sub: unpadded, an upper bound; subp: padded by spad) */
    {
        const double *sb = T->sbox + 6 * (size_t)n;
        if (!sub && !seg_box(o, d, 0.0, (double)tmax, sb, sb + 3)) {
            sub = 1;
            st[S_SUB_ROOTS]++;
        }
        if (!subp) {
            double lo[3], hi[3];
            for (int i = 0; i < 3; i++) {
                lo[i] = sb[i] - T->spad;
                hi[i] = sb[3 + i] + T->spad;
            }
            if (!seg_box(o, d, -T->spad, (double)tmax * (1 + 1e-5) + T->spad, lo, hi)) {
                subp = 1;
                st[S_SUBP_ROOTS]++;
            }
        }
    }
    /* entry: 0 root, 1 near-only / far-only step, 2 near child of a split, 3 far child of a split (the pop) */
    if (!subg && (T->is_leaf[n] ? T->count[n] > 0 : 1) &&
        (SUBMODE == 1 || entry == 0 || (SUBMODE == 2 && entry == 3) || (SUBMODE == 3 && entry >= 2))) {
        const Groups *G = T->sgrp + n;
        int skip = G->ng > 0 && !G->risky;
        for (int q = 0; q < G->ng && skip; q++)
            if (!group_skip(o, d, tmax, G->ax[q], G->ct[q], G->st[q], G->g[q], G->E[q], G->box[q])) skip = 0;
        if (skip) {
            subg = 1;
            st[S_SUBG_ROOTS]++;
        }
    }
    if (T->is_leaf[n]) {
        if (subg) {
            st[S_SUBG_LEAVES]++;
            st[S_SUBG_TESTS] += T->count[n];
        }
        st[S_LEAVES]++;
        if (sub) {
            st[S_SUB_LEAVES]++;
            st[S_SUB_TESTS] += T->count[n];
        }
        if (subp) {
            st[S_SUBP_LEAVES]++;
            st[S_SUBP_TESTS] += T->count[n];
        }
        leaf_census(T, n, o, d, tmax, st);
        int hit = 0;
        for (uint32_t j = 0; j < T->count[n]; j++) {
            const uint32_t id = T->refs[T->first[n] + j];
            if (shadow && id == excl) continue;
            st[S_TESTS]++;
            float t;
            if (mt(o, d, T->pos + 9 * (size_t)id, shadow ? tmax : *best, &t)) {
                if (shadow) return 1;
                *best = t;
                hit = 1;
            }
        }
        return hit;
    }
    st[S_INNER]++;
    if (sub) st[S_SUB_INNER]++;
    if (subp) st[S_SUBP_INNER]++;
    if (subg) st[S_SUBG_INNER]++;
    const uint32_t a = T->axis[n];
    const float pos = T->split[n];
    const float ts = (pos - o[a]) / d[a];
    const int below = o[a] < pos || (o[a] == pos && d[a] <= 0);
    const uint32_t nearc = T->child[n] + (1 - below), farc = T->child[n] + below;
    if (ts >= tmax || ts < 0) return node(T, nearc, o, d, tmin, tmax, shadow, excl, best, st, sub, subp, subg, 1);
    if (ts <= tmin) return node(T, farc, o, d, tmin, tmax, shadow, excl, best, st, sub, subp, subg, 1);
    if (!shadow) *best = ts;
    if (node(T, nearc, o, d, tmin, ts, shadow, excl, best, st, sub, subp, subg, 2)) return 1;
    if (!shadow) *best = tmax;
    return node(T, farc, o, d, ts, tmax, shadow, excl, best, st, sub, subp, subg, 3);
}

void census(uint32_t nn, const uint32_t *is_leaf, const uint32_t *axis, const float *split, const uint32_t *child,
            const uint32_t *first, const uint32_t *count, const uint32_t *refs, const float *box, const float *pos,
            uint32_t nr, const float *orig, const float *dir, const float *dist, const uint32_t *excl, int shadow,
            uint64_t *out, double spad_rel) {
    Tree T = {is_leaf, axis, child, first, count, refs, split, box, pos, NULL, NULL, 0.0, NULL, NULL, NULL};
    T.lbox = (double *)malloc(sizeof(double) * 6 * (size_t)nn);
    for (uint32_t n = 0; n < nn; n++) {
        double *b = T.lbox + 6 * (size_t)n;
        b[0] = b[1] = b[2] = INFINITY;
        b[3] = b[4] = b[5] = -INFINITY;
        if (!is_leaf[n]) continue;
        for (uint32_t j = 0; j < count[n]; j++) {
            const float *p = pos + 9 * (size_t)refs[first[n] + j];
            for (int v = 0; v < 3; v++)
                for (int i = 0; i < 3; i++) {
                    b[i] = fmin(b[i], p[3 * v + i]);
                    b[3 + i] = fmax(b[3 + i], p[3 * v + i]);
                }
        }
    }
    T.sbox = (double *)malloc(sizeof(double) * 6 * (size_t)nn);
    memcpy(T.sbox, T.lbox, sizeof(double) * 6 * (size_t)nn);
    for (uint32_t n = nn; n-- > 0;) /* children follow their parent in DFS order */
        if (!is_leaf[n])
            for (int c = 0; c < 2; c++) {
                const double *b = T.sbox + 6 * (size_t)(child[n] + c);
                for (int i = 0; i < 3; i++) {
                    T.sbox[6 * (size_t)n + i] = fmin(T.sbox[6 * (size_t)n + i], b[i]);
                    T.sbox[6 * (size_t)n + 3 + i] = fmax(T.sbox[6 * (size_t)n + 3 + i], b[3 + i]);
                }
            }
    {
        double ext = 0;
        for (int i = 0; i < 3; i++) ext = fmax(ext, (double)box[3 + i] - box[i]);
        T.spad = ext * spad_rel;
    }
    T.cone = (Cone *)calloc(nn, sizeof(Cone));
    for (uint32_t n = 0; n < nn; n++) {
        if (!is_leaf[n] || !count[n]) continue;
        Cone *K = T.cone + n;
        /* axis: principal direction of sum n n^T (normal lines, sign-free), then the widest angle */
        double M[9] = {0};
        double g = 0, E = 0;
        int bad = 0;
        for (uint32_t j = 0; j < count[n]; j++) {
            const float *p = pos + 9 * (size_t)refs[first[n] + j];
            double e1[3], e2[3];
            for (int i = 0; i < 3; i++) {
                e1[i] = (double)(p[3 + i] - p[i]);
                e2[i] = (double)(p[6 + i] - p[i]);
            }
            double nv[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]};
            double nl = sqrt(nv[0] * nv[0] + nv[1] * nv[1] + nv[2] * nv[2]);
            double e = fmax(fabs(e1[0]) + fabs(e1[1]) + fabs(e1[2]), fabs(e2[0]) + fabs(e2[1]) + fabs(e2[2]));
            E = fmax(E, e);
            if (!(nl > 0)) { /* degenerate: AA is rounding noise, the test rejects unless |AA_c| >= eps */
                bad = 1;
                continue;
            }
            g = fmax(g, e * e / nl);
            for (int a = 0; a < 3; a++)
                for (int b = 0; b < 3; b++) M[3 * a + b] += nv[a] * nv[b] / (nl * nl);
        }
        if (bad) continue;
        double v[3] = {1, 1, 1};
        for (int it = 0; it < 60; it++) {
            double w[3] = {M[0] * v[0] + M[1] * v[1] + M[2] * v[2], M[3] * v[0] + M[4] * v[1] + M[5] * v[2],
                           M[6] * v[0] + M[7] * v[1] + M[8] * v[2]};
            double l = sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
            if (!(l > 0)) break;
            for (int i = 0; i < 3; i++) v[i] = w[i] / l;
        }
        double cmin = 1.0;
        for (uint32_t j = 0; j < count[n]; j++) {
            const float *p = pos + 9 * (size_t)refs[first[n] + j];
            double e1[3], e2[3];
            for (int i = 0; i < 3; i++) {
                e1[i] = (double)(p[3 + i] - p[i]);
                e2[i] = (double)(p[6 + i] - p[i]);
            }
            double nv[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]};
            double nl = sqrt(nv[0] * nv[0] + nv[1] * nv[1] + nv[2] * nv[2]);
            cmin = fmin(cmin, fabs(nv[0] * v[0] + nv[1] * v[1] + nv[2] * v[2]) / nl);
        }
        cmin = fmax(0.0, cmin - 1e-9);
        for (int i = 0; i < 3; i++) K->ax[i] = v[i];
        K->ct = cmin;
        K->st = sqrt(1 - cmin * cmin);
        K->g = g;
        K->E = E;
        K->ok = 1;
    }
    T.grp = (Groups *)calloc((size_t)nn * KCFG, sizeof(Groups));
#pragma omp parallel for schedule(dynamic, 64)
    for (uint32_t n = 0; n < nn; n++) {
        if (!is_leaf[n] || !count[n]) continue;
        make_groups(pos, refs + first[n], count[n], T.grp + (size_t)n * KCFG);
    }
    /* subtree groups: the same over every reference of the subtree's leaves */
    T.sgrp = (Groups *)calloc((size_t)nn, sizeof(Groups));
#pragma omp parallel for schedule(dynamic, 1)
    for (uint32_t n = 0; n < nn; n++) {
        if (is_leaf[n]) {
            if (count[n]) {
                Groups G4[KCFG];
                make_groups(pos, refs + first[n], count[n], G4);
                T.sgrp[n] = G4[SUBK - 1];
            }
            continue;
        }
        uint32_t cap = 1024, c = 0, sp = 0, stk[256];
        uint32_t *ids = (uint32_t *)malloc(sizeof(uint32_t) * cap);
        stk[sp++] = n;
        while (sp) {
            uint32_t m = stk[--sp];
            if (!is_leaf[m]) {
                stk[sp++] = child[m];
                stk[sp++] = child[m] + 1;
                continue;
            }
            for (uint32_t j = 0; j < count[m]; j++) {
                if (c == cap) ids = (uint32_t *)realloc(ids, sizeof(uint32_t) * (cap *= 2));
                ids[c++] = refs[first[m] + j];
            }
        }
        if (c) {
            Groups G4[KCFG];
            make_groups(pos, ids, c, G4);
            T.sgrp[n] = G4[SUBK - 1];
        }
        free(ids);
    }
    memset(out, 0, sizeof(uint64_t) * S_N);
#pragma omp parallel
    {
        uint64_t st[S_N] = {0};
#pragma omp for schedule(dynamic, 256)
        for (uint32_t r = 0; r < nr; r++) {
            const float *o = orig + 3 * (size_t)r, *d = dir + 3 * (size_t)r;
            /* root slab test, kdtree.cpp:196-216 (std::min / max forms) */
            float t0 = -INFINITY, t1 = INFINITY;
            float tn[3], tf[3];
            for (int a = 0; a < 3; a++) {
                float inv = 1.f / d[a];
                float x = (box[a] - o[a]) * inv, y = (box[3 + a] - o[a]) * inv;
                tn[a] = y < x ? y : x;
                tf[a] = x < y ? y : x;
            }
            float tmin = tn[0] < tn[1] ? tn[1] : tn[0];
            tmin = tmin < tn[2] ? tn[2] : tmin;
            float tmax = tf[1] < tf[0] ? tf[1] : tf[0];
            tmax = tf[2] < tmax ? tf[2] : tmax;
            (void)t0;
            (void)t1;
            st[S_QUERIES]++;
            if (tmax < 0 || tmax < tmin) continue;
            if (shadow) {
                if (tmin > dist[r]) continue;
                tmax = dist[r] < tmax ? dist[r] : tmax;
            }
            float best = tmax;
            if (node(&T, 0, o, d, tmin, tmax, shadow, excl ? excl[r] : 0xffffffffu, &best, st, 0, 0, 0, 0) && shadow)
                st[S_OCCLUDED]++;
        }
#pragma omp critical
        for (int i = 0; i < S_N; i++) out[i] += st[i];
    }
    free(T.lbox);
    free(T.sbox);
    free(T.cone);
    free(T.grp);
    free(T.sgrp);
}
