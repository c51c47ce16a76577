/* bvh_census.c -- CPU census (diagnostic only): shadow queries answered by the reference's kd
 * traversal (kdtree.cpp:283-344, plain recursion) against an any-hit walk of a binned-SAH BVH over
 * the same triangles, whose answer is "some triangle != light passes Moller-Trumbore with t < D"
 * (D = the segment end).  Every kd OCCLUDED answer needs such a triangle (a leaf accepts with
 * t < tmax_leaf <= D), so a BVH walk that finds none proves VISIBLE; the census counts the work of
 * both and how often the BVH finds a triangle the kd traversal does not (then the kd answer rules).
 * Built by scripts/bvh_census.py. */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

enum { S_QUERIES, S_KD_OCC, S_KD_INNER, S_KD_LEAVES, S_KD_TESTS, S_BVH_FOUND, S_BVH_NODES, S_BVH_TESTS,
       S_BVH_VIS_NODES, S_BVH_VIS_TESTS, S_KD_VIS_INNER, S_KD_VIS_LEAVES, S_KD_VIS_TESTS, S_MISMATCH_FOUND,
       S_MISMATCH_OCC, S_BVH_OCC_NODES, S_BVH_OCC_TESTS, S_KD_OCC_INNER, S_KD_OCC_LEAVES, S_KD_OCC_TESTS,
       S_BVH_LEAVES, S_PR_FOUND, S_PR_NODES, S_PR_TESTS, S_PR_VIS_NODES, S_PR_VIS_TESTS, S_PR_MISS, S_N };

/* kdtree.cpp:293-320 (float, no contraction: gcc -ffp-contract=off) */
static int mt(const float o[3], const float d[3], const float *tri, float tmax, float *tout) {
    float e1[3], e2[3], p[3], s[3], q[3];
    for (int i = 0; i < 3; i++) {
        e1[i] = tri[3 + i] - tri[i];
        e2[i] = tri[6 + i] - tri[i];
    }
    p[0] = d[1] * e2[2] - d[2] * e2[1];
    p[1] = d[2] * e2[0] - d[0] * e2[2];
    p[2] = d[0] * e2[1] - d[1] * e2[0];
    const float a = (e1[0] * p[0] + e1[1] * p[1]) + e1[2] * p[2];
    if (fabsf(a) < FLT_EPSILON) return 0;
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
    if (t >= 0.f && t < tmax) {
        *tout = t;
        return 1;
    }
    return 0;
}

typedef struct {
    const uint32_t *is_leaf, *axis, *child, *first, *count, *refs;
    const float *split, *pos;
} Kd;

static int kd_node(const Kd *T, uint32_t n, const float o[3], const float d[3], float tmin, float tmax, uint32_t excl,
                   uint64_t *c) {
    if (T->is_leaf[n]) {
        c[0]++;
        for (uint32_t j = 0; j < T->count[n]; j++) {
            const uint32_t id = T->refs[T->first[n] + j];
            if (id == excl) continue;
            c[1]++;
            float t;
            if (mt(o, d, T->pos + 9 * (size_t)id, tmax, &t)) return 1;
        }
        return 0;
    }
    c[2]++;
    const uint32_t a = T->axis[n];
    const float sp = T->split[n];
    const float ts = (sp - o[a]) / d[a];
    const int below = o[a] < sp || (o[a] == sp && d[a] <= 0);
    const uint32_t nearc = T->child[n] + (1 - below), farc = T->child[n] + below;
    if (ts >= tmax || ts < 0) return kd_node(T, nearc, o, d, tmin, tmax, excl, c);
    if (ts <= tmin) return kd_node(T, farc, o, d, tmin, tmax, excl, c);
    if (kd_node(T, nearc, o, d, tmin, ts, excl, c)) return 1;
    return kd_node(T, farc, o, d, ts, tmax, excl, c);
}

/* ---- BVH: binned SAH (16 bins per axis over centroids), leaves of <= LEAF triangles ---- */
#ifndef LEAF
#define LEAF 4
#endif
typedef struct {
    float lo[3], hi[3];
    uint32_t left, first, count; /* inner: count 0, children left, left + 1 */
    /* proof data (double): cone of normal LINES (axis, half-angle), max E = |e1|_1 + |e2|_1, max g = E^2/|N| */
    double ax[3], rho, E, g;
    int degen;
} BNode;
typedef struct {
    BNode *n;
    uint32_t nn, cap;
    uint32_t *ids;
    const float *pos;
    float *cen;
} Bvh;

static void tri_box(const float *p, float lo[3], float hi[3]) {
    for (int i = 0; i < 3; i++) {
        lo[i] = fminf(p[i], fminf(p[3 + i], p[6 + i]));
        hi[i] = fmaxf(p[i], fmaxf(p[3 + i], p[6 + i]));
    }
}
static float area(const float lo[3], const float hi[3]) {
    const float x = hi[0] - lo[0], y = hi[1] - lo[1], z = hi[2] - lo[2];
    return x < 0 ? 0 : 2 * (x * y + y * z + z * x);
}
static uint32_t bvh_alloc(Bvh *B) {
    if (B->nn == B->cap) {
        B->cap = B->cap ? 2 * B->cap : 1024;
        B->n = (BNode *)realloc(B->n, sizeof(BNode) * B->cap);
    }
    return B->nn++;
}
static void bvh_build(Bvh *B, uint32_t node, uint32_t first, uint32_t count) {
    BNode *N = &B->n[node];
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    float clo[3] = {INFINITY, INFINITY, INFINITY}, chi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (uint32_t j = first; j < first + count; j++) {
        float a[3], b[3];
        tri_box(B->pos + 9 * (size_t)B->ids[j], a, b);
        for (int i = 0; i < 3; i++) {
            lo[i] = fminf(lo[i], a[i]);
            hi[i] = fmaxf(hi[i], b[i]);
            const float c = B->cen[3 * (size_t)B->ids[j] + i];
            clo[i] = fminf(clo[i], c);
            chi[i] = fmaxf(chi[i], c);
        }
    }
    memcpy(N->lo, lo, sizeof lo);
    memcpy(N->hi, hi, sizeof hi);
    N->first = first;
    N->count = count;
    N->left = 0;
    if (count <= LEAF) return;
    enum { NB = 16 };
    float best = INFINITY;
    int bax = -1, bsplit = 0;
    for (int ax = 0; ax < 3; ax++) {
        const float ext = chi[ax] - clo[ax];
        if (!(ext > 0)) continue;
        float blo[NB][3], bhi[NB][3];
        uint32_t bc[NB] = {0};
        for (int k = 0; k < NB; k++)
            for (int i = 0; i < 3; i++) {
                blo[k][i] = INFINITY;
                bhi[k][i] = -INFINITY;
            }
        for (uint32_t j = first; j < first + count; j++) {
            const uint32_t id = B->ids[j];
            int k = (int)((B->cen[3 * (size_t)id + ax] - clo[ax]) / ext * NB);
            k = k < 0 ? 0 : (k >= NB ? NB - 1 : k);
            float a[3], b[3];
            tri_box(B->pos + 9 * (size_t)id, a, b);
            bc[k]++;
            for (int i = 0; i < 3; i++) {
                blo[k][i] = fminf(blo[k][i], a[i]);
                bhi[k][i] = fmaxf(bhi[k][i], b[i]);
            }
        }
        for (int s = 1; s < NB; s++) {
            float l0[3] = {INFINITY, INFINITY, INFINITY}, l1[3] = {-INFINITY, -INFINITY, -INFINITY};
            float r0[3] = {INFINITY, INFINITY, INFINITY}, r1[3] = {-INFINITY, -INFINITY, -INFINITY};
            uint32_t nl = 0, nr = 0;
            for (int k = 0; k < NB; k++) {
                float *a0 = k < s ? l0 : r0, *a1 = k < s ? l1 : r1;
                if (k < s) nl += bc[k];
                else nr += bc[k];
                for (int i = 0; i < 3; i++) {
                    a0[i] = fminf(a0[i], blo[k][i]);
                    a1[i] = fmaxf(a1[i], bhi[k][i]);
                }
            }
            if (!nl || !nr) continue;
            const float cost = area(l0, l1) * nl + area(r0, r1) * nr;
            if (cost < best) {
                best = cost;
                bax = ax;
                bsplit = s;
            }
        }
    }
    if (bax < 0 || best >= area(lo, hi) * count) { /* no useful split: a leaf (large leaves split by median) */
        if (count <= 4 * LEAF || bax < 0) {
            if (bax < 0 && count > LEAF) { /* all centroids equal: split by index */
                const uint32_t l = bvh_alloc(B), r = bvh_alloc(B);
                (void)r;
                B->n[node].left = l;
                B->n[node].count = 0;
                bvh_build(B, l, first, count / 2);
                bvh_build(B, l + 1, first + count / 2, count - count / 2);
            }
            return;
        }
    }
    const float ext = chi[bax] - clo[bax];
    uint32_t m = first;
    for (uint32_t j = first; j < first + count; j++) {
        const uint32_t id = B->ids[j];
        int k = (int)((B->cen[3 * (size_t)id + bax] - clo[bax]) / ext * NB);
        k = k < 0 ? 0 : (k >= NB ? NB - 1 : k);
        if (k < bsplit) {
            const uint32_t t = B->ids[m];
            B->ids[m] = id;
            B->ids[j] = t;
            m++;
        }
    }
    if (m == first || m == first + count) m = first + count / 2;
    const uint32_t l = bvh_alloc(B), r = bvh_alloc(B);
    (void)r;
    B->n[node].left = l;
    B->n[node].count = 0;
    bvh_build(B, l, first, m - first);
    bvh_build(B, l + 1, m, first + count - m);
}

static int box_hit(const BNode *N, const float o[3], const float inv[3], float t1, float *tenter) {
    float tn = 0.f, tf = t1;
    for (int i = 0; i < 3; i++) {
        float a = (N->lo[i] - o[i]) * inv[i], b = (N->hi[i] - o[i]) * inv[i];
        if (a > b) {
            const float t = a;
            a = b;
            b = t;
        }
        if (a != a) a = -INFINITY; /* 0 * inf: the ray on a slab face */
        if (b != b) b = INFINITY;
        tn = fmaxf(tn, a);
        tf = fminf(tf, b);
    }
    *tenter = tn;
    return tn <= tf * (1 + 1e-6f) + 1e-6f; /* (a census: a slightly fat slab test) */
}

static int bvh_any(const Bvh *B, const float o[3], const float d[3], float D, uint32_t excl, uint64_t *c) {
    const float inv[3] = {1.f / d[0], 1.f / d[1], 1.f / d[2]};
    uint32_t stk[128], sp = 0, n = 0;
    float te;
    c[0]++;
    if (!box_hit(&B->n[0], o, inv, D, &te)) return 0;
    for (;;) {
        const BNode *N = &B->n[n];
        if (N->count) {
            c[2]++;
            for (uint32_t j = N->first; j < N->first + N->count; j++) {
                const uint32_t id = B->ids[j];
                if (id == excl) continue;
                c[1]++;
                float t;
                if (mt(o, d, B->pos + 9 * (size_t)id, D, &t)) return 1;
            }
        } else {
            float ta, tb;
            c[0] += 2;
            const int ha = box_hit(&B->n[N->left], o, inv, D, &ta), hb = box_hit(&B->n[N->left + 1], o, inv, D, &tb);
            if (ha && hb) {
                const uint32_t nearc = ta <= tb ? N->left : N->left + 1;
                stk[sp++] = nearc == N->left ? N->left + 1 : N->left;
                n = nearc;
                continue;
            }
            if (ha || hb) {
                n = ha ? N->left : N->left + 1;
                continue;
            }
        }
        if (!sp) return 0;
        n = stk[--sp];
    }
}

static void tri_normal(const float *p, double n[3], double *E, double *g, int *degen) {
    double e1[3], e2[3];
    for (int i = 0; i < 3; i++) {
        e1[i] = (double)(p[3 + i] - p[i]);
        e2[i] = (double)(p[6 + i] - p[i]);
    }
    double N[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]};
    double l = sqrt(N[0] * N[0] + N[1] * N[1] + N[2] * N[2]);
    *E = (fabs(e1[0]) + fabs(e1[1]) + fabs(e1[2])) + (fabs(e2[0]) + fabs(e2[1]) + fabs(e2[2]));
    *degen = !(l > 0);
    *g = l > 0 ? (*E) * (*E) / l : INFINITY;
    for (int i = 0; i < 3; i++) n[i] = l > 0 ? N[i] / l : 0;
}
static double angle_lines(const double a[3], const double b[3]) {
    double c = fabs(a[0] * b[0] + a[1] * b[1] + a[2] * b[2]);
    return acos(c > 1 ? 1 : c);
}
/* cones bottom-up: leaves from their triangles (axis = principal direction of n n^T), inner nodes from
   the children's cones (axis = sign-aligned sum, rho = max child offset + child rho) */
static void bvh_cones(Bvh *B, uint32_t node) {
    BNode *N = &B->n[node];
    if (N->count) {
        double M[9] = {0}, E = 0, g = 0;
        int degen = 0;
        for (uint32_t j = N->first; j < N->first + N->count; j++) {
            double n[3], e, gg;
            int dg;
            tri_normal(B->pos + 9 * (size_t)B->ids[j], n, &e, &gg, &dg);
            E = fmax(E, e);
            g = fmax(g, gg);
            degen |= dg;
            for (int a = 0; a < 3; a++)
                for (int b = 0; b < 3; b++) M[3 * a + b] += n[a] * n[b];
        }
        double v[3] = {0.577, 0.577, 0.577};
        for (int it = 0; it < 50; it++) {
            double w[3] = {M[0] * v[0] + M[1] * v[1] + M[2] * v[2], M[3] * v[0] + M[4] * v[1] + M[5] * v[2],
                           M[6] * v[0] + M[7] * v[1] + M[8] * v[2]};
            double l = sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
            if (!(l > 0)) break;
            for (int i = 0; i < 3; i++) v[i] = w[i] / l;
        }
        double rho = 0;
        for (uint32_t j = N->first; j < N->first + N->count; j++) {
            double n[3], e, gg;
            int dg;
            tri_normal(B->pos + 9 * (size_t)B->ids[j], n, &e, &gg, &dg);
            if (!dg) rho = fmax(rho, angle_lines(n, v));
        }
        memcpy(N->ax, v, sizeof v);
        N->rho = rho + 1e-9;
        N->E = E;
        N->g = g;
        N->degen = degen;
        return;
    }
    bvh_cones(B, N->left);
    bvh_cones(B, N->left + 1);
    const BNode *a = &B->n[N->left], *b = &B->n[N->left + 1];
    double s = (a->ax[0] * b->ax[0] + a->ax[1] * b->ax[1] + a->ax[2] * b->ax[2]) < 0 ? -1 : 1;
    double v[3] = {a->ax[0] + s * b->ax[0], a->ax[1] + s * b->ax[1], a->ax[2] + s * b->ax[2]};
    double l = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
    if (l > 0)
        for (int i = 0; i < 3; i++) v[i] /= l;
    else
        memcpy(v, a->ax, sizeof v);
    memcpy(N->ax, v, sizeof v);
    N->rho = fmin(M_PI / 2, fmax(angle_lines(v, a->ax) + a->rho, angle_lines(v, b->ax) + b->rho) + 1e-9);
    N->E = fmax(a->E, b->E);
    N->g = fmax(a->g, b->g);
    N->degen = a->degen | b->degen;
}

/* The proof walk (census, double precision): a node is skipped when no triangle below can pass
 * Moller-Trumbore with t < D for this ray:
 *   regime i  (the ray meets every normal of the node's cone at cos >= C1): the segment misses the
 *             node box padded by the leaf-cull bound at cb = C1 (leafcull.hpp, S from the box);
 *   plane     (otherwise): |h| > D cb_max + eps -- an accepting test needs the origin's distance h to the
 *             triangle's plane within D |d.n| + 10u g (D + S) (MT's t = s.N / (-d.N));
 * else the node is descended, and a leaf's triangles are tested exactly (float MT). */
#ifndef C1
#define C1 0.05
#endif
static int bvh_proof(const Bvh *B, const float o[3], const float d[3], float D, uint32_t excl, uint64_t *c) {
    const double u = 0x1p-24;
    uint32_t stk[128], sp = 0, n = 0;
    for (;;) {
        const BNode *N = &B->n[n];
        c[0]++;
        int skip = 0;
        double X[8][3], S = 0, R = 0, pmin = INFINITY, pmax = -INFINITY;
        for (int k = 0; k < 8; k++) {
            X[k][0] = (k & 1) ? N->hi[0] : N->lo[0];
            X[k][1] = (k & 2) ? N->hi[1] : N->lo[1];
            X[k][2] = (k & 4) ? N->hi[2] : N->lo[2];
            double r2 = 0;
            for (int i = 0; i < 3; i++) {
                const double dd = fabs((double)o[i] - X[k][i]);
                S = fmax(S, dd);
                r2 += dd * dd;
            }
            R = fmax(R, sqrt(r2));
            const double pa = N->ax[0] * X[k][0] + N->ax[1] * X[k][1] + N->ax[2] * X[k][2];
            pmin = fmin(pmin, pa);
            pmax = fmax(pmax, pa);
        }
        if (!N->degen && N->g < 1e15) {
            const double phi = angle_lines(N->ax, (const double[3]){d[0], d[1], d[2]});
            /* angle between d and a normal line: within [phi - rho, phi + rho]; |cos| of the angle between d
               and the plane's normal */
            const double cbmin = cos(fmin(phi + N->rho, M_PI / 2)), cbmax = cos(fmax(phi - N->rho, 0.0));
            if (cbmin >= C1) {
                const double pad = (20.11 * u * (N->E + 2 * S) * N->g / C1 + 6.21 * u * N->E + u * S) * 1.01 + 1e-12;
                const double dt = 10.06 * u * S * N->g / C1 * 1.01, t_hi = D * (1 + 10.06 * u * N->g / C1) * 1.01 + dt;
                double tn = -dt, tf = t_hi;
                for (int i = 0; i < 3; i++) {
                    const double lo = N->lo[i] - pad - o[i], hi = N->hi[i] + pad - o[i];
                    if (d[i] == 0) {
                        if (lo > 0 || hi < 0) tn = INFINITY;
                        continue;
                    }
                    double a = lo / d[i], b = hi / d[i];
                    if (a > b) {
                        const double t = a;
                        a = b;
                        b = t;
                    }
                    tn = fmax(tn, a);
                    tf = fmin(tf, b);
                }
                skip = tn > tf;
            } else {
                const double po = N->ax[0] * o[0] + N->ax[1] * o[1] + N->ax[2] * o[2];
                const double dista = fmax(0.0, fmax(po - pmax, pmin - po));
                const double eps = 10.1 * u * N->g * (D + S) + 1e-9;
                skip = dista - sin(N->rho) * R > D * cbmax * 1.001 + eps;
            }
        }
        if (!skip) {
            if (N->count) {
                c[2]++;
                for (uint32_t j = N->first; j < N->first + N->count; j++) {
                    const uint32_t id = B->ids[j];
                    if (id == excl) continue;
                    c[1]++;
                    float t;
                    if (mt(o, d, B->pos + 9 * (size_t)id, D, &t)) return 1;
                }
            } else {
                stk[sp++] = N->left + 1;
                n = N->left;
                continue;
            }
        }
        if (!sp) return 0;
        n = stk[--sp];
    }
}

void census(uint32_t nn, const uint32_t *is_leaf, const uint32_t *axis, const float *split, const uint32_t *child,
            const uint32_t *first, const uint32_t *count, const uint32_t *refs, const float *box, const float *pos,
            uint32_t ntris, uint32_t nr, const float *orig, const float *dir, const float *dist, const uint32_t *excl,
            uint64_t *out, uint32_t *bvh_nodes) {
    (void)nn;
    Kd T = {is_leaf, axis, child, first, count, refs, split, pos};
    Bvh B = {0};
    B.pos = pos;
    B.ids = (uint32_t *)malloc(sizeof(uint32_t) * ntris);
    B.cen = (float *)malloc(sizeof(float) * 3 * (size_t)ntris);
    for (uint32_t t = 0; t < ntris; t++) {
        B.ids[t] = t;
        for (int i = 0; i < 3; i++) B.cen[3 * (size_t)t + i] = (pos[9 * (size_t)t + i] + pos[9 * (size_t)t + 3 + i] +
                                                                pos[9 * (size_t)t + 6 + i]) / 3.f;
    }
    bvh_alloc(&B);
    bvh_build(&B, 0, 0, ntris);
    bvh_cones(&B, 0);
    *bvh_nodes = B.nn;
    memset(out, 0, sizeof(uint64_t) * S_N);
#pragma omp parallel
    {
        uint64_t st[S_N] = {0};
#pragma omp for schedule(dynamic, 256)
        for (uint32_t r = 0; r < nr; r++) {
            const float *o = orig + 3 * (size_t)r, *d = dir + 3 * (size_t)r;
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
            st[S_QUERIES]++;
            int occ = 0;
            uint64_t kc[3] = {0, 0, 0}, bc[3] = {0, 0, 0};
            if (!(tmax < 0 || tmax < tmin) && !(tmin > dist[r])) {
                tmax = dist[r] < tmax ? dist[r] : tmax;
                occ = kd_node(&T, 0, o, d, tmin, tmax, excl[r], kc);
            }
            const int found = bvh_any(&B, o, d, dist[r], excl[r], bc);
            st[S_KD_OCC] += occ;
            st[S_KD_LEAVES] += kc[0];
            st[S_KD_TESTS] += kc[1];
            st[S_KD_INNER] += kc[2];
            st[S_BVH_FOUND] += found;
            st[S_BVH_NODES] += bc[0];
            st[S_BVH_TESTS] += bc[1];
            st[S_BVH_LEAVES] += bc[2];
            if (occ) {
                st[S_BVH_OCC_NODES] += bc[0];
                st[S_BVH_OCC_TESTS] += bc[1];
                st[S_KD_OCC_INNER] += kc[2];
                st[S_KD_OCC_LEAVES] += kc[0];
                st[S_KD_OCC_TESTS] += kc[1];
            } else {
                st[S_BVH_VIS_NODES] += bc[0];
                st[S_BVH_VIS_TESTS] += bc[1];
                st[S_KD_VIS_INNER] += kc[2];
                st[S_KD_VIS_LEAVES] += kc[0];
                st[S_KD_VIS_TESTS] += kc[1];
            }
            uint64_t pc[3] = {0, 0, 0};
            const int pfound = bvh_proof(&B, o, d, dist[r], excl[r], pc);
            st[S_PR_FOUND] += pfound;
            st[S_PR_NODES] += pc[0];
            st[S_PR_TESTS] += pc[1];
            if (!occ) {
                st[S_PR_VIS_NODES] += pc[0];
                st[S_PR_VIS_TESTS] += pc[1];
            }
            st[S_PR_MISS] += occ && !pfound; /* must be 0 */
            st[S_MISMATCH_FOUND] += found && !occ; /* BVH found, kd VISIBLE: the kd answer rules */
            st[S_MISMATCH_OCC] += occ && !found;   /* must be 0: the BVH proof would be wrong */
        }
#pragma omp critical
        for (int i = 0; i < S_N; i++) out[i] += st[i];
    }
    free(B.n);
    free(B.ids);
    free(B.cen);
}
