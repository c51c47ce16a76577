/* rope_census.c -- CPU census (diagnostic only) of an exact rope traversal of the reference's kd tree.
 *
 * The reference's recursion (src/kdtree.cpp:248-281, 322-344) visits a leaf L with the interval
 * (lo, hi): lo = max(t0, tau of the ancestor planes L lies beyond), hi = min(T, tau >= 0 of the ancestor
 * planes L lies before), tau = (split - o[a]) / d[a] (the same float expression for every use of a plane),
 * "before / beyond" from the origin's side (belowFirst).  Per axis tau is monotone in the split position,
 * so these are the leaf's own faces: for a ray with every d[a] != 0, whose origin lies on no split plane
 * of the tree (o[a] != every split of axis a; then tau of a plane through the origin would be +-0 and the
 * recursion would take the side against the ray's travel), the leaves the recursion visits are the leaves
 * the ray's "tau clock" passes through, in order, and hi(L) = min(T, tau of L's exit faces).  The next
 * leaf after L is the one holding hi(L)+: across L's unique exit face (a rope to the deepest node holding
 * that whole face), then down, choosing at each node the side the clock is on just after hi(L) (crossed:
 * 0 <= tau <= hi(L)).  Two exit faces with the same tau (an edge or corner crossing) restart the descent
 * from the root with that rule, which is exact too; rays outside the conditions fall back to the recursion.
 *
 * The census checks, per query, that the rope walk visits the same (leaf, hi bits) sequence and gives
 * the same answer as the recursion, and counts the work of both.  Built by scripts/rope_census.py. */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

enum {
    C_QUERIES, C_ANSWER_TRUE, C_REC_INNER, C_REC_LEAVES, C_REC_TESTS, C_ROPE_QUERIES, C_FALLBACK_ZERO_DIR,
    C_FALLBACK_ON_SPLIT, C_FALLBACK_T0, C_LOCATE_STEPS, C_ROPE_LEAVES, C_EXIT_DIVS, C_EXIT_DIVS_NOCACHE,
    C_ROPE_DESC, C_RESTARTS, C_RESTART_STEPS, C_MISMATCH_SEQ, C_MISMATCH_ANS, C_REC_INNER_ROPED,
    C_REC_LEAVES_ROPED, C_VIS_QUERIES, C_VIS_REC_INNER, C_VIS_ROPE_WORK, C_FROM_HIT_LEAF, C_REC_FETCH,
    C_ROPE_FETCH, C_ROPE_REC, C_VIS_REC_FETCH, C_VIS_ROPE_FETCH, C_VIS_ROPE_DIVS, C_REC_FETCH_ROPED, C_N
};

#define NONE 0xffffffffu
#define MAXSEQ 4096

typedef struct {
    const uint32_t *is_leaf, *axis, *child, *first, *count, *refs;
    const float *split, *pos;
    float *lo, *hi;   /* [n][3] cell boxes */
    uint32_t *rope;   /* [n][6]: faces -x, +x, -y, +y, -z, +z (NONE: the scene box) */
    float *sorted[3]; /* the split positions of each axis, sorted */
    uint32_t nsorted[3];
} Kd;

/* kdtree.cpp:219-246 / 293-320 (float, no contraction); closest: *tout = t on accept */
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
    *tout = t;
    return t >= 0.f && t < tmax;
}

typedef struct {
    uint32_t leaf[MAXSEQ];
    uint32_t hib[MAXSEQ];
    int n, over;
} Seq;
static void seq_add(Seq *s, uint32_t leaf, float hi) {
    if (s->n < MAXSEQ) {
        s->leaf[s->n] = leaf;
        memcpy(&s->hib[s->n], &hi, 4);
        s->n++;
    } else {
        s->over = 1;
    }
}

/* one leaf's test with interval end hi: 1 = the query ends here (occluded / closest hit found) */
static int leaf_test(const Kd *T, uint32_t n, const float o[3], const float d[3], float hi, int shadow,
                     uint32_t excl, uint64_t *tests) {
    int ret = 0;
    float tmax = hi;
    for (uint32_t j = 0; j < T->count[n]; j++) {
        const uint32_t id = T->refs[T->first[n] + j];
        if (shadow && id == excl) continue;
        (*tests)++;
        float t;
        if (mt(o, d, T->pos + 9 * (size_t)id, tmax, &t)) {
            if (shadow) return 1;
            tmax = t;
            ret = 1;
        }
    }
    return ret;
}

/* the reference's recursion (near child first), recording (leaf, tmax bits) */
/* seg: inner steps of the current descent segment (a fat record per two levels: 1 + seg / 2 fetches) */
static int rec_node(const Kd *T, uint32_t n, const float o[3], const float d[3], float tmin, float tmax, int shadow,
                    uint32_t excl, uint64_t *c, Seq *sq, uint32_t seg) {
    if (T->is_leaf[n]) {
        c[C_REC_FETCH] += 1 + seg / 2;
        c[C_REC_LEAVES]++;
        seq_add(sq, n, tmax);
        return leaf_test(T, n, o, d, tmax, shadow, excl, &c[C_REC_TESTS]);
    }
    c[C_REC_INNER]++;
    const uint32_t a = T->axis[n];
    const float sp = T->split[n];
    const float ts = (sp - o[a]) / d[a];
    const uint32_t below = (o[a] < sp) || (o[a] == sp && d[a] <= 0);
    const uint32_t ch = T->child[n];
    if (ts >= tmax || ts < 0) return rec_node(T, ch + (1 - below), o, d, tmin, tmax, shadow, excl, c, sq, seg + 1);
    if (ts <= tmin) return rec_node(T, ch + below, o, d, tmin, tmax, shadow, excl, c, sq, seg + 1);
    return rec_node(T, ch + (1 - below), o, d, tmin, ts, shadow, excl, c, sq, seg + 1) ||
           rec_node(T, ch + below, o, d, ts, tmax, shadow, excl, c, sq, 0); /* (popped: a new segment) */
}

static int on_split(const Kd *T, const float o[3]) {
    for (int a = 0; a < 3; a++) {
        const float *s = T->sorted[a];
        uint32_t lo = 0, hi = T->nsorted[a];
        while (lo < hi) {
            const uint32_t m = (lo + hi) / 2;
            if (s[m] < o[a]) lo = m + 1;
            else hi = m;
        }
        if (lo < T->nsorted[a] && s[lo] == o[a]) return 1;
    }
    return 0;
}

/* descend from node n to the leaf holding the clock just after tb (0 <= tau <= tb: crossed) */
static uint32_t descend(const Kd *T, uint32_t n, const float o[3], const float d[3], float tb, uint64_t *steps) {
    while (!T->is_leaf[n]) {
        (*steps)++;
        const uint32_t a = T->axis[n];
        const float sp = T->split[n];
        const float ts = (sp - o[a]) / d[a];
        const uint32_t below = o[a] < sp; /* (no split holds o[a]) */
        const int crossed = ts >= 0.f && ts <= tb;
        n = T->child[n] + (crossed ? below : 1u - below);
    }
    return n;
}

/* the rope walk; returns the answer, -1 when the ray falls back to the recursion */
/* work: divisions; fetch[0]: node-record fetches (fat, two levels each), fetch[1]: leaf rope records */
static int rope_walk(const Kd *T, const float o[3], const float d[3], float t0, float Tend, int shadow, uint32_t excl,
                     uint32_t start_leaf, uint64_t *c, Seq *sq, uint64_t *work, uint64_t *fetch) {
    for (int a = 0; a < 3; a++)
        if (d[a] == 0.f || !isfinite(1.f / d[a])) {
            c[C_FALLBACK_ZERO_DIR]++;
            return -1;
        }
    if (!(t0 < 0.f)) {
        c[C_FALLBACK_T0]++;
        return -1;
    }
    if (on_split(T, o)) {
        c[C_FALLBACK_ON_SPLIT]++;
        return -1;
    }
    c[C_ROPE_QUERIES]++;
    uint32_t n = 0;
    /* the first leaf: the origin's (the clock just after t0 < 0 is on the origin's side of every plane) */
    if (start_leaf != NONE) {
        const float *lo = T->lo + 3 * (size_t)start_leaf, *hi = T->hi + 3 * (size_t)start_leaf;
        int in = 1;
        for (int a = 0; a < 3; a++) in &= (o[a] > lo[a] || lo[a] == T->lo[a]) && (o[a] < hi[a] || hi[a] == T->hi[a]);
        /* (a face on the scene box does not bound the point location; a split face must hold o strictly) */
        if (in) {
            n = start_leaf;
            c[C_FROM_HIT_LEAF]++;
        }
    }
    if (n == 0) {
        uint32_t k = 0;
        while (!T->is_leaf[n]) {
            c[C_LOCATE_STEPS]++;
            k++;
            n = T->child[n] + (o[T->axis[n]] < T->split[n] ? 0u : 1u);
        }
        fetch[0] += 1 + k / 2;
    }
    /* the exit-face cache: per axis the last plane position and its tau */
    float cpos[3] = {NAN, NAN, NAN}, ctau[3] = {0, 0, 0};
    for (;;) {
        c[C_ROPE_LEAVES]++;
        fetch[1]++;
        const float *lo = T->lo + 3 * (size_t)n, *hi = T->hi + 3 * (size_t)n;
        float tx[3];
        int face[3];
        for (int a = 0; a < 3; a++) {
            face[a] = 2 * a + (d[a] > 0.f);
            const float s = d[a] > 0.f ? hi[a] : lo[a];
            const int boxface = T->rope[6 * (size_t)n + face[a]] == NONE;
            if (boxface) {
                tx[a] = INFINITY;
                continue;
            }
            c[C_EXIT_DIVS_NOCACHE]++;
            if (s == cpos[a]) {
                tx[a] = ctau[a];
            } else {
                c[C_EXIT_DIVS]++;
                (*work)++;
                tx[a] = (s - o[a]) / d[a];
                cpos[a] = s;
                ctau[a] = tx[a];
            }
        }
        float h = Tend;
        int am = -1;
        for (int a = 0; a < 3; a++)
            if (tx[a] < h) {
                h = tx[a];
                am = a;
            }
        seq_add(sq, n, h);
        uint64_t tests = 0;
        if (leaf_test(T, n, o, d, h, shadow, excl, &tests)) return 1;
        if (am < 0) return 0; /* hi = T: the last leaf */
        int ties = 0;
        for (int a = 0; a < 3; a++) ties += tx[a] == h;
        uint32_t r;
        if (ties > 1) {
            c[C_RESTARTS]++;
            uint64_t st = 0;
            r = descend(T, 0, o, d, h, &st);
            c[C_RESTART_STEPS] += st;
            *work += st;
            fetch[0] += 1 + st / 2;
        } else {
            uint64_t st = 0;
            const uint32_t rt = T->rope[6 * (size_t)n + face[am]];
            r = descend(T, rt, o, d, h, &st);
            c[C_ROPE_DESC] += st;
            *work += st;
            /* a rope to a leaf: its (first, count) ride in the rope record, no node fetch */
            if (!T->is_leaf[rt]) fetch[0] += 1 + st / 2;
        }
        n = r;
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

static int cmpf(const void *a, const void *b) {
    const float x = *(const float *)a, y = *(const float *)b;
    return x < y ? -1 : x > y;
}

/* cell boxes and optimized ropes of every node (Havran's ropes, pushed down to the deepest node that holds
 * the whole face; a split on the face's own axis at the face's position holds the face on its far side) */
static void build(Kd *T, uint32_t nn, const float *box) {
    uint32_t *stack = malloc(sizeof(uint32_t) * (nn + 1));
    int sp = 0;
    memcpy(T->lo, box, 12);
    memcpy(T->hi, box + 3, 12);
    for (int f = 0; f < 6; f++) T->rope[f] = NONE;
    stack[sp++] = 0;
    while (sp) {
        const uint32_t n = stack[--sp];
        if (T->is_leaf[n]) continue;
        const uint32_t a = T->axis[n], c0 = T->child[n], c1 = c0 + 1;
        memcpy(T->lo + 3 * (size_t)c0, T->lo + 3 * (size_t)n, 12);
        memcpy(T->hi + 3 * (size_t)c0, T->hi + 3 * (size_t)n, 12);
        memcpy(T->lo + 3 * (size_t)c1, T->lo + 3 * (size_t)n, 12);
        memcpy(T->hi + 3 * (size_t)c1, T->hi + 3 * (size_t)n, 12);
        T->hi[3 * (size_t)c0 + a] = T->split[n];
        T->lo[3 * (size_t)c1 + a] = T->split[n];
        memcpy(T->rope + 6 * (size_t)c0, T->rope + 6 * (size_t)n, 24);
        memcpy(T->rope + 6 * (size_t)c1, T->rope + 6 * (size_t)n, 24);
        T->rope[6 * (size_t)c0 + 2 * a + 1] = c1;
        T->rope[6 * (size_t)c1 + 2 * a] = c0;
        stack[sp++] = c0;
        stack[sp++] = c1;
    }
    free(stack);
    for (uint32_t n = 0; n < nn; n++) {
        if (!T->is_leaf[n]) continue;
        const float *lo = T->lo + 3 * (size_t)n, *hi = T->hi + 3 * (size_t)n;
        for (int f = 0; f < 6; f++) {
            uint32_t r = T->rope[6 * (size_t)n + f];
            const int fa = f / 2, plus = f & 1;
            const float fpos = plus ? hi[fa] : lo[fa];
            while (r != NONE && !T->is_leaf[r]) {
                const uint32_t b = T->axis[r];
                const float s = T->split[r];
                if ((int)b == fa) { /* the child touching the face (a zero-width one: the other) */
                    if (plus) r = T->child[r] + (s > fpos ? 0u : 1u);
                    else r = T->child[r] + (s < fpos ? 1u : 0u);
                } else if (s <= lo[b]) {
                    r = T->child[r] + 1;
                } else if (s >= hi[b]) {
                    r = T->child[r];
                } else {
                    break;
                }
            }
            T->rope[6 * (size_t)n + f] = r;
        }
    }
}

typedef struct {
    Kd T;
} Ctx;

/* queries in the given order; start: per query a leaf hint (NONE: point location) */
void census(const uint32_t *is_leaf, const uint32_t *axis, const float *split, const uint32_t *child,
            const uint32_t *first, const uint32_t *count, const uint32_t *refs, const float *box, const float *pos,
            uint32_t nn, uint32_t nq, const float *o, const float *d, const float *dist, const uint32_t *excl,
            const uint32_t *start, int shadow, uint64_t *stats) {
    Kd T = {is_leaf, axis, child, first, count, refs, split, pos, NULL, NULL, NULL, {0}, {0}};
    T.lo = malloc(sizeof(float) * 3 * nn);
    T.hi = malloc(sizeof(float) * 3 * nn);
    T.rope = malloc(sizeof(uint32_t) * 6 * nn);
    build(&T, nn, box);
    for (int a = 0; a < 3; a++) {
        T.sorted[a] = malloc(sizeof(float) * nn);
        uint32_t k = 0;
        for (uint32_t n = 0; n < nn; n++)
            if (!is_leaf[n] && axis[n] == (uint32_t)a) T.sorted[a][k++] = split[n];
        qsort(T.sorted[a], k, sizeof(float), cmpf);
        T.nsorted[a] = k;
    }
    memset(stats, 0, sizeof(uint64_t) * C_N);
#pragma omp parallel
    {
        uint64_t c[C_N];
        memset(c, 0, sizeof c);
        Seq *s1 = malloc(sizeof(Seq)), *s2 = malloc(sizeof(Seq));
#pragma omp for schedule(dynamic, 256)
        for (uint32_t q = 0; q < nq; q++) {
            const float *oq = o + 3 * (size_t)q, *dq = d + 3 * (size_t)q;
            float t0, t1;
            ray_box(box, oq, dq, &t0, &t1);
            c[C_QUERIES]++;
            if (t1 < 0 || t1 < t0 || (shadow && t0 > dist[q])) continue;
            const float Tend = shadow ? fminf(t1, dist[q]) : t1;
            s1->n = s2->n = 0;
            s1->over = s2->over = 0;
            const uint64_t in0 = c[C_REC_INNER], lv0 = c[C_REC_LEAVES], f0 = c[C_REC_FETCH];
            const int ref = rec_node(&T, 0, oq, dq, t0, Tend, shadow, shadow ? excl[q] : 0, c, s1, 0);
            c[C_ANSWER_TRUE] += ref;
            uint64_t work = 0, fetch[2] = {0, 0};
            const int got = rope_walk(&T, oq, dq, t0, Tend, shadow, shadow ? excl[q] : 0, start ? start[q] : NONE, c,
                                      s2, &work, fetch);
            if (got < 0) continue;
            c[C_REC_INNER_ROPED] += c[C_REC_INNER] - in0;
            c[C_REC_LEAVES_ROPED] += c[C_REC_LEAVES] - lv0;
            c[C_REC_FETCH_ROPED] += c[C_REC_FETCH] - f0;
            c[C_ROPE_FETCH] += fetch[0];
            c[C_ROPE_REC] += fetch[1];
            if (!ref) {
                c[C_VIS_QUERIES]++;
                c[C_VIS_REC_INNER] += c[C_REC_INNER] - in0;
                c[C_VIS_REC_FETCH] += c[C_REC_FETCH] - f0;
                c[C_VIS_ROPE_WORK] += work;
                c[C_VIS_ROPE_FETCH] += fetch[0] + fetch[1];
            }
            c[C_MISMATCH_ANS] += got != ref;
            int same = s1->n == s2->n && !s1->over && !s2->over;
            for (int i = 0; same && i < s1->n; i++) same = s1->leaf[i] == s2->leaf[i] && s1->hib[i] == s2->hib[i];
            c[C_MISMATCH_SEQ] += !same;
        }
        free(s1);
        free(s2);
#pragma omp critical
        for (int i = 0; i < C_N; i++) stats[i] += c[i];
    }
    for (int a = 0; a < 3; a++) free(T.sorted[a]);
    free(T.lo);
    free(T.hi);
    free(T.rope);
}

/* the leaf holding each point (the closest trace's hit leaf, approximately: the leaf of the hit point) */
void locate(const uint32_t *is_leaf, const uint32_t *axis, const float *split, const uint32_t *child, uint32_t n,
            const float *p, uint32_t *leaf) {
#pragma omp parallel for
    for (uint32_t i = 0; i < n; i++) {
        uint32_t k = 0;
        while (!is_leaf[k]) k = child[k] + (p[3 * (size_t)i + axis[k]] < split[k] ? 0u : 1u);
        leaf[i] = k;
    }
}
