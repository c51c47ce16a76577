// leafcull_check.cpp -- CPU check of the leaf cull records (csrc/leafcull.hpp): a
// reference that leaf_cull_mask drops must be one whose Moller-Trumbore test REJECTS
// for that ray and segment (otherwise skipping it would change a result).
//
// Built by tests/test_leafcull.py with g++ -O2 -ffp-contract=off (the kernels' float
// semantics).  Leaves of up to 32 triangles are random and adversarial: coplanar walls,
// axis-aligned boxes, fans around a point (column-like normal spreads), slivers, tiny and
// huge triangles, degenerate ones.  Rays have unit directions (normalised as glm does)
// and start anywhere in the scene box, next to the triangles, on their planes, and aim at
// points on their edges and vertices (a few ulps off), along grazing directions (d in
// the plane up to 1e-9 ... 1e-1), axis-parallel from a vertex's coordinate planes, with tmax random or a few ulps around the hit distance.
// The kernels compute inv = v_rcp_f32(d) (1 ulp); the check perturbs inv by up to 2 ulp.
//   leafcull_check <seed> <leaves> [form: 0 per-ray, 1 fixed-pad, 2 packed, 3 compressed, 4 short]   prints "violations N tested M accepted A skipped K"
#include "leafcull.hpp"

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace {

struct V {
    float x, y, z;
};
V sub(V a, V b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
V add(V a, V b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
V muls(V a, float s) { return {a.x * s, a.y * s, a.z * s}; }
float dot(V a, V b) {
    const float x = a.x * b.x, y = a.y * b.y, z = a.z * b.z;
    return (x + y) + z;
}
V cross(V a, V b) { return {a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y}; }
V normalize(V v) { return muls(v, 1.f / sqrtf(dot(v, v))); } // glm: v * inversesqrt(dot(v, v))

// kdtree.cpp:219-246 / 293-320 as the kernels evaluate it (tri_test, render_common.hpp)
bool mt(V o, V d, V A, V e1, V e2, float tmax) {
    const V p = cross(d, e2);
    const float a = dot(e1, p);
    if (a < 1.19209290e-7F && a > -1.19209290e-7F) return false;
    const float f = 1.f / a;
    const V s = sub(o, A);
    const float u = f * dot(s, p);
    if (u < 0.f || u > 1.f) return false;
    const V q = cross(s, e1);
    const float v = f * dot(d, q);
    if (v < 0.f || v + u > 1.f) return false;
    const float t = f * dot(e2, q);
    return t >= 0.f && t < tmax;
}
float tri_t(V o, V d, V A, V e1, V e2) { // the test's t (for tmax near it)
    const V p = cross(d, e2);
    const float f = 1.f / dot(e1, p);
    const V q = cross(sub(o, A), e1);
    return f * dot(e2, q);
}

uint64_t rs = 88172645463325252ull;
double rnd() {
    rs ^= rs << 13;
    rs ^= rs >> 7;
    rs ^= rs << 17;
    return (double)(rs >> 11) * 0x1p-53;
}
double rr(double a, double b) { return a + (b - a) * rnd(); }
V rv(double s) { return {(float)rr(-s, s), (float)rr(-s, s), (float)rr(-s, s)}; }
V unit() {
    for (;;) {
        V v = rv(1.0);
        const float l = dot(v, v);
        if (l > 1e-4f && l <= 1.f) return normalize(v);
    }
}
float ulps(float x, int k) {
    for (int i = 0; i < (k < 0 ? -k : k); i++) x = nextafterf(x, k < 0 ? -INFINITY : INFINITY);
    return x;
}

// the compressed form's grid jitter: its own generator, so forms 2 and 3 see the same leaves and rays
uint64_t gs = 0x2545F4914F6CDD1Dull;
double grid_rnd() {
    gs = gs * 6364136223846793005ull + 1442695040888963407ull;
    return (double)(gs >> 11) * 0x1p-53;
}

struct Tri {
    V A, e1, e2;
};

// one random leaf: its triangles in list order
std::vector<Tri> make_leaf(double scale) {
    std::vector<Tri> t;
    const int kind = (int)(rnd() * 7);
    const int n = 1 + (int)(rnd() * 32);
    const V c = rv(scale);
    auto tri = [&](V a, V b, V cc) { t.push_back(Tri{a, sub(b, a), sub(cc, a)}); };
    for (int i = 0; i < n; i++) {
        const double s = scale * pow(10.0, rr(-4, 0));
        switch (kind) {
        case 0: { // random
            const V a = add(c, rv(s));
            tri(a, add(a, rv(s)), add(a, rv(s)));
            break;
        }
        case 1: { // a wall: coplanar, axis-aligned normal
            const int ax = (int)(rnd() * 3);
            V a = add(c, rv(s)), b = add(c, rv(s)), cc = add(c, rv(s));
            float *pa = &a.x, *pb = &b.x, *pc = &cc.x;
            pa[ax] = pb[ax] = pc[ax] = (&c.x)[ax];
            tri(a, b, cc);
            break;
        }
        case 2: { // a box's faces: two or three orientations
            const int ax = i % 3;
            V a = add(c, rv(s)), b = add(c, rv(s)), cc = add(c, rv(s));
            float *pa = &a.x, *pb = &b.x, *pc = &cc.x;
            const float w = (&c.x)[ax] + (float)((i & 1) ? s : -s);
            pa[ax] = pb[ax] = pc[ax] = w;
            tri(a, b, cc);
            break;
        }
        case 3: { // a fan around an axis (column): normals spread over a great circle
            const double ang = rr(0, 6.283185307), ang2 = ang + rr(0.05, 0.6);
            const V a = add(c, V{(float)(s * cos(ang)), (float)rr(-s, s), (float)(s * sin(ang))});
            const V b = add(c, V{(float)(s * cos(ang2)), (float)rr(-s, s), (float)(s * sin(ang2))});
            const V cc = add(b, V{0.f, (float)rr(-s, s), 0.f});
            tri(a, b, cc);
            break;
        }
        case 4: { // slivers and near-degenerate
            const V a = add(c, rv(s)), dir = rv(s);
            const V b = add(a, dir);
            const V cc = add(a, add(muls(dir, (float)rr(-2, 2)), rv(s * pow(10.0, rr(-9, -2)))));
            tri(a, b, cc);
            break;
        }
        case 5: { // exactly degenerate (collinear / repeated vertices) mixed with random
            const V a = add(c, rv(s)), b = add(a, rv(s));
            if (i & 1) tri(a, b, add(a, muls(sub(b, a), 2.f)));
            else tri(a, b, add(a, rv(s)));
            break;
        }
        default: { // coplanar, arbitrary orientation
            static V nrm;
            if (i == 0) nrm = unit();
            V a = add(c, rv(s)), b = add(c, rv(s)), cc = add(c, rv(s));
            a = sub(a, muls(nrm, dot(sub(a, c), nrm)));
            b = sub(b, muls(nrm, dot(sub(b, c), nrm)));
            cc = sub(cc, muls(nrm, dot(sub(cc, c), nrm)));
            tri(a, b, cc);
            break;
        }
        }
    }
    return t;
}

} // namespace

int main(int argc, char **argv) {
    const uint64_t seed = argc > 1 ? strtoull(argv[1], 0, 10) : 1;
    const int leaves = argc > 2 ? atoi(argv[2]) : 1000;
    rs ^= seed * 0x9E3779B97F4A7C15ull;
    for (int i = 0; i < 10; i++) rnd();
    uint64_t viol = 0, tested = 0, accepted = 0, skipped = 0;
    const int form = argc > 3 ? atoi(argv[3]) : 0; // 1: fixed-pad records (leaf_cull_fixed), 2: packed, 3: compressed, 4: short
    for (int L = 0; L < leaves; L++) {
        const double scale = pow(10.0, rr(-2, 3.5));
        const std::vector<Tri> t = make_leaf(scale);
        const uint32_t n = (uint32_t)t.size();
        float A[32][3], e1[32][3], e2[32][3];
        for (uint32_t j = 0; j < n; j++) {
            std::memcpy(A[j], &t[j].A, 12);
            std::memcpy(e1[j], &t[j].e1, 12);
            std::memcpy(e2[j], &t[j].e2, 12);
        }
        cr::LcFloat4 rec[cr::LC_REC];
        cr::leaf_cull_record(A, e1, e2, n, rec);
        float db_leaf = 1.f;
        for (uint32_t j = 0; j < n; j++)
            for (int i = 0; i < 3; i++)
                db_leaf = std::fmax(db_leaf, 1.01f * std::fmax(std::fabs(A[j][i]),
                                                               std::fmax(std::fabs(A[j][i] + e1[j][i]), std::fabs(A[j][i] + e2[j][i]))));
        for (int r = 0; r < 400; r++) {
            const Tri &T = t[(size_t)(rnd() * n)];
            V o, d;
            const int rk = (int)(rnd() * 8);
            const V edge_pt = add(T.A, add(muls(T.e1, (float)rnd()), muls(T.e2, (float)(rnd() * 0.2))));
            const V vtx = rnd() < 0.5 ? T.A : add(T.A, rnd() < 0.5 ? T.e1 : T.e2);
            const V nrm = normalize(cross(T.e1, T.e2));
            const bool nrm_ok = nrm.x == nrm.x;
            const V target = rk == 1 ? add(vtx, rv(scale * 1e-7)) : edge_pt;
            switch (rk) {
            case 0: // anywhere
                o = rv(scale * 4);
                d = unit();
                break;
            case 1:
            case 2: // at an edge / vertex point from anywhere
                o = add(target, muls(unit(), (float)(scale * pow(10.0, rr(-6, 0.5)))));
                d = normalize(sub(target, o));
                break;
            case 3: // from the triangle's plane (offset as sendRay's 0.001 n), outward
                o = add(edge_pt, muls(nrm_ok ? nrm : unit(), (float)(scale * pow(10.0, rr(-9, -2)))));
                d = unit();
                break;
            case 4: { // grazing: in the plane up to a small normal part
                const V inpl = normalize(cross(nrm_ok ? nrm : unit(), unit()));
                o = add(add(target, muls(inpl, (float)(-scale * rr(0.01, 3)))),
                        muls(nrm_ok ? nrm : unit(), (float)(scale * pow(10.0, rr(-10, -3)))));
                const V dd = add(inpl, muls(nrm_ok ? nrm : unit(), (float)(rr(-1, 1) * pow(10.0, rr(-9, -1)))));
                d = normalize(dd);
                break;
            }
            case 5: { // in the plane (up to 1e-12 .. 1e-4 of its scale), far to the side: where the
                      // test's rounding can accept nowhere near the triangle
                const V inpl = normalize(cross(nrm_ok ? nrm : unit(), unit()));
                const V side = normalize(cross(nrm_ok ? nrm : unit(), inpl));
                o = add(add(target, muls(side, (float)(scale * rr(-1e3, 1e3)))),
                        add(muls(inpl, (float)(-scale * rr(1, 1e3))),
                            muls(nrm_ok ? nrm : unit(), (float)(scale * pow(10.0, rr(-12, -4))))));
                d = rnd() < 0.5 ? inpl : normalize(add(inpl, muls(nrm_ok ? nrm : unit(), (float)(rr(-1, 1) * pow(10.0, rr(-12, -5))))));
                break;
            }
            case 7: { // axis-parallel (a zero direction component: inv infinite) from a vertex's coordinate planes
                o = add(target, rv(scale * 2));
                d = normalize(sub(target, o));
                const int z = (int)(rnd() * 3);
                (&d.x)[z] = 0.f;
                if (rnd() < 0.3) (&d.x)[(z + 1) % 3] = 0.f;
                d = normalize(d);
                (&o.x)[z] = (&vtx.x)[z];
                break;
            }
            default: // other triangles of the leaf behind / in front
                o = add(T.A, rv(scale * 2));
                d = normalize(sub(target, o));
                break;
            }
            if (!(d.x == d.x) || !cr::lc_unit(d.x, d.y, d.z)) continue;
            float tmax;
            const double pick = rnd();
            if (pick < 0.4) tmax = (float)(scale * pow(10.0, rr(-3, 1.5)));
            else if (pick < 0.5) tmax = INFINITY;
            else {
                const float th = tri_t(o, d, T.A, T.e1, T.e2);
                tmax = (th == th && std::fabs(th) < 1e30f) ? ulps(std::fabs(th), (int)(rnd() * 9) - 3) : 1.f;
            }
            const float ov[3] = {o.x, o.y, o.z}, dv[3] = {d.x, d.y, d.z};
            // db bounds every coordinate of the scene (origins and vertices), as the kernels' args.db
            const float db = std::fmax(db_leaf, 1.01f * std::fmax(std::fabs(o.x), std::fmax(std::fabs(o.y), std::fabs(o.z))));
            float inv[3];
            for (int i = 0; i < 3; i++) inv[i] = ulps(1.f / dv[i], (int)(rnd() * 5) - 2); // v_rcp_f32: within 1 ulp
            uint32_t keep;
            if (form) { // the scene constants this ray satisfies: |o|, |vertex| <= db, |o_i - v_i| <= smax
                double smax = 0;
                for (uint32_t j = 0; j < n; j++)
                    for (int i = 0; i < 3; i++) {
                        const double v[3] = {A[j][i], (double)A[j][i] + e1[j][i], (double)A[j][i] + e2[j][i]};
                        for (double x : v) smax = std::fmax(smax, std::fabs((double)ov[i] - x));
                    }
                cr::LcFloat4 fr[cr::LC_REC];
                cr::leaf_cull_fixed(rec, db, smax, fr);
                if (form >= 3) { // compressed: the leaf's boxes on a scene grid up to 1000x the leaf's scale wider
                    cr::LcFloat4 two[2 * cr::LC_REC];
                    for (int i = 0; i < cr::LC_REC; i++) two[i] = two[cr::LC_REC + i] = fr[i];
                    const double ext = scale * pow(10.0, grid_rnd() * 6 - 3);
                    for (int i = 0; i < 3; i++) {
                        (&two[cr::LC_REC].x)[i] = (float)((&fr[0].x)[i] - ext * grid_rnd());
                        (&two[cr::LC_REC + 1].x)[i] = (float)((&fr[1].x)[i] + ext * grid_rnd());
                    }
                    const uint32_t one = 1u;
                    std::memcpy(&two[cr::LC_REC + 6].x, &one, 4);
                    cr::LcGrid G = cr::lc_grid_make(two, 2, db);
                    if (form == 4) { // short: 32 B, the dt unit from the leaf's groups
                        cr::lc_grid_dt(G, fr, 1);
                        uint32_t w[8];
                        cr::leaf_cull_compress_s(rec, fr, n, G, w);
                        keep = cr::leaf_cull_mask_s(ov, dv, inv, true, tmax, w, n, G);
                    } else {
                        uint32_t w[12];
                        cr::leaf_cull_compress(rec, fr, n, G, w);
                        keep = cr::leaf_cull_mask_c(ov, dv, inv, true, tmax, w, n, G);
                    }
                } else if (form == 2) {
                    cr::LcFloat4 pr[cr::LC_RECP];
                    cr::leaf_cull_pack(fr, n, pr);
                    keep = cr::leaf_cull_mask_packed(ov, dv, inv, true, tmax, pr, n);
                } else {
                    keep = cr::leaf_cull_mask_fixed(ov, dv, inv, true, tmax, fr, n);
                }
            } else {
                keep = cr::leaf_cull_mask(ov, dv, inv, true, tmax, db, rec, n);
            }
            for (uint32_t j = 0; j < n; j++) {
                tested++;
                const bool acc = mt(o, d, t[j].A, t[j].e1, t[j].e2, tmax);
                accepted += acc;
                if (!((keep >> j) & 1u)) {
                    skipped++;
                    if (acc) {
                        viol++;
                        if (viol <= 5)
                            fprintf(stderr, "violation: leaf %d ray kind %d tri %u o (%g %g %g) d (%.9g %.9g %.9g) tmax %g\n",
                                    L, rk, j, o.x, o.y, o.z, d.x, d.y, d.z, tmax);
                    }
                }
            }
        }
    }
    printf("violations %llu tested %llu accepted %llu skipped %llu\n", (unsigned long long)viol,
           (unsigned long long)tested, (unsigned long long)accepted, (unsigned long long)skipped);
    return 0;
}
