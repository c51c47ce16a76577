// planecull_check.cpp -- CPU check of plane_record (csrc/planecull.hpp): for rays with
// normalized directions inside the scene box, every (ray, tmax) the Moller-Trumbore
// test ACCEPTS (0 <= t < tmax) must pass the plane check the trace kernels apply
// before the test (otherwise skipping the test would change a result).
//
// Built by tests/test_camcull.py with g++ -O2 -ffp-contract=off.  Triangles of every
// size and shape (slivers, tiny, scene-sized), rays through them, nearly parallel to
// their plane, starting on or within a few ulps of the plane, tmax ending just past
// or just before the hit; directions normalized as glm::normalize does.
//   planecull_check <seed> <cases>   prints "violations N tested M accepted A skipped S"
#include "planecull.hpp"

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

namespace {

struct V {
    float x, y, z;
};
V sub(V a, V b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
V muls(V a, float s) { return {a.x * s, a.y * s, a.z * s}; }
float dot(V a, V b) {
    const float x = a.x * b.x, y = a.y * b.y, z = a.z * b.z;
    return (x + y) + z;
}
V cross(V a, V b) { return {a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y}; }
V normalize(V v) { return muls(v, 1.0f / sqrtf(dot(v, v))); }

// kdtree.cpp:219-246 / 293-320 with the segment end: accepted iff 0 <= t < tmax
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

// the kernels' plane check (traverse.hpp): true = skip the test
bool skip(const float r[4], V o, V d, float tmax) {
    const V N = {r[0], r[1], r[2]};
    const float s0 = dot(N, o) - r[3];
    const float s1 = s0 + tmax * dot(N, d);
    return (s0 > 1.f && s1 > 1.f) || (s0 < -1.f && s1 < -1.f);
}

uint64_t rs = 88172645463325252ull;
double rnd() {
    rs ^= rs << 13;
    rs ^= rs >> 7;
    rs ^= rs << 17;
    return (double)(rs >> 11) * 0x1p-53;
}
double rr(double a, double b) { return a + (b - a) * rnd(); }
float nudge(float x, int k) {
    for (int i = 0; i < k; i++) x = nextafterf(x, rnd() < 0.5 ? -INFINITY : INFINITY);
    return x;
}

} // namespace

int main(int argc, char **argv) {
    rs ^= (uint64_t)strtoull(argc > 1 ? argv[1] : "1", nullptr, 10) * 0x9E3779B97F4A7C15ull;
    const int cases = argc > 2 ? atoi(argv[2]) : 2000;
    long long viol = 0, tested = 0, accepted = 0, skipped = 0;
    for (int cs = 0; cs < cases; cs++) {
        const double box = pow(10.0, rr(-1, 4)); // scene box [-box, box]^3
        const double Db = box + 1.0, Tb = 2.0 * sqrt(3.0) * box * 1.01 + 2.0;
        const int kind = cs % 5;
        const double size = box * pow(10.0, rr(kind == 1 ? -7 : -4, 0));
        double P[3][3], c[3];
        for (int i = 0; i < 3; i++) c[i] = rr(-box, box) * 0.9;
        for (int v = 0; v < 3; v++)
            for (int i = 0; i < 3; i++) P[v][i] = c[i] + rr(-1, 1) * size;
        if (kind == 2) // sliver: vertex 2 close to the line of edge 0-1
            for (int i = 0; i < 3; i++) P[2][i] = P[0][i] + (P[1][i] - P[0][i]) * rr(0, 1) + rr(-1, 1) * size * 1e-5;
        const V A = {(float)P[0][0], (float)P[0][1], (float)P[0][2]};
        const V B = {(float)P[1][0], (float)P[1][1], (float)P[1][2]};
        const V C = {(float)P[2][0], (float)P[2][1], (float)P[2][2]};
        const V e1 = sub(B, A), e2 = sub(C, A);
        const float Af[3] = {A.x, A.y, A.z}, e1f[3] = {e1.x, e1.y, e1.z}, e2f[3] = {e2.x, e2.y, e2.z};
        float rec[4];
        cr::plane_record(Af, e1f, e2f, Db, Tb, rec);
        double n[3] = {(double)e1.y * e2.z - (double)e1.z * e2.y, (double)e1.z * e2.x - (double)e1.x * e2.z,
                       (double)e1.x * e2.y - (double)e1.y * e2.x};
        const double nl = sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
        for (int k = 0; k < 160; k++) {
            // a target point on / near the triangle, an origin in the box
            const double b0 = rr(-0.05, 1.05), b1 = rr(-0.05, 1.05) * (1 - b0);
            double X[3], O[3];
            for (int i = 0; i < 3; i++) X[i] = P[0][i] + (P[1][i] - P[0][i]) * b0 + (P[2][i] - P[0][i]) * b1;
            const int mode = k % 4;
            for (int i = 0; i < 3; i++) O[i] = mode == 1 ? X[i] + rr(-1, 1) * size * 3 : rr(-box, box);
            if ((mode == 1 || mode == 2) && nl > 0) { // origin near (1) / on (2) the plane
                double dd = 0;
                for (int i = 0; i < 3; i++) dd += (O[i] - P[0][i]) * n[i] / nl;
                const double off = mode == 1 ? rr(-1, 1) * pow(10.0, rr(-8, -2)) * size : 0.0;
                for (int i = 0; i < 3; i++) O[i] -= (dd - off) * n[i] / nl;
            }
            V o = {(float)O[0], (float)O[1], (float)O[2]};
            if (mode == 2) o = {nudge(o.x, (int)(rnd() * 4)), nudge(o.y, (int)(rnd() * 4)), nudge(o.z, (int)(rnd() * 4))};
            const bool inside = fabs(o.x) <= Db && fabs(o.y) <= Db && fabs(o.z) <= Db;
            const V dir = normalize(sub(V{(float)X[0], (float)X[1], (float)X[2]}, o));
            if (!(std::isfinite(dir.x) && std::isfinite(dir.y) && std::isfinite(dir.z)) || !inside) continue;
            const double dist = sqrt((X[0] - o.x) * (X[0] - o.x) + (X[1] - o.y) * (X[1] - o.y) + (X[2] - o.z) * (X[2] - o.z));
            // tmax around the hit distance, a few ulps either side, and long segments
            for (int j = 0; j < 6; j++) {
                float tmax = j < 3 ? nudge((float)dist, (int)(rnd() * 8)) : (float)rr(0, Tb * 0.999);
                if (j == 2) tmax = (float)(dist * rr(0.999, 1.001));
                if (!(tmax > 0 && tmax <= Tb)) continue;
                tested++;
                const bool sk = skip(rec, o, dir, tmax);
                skipped += sk;
                if (mt(o, dir, A, e1, e2, tmax)) {
                    accepted++;
                    if (sk) {
                        if (viol < 10)
                            fprintf(stderr, "VIOLATION case %d kind %d mode %d tmax %.9g dist %.9g\n", cs, kind, mode,
                                    tmax, dist);
                        viol++;
                    }
                }
            }
        }
    }
    printf("violations %lld tested %lld accepted %lld skipped %lld\n", viol, tested, accepted, skipped);
    return viol ? 1 : 0;
}
