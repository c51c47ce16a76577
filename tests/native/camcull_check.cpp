// camcull_check.cpp -- CPU check of cam_cull_box (csrc/camcull.hpp): for camera rays,
// every sample position at which Moller-Trumbore ACCEPTS must lie inside the
// triangle's cull box (otherwise skipping the test would change a result).
//
// Built by tests/test_camcull.py with g++ -O2 -ffp-contract=off (the kernels' and the
// oracle's float semantics: IEEE single, no FMA contraction).  Cameras and triangles
// are random and adversarial: triangles far and near, tiny and huge, viewed edge-on
// (the eye close to their plane), straddling the eye plane, behind the eye; samples
// uniform over the screen and concentrated on and around the projected edges and
// vertices, down to a few float ulps of the screen position.
//   camcull_check <seed> <cases>     prints "violations N tested M accepted A culled C"
#include "camcull.hpp"

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

using cr::CullCam;

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

// kdtree.cpp:219-246 as the kernels evaluate it (tri_test, render_common.hpp)
bool mt(V o, V d, V A, V e1, V e2) {
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
    return f * dot(e2, q) >= 0.f;
}

uint64_t rs = 88172645463325252ull;
double rnd() { // [0, 1)
    rs ^= rs << 13;
    rs ^= rs >> 7;
    rs ^= rs << 17;
    return (double)(rs >> 11) * 0x1p-53;
}
double rr(double a, double b) { return a + (b - a) * rnd(); }

// camera basis in the layout of RenderArgs::cam (eye, leftUpper, dx, dy), from a random
// eye / target / up and field of view (the construction only needs to be a valid affine map)
CullCam make_cam(double scale) {
    CullCam c;
    const double X = (double)(64 + (int)(rnd() * 2000)), Y = (double)(64 + (int)(rnd() * 1200));
    c.xres = (float)X;
    c.yres = (float)Y;
    double eye[3], f[3], up[3] = {rr(-0.2, 0.2), 1.0, rr(-0.2, 0.2)};
    for (int i = 0; i < 3; i++) eye[i] = rr(-scale, scale);
    double n = 0;
    for (int i = 0; i < 3; i++) {
        f[i] = rr(-1, 1);
        n += f[i] * f[i];
    }
    n = sqrt(n);
    for (int i = 0; i < 3; i++) f[i] /= n;
    double s[3] = {f[1] * up[2] - f[2] * up[1], f[2] * up[0] - f[0] * up[2], f[0] * up[1] - f[1] * up[0]};
    n = sqrt(s[0] * s[0] + s[1] * s[1] + s[2] * s[2]);
    for (int i = 0; i < 3; i++) s[i] /= n;
    double u[3] = {s[1] * f[2] - s[2] * f[1], s[2] * f[0] - s[0] * f[2], s[0] * f[1] - s[1] * f[0]};
    const double yv = rr(0.2, 1.5), xv = yv * X / Y;
    for (int i = 0; i < 3; i++) {
        c.cam[i] = (float)eye[i];
        c.cam[3 + i] = (float)(f[i] - xv * s[i] + yv * u[i]); // left upper
        c.cam[6 + i] = (float)(2 * xv * s[i] / X);
        c.cam[9 + i] = (float)(-2 * yv * u[i] / Y);
    }
    return c;
}

V camera_dir(const CullCam &c, float sx, float sy) {
    const V lu = {c.cam[3], c.cam[4], c.cam[5]}, dx = {c.cam[6], c.cam[7], c.cam[8]}, dy = {c.cam[9], c.cam[10], c.cam[11]};
    return add(add(lu, muls(dx, sx)), muls(dy, sy));
}

// screen position (double) of world point w seen from the eye; false if behind
bool project(const CullCam &c, const double w[3], double &sx, double &sy) {
    double M[3][3], r[3];
    for (int i = 0; i < 3; i++) {
        M[i][0] = c.cam[6 + i];
        M[i][1] = c.cam[9 + i];
        M[i][2] = -(w[i] - c.cam[i]);
        r[i] = -c.cam[3 + i];
    }
    auto det3 = [](double a[3][3]) {
        return a[0][0] * (a[1][1] * a[2][2] - a[1][2] * a[2][1]) - a[0][1] * (a[1][0] * a[2][2] - a[1][2] * a[2][0]) +
               a[0][2] * (a[1][0] * a[2][1] - a[1][1] * a[2][0]);
    };
    const double det = det3(M);
    if (det == 0) return false;
    double sol[3];
    for (int k = 0; k < 3; k++) {
        double Mk[3][3];
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) Mk[i][j] = j == k ? r[i] : M[i][j];
        sol[k] = det3(Mk) / det;
    }
    sx = sol[0];
    sy = sol[1];
    return sol[2] > 0;
}

} // namespace

int main(int argc, char **argv) {
    rs ^= (uint64_t)strtoull(argc > 1 ? argv[1] : "1", nullptr, 10) * 0x9E3779B97F4A7C15ull;
    const int cases = argc > 2 ? atoi(argv[2]) : 2000;
    long long viol = 0, tested = 0, accepted = 0, culled = 0;
    for (int cs = 0; cs < cases; cs++) {
        const double scale = pow(10.0, rr(-3, 4));
        const CullCam c = make_cam(scale);
        const double X = c.xres, Y = c.yres;
        // a triangle: kind picks the geometry
        const int kind = cs % 6;
        double P[3][3];
        double fwd[3] = {c.cam[3] + c.cam[6] * X / 2 + c.cam[9] * Y / 2, c.cam[4] + c.cam[7] * X / 2 + c.cam[10] * Y / 2,
                         c.cam[5] + c.cam[8] * X / 2 + c.cam[11] * Y / 2};
        const double dist = scale * pow(10.0, rr(-2, 2)) * (kind == 5 ? 1e-3 : 1.0);
        const double size = dist * pow(10.0, rr(kind == 1 ? -6 : -3, kind == 2 ? 1.5 : 0.3));
        double ctr[3];
        for (int i = 0; i < 3; i++) ctr[i] = c.cam[i] + fwd[i] * dist * rr(0.5, 1.5) + rr(-1, 1) * dist * 0.5;
        for (int v = 0; v < 3; v++)
            for (int i = 0; i < 3; i++) P[v][i] = ctr[i] + rr(-1, 1) * size;
        if (kind == 3) { // edge-on: move vertex 2 into the plane through the eye and edge 0-1
            const double t = rr(-1e-4, 1e-4);
            for (int i = 0; i < 3; i++) P[2][i] = P[0][i] + (P[1][i] - P[0][i]) * rr(0, 1) + (P[0][i] - c.cam[i]) * rr(-1, 1) + t * size;
        }
        if (kind == 4) // straddling the eye plane / partly behind the eye
            for (int i = 0; i < 3; i++) P[2][i] = c.cam[i] - fwd[i] * dist * rr(0, 2) + rr(-1, 1) * size;
        const V A = {(float)P[0][0], (float)P[0][1], (float)P[0][2]};
        const V B = {(float)P[1][0], (float)P[1][1], (float)P[1][2]};
        const V C = {(float)P[2][0], (float)P[2][1], (float)P[2][2]};
        const V e1 = sub(B, A), e2 = sub(C, A), o = {c.cam[0], c.cam[1], c.cam[2]};
        const float Af[3] = {A.x, A.y, A.z}, e1f[3] = {e1.x, e1.y, e1.z}, e2f[3] = {e2.x, e2.y, e2.z};
        float box[4];
        cr::cam_cull_box(Af, e1f, e2f, c, box);
        auto check = [&](double sxd, double syd) {
            if (!(sxd >= 0 && sxd <= X && syd >= 0 && syd <= Y)) return;
            const float sx = (float)sxd, sy = (float)syd;
            if (!(sx >= 0 && sx <= (float)X && sy >= 0 && sy <= (float)Y)) return;
            tested++;
            const bool in = sx >= box[0] && sx <= box[1] && sy >= box[2] && sy <= box[3];
            culled += !in;
            if (mt(o, camera_dir(c, sx, sy), A, e1, e2)) {
                accepted++;
                if (!in) {
                    if (viol < 10)
                        fprintf(stderr, "VIOLATION case %d kind %d sx %.9g sy %.9g box %.9g %.9g %.9g %.9g\n", cs, kind,
                                sx, sy, box[0], box[1], box[2], box[3]);
                    viol++;
                }
            }
        };
        for (int k = 0; k < 64; k++) check(rr(0, X), rr(0, Y));
        // points on / near the edges and vertices, projected, then nudged by a few ulps
        for (int k = 0; k < 256; k++) {
            const int a = k % 3, b = (k + 1) % 3;
            double w[3], t = rr(0, 1), out = rr(-1, 1) * pow(10.0, rr(-9, -2));
            for (int i = 0; i < 3; i++)
                w[i] = P[a][i] + (P[b][i] - P[a][i]) * t + (P[a][i] + P[b][i] - 2 * P[(k + 2) % 3][i]) * out;
            double sx, sy;
            if (!project(c, w, sx, sy)) continue;
            for (int j = 0; j < 4; j++) {
                float fx = (float)sx, fy = (float)sy;
                for (int m = (int)(rnd() * 4); m > 0; m--) fx = nextafterf(fx, rnd() < 0.5 ? -INFINITY : INFINITY);
                for (int m = (int)(rnd() * 4); m > 0; m--) fy = nextafterf(fy, rnd() < 0.5 ? -INFINITY : INFINITY);
                check(fx, fy);
            }
        }
        // interior points
        for (int k = 0; k < 32; k++) {
            double b0 = rnd(), b1 = rnd() * (1 - b0), w[3], sx, sy;
            for (int i = 0; i < 3; i++) w[i] = P[0][i] + (P[1][i] - P[0][i]) * b0 + (P[2][i] - P[0][i]) * b1;
            if (project(c, w, sx, sy)) check(sx, sy);
        }
    }
    printf("violations %lld tested %lld accepted %lld culled %lld\n", viol, tested, accepted, culled);
    return viol ? 1 : 0;
}
