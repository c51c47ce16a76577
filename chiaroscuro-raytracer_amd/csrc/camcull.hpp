// camcull.hpp -- screen-space cull boxes for camera rays: an exact skip of
// Moller-Trumbore tests (kdtree.cpp:219-246) that cannot accept.
//
// Every camera ray starts at the eye o and has the direction
//     d = RN(RN(lu + RN(dx * sx)) + RN(dy * sy)),  sx = RN(x + ux), sy = RN(y + uy)
// (rayTracer.cpp:61, camera_dir): d is an affine function of the sample's screen
// position (sx, sy) up to three roundings.  With sv = RN(o - A) and the record's
// e1, e2, the quantities Moller-Trumbore rounds are, in exact arithmetic,
//     AA = d.(e2 x e1),  U = d.(e2 x sv),  V = d.(sv x e1),  T = e2.(sv x e1)
// -- all linear in d -- and the test accepts only if u = U/AA, v = V/AA and
// t = T/AA pass their range checks after rounding.  Bounding every rounding of the
// float evaluation (relative error u = 2^-24 per operation, plus an absolute slack
// for subnormal results) gives, for any sample the test ACCEPTS, with tau = sign(T):
//     tau*U >= -Ku,   tau*V >= -Kv,   tau*(AA - U - V) >= -Kw
// (the t >= 0 check fixes sign(AA) = tau once |T| exceeds its error bound).  These are
// three half-planes in (sx, sy); clipped to the screen rectangle they bound every
// sample position at which the test can accept.  cam_cull_box returns that region's
// bounding box, padded and rounded outwards to float: a camera ray whose (sx, sy)
// lies outside it is rejected by the test for certain, so skipping the test leaves
// every result bit unchanged.  A triangle whose bound cannot be established (huge
// or non-finite coordinates, the eye in its plane) gets the box of the whole plane
// (never skipped); one no camera ray can hit gets an empty box (always skipped).
//
// Error bounds (d componentwise bounded by D over the screen):
//   p = d x e2:  |dp_i| <= 2.01u P_i,  P = |d| x |e2| (absolute cross product)
//   AA = e1.p:   |dAA| <= 5.02u sum |e1_i| P_i = Ea    U = sv.p: Eu = 5.02u sum |sv_i| P_i
//   q = sv x e1: |dq_i| <= 2.01u Q_i,  Q = |sv| x |e1|
//   V = d.q:     Ev = 5.02u sum D_i Q_i                T = e2.q: Et = 5.02u sum |e2_i| Q_i
//   u + v > 1 with u, v >= 0 rounded: Kw = Ea + Eu + Ev + 3.1u |AA|max (+ slack)
//   d vs its affine map: |d_i - (lu + sx dx + sy dy)_i| <= 3.1u D_i
// (5.1u and 3.2u are used below: a margin only widens the box.)
#pragma once
#include <float.h>
#include <math.h>
#include <stdint.h>

#if defined(__HIPCC__)
#define CR_CULL_HD __host__ __device__
#else
#define CR_CULL_HD
#endif

namespace cr {

// eye, leftUpper, dx, dy as in RenderArgs::cam; the screen is [0, xres] x [0, yres]
struct CullCam {
    float cam[12];
    float xres, yres;
};

CR_CULL_HD inline float cull_down(double x) {
    float f = (float)x;
    if ((double)f > x) f = nextafterf(f, -INFINITY);
    return f;
}
CR_CULL_HD inline float cull_up(double x) {
    float f = (float)x;
    if ((double)f < x) f = nextafterf(f, INFINITY);
    return f;
}

// Box {xmin, xmax, ymin, ymax} of the sample positions at which the triangle record
// (A, e1 = B - A, e2 = C - A, exactly the floats the test uses) can accept a camera ray.
CR_CULL_HD inline void cam_cull_box(const float A[3], const float e1f[3], const float e2f[3], const CullCam &c,
                                    float out[4]) {
    const double u = 0x1p-24;
    const double X = c.xres, Y = c.yres;
    // never skipped / always skipped
    const float all[4] = {-INFINITY, INFINITY, -INFINITY, INFINITY};
    const float none[4] = {INFINITY, -INFINITY, INFINITY, -INFINITY};
    auto put = [&](const float *b) {
        for (int i = 0; i < 4; i++) out[i] = b[i];
    };
    double s[3], e1[3], e2[3], D[3], lu[3], dx[3], dy[3];
    for (int i = 0; i < 3; i++) {
        const float svf = c.cam[i] - A[i]; // the float subtraction the test performs
        s[i] = svf;
        e1[i] = e1f[i];
        e2[i] = e2f[i];
        lu[i] = c.cam[3 + i];
        dx[i] = c.cam[6 + i];
        dy[i] = c.cam[9 + i];
        D[i] = (fabs(lu[i]) + fabs(dx[i]) * X + fabs(dy[i]) * Y) * (1.0 + 1e-6);
    }
    auto cross = [](const double *a, const double *b, double *r) {
        r[0] = a[1] * b[2] - a[2] * b[1];
        r[1] = a[2] * b[0] - a[0] * b[2];
        r[2] = a[0] * b[1] - a[1] * b[0];
    };
    auto acr = [](const double *a, const double *b, double *r) { // |a| x |b|
        r[0] = fabs(a[1] * b[2]) + fabs(a[2] * b[1]);
        r[1] = fabs(a[2] * b[0]) + fabs(a[0] * b[2]);
        r[2] = fabs(a[0] * b[1]) + fabs(a[1] * b[0]);
    };
    auto adot = [](const double *a, const double *b) { return fabs(a[0] * b[0]) + fabs(a[1] * b[1]) + fabs(a[2] * b[2]); };
    double Na[3], Nu[3], Nv[3], Nw[3], P[3], Q[3];
    cross(e2, e1, Na);
    cross(e2, s, Nu);
    cross(s, e1, Nv);
    const double T = e2[0] * Nv[0] + e2[1] * Nv[1] + e2[2] * Nv[2];
    acr(D, e2, P);
    acr(s, e1, Q);
    const double AAb = adot(e1, P), Ub = adot(s, P), Vb = adot(D, Q), Tb = adot(e2, Q);
    const double lim = 1e30;
    double mag = 1.0;
    for (int i = 0; i < 3; i++) mag += fabs(s[i]) + fabs(e1[i]) + fabs(e2[i]) + D[i];
    if (!(AAb < lim && Ub < lim && Vb < lim && Tb < lim && mag < lim && X < 1e8 && Y < 1e8)) return put(all);
    const double slack = 0x1p-100 * mag + 0x1p-120 * AAb; // subnormal / underflow slack
    const double Ea = 5.1 * u * AAb, Eu = 5.1 * u * Ub, Ev = 5.1 * u * Vb, Et = 5.1 * u * Tb;
    // |AA| always below FLT_EPSILON: the test's first check rejects every ray
    if (AAb * (1.0 + 6.0 * u) + Ea + slack < (double)FLT_EPSILON) return put(none);
    if (!(fabs(T) > Et + slack)) return put(all); // eye (nearly) in the triangle's plane
    const double tau = T > 0 ? 1.0 : -1.0;
    for (int i = 0; i < 3; i++) Nw[i] = Na[i] - Nu[i] - Nv[i];
    double Nabs[3];
    for (int i = 0; i < 3; i++) Nabs[i] = fabs(Na[i]) + fabs(Nu[i]) + fabs(Nv[i]);
    const double dslack = 1e-12 * adot(Nabs, D); // double evaluation of the normals
    const double *N[3] = {Nu, Nv, Nw};
    const double K[3] = {Eu + slack, Ev + slack, Ea + Eu + Ev + 3.1 * u * AAb + 4.0 * slack};
    // half-planes h_e(x, y) = al + be x + ga y >= 0 over the screen
    double al[3], be[3], ga[3];
    for (int e = 0; e < 3; e++) {
        const double *n = N[e];
        const double a = tau * (n[0] * lu[0] + n[1] * lu[1] + n[2] * lu[2]);
        const double b = tau * (n[0] * dx[0] + n[1] * dx[1] + n[2] * dx[2]);
        const double g = tau * (n[0] * dy[0] + n[1] * dy[1] + n[2] * dy[2]);
        const double k = K[e] + 3.2 * u * adot(n, D) + dslack + 1e-12 * (fabs(a) + fabs(b) * X + fabs(g) * Y);
        al[e] = a + k;
        be[e] = b;
        ga[e] = g;
    }
    // clip the screen rectangle by the three half-planes (Sutherland-Hodgman)
    double px[8] = {0.0, X, X, 0.0}, py[8] = {0.0, 0.0, Y, Y};
    int n = 4;
    for (int e = 0; e < 3 && n > 0; e++) {
        double qx[8], qy[8];
        int m = 0;
        for (int i = 0; i < n; i++) {
            const int j = (i + 1) % n;
            const double hi = al[e] + be[e] * px[i] + ga[e] * py[i];
            const double hj = al[e] + be[e] * px[j] + ga[e] * py[j];
            if (hi >= 0.0 && m < 8) {
                qx[m] = px[i];
                qy[m++] = py[i];
            }
            if ((hi >= 0.0) != (hj >= 0.0) && m < 8) {
                const double t = hi / (hi - hj);
                qx[m] = px[i] + t * (px[j] - px[i]);
                qy[m++] = py[i] + t * (py[j] - py[i]);
            }
        }
        n = m;
        for (int i = 0; i < n; i++) {
            px[i] = qx[i];
            py[i] = qy[i];
        }
    }
    if (n == 0) return put(none);
    double x0 = px[0], x1 = px[0], y0 = py[0], y1 = py[0];
    for (int i = 1; i < n; i++) {
        x0 = fmin(x0, px[i]);
        x1 = fmax(x1, px[i]);
        y0 = fmin(y0, py[i]);
        y1 = fmax(y1, py[i]);
    }
    const double pad = 1e-3 + 1e-9 * (X + Y); // the clipping arithmetic (pixels)
    out[0] = cull_down(x0 - pad);
    out[1] = cull_up(x1 + pad);
    out[2] = cull_down(y0 - pad);
    out[3] = cull_up(y1 + pad);
}

} // namespace cr
