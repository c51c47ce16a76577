// planecull.hpp -- plane records: an exact skip of Moller-Trumbore tests
// (kdtree.cpp:219-246 / 293-320) whose segment [0, tmax) stays on one side of the
// triangle's plane.
//
// With n = e1 x e2 and sv = RN(o - A), the test's t is T/AA in exact arithmetic,
// T = sv.n, AA = -d.n, and it accepts only with 0 <= t < tmax after rounding.
// Bounding the rounding of T and AA (|dT| <= Et, |dAA| <= Ea: camcull.hpp's bounds)
// gives: if  g0 = T > Et  and  g1 = T - tmax*AA = n.(sv + tmax d) > Et + tmax*Ea +
// 2.1u*tmax*(|AA| + Ea),  the test rejects (its t is negative or >= tmax), and the
// same with both signs flipped.  g0 and g1 are the plane's values at the segment's
// ends.  For rays inside the scene box B (|o_i|, |A_i| <= Db), with |d_i| <= 1.001
// (the normalized directions of BRDF and light samples) and tmax <= Tb (the
// segment stays within the box), every bound is at most u*E*(21 Db + 12 Tb) with
// E = |e1|_1 |e2|_1, and so is the error of evaluating the plane in float.  The
// record is the plane scaled by mu = 4u*E*(21 Db + 12 Tb) (twice that):
//     N = n / mu,  W = n.A / mu,  s0 = N.o - W,  s1 = s0 + tmax * (N.d)
// and the kernel skips the test when s0 > 1 and s1 > 1, or s0 < -1 and s1 < -1.
// Degenerate, tiny or non-finite triangles get N = W = 0 (never skipped).
#pragma once
#include <math.h>

#if defined(__HIPCC__)
#define CR_PLANE_HD __host__ __device__
#else
#define CR_PLANE_HD
#endif

namespace cr {

// Db: max |coordinate| a ray origin or vertex can have (the padded scene box + 1);
// Tb: max segment length (the box diagonal, generously); out = {N, W}
CR_PLANE_HD inline void plane_record(const float A[3], const float e1f[3], const float e2f[3], double Db, double Tb,
                                     float out[4]) {
    const double u = 0x1p-24;
    double e1[3], e2[3], a[3];
    for (int i = 0; i < 3; i++) {
        e1[i] = e1f[i];
        e2[i] = e2f[i];
        a[i] = A[i];
    }
    const double n[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]};
    const double E = (fabs(e1[0]) + fabs(e1[1]) + fabs(e1[2])) * (fabs(e2[0]) + fabs(e2[1]) + fabs(e2[2]));
    const double mu = 4.0 * u * E * (21.0 * Db + 12.0 * Tb);
    const double w = n[0] * a[0] + n[1] * a[1] + n[2] * a[2];
    for (int i = 0; i < 4; i++) out[i] = 0.f;
    if (!(mu > 1e-20 && mu < 1e30 && E < 1e30 && fabs(w) < 1e30 && Db < 1e15 && Tb < 1e15)) return;
    for (int i = 0; i < 3; i++) out[i] = (float)(n[i] / mu);
    out[3] = (float)(w / mu);
}

} // namespace cr
