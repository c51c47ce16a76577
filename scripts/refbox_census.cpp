// refbox_census.cpp -- CPU census (diagnostic only): of the triangle tests the shadow trace still runs
// after the packed leaf cull records (csrc/leafcull.hpp, build 43), how many a per-reference box would
// skip exactly: the reference's tight box padded by its group's fixed pad, plus the group's time window
// turned into space (dt + D (tk - 1), D the scene diagonal), tested against the segment [0, tmax_leaf] --
// valid only for references whose group passed the cone test (|d.a| >= kappa), as the group skip is.
// Input (scripts/refbox_census.py): the oracle's kd tree, refs, triangle positions, shadow rays.
//   refbox_census <scene.bin> <rays.bin>   prints JSON counts
#include "../chiaroscuro-raytracer_amd/csrc/leafcull.hpp"

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

using namespace cr;

namespace {
struct Scene {
    uint32_t nn, nref, ntri;
    std::vector<uint32_t> is_leaf, axis, child, first, count, refs;
    std::vector<float> split, pos, box;
    std::vector<LcFloat4> rec;   // LC_RECP per node (packed, as cabi.cpp)
    std::vector<float> refbox;   // 6 per reference: padded tight box
    std::vector<uint8_t> refgrp; // 0 / 1 group, 2 always
};

uint64_t cnt[16];
enum { Q, OCC, LEAVES, MASKED_TESTS, BOXABLE, BOX_SKIP, INNER, TESTS_ALL };

// kdtree.cpp:293-320
bool mt(const float o[3], const float d[3], const float *A, const float *e1, const float *e2, float tmax) {
    float p[3] = {d[1] * e2[2] - d[2] * e2[1], d[2] * e2[0] - d[0] * e2[2], d[0] * e2[1] - d[1] * e2[0]};
    const float a = (e1[0] * p[0] + e1[1] * p[1]) + e1[2] * p[2];
    if (a < FLT_EPSILON && a > -FLT_EPSILON) return false;
    const float f = 1.f / a;
    const float s[3] = {o[0] - A[0], o[1] - A[1], o[2] - A[2]};
    const float u = f * ((s[0] * p[0] + s[1] * p[1]) + s[2] * p[2]);
    if (u < 0.f || u > 1.f) return false;
    const float q[3] = {s[1] * e1[2] - s[2] * e1[1], s[2] * e1[0] - s[0] * e1[2], s[0] * e1[1] - s[1] * e1[0]};
    const float v = f * ((d[0] * q[0] + d[1] * q[1]) + d[2] * q[2]);
    if (v < 0.f || u + v > 1.f) return false;
    const float t = f * ((e2[0] * q[0] + e2[1] * q[1]) + e2[2] * q[2]);
    return t >= 0.f && t < tmax;
}

// segment [0, T] against a box, in double (the census's own question; the kernel would bound its rounding)
bool seg_hits(const float o[3], const float d[3], double T, const float *b) {
    double t0 = 0, t1 = T;
    for (int i = 0; i < 3; i++) {
        if (d[i] == 0.f) {
            if (o[i] < b[i] || o[i] > b[3 + i]) return false;
            continue;
        }
        double a = (b[i] - (double)o[i]) / d[i], c = (b[3 + i] - (double)o[i]) / d[i];
        if (a > c) std::swap(a, c);
        t0 = std::max(t0, a);
        t1 = std::min(t1, c);
    }
    return t0 <= t1 * (1 + 1e-9) + 1e-12;
}

bool leaf(const Scene &S, uint32_t n, const float o[3], const float d[3], float tmax, uint32_t light) {
    cnt[LEAVES]++;
    const uint32_t c = S.count[n], f = S.first[n];
    const float inv[3] = {1.f / d[0], 1.f / d[1], 1.f / d[2]};
    const uint32_t m = leaf_cull_mask_packed(o, d, inv, lc_unit(d[0], d[1], d[2]), tmax, &S.rec[(size_t)LC_RECP * n], c);
    // which groups passed the cone test
    bool cone[2] = {false, false};
    if (c <= (uint32_t)LC_MAXREFS_P && lc_unit(d[0], d[1], d[2])) {
        for (int k = 0; k < 2; k++) {
            const LcFloat4 lo = S.rec[(size_t)LC_RECP * n + 3 * k], ax = S.rec[(size_t)LC_RECP * n + 3 * k + 2];
            const float dn = fabsf((d[0] * ax.x + d[1] * ax.y) + d[2] * ax.z);
            cone[k] = dn >= lo.w;
        }
    }
    for (uint32_t j = 0; j < c; j++) {
        const uint32_t r = f + j, t = S.refs[r];
        if (t == light) continue;
        cnt[TESTS_ALL]++;
        if (c <= 32 && !((m >> j) & 1u)) continue;
        cnt[MASKED_TESTS]++;
        const uint8_t g = S.refgrp[r];
        const bool boxable = g < 2 && cone[g];
        if (boxable) cnt[BOXABLE]++;
        if (boxable && !seg_hits(o, d, tmax, &S.refbox[6 * (size_t)r])) {
            cnt[BOX_SKIP]++;
            continue;
        }
        const float *P = &S.pos[9 * (size_t)t];
        const float e1[3] = {P[3] - P[0], P[4] - P[1], P[5] - P[2]}, e2[3] = {P[6] - P[0], P[7] - P[1], P[8] - P[2]};
        if (mt(o, d, P, e1, e2, tmax)) return true;
    }
    return false;
}

bool node(const Scene &S, uint32_t n, const float o[3], const float d[3], float tmin, float tmax, uint32_t light) {
    if (S.is_leaf[n]) return leaf(S, n, o, d, tmax, light);
    cnt[INNER]++;
    const uint32_t a = S.axis[n];
    const float tsplit = (S.split[n] - o[a]) / d[a];
    const uint32_t below = (o[a] < S.split[n]) || (o[a] == S.split[n] && d[a] <= 0);
    const uint32_t c = S.child[n];
    if (tsplit >= tmax || tsplit < 0) return node(S, c + (1 - below), o, d, tmin, tmax, light);
    if (tsplit <= tmin) return node(S, c + below, o, d, tmin, tmax, light);
    return node(S, c + (1 - below), o, d, tmin, tsplit, light) || node(S, c + below, o, d, tsplit, tmax, light);
}
} // namespace

int main(int argc, char **argv) {
    if (argc < 3) return 1;
    FILE *f = fopen(argv[1], "rb");
    Scene S;
    uint32_t h[3];
    if (fread(h, 4, 3, f) != 3) return 1;
    S.nn = h[0], S.nref = h[1], S.ntri = h[2];
    auto rd = [&](auto &v, size_t n) {
        v.resize(n);
        if (fread(v.data(), sizeof(v[0]), n, f) != n) exit(1);
    };
    rd(S.is_leaf, S.nn), rd(S.axis, S.nn), rd(S.split, S.nn), rd(S.child, S.nn), rd(S.first, S.nn), rd(S.count, S.nn);
    rd(S.refs, S.nref), rd(S.pos, 9 * (size_t)S.ntri), rd(S.box, 6);
    fclose(f);
    // cabi.cpp's records: leaf_cull_record -> leaf_cull_fixed -> leaf_cull_pack
    double db = 1.0, smax = 0.0, diag = 0.0;
    for (int i = 0; i < 3; i++) {
        db = std::max(db, std::max(std::fabs((double)S.box[i]), std::fabs((double)S.box[3 + i])) + 1.0);
        smax = std::max(smax, (double)S.box[3 + i] - (double)S.box[i] + 2.0);
        diag += ((double)S.box[3 + i] - S.box[i]) * ((double)S.box[3 + i] - S.box[i]);
    }
    db *= 1.0001;
    diag = std::sqrt(diag) * 1.01 + 2;
    S.rec.assign((size_t)LC_RECP * S.nn, LcFloat4{0, 0, 0, 0});
    S.refbox.assign(6 * (size_t)S.nref, 0.f);
    S.refgrp.assign(S.nref, 2);
    const double u = 0x1p-24, c0 = 1.0 / LC_C0_INV, Sx = smax * (1 + 4 * u) + 1e-6;
    for (uint32_t n = 0; n < S.nn; n++) {
        if (!S.is_leaf[n]) continue;
        const uint32_t c = S.count[n], fi = S.first[n], mm = std::min(c, (uint32_t)LC_MAXREFS);
        float A[LC_MAXREFS][3], e1[LC_MAXREFS][3], e2[LC_MAXREFS][3];
        for (uint32_t j = 0; j < mm; j++) {
            const float *P = &S.pos[9 * (size_t)S.refs[fi + j]];
            for (int i = 0; i < 3; i++) A[j][i] = P[i], e1[j][i] = P[3 + i] - P[i], e2[j][i] = P[6 + i] - P[i];
        }
        LcFloat4 r7[LC_REC], fx[LC_REC];
        leaf_cull_record(A, e1, e2, c, r7);
        leaf_cull_fixed(r7, db, smax, fx);
        leaf_cull_pack(fx, c, &S.rec[(size_t)LC_RECP * n]);
        if (c > (uint32_t)LC_MAXREFS_P) continue;
        uint32_t gm[2];
        memcpy(&gm[0], &r7[6].x, 4);
        memcpy(&gm[1], &r7[6].y, 4);
        for (int k = 0; k < 2; k++) {
            const double g = r7[3 * k].w, E = r7[3 * k + 1].w;
            const double pad = (20.11 * u * (E + 2 * Sx) * g / c0 + 6.21 * u * E + u * Sx) * (1 + 1e-6) + 4 * u * db;
            const double dt = 10.06 * u * Sx * g / c0 * (1 + 1e-6);
            const double tk = (1 + 10.06 * u * g / c0) * (1 + 3 * u) * (1 + 1e-6);
            const double ext = pad + dt + diag * (tk - 1);
            for (uint32_t j = 0; j < mm; j++) {
                if (!((gm[k] >> j) & 1u)) continue;
                S.refgrp[fi + j] = (uint8_t)k;
                float *b = &S.refbox[6 * (size_t)(fi + j)];
                for (int i = 0; i < 3; i++) {
                    const double a = A[j][i], bb = a + (double)e1[j][i], cc = a + (double)e2[j][i];
                    b[i] = (float)(std::min(a, std::min(bb, cc)) - ext);
                    b[3 + i] = (float)(std::max(a, std::max(bb, cc)) + ext);
                }
            }
        }
    }
    f = fopen(argv[2], "rb");
    uint32_t nr;
    if (fread(&nr, 4, 1, f) != 1) return 1;
    for (uint32_t i = 0; i < nr; i++) {
        float v[8];
        if (fread(v, 4, 8, f) != 8) return 1;
        const float *o = v, *d = v + 3;
        uint32_t light;
        memcpy(&light, &v[7], 4);
        // kdtree.cpp:283-290 root clip
        float tn[3], tf[3];
        for (int k = 0; k < 3; k++) {
            const float inv = 1.f / d[k];
            const float a = (S.box[k] - o[k]) * inv, b = (S.box[3 + k] - o[k]) * inv;
            tn[k] = b < a ? b : a;
            tf[k] = a < b ? b : a;
        }
        float t0 = tn[0] < tn[1] ? tn[1] : tn[0];
        t0 = t0 < tn[2] ? tn[2] : t0;
        float t1 = tf[1] < tf[0] ? tf[1] : tf[0];
        t1 = tf[2] < t1 ? tf[2] : t1;
        cnt[Q]++;
        if (t1 < 0 || t1 < t0 || t0 > v[6]) continue;
        if (node(S, 0, o, d, t0, std::min(t1, v[6]), light)) cnt[OCC]++;
    }
    printf("{\"queries\": %llu, \"occluded\": %llu, \"leaves\": %llu, \"inner\": %llu, \"tests_all\": %llu, "
           "\"tests_after_leaf_cull\": %llu, \"boxable\": %llu, \"box_skipped\": %llu}\n",
           (unsigned long long)cnt[Q], (unsigned long long)cnt[OCC], (unsigned long long)cnt[LEAVES],
           (unsigned long long)cnt[INNER], (unsigned long long)cnt[TESTS_ALL], (unsigned long long)cnt[MASKED_TESTS],
           (unsigned long long)cnt[BOXABLE], (unsigned long long)cnt[BOX_SKIP]);
    return 0;
}
