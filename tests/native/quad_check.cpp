// quad_check.cpp -- CPU model check of the two-level kd node records (csrc/quadnodes.hpp) and of the
// descent the secondary closest and shadow traces run over them (csrc/traverse.hpp, trav_round's QUAD
// path), against the per-ray recursion of kdtree.cpp:248-281 / 322-344.
//
// The model restates the kernel's steps per lane: a traversal position is a code slot << 2 | sel; one
// 16-B record per two descent levels; a far middle child is pushed as its parent's record with sel
// 1 / 2 and resumes with one step of that record before the two-level loop; stack entries
// {code, tmax at push} restored by the kd stack invariant (tmin = the current tmax at a pop).  Leaves
// answer from a table: a leaf holds random "hit distances" and accepts the smallest in [0, tmax) (a
// closest query ends at the first leaf that accepts; a shadow query at the first accept of any) --
// the traversal only decides WHICH leaves are tested with which intervals, the triangle test itself is
// the same code both ways.  For every ray the sequence of (leaf, tmin, tmax) tests and the answer must
// equal the recursion's.  The fat-record traversal the kernels ran before (two levels per fetch as a
// dwordx4 + dwordx2 pair) is modelled too, and both fetch counts are reported: the vector-memory
// instructions of the descent per query.
//
//   quad_check rand <seed> <cases> [mutant]          random trees, rays, intervals
//   quad_check file <tree.bin> <rays.bin> [mutant]    a scene's tree and rays (tests/test_quad_model.py)
// prints "violations V rays R leaf_tests L fat_fetch_insts F quad_fetch_insts Q mid_pops M"
// mutant 1: a middle child's children taken at gb_0 for both children; 2: a popped middle child resumed
// as a record root -- both must be caught.
#include "../../chiaroscuro-raytracer_amd/csrc/quadnodes.hpp"

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace {

uint64_t rs = 88172645463325252ull;
uint64_t next() {
    rs ^= rs << 13;
    rs ^= rs >> 7;
    rs ^= rs << 17;
    return rs;
}
double rnd() { return (double)(next() >> 11) * 0x1p-53; }

struct Tree {
    std::vector<cr::QuadNode> nodes; // cabi.cpp's encoding
    std::vector<std::vector<float>> hits; // per node (leaves): hit distances
};

// random tree: axis / split / depth random; leaves with 0..8 references and 0..3 hit distances
void fill(Tree &t, uint32_t id, int depth, const float lo[3], const float hi[3], uint32_t &nrefs) {
    if (depth == 0 || rnd() < 0.07) {
        const int nh = rnd() < 0.6 ? 0 : 1 + (int)(rnd() * 3);
        for (int i = 0; i < nh; i++) t.hits[id].push_back((float)(rnd() * 40.0 - 5.0));
        const uint32_t cnt = (uint32_t)(rnd() * 9);
        t.nodes[id] = {cnt ? nrefs : 0u, 3u | cnt << 2};
        nrefs += cnt;
        return;
    }
    const int a = (int)(rnd() * 3);
    // splits sometimes on an integer, which ray origins use exactly (ties of the below test)
    float s = lo[a] + (float)rnd() * (hi[a] - lo[a]);
    if (rnd() < 0.1) s = std::floor(s);
    const uint32_t c = (uint32_t)t.nodes.size();
    t.nodes.resize(c + 2, {0, 0});
    t.hits.resize(c + 2);
    uint32_t sb;
    std::memcpy(&sb, &s, 4);
    t.nodes[id] = {sb, (uint32_t)a | c << 2};
    for (int k = 0; k < 2; k++) {
        float l2[3], h2[3];
        std::memcpy(l2, lo, sizeof l2);
        std::memcpy(h2, hi, sizeof h2);
        if (k == 0) h2[a] = s;
        else l2[a] = s;
        fill(t, c + (uint32_t)k, depth - 1, l2, h2, nrefs);
    }
}

struct Ray {
    float o[3], d[3], tmin, tmax;
    bool shadow;
};
struct Test {
    uint32_t leaf;
    float tmin, tmax;
    bool operator==(const Test &b) const {
        return leaf == b.leaf && std::memcmp(&tmin, &b.tmin, 4) == 0 && std::memcmp(&tmax, &b.tmax, 4) == 0;
    }
};

// a leaf accepts its smallest hit distance in [0, tmax) (closest: tmax shrinks to it); leaf identity by its
// first reference (unique among non-empty leaves) and, for empty leaves, "empty"
bool leaf_accepts(const Tree &t, uint32_t node, float &tmax) {
    bool any = false;
    for (float h : t.hits[node])
        if (h >= 0.f && h < tmax) {
            tmax = h;
            any = true;
        }
    return any;
}

// kdtree.cpp:248-281 / 322-344, recursive as written
bool recurse(const Tree &t, const Ray &r, uint32_t n, float tmin, float tmax, std::vector<Test> &seq, float &thit) {
    const cr::QuadNode nd = t.nodes[n];
    if ((nd.y & 3u) == 3u) {
        seq.push_back({n, tmin, tmax});
        float tm = tmax;
        if (leaf_accepts(t, n, tm)) {
            thit = tm;
            return true;
        }
        return false;
    }
    const uint32_t a = nd.y & 3u, c = nd.y >> 2;
    float split;
    std::memcpy(&split, &nd.x, 4);
    const float oa = r.o[a], da = r.d[a];
    const float tsplit = (split - oa) / da;
    const uint32_t below = (oa < split) || (oa == split && da <= 0);
    if (tsplit >= tmax || tsplit < 0) return recurse(t, r, c + (1 - below), tmin, tmax, seq, thit);
    if (tsplit <= tmin) return recurse(t, r, c + below, tmin, tmax, seq, thit);
    return recurse(t, r, c + (1 - below), tmin, tsplit, seq, thit) || recurse(t, r, c + below, tsplit, tmax, seq, thit);
}

// the kernel's step at an inner node: returns the child side taken (0 / 1 of the node's children) and
// pushes the far child's position when both are crossed (trav_round's step, BF form)
struct Lane {
    float tmin, tmax;
    std::vector<std::pair<uint32_t, float>> stack; // {position, tmax at push}
};
uint32_t step(const Ray &r, Lane &L, uint32_t split_bits, uint32_t a, uint32_t far_pos0, uint32_t far_pos1,
              bool &pushed) {
    float split;
    std::memcpy(&split, &split_bits, 4);
    const float oa = r.o[a], da = r.d[a];
    const float tsplit = (split - oa) / da;
    const uint32_t below = (oa < split) || (oa == split && da <= 0);
    const bool near_only = (tsplit >= L.tmax) | (tsplit < 0);
    const bool far_only = !near_only & (tsplit <= L.tmin);
    pushed = !near_only & !far_only;
    const uint32_t k = far_only ? below : 1u - below;
    if (pushed) {
        L.stack.push_back({below ? far_pos1 : far_pos0, L.tmax});
        L.tmax = tsplit;
    }
    return k;
}
bool pop(Lane &L, uint32_t &pos) {
    if (L.stack.empty()) return false;
    pos = L.stack.back().first;
    L.tmin = L.tmax; // the popped entry's split distance (stack invariant)
    L.tmax = L.stack.back().second;
    L.stack.pop_back();
    return true;
}

// the fat-record traversal (build 26 / 43): a fetch = the node's word and both children's (2 insts)
bool fat_trace(const Tree &t, const Ray &r, std::vector<Test> &seq, uint64_t &insts) {
    Lane L{r.tmin, r.tmax, {}};
    uint32_t node = 0;
    for (;;) {
        insts += 2; // fetch(node): dwordx4 + dwordx2
        cr::QuadNode nd = t.nodes[node];
        while ((nd.y & 3u) != 3u) {
            bool p;
            const uint32_t c = nd.y >> 2;
            const uint32_t k = step(r, L, nd.x, nd.y & 3u, c, c + 1, p);
            node = c + k;
            nd = t.nodes[node]; // from the fat record
            if ((nd.y & 3u) != 3u) {
                const uint32_t c2 = nd.y >> 2;
                const uint32_t k2 = step(r, L, nd.x, nd.y & 3u, c2, c2 + 1, p);
                node = c2 + k2;
                insts += 2;
                nd = t.nodes[node];
            }
        }
        seq.push_back({node, L.tmin, L.tmax});
        float tm = L.tmax;
        if (leaf_accepts(t, node, tm)) return true;
        if (!pop(L, node)) return false;
    }
}

// owner[code]: the tree node at each position of the layout, walked from the root along the records'
// own meta words -- and every record word checked against the node it stands for
bool quad_owner(const Tree &t, const cr::QuadLayout &q, std::vector<uint32_t> &owner) {
    owner.assign(4 * (size_t)q.slots, 0xffffffffu);
    std::vector<std::pair<uint32_t, uint32_t>> work{{0u, 0u}};
    auto expect = [&](uint32_t n) {
        const cr::QuadNode nd = t.nodes[n];
        return (nd.y & 3u) == 3u ? cr::quad_leaf_word((nd.y >> 2) ? nd.x : 0u, nd.y >> 2, q.fbits) : nd.x;
    };
    while (!work.empty()) {
        const auto [slot, n] = work.back();
        work.pop_back();
        if (slot >= q.slots) return false;
        const uint32_t *R = q.rec.data() + 4 * (size_t)slot;
        owner[slot << 2] = n;
        const cr::QuadNode nd = t.nodes[n];
        if (R[0] != expect(n) || (R[3] & 3u) != (nd.y & 3u)) return false;
        if ((nd.y & 3u) == 3u) continue;
        const uint32_t c = nd.y >> 2;
        for (uint32_t k = 0; k < 2; k++) {
            owner[(slot << 2) | (1u + k)] = c + k;
            if (R[1 + k] != expect(c + k) || ((R[3] >> (2 + 2 * k)) & 3u) != (t.nodes[c + k].y & 3u)) return false;
            if ((t.nodes[c + k].y & 3u) == 3u) continue;
            const uint32_t g = (R[3] >> 6) + (k == 1 && ((R[3] >> 2) & 3u) != 3u ? 2u : 0u);
            const uint32_t gc = t.nodes[c + k].y >> 2;
            work.emplace_back(g, gc);
            work.emplace_back(g + 1, gc + 1);
        }
    }
    return true;
}

// the quad-record traversal (trav_round's QUAD path); leaf ids mapped back to tree nodes by `owner`
bool quad_trace(const Tree *T, const cr::QuadLayout &q, const std::vector<uint32_t> &owner, const Ray &r,
                std::vector<Test> &seq, uint64_t &insts, uint64_t &mid_pops, int mutant) {
    Lane L{r.tmin, r.tmax, {}};
    uint32_t code = 0;
    const uint32_t *R = nullptr;
    auto fetch = [&](uint32_t c) {
        insts += 1; // one dwordx4
        R = q.rec.data() + 4 * (size_t)(c >> 2);
    };
    auto gb = [&](uint32_t k) {
        const uint32_t base = R[3] >> 6;
        if (mutant == 1) return base;
        return base + (k == 1 && ((R[3] >> 2) & 3u) != 3u ? 2u : 0u);
    };
    for (;;) {
        if ((code >> 2) >= q.slots) {
            seq.push_back({0xffffffffu, 0.f, 0.f});
            return false;
        }
        fetch(code);
        uint32_t sel = code & 3u;
        if (mutant == 2) sel = 0;
        uint32_t w = sel ? R[sel] : R[0], a = sel ? (R[3] >> (2 * sel)) & 3u : R[3] & 3u;
        if (sel) mid_pops++;
        if (sel && a != 3u) { // mid start: the middle node's step, then its child's record
            bool p;
            const uint32_t g = gb(sel - 1);
            const uint32_t k2 = step(r, L, w, a, g << 2, (g + 1) << 2, p);
            code = (g + k2) << 2;
            fetch(code);
            w = R[0];
            a = R[3] & 3u;
        }
        while (a != 3u) {
            bool p;
            const uint32_t slot = code >> 2;
            const uint32_t k = step(r, L, w, a, (slot << 2) | 1u, (slot << 2) | 2u, p);
            code = (slot << 2) | (1u + k);
            w = R[1 + k];
            a = (R[3] >> (2 + 2 * k)) & 3u;
            if (a != 3u) {
                const uint32_t g = gb(k);
                const uint32_t k2 = step(r, L, w, a, g << 2, (g + 1) << 2, p);
                code = (g + k2) << 2;
                fetch(code);
                w = R[0];
                a = R[3] & 3u;
            }
        }
        (void)w;
        // (a broken traversal may wander: a position outside the layout or a runaway stack ends the ray,
        // and its sequence then differs from the recursion's)
        if (code >= owner.size() || owner[code] == 0xffffffffu || L.stack.size() > 4096 || seq.size() > 100000) {
            seq.push_back({0xffffffffu, 0.f, 0.f});
            return false;
        }
        seq.push_back({owner[code], L.tmin, L.tmax});
        float tm = L.tmax;
        if (leaf_accepts(*T, owner[code], tm)) return true;
        if (!pop(L, code)) return false;
    }
}

} // namespace

namespace {
// kdtree.cpp:196-208 root clip (the kernels' ray_box_inv: RN(1/d) products)
bool root_clip(const float bmin[3], const float bmax[3], Ray &r, float limit) {
    float t0 = -INFINITY, t1 = INFINITY;
    float tn[3], tf[3];
    for (int i = 0; i < 3; i++) {
        const float inv = 1.f / r.d[i];
        const float a = (bmin[i] - r.o[i]) * inv, b = (bmax[i] - r.o[i]) * inv;
        tn[i] = b < a ? b : a;
        tf[i] = a < b ? b : a;
    }
    t0 = tn[0] < tn[1] ? tn[1] : tn[0];
    t0 = t0 < tn[2] ? tn[2] : t0;
    t1 = tf[1] < tf[0] ? tf[1] : tf[0];
    t1 = tf[2] < t1 ? tf[2] : t1;
    if (t1 < 0 || t1 < t0) return false;
    if (r.shadow) {
        if (t0 > limit) return false;
        t1 = limit < t1 ? limit : t1;
    }
    r.tmin = t0;
    r.tmax = t1;
    return true;
}

struct Stats {
    uint64_t viol = 0, rays = 0, tests = 0, fat = 0, quad = 0, mid = 0;
};

void run(const Tree &t, uint32_t nrefs, std::vector<Ray> &rays, int mutant, Stats &st) {
    cr::QuadLayout q;
    std::string err;
    if (!cr::quad_build(t.nodes.data(), (uint32_t)t.nodes.size(), nrefs, q, err)) {
        std::printf("build failed: %s\n", err.c_str());
        std::exit(2);
    }
    std::vector<uint32_t> owner;
    if (!quad_owner(t, q, owner)) {
        std::printf("layout does not match the tree\n");
        std::exit(3);
    }
    std::vector<Test> a, b, c;
    for (const Ray &r : rays) {
        a.clear();
        b.clear();
        c.clear();
        float th = 0.f;
        const bool ra = recurse(t, r, 0, r.tmin, r.tmax, a, th);
        const bool rb = fat_trace(t, r, b, st.fat);
        const bool rc = quad_trace(&t, q, owner, r, c, st.quad, st.mid, mutant);
        st.rays++;
        st.tests += a.size();
        if (ra != rb || a != b) st.viol++; // (the fat model itself must agree with the recursion)
        if (ra != rc || a != c) st.viol++;
    }
}
} // namespace

int main(int argc, char **argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: quad_check rand <seed> <cases> [mutant] | file <tree.bin> <rays.bin> [mutant]\n");
        return 1;
    }
    Stats st;
    if (!std::strcmp(argv[1], "rand")) {
        rs ^= (uint64_t)std::atoll(argv[2]) * 0x9E3779B97F4A7C15ull;
        const int cases = std::atoi(argv[3]);
        const int mutant = argc > 4 ? std::atoi(argv[4]) : 0;
        for (int cs = 0; cs < cases; cs++) {
            Tree t;
            t.nodes.resize(1, {0, 0});
            t.hits.resize(1);
            const float lo[3] = {-10, -10, -10}, hi[3] = {10, 10, 10};
            uint32_t nrefs = 0;
            fill(t, 0, 3 + (int)(rnd() * 12), lo, hi, nrefs);
            std::vector<Ray> rays;
            for (int i = 0; i < 200; i++) {
                Ray r;
                for (int k = 0; k < 3; k++) {
                    r.o[k] = (float)(rnd() * 24 - 12);
                    if (rnd() < 0.15) r.o[k] = std::floor(r.o[k]); // on a split plane, sometimes
                    r.d[k] = (float)(rnd() * 2 - 1);
                    if (rnd() < 0.08) r.d[k] = 0.f; // axis-parallel components (inf / NaN splits)
                }
                r.shadow = rnd() < 0.5;
                const float limit = (float)(rnd() * 30);
                if (!root_clip(lo, hi, r, limit)) continue;
                rays.push_back(r);
            }
            run(t, nrefs, rays, mutant, st);
        }
    } else {
        // tree.bin: nn, nrefs, bmin[3], bmax[3], then nn x {x, y} in cabi's encoding, then per node a hit
        // count and its distances; rays.bin: n, then n x {o[3], d[3], limit, shadow (as float 0 / 1)}
        FILE *f = std::fopen(argv[2], "rb");
        if (!f) return 1;
        uint32_t nn = 0, nrefs = 0;
        float bmin[3], bmax[3];
        bool ok = std::fread(&nn, 4, 1, f) == 1 && std::fread(&nrefs, 4, 1, f) == 1 && std::fread(bmin, 4, 3, f) == 3 &&
                  std::fread(bmax, 4, 3, f) == 3;
        Tree t;
        t.nodes.resize(nn);
        t.hits.resize(nn);
        ok = ok && std::fread(t.nodes.data(), 8, nn, f) == nn;
        for (uint32_t i = 0; ok && i < nn; i++) {
            uint32_t nh = 0;
            ok = std::fread(&nh, 4, 1, f) == 1;
            t.hits[i].resize(nh);
            ok = ok && (nh == 0 || std::fread(t.hits[i].data(), 4, nh, f) == nh);
        }
        std::fclose(f);
        f = std::fopen(argv[3], "rb");
        uint32_t n = 0;
        ok = ok && f && std::fread(&n, 4, 1, f) == 1;
        std::vector<Ray> rays;
        for (uint32_t i = 0; ok && i < n; i++) {
            float v[8];
            ok = std::fread(v, 4, 8, f) == 8;
            Ray r;
            std::memcpy(r.o, v, 12);
            std::memcpy(r.d, v + 3, 12);
            r.shadow = v[7] != 0.f;
            if (ok && root_clip(bmin, bmax, r, v[6])) rays.push_back(r);
        }
        if (f) std::fclose(f);
        if (!ok) {
            std::fprintf(stderr, "bad input\n");
            return 1;
        }
        run(t, nrefs, rays, argc > 4 ? std::atoi(argv[4]) : 0, st);
    }
    std::printf("violations %llu rays %llu leaf_tests %llu fat_fetch_insts %llu quad_fetch_insts %llu mid_pops %llu\n",
                (unsigned long long)st.viol, (unsigned long long)st.rays, (unsigned long long)st.tests,
                (unsigned long long)st.fat, (unsigned long long)st.quad, (unsigned long long)st.mid);
    return 0;
}
