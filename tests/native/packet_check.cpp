// packet_check.cpp -- CPU model check of the packet camera-ray traversal of trace
// builds 17 / 18 (csrc/wavefront.hip wf_trace_packet): the algorithm, restated on
// plain arrays, against the per-ray recursive traversal of kdtree.cpp:248-281.
//
// Random kd trees (random axes and splits, random depth), rays from one common eye in
// random directions with random initial intervals, leaves holding random "hit
// distances" (a leaf accepts the smallest distance in [0, tmax) -- the traversal only
// needs WHICH leaf answers, the triangle test itself is the same code both ways), and
// random subtree / leaf culls per (node, ray) standing in for the cull boxes (a culled
// node is left exactly as if its subtree held nothing).  The packet model runs the
// kernel's steps: wave-uniform node stream, per-ray intervals and active flags, a
// stack entry per push holding each ray's tmax at push or INACTIVE, tmin restored on
// pop from the ray's current tmax (the kd stack invariant), far-only rays parked with
// tmax = tmin.  For every ray the sequence of (leaf, tmin, tmax) tests and the answer
// must equal the recursion's.
//   packet_check <seed> <cases> [mutant]   prints "violations N rays M leaf_tests L spec S spec_used U spec_bad B"
// mutant 1: far-only rays not parked (tmax kept); 2: every ray's tmax set at a push, active
// or not -- both must be caught (the check has teeth).
// The speculative load of build 48 (wf_trace_packet SPEC): at every fetch the kernel computes, from the
// fetched fat record alone, the near-near grandchild whose records it loads ahead.  The model encodes
// every node as the kernel's words (inner: split bits, axis | child << 2; leaf: first reference,
// 3 | count << 2 -- a leaf's `first` runs far past the node count) and checks each speculative index: it
// must come from an inner record and lie inside the tree (spec_bad counts the others; the run fails).
// mutant 3: the near child's record not checked for a leaf, its child index read from the word a leaf
// keeps its first reference in (the unguarded form) -- must be caught.  (An index from an inner record is
// a child of the tree, always inside it: the kernel's bound check only backs that up.)
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

struct Node {
    int axis = -1;  // -1: leaf
    float split = 0;
    int child = -1; // children at child, child + 1
    std::vector<float> hits; // leaf: hit distances
    uint32_t first = 0, count = 0; // leaf: its reference range (the kernel's leaf words)
};
std::vector<Node> tree;

int build(int depth, float lo[3], float hi[3]) {
    const int id = (int)tree.size();
    tree.push_back(Node());
    if (depth == 0 || rnd() < 0.06) {
        const int nh = rnd() < 0.7 ? 0 : 1 + (int)(rnd() * 3);
        for (int i = 0; i < nh; i++) tree[id].hits.push_back((float)(rnd() * 40.0 - 5.0));
        tree[id].count = 1 + (uint32_t)(rnd() * 12); // (first is numbered after the build, in node order)
        return id;
    }
    const int a = (int)(rnd() * 3);
    const float s = lo[a] + (float)rnd() * (hi[a] - lo[a]);
    tree[id].axis = a;
    tree[id].split = s;
    const int c = (int)tree.size();
    tree.push_back(Node());
    tree.push_back(Node());
    tree[id].child = c;
    float h0[3] = {hi[0], hi[1], hi[2]}, l1[3] = {lo[0], lo[1], lo[2]};
    h0[a] = s;
    l1[a] = s;
    // build the subtrees into fresh slots, then move them to c, c + 1
    const int s0 = build(depth - 1, lo, h0), s1 = build(depth - 1, l1, hi);
    tree[c] = tree[s0];
    tree[c + 1] = tree[s1];
    tree[s0] = Node(); // orphaned slots stay as empty leaves
    tree[s1] = Node();
    return id;
}

// deterministic per (node, ray) cull: the ray skips the node's subtree
uint32_t cull_seed;
int mutant = 0;
bool culled(int node, int ray) {
    uint32_t x = (uint32_t)node * 0x9E3779B1u ^ (uint32_t)ray * 0x85EBCA77u ^ cull_seed;
    x ^= x >> 15;
    x *= 0x2C1B3C6Du;
    x ^= x >> 12;
    return (x & 1023u) < 24u; // ~2.3%
}

struct Rec {
    int leaf;
    float t0, t1;
};
float eye[3];

// kdtree.cpp:248-281 as a recursion; a culled node returns "no hit" at once.
bool ref(int ray, int node, const float d[3], float tmin, float tmax, std::vector<Rec> &log, float &best) {
    if (culled(node, ray)) return false;
    const Node &n = tree[node];
    if (n.axis < 0) {
        log.push_back({node, tmin, tmax});
        bool f = false;
        for (float h : n.hits)
            if (h >= 0.f && h < tmax) {
                tmax = h;
                best = h;
                f = true;
            }
        return f;
    }
    const float oa = eye[n.axis], da = d[n.axis];
    const float tsplit = (n.split - oa) / da;
    const int below = oa < n.split ? 1 : 0;
    const int nearc = n.child + (1 - below), farc = n.child + below;
    if (tsplit >= tmax || tsplit < 0) return ref(ray, nearc, d, tmin, tmax, log, best);
    if (tsplit <= tmin) return ref(ray, farc, d, tmin, tmax, log, best);
    if (ref(ray, nearc, d, tmin, tsplit, log, best)) return true;
    return ref(ray, farc, d, tsplit, tmax, log, best);
}

// the kernel's two words of node n (cr_upload_scene's encoding)
void words(int n, uint32_t &x, uint32_t &y) {
    const Node &t = tree[n];
    if (t.axis < 0) {
        x = t.first;
        y = 3u | t.count << 2;
    } else {
        memcpy(&x, &t.split, 4);
        y = (uint32_t)t.axis | (uint32_t)t.child << 2;
    }
}
long long spec_n = 0, spec_used = 0, spec_bad = 0;
// build 48's speculative index after fetching node cn (0xffffffff: none), from the fat record's words
uint32_t speculate(int cn) {
    uint32_t x0, y0;
    words(cn, x0, y0);
    if ((y0 & 3u) == 3u) return 0xffffffffu;
    float s0;
    memcpy(&s0, &x0, 4);
    const uint32_t a0 = y0 & 3u, c0 = y0 >> 2;
    const bool below0 = eye[a0] < s0;
    uint32_t rx, ry;
    words((int)(below0 ? c0 : c0 + 1), rx, ry); // the near child's record, in the fat record
    uint32_t gc;
    if (mutant == 3) { // unguarded: a leaf's record taken for an inner one, its first word as the index
        gc = ((ry & 3u) == 3u) ? rx : (ry >> 2);
    } else {
        if ((ry & 3u) == 3u) return 0xffffffffu;
        float s1;
        memcpy(&s1, &rx, 4);
        gc = (ry >> 2) + (eye[ry & 3u] < s1 ? 0u : 1u);
    }
    if (mutant != 3 && gc >= tree.size()) return 0xffffffffu;
    spec_n++;
    const bool inner_src = (ry & 3u) != 3u;
    if (gc >= tree.size() || !inner_src) spec_bad++;
    return gc;
}

// The packet traversal of wf_trace_packet<R, S> (S rays per lane x 64 lanes = the packet).
void packet(int nr, const std::vector<std::vector<float>> &dir, std::vector<float> tmin, std::vector<float> tmax,
            std::vector<std::vector<Rec>> &log, std::vector<int> &found, std::vector<float> &best) {
    const uint32_t INACTIVE = 0xffffffffu;
    std::vector<char> active(nr, 1);
    struct Entry {
        int node;
        std::vector<uint32_t> t;
    };
    std::vector<Entry> stack;
    auto bits = [](float f) {
        uint32_t u;
        memcpy(&u, &f, 4);
        return u;
    };
    auto flt = [](uint32_t u) {
        float f;
        memcpy(&f, &u, 4);
        return f;
    };
    auto any = [&]() {
        for (int r = 0; r < nr; r++)
            if (active[r]) return true;
        return false;
    };
    int cn = 0;
    bool go = any();
    uint32_t spec = 0xffffffffu;
    int lvl_fetch = 0; // levels since the last fetch (the kernel fetches every two levels)
    while (go) {
        bool popit = true;
        if (lvl_fetch == 0) { // a fetch: the speculative index of its record (SPEC)
            if ((uint32_t)cn == spec) spec_used++;
            spec = speculate(cn);
        }
        for (;;) {
            for (int r = 0; r < nr; r++) active[r] = active[r] && !culled(cn, r); // the node's box
            if (!any()) break;
            const Node &n = tree[cn];
            if (n.axis < 0) {
                for (int r = 0; r < nr; r++) {
                    if (!active[r]) continue;
                    log[r].push_back({cn, tmin[r], tmax[r]});
                    for (float h : n.hits)
                        if (h >= 0.f && h < tmax[r]) {
                            tmax[r] = h;
                            best[r] = h;
                            found[r] = 1;
                        }
                }
                break;
            }
            const float oa = eye[n.axis];
            const int below = oa < n.split ? 1 : 0;
            const int nearc = n.child + (1 - below), farc = n.child + below;
            std::vector<float> tsp(nr);
            std::vector<char> crosses(nr), after(nr), to_near(nr), to_far(nr);
            bool anyn = false, anyf = false;
            for (int r = 0; r < nr; r++) {
                tsp[r] = (n.split - oa) / dir[r][n.axis];
                crosses[r] = !(tsp[r] >= tmax[r]) && !(tsp[r] < 0.f);
                after[r] = !(tsp[r] <= tmin[r]);
                to_near[r] = active[r] && (!crosses[r] || after[r]);
                to_far[r] = active[r] && crosses[r];
                anyn = anyn || to_near[r];
                anyf = anyf || to_far[r];
            }
            if (!anyn) {
                cn = farc;
            } else {
                if (anyf) {
                    Entry e{farc, std::vector<uint32_t>(nr)};
                    for (int r = 0; r < nr; r++) e.t[r] = to_far[r] ? bits(tmax[r]) : INACTIVE;
                    stack.push_back(e);
                }
                for (int r = 0; r < nr; r++) {
                    const float nt = after[r] ? tsp[r] : (mutant == 1 ? tmax[r] : tmin[r]);
                    tmax[r] = (to_far[r] || (mutant == 2 && crosses[r] && after[r])) ? nt : tmax[r];
                    active[r] = to_near[r];
                }
                cn = nearc;
            }
            popit = false;
            break; // fetch cn (the kernel's two-level fat step is the same sequence of decisions)
        }
        if (!popit) {
            lvl_fetch = (lvl_fetch + 1) & 1; // (two levels per fetched fat record)
            go = true;
            continue;
        }
        lvl_fetch = 0; // a pop fetches its node
        go = false;
        while (!stack.empty()) {
            Entry e = stack.back();
            stack.pop_back();
            cn = e.node;
            bool a = false;
            for (int r = 0; r < nr; r++) {
                const bool act = !found[r] && e.t[r] != INACTIVE;
                if (act) {
                    tmin[r] = tmax[r]; // the stack invariant
                    tmax[r] = flt(e.t[r]);
                }
                active[r] = act;
                a = a || act;
            }
            if (a) {
                go = true;
                break;
            }
        }
    }
}

} // namespace

int main(int argc, char **argv) {
    rs ^= (uint64_t)strtoull(argc > 1 ? argv[1] : "1", nullptr, 10) * 0x9E3779B97F4A7C15ull;
    const int cases = argc > 2 ? atoi(argv[2]) : 200;
    mutant = argc > 3 ? atoi(argv[3]) : 0;
    long long viol = 0, rays = 0, tests = 0;
    for (int cs = 0; cs < cases; cs++) {
        tree.clear();
        float lo[3] = {-10, -10, -10}, hi[3] = {10, 10, 10};
        build(6 + (int)(rnd() * 11), lo, hi);
        uint32_t refs = 0;
        for (Node &n : tree)
            if (n.axis < 0) {
                n.first = refs; // leaves' reference ranges in node order: past the node count soon
                refs += n.count;
            }
        cull_seed = (uint32_t)next();
        for (int i = 0; i < 3; i++) eye[i] = (float)(rnd() * 16.0 - 8.0);
        // an eye exactly on a split plane breaks the common near child: the host then uses
        // build 15 (RenderArgs::eye_on_split), so such cases are not the packet's
        bool on_split = false;
        for (const Node &n : tree)
            if (n.axis >= 0 && n.split == eye[n.axis]) on_split = true;
        if (on_split) continue;
        const int nr = 128; // build 18's packet (two rays per lane)
        std::vector<std::vector<float>> dir(nr, std::vector<float>(3));
        std::vector<float> t0(nr), t1(nr);
        const float base[3] = {(float)(rnd() * 2 - 1), (float)(rnd() * 2 - 1), (float)(rnd() * 2 - 1)};
        const float spread = (float)pow(10.0, rnd() * 3 - 3);
        for (int r = 0; r < nr; r++) {
            for (int i = 0; i < 3; i++) {
                dir[r][i] = base[i] + spread * (float)(rnd() * 2 - 1);
                if (rnd() < 0.02) dir[r][i] = 0.f; // axis-parallel components: infinite tsplit
            }
            t0[r] = rnd() < 0.5 ? 0.f : (float)(rnd() * 5);
            t1[r] = t0[r] + (float)(rnd() * 40);
        }
        std::vector<std::vector<Rec>> lr(nr), lp(nr);
        std::vector<int> fr(nr), fp(nr, 0);
        std::vector<float> br(nr, -1.f), bp(nr, -1.f);
        for (int r = 0; r < nr; r++) fr[r] = ref(r, 0, dir[r].data(), t0[r], t1[r], lr[r], br[r]) ? 1 : 0;
        packet(nr, dir, t0, t1, lp, fp, bp);
        for (int r = 0; r < nr; r++) {
            rays++;
            tests += (long long)lr[r].size();
            bool same = fr[r] == fp[r] && br[r] == bp[r] && lr[r].size() == lp[r].size();
            for (size_t i = 0; same && i < lr[r].size(); i++)
                same = lr[r][i].leaf == lp[r][i].leaf && lr[r][i].t0 == lp[r][i].t0 && lr[r][i].t1 == lp[r][i].t1;
            if (!same) {
                if (viol < 5)
                    fprintf(stderr, "VIOLATION case %d ray %d: ref %zu leaves found %d, packet %zu leaves found %d\n", cs,
                            r, lr[r].size(), fr[r], lp[r].size(), fp[r]);
                viol++;
            }
        }
    }
    printf("violations %lld rays %lld leaf_tests %lld spec %lld spec_used %lld spec_bad %lld\n", viol, rays, tests,
           spec_n, spec_used, spec_bad);
    return viol || spec_bad ? 1 : 0;
}
