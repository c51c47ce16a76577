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
//   packet_check <seed> <cases> [mutant]   prints "violations N rays M leaf_tests L"
// mutant 1: far-only rays not parked (tmax kept); 2: every ray's tmax set at a push, active
// or not -- both must be caught (the check has teeth).
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
};
std::vector<Node> tree;

int build(int depth, float lo[3], float hi[3]) {
    const int id = (int)tree.size();
    tree.push_back(Node());
    if (depth == 0 || rnd() < 0.06) {
        const int nh = rnd() < 0.7 ? 0 : 1 + (int)(rnd() * 3);
        for (int i = 0; i < nh; i++) tree[id].hits.push_back((float)(rnd() * 40.0 - 5.0));
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
    while (go) {
        bool popit = true;
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
            go = true;
            continue;
        }
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
    printf("violations %lld rays %lld leaf_tests %lld\n", viol, rays, tests);
    return viol ? 1 : 0;
}
