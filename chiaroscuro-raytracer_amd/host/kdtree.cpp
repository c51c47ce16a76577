// kdtree.cpp -- host kd-tree construction with the exact semantics of
// src/kdtree.cpp:34-194, parallelised without changing a single float:
//   * every split candidate keeps its own sequential cost sum over the node's
//     triangles in order (so candidates can run side by side, vectorised);
//   * the best candidate is picked in the reference's (axis, ratio) order with `<`;
//   * subtrees are built as OpenMP tasks into a temporary tree, then numbered in
//     the reference's allocation order (children pair appended when the parent is
//     built, left subtree completed before the right one).
#include "kdtree.hpp"

#include <cfloat>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <memory>
#include <stdexcept>

#ifdef _OPENMP
#include <omp.h>
#endif

namespace chiaro {

namespace {

struct TmpNode {
    bool leaf = true;
    uint32_t axis = 3;
    float split = 0.f;
    uint32_t depth = 0;
    std::vector<id_t> ids;
    std::unique_ptr<TmpNode> l, r;
};

struct Builder {
    const std::vector<Triangle> &tri;
    size_t leafSize;
    std::vector<float> ratios;
    explicit Builder(const std::vector<Triangle> &t, size_t ls) : tri(t), leafSize(ls) {
        for (float r = 0.01f; r < 1.0f; r += 0.01f) ratios.push_back(r); // kdtree.cpp:116
    }

    // kdtree.cpp:110-141 findSplit
    void findSplit(const std::vector<id_t> &tris, const vec3 &mx, const vec3 &mn, uint32_t &bestAxis,
                   float &bestSplit) const {
        const int NR = (int)ratios.size();
        const size_t n = tris.size();
        std::vector<float> split(3 * NR), cost(3 * NR, 0.f), omr(NR);
        std::vector<uint32_t> lc(3 * NR, 0), rc(3 * NR, 0);
        for (int i = 0; i < NR; i++) omr[i] = 1.f - ratios[i];
        for (int ax = 0; ax < 3; ax++)
            for (int i = 0; i < NR; i++) split[ax * NR + i] = mn[ax] + ratios[i] * (mx[ax] - mn[ax]);
        auto run_axis = [&](int ax) {
            float *c = cost.data() + ax * NR;
            uint32_t *L = lc.data() + ax * NR, *R = rc.data() + ax * NR;
            const float *sp = split.data() + ax * NR;
            const float *ra = ratios.data();
            for (size_t j = 0; j < n; j++) {
                const Triangle &t = tri[tris[j]];
                const float a = t.posFst[ax], b = t.posSnd[ax], cc = t.posTrd[ax];
                for (int i = 0; i < NR; i++) {
                    const float s = sp[i];
                    const bool l = (a <= s) | (b <= s) | (cc <= s); // inLeft, kdtree.cpp:22-24
                    const bool r = (a >= s) | (b >= s) | (cc >= s); // inRight, kdtree.cpp:26-28
                    c[i] += l ? ra[i] : 0.f; // += 0.f is exact: cost never becomes -0
                    c[i] += r ? omr[i] : 0.f;
                    L[i] += l;
                    R[i] += r;
                }
            }
        };
        if (n > 16384) {
#pragma omp taskloop grainsize(1)
            for (int ax = 0; ax < 3; ax++) run_axis(ax);
        } else {
            for (int ax = 0; ax < 3; ax++) run_axis(ax);
        }
        uint32_t bax = 3;
        float bsp = 0.f, bcost = float(n);
        for (int k = 0; k < 3 * NR; k++)
            if (lc[k] < n && rc[k] < n && cost[k] < bcost) {
                bax = (uint32_t)(k / NR);
                bsp = split[k];
                bcost = cost[k];
            }
        bestAxis = bax;
        bestSplit = bsp;
    }

    float triMin(id_t t, int a) const { // kdtree.cpp:16-20
        float m = tri[t].posFst[a];
        m = tri[t].posSnd[a] < m ? tri[t].posSnd[a] : m;
        return tri[t].posTrd[a] < m ? tri[t].posTrd[a] : m;
    }
    float triMax(id_t t, int a) const { // kdtree.cpp:10-14
        float m = tri[t].posFst[a];
        m = tri[t].posSnd[a] > m ? tri[t].posSnd[a] : m;
        return tri[t].posTrd[a] > m ? tri[t].posTrd[a] : m;
    }

    // kdtree.cpp:143-194 build
    void build(TmpNode *node, std::vector<id_t> tris, vec3 mx, vec3 mn) const {
        uint32_t ax = 3;
        float sp = 0.f;
        if (!(tris.size() <= leafSize)) findSplit(tris, mx, mn, ax, sp);
        if (tris.size() <= leafSize || ax == 3) {
            node->leaf = true;
            node->ids = std::move(tris);
            return;
        }
        node->leaf = false;
        node->axis = ax;
        node->split = sp;
        node->l.reset(new TmpNode());
        node->r.reset(new TmpNode());
        node->l->depth = node->r->depth = node->depth + 1;
        std::vector<id_t> kids[2];
        vec3 kmn[2], kmx[2];
        for (int side = 0; side < 2; side++) {
            vec3 cmn(FLT_MAX, FLT_MAX, FLT_MAX), cmx(-FLT_MAX, -FLT_MAX, -FLT_MAX);
            std::vector<id_t> &child = kids[side];
            for (id_t t : tris) {
                const Triangle &T = tri[t];
                const float a0 = T.posFst[ax], a1 = T.posSnd[ax], a2 = T.posTrd[ax];
                const bool in = side == 0 ? (a0 <= sp || a1 <= sp || a2 <= sp) : (a0 >= sp || a1 >= sp || a2 >= sp);
                if (!in) continue;
                child.push_back(t);
                int a = (int)ax;
                for (int q = 0; q < 3; q++) {
                    cmn[a] = std_min(cmn[a], triMin(t, a));
                    cmx[a] = std_max(cmx[a], triMax(t, a));
                    a = (a + 1) % 3;
                }
            }
            kmn[side] = cmn;
            kmx[side] = cmx;
        }
        std::vector<id_t>().swap(tris);
        for (int side = 0; side < 2; side++) {
            TmpNode *c = side == 0 ? node->l.get() : node->r.get();
            if (kids[side].size() > 4096) {
#pragma omp task firstprivate(c, side) shared(kids, kmn, kmx)
                build(c, std::move(kids[side]), kmx[side], kmn[side]);
            } else {
                build(c, std::move(kids[side]), kmx[side], kmn[side]);
            }
        }
#pragma omp taskwait
    }
};

} // namespace

KDTree::KDTree(Model &model, Scene &scene, int threads)
    : leafSize(scene.kdtreeLeafSize), minCoords(FLT_MAX, FLT_MAX, FLT_MAX), maxCoords(FLT_MIN, FLT_MIN, FLT_MIN) {
    size_t indicesCount = 0;
    for (auto &mesh : model.meshes) indicesCount += mesh.indices.size();
    triangles.reserve((indicesCount + 2) / 3);
    std::vector<id_t> triangleIDs;
    triangleIDs.reserve((indicesCount + 2) / 3);
    for (auto &tex : model.textures_loaded)
        if (tex.image) deviceTextures.push_back(&tex);

    // kdtree.cpp:44-85
    for (auto &mesh : model.meshes) {
        const bool isLight = mesh.materialColor.emissive.x > 0.f || mesh.materialColor.emissive.y > 0.f ||
                             mesh.materialColor.emissive.z > 0.f;
        for (unsigned i = 0; i + 2 < mesh.indices.size(); i += 3) {
            const id_t triangleId = (id_t)triangles.size();
            const Vertex &v0 = mesh.vertices[mesh.indices[i]], &v1 = mesh.vertices[mesh.indices[i + 1]],
                         &v2 = mesh.vertices[mesh.indices[i + 2]];
            triangles.push_back({v0.Position, v1.Position, v2.Position});
            Material m;
            m.BRDFtype = isLight ? BRDFT::Emissive : BRDFT::Diffuse;
            m.normal = (v0.Normal + v1.Normal + v2.Normal) / 3.f;
            m.Kd = mesh.materialColor.diffuse;
            m.Ke = mesh.materialColor.emissive;
            m.texDiffuse = mesh.textureDiffuse;
            m.texFst = v0.TexCoords;
            m.texSnd = v1.TexCoords;
            m.texTrd = v2.TexCoords;
            m.texIndex = (mesh.textureDiffuse && mesh.textureDiffuse->image) ? mesh.textureDiffuse->index : -1;
            materials.push_back(m);
            if (isLight) {
                const Triangle &T = triangles[triangleId];
                const float surface = 0.5f * length(cross(T.posSnd - T.posFst, T.posTrd - T.posFst));
                scene.lightTriangles.push_back(LightTriangle(triangleId, surface));
            }
            for (const Vertex *v : {&v0, &v1, &v2})
                for (int j = 0; j < 3; j++) {
                    if (!std::isfinite(v->Position[j])) throw std::runtime_error("non-finite vertex position");
                    minCoords[j] = std_min(v->Position[j], minCoords[j]);
                    maxCoords[j] = std_max(v->Position[j], maxCoords[j]);
                }
            triangleIDs.push_back(triangleId);
        }
    }

    // kdtree.cpp:89-90: build on the unpadded box
    Builder B(triangles, leafSize);
    TmpNode root;
#ifdef _OPENMP
    const int nth = threads > 0 ? threads : omp_get_max_threads();
#pragma omp parallel num_threads(nth)
#pragma omp single
#endif
    B.build(&root, std::move(triangleIDs), maxCoords, minCoords);
    (void)threads;

    // number in allocation order
    nodes.assign(1, KDNode());
    struct Frame {
        const TmpNode *t;
        uint32_t idx;
    };
    std::vector<Frame> st{{&root, 0}};
    while (!st.empty()) {
        Frame f = st.back();
        st.pop_back();
        if (f.t->depth > maxDepth) maxDepth = f.t->depth;
        KDNode n;
        if (f.t->leaf) {
            n.isLeaf = true;
            n.first = (uint32_t)refs.size();
            n.count = (uint32_t)f.t->ids.size();
            refs.insert(refs.end(), f.t->ids.begin(), f.t->ids.end());
            nodes[f.idx] = n;
        } else {
            n.isLeaf = false;
            n.split = {f.t->axis, f.t->split};
            n.child = (id_t)nodes.size();
            nodes.resize(nodes.size() + 2);
            nodes[f.idx] = n;
            // pre-order, left first: push right then left
            st.push_back({f.t->r.get(), n.child + 1});
            st.push_back({f.t->l.get(), n.child});
        }
    }

    if (!std::getenv("CHIARO_QUIET")) { // kdtree.cpp:91-104
        std::cout << "Triangles in scene: " << triangles.size() << "\n";
        std::cout << "Surface Lights in scene: " << scene.lightTriangles.size()
                  << (scene.lightTriangles.empty() ? " None.\n" : "\n");
    }
    // kdtree.cpp:106-107
    minCoords = vec3(minCoords.x - 0.0001f, minCoords.y - 0.0001f, minCoords.z - 0.0001f);
    maxCoords = vec3(maxCoords.x + 0.0001f, maxCoords.y + 0.0001f, maxCoords.z + 0.0001f);
}

void KDTree::describe(const Scene &scene, cr_scene_desc &d) {
    const size_t nt = triangles.size();
    cnodes_.resize(nodes.size());
    for (size_t i = 0; i < nodes.size(); i++) {
        const KDNode &n = nodes[i];
        cnodes_[i] = n.isLeaf ? cr_kdnode{0.f, 3u, n.first, n.count} : cr_kdnode{n.split.position, n.split.axis, n.child, 0u};
    }
    pos_.resize(9 * nt);
    nrm_.resize(3 * nt);
    kd_.resize(3 * nt);
    ke_.resize(3 * nt);
    uv_.resize(6 * nt);
    tex_.resize(nt);
    emis_.resize(nt);
    for (size_t t = 0; t < nt; t++) {
        const Triangle &T = triangles[t];
        const Material &M = materials[t];
        const vec3 P[3] = {T.posFst, T.posSnd, T.posTrd};
        for (int v = 0; v < 3; v++)
            for (int j = 0; j < 3; j++) pos_[9 * t + 3 * v + j] = P[v][j];
        for (int j = 0; j < 3; j++) {
            nrm_[3 * t + j] = M.normal[j];
            kd_[3 * t + j] = M.Kd[j];
            ke_[3 * t + j] = M.Ke[j];
        }
        const vec2 U[3] = {M.texFst, M.texSnd, M.texTrd};
        for (int v = 0; v < 3; v++) {
            uv_[6 * t + 2 * v] = U[v].x;
            uv_[6 * t + 2 * v + 1] = U[v].y;
        }
        tex_[t] = M.texIndex;
        emis_[t] = M.BRDFtype == BRDFT::Emissive ? 1 : 0;
    }
    lid_.clear();
    lsurf_.clear();
    for (auto &l : scene.lightTriangles) {
        lid_.push_back(l.id);
        lsurf_.push_back(l.surface);
    }
    ctex_.clear();
    for (const Texture *t : deviceTextures) ctex_.push_back(cr_texture{t->width, t->height, t->nrComponents, t->image});

    std::memset(&d, 0, sizeof d);
    d.n_nodes = (uint32_t)cnodes_.size();
    d.nodes = cnodes_.data();
    d.n_refs = (uint32_t)refs.size();
    d.refs = refs.data();
    d.max_depth = maxDepth;
    d.box_min[0] = minCoords.x; d.box_min[1] = minCoords.y; d.box_min[2] = minCoords.z;
    d.box_max[0] = maxCoords.x; d.box_max[1] = maxCoords.y; d.box_max[2] = maxCoords.z;
    d.n_tris = (uint32_t)nt;
    d.tri_pos = pos_.data();
    d.tri_normal = nrm_.data();
    d.tri_kd = kd_.data();
    d.tri_ke = ke_.data();
    d.tri_uv = uv_.data();
    d.tri_tex = tex_.data();
    d.tri_emissive = emis_.data();
    d.n_lights = (uint32_t)lid_.size();
    d.light_id = lid_.data();
    d.light_surface = lsurf_.data();
    d.n_textures = (uint32_t)ctex_.size();
    d.textures = ctex_.data();
}

bool KDTree::intersectRay(const vec3 &origin, const vec3 &dir, id_t &triangle, vec2 &baryPosition, float &distance) {
    if (!ctx_) {
        lastError = "KDTree not attached to a device context";
        return false;
    }
    const float o[3] = {origin.x, origin.y, origin.z}, d[3] = {dir.x, dir.y, dir.z};
    uint32_t hit = 0, tri = 0;
    float bary[2] = {0, 0}, dist = 0;
    if (cr_intersect(ctx_, 1, o, d, &hit, &tri, bary, &dist) != CR_OK) {
        lastError = cr_last_error(ctx_);
        return false;
    }
    if (!hit) return false;
    triangle = tri;
    baryPosition = vec2(bary[0], bary[1]);
    distance = dist;
    return true;
}

bool KDTree::intersectShadowRay(const vec3 &origin, const vec3 &dir, const float distance, const id_t lightTriangle) {
    if (!ctx_) {
        lastError = "KDTree not attached to a device context";
        return false;
    }
    const float o[3] = {origin.x, origin.y, origin.z}, d[3] = {dir.x, dir.y, dir.z};
    uint32_t occ = 0, light = lightTriangle;
    if (cr_intersect_shadow(ctx_, 1, o, d, &distance, &light, &occ) != CR_OK) {
        lastError = cr_last_error(ctx_);
        return false;
    }
    return occ != 0;
}

} // namespace chiaro
