// kdtree.hpp -- KDTree (mirror of include/kdtree.hpp:15-77).
//
// Built on the host exactly as src/kdtree.cpp:34-194 builds it (same triangle
// ids, light order, node order and split floats -- the kernels consume them), but
// with the 300 split candidates of every node evaluated in parallel and large
// subtrees built concurrently, then numbered in the reference's allocation order.
// Traversal (intersectRay / intersectShadowRay) runs on the GPU through the C-ABI.
#pragma once
#include "model.hpp"
#include "scene.hpp"

#include "chiaro_hip.h"

#include <vector>

namespace chiaro {

enum class BRDFT { Diffuse, Emissive }; // include/brdf.hpp:8

struct Triangle { // include/kdtree.hpp:15-18
    vec3 posFst, posSnd, posTrd;
};

struct Material { // include/kdtree.hpp:20-33
    BRDFT BRDFtype;
    vec3 normal;
    vec3 Kd;
    vec3 Ke;
    Texture *texDiffuse;
    vec2 texFst, texSnd, texTrd;
    int texIndex; // device texture id, -1 if none or not loaded
};

class KDTree {
  public:
    const size_t leafSize;
    KDTree(Model &model, Scene &scene, int threads = 0);

    // GPU-backed queries (KDTree::intersectRay / intersectShadowRay, src/kdtree.cpp:210-216, 283-290).
    // Require attach(); return false and set lastError on failure.
    bool intersectRay(const vec3 &origin, const vec3 &dir, id_t &triangle, vec2 &baryPosition, float &distance);
    bool intersectShadowRay(const vec3 &origin, const vec3 &dir, const float distance, const id_t lightTriangle);
    void attach(cr_ctx *ctx) { ctx_ = ctx; }

    std::vector<Triangle> triangles;
    std::vector<Material> materials;
    vec3 minCoords;
    vec3 maxCoords;

    struct KDNode { // include/kdtree.hpp:47-60 with the leaf list as a range of `refs`
        uint32_t first = 0, count = 0;
        id_t child = 0;
        struct Split {
            id_t axis;
            float position;
        } split{3, 0.f};
        bool isLeaf = true;
    };
    std::vector<KDNode> nodes;
    std::vector<id_t> refs;
    uint32_t maxDepth = 0;
    std::vector<const Texture *> deviceTextures; // index = Material::texIndex

    // Fill the C-ABI description (pointers stay valid while this KDTree lives).
    void describe(const Scene &scene, cr_scene_desc &d);

    std::string lastError;

  private:
    cr_ctx *ctx_ = nullptr;
    // flattened views for describe()
    std::vector<cr_kdnode> cnodes_;
    std::vector<float> pos_, nrm_, kd_, ke_, uv_;
    std::vector<int32_t> tex_;
    std::vector<uint8_t> emis_;
    std::vector<uint32_t> lid_;
    std::vector<float> lsurf_;
    std::vector<cr_texture> ctex_;
};

} // namespace chiaro
