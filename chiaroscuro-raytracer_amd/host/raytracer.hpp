// raytracer.hpp -- RayTracer (mirror of include/rayTracer.hpp:10-41).
//
// Same public API: RayTracer(Model&, Scene&), rayTrace(eye, center, up, yview),
// getData(), maxVal, normalizeImage(...), exportImage(filename).  rayTrace runs
// the render loop on the GPU through libchiaro_hip.so (include/chiaro_hip.h);
// there is no CPU render path in the product.
#pragma once
#include "kdtree.hpp"
#include "scene.hpp"

#include "chiaro_hip.h"

#include <cfloat>
#include <cstdint>
#include <stdexcept>
#include <vector>

namespace chiaro {

// Camera basis of src/rayTracer.cpp:41-49 (glm::lookAt + mat3 inverse, glm order).
cr_camera make_camera(vec3 eye, vec3 center, vec3 up, float yview, unsigned xres, unsigned yres);

class RayTracer {
  public:
    // device: HIP device index (scene.gpus > 1: GPUs device .. device + gpus - 1, the
    // layers tile-split over them, cr_group_*).  Throws std::runtime_error when no
    // GPU / the HIP library cannot be used (the product never falls back to the CPU).
    RayTracer(Model &_model, Scene &_scene, int device = 0);
    ~RayTracer();
    RayTracer(const RayTracer &) = delete;
    RayTracer &operator=(const RayTracer &) = delete;

    /* Fill pixels with rays shot on screen centered between eye and center. */
    void rayTrace(vec3 eye, vec3 center, vec3 up = vec3(0.f, 1.f, 0.f), float yview = 1.f);
    /* This build: n calls of rayTrace with the same view, rendered as pass groups
     * (cr_render_layers / cr_group_render_layers with the `gpus` key: several layers per pass group,
     * bit-identical). */
    void rayTraceLayers(unsigned n, vec3 eye, vec3 center, vec3 up = vec3(0.f, 1.f, 0.f), float yview = 1.f);
    /* Get RGB (24 bits per pixel) image location. */
    uint8_t *getData();
    /* The biggest single pixel color generated in last rayTrace() call. */
    float maxVal = 0.f;
    /* Normalize image so png and preview look somehow alike to exr output. */
    void normalizeImage(float exposure = FLT_MAX, float defog = 0.f, float kneeLow = 0.f, float kneeHigh = 5.f,
                        float gamma = 2.2f);
    /* Export: .pfm/.exr/.hdr in float, .ppm/.png 8-bit via normalizeImage. */
    void exportImage(const char *filename);

    // --- additions of this build (not in the reference API) ---
    const float *pixelData() const { return pixels.data(); } // [yres][xres][3], row 0 = top
    unsigned layers() const { return layers_; }
    cr_ctx *context() { return ctx_; }          // with gpus > 1: the root GPU's ctx
    cr_group *group() { return group_; }        // gpus > 1, else null
    KDTree &tree() { return kdtree; }
    const cr_counters &lastCounters() const { return counters_; }
    // checkpoint / resume of the progressive state (host/checkpoint.hpp); resume throws
    // std::runtime_error for a checkpoint of another frame, sampling or scene
    void saveCheckpoint(const char *path) const;
    void resume(const char *path);
    double lastSeconds() const { return lastSeconds_; }

  private:
    Scene &scene;
    std::vector<float> pixels; // replaces std::vector<std::vector<glm::vec3>>
    std::vector<uint8_t> data;
    KDTree kdtree;
    cr_ctx *ctx_ = nullptr;
    cr_group *group_ = nullptr;
    cr_counters counters_{};
    double lastSeconds_ = 0.0;
    // rayTracer.cpp:18-22 progressive-layer state (per instance here, not function-static)
    unsigned layers_ = 0;
    vec3 lastEye{FLT_MAX}, lastCenter{FLT_MAX}, lastUp{FLT_MAX};
    float lastYview = -1;
};

} // namespace chiaro
