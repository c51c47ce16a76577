// scene.hpp -- Scene: the .rtc configuration (mirror of include/scene.hpp:24-59).
#pragma once
#include "vec.hpp"

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace chiaro {

using id_t = uint32_t;

struct LightPoint { // include/scene.hpp:11-16 (parsed by nobody in the reference either)
    LightPoint(vec3 color, vec3 position, float intensity) : color(color), position(position), intensity(intensity) {}
    vec3 color, position;
    float intensity;
};

struct LightTriangle { // include/scene.hpp:18-22
    LightTriangle(id_t i, float s) : id(i), surface(s) {}
    id_t id;
    float surface;
};

class Scene {
  public:
    // src/scene.cpp:13-60: argv[1] = .rtc path (default cornell.rtc), argv[2..]
    // appended as further tokens, so they override the file.
    Scene(int argc, char **argv);

    std::string objPath;
    std::string renderPath;
    int k;
    unsigned xres;
    unsigned yres;
    vec3 VP, LA, UP;
    float yview;
    std::vector<LightPoint> lightPoints;
    bool usingOpenGLPreview;
    unsigned int previewHeight;
    size_t kdtreeLeafSize;
    vec3 background;
    unsigned int samples;
    std::vector<LightTriangle> lightTriangles; // filled by KDTree
    std::vector<std::string> params;
    float exposure;
    // additive keys of this build (not in the reference): "seed", "background",
    // "gpus" (the RayTracer tile-splits each layer over GPUs 0..gpus-1, cr_group_*)
    uint32_t seed;
    unsigned gpus;
    std::string rtcPath;   // argv[1] as given
    std::vector<std::string> errors; // "Invalid argument" lines also printed to stderr

  private:
    explicit Scene(const std::string &filename);
};

} // namespace chiaro
