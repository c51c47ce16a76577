// main.cpp -- offline front-end, the counterpart of the reference's main.cpp:5-21
// with the render loop on the MI355X:
//
//   bin/chiaroscuro scene.rtc [rtc tokens...]
//
// Scene(argc, argv) -> Model(scene) -> RayTracer(model, scene) ->
// rayTrace(VP, LA, UP, yview) -> exportImage(renderPath), as the reference's
// offline branch.  The OpenGL preview is not part of this build:
// with "preview" enabled in the .rtc the scene is rendered offline instead.
// Extra token "layers N" (this build): render N progressive layers of the same
// view (the reference's preview accumulates them the same way,
// src/rayTracer.cpp:17-33, src/openglPreview.cpp:247-255).
#include "model.hpp"
#include "raytracer.hpp"
#include "scene.hpp"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <string>
#include <vector>

int main(int argc, char **argv) {
    // strip this build's own tokens before Scene sees them
    unsigned layers = 1;
    std::vector<char *> args;
    for (int i = 0; i < argc; i++) {
        if (i > 1 && !std::strcmp(argv[i], "layers") && i + 1 < argc) {
            layers = (unsigned)std::max(1, std::atoi(argv[++i]));
            continue;
        }
        args.push_back(argv[i]);
    }
    try {
        chiaro::Scene scene((int)args.size(), args.data());
        if (scene.usingOpenGLPreview)
            std::fprintf(stderr, "chiaroscuro: OpenGL preview not built; rendering offline (add no-preview)\n");
        chiaro::Model model(scene);
        if (!model.error.empty()) std::fprintf(stderr, "%s\n", model.error.c_str());
        chiaro::RayTracer renderer(model, scene);
        // the layers in pass groups (RayTracer::rayTraceLayers, bit-identical to one rayTrace per layer)
        renderer.rayTraceLayers(layers, scene.VP, scene.LA, scene.UP, scene.yview);
        std::fprintf(stderr, "layers 1..%u: %.3f s, %llu rays\n", renderer.layers(), renderer.lastSeconds(),
                     (unsigned long long)(renderer.lastCounters().closest + renderer.lastCounters().shadow));
        renderer.exportImage(scene.renderPath.c_str());
    } catch (const std::exception &e) {
        std::fprintf(stderr, "chiaroscuro: %s\n", e.what());
        return 1;
    }
    return 0;
}
