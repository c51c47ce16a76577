// scene.cpp -- .rtc parsing with the semantics of src/scene.cpp:13-72.
#include "scene.hpp"

#include <fstream>
#include <iostream>

namespace chiaro {

// src/scene.cpp:63-72: defaults, then every non-empty line of the file is a token.
Scene::Scene(const std::string &filename)
    : renderPath("renders/output.exr"), k(3), xres(400), yres(300), VP(0, 0, 2), LA(0, 0, 0), UP(0, 1, 0), yview(1),
      usingOpenGLPreview(true), previewHeight(900), kdtreeLeafSize(8), background(0), samples(100), exposure(5),
      seed(0xC41A05C0u), gpus(1), rtcPath(filename) {
    std::ifstream file(filename);
    std::string input;
    while (std::getline(file, input)) {
        if (input.length() > 0) params.push_back(input);
    }
}

// src/scene.cpp:13-60.  std::stoi/stof throw on malformed numbers exactly as in
// the reference; the C API turns that into an error code.
Scene::Scene(int argc, char **argv) : Scene(std::string(argc > 1 ? argv[1] : "cornell.rtc")) {
    for (int i = 2; i < argc; i++) params.emplace_back(argv[i]);

    auto next = [&](unsigned &i) -> const std::string & {
        if (i + 1 >= params.size()) throw std::out_of_range("missing value after \"" + params[i] + "\"");
        return params[++i];
    };
    for (unsigned i = 0; i < params.size(); i++) {
        const std::string &p = params[i];
        if (p[0] == '#')
            continue;
        else if (p == "no-preview")
            usingOpenGLPreview = false;
        else if (p == "input")
            objPath = next(i);
        else if (p == "output")
            renderPath = next(i);
        else if (p == "k")
            k = std::stoi(next(i));
        else if (p == "xres")
            xres = std::stoi(next(i));
        else if (p == "yres")
            yres = std::stoi(next(i));
        else if (p == "VP" || p == "LA" || p == "UP" || p == "background") {
            const float x = std::stof(next(i));
            const float y = std::stof(next(i));
            const float z = std::stof(next(i));
            (p == "VP" ? VP : p == "LA" ? LA : p == "UP" ? UP : background) = vec3(x, y, z);
        } else if (p == "yview")
            yview = std::stof(next(i));
        else if (p == "preview-height")
            previewHeight = std::stoi(next(i));
        else if (p == "samples")
            samples = std::stoi(next(i));
        else if (p == "exposure")
            exposure = std::stof(next(i));
        else if (p == "kdtree-leaf-size")
            kdtreeLeafSize = std::stoi(next(i));
        else if (p == "seed")
            seed = (uint32_t)std::stoul(next(i), nullptr, 0);
        else if (p == "gpus")
            gpus = (unsigned)std::stoul(next(i));
        else {
            std::cerr << "Invalid argument \"" << p << "\"\n";
            errors.push_back(p);
        }
    }
}

} // namespace chiaro
