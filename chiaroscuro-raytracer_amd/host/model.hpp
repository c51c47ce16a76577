// model.hpp -- Model / Mesh / Texture / Color (mirror of include/model.hpp and
// include/mesh.hpp), GL-free.  The loader is this build's own OBJ/MTL reader
// (assimp is not available) reproducing the post-processing the reference asks
// assimp for (src/model.cpp:27): Triangulate | FlipUVs | GenNormals.
#pragma once
#include "vec.hpp"

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

namespace chiaro {

class Scene;

struct Vertex { // include/mesh.hpp:11-15
    vec3 Position;
    vec3 Normal;
    vec2 TexCoords;
};

struct Texture { // include/mesh.hpp:17-26 (image owned by the Model)
    unsigned int id = 0;
    std::string type;
    std::string path;
    unsigned char *image = nullptr;
    int width = 0, height = 0, nrComponents = 0;
    int index = -1; // position in Model::textures_loaded (device texture id)
};

struct Color { // include/mesh.hpp:28-36
    Color() : ambient(0.f), diffuse(0.f), specular(0.f), emissive(0.f), shininess(1) {}
    vec3 ambient, diffuse, specular, emissive;
    float shininess;
};

class Mesh { // include/mesh.hpp:38-59
  public:
    Mesh(std::vector<Vertex> vertices, std::vector<unsigned int> indices, std::vector<Texture> textures,
         Color materialColor);
    Mesh(const Mesh &o);
    Mesh &operator=(const Mesh &o);
    bool hasTexture() const { return textureNormal || textureHeight || textureDiffuse || textureSpecular; }

    std::vector<Vertex> vertices;
    std::vector<unsigned int> indices;
    std::vector<Texture> textures;
    Color materialColor;
    Texture *textureNormal = nullptr;
    Texture *textureHeight = nullptr;
    Texture *textureDiffuse = nullptr;
    Texture *textureSpecular = nullptr;

  private:
    void setupMesh(); // src/mesh.cpp:110-147 minus the GL buffers
};

class Model { // include/model.hpp:20-32
  public:
    explicit Model(Scene &scene);
    explicit Model(const std::string &path);
    std::vector<Mesh> meshes;
    std::vector<Texture> textures_loaded;
    std::string error; // non-empty if the file could not be read (reference prints ERROR::ASSIMP::)

  private:
    std::string directory;
    std::vector<std::unique_ptr<unsigned char[]>> images_;
    void loadModel(const std::string &path);
    Texture textureFromFile(const std::string &path, const std::string &typeName);
};

// PNG / binary-PPM decoder with stb_image's req_comp = 0 behaviour (native
// component count; palette -> RGB or RGBA; 16-bit -> 8-bit).  Returns false on failure.
bool load_image(const std::string &file, std::vector<unsigned char> &out, int &w, int &h, int &nc);

} // namespace chiaro
