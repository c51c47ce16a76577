// model.cpp -- own OBJ/MTL loader and PNG decoder (assimp and stb_image are
// third-party libraries the reference links, Makefile:6; assimp is absent here).
//
// Semantics kept from src/model.cpp:25-151 and assimp's OBJ importer as the
// reference configures it:
//   - one Mesh per (object/group, material run) in file order (processNode order)
//   - aiProcess_Triangulate: polygons fanned from their first corner
//   - aiProcess_FlipUVs: v -> 1 - v
//   - aiProcess_GenNormals: faces without `vn` get the flat face normal
//     normalize((v1 - v0) x (v2 - v0)) on all corners
//   - material index 0 is assimp's default material, which the reference skips
//     (`mMaterialIndex > 0`, src/model.cpp:85): faces before any usemtl -> Color()
//   - MTL Kd defaults to 0.6 grey when absent (assimp ObjFile::Material); Ke, Ka, Ks
//     as given; map_Kd loaded relative to the model directory, deduplicated by path
//     (Model::loadMaterialTextures, src/model.cpp:153-174)
#include "model.hpp"
#include "scene.hpp"

#include <zlib.h>

#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>
#include <map>
#include <sstream>

namespace chiaro {

// ------------------------------------------------------------------ Mesh --
Mesh::Mesh(std::vector<Vertex> v, std::vector<unsigned int> i, std::vector<Texture> t, Color c)
    : vertices(std::move(v)), indices(std::move(i)), textures(std::move(t)), materialColor(c) {
    setupMesh();
}
Mesh::Mesh(const Mesh &o) : vertices(o.vertices), indices(o.indices), textures(o.textures), materialColor(o.materialColor) {
    setupMesh();
}
Mesh &Mesh::operator=(const Mesh &o) {
    vertices = o.vertices;
    indices = o.indices;
    textures = o.textures;
    materialColor = o.materialColor;
    textureNormal = textureHeight = textureDiffuse = textureSpecular = nullptr;
    setupMesh();
    return *this;
}
// src/mesh.cpp:136-146
void Mesh::setupMesh() {
    for (auto &t : textures) {
        if (t.type == "texture_diffuse") textureDiffuse = &t;
        else if (t.type == "texture_specular") textureSpecular = &t;
        else if (t.type == "texture_normal") textureNormal = &t;
        else if (t.type == "texture_height") textureHeight = &t;
    }
}

// ------------------------------------------------------------------- PNG --
namespace {

uint32_t be32(const unsigned char *p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }

bool decode_png(const std::vector<unsigned char> &f, std::vector<unsigned char> &out, int &W, int &H, int &NC) {
    static const unsigned char sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
    if (f.size() < 8 || std::memcmp(f.data(), sig, 8) != 0) return false;
    size_t pos = 8;
    uint32_t w = 0, h = 0;
    int depth = 0, ctype = -1, interlace = 0;
    std::vector<unsigned char> idat, plte, trns;
    while (pos + 12 <= f.size()) {
        uint32_t len = be32(&f[pos]);
        if (pos + 12 + (size_t)len > f.size()) return false;
        const unsigned char *type = &f[pos + 4], *d = &f[pos + 8];
        if (!std::memcmp(type, "IHDR", 4)) {
            if (len < 13) return false;
            w = be32(d); h = be32(d + 4); depth = d[8]; ctype = d[9]; interlace = d[12];
        } else if (!std::memcmp(type, "PLTE", 4)) plte.assign(d, d + len);
        else if (!std::memcmp(type, "tRNS", 4)) trns.assign(d, d + len);
        else if (!std::memcmp(type, "IDAT", 4)) idat.insert(idat.end(), d, d + len);
        else if (!std::memcmp(type, "IEND", 4)) break;
        pos += 12 + (size_t)len;
    }
    if (!w || !h || w > (1u << 15) || h > (1u << 15) || interlace) return false; // Adam7 unsupported: load fails
    int chan;
    switch (ctype) {
    case 0: chan = 1; break;
    case 2: chan = 3; break;
    case 3: chan = 1; break;
    case 4: chan = 2; break;
    case 6: chan = 4; break;
    default: return false;
    }
    if (!(depth == 8 || depth == 16 || (depth < 8 && (ctype == 0 || ctype == 3)))) return false;
    const size_t bpp_bits = (size_t)chan * depth;
    const size_t stride = (w * bpp_bits + 7) / 8;
    const size_t bpp = (bpp_bits + 7) / 8;
    std::vector<unsigned char> raw((stride + 1) * h);
    uLongf rl = (uLongf)raw.size();
    if (uncompress(raw.data(), &rl, idat.data(), (uLong)idat.size()) != Z_OK || rl != raw.size()) return false;
    std::vector<unsigned char> img(stride * h), prev(stride, 0);
    for (uint32_t y = 0; y < h; y++) {
        const unsigned char ft = raw[y * (stride + 1)];
        const unsigned char *src = &raw[y * (stride + 1) + 1];
        unsigned char *dst = &img[y * stride];
        for (size_t x = 0; x < stride; x++) {
            const int a = x >= bpp ? dst[x - bpp] : 0, b = prev[x], c = x >= bpp ? prev[x - bpp] : 0;
            int v = src[x];
            switch (ft) {
            case 0: break;
            case 1: v += a; break;
            case 2: v += b; break;
            case 3: v += (a + b) >> 1; break;
            case 4: {
                const int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
                v += (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c);
                break;
            }
            default: return false;
            }
            dst[x] = (unsigned char)v;
        }
        std::memcpy(prev.data(), dst, stride);
    }
    // to 8-bit, native components (stb_image req_comp = 0)
    int oc = chan;
    if (ctype == 3) oc = trns.empty() ? 3 : 4;
    out.assign((size_t)w * h * oc, 0);
    for (uint32_t y = 0; y < h; y++) {
        const unsigned char *row = &img[y * stride];
        for (uint32_t x = 0; x < w; x++) {
            unsigned char *o = &out[((size_t)y * w + x) * oc];
            if (ctype == 3) {
                uint32_t idx;
                if (depth == 8) idx = row[x];
                else idx = (row[(x * depth) / 8] >> (8 - depth - (x * depth) % 8)) & ((1u << depth) - 1);
                if (3 * idx + 2 >= plte.size()) return false;
                o[0] = plte[3 * idx]; o[1] = plte[3 * idx + 1]; o[2] = plte[3 * idx + 2];
                if (oc == 4) o[3] = idx < trns.size() ? trns[idx] : 255;
            } else if (depth == 16) {
                for (int c = 0; c < chan; c++) o[c] = row[(x * chan + c) * 2]; // stb: high byte (>>8)
            } else if (depth == 8) {
                for (int c = 0; c < chan; c++) o[c] = row[x * chan + c];
            } else { // grey < 8 bit, stb scales to 0..255
                const uint32_t v = (row[(x * depth) / 8] >> (8 - depth - (x * depth) % 8)) & ((1u << depth) - 1);
                o[0] = (unsigned char)(v * (255 / ((1u << depth) - 1)));
            }
        }
    }
    W = (int)w; H = (int)h; NC = oc;
    return true;
}

bool decode_ppm(const std::vector<unsigned char> &f, std::vector<unsigned char> &out, int &W, int &H, int &NC) {
    if (f.size() < 2 || f[0] != 'P' || (f[1] != '6' && f[1] != '5')) return false;
    int vals[3], n = 0;
    size_t p = 2;
    while (n < 3 && p < f.size()) {
        while (p < f.size() && (isspace(f[p]) || f[p] == '#')) {
            if (f[p] == '#') while (p < f.size() && f[p] != '\n') p++;
            else p++;
        }
        int v = 0;
        bool any = false;
        while (p < f.size() && isdigit(f[p])) { v = v * 10 + (f[p++] - '0'); any = true; }
        if (!any) return false;
        vals[n++] = v;
    }
    p++;
    const int nc = f[1] == '6' ? 3 : 1;
    if (n != 3 || vals[2] != 255 || vals[0] <= 0 || vals[1] <= 0) return false;
    const size_t bytes = (size_t)vals[0] * vals[1] * nc;
    if (p + bytes > f.size()) return false;
    out.assign(f.begin() + p, f.begin() + p + bytes);
    W = vals[0]; H = vals[1]; NC = nc;
    return true;
}

} // namespace

bool load_image(const std::string &file, std::vector<unsigned char> &out, int &w, int &h, int &nc) {
    std::ifstream in(file, std::ios::binary);
    if (!in) return false;
    std::vector<unsigned char> f((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
    return decode_png(f, out, w, h, nc) || decode_ppm(f, out, w, h, nc);
}

// ------------------------------------------------------------------- OBJ --
namespace {

struct ObjMaterial {
    std::string name;
    vec3 Ka{0.f}, Kd{0.6f}, Ks{0.f}, Ke{0.f};
    float Ns = 0.f;
    std::string map_Kd;
};

std::string trim(const std::string &s) {
    size_t a = s.find_first_not_of(" \t\r\n"), b = s.find_last_not_of(" \t\r\n");
    return a == std::string::npos ? std::string() : s.substr(a, b - a + 1);
}

void parse_mtl(const std::string &file, std::vector<ObjMaterial> &mats, std::map<std::string, int> &index) {
    std::ifstream in(file);
    if (!in) {
        std::cerr << "OBJ: material library " << file << " not found\n";
        return;
    }
    std::string line;
    ObjMaterial *cur = nullptr;
    while (std::getline(in, line)) {
        std::istringstream ss(line);
        std::string key;
        if (!(ss >> key) || key[0] == '#') continue;
        if (key == "newmtl") {
            std::string name;
            std::getline(ss, name);
            name = trim(name);
            if (!index.count(name)) {
                index[name] = (int)mats.size();
                mats.push_back(ObjMaterial{});
                mats.back().name = name;
            }
            cur = &mats[index[name]];
        } else if (!cur) {
            continue;
        } else if (key == "Kd" || key == "Ka" || key == "Ks" || key == "Ke") {
            float r = 0, g = 0, b = 0;
            ss >> r;
            if (!(ss >> g)) g = b = r;
            else ss >> b;
            vec3 v(r, g, b);
            (key == "Kd" ? cur->Kd : key == "Ka" ? cur->Ka : key == "Ks" ? cur->Ks : cur->Ke) = v;
        } else if (key == "Ns") {
            ss >> cur->Ns;
        } else if (key == "map_Kd") {
            std::string rest;
            std::getline(ss, rest);
            rest = trim(rest);
            // skip options (-bm 1 ...) and keep the last token as the file name
            size_t sp = rest.find_last_of(" \t");
            cur->map_Kd = sp == std::string::npos ? rest : rest.substr(sp + 1);
        }
    }
}

int obj_index(int i, size_t n) { return i > 0 ? i - 1 : (int)n + i; }

} // namespace

Model::Model(Scene &scene) { loadModel(scene.objPath); }
Model::Model(const std::string &path) { loadModel(path); }

Texture Model::textureFromFile(const std::string &path, const std::string &typeName) {
    Texture t;
    t.path = path;
    t.type = typeName;
    std::vector<unsigned char> pixels;
    int w = 0, h = 0, nc = 0;
    const std::string file = directory + '/' + path;
    if (load_image(file, pixels, w, h, nc)) {
        images_.emplace_back(new unsigned char[pixels.size()]);
        std::memcpy(images_.back().get(), pixels.data(), pixels.size());
        t.image = images_.back().get();
        t.width = w;
        t.height = h;
        t.nrComponents = nc;
    } else {
        std::cout << "Texture failed to load at path: " << path << std::endl; // src/model.cpp:144-148
        t.image = nullptr;
    }
    return t;
}

void Model::loadModel(const std::string &path) {
    std::ifstream in(path);
    if (!in) {
        error = "unable to open file \"" + path + "\"";
        std::cout << "ERROR::ASSIMP::" << error << "\n"; // src/model.cpp:29-31
        return;
    }
    const size_t slash = path.find_last_of('/');
    directory = slash == std::string::npos ? path : path.substr(0, slash); // src/model.cpp:33 (same quirk)
    if (slash == std::string::npos) directory = ".";

    std::vector<vec3> V, N;
    std::vector<vec2> T;
    std::vector<ObjMaterial> mats(1); // 0 = assimp default material
    mats[0].name = "DefaultMaterial";
    std::map<std::string, int> matIndex;
    matIndex["DefaultMaterial"] = 0;

    struct Run {
        int material = 0;
        std::vector<Vertex> verts;
    };
    std::vector<Run> runs;
    runs.emplace_back();
    int curMat = 0;
    auto newRun = [&]() {
        if (!runs.back().verts.empty()) runs.emplace_back();
        runs.back().material = curMat;
    };

    std::string line;
    while (std::getline(in, line)) {
        std::istringstream ss(line);
        std::string key;
        if (!(ss >> key) || key[0] == '#') continue;
        if (key == "v") {
            float x = 0, y = 0, z = 0;
            ss >> x >> y >> z;
            V.emplace_back(x, y, z);
        } else if (key == "vn") {
            float x = 0, y = 0, z = 0;
            ss >> x >> y >> z;
            N.emplace_back(x, y, z);
        } else if (key == "vt") {
            float u = 0, v = 0;
            ss >> u >> v;
            T.emplace_back(u, v);
        } else if (key == "o" || key == "g") {
            newRun();
        } else if (key == "usemtl") {
            std::string name;
            std::getline(ss, name);
            name = trim(name);
            auto it = matIndex.find(name);
            curMat = it == matIndex.end() ? 0 : it->second;
            newRun();
        } else if (key == "mtllib") {
            std::string name;
            std::getline(ss, name);
            parse_mtl(directory + '/' + trim(name), mats, matIndex);
            // keep material indices 1.. in library order
        } else if (key == "f") {
            struct Corner { int v, t, n; };
            std::vector<Corner> cs;
            std::string tok;
            while (ss >> tok) {
                Corner c{-1, -1, -1};
                int part = 0;
                std::string num;
                for (size_t i = 0; i <= tok.size(); i++) {
                    if (i == tok.size() || tok[i] == '/') {
                        if (!num.empty()) {
                            int val = std::stoi(num);
                            if (part == 0) c.v = obj_index(val, V.size());
                            else if (part == 1) c.t = obj_index(val, T.size());
                            else c.n = obj_index(val, N.size());
                        }
                        num.clear();
                        part++;
                    } else {
                        num += tok[i];
                    }
                }
                if (c.v < 0 || c.v >= (int)V.size()) throw std::runtime_error("OBJ: vertex index out of range");
                cs.push_back(c);
            }
            if (cs.size() < 3) continue; // points/lines are not triangulated into the mesh
            Run &r = runs.back();
            r.material = curMat;
            for (size_t i = 1; i + 1 < cs.size(); i++) { // aiProcess_Triangulate (fan)
                const Corner tri[3] = {cs[0], cs[i], cs[i + 1]};
                const bool hasN = tri[0].n >= 0 && tri[1].n >= 0 && tri[2].n >= 0 && tri[0].n < (int)N.size() &&
                                  tri[1].n < (int)N.size() && tri[2].n < (int)N.size();
                vec3 fn(0.f);
                if (!hasN) { // aiProcess_GenNormals: flat face normal, aiVector3D::NormalizeSafe
                    const vec3 a = V[tri[0].v], b = V[tri[1].v], c = V[tri[2].v];
                    vec3 n = cross(b - a, c - a);
                    const float len = std::sqrt(n.x * n.x + n.y * n.y + n.z * n.z);
                    if (len > 0.f) n = vec3(n.x / len, n.y / len, n.z / len);
                    fn = n;
                }
                for (const Corner &c : tri) {
                    Vertex vx;
                    vx.Position = V[c.v];
                    vx.Normal = hasN ? N[c.n] : fn;
                    if (c.t >= 0 && c.t < (int)T.size()) vx.TexCoords = vec2(T[c.t].x, 1.0f - T[c.t].y); // FlipUVs
                    else vx.TexCoords = vec2(0.f, 0.f);
                    r.verts.push_back(vx);
                }
            }
        }
    }

    for (Run &r : runs) {
        if (r.verts.empty()) continue;
        std::vector<unsigned int> idx(r.verts.size());
        for (size_t i = 0; i < idx.size(); i++) idx[i] = (unsigned int)i;
        Color col;
        std::vector<Texture> textures;
        if (r.material > 0) { // src/model.cpp:85-111
            const ObjMaterial &m = mats[r.material];
            col.emissive = m.Ke;
            col.diffuse = m.Kd;
            col.ambient = m.Ka;
            col.specular = m.Ks;
            col.shininess = m.Ns;
            if (!m.map_Kd.empty()) {
                bool skip = false;
                for (auto &t : textures_loaded)
                    if (t.path == m.map_Kd) {
                        textures.push_back(t);
                        skip = true;
                        break;
                    }
                if (!skip) {
                    Texture t = textureFromFile(m.map_Kd, "texture_diffuse");
                    int loaded = 0;
                    for (auto &u : textures_loaded) loaded += u.image ? 1 : 0;
                    t.index = t.image ? loaded : -1; // device texture id = rank among loaded images
                    textures.push_back(t);
                    textures_loaded.push_back(t);
                }
            }
        }
        meshes.emplace_back(std::move(r.verts), std::move(idx), std::move(textures), col);
    }
}

} // namespace chiaro
