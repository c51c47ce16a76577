// capi.cpp -- extern "C" wrappers of the host classes (include/chiaroscuro.h).
#include "chiaroscuro.h"

#include "kdtree.hpp"
#include "model.hpp"
#include "preview.hpp"
#include "checkpoint.hpp"
#include "exr.hpp"
#include "raytracer.hpp"
#include "scene.hpp"

#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <memory>
#include <string>
#include <vector>

using namespace chiaro;

struct chiaro_scene {
    std::unique_ptr<Scene> s;
};
struct chiaro_model {
    std::unique_ptr<Model> m;
};
struct chiaro_kdtree {
    std::unique_ptr<KDTree> k;
};
struct chiaro_raytracer {
    std::unique_ptr<RayTracer> r;
};
struct chiaro_preview {
    std::unique_ptr<PreviewSession> p;
};

namespace {
thread_local std::string g_err;
template <class F> auto guard(F f, decltype(f()) bad) -> decltype(f()) {
    try {
        g_err.clear();
        return f();
    } catch (const std::exception &e) {
        g_err = e.what();
    } catch (...) {
        g_err = "unknown C++ exception";
    }
    return bad;
}
void cpy(char *dst, const std::string &s, size_t n) {
    std::strncpy(dst, s.c_str(), n - 1);
    dst[n - 1] = 0;
}
} // namespace

extern "C" {

const char *chiaro_last_error(void) { return g_err.c_str(); }

chiaro_scene *chiaro_scene_create(int argc, const char *const *argv) {
    return guard(
        [&]() -> chiaro_scene * {
            std::vector<char *> a;
            for (int i = 0; i < argc; i++) a.push_back(const_cast<char *>(argv[i]));
            a.push_back(nullptr);
            auto *s = new chiaro_scene();
            s->s.reset(new Scene(argc, a.data()));
            return s;
        },
        (chiaro_scene *)nullptr);
}

int chiaro_scene_info_get(const chiaro_scene *s, chiaro_scene_info *o) {
    if (!s || !o) return CR_E_INVALID;
    const Scene &S = *s->s;
    std::memset(o, 0, sizeof *o);
    o->xres = S.xres;
    o->yres = S.yres;
    o->samples = S.samples;
    o->preview_height = S.previewHeight;
    o->leaf_size = (uint32_t)S.kdtreeLeafSize;
    o->seed = S.seed;
    o->k = S.k;
    o->using_preview = S.usingOpenGLPreview ? 1 : 0;
    for (int i = 0; i < 3; i++) {
        o->VP[i] = S.VP[i];
        o->LA[i] = S.LA[i];
        o->UP[i] = S.UP[i];
        o->background[i] = S.background[i];
    }
    o->yview = S.yview;
    o->exposure = S.exposure;
    o->n_invalid = (uint32_t)S.errors.size();
    cpy(o->obj_path, S.objPath, sizeof o->obj_path);
    cpy(o->render_path, S.renderPath, sizeof o->render_path);
    o->gpus = S.gpus;
    return CR_OK;
}

void chiaro_scene_destroy(chiaro_scene *s) { delete s; }

chiaro_model *chiaro_model_create(chiaro_scene *s) {
    if (!s) return nullptr;
    return guard(
        [&]() -> chiaro_model * {
            auto *m = new chiaro_model();
            m->m.reset(new Model(*s->s));
            if (!m->m->error.empty()) {
                g_err = m->m->error;
                delete m;
                return nullptr;
            }
            return m;
        },
        (chiaro_model *)nullptr);
}

chiaro_model *chiaro_model_load(const char *path) {
    if (!path) return nullptr;
    return guard(
        [&]() -> chiaro_model * {
            auto *m = new chiaro_model();
            m->m.reset(new Model(std::string(path)));
            if (!m->m->error.empty()) {
                g_err = m->m->error;
                delete m;
                return nullptr;
            }
            return m;
        },
        (chiaro_model *)nullptr);
}

uint32_t chiaro_model_num_meshes(const chiaro_model *m) { return m ? (uint32_t)m->m->meshes.size() : 0; }

uint32_t chiaro_model_num_triangles(const chiaro_model *m) {
    if (!m) return 0;
    size_t n = 0;
    for (auto &mesh : m->m->meshes) n += mesh.indices.size() / 3;
    return (uint32_t)n;
}

uint32_t chiaro_model_num_textures(const chiaro_model *m) {
    if (!m) return 0;
    uint32_t n = 0;
    for (auto &t : m->m->textures_loaded) n += t.image ? 1 : 0;
    return n;
}

int chiaro_model_triangles(const chiaro_model *m, float *pos, float *vnrm, float *uv, float *kd, float *ke,
                           int32_t *tex) {
    if (!m) return CR_E_INVALID;
    size_t t = 0;
    for (auto &mesh : m->m->meshes) {
        const int ti = (mesh.textureDiffuse && mesh.textureDiffuse->image) ? mesh.textureDiffuse->index : -1;
        for (size_t i = 0; i + 2 < mesh.indices.size(); i += 3, t++) {
            for (int v = 0; v < 3; v++) {
                const Vertex &V = mesh.vertices[mesh.indices[i + v]];
                for (int j = 0; j < 3; j++) {
                    if (pos) pos[9 * t + 3 * v + j] = V.Position[j];
                    if (vnrm) vnrm[9 * t + 3 * v + j] = V.Normal[j];
                }
                if (uv) {
                    uv[6 * t + 2 * v] = V.TexCoords.x;
                    uv[6 * t + 2 * v + 1] = V.TexCoords.y;
                }
            }
            for (int j = 0; j < 3; j++) {
                if (kd) kd[3 * t + j] = mesh.materialColor.diffuse[j];
                if (ke) ke[3 * t + j] = mesh.materialColor.emissive[j];
            }
            if (tex) tex[t] = ti;
        }
    }
    return CR_OK;
}

int chiaro_model_texture(const chiaro_model *m, uint32_t i, int32_t *w, int32_t *h, int32_t *nc,
                         const uint8_t **data) {
    if (!m) return CR_E_INVALID;
    uint32_t k = 0;
    for (auto &t : m->m->textures_loaded) {
        if (!t.image) continue;
        if (k++ == i) {
            *w = t.width;
            *h = t.height;
            *nc = t.nrComponents;
            *data = t.image;
            return CR_OK;
        }
    }
    return CR_E_INVALID;
}

void chiaro_model_destroy(chiaro_model *m) { delete m; }

chiaro_kdtree *chiaro_kdtree_create(chiaro_model *m, chiaro_scene *s, int threads) {
    if (!m || !s) return nullptr;
    return guard(
        [&]() -> chiaro_kdtree * {
            auto *k = new chiaro_kdtree();
            k->k.reset(new KDTree(*m->m, *s->s, threads));
            return k;
        },
        (chiaro_kdtree *)nullptr);
}

uint32_t chiaro_kdtree_num_nodes(const chiaro_kdtree *k) { return k ? (uint32_t)k->k->nodes.size() : 0; }
uint32_t chiaro_kdtree_num_refs(const chiaro_kdtree *k) { return k ? (uint32_t)k->k->refs.size() : 0; }

int chiaro_kdtree_export(const chiaro_kdtree *k, uint32_t *is_leaf, uint32_t *axis, float *split, uint32_t *child,
                         uint32_t *leaf_first, uint32_t *leaf_count, uint32_t *refs, float *box) {
    if (!k) return CR_E_INVALID;
    const KDTree &K = *k->k;
    for (size_t i = 0; i < K.nodes.size(); i++) {
        const auto &n = K.nodes[i];
        is_leaf[i] = n.isLeaf;
        axis[i] = n.isLeaf ? 3u : n.split.axis;
        split[i] = n.isLeaf ? 0.f : n.split.position;
        child[i] = n.isLeaf ? 0u : n.child;
        leaf_first[i] = n.isLeaf ? n.first : 0u;
        leaf_count[i] = n.isLeaf ? n.count : 0u;
    }
    std::memcpy(refs, K.refs.data(), K.refs.size() * sizeof(uint32_t));
    box[0] = K.minCoords.x; box[1] = K.minCoords.y; box[2] = K.minCoords.z;
    box[3] = K.maxCoords.x; box[4] = K.maxCoords.y; box[5] = K.maxCoords.z;
    return CR_OK;
}

int chiaro_kdtree_describe(chiaro_kdtree *k, const chiaro_scene *s, cr_scene_desc *out) {
    if (!k || !s || !out) return CR_E_INVALID;
    return guard(
        [&]() -> int {
            k->k->describe(*s->s, *out);
            return CR_OK;
        },
        CR_E_INVALID);
}

void chiaro_kdtree_destroy(chiaro_kdtree *k) { delete k; }

chiaro_raytracer *chiaro_raytracer_create(chiaro_model *m, chiaro_scene *s, int device) {
    if (!m || !s) return nullptr;
    return guard(
        [&]() -> chiaro_raytracer * {
            auto *r = new chiaro_raytracer();
            try {
                r->r.reset(new RayTracer(*m->m, *s->s, device));
            } catch (...) {
                delete r;
                throw;
            }
            return r;
        },
        (chiaro_raytracer *)nullptr);
}

int chiaro_raytracer_raytrace(chiaro_raytracer *r, const float eye[3], const float center[3], const float up[3],
                              float yview) {
    if (!r) return CR_E_INVALID;
    return guard(
        [&]() -> int {
            r->r->rayTrace(vec3(eye[0], eye[1], eye[2]), vec3(center[0], center[1], center[2]),
                           vec3(up[0], up[1], up[2]), yview);
            return CR_OK;
        },
        CR_E_HIP);
}

int chiaro_raytracer_raytrace_layers(chiaro_raytracer *r, uint32_t n, const float eye[3], const float center[3],
                                     const float up[3], float yview) {
    if (!r || n < 1) return CR_E_INVALID;
    return guard(
        [&]() -> int {
            r->r->rayTraceLayers(n, vec3(eye[0], eye[1], eye[2]), vec3(center[0], center[1], center[2]),
                                 vec3(up[0], up[1], up[2]), yview);
            return CR_OK;
        },
        CR_E_HIP);
}

const float *chiaro_raytracer_pixels(const chiaro_raytracer *r) { return r ? r->r->pixelData() : nullptr; }
const uint8_t *chiaro_raytracer_data(chiaro_raytracer *r) { return r ? r->r->getData() : nullptr; }
float chiaro_raytracer_maxval(const chiaro_raytracer *r) { return r ? r->r->maxVal : 0.f; }
uint32_t chiaro_raytracer_layers(const chiaro_raytracer *r) { return r ? r->r->layers() : 0; }
int chiaro_raytracer_counters(const chiaro_raytracer *r, cr_counters *out) {
    if (!r || !out) return CR_E_INVALID;
    *out = r->r->lastCounters();
    return CR_OK;
}
int chiaro_raytracer_normalize(chiaro_raytracer *r, float exposure, float defog, float kl, float kh, float gamma) {
    if (!r) return CR_E_INVALID;
    return guard(
        [&]() -> int {
            r->r->normalizeImage(exposure, defog, kl, kh, gamma);
            return CR_OK;
        },
        CR_E_HIP);
}
int chiaro_raytracer_export(chiaro_raytracer *r, const char *filename) {
    if (!r || !filename) return CR_E_INVALID;
    return guard(
        [&]() -> int {
            r->r->exportImage(filename);
            return CR_OK;
        },
        CR_E_INVALID);
}
cr_ctx *chiaro_raytracer_ctx(chiaro_raytracer *r) { return r ? r->r->context() : nullptr; }

int chiaro_raytracer_checkpoint(chiaro_raytracer *r, const char *path) {
    if (!r || !path) return CR_E_INVALID;
    return guard(
        [&]() -> int {
            r->r->saveCheckpoint(path);
            return CR_OK;
        },
        CR_E_INVALID);
}

int chiaro_raytracer_resume(chiaro_raytracer *r, const char *path) {
    if (!r || !path) return CR_E_INVALID;
    return guard(
        [&]() -> int {
            r->r->resume(path);
            return CR_OK;
        },
        CR_E_INVALID);
}

uint64_t chiaro_kdtree_fingerprint(const chiaro_kdtree *k) { return k ? scene_fingerprint(*k->k) : 0; }

static void write_file(const char *path, const std::vector<unsigned char> &bytes) {
    FILE *f = std::fopen(path, "wb");
    if (!f) throw std::runtime_error("cannot open " + std::string(path));
    const bool ok = std::fwrite(bytes.data(), 1, bytes.size(), f) == bytes.size();
    if (std::fclose(f) != 0 || !ok) throw std::runtime_error("cannot write " + std::string(path));
}

int chiaro_exr_write(const char *path, const float *rgb, uint32_t w, uint32_t h) {
    if (!path || !rgb || !w || !h) return CR_E_INVALID;
    return guard(
        [&]() -> int {
            write_file(path, chiaro::exr_encode(rgb, (int)w, (int)h));
            return CR_OK;
        },
        CR_E_INVALID);
}

int chiaro_exr_write_half(const char *path, const uint16_t *rgb, uint32_t w, uint32_t h) {
    if (!path || !rgb || !w || !h) return CR_E_INVALID;
    return guard(
        [&]() -> int {
            write_file(path, chiaro::exr_encode_half(rgb, (int)w, (int)h));
            return CR_OK;
        },
        CR_E_INVALID);
}

int chiaro_exr_read_half(const char *path, uint32_t *w, uint32_t *h, uint16_t *rgb, size_t cap) {
    if (!path || !w || !h) return CR_E_INVALID;
    return guard(
        [&]() -> int {
            FILE *f = std::fopen(path, "rb");
            if (!f) throw std::runtime_error("cannot open " + std::string(path));
            std::vector<unsigned char> bytes;
            unsigned char buf[1 << 16];
            size_t n;
            while ((n = std::fread(buf, 1, sizeof(buf), f)) > 0) bytes.insert(bytes.end(), buf, buf + n);
            std::fclose(f);
            int W = 0, H = 0;
            std::vector<uint16_t> px;
            std::string err;
            if (!chiaro::exr_decode_half(bytes.data(), bytes.size(), W, H, px, err))
                throw std::runtime_error(std::string(path) + ": " + err);
            *w = (uint32_t)W;
            *h = (uint32_t)H;
            if (rgb) {
                if (cap < px.size()) throw std::runtime_error("rgb buffer too small");
                std::memcpy(rgb, px.data(), px.size() * sizeof(uint16_t));
            }
            return CR_OK;
        },
        CR_E_INVALID);
}

int chiaro_float_to_half(const float *in, uint16_t *out, size_t n) {
    if ((!in || !out) && n) return CR_E_INVALID;
    for (size_t i = 0; i < n; i++) out[i] = chiaro::float_to_half(in[i]);
    return CR_OK;
}

int chiaro_checkpoint_write(const char *path, const chiaro_checkpoint *h, const float *pixels) {
    if (!path || !h || !pixels) return CR_E_INVALID;
    return guard(
        [&]() -> int {
            checkpoint_write(path, *h, pixels);
            return CR_OK;
        },
        CR_E_INVALID);
}

int chiaro_checkpoint_read(const char *path, chiaro_checkpoint *h, float *pixels) {
    if (!path || !h) return CR_E_INVALID;
    return guard(
        [&]() -> int {
            checkpoint_read(path, *h, pixels);
            return CR_OK;
        },
        CR_E_INVALID);
}
void chiaro_raytracer_destroy(chiaro_raytracer *r) { delete r; }

int chiaro_camera(const float eye[3], const float center[3], const float up[3], float yview, uint32_t xres,
                  uint32_t yres, cr_camera *out) {
    if (!eye || !center || !up || !out || !xres || !yres) return CR_E_INVALID;
    *out = make_camera(vec3(eye[0], eye[1], eye[2]), vec3(center[0], center[1], center[2]), vec3(up[0], up[1], up[2]),
                       yview, xres, yres);
    return CR_OK;
}

} // extern "C"

chiaro_preview *chiaro_preview_create(chiaro_scene *s, chiaro_raytracer *r) {
    if (!s || !r) return nullptr;
    return guard(
        [&]() -> chiaro_preview * {
            auto *p = new chiaro_preview();
            p->p.reset(new PreviewSession(*s->s, *r->r));
            return p;
        },
        (chiaro_preview *)nullptr);
}

int chiaro_preview_key(chiaro_preview *p, int key, float dt, int shift) {
    if (!p) return CR_E_INVALID;
    return guard(
        [&]() -> int {
            PreviewSession &P = *p->p;
            switch (key) {
            case CHIARO_KEY_R: P.pressRender(); break;
            case CHIARO_KEY_TAB: P.toggleView(); break;
            case CHIARO_KEY_EQUAL: P.exposureUp(); break;
            case CHIARO_KEY_MINUS: P.exposureDown(); break;
            case CHIARO_KEY_W: P.move(FORWARD, dt, shift != 0); break;
            case CHIARO_KEY_S: P.move(BACKWARD, dt, shift != 0); break;
            case CHIARO_KEY_A: P.move(LEFT, dt, shift != 0); break;
            case CHIARO_KEY_D: P.move(RIGHT, dt, shift != 0); break;
            case CHIARO_KEY_E: P.move(UPWARD, dt, shift != 0); break;
            case CHIARO_KEY_Q: P.move(DOWNWARD, dt, shift != 0); break;
            case CHIARO_KEY_SHIFT: P.shiftState(shift != 0); break;
            default: return CR_E_INVALID;
            }
            return CR_OK;
        },
        CR_E_HIP);
}

int chiaro_preview_mouse(chiaro_preview *p, float xoffset, float yoffset) {
    if (!p) return CR_E_INVALID;
    p->p->look(xoffset, yoffset);
    return CR_OK;
}

int chiaro_preview_scroll(chiaro_preview *p, float yoffset) {
    if (!p) return CR_E_INVALID;
    p->p->scroll(yoffset);
    return CR_OK;
}

const uint8_t *chiaro_preview_texture(chiaro_preview *p, uint32_t *w, uint32_t *h) {
    if (!p) return nullptr;
    if (w) *w = p->p->width();
    if (h) *h = p->p->height();
    return p->p->texture();
}

int chiaro_preview_state(const chiaro_preview *p, float pos[3], float front[3], float up[3], float *zoom,
                         int *show_render, uint32_t *renders) {
    if (!p) return CR_E_INVALID;
    const PreviewCamera &c = p->p->camera;
    for (int i = 0; i < 3; i++) {
        if (pos) pos[i] = c.Position[i];
        if (front) front[i] = c.Front[i];
        if (up) up[i] = c.Up[i];
    }
    if (zoom) *zoom = c.Zoom;
    if (show_render) *show_render = p->p->showRender ? 1 : 0;
    if (renders) *renders = p->p->renders;
    return CR_OK;
}

void chiaro_preview_destroy(chiaro_preview *p) { delete p; }

int chiaro_preview_camera_replay(const float vp[3], const float la[3], const float up[3], float yview,
                                 const int32_t *ops, const float *args, int nops, float *out) {
    if (!vp || !la || !up || nops < 0 || (nops && (!ops || !args || !out))) return CR_E_INVALID;
    PreviewCamera c(vec3(vp[0], vp[1], vp[2]), vec3(la[0], la[1], la[2]), vec3(up[0], up[1], up[2]));
    c.Zoom = preview_zoom(yview);
    for (int i = 0; i < nops; i++) {
        const float a0 = args[2 * i], a1 = args[2 * i + 1];
        if (ops[i] >= 0 && ops[i] <= 5) c.ProcessKeyboard((CameraMovement)ops[i], a0);
        else if (ops[i] == 6) c.ProcessMouseMovement(a0, a1);
        else if (ops[i] == 7) c.ProcessMouseScroll(a0);
        else if (ops[i] == 8) c.MovementSpeed = a0;
        else return CR_E_INVALID;
        const vec3 v[4] = {c.Position, c.Front, c.Up, c.Right};
        float *o = out + 15 * (size_t)i;
        for (int k = 0; k < 4; k++)
            for (int j = 0; j < 3; j++) o[3 * k + j] = v[k][j];
        o[12] = c.Yaw;
        o[13] = c.Pitch;
        o[14] = c.Zoom;
    }
    return CR_OK;
}
