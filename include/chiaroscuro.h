/*
 * chiaroscuro.h -- C entry points of libchiaroscuro.so, the host mirror of the
 * reference's C++ classes (Scene, Model, KDTree, RayTracer), for FFI callers
 * (ctypes in this repo's tests and bench).  C++ callers use the host headers directly.
 *
 *   chiaro_scene_create      Scene::Scene(argc, argv)              src/scene.cpp:13-72
 *   chiaro_model_create      Model::Model(Scene&)                  src/model.cpp:17-36
 *   chiaro_raytracer_create  RayTracer::RayTracer(Model&, Scene&)  src/rayTracer.cpp:13-15
 *                            (builds KDTree, src/kdtree.cpp:34-108, uploads via cr_upload_scene)
 *   chiaro_raytracer_raytrace RayTracer::rayTrace                  src/rayTracer.cpp:17-74
 *   chiaro_raytracer_data / _maxval / _normalize / _export
 *                            getData / maxVal / normalizeImage / exportImage (rayTracer.cpp:171-279)
 *   chiaro_camera            the camera basis of rayTrace          src/rayTracer.cpp:41-49
 *   chiaro_preview_*         OpenGLPreview's render path without a window: camera,
 *                            key R / TAB / = / - / WASDQE, mouse, scroll, the screen
 *                            texture                               src/openglPreview.cpp:12-257,
 *                                                                  src/camera.cpp
 *
 * Errors: functions return NULL / a negative code; chiaro_last_error() (per thread)
 * gives the message.  C++ exceptions never cross this boundary.
 */
#ifndef CHIAROSCURO_H
#define CHIAROSCURO_H

#include "chiaro_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct chiaro_scene chiaro_scene;
typedef struct chiaro_model chiaro_model;
typedef struct chiaro_kdtree chiaro_kdtree;
typedef struct chiaro_raytracer chiaro_raytracer;

typedef struct {
    uint32_t xres, yres, samples, preview_height, leaf_size, seed;
    int32_t k;
    int32_t using_preview;
    float VP[3], LA[3], UP[3], background[3];
    float yview, exposure;
    uint32_t n_invalid; /* tokens reported as "Invalid argument" */
    char obj_path[1024];
    char render_path[1024];
    uint32_t gpus;      /* additive "gpus" key: GPUs the RayTracer splits a layer over */
} chiaro_scene_info;

const char *chiaro_last_error(void);

chiaro_scene *chiaro_scene_create(int argc, const char *const *argv);
int chiaro_scene_info_get(const chiaro_scene *s, chiaro_scene_info *out);
void chiaro_scene_destroy(chiaro_scene *s);

chiaro_model *chiaro_model_create(chiaro_scene *s);
chiaro_model *chiaro_model_load(const char *obj_path);
uint32_t chiaro_model_num_meshes(const chiaro_model *m);
uint32_t chiaro_model_num_triangles(const chiaro_model *m);
uint32_t chiaro_model_num_textures(const chiaro_model *m); /* loaded images */
/* Triangle soup in KDTree order: pos[9n], vnrm[9n] (vertex normals), uv[6n], kd[3n], ke[3n], tex[n]. */
int chiaro_model_triangles(const chiaro_model *m, float *pos, float *vnrm, float *uv, float *kd, float *ke,
                           int32_t *tex);
int chiaro_model_texture(const chiaro_model *m, uint32_t i, int32_t *w, int32_t *h, int32_t *nc,
                         const uint8_t **data);
void chiaro_model_destroy(chiaro_model *m);

/* KDTree without a device (host build only): for kd dumps and for callers that
 * drive libchiaro_hip.so themselves.  Appends to the scene's lightTriangles. */
chiaro_kdtree *chiaro_kdtree_create(chiaro_model *m, chiaro_scene *s, int threads);
uint32_t chiaro_kdtree_num_nodes(const chiaro_kdtree *k);
uint32_t chiaro_kdtree_num_refs(const chiaro_kdtree *k);
int chiaro_kdtree_export(const chiaro_kdtree *k, uint32_t *is_leaf, uint32_t *axis, float *split, uint32_t *child,
                         uint32_t *leaf_first, uint32_t *leaf_count, uint32_t *refs, float *box);
/* Fill the C-ABI scene description (pointers valid while k and s live). */
int chiaro_kdtree_describe(chiaro_kdtree *k, const chiaro_scene *s, cr_scene_desc *out);
void chiaro_kdtree_destroy(chiaro_kdtree *k);

chiaro_raytracer *chiaro_raytracer_create(chiaro_model *m, chiaro_scene *s, int device);
int chiaro_raytracer_raytrace(chiaro_raytracer *r, const float eye[3], const float center[3], const float up[3],
                              float yview);
/* n rayTrace calls with the same view (RayTracer::rayTraceLayers), rendered in pass groups -- on one
 * GPU (cr_render_layers) or across the `gpus` group (cr_group_render_layers); bit-identical. */
int chiaro_raytracer_raytrace_layers(chiaro_raytracer *r, uint32_t n, const float eye[3], const float center[3],
                                     const float up[3], float yview);
const float *chiaro_raytracer_pixels(const chiaro_raytracer *r);
const uint8_t *chiaro_raytracer_data(chiaro_raytracer *r);
float chiaro_raytracer_maxval(const chiaro_raytracer *r);
uint32_t chiaro_raytracer_layers(const chiaro_raytracer *r);
int chiaro_raytracer_counters(const chiaro_raytracer *r, cr_counters *out);
int chiaro_raytracer_normalize(chiaro_raytracer *r, float exposure, float defog, float knee_low, float knee_high,
                               float gamma);
int chiaro_raytracer_export(chiaro_raytracer *r, const char *filename);
cr_ctx *chiaro_raytracer_ctx(chiaro_raytracer *r);

/* Checkpoint / resume of a progressive render (the persisted counterpart of
 * src/rayTracer.cpp:18-33,64 -- layer count, last camera, running average).
 * A resumed RayTracer continues the layers where the checkpoint left them: the next
 * rayTrace at the same camera renders layer `layers + 1` and blends it into the saved
 * average, bit for bit as if the process had never stopped.  A checkpoint of another
 * frame size / spp / depth / seed / background / scene is refused (CR_E_INVALID). */
typedef struct {
    uint32_t xres, yres, samples, k, seed, layers;
    float eye[3], center[3], up[3], yview;
    float background[3];
    uint64_t scene; /* chiaro_kdtree_fingerprint of the scene the average belongs to */
} chiaro_checkpoint;
int chiaro_raytracer_checkpoint(chiaro_raytracer *r, const char *path);
int chiaro_raytracer_resume(chiaro_raytracer *r, const char *path);
uint64_t chiaro_kdtree_fingerprint(const chiaro_kdtree *k);
/* the file format itself (for a caller keeping its own frame, e.g. the multi-GPU
 * DistributedFrame): pixels [yres][xres][3]; read with pixels NULL = header only */
int chiaro_checkpoint_write(const char *path, const chiaro_checkpoint *h, const float *pixels);
int chiaro_checkpoint_read(const char *path, chiaro_checkpoint *h, float *pixels);
void chiaro_raytracer_destroy(chiaro_raytracer *r);

/* OpenEXR as the reference's exportImage writes it (FreeImage_Save(FIF_EXR, FIT_RGBF, 0),
 * src/rayTracer.cpp:229-272): channels B, G, R of HALF, PIZ compression, increasing-Y lines.
 * rgb [H][W][3] (R, G, B; row 0 = top); floats are rounded to half (nearest even, overflow to
 * infinity).  chiaro_exr_read_half reads scanline HALF R/G/B files with NO or PIZ compression;
 * with rgb NULL it returns the size only; cap = halves available at rgb. */
int chiaro_exr_write(const char *path, const float *rgb, uint32_t w, uint32_t h);
int chiaro_exr_write_half(const char *path, const uint16_t *rgb, uint32_t w, uint32_t h);
int chiaro_exr_read_half(const char *path, uint32_t *w, uint32_t *h, uint16_t *rgb, size_t cap);
int chiaro_float_to_half(const float *in, uint16_t *out, size_t n);

int chiaro_camera(const float eye[3], const float center[3], const float up[3], float yview, uint32_t xres,
                  uint32_t yres, cr_camera *out);

/* Headless preview session over a RayTracer (and its Scene: exposure keys change it). */
typedef struct chiaro_preview chiaro_preview;
enum {
    CHIARO_KEY_R = 0,     /* render a layer at the camera, show it            */
    CHIARO_KEY_TAB = 1,   /* toggle render / model view                        */
    CHIARO_KEY_EQUAL = 2, /* exposure + 0.2, re-normalise                      */
    CHIARO_KEY_MINUS = 3, /* exposure - 0.2, re-normalise                      */
    CHIARO_KEY_W = 4, CHIARO_KEY_S = 5, CHIARO_KEY_A = 6, CHIARO_KEY_D = 7, CHIARO_KEY_E = 8, CHIARO_KEY_Q = 9,
    /* a frame without a movement key: only the shift state (the speed of the next move) */
    CHIARO_KEY_SHIFT = 10
};
chiaro_preview *chiaro_preview_create(chiaro_scene *s, chiaro_raytracer *r);
/* one key press; dt = frame time for the movement keys, shift = LEFT_SHIFT held */
int chiaro_preview_key(chiaro_preview *p, int key, float dt, int shift);
int chiaro_preview_mouse(chiaro_preview *p, float xoffset, float yoffset);
int chiaro_preview_scroll(chiaro_preview *p, float yoffset);
/* the screen texture (RayTracer::getData after normalizeImage), width x height x RGB8 */
const uint8_t *chiaro_preview_texture(chiaro_preview *p, uint32_t *width, uint32_t *height);
/* camera Position, Front, Up, Zoom (degrees); show_render, renders so far */
int chiaro_preview_state(const chiaro_preview *p, float position[3], float front[3], float up[3], float *zoom,
                         int *show_render, uint32_t *renders);
void chiaro_preview_destroy(chiaro_preview *p);
/* The preview camera alone (no GPU): Camera(VP, LA, UP) with Zoom from yview, then
 * nops operations -- op 0..5 ProcessKeyboard(FORWARD..DOWNWARD, dt = a0), 6
 * ProcessMouseMovement(a0, a1), 7 ProcessMouseScroll(a0), 8 MovementSpeed = a0
 * (args: 2 per op) -- and after each: Position, Front, Up, Right, Yaw, Pitch, Zoom
 * (15 floats per op) into out.  A GL-free front-end can plan camera paths with it. */
int chiaro_preview_camera_replay(const float vp[3], const float la[3], const float up[3], float yview,
                                 const int32_t *ops, const float *args, int nops, float *out);

#ifdef __cplusplus
}
#endif
#endif
