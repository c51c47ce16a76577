/*
 * oracle.h -- CPU restatement of Chiaroscuro's per-pixel render loop.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load liboracle.so, and only as the checker /
 * the timed CPU baseline.  The product (libchiaro_hip.so + libchiaroscuro.so)
 * never links, loads or calls anything in this directory.
 *
 * Parity status (see DESIGN.md "Oracle"): the reference as shipped does not
 * build (src/prng.cpp and include/prng.hpp are missing; kdtree.cpp/rayTracer.cpp
 * need assimp/FreeImage headers absent from this image), so the traversal, kd
 * build, BRDF and integrator restated here are PARITY UNPINNED by the reference
 * itself.  The pieces that DO compile from the reference's own sources without
 * stand-ins -- Texture::getColorAt (src/mesh.cpp:21-35) and the vendored glm
 * 0.9.8.5 arithmetic used by rayTrace's camera (src/rayTracer.cpp:41-49) and by
 * normalize/cross/dot/distance -- are pinned against tests/golden/ref_*.json,
 * produced by oracle/ref (oracle/_ref build).
 */
#ifndef CHIARO_ORACLE_H
#define CHIARO_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct or_scene or_scene;

/* Counters, in the order of cr_counters (include/chiaro_hip.h). */
enum {
    OR_C_CLOSEST = 0, /* calls equivalent to KDTree::intersectRay          */
    OR_C_SHADOW,      /* calls equivalent to KDTree::intersectShadowRay    */
    OR_C_INNER,       /* inner kd nodes visited                            */
    OR_C_LEAF,        /* leaves visited                                    */
    OR_C_TRITEST,     /* Moller-Trumbore tests executed                    */
    OR_C_HIT,         /* closest-hit queries that hit                      */
    OR_C_TEXHIT,      /* hits shaded through Texture::getColorAt           */
    OR_C_PATHS,       /* camera paths                                      */
    OR_C_COUNT
};

/* Build the scene from the flattened triangle soup, in Model::meshes order
 * (src/kdtree.cpp:34-108).  Per triangle t:
 *   pos[9t..]   A,B,C world positions       vnrm[9t..] vertex normals n0,n1,n2
 *   uv[6t..]    texcoords of A,B,C           kd[3t..], ke[3t..] mesh colours
 *   tex[t]      diffuse texture index or -1  */
or_scene *or_scene_create(uint32_t ntri, const float *pos, const float *vnrm, const float *uv, const float *kd,
                          const float *ke, const int32_t *tex, uint32_t leaf_size, int build_threads);
int or_scene_add_texture(or_scene *s, int w, int h, int nc, const uint8_t *data);
void or_scene_destroy(or_scene *s);

/* kd-tree dump (G1).  Node i: meta = leaf ? (3 | count<<2) : (axis | child<<2) stored
 * as two arrays (is_leaf/axis/child + split bits); leaf lists concatenated. */
uint32_t or_kd_num_nodes(const or_scene *s);
uint32_t or_kd_num_refs(const or_scene *s);
uint32_t or_kd_max_depth(const or_scene *s);
void or_kd_export(const or_scene *s, uint32_t *is_leaf, uint32_t *axis, float *split, uint32_t *child,
                  uint32_t *leaf_first, uint32_t *leaf_count, uint32_t *refs, float *box /* min3 max3, padded */);
uint32_t or_num_lights(const or_scene *s);
void or_lights(const or_scene *s, uint32_t *ids, float *surface);

/* Camera basis exactly as src/rayTracer.cpp:41-49.  out = eye3, leftUpper3, dx3, dy3. */
void or_camera(const float eye[3], const float center[3], const float up[3], float yview, uint32_t xres,
               uint32_t yres, float out[12]);

/* Ray KAT (G2). hit[i]=0/1; tri, bary(2), dist written on hit. */
void or_intersect(or_scene *s, uint32_t n, const float *orig, const float *dir, uint32_t *hit, uint32_t *tri,
                  float *bary, float *dist);
void or_intersect_shadow(or_scene *s, uint32_t n, const float *orig, const float *dir, const float *dist,
                         const uint32_t *light, uint32_t *occluded);

/* BRDF KAT (G3): Diffuse::sample_wi with scripted disk draws sx, sy. */
void or_sample_wi(const float n[3], float sx, float sy, float wi[3], float *pdf);
void or_concentric(float sx, float sy, float *dx, float *dy);
void or_sincos(float x, float *s, float *c);

/* Texture KAT (G5). */
void or_tex_lookup(const or_scene *s, int tex, float u, float v, float out[3]);

/* RNG stream (DESIGN.md "RNG"): n raw u32 draws of stream (seed, layer, pixel, sample). */
void or_rng_draws(uint32_t seed, uint32_t layer, uint32_t pixel, uint32_t sample, uint32_t n, uint32_t *out);

/* Path KAT (G4): radiance of one camera sample, recursion exactly as sendRay. */
void or_path(or_scene *s, const float cam[12], uint32_t xres, uint32_t yres, int k, const float bg[3],
             uint32_t seed, uint32_t layer, uint32_t x, uint32_t y, uint32_t sample, float out[3]);

/* Render rows [y0, y1) with row stride ystep of layer `layer`:
 *   pixels = (old * (L-1) + mean) / L   (src/rayTracer.cpp:64)
 * `pix` is [yres][xres][3] in/out (only touched rows change).  threads<=0: all
 * OpenMP threads; otherwise that many.  counters: OR_C_COUNT uint64. */
void or_render(or_scene *s, const float cam[12], uint32_t xres, uint32_t yres, uint32_t spp, int k,
               const float bg[3], uint32_t seed, uint32_t layer, uint32_t y0, uint32_t y1, uint32_t ystep,
               int threads, float *pix, uint64_t *counters);

/* Batch means (no blend) of n listed pixels (px[i], py[i]) of layer `layer`:
 * mean[3i..] = (sum over samples of sendRay) * (1/spp); counters summed (may be NULL). */
void or_render_pixels(or_scene *s, const float cam[12], uint32_t xres, uint32_t yres, uint32_t spp, int k,
                      const float bg[3], uint32_t seed, uint32_t layer, uint32_t n, const uint32_t *px,
                      const uint32_t *py, int threads, float *mean, uint64_t *counters);

/* glm / kd-tree primitives (pinned by tests/golden/ref_glm.json) */
void or_glm_normalize(const float a[3], float out[3]);
void or_glm_cross(const float a[3], const float b[3], float out[3]);
float or_glm_dot(const float a[3], const float b[3]);
float or_glm_distance(const float a[3], const float b[3]);
void or_material_normal(const float n[9], float out[3]);
float or_light_surface(const float p[9]);
/* rayTracer.cpp:172-222 normalizeImage (glibc powf / logf), rows flipped */
void or_tonemap(const float *rgb, uint32_t xres, uint32_t yres, float exposure, float defog, float kneeLow,
                float kneeHigh, float gamma, uint8_t *out);

/* trig mode: 0 = restatement of glibc sinf / cosf (bit-exact with the HIP path and
 * with libm on every |x| < 120), 1 = call the host libm sinf / cosf */
void or_set_trig_mode(int mode);
uint64_t or_sincos_check(uint32_t lo, uint32_t hi, uint32_t stride, int both_signs, int threads);

#ifdef __cplusplus
}
#endif
#endif
