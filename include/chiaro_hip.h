/*
 * chiaro_hip.h -- the drop-in C-ABI boundary of the MI355X path-tracing core.
 *
 * Exported by libchiaro_hip.so.  Plain pointers and sizes only: no C++, no
 * glm, no torch, no hipError_t crosses this boundary.  Every call returns 0
 * (CR_OK) or a negative CR_E_* code; cr_last_error() gives the text.
 *
 * What each entry point replaces in the reference (Domingo1337/Chiaroscuro-RayTracer):
 *
 *   cr_upload_scene      KDTree::KDTree's products consumed by the render loop:
 *                        KDTree::triangles / materials / nodes / minCoords / maxCoords
 *                        (include/kdtree.hpp:43-76) and Scene::lightTriangles
 *                        (include/scene.hpp:47) -- built on the host by the caller
 *                        (src/kdtree.cpp:34-194), copied into device buffers here.
 *   cr_render            the body of RayTracer::rayTrace after the camera set-up:
 *                        the pixel x sample loop and the progressive blend
 *                        (src/rayTracer.cpp:52-70) with RayTracer::sendRay
 *                        (src/rayTracer.cpp:76-135), intersectRayKDTree (137-169),
 *                        KDTree traversal (src/kdtree.cpp:196-344), Diffuse /
 *                        Emissive BRDFs (src/brdf.cpp:10-85), Texture::getColorAt
 *                        (src/mesh.cpp:21-35) and Scene::randomLight (src/scene.cpp:79-82).
 *   cr_render_device     the same, into a caller-owned device framebuffer on a
 *                        caller-supplied HIP stream (no host copy).
 *   cr_render_tiles_device / cr_blend_tiles_device
 *                        the same loop split over ranks by 32x32 tiles (no
 *                        reference counterpart: the reference's only split is the
 *                        OpenMP row loop, src/rayTracer.cpp:55).
 *   cr_tonemap_setup / cr_tonemap / cr_tonemap_device
 *                        RayTracer::normalizeImage (src/rayTracer.cpp:172-222)
 *   cr_group_*           RayTracer::rayTrace (src/rayTracer.cpp:17-74) with the frame
 *                        tile-split over N GPUs of one process and gathered over
 *                        RCCL (the reference's single-process callers main.cpp:16,
 *                        src/openglPreview.cpp:247 through the host RayTracer).
 *   cr_comm_* / cr_render_dist_device
 *                        the same split with one process per GPU (RCCL
 *                        communicator from a unique id the caller distributes).
 *   cr_intersect         KDTree::intersectRay       (src/kdtree.cpp:210-216)
 *   cr_intersect_shadow  KDTree::intersectShadowRay (src/kdtree.cpp:283-290)
 *
 * Threading: one cr_ctx per GPU, not thread-safe; calls on one ctx are serialised.
 */
#ifndef CHIARO_HIP_H
#define CHIARO_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CR_OK 0
#define CR_E_INVALID (-1)  /* bad argument                         */
#define CR_E_HIP (-2)      /* HIP runtime error (no device, fault) */
#define CR_E_NOSCENE (-3)  /* render before cr_upload_scene        */
#define CR_E_DEPTH (-4)    /* kd-tree deeper than the kernels support */
#define CR_E_OOM (-5)      /* device allocation failed             */
#define CR_E_COMM (-6)     /* RCCL error (init, gather, a failed peer) */

typedef struct cr_ctx cr_ctx;

/* One kd node as KDTree::KDNode (include/kdtree.hpp:47-60):
 *   inner: axis in {0,1,2}, split = Split::position, child = KDNode::child
 *          (children at child and child+1, left = inLeft side)
 *   leaf:  axis == 3, first/count index the leaf reference list
 *          (KDNode::trianglesids, in order). */
typedef struct {
    float split;
    uint32_t axis;
    uint32_t child_or_first;
    uint32_t count;
} cr_kdnode;

typedef struct {
    int32_t width, height, components; /* Texture::width/height/nrComponents (include/mesh.hpp:173-182) */
    const uint8_t *data;               /* width*height*components bytes, stb layout */
} cr_texture;

typedef struct {
    /* kd tree, node 0 = root, DFS order exactly as KDTree::build allocates it */
    uint32_t n_nodes;
    const cr_kdnode *nodes;
    uint32_t n_refs;
    const uint32_t *refs;       /* concatenated leaf triangle id lists */
    uint32_t max_depth;         /* deepest leaf (root = 0) */
    float box_min[3], box_max[3]; /* KDTree::minCoords/maxCoords, AFTER the +-1e-4 pad */
    /* triangles + materials, id order (KDTree::triangles / materials) */
    uint32_t n_tris;
    const float *tri_pos;       /* [n][9]  posFst, posSnd, posTrd              */
    const float *tri_normal;    /* [n][3]  Material::normal ((n0+n1+n2)/3)     */
    const float *tri_kd;        /* [n][3]  Material::Kd                        */
    const float *tri_ke;        /* [n][3]  Material::Ke                        */
    const float *tri_uv;        /* [n][6]  texFst, texSnd, texTrd              */
    const int32_t *tri_tex;     /* [n]     texture index, -1 = none / not loaded */
    const uint8_t *tri_emissive;/* [n]     Material::BRDFtype == Emissive      */
    /* Scene::lightTriangles (include/scene.hpp:18-22), in push order */
    uint32_t n_lights;
    const uint32_t *light_id;
    const float *light_surface;
    /* textures referenced by tri_tex */
    uint32_t n_textures;
    const cr_texture *textures;
} cr_scene_desc;

/* Camera basis exactly as src/rayTracer.cpp:41-49 computes it (host side). */
typedef struct {
    float eye[3];
    float left_upper[3];
    float dx[3];
    float dy[3];
} cr_camera;

typedef struct {
    uint32_t xres, yres;  /* Scene::xres/yres */
    uint32_t spp;         /* Scene::samples (per layer) */
    int32_t k;            /* Scene::k, max path depth, 1..64 */
    float background[3];  /* Scene::background */
    uint32_t seed;        /* RNG stream key (DESIGN.md "RNG") */
    uint32_t layer;       /* progressive layer L >= 1 (src/rayTracer.cpp:18-33) */
    uint32_t rank, nranks;/* tile partition: tile slot s belongs to rank s % nranks (cr_tile_origin) */
    uint32_t tile;        /* tile edge in pixels, 0 -> 32 */
} cr_render_params;

/* Query counters of the last render / intersect call. */
typedef struct {
    uint64_t closest;     /* KDTree::intersectRay-equivalent queries      */
    uint64_t shadow;      /* KDTree::intersectShadowRay-equivalent queries (box-culled included) */
    uint64_t inner;       /* inner node visits  */
    uint64_t leaf;        /* leaf visits        */
    uint64_t tritest;     /* triangle tests     */
    uint64_t hit;         /* closest hits       */
    uint64_t texhit;      /* textured hits      */
    uint64_t paths;       /* camera paths       */
    uint64_t pixels;      /* pixels written     */
    /* SIMD-efficiency diagnostics of the persistent kernel (counting launches
     * only, cr_set_option "counters" 1): WAVE iterations executed by the kd
     * descent step, the leaf triangle loop, the traversal rounds (one leaf each)
     * and the per-query outer loop.  Lane efficiency of a phase =
     * lane work / (64 * wave iterations), e.g. inner / (64 * wave_desc). */
    uint64_t wave_desc;
    uint64_t wave_tri;
    uint64_t wave_round;
    uint64_t wave_query;
    /* of wave_desc / wave_tri: iterations whose node / triangle is the same for
     * every active lane (a scalar load would serve the whole wave) */
    uint64_t wave_desc_uniform;
    uint64_t wave_tri_uniform;
    /* of wave_desc / wave_tri: distinct 128-B cache lines the iteration's node /
     * first record load touches, summed (the cost unit of the vector memory
     * address path) */
    uint64_t wave_desc_lines;
    uint64_t wave_tri_lines;
    /* leaf rounds whose leaf is not wave-uniform: how many, the distinct leaves
     * and the triangle records they hold (summed), and how many of those rounds
     * hold at most 21 / 56 records (what a per-wave LDS staging area of 1 / 2.6
     * KiB would take) */
    uint64_t leaf_rounds;
    uint64_t leaf_distinct;
    uint64_t leaf_records;
    uint64_t leaf_fit21;
    uint64_t leaf_fit56;
    /* of `shadow`: NEE queries answered without a trace because their contribution is exactly zero
     * (cr_set_option "wf_nee_skip"; lean wavefront builds) */
    uint64_t nee_answered;
} cr_counters;

cr_ctx *cr_create(int device);
void cr_destroy(cr_ctx *ctx);
const char *cr_last_error(cr_ctx *ctx);

int cr_upload_scene(cr_ctx *ctx, const cr_scene_desc *desc);

/* Full-frame render of one progressive layer; blend on device into the ctx's
 * accumulator ((old*(L-1) + mean)/L), then copy [yres][xres][3] fp32 to
 * accum_rgb_out (host).  Layer 1 ignores the previous accumulator. */
int cr_render(cr_ctx *ctx, const cr_camera *cam, const cr_render_params *p, float *accum_rgb_out);

/* Resume a progressive render (checkpoint / resume of the accumulator, the persisted
 * counterpart of src/rayTracer.cpp:18-33,64): the ctx's accumulator becomes the host
 * frame rgb [yres][xres][3]; the next cr_render of layer L > 1 blends into it. */
int cr_set_accumulator(cr_ctx *ctx, uint32_t xres, uint32_t yres, const float *rgb);

/* Same, blending into the caller-owned device buffer d_frame [yres][xres][3]
 * (only this rank's tiles are touched) on `stream` (hipStream_t, NULL = null stream). */
int cr_render_device(cr_ctx *ctx, const cr_camera *cam, const cr_render_params *p, float *d_frame, void *stream);

/* Tonemap (RayTracer::normalizeImage, src/rayTracer.cpp:196-222).  The scalar
 * setup -- m = 2^(exposure+2.47393), s = 255*2^(-3.5*gamma), kl = 2^kneeLow and
 * the knee factor f = findKneeF(2^kneeHigh, 2^3.5 - kl) (:172-194) -- is host
 * arithmetic, done once by cr_tonemap_setup exactly as the reference does it.
 * The per-pixel transform runs on the device, one byte per thread:
 *   x = max(0, v - defog) * m;  x > kl: x = kl + log(1 + (x-kl)*f)/f;
 *   byte = (uint8) clamp(x^gamma * s, 0, 255)
 * with the rows flipped as the reference writes `data` ((yres-1-y)*xres + x). */
typedef struct cr_tonemap_params {
    float m, s, kl, f, defog, gamma;
} cr_tonemap_params;
void cr_tonemap_setup(float exposure, float defog, float kneeLow, float kneeHigh, float gamma, cr_tonemap_params *out);
/* d_rgb [yres][xres][3] fp32 (row 0 = top) -> d_bytes [yres][xres][3] uint8,
 * both device buffers, on `stream`. */
int cr_tonemap_device(cr_ctx *ctx, const cr_tonemap_params *t, uint32_t xres, uint32_t yres, const float *d_rgb,
                      uint8_t *d_bytes, void *stream);
/* The ctx's accumulator (the frame of the last cr_render) -> host bytes. */
int cr_tonemap(cr_ctx *ctx, const cr_tonemap_params *t, uint32_t xres, uint32_t yres, uint8_t *bytes_out);

/* Batch means (no blend) of this rank's tiles into compact d_tiles
 * [cr_tiles_for_rank][tile][tile][3]. */
int cr_render_tiles_device(cr_ctx *ctx, const cr_camera *cam, const cr_render_params *p, float *d_tiles,
                           void *stream);
/* Root side: d_gathered = [nranks][max_tiles][tile][tile][3] (rank r's compact
 * buffer at slot r, max_tiles = cr_tiles_for_rank(p, 0)); unpermute and blend
 * layer p->layer into d_frame [yres][xres][3]. */
int cr_blend_tiles_device(cr_ctx *ctx, const cr_render_params *p, const float *d_gathered, float *d_frame,
                          void *stream);
/* The same for layers p->layer .. + nlayers - 1 in ONE launch: d_gathered =
 * [nranks][nlayers][max_tiles][tile][tile][3] (rank r's nlayers compact buffers, as
 * cr_render_tiles_layers_device writes them, at slot r); each pixel blended layer after layer
 * in order, bit-identical to nlayers cr_blend_tiles_device calls. */
int cr_blend_tiles_layers_device(cr_ctx *ctx, const cr_render_params *p, uint32_t nlayers, const float *d_gathered,
                                 float *d_frame, void *stream);
uint32_t cr_tiles_for_rank(const cr_render_params *p, uint32_t rank);

/* Several progressive layers in ONE render pass (wavefront kernel): layers p->layer ..
 * p->layer + nlayers - 1 of the loop at src/rayTracer.cpp:18-33, each with its own samples and
 * RNG streams, so the result is bit-identical to nlayers calls of cr_render_device /
 * cr_render_tiles_device.  The paths of all layers share one chunk, so the latency-bound ends of
 * the generations (and the per-render cull boxes) are paid once per pass instead of per layer --
 * what a rank's small share of the frame needs when the frame is split over GPUs.
 * cr_layers_per_pass: how many of `want` layers fit one path chunk and one sample buffer (1 when
 * the kernel, lanes or counting build do not allow more); a larger nlayers is refused
 * (CR_E_INVALID) by cr_render_layers_device, which blends the layers in order into d_frame;
 * cr_render_tiles_layers_device writes layer j's batch means at
 * d_tiles + j * cr_tiles_for_rank(p, 0) * tile * tile * 3 floats, and with nranks > 1 takes up to
 * cr_layers_per_group layers (the rank's tiles in pieces). */
uint32_t cr_layers_per_pass(cr_ctx *ctx, const cr_render_params *p, uint32_t want);
int cr_render_layers_device(cr_ctx *ctx, const cr_camera *cam, const cr_render_params *p, uint32_t nlayers,
                            float *d_frame, void *stream);
int cr_render_tiles_layers_device(cr_ctx *ctx, const cr_camera *cam, const cr_render_params *p, uint32_t nlayers,
                                  float *d_tiles, void *stream);
/* cr_render of layers p->layer .. + nlayers - 1 of the whole frame (p->nranks 1) in pass groups:
 * up to 32 layers per pass, the frame cut into the fewest tile-split pieces (the ranks of a
 * pieces-way split, each blended in place) whose paths fit one chunk; bit-identical to nlayers
 * cr_render calls.  Counters, cr_last_kernel_ms and the trace stats sum over the passes. */
int cr_render_layers(cr_ctx *ctx, const cr_camera *cam, const cr_render_params *p, uint32_t nlayers,
                     float *accum_rgb_out);
/* How many of `want` layers (from p->layer) one pass group can render for p's share of the frame
 * (the whole frame with nranks 1, else rank p->rank's tiles), cutting the share into up to 64
 * pieces whose paths fit one chunk each: cr_render_layers plans the same for the frame, and
 * cr_render_tiles_layers_device renders that many layers of a rank's tiles in pieces (the ranks
 * r + kN of an N * m split; every tile slot keeps its pixels for any split of more than one rank). */
uint32_t cr_layers_per_group(cr_ctx *ctx, const cr_render_params *p, uint32_t want);
/* Triangles of the uploaded scene (0: none).  Frame pieces are used for scenes of at least 1024
 * triangles only: on a handful of triangles denser passes gain no coherence. */
uint32_t cr_scene_triangles(cr_ctx *ctx);
/* Pixel origin of rank's local tile `local` (slot rank + local * nranks of the frame's
 * row-major tile slots; with nranks > 1 each tile row is rotated by its index, so a
 * rank's tiles spread over every column class). */
int cr_tile_origin(const cr_render_params *p, uint32_t rank, uint32_t local, uint32_t *x0, uint32_t *y0);

/* Ray queries (host arrays). dir need not be normalised (the reference does not). */
int cr_intersect(cr_ctx *ctx, uint32_t n, const float *orig, const float *dir, uint32_t *hit, uint32_t *tri,
                 float *bary, float *dist);
int cr_intersect_shadow(cr_ctx *ctx, uint32_t n, const float *orig, const float *dir, const float *dist,
                        const uint32_t *light_tri, uint32_t *occluded);

int cr_get_counters(cr_ctx *ctx, cr_counters *out);
/* Device time (ms) of the last render kernel, HIP events on its own stream. */
float cr_last_kernel_ms(cr_ctx *ctx);
/* Per-kernel view of the last wavefront render ("kernel" 2) for the roofline.
 * Kinds: [0] the camera-ray trace (generation-1 closest-hit queries,
 * KDTree::intersectRay, src/kdtree.cpp:210-281), [1] the closest-hit traces of
 * later generations, [2] the shadow traces (intersectShadowRay, :283-344), [3]
 * the tail kernel that runs the last, small generations.  Per kind: launch
 * count, summed device time (a HIP event pair around every launch, on its
 * stream; [1] and [2] partly run side by side, so their times overlap) and, for
 * [0]-[2] after a counting render ("counters" 1), the inner-node / leaf /
 * triangle-test tallies of those launches (zero after a lean render and for [3]). */
typedef struct cr_trace_stats {
    uint64_t launches[4];
    double ms[4];
    uint64_t inner[4], leaf[4], tritest[4];
    /* wf_shade launches of the last render that reserved queue slots in chunks ("wf_app_chunk", or the
     * automatic chunks of scenes traced in append order) */
    uint64_t chunked_shades;
} cr_trace_stats;
int cr_get_trace_stats(cr_ctx *ctx, cr_trace_stats *out);
/* Kernel variant / tuning knobs: "kernel" (0 = persistent wave-regeneration,
 * 1 = one-thread-per-pixel), "variant" (persistent-kernel build, 0 = default),
 * "refill" (1..64: idle lanes of a wave that trigger a path-state step in the
 * dynamic-fetch variants), "counters" (1 = also count inner/leaf/tritest and
 * the wave_* diagnostics; 0 = only the per-query tallies, for timed launches),
 * "block", "waves_per_cu".  Returns CR_OK or CR_E_INVALID. */
int cr_set_option(cr_ctx *ctx, const char *key, int64_t value);
/* Diagnostics of the last counting render (wavefront trace kernels, option
 * "diag_kinds" = mask of trace kinds 1 camera / 2 closest / 4 shadow): leaf-round
 * shapes (what staging a wave's leaves in LDS would load) and a per-lane census of
 * repeated any-segment triangle misses.  Up to n of the DIAG_* values (csrc/kernels.hpp). */
int cr_get_diag(cr_ctx *ctx, uint64_t *out, int n);
/* Performed work of the last render with option "perf_counters" 1 (trace builds 18 / 26 / 40 / 42 /
 * 43 / 44 -- the defaults are 43 and 44 -- instantiated with counters; measurement only): per trace kind k (0 camera, 1 closest, 2 shadow,
 * 3 tail) the PERF_N = 12 values out[12k + i] -- queries, inner-node steps, leaves reached, leaf
 * cull records evaluated, triangle tests executed (all per ray), bytes of vector-memory loads and
 * stores (per lane), bytes of scalar-memory loads (per wave), wave iterations, and the shape of
 * the divergent leaf-cull loop: rounds, iterations, lanes with a test, tests (PERF_* in
 * csrc/kernels.hpp).  Where the counting build ("counters" 1) counts the reference algorithm's
 * work, these count what the culling kernels actually do.  Up to n values. */
int cr_get_perf(cr_ctx *ctx, uint64_t *out, int n);
/* 1 when wavefront trace build `build` (option "variant" with "kernel" 2) is compiled in:
 * the default compile holds 0, 15, 18 and 26 (the default); `make ALL_VARIANTS=1` every
 * measured build.  A render with a missing build returns CR_E_INVALID. */
int cr_trace_build_available(int build);
/* The wavefront trace build the last render on ctx ran (its "variant": the scene-size default 43 / 44
 * unless set), -1 when it was the counting build ("counters" 1), -2 when it was not a wavefront render
 * (or none has run).  Lets a caller name the kernels a result came from (bench.py, smoke()). */
int cr_last_trace_build(cr_ctx *ctx);
int cr_synchronize(cr_ctx *ctx);

/* ---------------------------------------------------------- multi-GPU --
 * The frame split of SURVEY §8e behind the C-ABI, RCCL inside (csrc/group.cpp):
 * tile slot s of the frame belongs to rank s % nranks (cr_tile_origin); each rank renders its tiles'
 * batch means, the root (rank 0) gathers them over RCCL (xGMI) and blends the
 * layer into its frame ((old*(L-1) + mean)/L, src/rayTracer.cpp:64) on the
 * device.  The image equals the single-GPU render bit for bit. */

/* One process per GPU.  Rank 0 makes the id (cr_comm_unique_id), the caller
 * hands it to every rank (any channel), each rank calls cr_comm_init on its ctx
 * (collective: returns once all nranks have joined). */
#define CR_COMM_ID_BYTES 128
int cr_comm_unique_id(uint8_t *id_out, size_t id_bytes);
int cr_comm_init(cr_ctx *ctx, int nranks, int rank, const uint8_t *id);
int cr_comm_destroy(cr_ctx *ctx);
/* Collective over the communicator: this rank's tiles of layer p->layer (p->rank /
 * p->nranks are taken from the communicator), gathered to rank 0 and blended into
 * d_frame [yres][xres][3] there (other ranks: d_frame unused, may be NULL).
 * Returns when the layer is complete on this rank's stream. */
int cr_render_dist_device(cr_ctx *ctx, const cr_camera *cam, const cr_render_params *p, float *d_frame,
                          void *stream);
/* Pass groups over the communicator: layers p->layer .. + nlayers - 1 of this rank's tiles in one
 * render pass group (cr_render_tiles_layers_device: the rank's tiles in pieces when they do not fit
 * one chunk), ONE grouped send / receive of all nlayers compact buffers to rank 0 and one blend of
 * the layers there (cr_blend_tiles_layers_device); bit-identical to nlayers cr_render_dist_device
 * calls.  nlayers must fit: at most min over the ranks of cr_layers_per_group -- every rank must
 * pass the same nlayers (the caller agrees on it, e.g. an all-reduce MIN). */
int cr_render_dist_layers_device(cr_ctx *ctx, const cr_camera *cam, const cr_render_params *p, uint32_t nlayers,
                                 float *d_frame, void *stream);

/* One process driving N GPUs: a ctx per device (devices NULL -> 0..ngpus-1), the
 * passes on one host thread per GPU, grouped RCCL send / receive to rank 0.  A
 * device listed twice cannot join a RCCL communicator: such a group gathers with
 * device-to-device copies (same protocol, for one-GPU tests).  Errors of create
 * show on the first call / cr_group_last_error. */
typedef struct cr_group cr_group;
int cr_device_count(void); /* HIP devices visible to this process (0 without a GPU) */
cr_group *cr_group_create(int ngpus, const int *devices);
void cr_group_destroy(cr_group *g);
const char *cr_group_last_error(cr_group *g);
int cr_group_size(cr_group *g);
/* 1 when every rank has a device and, for distinct devices, the RCCL communicator
 * exists; 0 after a failed create (cr_group_last_error says why; cr_group_destroy
 * is still required). */
int cr_group_ok(cr_group *g);
int cr_group_upload_scene(cr_group *g, const cr_scene_desc *desc);
int cr_group_set_option(cr_group *g, const char *key, int64_t value); /* on every rank's ctx */
/* cr_render across the group: layer p->layer of the whole frame (p->rank / p->nranks
 * ignored, p->tile used), blended into the root's accumulator, copied to
 * accum_rgb_out [yres][xres][3] (host). */
int cr_group_render(cr_group *g, const cr_camera *cam, const cr_render_params *p, float *accum_rgb_out);
/* cr_group_render of layers p->layer .. + nlayers - 1 in pass groups (cr_render_layers across the
 * group): per group of up to 32 layers -- as many as every rank's tiles fit (min over the ranks of
 * cr_layers_per_group) -- each rank renders its tiles of all of them in one pass group, one gather
 * of the group's buffers and one blend of its layers at the root; bit-identical to nlayers
 * cr_group_render calls.  Counters and cr_group_rank_ms sum over the groups. */
int cr_group_render_layers(cr_group *g, const cr_camera *cam, const cr_render_params *p, uint32_t nlayers,
                           float *accum_rgb_out);
int cr_group_get_counters(cr_group *g, cr_counters *out); /* summed over the ranks */
int cr_group_rank_ms(cr_group *g, float *ms_out);          /* [ngpus] each rank's last pass (HIP events) */
/* rank's ctx (rank 0: the root, which also answers cr_intersect*), NULL if out of range */
cr_ctx *cr_group_ctx(cr_group *g, int rank);
/* cr_set_accumulator for the group's root accumulator */
int cr_group_set_accumulator(cr_group *g, uint32_t xres, uint32_t yres, const float *rgb);
/* cr_tonemap on the root's accumulator (the frame of the last cr_group_render) */
int cr_group_tonemap(cr_group *g, const cr_tonemap_params *t, uint32_t xres, uint32_t yres, uint8_t *bytes_out);

#ifdef __cplusplus
}
#endif
#endif
