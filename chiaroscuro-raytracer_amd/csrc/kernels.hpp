// kernels.hpp -- device-side data layout shared by kernels.hip and cabi.cpp.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "leafcull.hpp"

namespace cr {

enum { MODE_BLEND = 0, MODE_TILES = 1 };
// float4 per triangle record.  3 (48 B, 1.5 lines per test on average) beat 4
// (one 64-B line per test, +33% footprint): 561 vs 547 Mray/s, sponza 8 spp.
enum { REC_STRIDE = 3 };
enum { CTR_N = 22, CTR_SLOTS = 112 }; // Ctr fields (cr_counters order); device counter buffer entries
// Wavefront trace launches by kind (cr_trace_stats order): camera rays (generation-1
// closest trace), closest traces of later generations, shadow traces, the tail kernel.
enum { TK_CAMERA = 0, TK_CLOSEST = 1, TK_SHADOW = 2, TK_TAIL = 3, TK_N = 4 };
// Counting builds of the trace kernels also tally inner / leaf / tritest per kind
// (not the tail): slots CTR_TRACE + 3 * kind + {0, 1, 2}.
enum { CTR_TRACE = 24 };
// slot of cr_counters::nee_answered (shadow queries answered without a trace, WfArgs::nee_skip)
enum { CTR_NEE = 22 };
// Leaf-round and repeated-miss diagnostics of counting builds (cr_get_diag, DIAG_* order),
// for the trace kinds in RenderArgs::diag_kinds (bit 1 << TK_*): slots CTR_DIAG + i.
enum { CTR_DIAG = 40, DIAG_N = 16 };
enum {
    DIAG_ROUNDS = 0,    // divergent leaf rounds (the wave's busy lanes at more than one leaf)
    DIAG_LANES = 1,     //   lanes at a leaf with triangles, summed over those rounds
    DIAG_DISTINCT = 2,  //   distinct leaves with triangles, summed
    DIAG_RECORDS = 3,   //   records of the distinct leaves, summed (what LDS staging would load)
    DIAG_MAXCOUNT = 4,  //   the largest leaf of the round, summed (wave iterations of the leaf loop)
    DIAG_LANETESTS = 5, //   records of every lane's leaf, summed (lane work of the leaf loop)
    DIAG_FIT64 = 6,     //   rounds with at most 64 / 128 staged records
    DIAG_FIT128 = 7,
    DIAG_UROUNDS = 8,   // uniform leaf rounds
    DIAG_TESTS = 9,     // triangle tests (lane)
    DIAG_GEOMISS = 10,  //   rejected for any segment (det, u, v or t < 0): exact to skip later in the query
    DIAG_REP1 = 11,     //   of those: the triangle was such a miss in the lane's last 1 / 4 / 8 such misses
    DIAG_REP4 = 12,
    DIAG_REP8 = 13,
};
// Performed work of the default trace build's kernels (RenderArgs::perf_counters, cr_get_perf):
// per trace kind, slots CTR_PERF + PERF_N * kind + PERF_*.  What the kernels actually execute
// and load -- after the cull boxes, leaf cull records and packet traversal skipped work --
// where the counting build (full_counters) counts the reference algorithm's work.
enum { CTR_PERF = 64, PERF_N = 12 };
enum {
    PERF_QUERIES = 0, // queries started (ray fetched from the queue)
    PERF_STEPS = 1,   // inner-node decisions, per ray
    PERF_LEAVES = 2,  // leaves reached, per ray
    PERF_MASKS = 3,   // leaf cull records evaluated, per ray
    PERF_TESTS = 4,   // triangle tests executed, per ray
    PERF_VBYTES = 5,  // bytes of vector-memory loads and stores (per lane) of the trace
    PERF_SBYTES = 6,  // bytes of scalar-memory loads (per wave)
    PERF_WAVES = 7,   // wave iterations: traversal rounds (wf_trace, tail) / node fetches (packet)
    PERF_DROUNDS = 8, // divergent leaf rounds of the leaf-cull loop with a test to run (wave)
    PERF_DITERS = 9,  //   their loop iterations (the largest lane mask's popcount, summed; wave)
    PERF_DLANES = 10, //   lanes with a test, summed (wave)
    PERF_DTESTS = 11, //   tests, summed (lane)
};

// Zero bytes appended after every texture: the reference's getColorAt reads one
// texel past the row/image end for coords == 1.0 (src/mesh.cpp:23-30) and three
// bytes for 1-channel images; the pad makes that read defined (zeros).
__host__ __device__ inline uint64_t tex_pad(int w, int nc) { return (uint64_t)(w + 1) * nc + 4; }

// Tile split (nranks > 1): slot s = rank + lt * nranks of the frame's row-major tile
// slots belongs to the rank; slot s is tile (column (s % tiles_x + row) % tiles_x, row
// s / tiles_x) -- each tile row rotated by its index, so a rank's tiles cycle through
// every column class mod nranks instead of forming vertical stripes (cost varies
// across the frame: plain t % nranks left 2.6% imbalance at 8 ranks).  One rank: the
// identity.  cr_tile_origin and chiaroscuro_amd.tiles.TileLayout are the same map.
__host__ __device__ inline uint32_t tile_slot_column(uint32_t slot, uint32_t tiles_x, uint32_t nranks) {
    const uint32_t row = slot / tiles_x, c = slot - row * tiles_x;
    return nranks > 1 ? (c + row % tiles_x) % tiles_x : c;
}
// ... and back: the slot of tile (column gx, row gy)
__host__ __device__ inline uint32_t tile_slot(uint32_t gx, uint32_t gy, uint32_t tiles_x, uint32_t nranks) {
    const uint32_t c = nranks > 1 ? (gx + tiles_x - gy % tiles_x) % tiles_x : gx;
    return gy * tiles_x + c;
}

struct DevScene {
    const uint2 *nodes;   // {split bits | first ref, axis | child<<2 ; leaf: 3 | count<<2}
    const uint4 *fat;     // 2 per node: {self, child 0}, {child 1, 0, 0} (two-level descent)
    // REC_STRIDE float4 per leaf reference, AoS: {A, tri id bits}, {e1 = B-A, 0},
    // {e2 = C-A, 0} -- bitwise what the reference computes per test.  (A 40-B SoA
    // split measured 15% slower: three cache lines per test instead of one or two.)
    const float4 *recs;
    // leaf cull records (leafcull.hpp) per kd node: a leaf's references in two normal groups, each with
    // its box and normal cone -- the exact skip of the tests a unit-direction ray cannot pass
    const float4 *lcullp; // packed (LC_RECP float4 per node, leaf_cull_pack, LC 4)
    const uint4 *lcullc;  // compressed (LC_RECC uint4 per node on grid lcg, leaf_cull_compress, LC 5)
    LcGrid lcg;
    float db;             // bound on |coordinate| of any origin or vertex (padded box + 1)
    const float4 *tri;    // 3 per triangle: A, B, C
    const float4 *mat_n;  // normal, w = emissive flag bits
    const float4 *mat_kd; // Kd, w = texture index (int bits, -1 none)
    const float4 *mat_ke; // Ke
    const float2 *mat_uv; // 3 per triangle
    const uint2 *lights;  // {triangle id, surface bits}
    const uint4 *texs;    // {w, h, nc, byte offset}
    const uint8_t *texels;
    uint32_t nlights;
    uint32_t n_nodes;
    float3 bmin, bmax;    // padded root box
};
// cr_upload_scene numbers the first NODE_BFS nodes breadth-first (sibling pairs kept
// adjacent, the rest in the reference's depth-first order), so the top of the tree
// is nodes 0..NODE_BFS-1 (the LDS node tile of trace builds 10-11).
enum : uint32_t { NODE_BFS = 512 };

struct RenderArgs {
    DevScene S;
    float cam[12];        // eye, leftUpper, dx, dy
    uint32_t xres, yres, spp;
    int K;
    float bg[3];
    uint32_t seed, layer;
    // layers rendered by this pass (wavefront kernel): layers layer .. layer + nl - 1, their samples
    // one run per item ("virtual" sample s -> layer + s / spp, sample s % spp); MODE_TILES writes
    // layer j's tile means at out + j * layer_stride floats
    uint32_t nl;
    uint64_t layer_stride;
    // MODE_TILES of one piece of a rank's tiles (cr_render_tiles_layers_device): this launch renders
    // rank r + piece_k * N of an N * piece_m split, whose local tile j is the rank's local tile
    // piece_k + j * piece_m (tile slots keep their pixels for any split of more than one rank)
    uint32_t piece_k, piece_m;
    uint32_t rank, nranks, tile, tiles_x;
    uint32_t n_items;     // my_tiles * tile * tile
    uint32_t stack_depth;
    int mode;
    float *out;
    unsigned long long *counters; // 9 x u64
    uint2 *gstack;                // traversal-stack overflow [stack_depth][gstride] {node, tmax bits}
    uint32_t gstride;             // threads in the persistent trace grid
    int full_counters;            // 1: also count inner/leaf/tritest (SURVEY §8d bytes)
    int perf_counters;            // 1: the default build's kernels with performed-work counts (CTR_PERF)
    int variant;                  // wavefront trace build (wavefront.hip kWf)
    uint32_t refill;              // idle lanes of a wave that trigger a path-state step / ray fetch
    uint32_t refill_shadow;       // wavefront shadow-trace kernel's threshold
    uint32_t refill_camera;       // wavefront closest trace of generation 1 (camera rays)
    // (pixel, sample) work items of one launch: samples [s0, s0 + s_count) of
    // every item, w = item * s_count + (s - s0), n_work = n_items * s_count
    uint32_t s0, s_count, n_work;
    float *samples;               // [n_items][s_count][3] path radiance per work item
    float *run;                   // [n_items][3] running per-pixel sum across sample chunks
    // wavefront camera trace builds with the screen-space cull (camcull.hpp): per leaf
    // reference {xmin, xmax, ymin, ymax} of the sample positions at which its triangle can
    // accept a camera ray of this camera (null: no cull)
    const float4 *cull;
    const float4 *cull_node;      // [n_nodes] the union of the boxes of the node's subtree
    // 1: the eye lies exactly on a split plane of its axis, where camera rays may disagree on
    // a node's near child -- the packet camera trace (build 17) is not used for this render
    int eye_on_split;
    uint32_t diag_kinds;          // counting builds: trace kinds (1 << TK_*) the DIAG_* slots describe
    int lc_debug;                 // measurement only: leaf-cull masks 1 = every reference, 2 = none (wrong images)
    uint32_t lc_min;              // leaf-cull builds: leaves with fewer references are tested without the check
    uint32_t desc_quorum;         // lean wavefront traces: a round's descent stops once at most desc_quorum / 64
                                  // of its lanes still descend (they go on next round); 0: every lane reaches a leaf
};
// Traversal-stack overflow area of a persistent trace grid of `threads` lanes: [depth][threads] x 8 B.
inline size_t gstack_bytes(uint32_t depth, uint32_t threads) { return (size_t)depth * threads * 8; }
// Sample buffer budget: a render is split into sample chunks whose per-sample
// buffer fits in this many bytes (whole 1080p x 128 spp frames fit in one).
enum : uint64_t { SAMPLE_BUF_BYTES = 4ull << 30 };
// Per-pixel in-order sum of one chunk's samples; `last` blends / writes the pixel.
int launch_sum_samples(const RenderArgs &A, bool first, bool last, hipStream_t st, uint32_t lds = 0, bool staged = true);

// Wavefront path tracer (wavefront.hip, cr_set_option "kernel" 2): the paths of
// work items [w0, w0 + P) advance one bounce per generation through separate
// kernels (camera, closest trace, shade, shadow trace, bounce) that exchange
// rays through queues in HBM.
// counters: closest count [g], shadow count [WF_G+g], work [2*WF_G+g], [3*WF_G+g], (unused) [4*WF_G+g];
// g <= K + 1 <= 65;
// then the per-XCD work counters of the partitioned queues (WfArgs::xcd), WF_XSTRIDE apart
// (one 64-B line each): closest [WF_XBASE + (g*8 + x)*WF_XSTRIDE], shadow after WF_G*8 of those
enum : uint32_t { WF_G = 66, WF_XCDS = 8, WF_XSTRIDE = 16, WF_XBASE = 5 * WF_G,
                  WF_CNT = WF_XBASE + 2 * WF_G * WF_XCDS * WF_XSTRIDE };
enum { WF_STATE = 6 };            // path-state float4 slots per path (wavefront.hip PS)
struct WfArgs {
    uint32_t P;       // path slots of this chunk
    uint32_t w0;      // first work item of the chunk
    float4 *ray[2];   // closest rays, by generation parity: [2P] {o, path}, {d, 0}
    uint4 *hit[2];    // [P] closest result of ray i of generation g in hit[g & 1]: {tri, bx, by bits, 1} / 0
    float4 *sray;     // [2P] shadow rays {o, path}, {d, limit}
    uint32_t *sexcl;  // [P] light triangle the shadow ray ignores
    uint32_t *occ;    // [P] shadow result of shadow ray j
    uint32_t *cnt;    // [WF_CNT] zeroed per chunk
    float4 *ps;       // [WF_STATE][P] path state
    float4 *dw;       // [2K][P] (direct, w) per bounce
    uint2 *gstack;    // trace kernels' stack overflow [depth][gstride]
    uint2 *gstack2;   // ... of a closest trace running beside a shadow trace
    uint32_t gstride; // threads of the trace grid
    // queue ordering (raysort.hip): wf_shade writes a sort key and the slot per
    // appended ray into key[q][0] / perm[q][0] (q = 0 shadow queue, 1 closest
    // queue); the host sorts them (double buffers [q][0..1]) and hands the trace
    // kernel the permutation (`order`, null = queue order)
    uint32_t *key[2][2], *perm[2][2];
    const uint32_t *order;
    void *sort_tmp;
    size_t sort_tmp_bytes;
    int sort;         // 1: write keys and sort the queues of large generations
    int key_bits;     // significant key bits (world keys included)
    int key_bits_pixel; // significant bits of the pixel keys (generation-1 queues): fewer digit passes
    uint32_t sort_min;   // queues shorter than this are traced in append order
    uint32_t sort_tile;  // log2 of the pixel sub-tile edge of the key (3: 8x8 pixels)
    uint32_t dir_res;    // octahedral direction bins per axis (8: 64 bins; power of two)
    int world_keys;      // g > 0: world-space origin keys for queues whose rays start at hits of
                         // generation >= g (shadow queue g, closest queue g + 1); 0: pixel keys only
    uint32_t world_bits; // bits per axis of the origin's Morton code
    uint32_t tail_min;   // a closest queue shorter than this hands the rest of the chunk to wf_tail (0: never)
    float2 *cxy;         // [P] screen position (sx, sy) of path p's camera sample (written when A.cull)
    // XCD-partitioned queues (bit 0 shadow, bit 1 secondary closest, bit 2 camera rays): the
    // queue's (sorted) order is cut into WF_XCDS contiguous ranges and a block of XCD
    // blockIdx % WF_XCDS (the dispatcher's round-robin) takes rays from its own range first,
    // then from the others' -- each XCD's L2 then holds the data of one region of key space
    uint32_t xcd;
    // 1: queue keys are (leaf of the hit the ray starts from, direction bin) -- the hit
    // record's w carries the leaf + 1 -- instead of pixel / world-position keys
    int leaf_keys;
    uint32_t resolve_paths; // wf_resolve sweeps queues of >= P / this rays in path order (0: never)
    // measurement only (option "wf_measure_skip", WRONG images): bit 0 no wf_resolve launch, bit 1 no queue
    // sort -- upper bounds of what a cheaper resolve / sort could gain
    uint32_t measure_skip;
    uint32_t leaf_shift; // leaf keys: the node index >> leaf_shift (depth-first numbering: a run of
                         // consecutive nodes is one region of the tree)
    // Overlapped tail (launch_wavefront_chunk): the tail kernel for closest queue g + 1 starts beside
    // the shadow trace of generation g.  tail_shadow_gen = g: wf_tail first traces each of its paths'
    // generation-g shadow ray and resolves that bounce itself; ended_only = 1: the shadow trace and
    // wf_resolve of generation g take only the paths that ended at g (bit 0 of the PS3 mark).
    uint32_t tail_shadow_gen;
    uint32_t ended_only;
    int tail_overlap; // 1: hand the rest of a chunk to an overlapped tail (option "wf_tail_overlap")
    uint32_t sort_g1; // generation-1 queues that are sorted: bit 0 the shadow queue, bit 1 the closest queue
    int cam_lean;     // 1: wf_camera leaves generation 1's RNG state to wf_shade (option "wf_cam_lean")
    uint32_t dir_res_s; // leaf keys: direction bins per axis of the SHADOW queues' keys
    int key_bits_s;     // significant bits of the shadow queues' keys
    int tail_waves;     // waves per SIMD of the lean tail launch (4, 5, 6)
    int shade_waves;    // wf_shade's build: 8 waves per SIMD (64 VGPRs, spills) or else its natural 6
    // wf_shade's queue appends in chunks (set per launch by launch_wavefront_chunk): a block reserves
    // app_chunk slots of a queue with one atomic and fills them over its iterations; the unused end of
    // its last chunk becomes dead entries (ray w = NO_PATH, key ~0) that the consumers skip.  0: one
    // atomic per block iteration.  Same-address device atomics serialise (~5.7 ns each on MI355X,
    // scripts/append_bench.hip): the per-iteration form bound wf_shade of a full chunk.
    uint32_t app_chunk;
    uint32_t qspare;    // queue slots past P in every queue-indexed array (the dead entries' room; 0: no chunks)
    uint32_t app_force; // option "wf_app_chunk": this chunk size (>= 256) for every launch that has room (tests)
    uint32_t shade_block; // wf_shade's threads per block for the per-iteration appends (256, 512, 1024)
    // 1: no wf_camera launch -- the packet camera trace derives each path's camera ray from its
    // (pixel, sample) itself, and wf_shade(1) / wf_resolve(1) take path p = ray p and the eye as
    // its origin (set per chunk by launch_wavefront_chunk; option "wf_cam_fuse")
    int cam_fused;
    // 1: a secondary closest ray carries its path's RNG counter in the direction's w and the key is
    // re-derived from the path's (pixel, sample) -- wf_shade neither reads nor writes the control slot
    // (PS_CTL) of generations >= 2; wf_tail writes it at pickup (option "wf_ctl_ray")
    int ctl_ray;
    // [P] resolve marks, one byte per path: (k << 1) | ended of the path's last closest hit (wf_shade), 0 for
    // a path that missed -- wf_resolve's path-order sweep reads these, not the 16-B PS3 records
    uint8_t *mark;
    // 1: the shadow trace writes each query's result over the slot in the w of its path's dw record of
    // that bounce (SHADOW_VIS / SHADOW_OCC) instead of occ[slot] -- wf_resolve then reads no occ entries,
    // which a sorted shadow queue scatters over the paths (option "wf_vis_dw")
    int vis_dw;
    // 1 (option "wf_vis_mark", no overlapped tail, K <= 63): the resolve marks are
    // (k << 2) | visible << 1 | ended; wf_shade writes PS3 = direct + contrib (the reference's add for a
    // visible NEE ray, done there) and a mark with visible 0, the shadow trace sets visible for an
    // unoccluded answer (one byte, nothing for an occluded one), and wf_resolve touches only the paths
    // whose bounce is visible (copy PS3 over dw) or ended (fold) -- no dw read / write for the rest
    int vis_mark;
    // 1: an NEE query whose contribution is exactly zero is answered without a trace (wavefront.hip
    // nee_zero; lean builds only -- the counting and performed-work builds trace every query) and
    // counted as a shadow query (option "wf_nee_skip")
    int nee_skip;
};
// rays 2x2 float4, hits 2, shadow ray 2, exclude + occ 8 B, state, (direct, w) pairs, 2 x 2 sort keys + perms,
// camera sample position, resolve mark
// spare: + 21 for the queue arrays' spare slots of chunked appends, P / 8 of them at 168 B (cabi.cpp spare_for)
inline size_t wf_bytes_per_path(int K, bool spare) {
    return (size_t)(4 + 2 + 2 + WF_STATE + 2 * K) * 16 + 8 + 32 + 8 + 1 + (spare ? 21 : 0);
}
// Second stream and fork / join events of a render (shadow trace g beside closest trace g + 1).
struct WfStreams {
    hipStream_t side;
    hipEvent_t fork, join;
};
int num_wf_variants();
// the most blocks a chunked-append wf_shade launch has at the ctx's wf_shade_waves (spare-slot sizing)
uint32_t wf_shade_blocks(int num_cus, int shade_waves);
// true when the variant's camera trace skips Moller-Trumbore tests by the cull boxes
bool wf_variant_culls(int variant);
bool wf_variant_available(int variant); // compiled in (the default compile holds builds 0, 15, 18, 26)
bool wf_perf_available(int variant);    // a performed-work instance of this trace build exists (18, 26)
// cull boxes of this render's camera for the nrefs leaf references (+ 4 padding boxes)
// and their unions per subtree (node_boxes[n_nodes]): leaves first, then the inner
// nodes level by level from the deepest (levels: inner node ids grouped by depth,
// level_off[i] = {offset, count} of level i, deepest first)
int launch_cam_cull(const RenderArgs &A, uint32_t nrefs, float4 *boxes, float4 *node_boxes, const uint32_t *levels,
                    const uint32_t (*level_off)[2], int nlevels, hipStream_t st);
void wf_trace_geometry(int variant, int num_cus, uint32_t &block, uint32_t &blocks);
void wf_tail_geometry(int num_cus, uint32_t &block, uint32_t &blocks);
// HIP events bracketing every trace launch (start, stop), recorded on the launch
// stream; kind[i] = TK_* of pair i.  Grown by the launcher.
struct TraceEvents {
    hipEvent_t *ev = nullptr; // [2 * cap]
    int *kind = nullptr;      // [cap]
    int cap = 0, n = 0;
    int chunked = 0; // wf_shade launches that appended in chunks (WfArgs::app_chunk != 0)
};
// One chunk: camera, closest 1, then per generation shade, shadow || next closest, resolve.
// Two chunks in flight (cr_set_option "wf_lanes" 2): each lane owns a buffer set
// (W, W.P = its capacity), a main and a side stream with fork / join events, an
// event marking its queue lengths copied, and 2 pinned host words for them.  The
// host advances both lanes' generations without blocking (event polling); a
// chunk starts on a free lane once the other lane's chunk is past its camera-ray
// trace, so a VALU-bound camera trace runs beside address-bound secondary traces
// and one chunk's generation tails beside the other's work.  Lane 0's main
// stream is `st`; lane 1's joins `st` at entry and exit.
struct WfLane {
    WfArgs W;
    hipStream_t st, side;
    hipEvent_t fork, join, ready;
    uint32_t *hcnt;
};
int run_wavefront_lanes(const RenderArgs &A, WfLane *lanes, int nlanes, int num_cus, hipStream_t st,
                        TraceEvents *te);
int launch_wavefront_chunk(const RenderArgs &A, const WfArgs &W, int num_cus, hipStream_t st, const WfStreams &ss,
                           TraceEvents *te = nullptr);
// raysort.hip: stable radix sort of (key, value) pairs; lib: hipcub's instead
int sort_queue(uint32_t *keys[2], uint32_t *vals[2], uint32_t n, int end_bit, void *tmp, size_t &tmp_bytes,
               hipStream_t st, bool lib = false, bool iota = false, bool keep_keys = true);
size_t wf_sort_tmp_bytes(uint32_t n, int key_bits);

struct QueryArgs {
    DevScene S;
    uint32_t n, shadow, stack_depth;
    const float *orig, *dir, *dist;
    const uint32_t *light;
    uint32_t *hit, *tri;
    float *bary, *dist_out;
    unsigned long long *counters;
};

// gathered: [nranks][nl][max_tiles][T][T][3] -- every rank's compact tile buffers of layers
// layer .. layer + nl - 1, blended into the frame in layer order by one launch
struct BlendArgs {
    const float *gathered;
    float *frame;
    uint32_t xres, yres, tile, tiles_x, nranks, max_tiles, layer, nl;
};

// RayTracer::normalizeImage's per-pixel transform (src/rayTracer.cpp:207-221)
struct TonemapArgs {
    const float *rgb; // [yres][xres][3], row 0 = top
    uint8_t *out;     // [yres][xres][3], rows flipped as the reference's data
    uint32_t xres, yres;
    float m, s, kl, f, defog, gamma;
};

int launch_intersect(const QueryArgs &Q, hipStream_t st);
int launch_blend(const BlendArgs &B, hipStream_t st);
int launch_tonemap(const TonemapArgs &T, hipStream_t st);

} // namespace cr
