// ctx.hpp -- the state behind one cr_ctx (one GPU) and the render entry shared by
// the single-GPU C-ABI (cabi.cpp) and the multi-GPU one (group.cpp).
#pragma once
#include "chiaro_hip.h"
#include "kernels.hpp"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <string>
#include <vector>

struct cr_ctx {
    int device = -1;
    int num_cus = 0;
    std::string err;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    cr::WfStreams wfs{nullptr, nullptr, nullptr}; // wavefront side stream + fork / join events
    // second wavefront lane (wf_lanes 2): its main / side streams, fork / join events;
    // per lane a queue-length event and pinned host words for the lengths
    hipStream_t stream2 = nullptr, side2 = nullptr;
    hipEvent_t fork2 = nullptr, join2 = nullptr, lane_ev[2] = {nullptr, nullptr};
    uint32_t *hcnt = nullptr;
    void *d_wf2 = nullptr;
    size_t wf2_bytes = 0;
    // HBM the path-chunk buffers may take: free + their size at the first query, kept (wf_path_cap)
    uint64_t wf_mem_budget = 0;
    float last_ms = 0.f;
    int last_build = -2; // cr_last_trace_build
    // scene
    bool has_scene = false;
    cr::DevScene S{};
    uint32_t stack_depth = 1;
    uint32_t n_refs = 0;     // leaf references (triangle records) of the scene
    uint32_t n_tris = 0;     // triangles of the scene (the default trace build depends on it)
    std::vector<float> splits[3]; // split positions of the inner nodes per axis, sorted (eye_on_split)
    // inner kd nodes grouped by depth (device ids, deepest level first) and the
    // [offset, count) of each level: the bottom-up pass of the subtree cull boxes
    const uint32_t *d_levels = nullptr;
    std::vector<std::pair<uint32_t, uint32_t>> levels;
    std::vector<void *> scene_bufs;
    // work buffers
    unsigned long long *d_counters = nullptr;
    float *d_accum = nullptr;
    size_t accum_elems = 0;
    void *d_gstack = nullptr, *d_samples = nullptr, *d_run = nullptr, *d_wf = nullptr;
    size_t gstack_bytes = 0, samples_bytes = 0, run_bytes = 0, wf_bytes = 0;
    void *d_cull = nullptr;  // camera-ray cull boxes, one per leaf reference (+ 4), per render
    size_t cull_bytes = 0;
    void *d_cull_node = nullptr; // ... their per-leaf unions, one per kd node
    size_t cull_node_bytes = 0;
    cr_counters last{};
    cr::TraceEvents tev;     // wavefront trace launches of the last render (cr_get_trace_stats)
    cr_trace_stats last_trace{};
    // options
    // Defaults from sweeps on MI355X, sponza stand-in 1080p x 128 spp:
    //   wavefront (kernel 2), trace variant 9, refill 64/56/48, sorted queues, tail below 1M rays
    //   (the persistent megakernel, kernel 0: 615 Mray/s; one thread per pixel, kernel 1: ~60; both removed)
    int kernel = 2;
    int full_counters = 1;
    int lc_debug = 0;                      // measurement only (RenderArgs::lc_debug)
    uint32_t lc_min = 0;                   // RenderArgs::lc_min
    int desc_quorum = -1;                  // RenderArgs::desc_quorum; -1: 8, 0 (off) for SORT_MIN_TRIS <= tris < LEAF_CULL_MIN_TRIS
    uint32_t diag_kinds = 0;               // counting renders: trace kinds of the DIAG_* census (1 << TK_*)
    unsigned long long last_diag[cr::DIAG_N] = {};
    int perf_counters = 0;                 // RenderArgs::perf_counters (option "perf_counters")
    unsigned long long last_perf[cr::TK_N * cr::PERF_N] = {};
    int variant = -1;       // -1: the kernel's default build
    uint32_t refill = 0;    // 0: the default (48)
    uint32_t refill_shadow = 0; // wavefront shadow trace; 0: refill if set, else 56
    uint32_t refill_camera = 0; // wavefront generation-1 closest trace; 0: refill if set, else 64
    uint32_t wf_paths = 256u << 20; // wavefront: paths in flight per chunk (capped by free HBM)
    int wf_sort = -1;               // wavefront: sort large shadow / secondary queues for coherence (-1: scenes
                                    // of at least SORT_MIN_TRIS triangles, cabi.cpp)
    uint32_t wf_sort_min = 1u << 20; // ... of at least this many rays
    // sweep (1080p x 128 spp, refill 56): no sort 807; (8x8 px, 8x8 dirs) 891; (16x16, 16x16) 912;
    // (16x16, 32x32 Morton) 930; (32x32, 32x32) 914 Mray/s
    uint32_t wf_sort_tile = 4;      // key: log2 pixel sub-tile edge
    // direction bins per octahedral axis: 32 -> 64 575.6 -> 570.2 ms per pass, rank 0 of 8 79.6 -> 78.0
    // (world bits 5 / 7 and 16 bins measured slower; 7 bits x 64 bins: 31-bit keys, 607 ms)
    uint32_t wf_dir_res = 128;      // key: direction bins per octahedral axis (round 3: 128 at leaf shift 1,
                                    // 365.1 vs 367.1 ms per pass; halved for leaf keys until they fit 32 bits)
    int wf_world_keys = 2;          // key: world-space origins for queues starting at hits of gen >= 2
    uint32_t wf_world_bits = 6;     // key: Morton bits per axis of the origin
    // closest queues shorter than this finish in one wf_tail launch (0: never).  Sweep, sponza
    // 1080p x 128 spp: 0 / 256K / 1M / 4M / 16M -> 594.7 / 591.6 / 590.2 / 592.9 / 626.5 ms;
    // rank 0 of an 8-way split: 0 / 64K / 256K / 1M / 4M -> 88.8 / 85.9 / 83.3 / 83.1 / 84.2 ms
    uint32_t wf_tail_min = 1u << 20;
    // the tail starts beside the last shadow trace (WfArgs::tail_overlap); measured neutral (round 3:
    // 366.5 / 367.2 vs 366.9 / 366.8 ms per pass, rank 0 of 8 57.25 vs 57.36 ms -- the tail's chains
    // gain one shadow query each and share the GPU with that trace), so off by default
    int wf_tail_overlap = 0;
    uint32_t wf_sort_g1 = 3;        // generation-1 queues sorted: bit 0 shadow, bit 1 closest (WfArgs::sort_g1)
    int wf_cam_lean = 1;            // WfArgs::cam_lean
    // WfArgs::cam_fused (no wf_camera: the packet trace makes the rays) and WfArgs::ctl_ray (the RNG
    // counter in the closest ray, no control slot for generations >= 2); round 4, two interleaved rounds,
    // ms per layer: sponza 1080p x 128 spp 321.8 / 322.3 -> fused 320.1 / 320.5 -> both 318.8 / 319.4;
    // cornell_box 1024^2 x 500 spp 112.9 / 112.4 -> both 108.5 / 106.0 (C2 moves path state, not rays)
    int wf_cam_fuse = 1;
    int wf_ctl_ray = 1;
    // WfArgs::vis_dw; round 4, two interleaved rounds: sponza 318.1 / 317.9 -> 318.0 / 318.3 ms per layer,
    // cornell_box 105.7 / 106.1 -> 105.1 / 105.1 ms per pass
    int wf_vis_dw = 1;
    // WfArgs::vis_mark (round 5)
    int wf_vis_mark = 1;
    // WfArgs::nee_skip; round 4, two interleaved rounds: sponza 316.6 / 317.0 -> 293.7 / 293.1 ms per
    // layer, cornell_box 103.2 / 102.3 -> 95.1 / 95.3 ms per pass, nanobox 144.6 / 145.0 -> 142.9 / 143.0
    int wf_nee_skip = 1;
    uint32_t sum_lds = 0;           // launch_sum_samples' LDS reservation per block (occupancy cap)
    int sum_staged = 1;             // sum_samples_lds (sample runs staged through LDS) when aligned
    int wf_tail_waves = 4;          // WfArgs::tail_waves
    uint32_t wf_dir_res_shadow = 0; // shadow queues' direction bins per axis with leaf keys (0: wf_dir_res)
    // per-sample buffer budget of one sample chunk (cr_set_option "sample_buf_bytes"); a
    // render whose n_items * 12 B * spp exceeds it runs in sample chunks whose running sum
    // carries over in d_run (sum_samples) -- the 4K x 100 spp batches of C5 do
    uint64_t sample_buf = cr::SAMPLE_BUF_BYTES;
    int wf_lanes = 1;                 // wavefront chunks in flight at once (1 or 2)
    // XCD-partitioned queues (WfArgs::xcd bits: 1 shadow, 2 secondary closest, 4 camera rays);
    // sponza 1080p x 128 spp, 2 interleaved rounds: 0 / 1 / 3 / 7 -> 435.1 / 432.4 / 431.4 / 423.1 ms
    // per pass (build 15); build 17: 429.3 -> 416.5 ms with 7
    uint32_t wf_xcd = 7;
    // queue keys from the starting hit's kd leaf (WfArgs::leaf_keys), sponza 1080p x 128 spp,
    // 2 interleaved rounds: pixel / world keys 409.5 -> leaf keys 396.4 ms per pass; coarser
    // regions (node index >> 3 / 6 / 9) 405.2 / 418.7 / 440.2 vs 401.6 ms, 32 direction bins 409.3
    int wf_leaf_keys = 1;
    uint32_t wf_leaf_shift = 1; // ... its node index >> this (a leaf and its sibling share a key region)
    // sweep (1080p x 128 spp, 2 rounds): 0 / 1 / 2 / 4 / 8 / 16 / 64 -> 399.2 / 394.6 / 394.8 / 394.8 / 393.8 / 393.6 / 394.5 ms
    uint32_t wf_resolve_paths = 16; // wf_resolve in path order for queues of at least P / this rays (0: never)
    uint32_t wf_measure_skip = 0;   // WfArgs::measure_skip (measurement only: wrong images)
    // WfArgs::shade_waves (option "wf_shade_waves": 6 or 8); round 4, two interleaved rounds: sponza
    // 322.5 / 322.9 vs 322.6 / 322.2 ms per layer, cornell_box 108.4 / 108.7 vs 107.6 / 107.3 ms per pass
    int wf_shade_waves = 8;
    // wf_shade's append chunk (WfArgs::app_force): 0 = by the queue's length (launch_wavefront_chunk), else
    // this power of two >= 256 whenever the queue arrays have room (tests: the dead entries at small sizes)
    int wf_app_chunk = 0;
    // WfArgs::shade_block (option "wf_shade_block"): threads per wf_shade block, i.e. rays per queue append on
    // sorted queues (round 5, sponza stand-in, two interleaved rounds: 256 -> 2270.9 / 2276.0, 512 -> 2313.8 /
    // 2314.6, 1024 -> 2318.1 / 2314.2 Mray/s -- the same-address append atomics, scripts/append_bench.hip)
    int wf_shade_block = 1024;
    uint32_t node_bfs = cr::NODE_BFS; // nodes numbered breadth-first at the next cr_upload_scene
    // multi-process frame split (cr_comm_init / cr_render_dist_device): one RCCL
    // communicator per process, this rank's compact tile buffer, the root's gather area
    ncclComm_t comm = nullptr;
    int comm_rank = 0, comm_nranks = 1;
    uint32_t comm_timeout_ms = 120000; // cr_comm_init: peers must join within this (option "comm_timeout_ms")
    float *d_tiles = nullptr, *d_gathered = nullptr;
    size_t tiles_bytes = 0, gathered_bytes = 0;
    int *d_flag = nullptr; // one word: the ranks' agreement on a pass group before its gather
    size_t flag_bytes = 0;
};


#define HIPCHK(call)                                                                                                 \
    do {                                                                                                             \
        hipError_t e_ = (call);                                                                                      \
        if (e_ != hipSuccess) return crx::hip_fail(c, e_, #call);                                                    \
    } while (0)

namespace crx {
int fail(cr_ctx *c, int code, const std::string &msg);
int hip_fail(cr_ctx *c, hipError_t e, const char *what);
int check_params(cr_ctx *c, const cr_render_params *p);
uint32_t tile_of(const cr_render_params *p);
int grow(cr_ctx *c, void **buf, size_t &cap, size_t need);
// one render pass of p's tiles (MODE_TILES: compact [tiles][T][T][3] batch means
// into out) or of the whole frame blended into out (MODE_BLEND), on stream st;
// returns after the pass, counters and trace stats are read back
// nl > 1 (wavefront kernel): layers p->layer .. p->layer + nl - 1 in one pass (cr_render_layers_device)
// piece_m > 1 (MODE_TILES): p is piece piece_k of a rank's tiles (rank r + piece_k * N of an
// N * piece_m split), written into the rank's compact buffer of layer stride `stride` floats
int run_render(cr_ctx *c, const cr_camera *cam, const cr_render_params *p, float *out, int mode, hipStream_t st,
               uint32_t nl = 1, uint32_t piece_k = 0, uint32_t piece_m = 1, uint64_t stride = 0);
// group.cpp: the communicator and buffers of the multi-process split (cr_destroy)
void release_dist(cr_ctx *c);
// The largest nl <= want (>= 1) whose paths fit one chunk when p's share (the frame for nranks 1, else rank
// p->rank's tiles) is cut into *m_out pieces, the fewest (cabi.cpp; cr_layers_per_group)
uint32_t group_layers(cr_ctx *c, const cr_render_params *p, uint32_t want, uint32_t *m_out);
// the counters, pass time and trace stats of several passes, summed (pass groups)
struct PassTotals {
    uint64_t ctr[sizeof(cr_counters) / sizeof(uint64_t)] = {};
    float ms = 0.f;
    cr_trace_stats ts{};
    void add(const cr_ctx *c) {
        const uint64_t *h = (const uint64_t *)&c->last;
        for (size_t i = 0; i < sizeof(cr_counters) / sizeof(uint64_t); i++) ctr[i] += h[i];
        ms += c->last_ms;
        for (int kind = 0; kind < 4; kind++) {
            ts.launches[kind] += c->last_trace.launches[kind];
            ts.ms[kind] += c->last_trace.ms[kind];
            ts.inner[kind] += c->last_trace.inner[kind];
            ts.leaf[kind] += c->last_trace.leaf[kind];
            ts.tritest[kind] += c->last_trace.tritest[kind];
        }
    }
    void store(cr_ctx *c) const {
        std::memcpy(&c->last, ctr, sizeof(cr_counters));
        c->last_ms = ms;
        c->last_trace = ts;
    }
};
} // namespace crx
