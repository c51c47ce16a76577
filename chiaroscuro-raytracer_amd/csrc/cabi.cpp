// cabi.cpp -- libchiaro_hip.so: the C-ABI boundary (include/chiaro_hip.h).
//
// Owns the device copies of the scene (re-laid out for the kernels, see
// kernels.hip header), the progressive accumulator, the counters and the
// per-launch HIP events.  No C++ exception or hipError_t crosses the ABI.
#include "ctx.hpp"
#include "leafcull.hpp"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

namespace crx {

int fail(cr_ctx *c, int code, const std::string &msg) {
    if (c) c->err = msg;
    return code;
}
int hip_fail(cr_ctx *c, hipError_t e, const char *what) {
    return fail(c, CR_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
}


void free_scene(cr_ctx *c) {
    for (void *p : c->scene_bufs) hipFree(p);
    c->scene_bufs.clear();
    c->has_scene = false;
    c->S = cr::DevScene{};
    c->d_levels = nullptr;
    c->levels.clear();
}

template <class T> int upload(cr_ctx *c, const std::vector<T> &h, const T **out) {
    void *d = nullptr;
    size_t bytes = h.size() * sizeof(T);
    if (bytes == 0) bytes = 16;
    hipError_t e = hipMalloc(&d, bytes);
    if (e != hipSuccess) return fail(c, CR_E_OOM, std::string("hipMalloc: ") + hipGetErrorString(e));
    c->scene_bufs.push_back(d);
    if (!h.empty()) {
        e = hipMemcpy(d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice);
        if (e != hipSuccess) return hip_fail(c, e, "hipMemcpy(scene)");
    }
    *out = (const T *)d;
    return CR_OK;
}

int check_params(cr_ctx *c, const cr_render_params *p) {
    if (!p) return fail(c, CR_E_INVALID, "null params");
    if (!c->has_scene) return fail(c, CR_E_NOSCENE, "no scene uploaded");
    if (p->xres == 0 || p->yres == 0 || p->spp == 0) return fail(c, CR_E_INVALID, "xres/yres/spp must be > 0");
    if (p->k < 1 || p->k > 64) return fail(c, CR_E_INVALID, "k must be in [1, 64]");
    if (p->layer < 1) return fail(c, CR_E_INVALID, "layer must be >= 1");
    if (p->nranks < 1 || p->rank >= p->nranks) return fail(c, CR_E_INVALID, "bad rank/nranks");
    uint64_t px = (uint64_t)p->xres * p->yres;
    if (px > (1ull << 31)) return fail(c, CR_E_INVALID, "image too large");
    return CR_OK;
}

uint32_t tile_of(const cr_render_params *p) { return p->tile ? p->tile : 32u; }

// Grow-only device work buffer.
int grow(cr_ctx *c, void **buf, size_t &cap, size_t need) {
    if (need <= cap && *buf) return CR_OK;
    if (*buf) hipFree(*buf);
    *buf = nullptr;
    cap = 0;
    if (hipMalloc(buf, need ? need : 16) != hipSuccess) return fail(c, CR_E_OOM, "work buffer");
    cap = need;
    return CR_OK;
}

// scenes with fewer triangles default to trace build 18 instead of 26 (fill_args)
const uint32_t LEAF_CULL_MIN_TRIS = 65536;
// scenes with fewer triangles trace their queues in append order (wf_sort -1, the default): on a
// handful of triangles the whole scene stays in cache whatever the order, and the sort plus the
// trace's reads through the permutation cost more than coherence gains (round 4, cornell_box 1024^2 x
// 500 spp, two interleaved rounds: sorted 9050 / 8894, unsorted 11140 / 11130 Mray/s)
const uint32_t SORT_MIN_TRIS = 1024;

void fill_args(cr_ctx *c, cr::RenderArgs &A, const cr_camera *cam, const cr_render_params *p, float *out, int mode) {
    A.S = c->S;
    std::memcpy(A.cam, cam->eye, 3 * sizeof(float));
    std::memcpy(A.cam + 3, cam->left_upper, 3 * sizeof(float));
    std::memcpy(A.cam + 6, cam->dx, 3 * sizeof(float));
    std::memcpy(A.cam + 9, cam->dy, 3 * sizeof(float));
    A.xres = p->xres;
    A.yres = p->yres;
    A.spp = p->spp;
    A.K = p->k;
    A.bg[0] = p->background[0];
    A.bg[1] = p->background[1];
    A.bg[2] = p->background[2];
    A.seed = p->seed;
    A.layer = p->layer;
    A.nl = 1;
    A.layer_stride = 0;
    A.piece_k = 0;
    A.piece_m = 1;
    A.rank = p->rank;
    A.nranks = p->nranks;
    A.tile = tile_of(p);
    A.tiles_x = (p->xres + A.tile - 1) / A.tile;
    A.n_items = cr_tiles_for_rank(p, p->rank) * A.tile * A.tile;
    A.stack_depth = c->stack_depth;
    A.mode = mode;
    A.out = out;
    A.counters = c->d_counters;
    A.full_counters = c->full_counters;
    A.perf_counters = c->perf_counters;
    A.diag_kinds = c->diag_kinds;
    A.lc_debug = c->lc_debug;
    A.lc_min = c->lc_min;
    // descent rounds end once at most 8 / 64 of a wave's lanes still descend (sponza: 299.9 / 300.6 -> 296.1 /
    // 296.5 ms per layer, 293 with the loop-exit form; 4 / 6 / 12 / 16 / 20 / 32 / 48 slower; cornell_box 97.6 ->
    // 95.8 ms), except on scenes that sort their queues without the leaf-cull build, where full descents
    // measured faster (nanobox stand-in 142.7 -> 146.1 ms at 8)
    A.desc_quorum = c->desc_quorum >= 0 ? (uint32_t)c->desc_quorum
                    : ((c->n_tris >= SORT_MIN_TRIS && c->n_tris < LEAF_CULL_MIN_TRIS) ? 0u : 8u);
    // wavefront: closest 56 / shadow 48 -> 811 Mray/s (48/48: 802, 64/48: 780, 40/48: 783);
    // re-swept under leaf-keyed queues (scripts/gpu_leaf_sweep.sh, 1080p x 128 spp, closest /
    // shadow): 56/48 397.4, 48/56 394.5, 48/48 395.9, 56/56 396.2 ms per pass; a rank of 8:
    // 59.96 vs 59.64 ms -> closest 48 / shadow 56
    A.refill = c->refill ? c->refill : 48u;
    // round 4: 60 on scenes whose queues are sorted (sponza 290.8 / 290.7 -> 289.8 / 290.1 ms per layer, nanobox
    // 143.4 / 143.3 -> 141.8 / 141.6), 56 on the unsorted small ones (cornell_box 95.7 -> 97.7 ms at 60)
    A.refill_shadow = c->refill_shadow ? c->refill_shadow
                                       : (c->refill ? c->refill : (c->n_tris >= SORT_MIN_TRIS ? 60u : 56u));
    // camera rays (64 samples of one pixel per wave): lock-step is best, 64 -> 933 vs 56 -> 924 Mray/s
    A.refill_camera = c->refill_camera ? c->refill_camera : (c->refill ? c->refill : 64u);
    // wavefront trace builds (wavefront.hip kWf): 2 = LDS ring 8, 8 waves/SIMD, scalar loads for
    // wave-uniform nodes / leaves: 1003 vs 935 Mray/s for the same build without them (variant 1);
    // 6 = 2 + fat node records (a node and both children in 32 B: one dependent load per two
    // descent levels): 595.0 vs 597.5 ms per 1080p x 128 spp pass, 83.0 vs 84.2 ms for rank 0 of 8;
    // 9 = 6 with branch-light descent steps and uniform-leaf tests (fewer scalar-unit exec-mask
    // instructions): 563.8 vs 565.5 ms, rank 0 of 8 77.48 vs 77.64 ms (5 interleaved rounds);
    // 14 = 9 whose camera-ray trace skips triangle tests (and whole leaves) outside their
    // screen-space cull boxes (camcull.hpp): camera trace 193 -> 119 ms, 565 -> 489 ms per pass;
    // 15 = 14 that also skips every fetched subtree whose box excludes the sample:
    // camera trace 118 -> 70 ms, 488 -> 439 ms per pass;
    // 17 = 15 whose camera rays traverse one packet (one pixel's 64 samples) per wave:
    // 429.3 vs 435.1 ms per pass (2 interleaved rounds), 416.5 vs 423.1 ms with wf_xcd 7;
    // 18 = 17 with two camera rays per lane (128-ray packets): camera trace 44.1 -> 40.5 ms,
    // 409.7 -> 406.9 ms per pass;
    // 26 = 18 whose secondary closest and shadow traces (and the tail) skip the references a
    // leaf's cull record excludes for the ray (leafcull.hpp, packed fixed-pad form): shadow trace
    // 58.2 -> 53.3 ms per launch, closest 99.8 -> 91.5 ms beside it, 391.5 -> 367 ms per pass
    // the leaf cull (26) pays on large scenes only (round 3, 1080p): sponza stand-in (261k triangles)
    // 391.5 -> 366 ms per pass, nanobox stand-in (20k) 167.6 -> 171.0, cornell_box (36) 147.9 -> 149.3
    // -- on small trees a leaf's references lie close to its cell and the record costs more than
    // the tests it removes -- so scenes below LEAF_CULL_MIN_TRIS triangles default to 18;
    // 40 / 42 = 26 / 18 whose camera packet divides by the rays' RN(1/d) (exact short division,
    // round 3): camera trace 41.1 -> 37.1 ms on the sponza stand-in, 24.1 -> 22.1 on nanobox,
    // 3.54 -> 3.55 on cornell_box (short packets: the reciprocals cost what they save);
    // 43 / 44 = 40 / 42 with the short division in the shadow trace too: 358.2 -> 356.4 ms, nanobox
    // 163.7 -> 162.4 ms; 49 = 43 with the compressed leaf cull records (round 5: 48 B per leaf, three
    // loads instead of six): 2179 -> 2252 Mray/s at the driver's command, shadow 41.7 -> 40.0 ms;
    // 54 = 49 with the leaf exchange in the shadow and secondary closest traces (round 6: a divergent leaf
    // round's masked tests spread over the whole wave): 2315 -> 2362 Mray/s, shadow 39.2 -> 38.3 ms
    // 59 = 54 with the exchange's prefix by a DPP scan: 2348 -> 2395 Mray/s, shadow 38.4 -> 37.6 ms
    A.variant = c->variant >= 0 ? c->variant : (c->n_tris >= LEAF_CULL_MIN_TRIS ? 59 : 44);
    A.eye_on_split = 0;
    for (int a = 0; a < 3; a++)
        if (std::binary_search(c->splits[a].begin(), c->splits[a].end(), cam->eye[a])) A.eye_on_split = 1;
}

// path slots one wavefront chunk may hold: ~45% of the HBM that was free (plus the chunk buffers then
// held) when the ctx first asked after its scene upload.  Kept until the next upload: the plan of a pass group (cr_layers_per_group,
// cr_layers_per_pass) must not change as this ctx's own buffers grow, or ranks that asked at different
// moments would plan different groups and their per-layer gathers would not pair up
// wf_shade may append in chunks (WfArgs::app_chunk: the queues traced in append order, or a forced chunk):
// only then do the queue arrays carry spare slots -- a sorted scene's path cap, and with it the pieces of a
// pass group, stays what it was
bool wf_chunked(const cr_ctx *c) {
    return c->wf_app_chunk || c->wf_sort == 0 || (c->wf_sort < 0 && c->n_tris < SORT_MIN_TRIS);
}
uint64_t wf_path_cap(cr_ctx *c, int k) {
    if (!c->wf_mem_budget) {
        size_t freeb = 0, totalb = 0;
        if (hipMemGetInfo(&freeb, &totalb) != hipSuccess) return ~0ull;
        c->wf_mem_budget = freeb + c->wf_bytes + c->wf2_bytes;
    }
    return (uint64_t)(c->wf_mem_budget * 0.45) / cr::wf_bytes_per_path(k, wf_chunked(c));
}

int run_render(cr_ctx *c, const cr_camera *cam, const cr_render_params *p, float *out, int mode, hipStream_t st,
               uint32_t nl, uint32_t piece_k, uint32_t piece_m, uint64_t stride) {
    if (!cam || !out) return fail(c, CR_E_INVALID, "null camera/output");
    int rc = check_params(c, p);
    if (rc) return rc;
    if (nl < 1 || (nl > 1 && (c->kernel != 2 || c->wf_lanes != 1)))
        return fail(c, CR_E_INVALID, "layers per pass: >= 1, and > 1 only with the wavefront kernel in one lane");
    HIPCHK(hipSetDevice(c->device));
    cr::RenderArgs A{};
    fill_args(c, A, cam, p, out, mode);
    // nl layers in one pass: every item holds nl * spp samples (layer p->layer + s / spp)
    const uint64_t spp_pass = (uint64_t)p->spp * nl;
    if (spp_pass >= (1ull << 31)) return fail(c, CR_E_INVALID, "layers x spp too large");
    A.nl = nl;
    A.layer_stride = (uint64_t)cr_tiles_for_rank(p, 0) * A.tile * A.tile * 3;
    if (piece_m > 1) {
        if (mode != cr::MODE_TILES || piece_k >= piece_m || !stride) return fail(c, CR_E_INVALID, "bad piece");
        A.piece_k = piece_k;
        A.piece_m = piece_m;
        A.layer_stride = stride;
    }
    if (c->kernel == 2 && !c->full_counters && !cr::wf_variant_available(A.variant))
        return fail(c, CR_E_INVALID, "trace build " + std::to_string(A.variant) +
                                         " does not exist (DESIGN.md §3 lists the measured builds that were removed)");
    if (c->perf_counters && (c->kernel != 2 || c->full_counters || !cr::wf_perf_available(A.variant)))
        return fail(c, CR_E_INVALID, "perf_counters: the wavefront kernel's trace builds 18, 26, 40, 42, 43, 44, "
                                     "49, 53, 54 and 59 only, without the counting build");
    c->last_build = c->kernel == 2 ? (c->full_counters ? -1 : A.variant) : -2;
    HIPCHK(hipMemsetAsync(c->d_counters, 0, cr::CTR_SLOTS * sizeof(unsigned long long), st));
    {
        const bool wf = true; // (the wavefront path tracer is the render kernel)
        uint32_t blk, blocks;
        cr::wf_trace_geometry(c->full_counters ? -1 : A.variant, c->num_cus, blk, blocks);
        A.gstride = blk * blocks;
        // samples per chunk: the per-sample buffer stays within SAMPLE_BUF_BYTES
        // and the work index within 31 bits
        const uint64_t per_sample = (uint64_t)A.n_items * 12u;
        uint64_t chunk = std::max<uint64_t>(1, c->sample_buf / std::max<uint64_t>(per_sample, 1));
        chunk = std::min<uint64_t>(chunk, std::max<uint64_t>(1, (1ull << 31) / std::max<uint32_t>(A.n_items, 1)));
        chunk = std::min<uint64_t>(chunk, spp_pass);
        // a chunk of a multiple of 16 samples (sum_samples_lds stages 16 at a time and needs runs of a
        // multiple of 4; the last chunk then has spp mod 4 == its own mod 4)
        if (chunk < spp_pass && chunk >= 16) chunk &= ~(uint64_t)15;
        const bool chunked = chunk < spp_pass;
        if (nl > 1 && chunked) return fail(c, CR_E_INVALID, "layers per pass: the samples do not fit one buffer");
        // wavefront: a second stack-overflow area for the closest trace that runs beside a
        // shadow trace, per lane
        if (cr::gstack_bytes(c->stack_depth, A.gstride) >= (1ull << 32)) // (gstack_at's 32-bit offsets)
            return fail(c, CR_E_INVALID, "stack-overflow area above 4 GiB");
        if (int r = grow(c, &c->d_gstack, c->gstack_bytes, 2 * c->wf_lanes * cr::gstack_bytes(c->stack_depth, A.gstride)))
            return r;
        // large renders reserve the whole sample budget at once: a later pass of another shape (a pass
        // group's frame piece, cr_render_layers) then reuses the buffer instead of regrowing it
        {
            const uint64_t need = per_sample * chunk;
            if (int r = grow(c, &c->d_samples, c->samples_bytes, need * 4 > c->sample_buf ? std::max<uint64_t>(need, c->sample_buf) : need))
                return r;
        }
        if (chunked)
            if (int r = grow(c, &c->d_run, c->run_bytes, per_sample)) return r;
        A.gstack = (uint2 *)c->d_gstack;
        A.samples = (float *)c->d_samples;
        A.run = (float *)c->d_run;
        cr::WfArgs W{};
        cr::WfArgs W2{};
        const int lanes = c->wf_lanes;
        {
            // path slots per wavefront chunk, and the queues / state carved from one buffer
            // per lane ... at most ~45% of the currently free HBM in all (the buffers are
            // reused, so only a growth needs the headroom).  Two lanes: two chunks in flight,
            // the second starting once the first is past its camera-ray trace.
            uint64_t P = (uint64_t)A.n_items * chunk;
            if (lanes == 2) P = (P + 1) / 2;
            P = std::min<uint64_t>(P, c->wf_paths);
            {
                const uint64_t cap = wf_path_cap(c, p->k) / (uint64_t)lanes;
                P = std::max<uint64_t>(std::min<uint64_t>(P, cap), std::min<uint64_t>(P, 1u << 20));
            }
            const size_t f4 = 16 * (size_t)P;
            // queue-indexed arrays hold qspare more slots: the dead entries of wf_shade's chunked appends
            // (WfArgs::app_chunk; at most one partial chunk per block and queue)
            // (option "wf_app_chunk" forces a chunk size: room for it on every block)
            const uint64_t forced = c->wf_app_chunk ? (uint64_t)cr::wf_shade_blocks(c->num_cus, c->wf_shade_waves) * c->wf_app_chunk : 0;
            const bool chunked = wf_chunked(c);
            auto spare_for = [&](uint64_t Pn) {
                return chunked ? std::max<uint64_t>(std::min<uint64_t>(Pn / 8, 8u << 20), forced) : (uint64_t)0;
            };
            const uint64_t Q = P + spare_for(P);
            const size_t fq = 16 * (size_t)Q;
            // queue sorting: by default for scenes of at least SORT_MIN_TRIS triangles only (wf_sort -1)
            const int sort = c->wf_sort >= 0 ? c->wf_sort : (c->n_tris >= SORT_MIN_TRIS ? 1 : 0);
            // queue-sort keys: (pixel sub-tile, octahedral direction bin)
            const uint32_t T = A.tile, sub = (T + (1u << c->wf_sort_tile) - 1) >> c->wf_sort_tile;
            const uint64_t nkeys = (uint64_t)(A.n_items / (T * T)) * sub * sub * c->wf_dir_res * c->wf_dir_res;
            int key_bits = 1;
            while (key_bits < 32 && (1ull << key_bits) < nkeys) key_bits++;
            const int key_bits_pixel = key_bits;
            const uint64_t nworld = (1ull << (3 * c->wf_world_bits)) * c->wf_dir_res * c->wf_dir_res;
            while (c->wf_world_keys && key_bits < 32 && (1ull << key_bits) < nworld) key_bits++;
            // leaf keys: (leaf node >> wf_leaf_shift, direction bin); the direction grid is halved
            // until the key fits 32 bits (the sponza stand-in keeps 128 x 128 bins at shift 1)
            auto leaf_width = [&](uint64_t dres) {
                int b = 1;
                while (b < 40 && (1ull << b) < (((uint64_t)A.S.n_nodes >> c->wf_leaf_shift) + 1) * dres * dres) b++;
                return b;
            };
            uint32_t dres_l = c->wf_dir_res;
            while (dres_l > 8 && leaf_width(dres_l) > 32) dres_l >>= 1;
            const int leaf_bits = leaf_width(dres_l);
            const bool leaf_keys = c->wf_leaf_keys && leaf_bits <= 32;
            // the shadow queues' leaf keys may use another direction grid (option "wf_dir_res_shadow")
            uint32_t dres_s = c->wf_dir_res_shadow ? c->wf_dir_res_shadow : dres_l;
            while (dres_s > 1 && leaf_width(dres_s) > 32) dres_s >>= 1;
            const int leaf_bits_s = leaf_width(dres_s);
            // (leaf keys replace the pixel and world keys in every queue: their width alone sets the
            // digit passes)
            if (leaf_keys) key_bits = leaf_bits;
            // bytes of the buffers of a chunk of Pn paths with kb-bit sort keys
            auto need_for = [&](uint64_t Pn, int kb) -> size_t {
                const uint64_t Qn = Pn + spare_for(Pn);
                const size_t st = sort ? cr::wf_sort_tmp_bytes((uint32_t)Qn, kb) : 0;
                return (4 + 2 + 2) * 16 * (size_t)Qn + 8 * (size_t)Qn +
                       (cr::WF_STATE + 2 * (size_t)p->k) * 16 * (size_t)Pn + 9 * (size_t)Pn +
                       (sort ? 32 * (size_t)Qn + st : 0) + cr::WF_CNT * sizeof(uint32_t) + 8192;
            };
            const size_t sort_tmp = sort ? cr::wf_sort_tmp_bytes((uint32_t)Q, key_bits) : 0;
            const size_t need = need_for(P, key_bits);
            // a chunk of more than a quarter of the path cap reserves the buffers of a whole-cap chunk
            // with the widest keys, so passes of other sizes (a pass group's frame pieces, the next
            // layer) reuse them instead of regrowing ~100 GB inside a timed render
            size_t need_alloc = need;
            {
                const uint64_t pcap = std::min<uint64_t>(c->wf_paths, wf_path_cap(c, p->k) / (uint64_t)lanes);
                if (P * 4 > pcap) need_alloc = std::max(need, need_for(std::max<uint64_t>(P, pcap), 32));
            }
            if (int r = grow(c, &c->d_wf, c->wf_bytes, need_alloc)) return r;
            if (lanes == 2)
                if (int r = grow(c, &c->d_wf2, c->wf2_bytes, need_alloc)) return r;
            auto carve = [&](void *base, cr::WfArgs &W, int lane) {
                char *b = (char *)base;
                auto take = [&](size_t bytes) {
                    char *r = b;
                    b += (bytes + 255) & ~(size_t)255;
                    return r;
                };
                W.ray[0] = (float4 *)take(2 * fq);
                W.ray[1] = (float4 *)take(2 * fq);
                W.hit[0] = (uint4 *)take(fq);
                W.hit[1] = (uint4 *)take(fq);
                W.sray = (float4 *)take(2 * fq);
                W.ps = (float4 *)take(cr::WF_STATE * f4);
                W.dw = (float4 *)take(2 * (size_t)p->k * f4);
                W.sexcl = (uint32_t *)take(4 * (size_t)Q);
                W.occ = (uint32_t *)take(4 * (size_t)Q);
                W.qspare = (uint32_t)(Q - P);
                W.app_force = (uint32_t)c->wf_app_chunk;
                W.shade_block = (uint32_t)c->wf_shade_block;
                W.cnt = (uint32_t *)take(cr::WF_CNT * sizeof(uint32_t));
                W.cxy = (float2 *)take(8 * (size_t)P);
                W.mark = (uint8_t *)take((size_t)P);
                W.shade_waves = c->wf_shade_waves;
                W.sort = sort && nkeys <= (1ull << 32);
                W.key_bits = key_bits;
                W.key_bits_pixel = key_bits_pixel;
                W.sort_min = c->wf_sort_min;
                W.sort_tile = c->wf_sort_tile;
                W.dir_res = leaf_keys ? dres_l : c->wf_dir_res;
                W.dir_res_s = leaf_keys ? dres_s : c->wf_dir_res;
                W.key_bits_s = leaf_keys ? leaf_bits_s : key_bits;
                W.world_keys = nworld <= (1ull << 32) ? c->wf_world_keys : 0;
                W.world_bits = c->wf_world_bits;
                W.tail_min = c->wf_tail_min;
                W.xcd = c->wf_xcd;
                W.leaf_keys = leaf_keys ? 1 : 0;
                W.leaf_shift = c->wf_leaf_shift;
                W.resolve_paths = c->wf_resolve_paths;
                W.measure_skip = c->wf_measure_skip;
                W.tail_overlap = c->wf_tail_overlap;
                W.sort_g1 = c->wf_sort_g1;
                W.cam_lean = c->wf_cam_lean;
                W.cam_fused = c->wf_cam_fuse;
                W.ctl_ray = c->wf_ctl_ray;
                W.vis_dw = c->wf_vis_dw;
                W.vis_mark = c->wf_vis_mark && !c->wf_tail_overlap && p->k <= 63 ? 1 : 0;
                W.nee_skip = c->wf_nee_skip;
                W.tail_waves = c->wf_tail_waves;
                if (sort) {
                    for (int q = 0; q < 2; q++)
                        for (int i = 0; i < 2; i++) {
                            W.key[q][i] = (uint32_t *)take(4 * (size_t)Q);
                            W.perm[q][i] = (uint32_t *)take(4 * (size_t)Q);
                        }
                    W.sort_tmp = take(sort_tmp);
                    W.sort_tmp_bytes = sort_tmp;
                }
                const size_t area = (size_t)c->stack_depth * A.gstride;
                W.gstack = A.gstack + 2 * (size_t)lane * area;
                W.gstack2 = W.gstack + area;
                W.gstride = A.gstride;
                W.P = (uint32_t)P;
            };
            carve(c->d_wf, W, 0);
            if (lanes == 2) carve(c->d_wf2, W2, 1);
        }
        // screen-space cull boxes of this camera for the camera-ray trace (camcull.hpp),
        // computed inside the timed region of every render
        // (built for triangle-less scenes too: the culling kernels read them unconditionally, and
        // with n_refs + 4 empty boxes every sample is outside)
        const bool cull = wf && !c->full_counters && cr::wf_variant_culls(A.variant);
        if (cull) {
            if (int r = grow(c, &c->d_cull, c->cull_bytes, 16 * ((size_t)c->n_refs + 4))) return r;
            if (int r = grow(c, &c->d_cull_node, c->cull_node_bytes, 16 * (size_t)c->S.n_nodes)) return r;
        }
        A.cull = cull ? (const float4 *)c->d_cull : nullptr;
        A.cull_node = cull ? (const float4 *)c->d_cull_node : nullptr;
        c->tev.n = 0;
        c->tev.chunked = 0;
        HIPCHK(hipEventRecord(c->ev0, st));
        if (cull)
            if (int e = cr::launch_cam_cull(A, c->n_refs, (float4 *)c->d_cull, (float4 *)c->d_cull_node, c->d_levels,
                                            (const uint32_t(*)[2])c->levels.data(), (int)c->levels.size(), st))
                return hip_fail(c, (hipError_t)e, "cull-box kernel launch");
        for (uint32_t s0 = 0; s0 < spp_pass; s0 += (uint32_t)chunk) {
            A.s0 = s0;
            A.s_count = (uint32_t)std::min<uint64_t>(chunk, spp_pass - s0);
            A.n_work = A.n_items * A.s_count;
            int e = 0;
            if (lanes == 2) {
                cr::WfLane L[2] = {{W, st, c->wfs.side, c->wfs.fork, c->wfs.join, c->lane_ev[0], c->hcnt},
                                   {W2, c->stream2, c->side2, c->fork2, c->join2, c->lane_ev[1], c->hcnt + 2}};
                e = cr::run_wavefront_lanes(A, L, 2, c->num_cus, st, &c->tev);
            } else {
                const uint32_t P = W.P;
                for (uint32_t w0 = 0; w0 < A.n_work && !e; w0 += P) {
                    W.w0 = w0;
                    W.P = std::min(P, A.n_work - w0);
                    HIPCHK(hipMemsetAsync(W.cnt, 0, cr::WF_CNT * sizeof(uint32_t), st));
                    e = cr::launch_wavefront_chunk(A, W, c->num_cus, st, c->wfs, &c->tev);
                }
                W.P = P;
            }
            if (!e) e = cr::launch_sum_samples(A, s0 == 0, s0 + A.s_count == spp_pass, st, c->sum_lds, c->sum_staged != 0);
            if (e) return hip_fail(c, (hipError_t)e, "render kernel launch");
        }
        HIPCHK(hipEventRecord(c->ev1, st));
    }
    unsigned long long h[cr::CTR_SLOTS];
    HIPCHK(hipMemcpyAsync(h, c->d_counters, sizeof(h), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    HIPCHK(hipEventElapsedTime(&c->last_ms, c->ev0, c->ev1));
    c->last = cr_counters{h[0], h[1],  h[2],  h[3],  h[4],  h[5],  h[6],  h[7], h[8],
                          h[9], h[10], h[11], h[12], h[13], h[14], h[15], h[16],
                          h[17], h[18], h[19], h[20], h[21], h[cr::CTR_NEE]};
    for (int i = 0; i < cr::DIAG_N; i++) c->last_diag[i] = h[cr::CTR_DIAG + i];
    for (int i = 0; i < cr::TK_N * cr::PERF_N; i++) c->last_perf[i] = h[cr::CTR_PERF + i];
    c->last_trace = cr_trace_stats{};
    if (c->kernel == 2) {
        for (int i = 0; i < c->tev.n; i++) {
            float ms = 0.f;
            HIPCHK(hipEventElapsedTime(&ms, c->tev.ev[2 * i], c->tev.ev[2 * i + 1]));
            const int k = c->tev.kind[i];
            c->last_trace.launches[k]++;
            c->last_trace.ms[k] += ms;
        }
        c->last_trace.chunked_shades = (uint64_t)c->tev.chunked;
        for (int k = 0; k < cr::TK_TAIL; k++) { // the tail kernel's work is not split by kind
            c->last_trace.inner[k] = h[cr::CTR_TRACE + 3 * k];
            c->last_trace.leaf[k] = h[cr::CTR_TRACE + 3 * k + 1];
            c->last_trace.tritest[k] = h[cr::CTR_TRACE + 3 * k + 2];
        }
    }
    return CR_OK;
}

} // namespace crx

using namespace crx;

extern "C" {

cr_ctx *cr_create(int device) {
    cr_ctx *c = new cr_ctx();
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
        c->err = "no HIP device";
        return c; // error surfaced on first use; cr_last_error explains
    }
    if (device < 0 || device >= n) {
        c->err = "bad device index";
        return c;
    }
    c->device = device;
    if (hipSetDevice(device) != hipSuccess) {
        c->err = "hipSetDevice failed";
        c->device = -1;
        return c;
    }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess) c->num_cus = prop.multiProcessorCount;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&c->wfs.side, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&c->wfs.fork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->wfs.join, hipEventDisableTiming) != hipSuccess ||
        hipStreamCreateWithFlags(&c->stream2, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&c->side2, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&c->fork2, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->join2, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->lane_ev[0], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->lane_ev[1], hipEventDisableTiming) != hipSuccess ||
        hipHostMalloc((void **)&c->hcnt, 4 * sizeof(uint32_t), hipHostMallocDefault) != hipSuccess ||
        hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess ||
        hipMalloc(&c->d_counters, cr::CTR_SLOTS * sizeof(unsigned long long)) != hipSuccess) {
        c->err = "device init failed";
        c->device = -1;
    }
    return c;
}

void cr_destroy(cr_ctx *c) {
    if (!c) return;
    if (c->device >= 0) {
        hipSetDevice(c->device);
        release_dist(c);
        free_scene(c);
        if (c->d_accum) hipFree(c->d_accum);
        if (c->d_gstack) hipFree(c->d_gstack);
        if (c->d_samples) hipFree(c->d_samples);
        if (c->d_run) hipFree(c->d_run);
        if (c->d_wf) hipFree(c->d_wf);
        if (c->d_cull) hipFree(c->d_cull);
        if (c->d_cull_node) hipFree(c->d_cull_node);
        if (c->d_counters) hipFree(c->d_counters);
        if (c->ev0) hipEventDestroy(c->ev0);
        for (int i = 0; i < 2 * c->tev.cap; i++) hipEventDestroy(c->tev.ev[i]);
        delete[] c->tev.ev;
        delete[] c->tev.kind;
        if (c->ev1) hipEventDestroy(c->ev1);
        if (c->stream) hipStreamDestroy(c->stream);
        if (c->wfs.side) hipStreamDestroy(c->wfs.side);
        if (c->wfs.fork) hipEventDestroy(c->wfs.fork);
        if (c->wfs.join) hipEventDestroy(c->wfs.join);
        if (c->stream2) hipStreamDestroy(c->stream2);
        if (c->side2) hipStreamDestroy(c->side2);
        if (c->fork2) hipEventDestroy(c->fork2);
        if (c->join2) hipEventDestroy(c->join2);
        for (hipEvent_t e : c->lane_ev)
            if (e) hipEventDestroy(e);
        if (c->hcnt) hipHostFree(c->hcnt);
        if (c->d_wf2) hipFree(c->d_wf2);
    }
    delete c;
}

const char *cr_last_error(cr_ctx *c) { return c ? c->err.c_str() : "null context"; }

int cr_upload_scene(cr_ctx *c, const cr_scene_desc *d) {
    if (!c) return CR_E_INVALID;
    if (c->device < 0) return fail(c, CR_E_HIP, c->err.empty() ? "no device" : c->err);
    if (!d || !d->nodes || d->n_nodes == 0) return fail(c, CR_E_INVALID, "empty kd tree");
    if (d->n_tris && (!d->tri_pos || !d->tri_normal || !d->tri_kd || !d->tri_ke || !d->tri_uv))
        return fail(c, CR_E_INVALID, "missing triangle arrays");
    if (d->max_depth > 256) return fail(c, CR_E_DEPTH, "kd tree deeper than 256");
    HIPCHK(hipSetDevice(c->device));
    free_scene(c);
    // a new scene re-queries the path budget at its first plan (wf_path_cap): buffers grown since the last
    // query (gather and tile buffers, the caller's own tensors) must not leave the chunk cap above the HBM
    // that is free now.  Ranks still agree on a group's plan: plan_layers' all-reduce MIN, and the per-group
    // agreement of cr_render_dist_layers_device / cr_group_render_layers
    c->wf_mem_budget = 0;
    const uint32_t nt = d->n_tris;
    // nodes -> {split bits | first, axis | child<<2}, validated first
    const uint32_t NN = d->n_nodes;
    for (uint32_t i = 0; i < NN; i++) {
        const cr_kdnode &n = d->nodes[i];
        if (n.axis == 3) {
            if (n.count >= (1u << 30) || (uint64_t)n.child_or_first + n.count > d->n_refs)
                return fail(c, CR_E_INVALID, "bad leaf range");
        } else if (n.axis > 2 || (uint64_t)n.child_or_first + 1 >= NN || n.child_or_first >= (1u << 30)) {
            return fail(c, CR_E_INVALID, "bad inner node");
        }
    }
    // node numbering: the first NODE_BFS nodes breadth-first from the root (each inner
    // node's two children take consecutive ids, as KDTree::build allocates them), the
    // rest in the reference's depth-first order -- the top of the tree is nodes
    // 0..NODE_BFS-1 for the LDS node tile; only addresses change, not the traversal
    std::vector<uint32_t> newid(NN, 0xffffffffu), order;
    order.reserve(NN);
    order.push_back(0);
    newid[0] = 0;
    for (size_t h = 0; h < order.size() && order.size() + 2 <= c->node_bfs; h++) {
        const cr_kdnode &n = d->nodes[order[h]];
        if (n.axis == 3) continue;
        for (uint32_t k = 0; k < 2; k++) {
            const uint32_t ch = n.child_or_first + k;
            if (newid[ch] != 0xffffffffu) return fail(c, CR_E_INVALID, "kd node with two parents");
            newid[ch] = (uint32_t)order.size();
            order.push_back(ch);
        }
    }
    for (uint32_t i = 0; i < NN; i++)
        if (newid[i] == 0xffffffffu) {
            newid[i] = (uint32_t)order.size();
            order.push_back(i);
        }
    std::vector<uint2> nodes(NN);
    for (uint32_t i = 0; i < NN; i++) {
        const cr_kdnode &n = d->nodes[i];
        if (n.axis == 3) {
            nodes[newid[i]] = make_uint2(n.child_or_first, 3u | (n.count << 2));
        } else {
            const uint32_t ch = newid[n.child_or_first];
            if (newid[n.child_or_first + 1] != ch + 1) return fail(c, CR_E_INVALID, "kd siblings not adjacent");
            uint32_t sb;
            std::memcpy(&sb, &n.split, 4);
            nodes[newid[i]] = make_uint2(sb, n.axis | (ch << 2));
        }
    }
    // fat node records: a node's own record followed by both children's
    if ((uint64_t)32 * d->n_nodes > 0xFFFFFFFFull) return fail(c, CR_E_INVALID, "more than 134 M kd nodes");
    std::vector<uint4> fat((size_t)2 * d->n_nodes, make_uint4(0u, 0u, 0u, 0u));
    for (uint32_t i = 0; i < d->n_nodes; i++) {
        const uint2 n = nodes[i];
        fat[2 * (size_t)i].x = n.x;
        fat[2 * (size_t)i].y = n.y;
        if ((n.y & 3u) != 3u) {
            const uint32_t ch = n.y >> 2;
            fat[2 * (size_t)i].z = nodes[ch].x;
            fat[2 * (size_t)i].w = nodes[ch].y;
            fat[2 * (size_t)i + 1] = make_uint4(nodes[ch + 1].x, nodes[ch + 1].y, 0u, 0u);
        }
    }
    // leaf-ordered triangle records {A,id},{B-A},{C-A}: e1/e2 computed exactly as
    // intersectRayTriangle does each time (kdtree.cpp:222-223), so bit-identical.
    // load_rec addresses records with a 32-bit byte offset
    if ((uint64_t)16 * cr::REC_STRIDE * ((uint64_t)d->n_refs + 1) > 0xFFFFFFFFull)
        return fail(c, CR_E_INVALID, "more than 89 M leaf references (triangle records exceed 4 GiB)");
    // + one zero record past the last (an empty leaf's `first` may be n_refs)
    std::vector<float4> recs((size_t)cr::REC_STRIDE * ((size_t)d->n_refs + 1), make_float4(0.f, 0.f, 0.f, 0.f));
    for (uint32_t r = 0; r < d->n_refs; r++) {
        const uint32_t t = d->refs[r];
        if (t >= nt) return fail(c, CR_E_INVALID, "leaf ref out of range");
        const float *p = d->tri_pos + 9 * (size_t)t;
        float idf;
        std::memcpy(&idf, &t, 4);
        float4 *q = recs.data() + (size_t)cr::REC_STRIDE * r;
        q[0] = make_float4(p[0], p[1], p[2], idf);
        q[1] = make_float4(p[3] - p[0], p[4] - p[1], p[5] - p[2], 0.f);
        q[2] = make_float4(p[6] - p[0], p[7] - p[1], p[8] - p[2], 0.f);
    }
    // leaf cull records (leafcull.hpp), per node of the new numbering; host threads.  The per-ray and
    // fixed-pad forms stay on the host: they are the steps from which the packed (LC 4) and the
    // compressed (LC 5) records the traces read are derived
    std::vector<float4> lcull((size_t)cr::LC_REC * NN, make_float4(0.f, 0.f, 0.f, 0.f));
    {
        const unsigned nth = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
        std::vector<std::thread> th;
        for (unsigned w = 0; w < nth; w++)
            th.emplace_back([&, w] {
                float A[cr::LC_MAXREFS][3], e1[cr::LC_MAXREFS][3], e2[cr::LC_MAXREFS][3];
                for (uint32_t i = w; i < NN; i += nth) {
                    if ((nodes[i].y & 3u) != 3u) continue;
                    const uint32_t first = nodes[i].x, cnt = nodes[i].y >> 2;
                    const uint32_t m = std::min(cnt, (uint32_t)cr::LC_MAXREFS);
                    for (uint32_t j = 0; j < m; j++) {
                        const float4 *q = recs.data() + (size_t)cr::REC_STRIDE * (first + j);
                        A[j][0] = q[0].x, A[j][1] = q[0].y, A[j][2] = q[0].z;
                        e1[j][0] = q[1].x, e1[j][1] = q[1].y, e1[j][2] = q[1].z;
                        e2[j][0] = q[2].x, e2[j][1] = q[2].y, e2[j][2] = q[2].z;
                    }
                    cr::leaf_cull_record(A, e1, e2, cnt, (cr::LcFloat4 *)(lcull.data() + (size_t)cr::LC_REC * i));
                }
            });
        for (auto &t : th) t.join();
    }
    // ... and in the fixed-pad form: origins and vertices inside the padded box (+1: the 0.001 n offsets)
    std::vector<float4> lcullf((size_t)cr::LC_REC * NN, make_float4(0.f, 0.f, 0.f, 0.f));
    double lc_db = 1.0;
    {
        double &db = lc_db, smax = 0.0;
        for (int i = 0; i < 3; i++) {
            db = std::max(db, std::max(std::fabs((double)d->box_min[i]), std::fabs((double)d->box_max[i])) + 1.0);
            smax = std::max(smax, (double)d->box_max[i] - (double)d->box_min[i] + 2.0);
        }
        db *= 1.0001;
        for (uint32_t i = 0; i < NN; i++)
            cr::leaf_cull_fixed((const cr::LcFloat4 *)(lcull.data() + (size_t)cr::LC_REC * i), db, smax,
                                (cr::LcFloat4 *)(lcullf.data() + (size_t)cr::LC_REC * i));
    }
    std::vector<float4> lcullp((size_t)cr::LC_RECP * NN, make_float4(0.f, 0.f, 0.f, 0.f));
    for (uint32_t i = 0; i < NN; i++)
        cr::leaf_cull_pack((const cr::LcFloat4 *)(lcullf.data() + (size_t)cr::LC_REC * i),
                           (nodes[i].y & 3u) == 3u ? nodes[i].y >> 2 : 0u,
                           (cr::LcFloat4 *)(lcullp.data() + (size_t)cr::LC_RECP * i));
    // ... and compressed on the scene's grid (48 B per node, LC 5)
    cr::LcGrid lcg = cr::lc_grid_make((const cr::LcFloat4 *)lcullf.data(), NN, lc_db);
    cr::lc_grid_dt(lcg, (const cr::LcFloat4 *)lcullf.data(), NN);
    std::vector<uint4> lcullc((size_t)cr::LC_RECC * NN, make_uint4(0u, 0u, 0u, 0u));
    for (uint32_t i = 0; i < NN; i++)
        cr::leaf_cull_compress((const cr::LcFloat4 *)(lcull.data() + (size_t)cr::LC_REC * i),
                               (const cr::LcFloat4 *)(lcullf.data() + (size_t)cr::LC_REC * i),
                               (nodes[i].y & 3u) == 3u ? nodes[i].y >> 2 : 0u, lcg,
                               (uint32_t *)(lcullc.data() + (size_t)cr::LC_RECC * i));
    std::vector<float4> tri((size_t)3 * nt), mn(nt), mkd(nt), mke(nt);
    std::vector<float2> muv((size_t)3 * nt);
    for (uint32_t t = 0; t < nt; t++) {
        const float *p = d->tri_pos + 9 * (size_t)t;
        for (int v = 0; v < 3; v++) tri[3 * (size_t)t + v] = make_float4(p[3 * v], p[3 * v + 1], p[3 * v + 2], 0.f);
        const uint32_t em = d->tri_emissive ? (d->tri_emissive[t] ? 1u : 0u)
                                            : ((d->tri_ke[3 * t] > 0.f || d->tri_ke[3 * t + 1] > 0.f ||
                                                d->tri_ke[3 * t + 2] > 0.f) ? 1u : 0u);
        float emf;
        std::memcpy(&emf, &em, 4);
        mn[t] = make_float4(d->tri_normal[3 * t], d->tri_normal[3 * t + 1], d->tri_normal[3 * t + 2], emf);
        int32_t ti = d->tri_tex ? d->tri_tex[t] : -1;
        if (ti >= (int32_t)d->n_textures) return fail(c, CR_E_INVALID, "texture index out of range");
        float tif;
        std::memcpy(&tif, &ti, 4);
        mkd[t] = make_float4(d->tri_kd[3 * t], d->tri_kd[3 * t + 1], d->tri_kd[3 * t + 2], tif);
        mke[t] = make_float4(d->tri_ke[3 * t], d->tri_ke[3 * t + 1], d->tri_ke[3 * t + 2], 0.f);
        for (int v = 0; v < 3; v++)
            muv[3 * (size_t)t + v] = make_float2(d->tri_uv[6 * t + 2 * v], d->tri_uv[6 * t + 2 * v + 1]);
    }
    std::vector<uint2> lights(d->n_lights);
    for (uint32_t i = 0; i < d->n_lights; i++) {
        if (d->light_id[i] >= nt) return fail(c, CR_E_INVALID, "light id out of range");
        uint32_t sb;
        std::memcpy(&sb, &d->light_surface[i], 4);
        lights[i] = make_uint2(d->light_id[i], sb);
    }
    std::vector<uint4> texs(d->n_textures);
    std::vector<uint8_t> texels;
    for (uint32_t i = 0; i < d->n_textures; i++) {
        const cr_texture &t = d->textures[i];
        if (t.width <= 0 || t.height <= 0 || t.components <= 0 || !t.data)
            return fail(c, CR_E_INVALID, "bad texture");
        size_t off = (texels.size() + 15) & ~(size_t)15;
        size_t bytes = (size_t)t.width * t.height * t.components;
        texels.resize(off + bytes + cr::tex_pad(t.width, t.components), 0);
        std::memcpy(texels.data() + off, t.data, bytes);
        if (off > 0xffffffffull) return fail(c, CR_E_INVALID, "texture atlas > 4 GiB");
        texs[i] = make_uint4((uint32_t)t.width, (uint32_t)t.height, (uint32_t)t.components, (uint32_t)off);
    }
    // inner nodes grouped by depth, deepest level first (children have larger ids than
    // their parent in this numbering: one forward pass gives the depths)
    std::vector<uint32_t> depth(NN, 0), levels;
    std::vector<std::pair<uint32_t, uint32_t>> level_off;
    uint32_t tree_depth = 0; // deepest node (root = 0): the most entries a traversal stack holds
    {
        uint32_t maxd = 0;
        for (uint32_t i = 0; i < NN; i++) {
            tree_depth = std::max(tree_depth, depth[i]);
            if ((nodes[i].y & 3u) == 3u) continue;
            const uint32_t ch = nodes[i].y >> 2;
            if (ch <= i) return fail(c, CR_E_INVALID, "kd child numbered before its parent");
            depth[ch] = depth[ch + 1] = depth[i] + 1;
            maxd = std::max(maxd, depth[i]);
        }
        // the stacks (LDS rings, gstack, the packet trace's PACKET_DEPTH node stack) are sized
        // from the tree itself, never from the caller's declared max_depth
        if (tree_depth > 256) return fail(c, CR_E_DEPTH, "kd tree deeper than 256");
        std::vector<uint32_t> cnt(maxd + 1, 0);
        for (uint32_t i = 0; i < NN; i++)
            if ((nodes[i].y & 3u) != 3u) cnt[depth[i]]++;
        uint32_t off = 0;
        for (int dd = (int)maxd; dd >= 0; dd--) {
            level_off.emplace_back(off, cnt[dd]);
            off += cnt[dd];
        }
        levels.resize(off);
        std::vector<uint32_t> pos(maxd + 1);
        for (uint32_t dd = 0; dd <= maxd; dd++) pos[dd] = level_off[maxd - dd].first;
        for (uint32_t i = 0; i < NN; i++)
            if ((nodes[i].y & 3u) != 3u) levels[pos[depth[i]]++] = i;
    }
    const uint32_t *levels_dev = nullptr;
    int rc;
    if ((rc = upload(c, levels, &levels_dev))) {
        free_scene(c);
        return rc;
    }
    if ((rc = upload(c, nodes, &c->S.nodes)) || (rc = upload(c, fat, &c->S.fat)) || (rc = upload(c, recs, &c->S.recs)) ||
        (rc = upload(c, lcullp, &c->S.lcullp)) || (rc = upload(c, lcullc, &c->S.lcullc)) || (rc = upload(c, tri, &c->S.tri)) ||
        (rc = upload(c, mn, &c->S.mat_n)) || (rc = upload(c, mkd, &c->S.mat_kd)) || (rc = upload(c, mke, &c->S.mat_ke)) ||
        (rc = upload(c, muv, &c->S.mat_uv)) || (rc = upload(c, lights, &c->S.lights)) ||
        (rc = upload(c, texs, &c->S.texs)) || (rc = upload(c, texels, &c->S.texels))) {
        free_scene(c);
        return rc;
    }
    c->S.lcg = lcg;
    c->S.nlights = d->n_lights;
    c->S.n_nodes = d->n_nodes;
    c->S.bmin = make_float3(d->box_min[0], d->box_min[1], d->box_min[2]);
    c->S.bmax = make_float3(d->box_max[0], d->box_max[1], d->box_max[2]);
    {
        double db = 1.0; // every origin (a hit point + 0.001 n) and vertex lies in the padded box
        for (int i = 0; i < 3; i++)
            db = std::max(db, std::max(std::fabs((double)d->box_min[i]), std::fabs((double)d->box_max[i])) + 1.0);
        c->S.db = (float)(db * 1.0001);
    }
    c->stack_depth = std::max(tree_depth, std::max(d->max_depth, 1u));
    c->n_refs = d->n_refs;
    c->n_tris = d->n_tris;
    for (int a = 0; a < 3; a++) c->splits[a].clear();
    for (uint32_t i = 0; i < NN; i++)
        if (d->nodes[i].axis < 3) c->splits[d->nodes[i].axis].push_back(d->nodes[i].split);
    for (int a = 0; a < 3; a++) std::sort(c->splits[a].begin(), c->splits[a].end());
    c->d_levels = levels_dev;
    c->levels = std::move(level_off);
    c->has_scene = true;
    return CR_OK;
}

int cr_tile_origin(const cr_render_params *p, uint32_t rank, uint32_t local, uint32_t *x0, uint32_t *y0) {
    if (!p || !x0 || !y0 || local >= cr_tiles_for_rank(p, rank)) return CR_E_INVALID;
    const uint32_t T = tile_of(p), tx = (p->xres + T - 1) / T, s = rank + local * p->nranks;
    *x0 = cr::tile_slot_column(s, tx, p->nranks) * T;
    *y0 = s / tx * T;
    return CR_OK;
}

uint32_t cr_tiles_for_rank(const cr_render_params *p, uint32_t rank) {
    if (!p || p->nranks == 0 || rank >= p->nranks || p->xres == 0 || p->yres == 0) return 0;
    const uint32_t T = tile_of(p);
    const uint32_t nt = ((p->xres + T - 1) / T) * ((p->yres + T - 1) / T);
    return nt > rank ? (nt - rank + p->nranks - 1) / p->nranks : 0;
}

int cr_render(cr_ctx *c, const cr_camera *cam, const cr_render_params *p, float *accum_rgb_out) {
    if (!c) return CR_E_INVALID;
    if (c->device < 0) return fail(c, CR_E_HIP, c->err.empty() ? "no device" : c->err);
    if (!accum_rgb_out || !p) return fail(c, CR_E_INVALID, "null output/params");
    cr_render_params q = *p;
    if (q.nranks == 0) q.nranks = 1;
    int rc = check_params(c, &q);
    if (rc) return rc;
    HIPCHK(hipSetDevice(c->device));
    const size_t elems = (size_t)q.xres * q.yres * 3;
    if (elems != c->accum_elems) {
        if (c->d_accum) hipFree(c->d_accum);
        c->d_accum = nullptr;
        c->accum_elems = 0;
        if (hipMalloc(&c->d_accum, elems * sizeof(float)) != hipSuccess) return fail(c, CR_E_OOM, "accumulator");
        c->accum_elems = elems;
        HIPCHK(hipMemset(c->d_accum, 0, elems * sizeof(float)));
    }
    rc = run_render(c, cam, &q, c->d_accum, cr::MODE_BLEND, c->stream);
    if (rc) return rc;
    HIPCHK(hipMemcpy(accum_rgb_out, c->d_accum, elems * sizeof(float), hipMemcpyDeviceToHost));
    return CR_OK;
}


// cr_render over nlayers layers in pass groups: up to LAYER_GROUP layers per pass, the frame cut
// into the fewest tile-split pieces whose paths fit one chunk (DistributedFrame.plan_layers)
static const uint32_t LAYER_GROUP = 32, MAX_PIECES = 64;
// frame pieces pay on scenes with real geometry (sponza stand-in 353 -> 324 ms per layer, 4K 1122 ->
// 987, nanobox stand-in 1922 -> 2173 Mray/s) and lose on a handful of triangles (cornell_box, 36:
// 147.6 -> 153.8 ms per layer), whose queues gain no coherence from denser passes
static const uint32_t PIECES_MIN_TRIS = 1024;
uint32_t cr_scene_triangles(cr_ctx *c) { return c && c->has_scene ? c->n_tris : 0u; }
// The largest nl <= want (>= 1) whose paths fit one chunk when p's share is cut into *m pieces (the
// fewest; scenes of at least PIECES_MIN_TRIS triangles only): for the whole frame (nranks 1) the
// ranks of an m-way split, for rank r of N the ranks r + kN of an N * m split
} // extern "C"
uint32_t crx::group_layers(cr_ctx *c, const cr_render_params *p, uint32_t want, uint32_t *m_out) {
    *m_out = 1;
    const uint32_t N = p->nranks ? p->nranks : 1;
    const uint32_t share = cr_tiles_for_rank(p, p->rank);
    const uint32_t maxm = c->n_tris < PIECES_MIN_TRIS ? 1u : std::min(MAX_PIECES, std::max(share, 1u));
    for (uint32_t nl = std::max(want, 1u); nl > 1; nl--)
        for (uint32_t m = 1; m <= maxm; m++) {
            cr_render_params t = *p;
            t.nranks = N * m;
            t.rank = N == 1 ? 0 : p->rank; // the largest piece
            if (cr_layers_per_pass(c, &t, nl) == nl) {
                *m_out = m;
                return nl;
            }
        }
    return 1;
}
extern "C" {

uint32_t cr_layers_per_group(cr_ctx *c, const cr_render_params *p, uint32_t want) {
    if (!c || c->device < 0 || !c->has_scene || !p || want < 1 || check_params(c, p) != CR_OK) return 1;
    uint32_t m = 1;
    return group_layers(c, p, want, &m);
}

int cr_render_layers(cr_ctx *c, const cr_camera *cam, const cr_render_params *p, uint32_t nlayers,
                     float *accum_rgb_out) {
    if (!c) return CR_E_INVALID;
    if (c->device < 0) return fail(c, CR_E_HIP, c->err.empty() ? "no device" : c->err);
    if (!accum_rgb_out || !p || nlayers < 1) return fail(c, CR_E_INVALID, "null output/params or no layers");
    cr_render_params q = *p;
    if (q.nranks == 0) q.nranks = 1;
    if (q.nranks != 1) return fail(c, CR_E_INVALID, "cr_render_layers: the whole frame (nranks 1)");
    int rc = check_params(c, &q);
    if (rc) return rc;
    HIPCHK(hipSetDevice(c->device));
    const size_t elems = (size_t)q.xres * q.yres * 3;
    if (elems != c->accum_elems) {
        if (c->d_accum) hipFree(c->d_accum);
        c->d_accum = nullptr;
        c->accum_elems = 0;
        if (hipMalloc(&c->d_accum, elems * sizeof(float)) != hipSuccess) return fail(c, CR_E_OOM, "accumulator");
        c->accum_elems = elems;
        HIPCHK(hipMemset(c->d_accum, 0, elems * sizeof(float)));
    }
    PassTotals sum;
    for (uint32_t done = 0; done < nlayers;) {
        uint32_t m = 1;
        const uint32_t nl = group_layers(c, &q, std::min(LAYER_GROUP, nlayers - done), &m);
        for (uint32_t k = 0; k < m; k++) {
            cr_render_params t = q;
            t.layer = q.layer + done;
            t.rank = k;
            t.nranks = m;
            if ((rc = run_render(c, cam, &t, c->d_accum, cr::MODE_BLEND, c->stream, nl))) return rc;
            sum.add(c);
        }
        done += nl;
    }
    sum.store(c);
    HIPCHK(hipMemcpy(accum_rgb_out, c->d_accum, elems * sizeof(float), hipMemcpyDeviceToHost));
    return CR_OK;
}

int cr_set_accumulator(cr_ctx *c, uint32_t xres, uint32_t yres, const float *rgb) {
    if (!c) return CR_E_INVALID;
    if (c->device < 0) return fail(c, CR_E_HIP, c->err.empty() ? "no device" : c->err);
    if (!rgb || !xres || !yres) return fail(c, CR_E_INVALID, "null / empty accumulator");
    HIPCHK(hipSetDevice(c->device));
    const size_t elems = (size_t)xres * yres * 3;
    if (elems != c->accum_elems) {
        if (c->d_accum) hipFree(c->d_accum);
        c->d_accum = nullptr;
        c->accum_elems = 0;
        if (hipMalloc(&c->d_accum, elems * sizeof(float)) != hipSuccess) return fail(c, CR_E_OOM, "accumulator");
        c->accum_elems = elems;
    }
    HIPCHK(hipMemcpy(c->d_accum, rgb, elems * sizeof(float), hipMemcpyHostToDevice));
    return CR_OK;
}

int cr_render_device(cr_ctx *c, const cr_camera *cam, const cr_render_params *p, float *d_frame, void *stream) {
    if (!c) return CR_E_INVALID;
    if (c->device < 0) return fail(c, CR_E_HIP, c->err.empty() ? "no device" : c->err);
    return run_render(c, cam, p, d_frame, cr::MODE_BLEND, (hipStream_t)stream);
}

int cr_render_tiles_device(cr_ctx *c, const cr_camera *cam, const cr_render_params *p, float *d_tiles,
                           void *stream) {
    if (!c) return CR_E_INVALID;
    if (c->device < 0) return fail(c, CR_E_HIP, c->err.empty() ? "no device" : c->err);
    return run_render(c, cam, p, d_tiles, cr::MODE_TILES, (hipStream_t)stream);
}

uint32_t cr_layers_per_pass(cr_ctx *c, const cr_render_params *p, uint32_t want) {
    if (!c || c->device < 0 || !c->has_scene || !p || want < 1 || check_params(c, p) != CR_OK) return 1;
    if (c->kernel != 2 || c->wf_lanes != 1 || c->full_counters) return 1;
    if (hipSetDevice(c->device) != hipSuccess) return 1;
    const uint64_t items = (uint64_t)cr_tiles_for_rank(p, p->rank) * tile_of(p) * tile_of(p);
    const uint64_t paths_cap = std::min<uint64_t>(c->wf_paths, wf_path_cap(c, p->k));
    uint32_t nl = want;
    // one chunk of paths, one sample buffer, a 31-bit work index
    while (nl > 1 && (items * p->spp * nl > paths_cap || items * 12u * p->spp * nl > c->sample_buf ||
                      items * p->spp * nl >= (1ull << 31)))
        nl--;
    return nl;
}

int cr_render_layers_device(cr_ctx *c, const cr_camera *cam, const cr_render_params *p, uint32_t nlayers,
                            float *d_frame, void *stream) {
    if (!c) return CR_E_INVALID;
    if (c->device < 0) return fail(c, CR_E_HIP, c->err.empty() ? "no device" : c->err);
    return run_render(c, cam, p, d_frame, cr::MODE_BLEND, (hipStream_t)stream, nlayers);
}

int cr_render_tiles_layers_device(cr_ctx *c, const cr_camera *cam, const cr_render_params *p, uint32_t nlayers,
                                  float *d_tiles, void *stream) {
    if (!c) return CR_E_INVALID;
    if (c->device < 0) return fail(c, CR_E_HIP, c->err.empty() ? "no device" : c->err);
    if (!p || p->nranks <= 1 || nlayers <= 1 || cr_layers_per_pass(c, p, nlayers) == nlayers)
        return run_render(c, cam, p, d_tiles, cr::MODE_TILES, (hipStream_t)stream, nlayers);
    // the rank's tiles in pieces (ranks r + kN of an N * m split: every tile slot keeps its pixels
    // for any split of more than one rank), each written into the rank's compact buffer
    uint32_t m = 1;
    if (group_layers(c, p, nlayers, &m) != nlayers)
        return fail(c, CR_E_INVALID, "layers per pass: the rank's share does not fit in pieces");
    const uint64_t stride = (uint64_t)cr_tiles_for_rank(p, 0) * tile_of(p) * tile_of(p) * 3;
    PassTotals sum;
    for (uint32_t k = 0; k < m; k++) {
        cr_render_params t = *p;
        t.rank = p->rank + k * p->nranks;
        t.nranks = p->nranks * m;
        if (cr_tiles_for_rank(&t, t.rank) == 0) continue;
        if (int rc = run_render(c, cam, &t, d_tiles, cr::MODE_TILES, (hipStream_t)stream, nlayers, k, m, stride))
            return rc;
        sum.add(c);
    }
    sum.store(c);
    return CR_OK;
}

int cr_blend_tiles_device(cr_ctx *c, const cr_render_params *p, const float *d_gathered, float *d_frame,
                          void *stream) {
    return cr_blend_tiles_layers_device(c, p, 1, d_gathered, d_frame, stream);
}

int cr_blend_tiles_layers_device(cr_ctx *c, const cr_render_params *p, uint32_t nlayers, const float *d_gathered,
                                 float *d_frame, void *stream) {
    if (!c) return CR_E_INVALID;
    if (c->device < 0) return fail(c, CR_E_HIP, c->err.empty() ? "no device" : c->err);
    if (!p || !d_gathered || !d_frame || p->nranks < 1 || p->layer < 1 || nlayers < 1)
        return fail(c, CR_E_INVALID, "bad blend args");
    HIPCHK(hipSetDevice(c->device));
    cr::BlendArgs B{};
    B.gathered = d_gathered;
    B.frame = d_frame;
    B.xres = p->xres;
    B.yres = p->yres;
    B.tile = tile_of(p);
    B.tiles_x = (p->xres + B.tile - 1) / B.tile;
    B.nranks = p->nranks;
    B.max_tiles = cr_tiles_for_rank(p, 0);
    B.layer = p->layer;
    B.nl = nlayers;
    int e = cr::launch_blend(B, (hipStream_t)stream);
    if (e) return hip_fail(c, (hipError_t)e, "blend kernel launch");
    return CR_OK;
}

// rayTracer.cpp:172-205: host scalars of normalizeImage, glibc powf / logf as the reference
static inline float tm_knee(double x, double f) { return logf(x * f + 1) / f; }
static float tm_find_knee_f(float x, float y) {
    float f0 = 0, f1 = 1;
    while (tm_knee(x, f1) > y) {
        f0 = f1;
        f1 = f1 * 2;
    }
    for (int i = 0; i < 30; ++i) {
        const float f2 = (f0 + f1) / 2;
        if (tm_knee(x, f2) < y) f1 = f2;
        else f0 = f2;
    }
    return (f0 + f1) / 2;
}

void cr_tonemap_setup(float exposure, float defog, float kneeLow, float kneeHigh, float gamma, cr_tonemap_params *t) {
    if (!t) return;
    t->m = powf(2.f, exposure + 2.47393f);
    t->s = 255.f * powf(2.f, -3.5f * gamma);
    t->kl = powf(2.f, kneeLow);
    t->f = tm_find_knee_f(powf(2.f, kneeHigh), powf(2.f, 3.5) - t->kl);
    t->defog = defog;
    t->gamma = gamma;
}

int cr_tonemap_device(cr_ctx *c, const cr_tonemap_params *t, uint32_t xres, uint32_t yres, const float *d_rgb,
                      uint8_t *d_bytes, void *stream) {
    if (!c) return CR_E_INVALID;
    if (c->device < 0) return fail(c, CR_E_HIP, c->err.empty() ? "no device" : c->err);
    if (!t || !d_rgb || !d_bytes) return fail(c, CR_E_INVALID, "bad tonemap args");
    if ((uint64_t)xres * yres > (1ull << 31)) return fail(c, CR_E_INVALID, "image too large");
    HIPCHK(hipSetDevice(c->device));
    const cr::TonemapArgs T{d_rgb, d_bytes, xres, yres, t->m, t->s, t->kl, t->f, t->defog, t->gamma};
    const int e = cr::launch_tonemap(T, (hipStream_t)stream);
    if (e) return hip_fail(c, (hipError_t)e, "tonemap kernel launch");
    return CR_OK;
}

int cr_tonemap(cr_ctx *c, const cr_tonemap_params *t, uint32_t xres, uint32_t yres, uint8_t *bytes_out) {
    if (!c) return CR_E_INVALID;
    if (c->device < 0) return fail(c, CR_E_HIP, c->err.empty() ? "no device" : c->err);
    if (!bytes_out) return fail(c, CR_E_INVALID, "null output");
    const size_t n = (size_t)3 * xres * yres;
    if (!c->d_accum || c->accum_elems != n) return fail(c, CR_E_INVALID, "no rendered frame of this size");
    HIPCHK(hipSetDevice(c->device));
    void *d_bytes = nullptr;
    if (hipMalloc(&d_bytes, n ? n : 1) != hipSuccess) return fail(c, CR_E_OOM, "tonemap buffer");
    int rc = cr_tonemap_device(c, t, xres, yres, c->d_accum, (uint8_t *)d_bytes, c->stream);
    if (rc == CR_OK) {
        const hipError_t e = hipMemcpyAsync(bytes_out, d_bytes, n, hipMemcpyDeviceToHost, c->stream);
        const hipError_t e2 = e == hipSuccess ? hipStreamSynchronize(c->stream) : e;
        if (e2 != hipSuccess) rc = hip_fail(c, e2, "tonemap copy");
    }
    hipFree(d_bytes);
    return rc;
}

static int run_query(cr_ctx *c, uint32_t n, bool shadow, const float *orig, const float *dir, const float *dist,
                     const uint32_t *light, uint32_t *hit, uint32_t *tri, float *bary, float *dist_out) {
    if (!c) return CR_E_INVALID;
    if (c->device < 0) return fail(c, CR_E_HIP, c->err.empty() ? "no device" : c->err);
    if (!c->has_scene) return fail(c, CR_E_NOSCENE, "no scene uploaded");
    if (n == 0) return CR_OK;
    if (!orig || !dir || !hit) return fail(c, CR_E_INVALID, "null query arrays");
    if (shadow && (!dist || !light)) return fail(c, CR_E_INVALID, "null shadow distance / light arrays");
    HIPCHK(hipSetDevice(c->device));
    char *buf = nullptr;
    const size_t fbytes = (size_t)n * 3 * sizeof(float);
    const size_t total = 2 * fbytes + 4 * (size_t)n * sizeof(uint32_t) + 3 * (size_t)n * sizeof(float) + 256;
    if (hipMalloc(&buf, total) != hipSuccess) return fail(c, CR_E_OOM, "query buffers");
    char *p = buf;
    auto take = [&](size_t b) { char *r = p; p += (b + 15) & ~(size_t)15; return r; };
    cr::QueryArgs Q{};
    Q.S = c->S;
    Q.n = n;
    Q.shadow = shadow ? 1u : 0u;
    Q.stack_depth = c->stack_depth;
    float *d_orig = (float *)take(fbytes), *d_dir = (float *)take(fbytes);
    const size_t nb = (size_t)n * 4u; // bytes of one float / uint32 per query
    float *d_dist = (float *)take(nb);
    uint32_t *d_light = (uint32_t *)take(nb);
    uint32_t *d_hit = (uint32_t *)take(nb), *d_tri = (uint32_t *)take(nb);
    float *d_bary = (float *)take(2 * nb), *d_do = (float *)take(nb);
    hipError_t e = hipMemcpy(d_orig, orig, fbytes, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(d_dir, dir, fbytes, hipMemcpyHostToDevice);
    if (e == hipSuccess && shadow) e = hipMemcpy(d_dist, dist, n * sizeof(float), hipMemcpyHostToDevice);
    if (e == hipSuccess && shadow) e = hipMemcpy(d_light, light, n * sizeof(uint32_t), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemset(c->d_counters, 0, cr::CTR_SLOTS * sizeof(unsigned long long));
    Q.orig = d_orig; Q.dir = d_dir; Q.dist = d_dist; Q.light = d_light;
    Q.hit = d_hit; Q.tri = d_tri; Q.bary = d_bary; Q.dist_out = d_do;
    Q.counters = c->d_counters;
    if (e == hipSuccess) e = (hipError_t)cr::launch_intersect(Q, nullptr);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(hit, d_hit, n * sizeof(uint32_t), hipMemcpyDeviceToHost);
    if (e == hipSuccess && !shadow && tri) e = hipMemcpy(tri, d_tri, n * sizeof(uint32_t), hipMemcpyDeviceToHost);
    if (e == hipSuccess && !shadow && bary) e = hipMemcpy(bary, d_bary, 2 * n * sizeof(float), hipMemcpyDeviceToHost);
    if (e == hipSuccess && !shadow && dist_out) e = hipMemcpy(dist_out, d_do, n * sizeof(float), hipMemcpyDeviceToHost);
    unsigned long long h[cr::CTR_SLOTS] = {};
    if (e == hipSuccess) e = hipMemcpy(h, c->d_counters, sizeof(h), hipMemcpyDeviceToHost);
    hipFree(buf);
    if (e != hipSuccess) return hip_fail(c, e, "intersect");
    c->last = cr_counters{h[0], h[1],  h[2],  h[3],  h[4],  h[5],  h[6],  h[7], h[8],
                          h[9], h[10], h[11], h[12], h[13], h[14], h[15], h[16],
                          h[17], h[18], h[19], h[20], h[21], h[cr::CTR_NEE]};
    return CR_OK;
}

int cr_intersect(cr_ctx *c, uint32_t n, const float *orig, const float *dir, uint32_t *hit, uint32_t *tri,
                 float *bary, float *dist) {
    return run_query(c, n, false, orig, dir, nullptr, nullptr, hit, tri, bary, dist);
}

int cr_intersect_shadow(cr_ctx *c, uint32_t n, const float *orig, const float *dir, const float *dist,
                        const uint32_t *light_tri, uint32_t *occluded) {
    if (c && n && (!dist || !light_tri)) return fail(c, CR_E_INVALID, "null dist/light");
    return run_query(c, n, true, orig, dir, dist, light_tri, occluded, nullptr, nullptr, nullptr);
}

int cr_get_counters(cr_ctx *c, cr_counters *out) {
    if (!c || !out) return CR_E_INVALID;
    *out = c->last;
    return CR_OK;
}

float cr_last_kernel_ms(cr_ctx *c) { return c ? c->last_ms : 0.f; }

int cr_get_trace_stats(cr_ctx *c, cr_trace_stats *out) {
    if (!c || !out) return CR_E_INVALID;
    *out = c->last_trace;
    return CR_OK;
}

int cr_trace_build_available(int build) { return cr::wf_variant_available(build) ? 1 : 0; }
int cr_last_trace_build(cr_ctx *c) { return c ? c->last_build : -2; }

int cr_get_diag(cr_ctx *c, uint64_t *out, int n) {
    if (!c || !out || n < 0) return CR_E_INVALID;
    for (int i = 0; i < n && i < cr::DIAG_N; i++) out[i] = c->last_diag[i];
    return CR_OK;
}

int cr_get_perf(cr_ctx *c, uint64_t *out, int n) {
    if (!c || !out || n < 0) return CR_E_INVALID;
    for (int i = 0; i < n && i < cr::TK_N * cr::PERF_N; i++) out[i] = c->last_perf[i];
    return CR_OK;
}

int cr_set_option(cr_ctx *c, const char *key, int64_t v) {
    if (!c || !key) return CR_E_INVALID;
    const int64_t nvar = cr::num_wf_variants();
    // (the megakernel (0) and the thread-per-pixel kernel (1) were measured slower and removed: DESIGN.md §3)
    if (!std::strcmp(key, "kernel") && v == 2) c->kernel = (int)v;
    else if (!std::strcmp(key, "counters") && (v == 0 || v == 1)) c->full_counters = (int)v;
    else if (!std::strcmp(key, "perf_counters") && (v == 0 || v == 1)) c->perf_counters = (int)v;
    else if (!std::strcmp(key, "wf_tail_overlap") && (v == 0 || v == 1)) c->wf_tail_overlap = (int)v;
    else if (!std::strcmp(key, "wf_sort_g1") && v >= 0 && v <= 3) c->wf_sort_g1 = (uint32_t)v;
    else if (!std::strcmp(key, "wf_cam_lean") && (v == 0 || v == 1)) c->wf_cam_lean = (int)v;
    else if (!std::strcmp(key, "wf_cam_fuse") && (v == 0 || v == 1)) c->wf_cam_fuse = (int)v;
    else if (!std::strcmp(key, "wf_ctl_ray") && (v == 0 || v == 1)) c->wf_ctl_ray = (int)v;
    else if (!std::strcmp(key, "wf_vis_dw") && (v == 0 || v == 1)) c->wf_vis_dw = (int)v;
    else if (!std::strcmp(key, "wf_vis_mark") && (v == 0 || v == 1)) c->wf_vis_mark = (int)v;
    else if (!std::strcmp(key, "sum_lds") && v >= 0 && v <= 65536) c->sum_lds = (uint32_t)v;
    else if (!std::strcmp(key, "wf_nee_skip") && (v == 0 || v == 1)) c->wf_nee_skip = (int)v;
    else if (!std::strcmp(key, "sum_staged") && (v == 0 || v == 1)) c->sum_staged = (int)v;
    else if (!std::strcmp(key, "wf_tail_waves") && v >= 4 && v <= 6) c->wf_tail_waves = (int)v;
    else if (!std::strcmp(key, "wf_side_priority") && (v == 0 || v == 1)) {
        // the second stream (closest trace g + 1 beside shadow trace g) at the device's highest
        // stream priority (1) or the default (0): which persistent grid takes the CUs first
        int lo = 0, hi = 0;
        if (hipSetDevice(c->device) != hipSuccess || hipDeviceSynchronize() != hipSuccess ||
            hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess)
            return CR_E_HIP;
        hipStream_t s = nullptr;
        if (hipStreamCreateWithPriority(&s, hipStreamNonBlocking, v ? hi : lo) != hipSuccess) return CR_E_HIP;
        hipStreamDestroy(c->wfs.side);
        c->wfs.side = s;
    }
    else if (!std::strcmp(key, "diag_kinds") && v >= 0 && v <= 7) c->diag_kinds = (uint32_t)v;
    else if (!std::strcmp(key, "lc_debug") && v >= 0 && v <= 2) c->lc_debug = (int)v;
    else if (!std::strcmp(key, "lc_min") && v >= 0 && v <= 33) c->lc_min = (uint32_t)v;
    else if (!std::strcmp(key, "desc_quorum") && v >= -1 && v <= 64) c->desc_quorum = (int)v;
    else if (!std::strcmp(key, "comm_timeout_ms") && v >= 1 && v <= 3600000) c->comm_timeout_ms = (uint32_t)v;
    else if (!std::strcmp(key, "variant") && v >= -1 && v < nvar) c->variant = (int)v; // -1 default; clamped per kernel
    else if (!std::strcmp(key, "refill") && v >= 0 && v <= 64) c->refill = (uint32_t)v; // 0: per-kernel default
    else if (!std::strcmp(key, "refill_shadow") && v >= 0 && v <= 64) c->refill_shadow = (uint32_t)v;
    else if (!std::strcmp(key, "refill_camera") && v >= 0 && v <= 64) c->refill_camera = (uint32_t)v;
    else if (!std::strcmp(key, "wf_sort") && v >= -1 && v <= 1) c->wf_sort = (int)v;
    else if (!std::strcmp(key, "wf_world_keys") && v >= 0 && v <= 64) c->wf_world_keys = (int)v;
    else if (!std::strcmp(key, "wf_world_bits") && v >= 1 && v <= 10) c->wf_world_bits = (uint32_t)v;
    else if (!std::strcmp(key, "wf_sort_min") && v >= 0 && v <= (1ll << 31)) c->wf_sort_min = (uint32_t)v;
    else if (!std::strcmp(key, "wf_tail_min") && v >= 0 && v <= 0xffffffffll) c->wf_tail_min = (uint32_t)v;
    else if (!std::strcmp(key, "wf_sort_tile") && v >= 0 && v <= 5) c->wf_sort_tile = (uint32_t)v;
    else if (!std::strcmp(key, "wf_dir_res") && v >= 1 && v <= 256 && (v & (v - 1)) == 0)
        c->wf_dir_res = (uint32_t)v;
    else if (!std::strcmp(key, "wf_dir_res_shadow") && v >= 0 && v <= 256 && (v & (v - 1)) == 0)
        c->wf_dir_res_shadow = (uint32_t)v;
    else if (!std::strcmp(key, "wf_paths") && v >= 4096 && v <= (1ll << 30)) c->wf_paths = (uint32_t)v;
    else if (!std::strcmp(key, "wf_lanes") && (v == 1 || v == 2)) c->wf_lanes = (int)v;
    else if (!std::strcmp(key, "wf_xcd") && v >= 0 && v <= 7) c->wf_xcd = (uint32_t)v;
    else if (!std::strcmp(key, "wf_leaf_keys") && (v == 0 || v == 1)) c->wf_leaf_keys = (int)v;
    else if (!std::strcmp(key, "wf_resolve_paths") && v >= 0 && v <= 64) c->wf_resolve_paths = (uint32_t)v;
    else if (!std::strcmp(key, "wf_measure_skip") && v >= 0 && v <= 3) c->wf_measure_skip = (uint32_t)v;
    else if (!std::strcmp(key, "wf_shade_waves") && (v == 6 || v == 8)) c->wf_shade_waves = (int)v;
    else if (!std::strcmp(key, "wf_shade_block") && (v == 256 || v == 512 || v == 1024)) c->wf_shade_block = (int)v;
    else if (!std::strcmp(key, "wf_app_chunk") && (v == 0 || (v >= 256 && v <= 65536 && !(v & (v - 1))))) c->wf_app_chunk = (int)v;
    else if (!std::strcmp(key, "wf_leaf_shift") && v >= 0 && v <= 24) c->wf_leaf_shift = (uint32_t)v;
    else if (!std::strcmp(key, "node_bfs") && v >= 1 && v <= (1ll << 30)) c->node_bfs = (uint32_t)v;
    else if (!std::strcmp(key, "sample_buf_bytes") && v >= 1 && v <= (1ll << 40)) c->sample_buf = (uint64_t)v;
    else return fail(c, CR_E_INVALID, std::string("unknown option or value: ") + key);
    return CR_OK;
}

int cr_synchronize(cr_ctx *c) {
    if (!c) return CR_E_INVALID;
    if (c->device < 0) return fail(c, CR_E_HIP, "no device");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipDeviceSynchronize());
    return CR_OK;
}

} // extern "C"
