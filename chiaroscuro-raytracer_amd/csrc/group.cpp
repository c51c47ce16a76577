// group.cpp -- the multi-GPU frame split at the C-ABI, RCCL inside.
//
// The frame is cut into tile x tile tiles, tile t belongs to rank t % nranks;
// every rank renders the batch means of its tiles into a compact buffer
// [tiles][T][T][3], the root gathers the buffers over RCCL (xGMI between the
// GPUs of a node) and unpermutes + blends the layer into its frame on the
// device: frame = (frame * (L - 1) + mean) / L (src/rayTracer.cpp:64).  The
// RNG key holds the global pixel index, so the image does not depend on the
// number of ranks (tests/test_gpu_parity.py tile tests, tests/test_gpu_group.py).
//
// Two shapes of the same protocol:
//   cr_comm_* / cr_render_dist_device  one process per GPU (the MI355X layout:
//       bench.py under torch.distributed.run); a ncclComm per process from a
//       unique id the caller distributes; grouped ncclSend / ncclRecv to rank 0
//   cr_group_*  one host process driving N GPUs (the reference's callers --
//       main.cpp:16, src/openglPreview.cpp:247 -- are single-process): a
//       cr_ctx per GPU, the passes on one host thread per GPU (a pass waits on
//       its queue lengths), ncclCommInitAll and the grouped send / receive from
//       one thread.  A device listed twice cannot join a RCCL communicator; such
//       a group gathers with device-to-device copies instead (the one-GPU tests
//       of the N-rank protocol use that).
// After every gather the host polls ncclCommGetAsyncError while it waits, so a
// failed peer surfaces as CR_E_COMM instead of a hang.
#include "ctx.hpp"

#include <algorithm>
#include <chrono>
#include <cstring>
#include <thread>

namespace crx {

static int nccl_fail(cr_ctx *c, ncclResult_t r, const char *what) {
    return fail(c, CR_E_COMM, std::string(what) + ": " + ncclGetErrorString(r));
}

void release_dist(cr_ctx *c) {
    if (c->comm) ncclCommDestroy(c->comm);
    c->comm = nullptr;
    c->comm_rank = 0;
    c->comm_nranks = 1;
    if (c->d_tiles) hipFree(c->d_tiles);
    if (c->d_gathered) hipFree(c->d_gathered);
    if (c->d_flag) hipFree(c->d_flag);
    c->d_tiles = c->d_gathered = nullptr;
    c->d_flag = nullptr;
    c->tiles_bytes = c->gathered_bytes = c->flag_bytes = 0;
}

// A non-blocking communicator's state once its pending work is enqueued (or failed).
static ncclResult_t nccl_settle(ncclComm_t comm) {
    ncclResult_t st = ncclInProgress;
    while (ncclCommGetAsyncError(comm, &st) == ncclSuccess && st == ncclInProgress)
        std::this_thread::sleep_for(std::chrono::microseconds(20));
    return st;
}

// Wait for the stream's work while watching the communicator's asynchronous error.
static int wait_comm(cr_ctx *c, ncclComm_t comm, hipStream_t st, const char *what) {
    for (;;) {
        const hipError_t q = hipStreamQuery(st);
        if (q == hipSuccess) break;
        if (q != hipErrorNotReady) return hip_fail(c, q, what);
        ncclResult_t ae = ncclSuccess;
        if (comm && ncclCommGetAsyncError(comm, &ae) == ncclSuccess && ae != ncclSuccess && ae != ncclInProgress) {
            ncclCommAbort(comm);
            if (c->comm == comm) c->comm = nullptr;
            return nccl_fail(c, ae, what);
        }
        std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
    ncclResult_t ae = ncclSuccess;
    if (comm && ncclCommGetAsyncError(comm, &ae) == ncclSuccess && ae != ncclSuccess) return nccl_fail(c, ae, what);
    return CR_OK;
}

// Every rank's verdict on a pass group before anything of it is rendered or exchanged: an all-reduce MIN
// of `ok` over the communicator.  A rank whose share cannot hold the group (a plan that differs between
// the ranks, a buffer that cannot grow) then makes EVERY rank fail here with the same error, instead of
// returning before the grouped send / receive and leaving its peers blocked in it until comm_timeout_ms.
static int agree(cr_ctx *c, bool ok, hipStream_t st, const char *what) {
    // (d_flag exists since cr_comm_init: nothing that can fail on one rank alone precedes the all-reduce)
    HIPCHK(hipMemsetD32Async((hipDeviceptr_t)c->d_flag, ok ? 1 : 0, 1, st));
    ncclResult_t r = ncclAllReduce(c->d_flag, c->d_flag, 1, ncclInt32, ncclMin, c->comm, st);
    if (r == ncclInProgress) r = nccl_settle(c->comm);
    if (r != ncclSuccess) return nccl_fail(c, r, what);
    if (int rc = wait_comm(c, c->comm, st, what)) return rc;
    int all = 0;
    HIPCHK(hipMemcpy(&all, c->d_flag, sizeof(int), hipMemcpyDeviceToHost));
    if (all == 1) return CR_OK;
    return fail(c, CR_E_INVALID, std::string(what) + ": " +
                                     (ok ? "another rank cannot render this pass group (plan the group with "
                                           "cr_layers_per_group on every rank and agree on the minimum)"
                                         : c->err));
}

// Elements of one rank's compact tile buffer (the root's largest: rank 0 owns
// the most tiles), so every rank sends and the root receives the same count.
static size_t slot_elems(const cr_render_params *p) {
    const size_t T = tile_of(p);
    return (size_t)cr_tiles_for_rank(p, 0) * T * T * 3;
}

static cr::BlendArgs blend_args(const cr_render_params *p, const float *gathered, float *frame) {
    cr::BlendArgs B{};
    B.gathered = gathered;
    B.frame = frame;
    B.xres = p->xres;
    B.yres = p->yres;
    B.tile = tile_of(p);
    B.tiles_x = (p->xres + B.tile - 1) / B.tile;
    B.nranks = p->nranks;
    B.max_tiles = cr_tiles_for_rank(p, 0);
    B.layer = p->layer;
    B.nl = 1;
    return B;
}

// Layers q->layer .. + nlayers - 1 of the whole frame (nranks 1) blended into d_frame on st, in the
// pieces cr_layers_per_group plans (cr_render_layers' scheme on a device frame); counters summed.
static int frame_layers(cr_ctx *c, const cr_camera *cam, const cr_render_params *q, uint32_t nlayers, float *d_frame,
                        hipStream_t st) {
    cr_render_params f = *q;
    f.rank = 0;
    f.nranks = 1;
    uint32_t m = 1;
    if (nlayers > 1 && group_layers(c, &f, nlayers, &m) != nlayers)
        return fail(c, CR_E_INVALID, "layers per pass: the frame does not fit in pieces");
    PassTotals sum;
    for (uint32_t k = 0; k < m; k++) {
        cr_render_params t = f;
        t.rank = k;
        t.nranks = m;
        if (int rc = run_render(c, cam, &t, d_frame, cr::MODE_BLEND, st, nlayers)) return rc;
        sum.add(c);
    }
    sum.store(c);
    return CR_OK;
}

} // namespace crx

using namespace crx;

// ------------------------------------------------------ one process per GPU --
extern "C" {

int cr_comm_unique_id(uint8_t *out, size_t n) {
    if (!out || n < CR_COMM_ID_BYTES || sizeof(ncclUniqueId) > CR_COMM_ID_BYTES) return CR_E_INVALID;
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return CR_E_COMM;
    std::memset(out, 0, CR_COMM_ID_BYTES);
    std::memcpy(out, &id, sizeof(id));
    return CR_OK;
}

int cr_comm_init(cr_ctx *c, int nranks, int rank, const uint8_t *id) {
    if (!c) return CR_E_INVALID;
    if (c->device < 0) return fail(c, CR_E_HIP, c->err.empty() ? "no device" : c->err);
    if (nranks < 1 || rank < 0 || rank >= nranks || !id) return fail(c, CR_E_INVALID, "bad nranks/rank/id");
    HIPCHK(hipSetDevice(c->device));
    release_dist(c);
    // agree()'s flag word is allocated here, before any collective: a rank whose allocation fails then
    // fails before the communicator exists, never between its peers' entry into an all-reduce and its own
    if (int rr = grow(c, (void **)&c->d_flag, c->flag_bytes, sizeof(int))) return rr;
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof(uid));
    // non-blocking init, polled against a deadline: a rank whose peers never join (a dead
    // launcher, a wrong nranks, one GPU for two ranks) gets CR_E_COMM instead of a hang
    ncclComm_t comm = nullptr;
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    ncclResult_t r = ncclCommInitRankConfig(&comm, nranks, uid, rank, &cfg);
    if (r != ncclSuccess && r != ncclInProgress) {
        if (comm) ncclCommAbort(comm);
        return nccl_fail(c, r, "ncclCommInitRankConfig");
    }
    const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(c->comm_timeout_ms);
    for (;;) {
        ncclResult_t st = ncclInProgress;
        if ((r = ncclCommGetAsyncError(comm, &st)) != ncclSuccess || (st != ncclSuccess && st != ncclInProgress)) {
            ncclCommAbort(comm);
            return nccl_fail(c, r != ncclSuccess ? r : st, "ncclCommInitRankConfig");
        }
        if (st == ncclSuccess) break;
        if (std::chrono::steady_clock::now() > deadline) {
            ncclCommAbort(comm);
            return fail(c, CR_E_COMM, "cr_comm_init: the " + std::to_string(nranks) +
                                          "-rank communicator did not form within " +
                                          std::to_string(c->comm_timeout_ms) + " ms (peers missing)");
        }
        std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
    c->comm = comm;
    c->comm_rank = rank;
    c->comm_nranks = nranks;
    return CR_OK;
}

int cr_comm_destroy(cr_ctx *c) {
    if (!c) return CR_E_INVALID;
    if (c->device >= 0) {
        HIPCHK(hipSetDevice(c->device));
        release_dist(c);
    }
    return CR_OK;
}

int cr_render_dist_device(cr_ctx *c, const cr_camera *cam, const cr_render_params *p, float *d_frame, void *stream) {
    if (!c) return CR_E_INVALID;
    if (c->device < 0) return fail(c, CR_E_HIP, c->err.empty() ? "no device" : c->err);
    if (!p || !cam) return fail(c, CR_E_INVALID, "null camera/params");
    if (!c->comm) return fail(c, CR_E_INVALID, "no communicator (cr_comm_init)");
    cr_render_params q = *p;
    q.rank = (uint32_t)c->comm_rank;
    q.nranks = (uint32_t)c->comm_nranks;
    const bool root = c->comm_rank == 0;
    if (root && !d_frame) return fail(c, CR_E_INVALID, "root needs a frame");
    if (int rc = check_params(c, &q)) return rc;
    HIPCHK(hipSetDevice(c->device));
    hipStream_t st = (hipStream_t)stream;
    if (q.nranks == 1) return run_render(c, cam, &q, d_frame, cr::MODE_BLEND, st);
    const size_t slot = slot_elems(&q);
    float *mine;
    if (root) {
        if (int r = grow(c, (void **)&c->d_gathered, c->gathered_bytes, slot * q.nranks * sizeof(float))) return r;
        mine = c->d_gathered; // the root's own tiles land in slot 0
    } else {
        if (int r = grow(c, (void **)&c->d_tiles, c->tiles_bytes, slot * sizeof(float))) return r;
        mine = c->d_tiles;
    }
    if (int rc = run_render(c, cam, &q, mine, cr::MODE_TILES, st)) return rc;
    ncclResult_t r = ncclGroupStart();
    if (r == ncclSuccess) {
        // (a non-blocking communicator may answer ncclInProgress: queued, not failed)
        if (root) {
            for (uint32_t k = 1; k < q.nranks && (r == ncclSuccess || r == ncclInProgress); k++)
                r = ncclRecv(c->d_gathered + k * slot, slot, ncclFloat32, (int)k, c->comm, st);
        } else {
            r = ncclSend(mine, slot, ncclFloat32, 0, c->comm, st);
        }
        if (r == ncclInProgress) r = ncclSuccess;
        ncclResult_t e = ncclGroupEnd();
        if (e == ncclInProgress) e = nccl_settle(c->comm); // non-blocking: enqueued before the blend
        if (r == ncclSuccess) r = e;
    }
    if (r != ncclSuccess) return nccl_fail(c, r, "tile gather");
    if (root) {
        const int e = cr::launch_blend(blend_args(&q, c->d_gathered, d_frame), st);
        if (e) return hip_fail(c, (hipError_t)e, "blend kernel launch");
    }
    return wait_comm(c, c->comm, st, "tile gather");
}

int cr_render_dist_layers_device(cr_ctx *c, const cr_camera *cam, const cr_render_params *p, uint32_t nlayers,
                                 float *d_frame, void *stream) {
    if (!c) return CR_E_INVALID;
    if (c->device < 0) return fail(c, CR_E_HIP, c->err.empty() ? "no device" : c->err);
    if (!p || !cam || nlayers < 1) return fail(c, CR_E_INVALID, "null camera/params or no layers");
    if (!c->comm) return fail(c, CR_E_INVALID, "no communicator (cr_comm_init)");
    if (nlayers == 1) return cr_render_dist_device(c, cam, p, d_frame, stream);
    cr_render_params q = *p;
    q.rank = (uint32_t)c->comm_rank;
    q.nranks = (uint32_t)c->comm_nranks;
    const bool root = c->comm_rank == 0;
    if (root && !d_frame) return fail(c, CR_E_INVALID, "root needs a frame");
    if (int rc = check_params(c, &q)) return rc;
    HIPCHK(hipSetDevice(c->device));
    hipStream_t st = (hipStream_t)stream;
    if (q.nranks == 1) return frame_layers(c, cam, &q, nlayers, d_frame, st);
    // every rank's nlayers compact buffers in one piece: [nlayers][slot], the root's in its slot 0 of
    // [nranks][nlayers][slot]; ONE grouped send / receive of the whole group, one blend of its layers
    const size_t slot = slot_elems(&q), span = slot * nlayers;
    // this rank's checks first, then every rank's verdict (agree): the group is rendered and exchanged
    // only when the plan holds on all of them
    uint32_t m = 1;
    bool ok = group_layers(c, &q, nlayers, &m) == nlayers;
    if (!ok) fail(c, CR_E_INVALID, "layers per pass: the rank's share does not fit " + std::to_string(nlayers) +
                                      " layers in pieces");
    float *mine = nullptr;
    if (ok) {
        const int r = root ? grow(c, (void **)&c->d_gathered, c->gathered_bytes, span * q.nranks * sizeof(float))
                           : grow(c, (void **)&c->d_tiles, c->tiles_bytes, span * sizeof(float));
        ok = r == CR_OK;
        mine = root ? c->d_gathered : c->d_tiles;
    }
    if (int rc = agree(c, ok, st, "pass group plan")) return rc;
    if (int rc = cr_render_tiles_layers_device(c, cam, &q, nlayers, mine, st)) return rc;
    ncclResult_t r = ncclGroupStart();
    if (r == ncclSuccess) {
        if (root) {
            for (uint32_t k = 1; k < q.nranks && (r == ncclSuccess || r == ncclInProgress); k++)
                r = ncclRecv(c->d_gathered + k * span, span, ncclFloat32, (int)k, c->comm, st);
        } else {
            r = ncclSend(mine, span, ncclFloat32, 0, c->comm, st);
        }
        if (r == ncclInProgress) r = ncclSuccess;
        ncclResult_t e = ncclGroupEnd();
        if (e == ncclInProgress) e = nccl_settle(c->comm);
        if (r == ncclSuccess) r = e;
    }
    if (r != ncclSuccess) return nccl_fail(c, r, "tile gather");
    if (root) {
        cr::BlendArgs B = blend_args(&q, c->d_gathered, d_frame);
        B.nl = nlayers;
        if (const int e = cr::launch_blend(B, st)) return hip_fail(c, (hipError_t)e, "blend kernel launch");
    }
    return wait_comm(c, c->comm, st, "tile gather");
}

} // extern "C"

// ---------------------------------------------------- one process, N GPUs --
struct cr_group {
    std::vector<int> devices;
    std::vector<cr_ctx *> ctx;
    std::vector<ncclComm_t> comm; // empty: gather by device copies (a device listed twice)
    std::vector<float *> tiles;   // rank r >= 1: compact buffer on device r
    std::vector<size_t> tiles_bytes;
    float *gathered = nullptr;    // root device: [nranks][slot]
    size_t gathered_bytes = 0;
    float *frame = nullptr;       // root device: the progressive accumulator [yres][xres][3]
    size_t frame_elems = 0;
    std::string err;
    cr_counters last{};
    std::vector<float> rank_ms;
};

namespace {
int gfail(cr_group *g, int code, const std::string &msg) {
    g->err = msg;
    return code;
}
int gctx_fail(cr_group *g, size_t r, int code) {
    return gfail(g, code, "rank " + std::to_string(r) + " (device " + std::to_string(g->devices[r]) + "): " +
                              cr_last_error(g->ctx[r]));
}
// run f(r) for every rank on its own host thread; first failure wins
template <class F> int for_ranks(cr_group *g, F f) {
    const size_t n = g->ctx.size();
    std::vector<int> rc(n, CR_OK);
    std::vector<std::thread> th;
    for (size_t r = 1; r < n; r++) th.emplace_back([&, r] { rc[r] = f(r); });
    rc[0] = f(0);
    for (auto &t : th) t.join();
    for (size_t r = 0; r < n; r++)
        if (rc[r]) return gctx_fail(g, r, rc[r]);
    return CR_OK;
}
} // namespace

extern "C" {

int cr_device_count(void) {
    int n = 0;
    return hipGetDeviceCount(&n) == hipSuccess ? n : 0;
}

cr_group *cr_group_create(int ngpus, const int *devices) {
    cr_group *g = new cr_group();
    if (ngpus < 1 || ngpus > 64) {
        g->err = "ngpus must be in [1, 64]";
        return g;
    }
    for (int r = 0; r < ngpus; r++) g->devices.push_back(devices ? devices[r] : r);
    // per-rank buffers sized before any ctx exists: cr_group_destroy walks them for every
    // created ctx, also after a failed create
    g->tiles.assign(ngpus, nullptr);
    g->tiles_bytes.assign(ngpus, 0);
    g->rank_ms.assign(ngpus, 0.f);
    for (int r = 0; r < ngpus; r++) {
        g->ctx.push_back(cr_create(g->devices[r]));
        if (!g->ctx.back() || g->ctx.back()->device < 0) {
            g->err = "rank " + std::to_string(r) + " (device " + std::to_string(g->devices[r]) +
                     "): " + cr_last_error(g->ctx.back());
            return g;
        }
    }
    std::vector<int> sorted = g->devices;
    std::sort(sorted.begin(), sorted.end());
    if (std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end()) {
        g->comm.assign(ngpus, nullptr);
        const ncclResult_t r = ncclCommInitAll(g->comm.data(), ngpus, g->devices.data());
        if (r != ncclSuccess) {
            g->comm.clear();
            g->err = std::string("ncclCommInitAll: ") + ncclGetErrorString(r);
        }
    }
    return g;
}

void cr_group_destroy(cr_group *g) {
    if (!g) return;
    for (ncclComm_t c : g->comm)
        if (c) ncclCommDestroy(c);
    for (size_t r = 0; r < g->ctx.size(); r++) {
        if (!g->ctx[r]) continue;
        if (g->ctx[r]->device >= 0) {
            hipSetDevice(g->devices[r]);
            if (r < g->tiles.size() && g->tiles[r]) hipFree(g->tiles[r]);
            if (r == 0) {
                if (g->gathered) hipFree(g->gathered);
                if (g->frame) hipFree(g->frame);
            }
        }
        cr_destroy(g->ctx[r]);
    }
    delete g;
}

const char *cr_group_last_error(cr_group *g) { return g ? g->err.c_str() : "null group"; }
static bool group_ok(cr_group *g);

int cr_group_size(cr_group *g) { return g ? (int)g->ctx.size() : 0; }

int cr_group_ok(cr_group *g) { return g && group_ok(g) ? 1 : 0; }

// Usable: every ctx on a device, and a communicator unless a device repeats.
static bool group_ok(cr_group *g) {
    if (g->ctx.empty() || g->ctx.size() != g->devices.size()) return false;
    for (cr_ctx *c : g->ctx)
        if (!c || c->device < 0) return false;
    std::vector<int> sorted = g->devices;
    std::sort(sorted.begin(), sorted.end());
    const bool distinct = std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
    return !distinct || !g->comm.empty();
}

int cr_group_upload_scene(cr_group *g, const cr_scene_desc *d) {
    if (!g) return CR_E_INVALID;
    if (!group_ok(g)) return CR_E_HIP;
    return for_ranks(g, [&](size_t r) { return cr_upload_scene(g->ctx[r], d); });
}

int cr_group_set_option(cr_group *g, const char *key, int64_t value) {
    if (!g || g->ctx.empty()) return CR_E_INVALID;
    for (size_t r = 0; r < g->ctx.size(); r++)
        if (int rc = cr_set_option(g->ctx[r], key, value)) return gctx_fail(g, r, rc);
    return CR_OK;
}

// One pass group of the whole group: layers q->layer .. + nl - 1 (q->nranks = the group size), every
// rank its tiles of all nl layers (one pass, in pieces when they do not fit one chunk), the gather of
// the nl compact buffers per rank into the root's [nranks][nl][slot], one blend of the nl layers into
// the root's frame; counters and rank times added to sum / ms.
static int group_pass(cr_group *g, const cr_camera *cam, const cr_render_params *q, uint32_t nl, PassTotals *sum,
                      std::vector<float> &ms) {
    const uint32_t n = (uint32_t)g->ctx.size();
    hipStream_t st0 = g->ctx[0]->stream;
    if (n == 1) {
        if (hipSetDevice(g->devices[0]) != hipSuccess) return gfail(g, CR_E_HIP, "hipSetDevice");
        cr_render_params f = *q;
        if (int rc = nl == 1 ? run_render(g->ctx[0], cam, &f, g->frame, cr::MODE_BLEND, st0)
                             : frame_layers(g->ctx[0], cam, &f, nl, g->frame, st0))
            return gctx_fail(g, 0, rc);
        sum[0].add(g->ctx[0]);
        ms[0] += g->ctx[0]->last_ms;
        return CR_OK;
    }
    const size_t slot = slot_elems(q), span = slot * nl;
    if (hipSetDevice(g->devices[0]) != hipSuccess) return gfail(g, CR_E_HIP, "hipSetDevice");
    if (int rc = grow(g->ctx[0], (void **)&g->gathered, g->gathered_bytes, span * n * sizeof(float)))
        return gctx_fail(g, 0, rc);
    int rc = for_ranks(g, [&](size_t r) -> int {
        cr_ctx *c = g->ctx[r];
        if (hipSetDevice(g->devices[r]) != hipSuccess) return fail(c, CR_E_HIP, "hipSetDevice");
        float *mine = g->gathered;
        if (r > 0) {
            if (int e = grow(c, (void **)&g->tiles[r], g->tiles_bytes[r], span * sizeof(float))) return e;
            mine = g->tiles[r];
        }
        cr_render_params qr = *q;
        qr.rank = (uint32_t)r;
        const int e = nl == 1 ? run_render(c, cam, &qr, mine, cr::MODE_TILES, c->stream)
                              : cr_render_tiles_layers_device(c, cam, &qr, nl, mine, c->stream);
        if (!e) {
            sum[r].add(c);
            ms[r] += c->last_ms;
        }
        return e;
    });
    if (rc) return rc;
    if (g->comm.empty()) { // a device listed twice: device-to-device copies into the root's slots
        for (uint32_t r = 1; r < n; r++)
            if (hipMemcpyPeerAsync(g->gathered + r * span, g->devices[0], g->tiles[r], g->devices[r],
                                   span * sizeof(float), st0) != hipSuccess)
                return gfail(g, CR_E_HIP, "tile copy");
    } else {
        ncclResult_t r = ncclGroupStart();
        for (uint32_t k = 1; k < n && r == ncclSuccess; k++) {
            r = ncclSend(g->tiles[k], span, ncclFloat32, 0, g->comm[k], g->ctx[k]->stream);
            if (r == ncclSuccess) r = ncclRecv(g->gathered + k * span, span, ncclFloat32, (int)k, g->comm[0], st0);
        }
        const ncclResult_t e = ncclGroupEnd();
        if (r == ncclSuccess) r = e;
        if (r != ncclSuccess) return gfail(g, CR_E_COMM, std::string("tile gather: ") + ncclGetErrorString(r));
    }
    if (hipSetDevice(g->devices[0]) != hipSuccess) return gfail(g, CR_E_HIP, "hipSetDevice");
    cr::BlendArgs B = blend_args(q, g->gathered, g->frame);
    B.nl = nl;
    const int e = cr::launch_blend(B, st0);
    if (e) return gfail(g, CR_E_HIP, std::string("blend kernel launch: ") + hipGetErrorString((hipError_t)e));
    for (uint32_t k = 0; k < n; k++) {
        hipSetDevice(g->devices[k]);
        if (int w = wait_comm(g->ctx[k], g->comm.empty() ? nullptr : g->comm[k], g->ctx[k]->stream, "tile gather"))
            return gctx_fail(g, k, w);
    }
    hipSetDevice(g->devices[0]);
    return CR_OK;
}

// cr_group_render(_layers): layers p->layer .. + nlayers - 1, pass groups of up to `group` layers
static int group_render(cr_group *g, const cr_camera *cam, const cr_render_params *p, uint32_t nlayers,
                        uint32_t group, float *accum_rgb_out) {
    if (!g) return CR_E_INVALID;
    if (!group_ok(g)) return gfail(g, CR_E_HIP, g->err.empty() ? "group not initialised" : g->err);
    if (!cam || !p || !accum_rgb_out || nlayers < 1) return gfail(g, CR_E_INVALID, "null camera/params/output");
    const uint32_t n = (uint32_t)g->ctx.size();
    cr_render_params q = *p;
    q.rank = 0;
    q.nranks = n;
    if (int rc = check_params(g->ctx[0], &q)) return gctx_fail(g, 0, rc);
    const size_t elems = (size_t)q.xres * q.yres * 3;
    if (hipSetDevice(g->devices[0]) != hipSuccess) return gfail(g, CR_E_HIP, "hipSetDevice");
    if (elems != g->frame_elems) {
        if (g->frame) hipFree(g->frame);
        g->frame = nullptr;
        g->frame_elems = 0;
        if (hipMalloc(&g->frame, elems * sizeof(float)) != hipSuccess) return gfail(g, CR_E_OOM, "frame");
        g->frame_elems = elems;
        if (hipMemset(g->frame, 0, elems * sizeof(float)) != hipSuccess) return gfail(g, CR_E_HIP, "frame");
    }
    std::vector<PassTotals> sum(n);
    std::vector<float> ms(n, 0.f);
    for (uint32_t done = 0; done < nlayers;) {
        cr_render_params t = q;
        t.layer = q.layer + done;
        // the group's size: what every rank's share fits (each rank's tiles in up to 64 pieces)
        uint32_t nl = std::min(group, nlayers - done);
        for (uint32_t r = 0; r < n && nl > 1; r++) {
            cr_render_params tr = t;
            tr.rank = r;
            if (n == 1) tr.nranks = 1;
            uint32_t m = 1;
            nl = std::min(nl, group_layers(g->ctx[r], &tr, nl, &m));
        }
        if (int rc = group_pass(g, cam, &t, nl, sum.data(), ms)) return rc;
        done += nl;
    }
    if (hipMemcpy(accum_rgb_out, g->frame, elems * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess)
        return gfail(g, CR_E_HIP, "frame copy");
    // counters summed over ranks (and groups); each rank's pass time
    cr_counters tot{};
    uint64_t *s = (uint64_t *)&tot;
    for (uint32_t k = 0; k < n; k++) {
        for (size_t i = 0; i < sizeof(cr_counters) / sizeof(uint64_t); i++) s[i] += sum[k].ctr[i];
        g->rank_ms[k] = ms[k];
    }
    g->last = tot;
    return CR_OK;
}

int cr_group_render(cr_group *g, const cr_camera *cam, const cr_render_params *p, float *accum_rgb_out) {
    return group_render(g, cam, p, 1, 1, accum_rgb_out);
}

int cr_group_render_layers(cr_group *g, const cr_camera *cam, const cr_render_params *p, uint32_t nlayers,
                           float *accum_rgb_out) {
    return group_render(g, cam, p, nlayers, 32, accum_rgb_out);
}

int cr_group_set_accumulator(cr_group *g, uint32_t xres, uint32_t yres, const float *rgb) {
    if (!g) return CR_E_INVALID;
    if (!group_ok(g)) return gfail(g, CR_E_HIP, g->err.empty() ? "group not initialised" : g->err);
    if (!rgb || !xres || !yres) return gfail(g, CR_E_INVALID, "null / empty accumulator");
    const size_t elems = (size_t)xres * yres * 3;
    if (hipSetDevice(g->devices[0]) != hipSuccess) return gfail(g, CR_E_HIP, "hipSetDevice");
    if (elems != g->frame_elems) {
        if (g->frame) hipFree(g->frame);
        g->frame = nullptr;
        g->frame_elems = 0;
        if (hipMalloc(&g->frame, elems * sizeof(float)) != hipSuccess) return gfail(g, CR_E_OOM, "frame");
        g->frame_elems = elems;
    }
    if (hipMemcpy(g->frame, rgb, elems * sizeof(float), hipMemcpyHostToDevice) != hipSuccess)
        return gfail(g, CR_E_HIP, "frame copy");
    return CR_OK;
}

cr_ctx *cr_group_ctx(cr_group *g, int rank) {
    return g && rank >= 0 && rank < (int)g->ctx.size() ? g->ctx[rank] : nullptr;
}

int cr_group_tonemap(cr_group *g, const cr_tonemap_params *t, uint32_t xres, uint32_t yres, uint8_t *bytes_out) {
    if (!g || !t || !bytes_out) return CR_E_INVALID;
    const size_t n = (size_t)3 * xres * yres;
    if (!g->frame || g->frame_elems != n) return gfail(g, CR_E_INVALID, "no rendered frame of this size");
    if (hipSetDevice(g->devices[0]) != hipSuccess) return gfail(g, CR_E_HIP, "hipSetDevice");
    void *d_bytes = nullptr;
    if (hipMalloc(&d_bytes, n ? n : 1) != hipSuccess) return gfail(g, CR_E_OOM, "tonemap buffer");
    cr_ctx *c = g->ctx[0];
    int rc = cr_tonemap_device(c, t, xres, yres, g->frame, (uint8_t *)d_bytes, c->stream);
    if (rc == CR_OK && (hipMemcpyAsync(bytes_out, d_bytes, n, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
                        hipStreamSynchronize(c->stream) != hipSuccess))
        rc = fail(c, CR_E_HIP, "tonemap copy");
    hipFree(d_bytes);
    return rc ? gctx_fail(g, 0, rc) : CR_OK;
}

int cr_group_get_counters(cr_group *g, cr_counters *out) {
    if (!g || !out) return CR_E_INVALID;
    *out = g->last;
    return CR_OK;
}

int cr_group_rank_ms(cr_group *g, float *out) {
    if (!g || !out) return CR_E_INVALID;
    std::copy(g->rank_ms.begin(), g->rank_ms.end(), out);
    return CR_OK;
}

} // extern "C"
