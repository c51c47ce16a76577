// kernels.hip -- CDNA4 (gfx950) kernels around the render loop: the ray-query kernel behind
// cr_intersect / cr_intersect_shadow (KDTree::intersectRay / intersectShadowRay, one query per
// thread with the reference's recursion as an LDS stack), the root-side tile blend and the tonemap.
// The render loop itself is the wavefront path tracer (wavefront.hip), its sample sum samples.hip.
//
// Layout in HBM (built by cabi.cpp):
//   nodes  : uint2 per kd node {split bits | first ref, axis | child<<2 (axis 3 = leaf, count<<2)}
//   recs   : 3 x float4 per leaf reference, leaf-ordered: {A, id}, {B-A}, {C-A}
//   tri    : 3 x float4 per triangle {A, B, C} (hit reconstruction only)
//   mat    : float4 normal (w: emissive flag), float4 Kd (w: texture index), float4 Ke, 3 x float2 uv
//   lights : uint2 {triangle id, surface bits}
#include "render_common.hpp"

namespace cr {

// Full (node, tmin, tmax) stack in LDS, [depth][thread]: every lane's push/pop
// hits its own bank whatever its depth.
struct Stack {
    uint32_t *node;
    float *tmin;
    float *tmax;
    uint32_t stride; // = blockDim.x
};

// Unified kd traversal (recursion of the reference emulated with a stack).
//   closest (SHADOW=false): KDTree::intersectRay, src/kdtree.cpp:210-281 -- the
//     first leaf (near-to-far) holding an accepted hit ends the query.
//   shadow  (SHADOW=true):  KDTree::intersectShadowRay, src/kdtree.cpp:283-344 --
//     any accepted triangle other than `exclude` ends it.
template <bool SHADOW>
__device__ __forceinline__ bool traverse(const DevScene &S, const Stack &stk, f3 o, f3 d, float limit,
                                         uint32_t exclude, uint32_t &tri, float &bx, float &by, float &dist,
                                         Ctr &c) {
    float tmin, tmax;
    ray_box(S, o, d, tmin, tmax);
    if (SHADOW) {
        if (tmax < 0 || tmax < tmin || tmin > limit) return false;
        tmax = std_min(tmax, limit);
    } else {
        if (tmax < 0 || tmax < tmin) return false;
    }
    const uint32_t tid = threadIdx.x;
    uint32_t sp = 0;
    uint32_t node = 0;
    for (;;) {
        uint2 nd = S.nodes[node];
        while ((nd.y & 3u) != 3u) {
            c.inner++;
            const uint32_t a = nd.y & 3u;
            const float split = __uint_as_float(nd.x);
            const float oa = comp(o, a), da = comp(d, a);
            const float tsplit = split_distance(split, oa, da);
            const uint32_t below = (oa < split) || (oa == split && da <= 0);
            const uint32_t child = nd.y >> 2;
            if (tsplit >= tmax || tsplit < 0) {
                node = child + (1u - below);
            } else if (tsplit <= tmin) {
                node = child + below;
            } else {
                stk.node[sp * stk.stride + tid] = child + below;
                stk.tmin[sp * stk.stride + tid] = tsplit;
                stk.tmax[sp * stk.stride + tid] = tmax;
                sp++;
                node = child + (1u - below);
                tmax = tsplit;
            }
            nd = S.nodes[node];
        }
        c.leaf++;
        const uint32_t first = nd.x, count = nd.y >> 2;
        bool found = false;
        for (uint32_t j = 0; j < count; j++) {
            const TriRec r = load_rec(S, first + j);
            const uint32_t id = rec_id(r);
            if (SHADOW && id == exclude) continue;
            c.tritest++;
            float ux, uy, t;
            if (tri_test(o, d, r, tmax, ux, uy, t)) {
                if (SHADOW) return true;
                bx = ux;
                by = uy;
                tmax = t;
                tri = id;
                found = true;
            }
        }
        if (!SHADOW && found) {
            dist = tmax;
            return true;
        }
        if (sp == 0) return false;
        sp--;
        node = stk.node[sp * stk.stride + tid];
        tmin = stk.tmin[sp * stk.stride + tid];
        tmax = stk.tmax[sp * stk.stride + tid];
    }
}

// Ray-query kernel (cr_intersect / cr_intersect_shadow).
__global__ void __launch_bounds__(128) intersect_kernel(QueryArgs Q) {
    extern __shared__ uint32_t lds[];
    const uint32_t depth = Q.stack_depth;
    Stack stk{lds, (float *)(lds + depth * blockDim.x), (float *)(lds + 2 * depth * blockDim.x), blockDim.x};
    Ctr c = {};
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < Q.n) {
        const f3 o = mk(Q.orig[3 * i], Q.orig[3 * i + 1], Q.orig[3 * i + 2]);
        const f3 d = mk(Q.dir[3 * i], Q.dir[3 * i + 1], Q.dir[3 * i + 2]);
        uint32_t t = 0;
        float bx = 0.f, by = 0.f, ds = 0.f;
        if (Q.shadow) {
            c.shadow++;
            Q.hit[i] = traverse<true>(Q.S, stk, o, d, Q.dist[i], Q.light[i], t, bx, by, ds, c) ? 1u : 0u;
        } else {
            c.closest++;
            const bool h = traverse<false>(Q.S, stk, o, d, 0.f, 0xffffffffu, t, bx, by, ds, c);
            Q.hit[i] = h ? 1u : 0u;
            if (h) {
                c.hit++;
                Q.tri[i] = t;
                Q.bary[2 * i] = bx;
                Q.bary[2 * i + 1] = by;
                Q.dist_out[i] = ds;
            }
        }
    }
    flush_counters(Q.counters, c);
}

// Root-side unpermute + progressive blend of gathered tile buffers.
__global__ void __launch_bounds__(256) blend_tiles_kernel(BlendArgs B) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; // pixel in frame
    if (i >= B.xres * B.yres) return;
    const uint32_t y = i / B.xres, x = i - y * B.xres;
    const uint32_t T = B.tile;
    const uint32_t s = tile_slot(x / T, y / T, B.tiles_x, B.nranks);
    const uint32_t r = s % B.nranks, lt = s / B.nranks;
    const size_t layer_elems = (size_t)B.max_tiles * T * T; // one rank's buffer of one layer, in pixels
    const size_t src = ((size_t)r * B.nl * B.max_tiles + lt) * T * T + (y % T) * T + (x % T);
    float *o = B.frame + 3 * (size_t)i;
    f3 nw = (B.layer > 1) ? mk(o[0], o[1], o[2]) : mk(0.f, 0.f, 0.f);
    // rayTracer.cpp:64 per layer, in layer order (mean = temp * invSamples already applied by the
    // rank); the running value stays in registers, bit-identical to one blend launch per layer
    for (uint32_t j = 0; j < B.nl; j++) {
        const size_t q = 3 * (src + j * layer_elems);
        const f3 m = mk(B.gathered[q], B.gathered[q + 1], B.gathered[q + 2]);
        const uint32_t L = B.layer + j;
        nw = divs(add(muls(nw, (float)(L - 1)), m), (float)L);
    }
    o[0] = nw.x;
    o[1] = nw.y;
    o[2] = nw.z;
}

// Tonemap, one byte per thread (reads coalesced, writes row-contiguous).
// knee (rayTracer.cpp:172): logf((float)(x*f + 1)) / f in double, returned as
// float; logf and powf are evaluated in double and rounded once (glibc's logf /
// powf are double-evaluated too; the two agree except where the value lies
// within their error of a float rounding boundary -- tests/test_gpu_tonemap.py).
__global__ void __launch_bounds__(256) tonemap_kernel(TonemapArgs T) {
    const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t n = 3ull * T.xres * T.yres;
    if (e >= n) return;
    const uint32_t p = (uint32_t)(e / 3), ch = (uint32_t)(e - 3ull * p);
    const uint32_t y = p / T.xres, x = p - y * T.xres;
    float v = std_max(0.f, T.rgb[e] - T.defog);
    v *= T.m;
    if (v > T.kl) {
        const float lg = (float)log((double)(float)((double)(v - T.kl) * (double)T.f + 1.0));
        v = T.kl + (float)((double)lg / (double)T.f);
    }
    const float w = (float)pow((double)v, (double)T.gamma) * T.s;
    const float c = (w > 0.f ? w : 0.f) < 255.f ? (w > 0.f ? w : 0.f) : 255.f; // glm::clamp
    T.out[3ull * ((uint64_t)(T.yres - 1 - y) * T.xres + x) + ch] = (uint8_t)c;
}

// ---------------------------------------------------------------- launch --
int launch_intersect(const QueryArgs &Q, hipStream_t st) {
    const uint32_t block = 128;
    const size_t lds = (size_t)3 * Q.stack_depth * block * sizeof(uint32_t);
    const uint32_t grid = (Q.n + block - 1) / block;
    if (grid == 0) return 0;
    hipLaunchKernelGGL(intersect_kernel, dim3(grid), dim3(block), lds, st, Q);
    return (int)hipGetLastError();
}

int launch_blend(const BlendArgs &B, hipStream_t st) {
    const uint32_t n = B.xres * B.yres;
    if (n == 0) return 0;
    hipLaunchKernelGGL(blend_tiles_kernel, dim3((n + 255) / 256), dim3(256), 0, st, B);
    return (int)hipGetLastError();
}

int launch_tonemap(const TonemapArgs &T, hipStream_t st) {
    const uint64_t n = 3ull * T.xres * T.yres;
    if (n == 0) return 0;
    hipLaunchKernelGGL(tonemap_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st, T);
    return (int)hipGetLastError();
}

} // namespace cr
