// samples.hip -- the per-pixel sample sum and layer blend of a render pass (rayTracer.cpp:59-64):
// every path of the pass wrote its radiance to samples[item][sample]; these kernels add each pixel's
// samples in sample order -- the reference's order -- and blend the layer into the frame (or write the
// tile mean), so the result is bit-identical to the sequential loop whatever order the paths were
// traced in.
#include "traverse.hpp"

namespace cr {

// Per pixel: add this launch's samples in sample order onto the running sum
// (A.run, carried across sample chunks), then on the last chunk blend the
// layer into the frame / write the tile mean (write_pixel).
__global__ void __launch_bounds__(256) sum_samples(RenderArgs A, int first, int last) {
    const uint32_t item = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t px = 0, py = 0;
    const bool valid = item < A.n_items && item_pixel(A, item, px, py);
    if (valid) {
        f3 temp = mk(0.f, 0.f, 0.f);
        if (!first) temp = mk(A.run[3 * (size_t)item], A.run[3 * (size_t)item + 1], A.run[3 * (size_t)item + 2]);
        const float *sm = A.samples + 3 * (size_t)item * A.s_count;
        // A.nl layers in one pass (never sample-chunked): each layer's run of A.spp samples is
        // summed in sample order and blended / written as its own layer, in layer order
        for (uint32_t j = 0; j + 1 < A.nl; j++) {
            for (uint32_t s = j * A.spp; s < (j + 1) * A.spp; s++)
                temp = add(temp, mk(sm[3 * s], sm[3 * s + 1], sm[3 * s + 2]));
            write_pixel(A, px, py, item, temp, j);
            temp = mk(0.f, 0.f, 0.f);
        }
        const uint32_t s_first = (A.nl - 1) * A.spp;
        for (uint32_t s = s_first; s < A.s_count; s++) temp = add(temp, mk(sm[3 * s], sm[3 * s + 1], sm[3 * s + 2]));
        if (last) {
            write_pixel(A, px, py, item, temp, A.nl - 1);
        } else {
            A.run[3 * (size_t)item] = temp.x;
            A.run[3 * (size_t)item + 1] = temp.y;
            A.run[3 * (size_t)item + 2] = temp.z;
        }
    }
    const uint64_t b = __ballot(valid && last);
    // (pixels written: one per layer of the pass)
    if (b && (threadIdx.x & 63u) == 0) atomicAdd(&A.counters[T_PIXELS], (unsigned long long)__popcll(b) * A.nl);
}

// sum_samples with the sample runs staged through LDS: a block's 256 pixels read their next SUM_C samples
// together (each pixel's run of SUM_C x 12 B read by consecutive lanes, 16 B each), then each thread adds
// its pixel's from LDS -- the same adds in the same order as sum_samples.  The thread-per-pixel reads of
// sum_samples touch 64 lines per wave-load and re-read each line ~10 loads later, by which time the many
// waves streaming beside it have evicted it from L2 (2-3x the sample bytes at the fabric).  Needs
// s_count % 4 == 0 (16-B aligned runs).
enum : uint32_t { SUM_C = 16, SUM_ROW = 3 * SUM_C + 1 }; // (+1: the rows of consecutive pixels start in other banks)
__global__ void __launch_bounds__(256) sum_samples_lds(RenderArgs A, int first, int last) {
    __shared__ float buf[256 * SUM_ROW];
    const uint32_t item0 = blockIdx.x * blockDim.x, item = item0 + threadIdx.x;
    const uint32_t nitems = min((uint32_t)blockDim.x, A.n_items - item0);
    uint32_t px = 0, py = 0;
    const bool valid = item < A.n_items && item_pixel(A, item, px, py);
    f3 temp = mk(0.f, 0.f, 0.f);
    if (valid && !first) temp = mk(A.run[3 * (size_t)item], A.run[3 * (size_t)item + 1], A.run[3 * (size_t)item + 2]);
    const uint32_t S = A.s_count;
    const float4 *run4 = (const float4 *)(A.samples + 3 * (size_t)item0 * S); // S % 4 == 0: 16-B aligned
    const size_t stride4 = 3 * (size_t)S / 4;                                   // float4 per pixel run
    uint32_t lj = 0;                                                            // the layer of the pass
    for (uint32_t s0 = 0; s0 < S; s0 += SUM_C) {
        const uint32_t cs = min((uint32_t)SUM_C, S - s0), q = 3 * cs / 4; // samples and float4 per pixel this chunk
        __syncthreads(); // (the previous chunk is consumed)
        for (uint32_t k = threadIdx.x; k < nitems * q; k += blockDim.x) {
            const uint32_t pix = k / q, part = k - pix * q;
            const float4 v = run4[pix * stride4 + 3 * (size_t)s0 / 4 + part];
            float *d = buf + pix * SUM_ROW + 4 * part;
            d[0] = v.x;
            d[1] = v.y;
            d[2] = v.z;
            d[3] = v.w;
        }
        __syncthreads();
        if (valid) {
            const float *b = buf + threadIdx.x * SUM_ROW;
            for (uint32_t t = 0; t < cs; t++) {
                temp = add(temp, mk(b[3 * t], b[3 * t + 1], b[3 * t + 2]));
                // A.nl layers in one pass (never sample-chunked): a layer's run ends -> blend / write it
                const uint32_t s = s0 + t + 1;
                if (A.nl > 1 && s < S && s % A.spp == 0) {
                    write_pixel(A, px, py, item, temp, lj);
                    temp = mk(0.f, 0.f, 0.f);
                    lj++;
                }
            }
        }
    }
    if (valid) {
        if (last) {
            write_pixel(A, px, py, item, temp, A.nl - 1);
        } else {
            A.run[3 * (size_t)item] = temp.x;
            A.run[3 * (size_t)item + 1] = temp.y;
            A.run[3 * (size_t)item + 2] = temp.z;
        }
    }
    const uint64_t bl = __ballot(valid && last);
    if (bl && (threadIdx.x & 63u) == 0) atomicAdd(&A.counters[T_PIXELS], (unsigned long long)__popcll(bl) * A.nl);
}

// lds: dynamic LDS reserved per block (unused: it only caps the blocks per CU, so fewer waves share
// each CU's slice of L2 while they stream their pixels' sample runs; option "sum_lds")
// staged: sum_samples_lds when the runs are 16-B aligned (option "sum_staged", default)
int launch_sum_samples(const RenderArgs &A, bool first, bool last, hipStream_t st, uint32_t lds, bool staged) {
    const uint32_t blocks = (A.n_items + 255) / 256;
    if (!blocks) return (int)hipGetLastError();
    if (staged && A.s_count % 4 == 0)
        hipLaunchKernelGGL(sum_samples_lds, dim3(blocks), dim3(256), lds, st, A, first ? 1 : 0, last ? 1 : 0);
    else
        hipLaunchKernelGGL(sum_samples, dim3(blocks), dim3(256), lds, st, A, first ? 1 : 0, last ? 1 : 0);
    return (int)hipGetLastError();
}

} // namespace cr
