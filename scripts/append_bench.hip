// append_bench.hip -- cost of wf_shade's queue-append pattern alone on one MI355X: every block of a
// grid-stride launch (the shade grid: 8 blocks of 256 per CU) takes `iters` rounds, each a block barrier,
// one device-scope atomicAdd per queue by thread 0 (two queues, both in flight) and a second barrier --
// block_append_n's shape with no shading around it.  Variants: the counters in one 128-B line, in
// separate lines, or one counter pair per group of 8 blocks (8 pairs).  Measurement only.
//   hipcc --offload-arch=gfx950 -O3 -o append_bench scripts/append_bench.hip && ./append_bench
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void __launch_bounds__(256) appends(unsigned *cnt, unsigned iters, unsigned stride, unsigned groups,
                                                unsigned *sink) {
    __shared__ unsigned base[2];
    unsigned acc = 0;
    unsigned *c = cnt + (blockIdx.x % groups) * 2u * stride;
    for (unsigned it = 0; it < iters; it++) {
        __syncthreads();
        if (threadIdx.x == 0) {
            base[0] = atomicAdd(c, 200u);
            base[1] = atomicAdd(c + stride, 150u);
        }
        __syncthreads();
        acc += base[0] ^ base[1];
    }
    if (acc == 0x12345678u) sink[0] = acc; // (keeps the loop)
}

int main() {
    int dev = 0, cus = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    unsigned *cnt, *sink;
    hipMalloc(&cnt, 1 << 20);
    hipMalloc(&sink, 64);
    const unsigned blocks = (unsigned)cus * 8u;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    struct V {
        const char *name;
        unsigned stride, groups;
    } vs[] = {{"one line, 1 pair", 1, 1}, {"separate lines, 1 pair", 32, 1}, {"8 pairs", 32, 8}, {"64 pairs", 32, 64}};
    for (unsigned iters : {64u, 256u, 506u}) {
        for (const V &v : vs) {
            float best = 1e30f;
            for (int rep = 0; rep < 4; rep++) {
                hipMemset(cnt, 0, 1 << 20);
                hipEventRecord(a);
                hipLaunchKernelGGL(appends, dim3(blocks), dim3(256), 0, 0, cnt, iters, v.stride, v.groups, sink);
                hipEventRecord(b);
                hipEventSynchronize(b);
                float ms = 0.f;
                hipEventElapsedTime(&ms, a, b);
                if (rep && ms < best) best = ms;
            }
            const double atom = 2.0 * blocks * iters;
            printf("%u blocks x %u rounds, %-24s %8.3f ms  %.2f ns per atomic\n", blocks, iters, v.name, best,
                   best * 1e6 / atom);
        }
    }
    return 0;
}
