// GPU check of the exact fast-division helpers of device_math.hpp against the
// correctly rounded hardware-sequence division (what the reference's float
// division gives).  Built and run by tests/test_gpu_numerics.py.
//   rcp_rn      : every one of the 2^32 float bit patterns
//   div_by_rcp  : random bit patterns of a and b (all classes, all exponents)
//                 and pairs whose quotient sits next to a rounding midpoint
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "device_math.hpp"

using namespace cr;

__device__ __forceinline__ bool same(float x, float y) {
    return __float_as_uint(x) == __float_as_uint(y) || (x != x && y != y);
}
__device__ __forceinline__ uint64_t h64(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdULL;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ULL;
    x ^= x >> 33;
    return x;
}

__global__ void rcp_all(unsigned long long *bad, unsigned int *first) {
    const uint64_t base = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 64;
    unsigned int n = 0;
    for (int i = 0; i < 64; i++) {
        const uint32_t u = (uint32_t)(base + i);
        const float a = __uint_as_float(u);
        if (!same(rcp_rn(a), 1.f / a)) {
            n++;
            atomicCAS(first, 0u, u);
        }
    }
    if (n) atomicAdd(bad, (unsigned long long)n);
}

__global__ void div_random(uint64_t seed, unsigned long long *bad, unsigned long long *fast, unsigned int *first) {
    const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    unsigned int n = 0, nf = 0;
    for (int i = 0; i < 64; i++) {
        const uint64_t s = h64(seed ^ (gid * 64 + i));
        float a, b;
        if (i & 1) {
            // b in the reciprocal range, a/b next to a midpoint
            const uint32_t sb = (uint32_t)s & 0x807fffffu;
            b = __uint_as_float(sb | ((uint32_t)(((s >> 32) % 81) + 127 - 40) << 23));
            const uint32_t qe = (uint32_t)(((s >> 40) % 121) + 127 - 60);
            const float q = __uint_as_float((qe << 23) | ((uint32_t)(s >> 9) & 0x7fffffu));
            const double mid = ((double)q + (double)__uint_as_float(__float_as_uint(q) + 1u)) * 0.5;
            a = (float)(mid * (double)b);
            if (s & (1ull << 62)) a = __uint_as_float(__float_as_uint(a) + 1u);
        } else {
            a = __uint_as_float((uint32_t)s);
            b = __uint_as_float((uint32_t)(s >> 32));
        }
        const float y = rcp_for_div(b);
        const float q0 = a * y;
        if (fabsf(q0) >= 0x1p-60f && fabsf(q0) <= 0x1p60f) nf++;
        if (!same(div_by_rcp(a, b, y), a / b)) {
            n++;
            atomicCAS(first, 0u, __float_as_uint(a));
        }
    }
    if (n) atomicAdd(bad, (unsigned long long)n);
    atomicAdd(fast, (unsigned long long)nf);
}

int main(int argc, char **argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 16;
    unsigned long long *d;
    unsigned int *f;
    if (hipMalloc(&d, 3 * sizeof(unsigned long long)) != hipSuccess || hipMalloc(&f, 2 * sizeof(unsigned int)))
        return 2;
    (void)hipMemset(d, 0, 3 * sizeof(unsigned long long));
    (void)hipMemset(f, 0, 2 * sizeof(unsigned int));
    // 2^32 patterns: 2^26 threads x 64
    hipLaunchKernelGGL(rcp_all, dim3(1u << 18), dim3(256), 0, 0, d, f);
    for (int r = 0; r < rounds; r++)
        hipLaunchKernelGGL(div_random, dim3(1u << 16), dim3(256), 0, 0, 0x9E3779B97F4A7C15ull * (r + 1), d + 1,
                           d + 2, f + 1);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    unsigned long long h[3];
    unsigned int hf[2];
    (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    (void)hipMemcpy(hf, f, sizeof(hf), hipMemcpyDeviceToHost);
    const unsigned long long pairs = (unsigned long long)rounds * (1ull << 16) * 256 * 64;
    printf("{\"rcp_patterns\": 4294967296, \"rcp_mismatch\": %llu, \"rcp_first\": \"0x%08x\", "
           "\"div_pairs\": %llu, \"div_fast_path\": %llu, \"div_mismatch\": %llu, \"div_first_a\": \"0x%08x\"}\n",
           h[0], hf[0], pairs, h[2], h[1], hf[1]);
    return (h[0] || h[1]) ? 1 : 0;
}
