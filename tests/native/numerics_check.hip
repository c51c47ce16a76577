// GPU check of the exact fast-division helpers of device_math.hpp against the
// correctly rounded hardware-sequence division (what the reference's float
// division gives), and of the kernels' sinf / cosf against the host's glibc
// libm (what src/brdf.cpp:52-53 calls).  Built and run by tests/test_gpu_numerics.py.
//   rcp_rn      : every one of the 2^32 float bit patterns
//   div_by_rcp  : random bit patterns of a and b (all classes, all exponents)
//                 and pairs whose quotient sits next to a rounding midpoint
//   cr_sincosf  : every float in [-2pi, 2pi] (concentric()'s theta lies in [0, 2pi])
//                 against libm sinf / cosf on the host
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

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

__global__ void sincos_batch(uint32_t u0, uint32_t n, float2 *out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float sn, cs;
    cr_sincosf(__uint_as_float(u0 + i), sn, cs);
    out[i] = make_float2(sn, cs);
}

// device sincos vs host libm over float patterns [0, hi] of both signs
static int sincos_sweep(uint32_t hi, unsigned long long &bad, uint32_t &first, unsigned long long &tested) {
    const uint32_t B = 1u << 25;
    float2 *d = nullptr;
    if (hipMalloc(&d, (size_t)B * sizeof(float2)) != hipSuccess) return 2;
    std::vector<float2> h(B);
    bad = tested = 0;
    first = 0;
    for (int sg = 0; sg < 2; sg++) {
        for (uint64_t u0 = 0; u0 <= hi; u0 += B) {
            const uint32_t n = (uint32_t)std::min<uint64_t>(B, (uint64_t)hi + 1 - u0);
            const uint32_t base = (uint32_t)u0 | (sg ? 0x80000000u : 0u);
            hipLaunchKernelGGL(sincos_batch, dim3((n + 255) / 256), dim3(256), 0, 0, base, n, d);
            if (hipMemcpy(h.data(), d, (size_t)n * sizeof(float2), hipMemcpyDeviceToHost) != hipSuccess) return 2;
            unsigned long long b = 0;
            uint32_t f = 0;
#pragma omp parallel for reduction(+ : b) schedule(static)
            for (uint32_t i = 0; i < n; i++) {
                const uint32_t u = base + i;
                float x;
                std::memcpy(&x, &u, 4);
                const float es = sinf(x), ec = cosf(x);
                if (std::memcmp(&es, &h[i].x, 4) || std::memcmp(&ec, &h[i].y, 4)) {
                    b++;
#pragma omp critical
                    if (!f) f = u;
                }
            }
            bad += b;
            if (!first) first = f;
            tested += n;
        }
    }
    (void)hipFree(d);
    return 0;
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
    unsigned long long sc_bad = 0, sc_tested = 0;
    uint32_t sc_first = 0;
    float two_pi = 6.2831855f; // float above 2pi
    uint32_t hi;
    std::memcpy(&hi, &two_pi, 4);
    if (sincos_sweep(hi, sc_bad, sc_first, sc_tested)) return 2;
    printf("{\"rcp_patterns\": 4294967296, \"rcp_mismatch\": %llu, \"rcp_first\": \"0x%08x\", "
           "\"div_pairs\": %llu, \"div_fast_path\": %llu, \"div_mismatch\": %llu, \"div_first_a\": \"0x%08x\", "
           "\"sincos_tested\": %llu, \"sincos_mismatch\": %llu, \"sincos_first\": \"0x%08x\"}\n",
           h[0], hf[0], pairs, h[2], h[1], hf[1], sc_tested, sc_bad, sc_first);
    return (h[0] || h[1] || sc_bad) ? 1 : 0;
}
