// Micro-benchmark: cost of a wave64 global_load_dwordx4 vs the number of active
// lanes and address divergence (does the vector-memory address path charge per
// active lane or per instruction?).  L2-resident table, dependent-free loads.
//   hipcc --offload-arch=gfx950 -O3 scripts/ta_bench.hip -o /tmp/ta && /tmp/ta
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

__global__ void __launch_bounds__(256) probe(const float4 *tab, uint32_t mask, int active, int coherent, int iters,
                                             float *out) {
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t h = (blockIdx.x * 256u + threadIdx.x) * 2654435761u;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    if ((int)lane < active) {
        for (int i = 0; i < iters; i++) {
            h = h * 1664525u + 1013904223u;
            const uint32_t idx = coherent ? __builtin_amdgcn_readfirstlane(h) & mask : (h >> 4) & mask;
            const float4 v = tab[idx];
            acc.x += v.x;
            acc.y += v.y;
            acc.z += v.z;
            acc.w += v.w;
        }
    }
    if (acc.x + acc.y + acc.z + acc.w == 12345.f) out[0] = 1.f;
}

int main() {
    const uint32_t n = 1u << 17; // 2 MiB of float4: L2-resident
    float4 *tab;
    float *out;
    (void)hipMalloc(&tab, n * sizeof(float4));
    (void)hipMalloc(&out, 4);
    (void)hipMemset(tab, 0, n * sizeof(float4));
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const int iters = 2000;
    const int blocks = 256 * 8;
    for (int coherent = 0; coherent < 2; coherent++) {
        for (int active : {64, 48, 32, 16, 8, 4, 1}) {
            hipLaunchKernelGGL(probe, dim3(blocks), dim3(256), 0, 0, tab, n - 1, active, coherent, 50, out);
            (void)hipEventRecord(a, 0);
            hipLaunchKernelGGL(probe, dim3(blocks), dim3(256), 0, 0, tab, n - 1, active, coherent, iters, out);
            (void)hipEventRecord(b, 0);
            (void)hipEventSynchronize(b);
            float ms = 0.f;
            (void)hipEventElapsedTime(&ms, a, b);
            const double winstr = (double)blocks * 4 * iters; // wave-level load instructions
            printf("{\"coherent\": %d, \"active_lanes\": %d, \"ms\": %.3f, \"ns_per_wave_load_per_CU\": %.3f}\n",
                   coherent, active, ms, ms * 1e6 / (winstr / 256.0));
        }
    }
    return 0;
}
