// GPU check of the queue sort (csrc/raysort.hip): the hand-written stable LSD
// radix sort against std::stable_sort on the host and against hipcub's
// DeviceRadixSort, over tile-edge sizes and key widths.  Built and run by
// tests/test_gpu_sort.py; prints one JSON line.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <random>
#include <vector>

#include "../../chiaroscuro-raytracer_amd/csrc/raysort.hip"

// iota: the values are not uploaded (vals[0] holds garbage) and the sort takes the identity
static int run(uint32_t n, int bits, uint64_t seed, bool lib, std::vector<uint32_t> &ko, std::vector<uint32_t> &vo,
               bool iota = false) {
    std::mt19937_64 rng(seed);
    std::vector<uint32_t> k(n), v(n);
    const uint32_t mask = bits >= 32 ? 0xffffffffu : ((1u << bits) - 1u);
    for (uint32_t i = 0; i < n; i++) {
        k[i] = (uint32_t)rng() & mask;
        if (seed & 1) k[i] &= ~0x0f0u; // clustered keys: many equal digits
        v[i] = iota ? 0xdeadbeefu : i;
    }
    uint32_t *d[4];
    for (auto &p : d)
        if (hipMalloc(&p, (size_t)std::max<uint32_t>(n, 1) * 4) != hipSuccess) return 2;
    hipMemcpy(d[0], k.data(), (size_t)n * 4, hipMemcpyHostToDevice);
    hipMemcpy(d[2], v.data(), (size_t)n * 4, hipMemcpyHostToDevice);
    uint32_t *keys[2] = {d[0], d[1]}, *vals[2] = {d[2], d[3]};
    size_t tb = 0;
    cr::sort_queue(keys, vals, n, bits, nullptr, tb, nullptr, lib, false);
    void *tmp = nullptr;
    if (hipMalloc(&tmp, tb ? tb : 16) != hipSuccess) return 2;
    const int sel = cr::sort_queue(keys, vals, n, bits, tmp, tb, nullptr, lib, iota);
    if (sel < 0 || hipDeviceSynchronize() != hipSuccess) return 3;
    ko.resize(n);
    vo.resize(n);
    hipMemcpy(ko.data(), keys[sel], (size_t)n * 4, hipMemcpyDeviceToHost);
    hipMemcpy(vo.data(), vals[sel], (size_t)n * 4, hipMemcpyDeviceToHost);
    for (auto p : d) hipFree(p);
    hipFree(tmp);
    // host reference: stable order of (key, original index)
    std::vector<uint32_t> idx(n);
    std::iota(idx.begin(), idx.end(), 0u);
    std::stable_sort(idx.begin(), idx.end(), [&](uint32_t a, uint32_t b) { return k[a] < k[b]; });
    for (uint32_t i = 0; i < n; i++)
        if (vo[i] != idx[i] || ko[i] != k[idx[i]]) return 1;
    return 0;
}

int main() {
    const uint32_t sizes[] = {0, 1, 63, 64, 4095, 4096, 4097, 12289, 16383, 16384, 16385, 100000, 1048577, 3000001};
    const int widths[] = {1, 7, 8, 12, 25, 30, 32};
    int cases = 0, bad = 0, lib_diff = 0;
    for (uint32_t n : sizes)
        for (int bits : widths)
            for (uint64_t seed = 1; seed <= 2; seed++) {
                std::vector<uint32_t> k0, v0, k1, v1;
                const int r = run(n, bits, seed * 977 + n + bits, false, k0, v0);
                cases++;
                if (r) {
                    bad++;
                    fprintf(stderr, "mismatch n=%u bits=%d seed=%llu rc=%d\n", n, bits, (unsigned long long)seed, r);
                    continue;
                }
                if (n <= 100000 && run(n, bits, seed * 977 + n + bits, true, k1, v1) == 0 && (k0 != k1 || v0 != v1))
                    lib_diff++;
                // the identity taken by the first pass instead of uploaded values: the same result
                if (n == 0) continue;
                std::vector<uint32_t> k2, v2;
                cases++;
                if (run(n, bits, seed * 977 + n + bits, false, k2, v2, true) || k2 != k0 || v2 != v0) {
                    bad++;
                    fprintf(stderr, "iota mismatch n=%u bits=%d seed=%llu\n", n, bits, (unsigned long long)seed);
                }
            }
    printf("{\"cases\": %d, \"mismatch\": %d, \"differs_from_hipcub\": %d}\n", cases, bad, lib_diff);
    return bad ? 1 : 0;
}
