// raysort.hip -- queue ordering for the wavefront tracer: a stable LSD radix sort
// of (coherence key, queue slot) pairs, so that a trace wave takes rays that start
// near each other and point the same way (fewer distinct cache lines per load).
// Only the processing order changes; every ray's result is written to its
// original queue slot, so the image is unchanged.
//
// Hand-written for gfx950, 8-bit digits, one pass per digit of the key's
// significant bits, each pass three steps over tiles of 4096 pairs (a 256-thread
// block, 4 waves x 16 rounds x 64 lanes, tile order = wave, round, lane):
//   upsweep   per-tile digit histogram (LDS atomics) -> H[digit][tile]
//   scan      exclusive prefix of H in digit-major order (segment sums, one-block
//             scan of those, segment rescan): H[d][t] = where tile t's digit-d
//             pairs start in the output
//   downsweep stable rank of each pair inside its tile: per round the lanes with
//             the same digit find each other with 8 ballots (peer mask), a
//             per-wave digit counter in LDS gives the rank within the wave, a
//             block scan of the 4 x 256 counters the rank within the tile; the
//             pairs are staged in LDS in sorted order and written out so that
//             consecutive threads write consecutive addresses of a digit's run.
// No step waits on another block (no look-back chains): every kernel ends after
// a fixed amount of work whatever the scheduling.
// Traffic per pass: 4 B read (upsweep) + 8 B read + 8 B written (downsweep) per pair.
// The hipcub DeviceRadixSort this replaced is the checker of tests/test_gpu_sort.py
// (tests/native/sort_check.hip compiles this file with CR_SORT_LIB; the product does not).
#ifdef CR_SORT_LIB // (the sort test's comparison path: hipcub's DeviceRadixSort)
#include <hipcub/hipcub.hpp>
#endif

#include "kernels.hpp"

namespace cr {

namespace {

constexpr uint32_t RS_BITS = 8, RS_BINS = 1u << RS_BITS;
constexpr uint32_t RS_THREADS = 256, RS_WAVES = RS_THREADS / 64, RS_ROUNDS = 16;
constexpr uint32_t RS_TILE = RS_THREADS * RS_ROUNDS; // 4096 pairs
constexpr uint32_t RS_SEG = RS_THREADS * 16;         // scan segment: 4096 histogram entries

__device__ __forceinline__ uint32_t tile_item(uint32_t wave, uint32_t round, uint32_t lane) {
    return (wave * RS_ROUNDS + round) * 64u + lane;
}

// Per-wave histograms (no LDS atomic contention between waves); a round whose
// valid lanes all hold one digit -- common: neighbouring queue entries are rays of
// the same pixel -- adds its count with one atomic instead of 64 conflicting ones.
__global__ void __launch_bounds__(RS_THREADS) rs_upsweep(const uint32_t *keys, uint32_t n, uint32_t shift,
                                                         uint32_t ntiles, uint32_t *H) {
    __shared__ uint32_t hist[RS_WAVES][RS_BINS];
    const uint32_t tile = blockIdx.x, lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    for (uint32_t w = 0; w < RS_WAVES; w++) hist[w][threadIdx.x] = 0;
    __syncthreads();
    const uint32_t base = tile * RS_TILE;
    const uint32_t count = min(RS_TILE, n - base);
#pragma unroll 4
    for (uint32_t r = 0; r < RS_ROUNDS; r++) {
        const uint32_t i = tile_item(wave, r, lane);
        const bool ok = i < count;
        const uint32_t d = ok ? (keys[base + i] >> shift) & (RS_BINS - 1) : 0u;
        const uint32_t d0 = (uint32_t)__shfl((int)d, 0, 64);
        const uint64_t m_ok = __ballot(ok);
        if (__ballot(ok && d == d0) == m_ok) {
            if (lane == 0 && m_ok) atomicAdd(&hist[wave][d0], (uint32_t)__popcll(m_ok));
        } else if (ok) {
            atomicAdd(&hist[wave][d], 1u);
        }
    }
    __syncthreads();
    uint32_t t = 0;
    for (uint32_t w = 0; w < RS_WAVES; w++) t += hist[w][threadIdx.x];
    H[(size_t)threadIdx.x * ntiles + tile] = t;
}

// Block-wide exclusive scan of one value per thread; returns the block total in *total.
__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t v, uint32_t *lds /* [RS_WAVES] */,
                                                         uint32_t *total) {
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    uint32_t x = v; // inclusive scan inside the wave
#pragma unroll
    for (uint32_t off = 1; off < 64; off <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, off, 64);
        if (lane >= off) x += y;
    }
    if (lane == 63) lds[wave] = x;
    __syncthreads();
    uint32_t before = 0, all = 0;
    for (uint32_t w = 0; w < RS_WAVES; w++) {
        const uint32_t s = lds[w];
        before += w < wave ? s : 0u;
        all += s;
    }
    __syncthreads(); // lds reused by the caller
    *total = all;
    return before + x - v;
}

// segment sums of H (RS_SEG entries per block)
__global__ void __launch_bounds__(RS_THREADS) rs_scan_sums(const uint32_t *H, uint32_t m, uint32_t *sums) {
    __shared__ uint32_t lds[RS_WAVES];
    const size_t base = (size_t)blockIdx.x * RS_SEG + threadIdx.x * 16u;
    uint32_t s = 0;
    for (uint32_t k = 0; k < 16; k++)
        if (base + k < m) s += H[base + k];
    uint32_t total;
    block_exclusive_scan(s, lds, &total);
    if (threadIdx.x == 0) sums[blockIdx.x] = total;
}

// exclusive scan of the segment sums, one block
__global__ void __launch_bounds__(RS_THREADS) rs_scan_top(uint32_t *sums, uint32_t nseg) {
    __shared__ uint32_t lds[RS_WAVES];
    uint32_t carry = 0;
    for (uint32_t b = 0; b < nseg; b += RS_THREADS) {
        const uint32_t i = b + threadIdx.x;
        const uint32_t v = i < nseg ? sums[i] : 0u;
        uint32_t total;
        const uint32_t ex = block_exclusive_scan(v, lds, &total);
        if (i < nseg) sums[i] = carry + ex;
        carry += total;
    }
}

// exclusive prefix of each segment, offset by the segment's start
__global__ void __launch_bounds__(RS_THREADS) rs_scan_apply(uint32_t *H, uint32_t m, const uint32_t *sums) {
    __shared__ uint32_t lds[RS_WAVES];
    const size_t base = (size_t)blockIdx.x * RS_SEG + threadIdx.x * 16u;
    uint32_t v[16], s = 0;
#pragma unroll
    for (uint32_t k = 0; k < 16; k++) {
        v[k] = base + k < m ? H[base + k] : 0u;
        s += v[k];
    }
    uint32_t total;
    uint32_t run = sums[blockIdx.x] + block_exclusive_scan(s, lds, &total);
#pragma unroll
    for (uint32_t k = 0; k < 16; k++) {
        if (base + k < m) H[base + k] = run;
        run += v[k];
    }
}

__global__ void __launch_bounds__(RS_THREADS) rs_downsweep(const uint32_t *keys_in, const uint32_t *vals_in,
                                                           uint32_t *keys_out, uint32_t *vals_out, uint32_t n,
                                                           uint32_t shift, uint32_t ntiles, const uint32_t *H) {
    __shared__ uint32_t wave_cnt[RS_WAVES][RS_BINS]; // per-wave digit counts, then per-wave digit starts
    __shared__ uint32_t digit_start[RS_BINS];        // tile-local start of each digit
    __shared__ uint32_t out_base[RS_BINS];           // global start of this tile's digit run
    __shared__ uint32_t skey[RS_TILE], sval[RS_TILE];
    __shared__ uint32_t lds[RS_WAVES];
    const uint32_t tile = blockIdx.x, lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint32_t base = tile * RS_TILE;
    const uint32_t count = min(RS_TILE, n - base);
    for (uint32_t w = 0; w < RS_WAVES; w++) wave_cnt[w][threadIdx.x] = 0;
    out_base[threadIdx.x] = H[(size_t)threadIdx.x * ntiles + tile];
    __syncthreads();
    const uint64_t below = (lane ? (~0ull >> (64 - lane)) : 0ull);
    uint32_t key[RS_ROUNDS], val[RS_ROUNDS], rank[RS_ROUNDS];
#pragma unroll
    for (uint32_t r = 0; r < RS_ROUNDS; r++) {
        const uint32_t i = tile_item(wave, r, lane);
        const bool ok = i < count;
        key[r] = ok ? keys_in[base + i] : 0u;
        val[r] = ok ? (vals_in ? vals_in[base + i] : base + i) : 0u; // (no vals_in: the identity)
        const uint32_t d = (key[r] >> shift) & (RS_BINS - 1);
        const uint64_t m_ok = __ballot(ok);
        uint64_t peers = m_ok;
        if (__ballot(ok && d == (uint32_t)__shfl((int)d, 0, 64)) != m_ok) { // more than one digit this round
#pragma unroll
            for (uint32_t b = 0; b < RS_BITS; b++) {
                const bool bit = (d >> b) & 1u;
                const uint64_t m = __ballot(bit);
                peers &= bit ? m : ~m;
            }
        }
        // lanes of this round with my digit, then the wave's earlier rounds
        const uint32_t before = wave_cnt[wave][d];
        rank[r] = before + (uint32_t)__popcll(peers & below);
        if (ok && (peers & below) == 0) wave_cnt[wave][d] = before + (uint32_t)__popcll(peers);
        if (!ok) rank[r] = 0xffffffffu;
    }
    __syncthreads();
    // tile-local digit starts (scan over digits), then per-wave starts inside each digit
    uint32_t tot = 0;
    for (uint32_t w = 0; w < RS_WAVES; w++) tot += wave_cnt[w][threadIdx.x];
    uint32_t total;
    const uint32_t ds = block_exclusive_scan(tot, lds, &total);
    digit_start[threadIdx.x] = ds;
    uint32_t run = ds;
    for (uint32_t w = 0; w < RS_WAVES; w++) {
        const uint32_t c = wave_cnt[w][threadIdx.x];
        wave_cnt[w][threadIdx.x] = run;
        run += c;
    }
    __syncthreads();
#pragma unroll
    for (uint32_t r = 0; r < RS_ROUNDS; r++) {
        if (rank[r] == 0xffffffffu) continue;
        const uint32_t d = (key[r] >> shift) & (RS_BINS - 1);
        const uint32_t pos = wave_cnt[wave][d] + rank[r];
        skey[pos] = key[r];
        sval[pos] = val[r];
    }
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < count; j += RS_THREADS) {
        const uint32_t k = skey[j];
        const uint32_t d = (k >> shift) & (RS_BINS - 1);
        const uint32_t o = out_base[d] + (j - digit_start[d]);
        if (keys_out) keys_out[o] = k; // (null: the last pass of a sort whose keys are not read again)
        vals_out[o] = sval[j];
    }
}

} // namespace

// Workspace: H [256][ntiles] + segment sums.
static size_t rs_tmp_bytes(uint32_t n) {
    const size_t ntiles = (n + RS_TILE - 1) / RS_TILE;
    const size_t m = RS_BINS * ntiles, nseg = (m + RS_SEG - 1) / RS_SEG;
    return (m + nseg) * sizeof(uint32_t) + 256;
}

// keys/vals are double buffers of n entries; returns the index (0/1) of the buffer
// holding the sorted permutation, or -1 on error.  tmp == nullptr asks for the
// temp size in tmp_bytes.  lib: hipcub's DeviceRadixSort instead (comparison).
// iota: vals[0] is not read -- the first digit pass takes the identity 0..n-1 (the
// queue's own order), so the producer need not write it (hand-written sort only).
// keep_keys false: the last digit pass writes only the permutation (the caller reads vals only)
int sort_queue(uint32_t *keys[2], uint32_t *vals[2], uint32_t n, int end_bit, void *tmp, size_t &tmp_bytes,
               hipStream_t st, bool lib, bool iota, bool keep_keys) {
    if (iota && (lib || end_bit <= 0)) return -1;
    if (lib) {
#ifdef CR_SORT_LIB
        hipcub::DoubleBuffer<uint32_t> k(keys[0], keys[1]), v(vals[0], vals[1]);
        if (hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, k, v, (int)n, 0, end_bit, st) != hipSuccess)
            return -1;
        return v.selector;
#else
        return -1; // not compiled in
#endif
    }
    if (!tmp) {
        tmp_bytes = rs_tmp_bytes(n);
        return 0;
    }
    if (tmp_bytes < rs_tmp_bytes(n)) return -1;
    if (n == 0) return 0;
    const uint32_t ntiles = (n + RS_TILE - 1) / RS_TILE;
    const uint32_t m = RS_BINS * ntiles, nseg = (m + RS_SEG - 1) / RS_SEG;
    uint32_t *H = (uint32_t *)tmp, *sums = H + m;
    int sel = 0;
    for (int shift = 0; shift < end_bit; shift += (int)RS_BITS, sel ^= 1) {
        hipLaunchKernelGGL(rs_upsweep, dim3(ntiles), dim3(RS_THREADS), 0, st, keys[sel], n, (uint32_t)shift, ntiles,
                           H);
        hipLaunchKernelGGL(rs_scan_sums, dim3(nseg), dim3(RS_THREADS), 0, st, H, m, sums);
        hipLaunchKernelGGL(rs_scan_top, dim3(1), dim3(RS_THREADS), 0, st, sums, nseg);
        hipLaunchKernelGGL(rs_scan_apply, dim3(nseg), dim3(RS_THREADS), 0, st, H, m, sums);
        const bool last = shift + (int)RS_BITS >= end_bit;
        hipLaunchKernelGGL(rs_downsweep, dim3(ntiles), dim3(RS_THREADS), 0, st, keys[sel],
                           (iota && shift == 0) ? (const uint32_t *)nullptr : vals[sel],
                           (last && !keep_keys) ? (uint32_t *)nullptr : keys[sel ^ 1], vals[sel ^ 1], n,
                           (uint32_t)shift, ntiles, H);
    }
    if (hipGetLastError() != hipSuccess) return -1;
    return sel;
}

} // namespace cr
