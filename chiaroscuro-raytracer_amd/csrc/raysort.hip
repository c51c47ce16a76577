// raysort.hip -- queue ordering for the wavefront tracer: a device radix sort of
// (8x8-pixel sub-tile, direction bin) keys so that a trace wave takes rays that
// start near each other and point the same way (fewer distinct cache lines per
// load).  Only the processing order changes; every ray's result is written to
// its original queue slot, so the image is unchanged.
#include <hipcub/hipcub.hpp>

#include "kernels.hpp"

namespace cr {

// keys/vals are double buffers of n entries; returns the index (0/1) of the
// buffer holding the sorted permutation, or -1 on error.  tmp == nullptr asks
// for the temp size in tmp_bytes.
int sort_queue(uint32_t *keys[2], uint32_t *vals[2], uint32_t n, int end_bit, void *tmp, size_t &tmp_bytes,
               hipStream_t st) {
    hipcub::DoubleBuffer<uint32_t> k(keys[0], keys[1]), v(vals[0], vals[1]);
    if (hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, k, v, (int)n, 0, end_bit, st) != hipSuccess) return -1;
    return v.selector;
}

} // namespace cr
