// rt_sort.hip -- longest-first ordering of pixel units between chunk launches (hipcub radix
// sort of the rays each unit cost in the previous chunk; descending = LPT scheduling).
#include <hipcub/hipcub.hpp>

#include "rt_kernels.hpp"

namespace rtk {

size_t sort_temp_bytes(uint32_t n) {
    size_t bytes = 0;
    (void)hipcub::DeviceRadixSort::SortPairsDescending(nullptr, bytes, (const unsigned *)nullptr, (unsigned *)nullptr,
                                                 (const unsigned *)nullptr, (unsigned *)nullptr, (int)n);
    return bytes;
}

hipError_t sort_units_by_cost(const unsigned *cost, unsigned *keys_tmp, const unsigned *iota, unsigned *order,
                              uint32_t n, void *temp, size_t temp_bytes, hipStream_t s) {
    return hipcub::DeviceRadixSort::SortPairsDescending(temp, temp_bytes, cost, keys_tmp, iota, order, (int)n, 0, 32, s);
}

size_t sort_pairs_temp_bytes(size_t n, int end_bit) {
    size_t bytes = 0;
    (void)hipcub::DeviceRadixSort::SortPairsDescending(nullptr, bytes, (const unsigned *)nullptr, (unsigned *)nullptr,
                                                       (const unsigned *)nullptr, (unsigned *)nullptr, (int)n, 0,
                                                       end_bit);
    return bytes;
}

hipError_t sort_pairs_desc(const unsigned *keys_in, unsigned *keys_out, const unsigned *vals_in, unsigned *vals_out,
                           size_t n, void *temp, size_t temp_bytes, int end_bit, hipStream_t s) {
    return hipcub::DeviceRadixSort::SortPairsDescending(temp, temp_bytes, keys_in, keys_out, vals_in, vals_out, (int)n,
                                                        0, end_bit, s);
}

}  // namespace rtk
