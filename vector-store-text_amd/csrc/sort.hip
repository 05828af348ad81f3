// sort.hip — radix sort of the batch's reverse-link pairs by (level, v, u),
// so every (level, v) segment is contiguous for hnsw_reverse_kernel.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "vsg_kernels.hpp"

namespace vsg {

hipError_t sort_pairs(void* temp, size_t& temp_bytes, const uint64_t* keys_in, uint64_t* keys_out,
                      const uint32_t* vals_in, uint32_t* vals_out, size_t n, hipStream_t s) {
    return hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, keys_in, keys_out, vals_in, vals_out, (int)n, 0,
                                              PAIR_L_SHIFT + 5, s);
}

}  // namespace vsg
