#include "sisort.h"

#include <hipcub/hipcub.hpp>

namespace gbgpu {
hipError_t si_sort_pairs(void *tmp, size_t &tmp_bytes, const uint64_t *kin, uint64_t *kout, const uint32_t *vin,
                         uint32_t *vout, uint32_t n, hipStream_t st, int end_bit) {
  return hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, kin, kout, vin, vout, (int)n, 0, end_bit, st);
}
}  // namespace gbgpu
