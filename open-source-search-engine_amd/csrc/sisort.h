// Stable LSD radix sort of (u64 key, u32 value) pairs, hand-written for
// gfx950: the docid sort of the survivors for the second pass's
// getWordPosList emulation (engine.hip, score_info), of the facet votes
// (facet_pass) and of the stale-mbuf survivors (stale_fix), and the (term,
// key) sort of the shards' facet entries in the Msg3a exchange
// (exchange.hip).
#ifndef GBGPU_SISORT_H
#define GBGPU_SISORT_H

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace gbgpu {
// (key, value) pairs by the key's low end_bit bits (docids: 38), stable;
// tmp == nullptr returns the scratch size in tmp_bytes.  kin/vin are not
// written; kout/vout receive the sorted pairs.
hipError_t si_sort_pairs(void *tmp, size_t &tmp_bytes, const uint64_t *kin, uint64_t *kout, const uint32_t *vin,
                         uint32_t *vout, uint32_t n, hipStream_t st, int end_bit = 38);
}  // namespace gbgpu

#endif
