// Batched posdb list merge on the GPU (RdbList::posdbMerge_r,
// RdbList.cpp:3065-3568).  Internal interface between merge.hip and the
// C-ABI glue in engine.hip (gbgpu_merge_posdb / gbgpu_merge_posdb_device).
#ifndef GBGPU_MERGE_H
#define GBGPU_MERGE_H

#include <stdint.h>

namespace gbmerge {

struct MergeState;

int state_new(MergeState **out);
void state_free(MergeState *s);

// Merge n device-resident posdb lists (oldest first; each 16-B aligned and
// readable up to its size rounded up to 16 bytes) into dev_out (2-B aligned,
// out_cap bytes).  Same contract and return codes as gbgpu_merge_posdb.
int merge_device(MergeState *s, const uint8_t *const *lists, const int64_t *sizes, int n, int remove_neg_keys,
                 int64_t min_rec_sizes, uint8_t *out, int64_t out_cap, int64_t *out_size);

// Host buffers in, host buffer out (uploads, merges, downloads).
int merge_host(MergeState *s, const uint8_t *const *lists, const int64_t *sizes, int n, int remove_neg_keys,
               int64_t min_rec_sizes, uint8_t *out, int64_t out_cap, int64_t *out_size);

// The last key the last merge wrote, decompressed (RdbList::m_lastKey):
// 0, or ENOENT when it wrote nothing; *more (may be NULL): whether input
// keys were left unmerged behind the cut.
int last_key(MergeState *s, uint8_t *key18, int32_t *more = nullptr);

// Phase timings of the last merge (HIP events), ms: [0] total, [1] decode
// (count + scan + decode), [2] partition (samples, rank, offsets), [3] tile
// merge, [4] tile offsets + cut, [5] copy to the output.  Plus the key and
// tile counts.
void last_timings(MergeState *s, float *ms6, int64_t *nkeys, int64_t *ntiles);

// Which pipeline ran the last merge: 2 (keys decoded to HBM), 0 none.
int last_path(MergeState *s);

}  // namespace gbmerge

#endif
