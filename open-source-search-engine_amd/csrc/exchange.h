// Msg3a::mergeLists whole (Msg3a.cpp:971-1503) over full Msg39Replies:
// the reply pack the RCCL exchange moves, the device merge of the gathered
// packs (site cap, docid dedup, facet tables, summed counts) and the same
// merge on the host.  engine.hip owns the context, the communicator and the
// sequencing; this unit owns the format and the kernels.
#ifndef GBGPU_EXCHANGE_H
#define GBGPU_EXCHANGE_H

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "../../include/gbgpu.h"

namespace gbx {

constexpr int MAXQT = 64;          // query terms the request may name
constexpr uint32_t XFMAX = 4096;   // merged entries (docsToGet) on the device
constexpr int MAXSEC = 64;         // facet sections a reply may hold

// a rank's pack: this head, then n records, then nqt facet doc counts, then
// the reply's facet list bytes as Msg39 serialized them (8-byte padded)
struct XFHead {
  int32_t n;           // m_numDocIds
  int32_t hits;        // m_estimatedHits
  int32_t has_recs;    // size_clusterRecs > 0
  int32_t nqt;         // m_nqt
  int32_t facet_bytes; // size_facetHashList
  int32_t has_fdocs;   // ptr_numDocsThatHaveFacetList given
  int32_t empty;       // no reply (a failed shard): nothing of it is read
  int32_t pad;
};
struct XFRec {
  int64_t docid;
  double score;
  uint8_t rec[12];     // the clusterdb key_t: n0 (8 bytes), n1 (4)
  uint32_t pad;
};
static_assert(sizeof(XFHead) == 32 && sizeof(XFRec) == 32, "pack layout");

// the request's fields the device merge reads
struct XFReq {
  int32_t docs_to_get, clus, hide, family, nqt, pad;
  int64_t tids[MAXQT];
  int32_t fcs[MAXQT];
};

// bytes of a reply's pack (head included), 0 for a reply that cannot be
// packed (bad sizes)
size_t pack_bytes(const gbgpu_reply *r);
// writes the pack of `r` (NULL: an empty reply) at dst
void pack_reply(const gbgpu_reply *r, int32_t nqt, uint8_t *dst);
// checks a request; fills the device view
int make_req(const gbgpu_merge_req *req, XFReq *x);

// device scratch merge_device needs for nranks packs holding facet_bytes[r]
// bytes of facet lists (0: more entries than it handles)
size_t merge_scratch_bytes(int nranks, const int32_t *facet_bytes);
// pinned host bytes merge_device reads its result through
size_t merge_stage_bytes();

// device merge of nranks packs laid `stride` bytes apart in d_recv (device
// memory), synchronously on stream st; result into `out` (host arrays).
// The caller owns the scratch (device, merge_scratch_bytes) and the stage
// (pinned host, merge_stage_bytes): the merge allocates nothing.
int merge_device(hipStream_t st, const uint8_t *d_recv, int nranks, size_t stride, const XFReq &req,
                 const int32_t *facet_bytes, uint8_t *scratch, size_t scratch_bytes, uint8_t *stage,
                 gbgpu_merged *out);

// the same merge on the host
int merge_host(const gbgpu_merge_req *req, const gbgpu_reply *replies, int nshards, gbgpu_merged *out);

}  // namespace gbx

#endif
