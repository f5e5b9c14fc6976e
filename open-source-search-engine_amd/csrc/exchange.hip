// Msg3a::mergeLists whole (Msg3a.cpp:971-1503) over full Msg39Replies
// (exchange.h).  A reply's pack is what the RCCL all-gather moves: a 32-byte
// head, n 32-byte records (docid, double score, the 12-byte clusterdb key),
// the nqt facet doc counts and the facet list bytes exactly as Msg39
// serialized them (Msg39.cpp:1457-1555).  After the gather every rank merges
// the same packs on the device:
//   k_xf_merge     one wave: the shard-head loop of Msg3a.cpp:1315-1467 with
//                  the clusterdb site cap (1342-1379) over an LDS hash table
//                  of site counts, the docid test over an LDS list of the
//                  docids taken, the summed hits and facet doc counts
//                  (gotAllShardReplies, 792-802);
//   k_xf_sections  one lane per pack walks its facet list's sections (termid
//                  -> query term, getQueryTermByTermId64; an unknown termid
//                  ends that reply's lists, 1156-1162);
//   k_xf_keys      one thread per facet entry: (term, key) sort key, the
//                  entry's byte offset as the value;
//   si_sort_pairs  stable by (term, key), so equal keys stay in reply order;
//   k_xf_heads / k_xf_bscan / k_xf_emit
//                  the first entry of each (term, key) run is a table entry:
//                  its rank among the heads places it, and it folds the run
//                  in reply order with the reference's rules (1189-1234).
#include "exchange.h"

#include <algorithm>
#include <cerrno>
#include <cstring>
#include <unordered_map>
#include <vector>

#include "sisort.h"

namespace gbx {
namespace {

constexpr int SITE_SLOTS = 8192;     // the site-count table (LDS)
constexpr int SITE_MAX = 6144;       // distinct sites before ECAPACITY
constexpr uint32_t TERM_NONE = 0xff; // a sort key past every entry

__host__ __device__ inline uint64_t rd64(const uint8_t *p) {
  uint64_t v;
  memcpy(&v, p, 8);
  return v;
}
__host__ __device__ inline uint32_t rd32(const uint8_t *p) {
  uint32_t v;
  memcpy(&v, p, 4);
  return v;
}

inline size_t facet_off(int32_t n, int32_t nqt) { return sizeof(XFHead) + sizeof(XFRec) * (size_t)n + 8 * (size_t)nqt; }
__device__ inline size_t dfacet_off(int32_t n, int32_t nqt) {
  return sizeof(XFHead) + sizeof(XFRec) * (size_t)n + 8 * (size_t)nqt;
}

// the merged result block the device writes
struct XFOut {
  int32_t n, err;
  int64_t hits;
  int32_t nfacets, pad;
  int64_t pad2;
};
constexpr size_t OUT_DOCS = sizeof(XFOut);
constexpr size_t OUT_SCORES = OUT_DOCS + 8 * (size_t)XFMAX;
constexpr size_t OUT_RECS = OUT_SCORES + 8 * (size_t)XFMAX;
constexpr size_t OUT_FDOCS = OUT_RECS + 12 * (size_t)XFMAX;
constexpr size_t OUT_BYTES = OUT_FDOCS + 8 * (size_t)MAXQT;

// ---------------------------------------------------------------- the merge
// One wave.  Lane r < nranks holds pack r's head; the pick walks the heads in
// pack order exactly as the reference's scan over j (k_xmerge's rule).
__global__ void __launch_bounds__(64) k_xf_merge(const uint8_t *recv, int nranks, size_t stride, XFReq rq,
                                                 uint8_t *out) {
  const int lane = threadIdx.x;
  XFOut *oh = reinterpret_cast<XFOut *>(out);
  int64_t *odoc = reinterpret_cast<int64_t *>(out + OUT_DOCS);
  double *osc = reinterpret_cast<double *>(out + OUT_SCORES);
  uint8_t *orec = out + OUT_RECS;
  int64_t *ofd = reinterpret_cast<int64_t *>(out + OUT_FDOCS);
  __shared__ uint64_t s_doc[XFMAX];
  __shared__ uint32_t s_site[SITE_SLOTS];
  for (int i = lane; i < SITE_SLOTS; i += 64) s_site[i] = 0;
  uint32_t cur = 0, n = 0;
  const XFRec *rr = nullptr;
  int64_t hits = 0;
  if (lane < nranks) {
    const uint8_t *pk = recv + stride * lane;
    const XFHead *h = reinterpret_cast<const XFHead *>(pk);
    if (!h->empty) {
      n = (uint32_t)h->n;
      hits = h->hits;  // 792: int64 += int32
      rr = reinterpret_cast<const XFRec *>(pk + sizeof(XFHead));
    }
  }
  for (int off = 32; off > 0; off >>= 1) hits += __shfl_xor(hits, off, 64);
  // 794-802: every term's facet doc count summed over the replies
  for (int t = lane; t < rq.nqt; t += 64) {
    int64_t c = 0;
    for (int r = 0; r < nranks; r++) {
      const uint8_t *pk = recv + stride * r;
      const XFHead *h = reinterpret_cast<const XFHead *>(pk);
      if (h->empty || !h->has_fdocs) continue;
      c += reinterpret_cast<const int64_t *>(pk + sizeof(XFHead) + sizeof(XFRec) * (size_t)h->n)[t];
    }
    ofd[t] = c;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  uint32_t taken = 0, nsites = 0;
  int err = 0;
  const uint32_t want = (uint32_t)rq.docs_to_get;
  while (taken < want) {
    const bool has = lane < nranks && cur < n;
    const double hs = has ? rr[cur].score : 0.0;
    const uint64_t hd = has ? (uint64_t)rr[cur].docid : ~0ull;
    const uint64_t hm = __ballot(has);
    int bl = 64;
    double bs = 0.0;
    uint64_t bd = 0;
    for (int j = 0; j < nranks; j++) {  // Msg3a.cpp:1323-1334, uniform over the wave
      const double sj = __shfl(hs, j, 64);
      const uint64_t dj = __shfl(hd, j, 64);
      if (!((hm >> j) & 1)) continue;
      if (bl == 64) {
        bl = j, bs = sj, bd = dj;
        continue;
      }
      if (sj < bs) continue;
      if (sj > bs || dj < bd) bl = j, bs = sj, bd = dj;
    }
    if (bl == 64) break;  // every reply exhausted
    // the winner's clusterdb record (its pack's record at the head)
    uint64_t n0 = 0;
    uint32_t n1 = 0;
    if (lane == bl && rq.clus) {
      n0 = rd64(rr[cur].rec);
      n1 = rd32(rr[cur].rec + 8);
    }
    n0 = __shfl(n0, bl, 64);
    n1 = __shfl(n1, bl, 64);
    if (lane == bl) cur++;  // skip: the cursor moves on whatever follows (1461-1465)
    if (rq.clus && n0 != 0 && n1 != 0) {
      // 1348-1351: the family filter drops adult records
      if (rq.family && ((n0 >> 34) & 1)) continue;
      // 1353-1378: at most 2 a site (1 with hideAllClustered); site hash 0
      // is counted but never capped
      const uint32_t sh = (uint32_t)(n0 >> 2) & 0x03FFFFFFu;
      const uint32_t tag = (sh + 1) << 2;
      uint32_t h = (sh * 2654435761u) >> 19;
      int slot = -1, cnt = 0;
      for (int probe = 0; probe < SITE_SLOTS / 64; probe++, h += 64) {
        const uint32_t at = (h + lane) & (SITE_SLOTS - 1);
        const uint32_t v = s_site[at];
        const uint64_t mb = __ballot(v != 0 && (v & ~3u) == tag);
        const uint64_t eb = __ballot(v == 0);
        const int pm = mb ? __builtin_ctzll(mb) : 64, pe = eb ? __builtin_ctzll(eb) : 64;
        if (pm < pe) {  // found before the first free slot
          slot = (int)((h + pm) & (SITE_SLOTS - 1));
          cnt = (int)(__shfl(v, pm, 64) & 3u);
          break;
        }
        if (pe < 64) {
          slot = (int)((h + pe) & (SITE_SLOTS - 1));
          cnt = -1;  // new
          break;
        }
      }
      if (slot < 0) {
        err = GBGPU_ECAPACITY;
        break;
      }
      if (cnt >= 0) {
        if (sh && cnt >= 2) continue;
        if (sh && cnt >= 1 && rq.hide) continue;
        if (lane == 0) s_site[slot] = tag | (uint32_t)min(cnt + 1, 3);
      } else {
        if (++nsites > (uint32_t)SITE_MAX) {
          err = GBGPU_ECAPACITY;
          break;
        }
        if (lane == 0) s_site[slot] = tag | 1u;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    // 1381-1385: a docid merged already is passed over
    bool dup = false;
    for (uint32_t t = lane; t < taken; t += 64) dup |= s_doc[t] == bd;
    if (__ballot(dup)) continue;
    if (lane == 0) {
      s_doc[taken] = bd;
      odoc[taken] = (int64_t)bd;
      osc[taken] = bs;
    }
    if (rq.clus && lane < 3) {
      const uint32_t w = lane == 0 ? (uint32_t)n0 : lane == 1 ? (uint32_t)(n0 >> 32) : n1;
      memcpy(orec + 12 * (size_t)taken + 4 * lane, &w, 4);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    taken++;
  }
  if (lane == 0) {
    oh->n = (int32_t)taken;
    oh->err = err;
    oh->hits = hits;
  }
}

// ------------------------------------------------------------- facet tables
struct XFSec {
  uint32_t off;   // byte offset of the section's first entry in recv
  int32_t nh;     // entries
  int32_t term;   // query term
  uint32_t base;  // index of its first entry among its reply's entries
};

__global__ void __launch_bounds__(64) k_xf_sections(const uint8_t *recv, int nranks, size_t stride, XFReq rq,
                                                    XFSec *sec, int32_t *nsec, uint32_t *rbase, int32_t *err,
                                                    uint32_t *total) {
  const int lane = threadIdx.x;
  uint32_t cnt = 0;
  int ns = 0;
  int e = 0, stop = 0;
  if (lane < nranks) {
    const uint8_t *pk = recv + stride * lane;
    const XFHead *h = reinterpret_cast<const XFHead *>(pk);
    if (!h->empty && h->facet_bytes > 0) {
      size_t p = dfacet_off(h->n, h->nqt);
      const size_t end = p + (size_t)h->facet_bytes;
      while (p < end) {  // ploop, Msg3a.cpp:1147-1239
        if (end - p < 12) {
          e = GBGPU_ECORRUPT;
          break;
        }
        const int64_t tid = (int64_t)rd64(pk + p);
        const int32_t nh = (int32_t)rd32(pk + p + 8);
        p += 12;
        int term = -1;
        for (int i = 0; i < rq.nqt; i++)
          if (rq.tids[i] == tid) {
            term = i;
            break;
          }
        if (term < 0) {  // 1157-1162: `break` leaves the loop over the replies
          stop = 1;
          break;
        }
        if (nh < 0 || (size_t)nh * 36 > end - p) {
          e = GBGPU_ECORRUPT;
          break;
        }
        if (ns == MAXSEC) {
          e = GBGPU_ECAPACITY;
          break;
        }
        sec[lane * MAXSEC + ns] = XFSec{(uint32_t)(stride * lane + p), nh, term, cnt};
        ns++;
        cnt += (uint32_t)nh;
        p += 36 * (size_t)nh;
      }
    }
  }
  // an unknown termid ends the walk over the replies: packs after the first
  // that met one contribute nothing
  const uint64_t sb = __ballot(stop != 0);
  if (sb && lane > __builtin_ctzll(sb)) {
    ns = 0;
    cnt = 0;
    e = 0;
  }
  // the packs' entries numbered in pack order
  uint32_t x = cnt;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane < nranks) {
    nsec[lane] = ns;
    rbase[lane] = x - cnt;
  }
  // the shuffles run with every lane active: a lane read by ds_bpermute must
  // be in the exec mask, or the read returns 0
  const uint64_t eb = __ballot(e != 0);
  const uint32_t tot = __shfl(x, 63, 64);
  const int e0 = __shfl(e, eb ? __builtin_ctzll(eb) : 0, 64);
  if (lane == 0) {
    *total = tot;
    *err = eb ? e0 : 0;
  }
}

__global__ void k_xf_keys(const uint8_t *recv, int nranks, const XFSec *sec, const int32_t *nsec,
                          const uint32_t *rbase, const uint32_t *total, uint32_t emax, uint64_t *keys,
                          uint32_t *vals) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= emax) return;
  const uint32_t E = *total;
  if (i >= E) {
    keys[i] = ((uint64_t)TERM_NONE << 32) | 0xffffffffu;
    vals[i] = 0;
    return;
  }
  int r = 0;
  while (r + 1 < nranks && rbase[r + 1] <= i) r++;
  const XFSec *s = sec + r * MAXSEC;
  const uint32_t li = i - rbase[r];  // the entry's index inside its reply
  int k = 0;
  while (k + 1 < nsec[r] && s[k + 1].base <= li) k++;
  const uint32_t off = s[k].off + 36 * (li - s[k].base);
  const uint32_t key = rd32(recv + off);
  keys[i] = ((uint64_t)(uint32_t)s[k].term << 32) | (key ^ 0x80000000u);  // signed key order
  vals[i] = off;
}

__device__ inline bool is_head(const uint64_t *keys, uint32_t i, uint32_t E) {
  return i < E && (i == 0 || keys[i] != keys[i - 1]);
}

// heads a 256-thread block holds
__global__ void __launch_bounds__(256) k_xf_heads(const uint64_t *keys, const uint32_t *total, uint32_t emax,
                                                  uint32_t *bcnt) {
  __shared__ uint32_t wc[4];
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  const bool h = i < emax && is_head(keys, i, *total);
  const uint64_t b = __ballot(h);
  if ((threadIdx.x & 63) == 0) wc[threadIdx.x >> 6] = __popcll(b);
  __syncthreads();
  if (threadIdx.x == 0) bcnt[blockIdx.x] = wc[0] + wc[1] + wc[2] + wc[3];
}

// exclusive scan of nb block counts, the total at [nb]; one block
__global__ void __launch_bounds__(1024) k_xf_bscan(uint32_t *c, uint32_t nb) {
  __shared__ uint32_t ws[16];
  const uint32_t per = (nb + 1023) / 1024;
  const uint32_t b = threadIdx.x * per, e = min(nb, b + per);
  uint32_t s = 0;
  for (uint32_t i = b; i < e; i++) s += c[i];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t x = s;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) ws[w] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t a = 0;
    for (int i = 0; i < 16; i++) {
      const uint32_t t = ws[i];
      ws[i] = a;
      a += t;
    }
    c[nb] = a;
  }
  __syncthreads();
  uint32_t run = ws[w] + x - s;
  for (uint32_t i = b; i < e; i++) {
    const uint32_t t = c[i];
    c[i] = run;
    run += t;
  }
}

// one head per thread: fold its run in reply order (Msg3a.cpp:1189-1234)
__global__ void __launch_bounds__(256) k_xf_emit(const uint8_t *recv, const uint64_t *keys, const uint32_t *vals,
                                                 const uint32_t *total, uint32_t emax, const uint32_t *boff, XFReq rq,
                                                 gbgpu_facet_entry *out) {
  __shared__ uint32_t wc[4];
  const uint32_t E = *total;
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  const bool h = i < emax && is_head(keys, i, E);
  const uint64_t b = __ballot(h);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) wc[w] = __popcll(b);
  __syncthreads();
  if (!h) return;
  uint32_t pos = boff[blockIdx.x] + __popcll(b & ((1ull << lane) - 1));
  for (int x = 0; x < w; x++) pos += wc[x];
  const int term = (int)(keys[i] >> 32);
  const bool isfloat = rq.fcs[term] == 65, isint = rq.fcs[term] == 64;
  const uint8_t *p = recv + vals[i];
  gbgpu_facet_entry f;
  f.term = term;
  f.key = (int32_t)rd32(p);
  f.count = (int32_t)rd32(p + 4);
  f.outside = (int32_t)rd32(p + 8);
  f.docid = (int64_t)rd64(p + 12);
  f.sum = (int64_t)rd64(p + 20);
  f.max = (int32_t)rd32(p + 28);
  f.min = (int32_t)rd32(p + 32);
  for (uint32_t j = i + 1; j < E && keys[j] == keys[i]; j++) {
    const uint8_t *q = recv + vals[j];
    const int32_t c1 = (int32_t)rd32(q + 4);
    const int64_t s1 = (int64_t)rd64(q + 20);
    const int32_t mx1 = (int32_t)rd32(q + 28), mn1 = (int32_t)rd32(q + 32);
    if (isfloat) {
      const double sum = __longlong_as_double(f.sum) + __longlong_as_double(s1);
      f.sum = __double_as_longlong(sum);
      if (f.count == 0 || (c1 != 0 && __int_as_float(mn1) < __int_as_float(f.min))) f.min = mn1;
      if (f.count == 0 || (c1 != 0 && __int_as_float(mx1) > __int_as_float(f.max))) f.max = mx1;
    }
    if (isint) {
      f.sum = (int64_t)((uint64_t)f.sum + (uint64_t)s1);
      if (f.count == 0 || (c1 != 0 && mn1 < f.min)) f.min = mn1;
      if (f.count == 0 || (c1 != 0 && mx1 > f.max)) f.max = mx1;
    }
    f.count = (int32_t)((uint32_t)f.count + (uint32_t)c1);
    f.outside = (int32_t)((uint32_t)f.outside + rd32(q + 8));
    // m_docId: the first entry's (the reference picks at random, 1232-1233)
  }
  out[pos] = f;
}

inline size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

#define XCHECK(x)                      \
  do {                                 \
    if ((x) != hipSuccess) {           \
      rc = GBGPU_EHIP;                 \
      goto done;                       \
    }                                  \
  } while (0)

}  // namespace

// ---------------------------------------------------------------- host side
size_t pack_bytes(const gbgpu_reply *r) {
  if (!r) return sizeof(XFHead);
  if (r->n < 0 || r->facet_list_size < 0 || r->nqt < 0 || r->nqt > MAXQT) return 0;
  return (facet_off(r->n, r->nqt) + (size_t)r->facet_list_size + 7) & ~(size_t)7;
}

void pack_reply(const gbgpu_reply *r, int32_t nqt, uint8_t *dst) {
  XFHead h;
  std::memset(&h, 0, sizeof h);
  if (!r) {
    h.empty = 1;
    h.nqt = nqt;
    std::memcpy(dst, &h, sizeof h);
    return;
  }
  h.n = r->n;
  h.hits = r->hits;
  h.has_recs = r->cluster_recs != nullptr;
  h.nqt = r->nqt;
  h.facet_bytes = r->facet_list ? r->facet_list_size : 0;
  h.has_fdocs = r->facet_docs != nullptr;
  std::memcpy(dst, &h, sizeof h);
  XFRec *rec = reinterpret_cast<XFRec *>(dst + sizeof(XFHead));
  for (int32_t i = 0; i < r->n; i++) {
    XFRec x;
    std::memset(&x, 0, sizeof x);
    x.docid = r->docids[i];
    x.score = r->scores[i];
    if (r->cluster_recs) std::memcpy(x.rec, r->cluster_recs + 12 * (size_t)i, 12);
    std::memcpy(&rec[i], &x, sizeof x);
  }
  uint8_t *fd = dst + sizeof(XFHead) + sizeof(XFRec) * (size_t)r->n;
  if (r->facet_docs) std::memcpy(fd, r->facet_docs, 8 * (size_t)r->nqt);
  else std::memset(fd, 0, 8 * (size_t)r->nqt);
  if (h.facet_bytes) std::memcpy(fd + 8 * (size_t)r->nqt, r->facet_list, (size_t)h.facet_bytes);
}

int make_req(const gbgpu_merge_req *req, XFReq *x) {
  if (!req || req->docs_to_get <= 0 || req->nqt < 0 || req->nqt > MAXQT || (req->nqt > 0 && !req->term_ids) ||
      (req->nqt > 0 && !req->field_codes))
    return EINVAL;
  std::memset(x, 0, sizeof *x);
  x->docs_to_get = req->docs_to_get;
  x->clus = req->site_clustering != 0;
  x->hide = req->hide_all_clustered != 0;
  x->family = req->family_filter != 0;
  x->nqt = req->nqt;
  for (int i = 0; i < req->nqt; i++) {
    x->tids[i] = req->term_ids[i];
    x->fcs[i] = req->field_codes[i];
  }
  return 0;
}

namespace {
// the scratch a merge of these packs lays out (device)
struct Layout {
  uint32_t emax = 0, nb = 0;
  size_t sort_tmp = 0, o_out = 0, o_sec = 0, o_nsec = 0, o_rbase = 0, o_misc = 0, o_k = 0, o_ks = 0, o_v = 0,
         o_vs = 0, o_bc = 0, o_fac = 0, o_tmp = 0, bytes = 0;
  bool set(int nranks, const int32_t *facet_bytes) {
    uint64_t e = 1;
    for (int r = 0; r < nranks; r++) e += (uint64_t)std::max(0, facet_bytes[r]) / 36;
    if (e > (1u << 30)) return false;
    emax = (uint32_t)e;
    nb = (emax + 255) / 256;
    (void)gbgpu::si_sort_pairs(nullptr, sort_tmp, nullptr, nullptr, nullptr, nullptr, emax, nullptr, 40);
    o_out = 0;
    o_sec = o_out + al256(OUT_BYTES);
    o_nsec = o_sec + al256(sizeof(XFSec) * 64 * MAXSEC);
    o_rbase = o_nsec + 256;
    o_misc = o_rbase + 256;  // err, total
    o_k = o_misc + 256;
    o_ks = o_k + al256(8 * (size_t)emax);
    o_v = o_ks + al256(8 * (size_t)emax);
    o_vs = o_v + al256(4 * (size_t)emax);
    o_bc = o_vs + al256(4 * (size_t)emax);
    o_fac = o_bc + al256(4 * ((size_t)nb + 1));
    o_tmp = o_fac + al256(sizeof(gbgpu_facet_entry) * (size_t)emax);
    bytes = o_tmp + al256(sort_tmp);
    return true;
  }
};
// the stage: the merged block, then the section walk's error and entry
// count, then the table size
constexpr size_t ST_MISC = OUT_BYTES;
constexpr size_t ST_NFAC = OUT_BYTES + 8;
constexpr size_t ST_BYTES = OUT_BYTES + 16;
}  // namespace

size_t merge_scratch_bytes(int nranks, const int32_t *facet_bytes) {
  Layout L;
  return nranks >= 1 && nranks <= 64 && L.set(nranks, facet_bytes) ? L.bytes : 0;
}

size_t merge_stage_bytes() { return ST_BYTES; }

int merge_device(hipStream_t st, const uint8_t *d_recv, int nranks, size_t stride, const XFReq &rq,
                 const int32_t *facet_bytes, uint8_t *s, size_t scratch_bytes, uint8_t *stage, gbgpu_merged *out) {
  if (nranks < 1 || nranks > 64 || (uint32_t)rq.docs_to_get > XFMAX || !out || !s || !stage) return EINVAL;
  Layout L;
  if (!L.set(nranks, facet_bytes)) return GBGPU_ECAPACITY;
  if (scratch_bytes < L.bytes) return EINVAL;
  const uint32_t emax = L.emax, nb = L.nb;
  int rc = 0;
  {
    hipLaunchKernelGGL(k_xf_merge, dim3(1), dim3(64), 0, st, d_recv, nranks, stride, rq, s + L.o_out);
    XCHECK(hipGetLastError());
    int32_t *derr = reinterpret_cast<int32_t *>(s + L.o_misc);
    uint32_t *dtot = reinterpret_cast<uint32_t *>(s + L.o_misc + 4);
    hipLaunchKernelGGL(k_xf_sections, dim3(1), dim3(64), 0, st, d_recv, nranks, stride, rq,
                       reinterpret_cast<XFSec *>(s + L.o_sec), reinterpret_cast<int32_t *>(s + L.o_nsec),
                       reinterpret_cast<uint32_t *>(s + L.o_rbase), derr, dtot);
    XCHECK(hipGetLastError());
    uint64_t *k = reinterpret_cast<uint64_t *>(s + L.o_k), *ks = reinterpret_cast<uint64_t *>(s + L.o_ks);
    uint32_t *v = reinterpret_cast<uint32_t *>(s + L.o_v), *vs = reinterpret_cast<uint32_t *>(s + L.o_vs);
    uint32_t *bc = reinterpret_cast<uint32_t *>(s + L.o_bc);
    gbgpu_facet_entry *fac = reinterpret_cast<gbgpu_facet_entry *>(s + L.o_fac);
    hipLaunchKernelGGL(k_xf_keys, dim3(nb), dim3(256), 0, st, d_recv, nranks, reinterpret_cast<XFSec *>(s + L.o_sec),
                       reinterpret_cast<int32_t *>(s + L.o_nsec), reinterpret_cast<uint32_t *>(s + L.o_rbase), dtot,
                       emax, k, v);
    XCHECK(hipGetLastError());
    size_t tmp = L.sort_tmp;
    XCHECK(gbgpu::si_sort_pairs(s + L.o_tmp, tmp, k, ks, v, vs, emax, st, 40));
    hipLaunchKernelGGL(k_xf_heads, dim3(nb), dim3(256), 0, st, ks, dtot, emax, bc);
    hipLaunchKernelGGL(k_xf_bscan, dim3(1), dim3(1024), 0, st, bc, nb);
    hipLaunchKernelGGL(k_xf_emit, dim3(nb), dim3(256), 0, st, d_recv, ks, vs, dtot, emax, bc, rq, fac);
    XCHECK(hipGetLastError());
    // the merged block, the section walk's error and the table size, in one
    // round trip through the pinned stage
    XCHECK(hipMemcpyAsync(stage, s + L.o_out, OUT_BYTES, hipMemcpyDeviceToHost, st));
    XCHECK(hipMemcpyAsync(stage + ST_MISC, s + L.o_misc, 8, hipMemcpyDeviceToHost, st));
    XCHECK(hipMemcpyAsync(stage + ST_NFAC, bc + nb, 4, hipMemcpyDeviceToHost, st));
    XCHECK(hipStreamSynchronize(st));
    XFOut ho;
    std::memcpy(&ho, stage, sizeof ho);
    int32_t serr;
    uint32_t nfac;
    std::memcpy(&serr, stage + ST_MISC, 4);
    std::memcpy(&nfac, stage + ST_NFAC, 4);
    if (ho.err) return ho.err;
    if (serr) return serr;
    out->n = ho.n;
    out->hits = ho.hits;
    out->n_facets = (int32_t)nfac;
    const size_t n = (size_t)ho.n;
    const bool fit = !out->facets || (int32_t)nfac <= out->facets_cap;
    if (out->facets && fit && nfac) {
      XCHECK(hipMemcpyAsync(out->facets, fac, sizeof(gbgpu_facet_entry) * nfac, hipMemcpyDeviceToHost, st));
      XCHECK(hipStreamSynchronize(st));
    }
    if ((int32_t)n > out->cap) return ENOSPC;
    for (size_t i = 0; i < n; i++) {
      if (out->docids) std::memcpy(&out->docids[i], stage + OUT_DOCS + 8 * i, 8);
      if (out->scores) std::memcpy(&out->scores[i], stage + OUT_SCORES + 8 * i, 8);
    }
    if (out->cluster_recs && rq.clus) std::memcpy(out->cluster_recs, stage + OUT_RECS, 12 * n);
    if (out->facet_docs) std::memcpy(out->facet_docs, stage + OUT_FDOCS, 8 * (size_t)rq.nqt);
    if (!fit) rc = ENOSPC;
  }
done:
  if (rc == GBGPU_EHIP) (void)hipStreamSynchronize(st);
  return rc;
}

int merge_host(const gbgpu_merge_req *req, const gbgpu_reply *rep, int nshards, gbgpu_merged *out) {
  XFReq rq;
  int rc = make_req(req, &rq);
  if (rc) return rc;
  if (!out || nshards < 0 || (nshards > 0 && !rep)) return EINVAL;
  const int32_t nqt = rq.nqt;
  int64_t hits = 0;
  for (int j = 0; j < nshards; j++) {
    if (rep[j].n < 0 || rep[j].nqt != nqt || rep[j].facet_list_size < 0) return EINVAL;  // 755-761
    if (rq.clus && rep[j].n > 0 && !rep[j].cluster_recs) return EINVAL;
    hits += rep[j].hits;
  }
  // 794-802
  std::vector<int64_t> fd(nqt, 0);
  for (int j = 0; j < nshards; j++)
    if (rep[j].facet_docs)
      for (int k = 0; k < nqt; k++) fd[k] += rep[j].facet_docs[k];
  // 1129-1240: the tables, reply by reply, entry by entry
  std::vector<gbgpu_facet_entry> tab;
  std::unordered_map<uint64_t, size_t> at;
  bool stop = false;
  for (int j = 0; j < nshards && !stop; j++) {
    const uint8_t *p = rep[j].facet_list;
    if (!p) continue;
    const uint8_t *last = p + rep[j].facet_list_size;
    while (p < last) {
      if (last - p < 12) return GBGPU_ECORRUPT;
      const int64_t tid = (int64_t)rd64(p);
      const int32_t nh = (int32_t)rd32(p + 8);
      p += 12;
      int term = -1;
      for (int i = 0; i < nqt; i++)
        if (rq.tids[i] == tid) {
          term = i;
          break;
        }
      if (term < 0) {  // 1157-1162: `break` ends the walk over the replies
        stop = true;
        break;
      }
      if (nh < 0 || (int64_t)nh * 36 > last - p) return GBGPU_ECORRUPT;
      const bool isfloat = rq.fcs[term] == 65, isint = rq.fcs[term] == 64;
      for (int32_t e = 0; e < nh; e++, p += 36) {
        gbgpu_facet_entry f;
        f.term = term;
        f.key = (int32_t)rd32(p);
        f.count = (int32_t)rd32(p + 4);
        f.outside = (int32_t)rd32(p + 8);
        f.docid = (int64_t)rd64(p + 12);
        f.sum = (int64_t)rd64(p + 20);
        f.max = (int32_t)rd32(p + 28);
        f.min = (int32_t)rd32(p + 32);
        const uint64_t hk = ((uint64_t)(uint32_t)term << 32) | (uint32_t)f.key;
        auto it = at.find(hk);
        if (it == at.end()) {
          at.emplace(hk, tab.size());
          tab.push_back(f);
          continue;
        }
        gbgpu_facet_entry &g = tab[it->second];
        if (isfloat) {
          double s1, s2;
          float a, b;
          std::memcpy(&s1, &f.sum, 8);
          std::memcpy(&s2, &g.sum, 8);
          s2 += s1;
          std::memcpy(&g.sum, &s2, 8);
          std::memcpy(&a, &f.min, 4);
          std::memcpy(&b, &g.min, 4);
          if (g.count == 0 || (f.count != 0 && a < b)) g.min = f.min;
          std::memcpy(&a, &f.max, 4);
          std::memcpy(&b, &g.max, 4);
          if (g.count == 0 || (f.count != 0 && a > b)) g.max = f.max;
        }
        if (isint) {
          g.sum = (int64_t)((uint64_t)g.sum + (uint64_t)f.sum);
          if (g.count == 0 || (f.count != 0 && f.min < g.min)) g.min = f.min;
          if (g.count == 0 || (f.count != 0 && f.max > g.max)) g.max = f.max;
        }
        g.count = (int32_t)((uint32_t)g.count + (uint32_t)f.count);
        g.outside = (int32_t)((uint32_t)g.outside + (uint32_t)f.outside);
      }
    }
  }
  std::stable_sort(tab.begin(), tab.end(), [](const gbgpu_facet_entry &a, const gbgpu_facet_entry &b) {
    return a.term != b.term ? a.term < b.term : a.key < b.key;
  });
  // 1315-1467: the merge loop, the site cap before the docid test
  std::vector<int32_t> cur(nshards, 0);
  std::unordered_map<int64_t, char> seen;
  std::unordered_map<uint32_t, int32_t> site;
  int32_t n = 0;
  while (n < rq.docs_to_get) {
    int maxj = -1;
    for (int j = 0; j < nshards; j++) {
      if (cur[j] >= rep[j].n) continue;
      if (maxj == -1) {
        maxj = j;
        continue;
      }
      const double sj = rep[j].scores[cur[j]], sm = rep[maxj].scores[cur[maxj]];
      if (sj < sm) continue;
      if (sj > sm || rep[j].docids[cur[j]] < rep[maxj].docids[cur[maxj]]) maxj = j;
    }
    if (maxj < 0) break;
    const int32_t c = cur[maxj]++;
    const int64_t d = rep[maxj].docids[c];
    const uint8_t *rec = rq.clus ? rep[maxj].cluster_recs + 12 * (size_t)c : nullptr;
    if (rec) {
      const uint64_t n0 = rd64(rec);
      const uint32_t n1 = rd32(rec + 8);
      if (n0 != 0 && n1 != 0) {
        if (rq.family && ((n0 >> 34) & 1)) continue;
        const uint32_t sh = (uint32_t)(n0 >> 2) & 0x03FFFFFFu;
        auto it = site.find(sh);
        if (it != site.end()) {
          if (sh && it->second >= 2) continue;
          if (sh && it->second >= 1 && rq.hide) continue;
          it->second++;
        } else {
          site.emplace(sh, 1);
        }
      }
    }
    if (!seen.emplace(d, 1).second) continue;
    if (n >= out->cap) return ENOSPC;
    if (out->docids) out->docids[n] = d;
    if (out->scores) out->scores[n] = rep[maxj].scores[c];
    if (out->cluster_recs && rec) std::memcpy(out->cluster_recs + 12 * (size_t)n, rec, 12);
    n++;
  }
  out->n = n;
  out->hits = hits;
  if (out->facet_docs) std::memcpy(out->facet_docs, fd.data(), 8 * (size_t)nqt);
  out->n_facets = (int32_t)tab.size();
  if (out->facets) {
    if ((int32_t)tab.size() > out->facets_cap) return ENOSPC;
    std::memcpy(out->facets, tab.data(), sizeof(gbgpu_facet_entry) * tab.size());
  }
  return 0;
}

}  // namespace gbx
