// gbgpu engine: MI355X (gfx950) kernels for PosdbTable::intersectLists10_r
// and the C-ABI around them (include/gbgpu.h).
//
// Per query, with every list resident in HBM (first key swapped to 12 bytes
// at upload, Posdb.cpp:5671-5703), ONE host->device copy of the query tables
// is followed by these launches on the context's stream:
//
//   k_reset            zero the per-query counters and top-k select state
//   k_write_runs
//        candidate docids = run starts of the sublists of the smallest group
//        (addDocIdVotes group 0, Posdb.cpp:5178-5332), one sorted array per
//        sublist; array 0's own run locations are recorded here.
//   k_probe
//        scan of every other list, one wave per contiguous span, no block
//        barrier: each lane classifies 8 six-byte units by the alignment bit
//        (Posdb.h:887-889), the wave compacts the run starts into LDS with a
//        ballot prefix sum, and either the chunk's candidates binary-search
//        them (dense lists) or each run start looks its docid up in the
//        candidate arrays' bucket directory (sparse lists) -- addDocIdVotes
//        g>0 / rmDocIdVotes, Posdb.cpp:5086-5171, 4871-4946.  A hit sets the
//        list's bit in the candidate's list mask and records (unit, length)
//        of the docid's run.
//   k_cmp_count, k_cmp_place (+ k_ext_walk)
//        survivors = candidates whose lists cover every positive group and
//        no negative one (the final m_docIdVoteBuf), plus the shrunk-sublist
//        non-empty flags (shrinkSubLists, Posdb.cpp:5334-5428), placed by
//        size bucket for k_score.
//   k_score<NQ, NS>
//        one lane per survivor: mini-merge of each group (Posdb.cpp:6559-
//        6778) into the survivor's arena records, then the scorers of
//        scoring.h (weight tables staged in LDS).
//   k_topk
//        the k best (score desc, docid asc) replacing TopTree (TopTree.cpp:
//        195-516): k_score's 16-bit key histogram, one gather, the last block
//        narrows the k-th key in LDS and sorts.
//
// ONE device->host copy returns counters + top list.  No host
// synchronisation happens between kernels: counts live in device memory and
// grids are sized from host-known upper bounds.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <type_traits>
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <vector>
#include <map>
#include <array>

#include "../../include/gbgpu.h"
#include "merge.h"
#include "plan.h"
#include "posdb_key.h"
#include "scoring.h"
#include "sisort.h"
#include "exchange.h"

namespace gbgpu {

constexpr int BLOCK = 256;
constexpr int UPT = 8;                           // units per thread
constexpr int CHUNK_UNITS = BLOCK * UPT;         // 2048 units = 12 KiB per chunk
constexpr int CHUNK_BYTES = CHUNK_UNITS * 6;
constexpr int CHUNK_LOAD = CHUNK_BYTES + 16;     // + the tail of a 12-byte key
constexpr int MAX_RUNS = CHUNK_UNITS / 2;        // a run is >= 2 units
constexpr int TILE = 2048;                       // final top-k sort capacity
constexpr int MAX_K = 1536;                      // TILE - MAX_K ties merged per round
constexpr int TILE_BIG = 8192;                   // ... for a larger TopTree (k_topk<TILE_BIG>, 96 KiB of LDS)
constexpr int MAX_K_BIG = 6144;                  // docsToGet up to 3072 (m_docsWanted = 2 docsToGet)
constexpr int SEL_HBINS = 65536;                 // top-k histogram bins (key >> 16)
constexpr int TREE_CAP = 4096;                   // site-clustering TopTree nodes held in LDS
constexpr int LIST_PAD = CHUNK_LOAD + 128;

// A list re-shrunk by a later group (DevList::owner_group): its buffer then
// holds the first shrink's output P (the survivors' runs) followed by the
// list's own bytes from offset |P| on, and the re-shrink's copy of the LAST
// survivor run takes every following unit whose byte 0 has the 6-byte bit
// (Posdb.cpp:5384-5395 reads past P): that run grows by E units.
struct ListExt {
  unsigned long long units;  // |P| in 6-byte units
  unsigned long long dmax;   // docid of the last survivor with a run in the list
  unsigned long long off;    // arena offset of that survivor's relocated records (reloc)
  uint32_t E;                // units the re-shrunk copy of that run gains
  uint32_t slot1;            // its candidate slot + 1 (0: none)
  uint32_t reloc;            // its mini-merge records live at `off` (room for the extra units)
  uint32_t pad;
};

// The buckets are narrow where a wave's lanes are one survivor each: a
// lane's merge loop and scorers run for as many steps as its survivor has
// units and records, and the wave for as many as its largest lane, so the
// lanes of one wave should hold survivors of one size.  Buckets 5..15 are
// the unit counts rc, rc - 1, ... (rc <= 12: one count a bucket; wider
// steps for larger rc), 2..4 the thirds of (rc, 2rc] (two lanes a
// survivor), 1 (2rc, 4rc] and 0 above (four and eight lanes).
constexpr int NBKT = 16;
static_assert(NBKT % 4 == 0, "count rows are read as 16-byte vectors");
__host__ __device__ __forceinline__ int size_bucket(uint32_t u, uint32_t rc) {
  if (u > 4 * rc) return 0;
  if (u > 2 * rc) return 1;
  if (u > rc) {
    const uint32_t d = u - rc - 1;  // 0 .. rc - 1
    const uint32_t t = (3 * d) / rc;
    return 4 - (int)(t < 2 ? t : 2u);
  }
  const uint32_t w = rc <= 12 ? 1u : (rc + 10) / 11;
  const uint32_t k = (rc - u) / w;
  return 5 + (int)(k < 10 ? k : 10u);
}
__host__ __device__ __forceinline__ int bucket_shift(int b) { return b == 0 ? 3 : b == 1 ? 4 : b <= 4 ? 5 : 6; }

struct Counters {
  uint32_t filtered;  // m_filtered: scored docids dropped by the paging filter (Posdb.cpp:7327-7347)
  uint32_t corrupt;
  unsigned long long surv_top;  // survivors << 36 | their run units (k_cmp_place block 0)
  uint32_t g0count[MAXG0];
  uint32_t anysurv;  // bit l: list l has a run in some survivor
  uint32_t tree_n;   // site clustering: TopTree nodes written by k_tree_replay
  uint32_t tree_err; // site clustering: the tree outgrew the replay's LDS (TC nodes)
  uint32_t unsup;    // a re-shrink would copy a misparsed run (not emulated): EUNSUPPORTED
  uint32_t pad[2];
  uint32_t rdbg_t, rdbg_total;  // diagnostic: replay us in tree_add / in all
  unsigned long long dmax_all;  // largest survivor docid
  ListExt ext[MAXL];
  uint32_t bcnt[NBKT];    // survivors per size bucket (k_cmp_place block 0)
  uint32_t bstart[NBKT];  // each bucket's first survivor position
  unsigned long long arena_top;  // global record arena: units handed out (k_ext_walk, k_score, k_scoreinfo)
  uint32_t nstale;               // survivors whose trailing group merged empty (k_score: the stale list)
  uint32_t pad2;
  uint32_t sq_dbg[4];  // diagnostic (GBGPU_DIAG + GBGPU_TOPK_DEBUG): k_tree_seq clocks, 10 ns units
};

// top-k select state (k_score's histogram, k_topk's gathers)
struct Select {
  uint32_t hist[SEL_HBINS];  // scored keys per top-16-bit prefix (k_score)
  // k_topk's gathers and hand-off in ONE word, so a block's round takes both
  // offsets with one atomic and the last block's done-add returns the final
  // sizes: bits 0-15 |A| (prefix above P, < k <= MAX_K), 16-47 |B| (prefix
  // P), 48-63 blocks finished
  unsigned long long cnt;
  unsigned long long tdbg[8];  // diagnostic (GBGPU_TOPK_DEBUG): k_topk phase clocks (s_memrealtime)
};

// where a docid's run sits in one list: first unit and length in units
struct Loc {
  uint32_t unit, len;
};

struct G0Chunk {
  uint32_t array;  // candidate array index
  uint32_t u0;     // first unit
};
struct ProbeWork {
  uint32_t list;
  uint32_t u0, u1;
  uint32_t has_dfirst;  // dfirst is known (the list's granule table, ListEntry::gfirst)
  uint64_t dfirst;      // docid of the first run start at or after u0 (~0: none in the list)
};

#define HIPCHECK(x)                                                        \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      std::fprintf(stderr, "gbgpu: %s failed: %s (%s:%d)\n", #x,           \
                   hipGetErrorString(e_), __FILE__, __LINE__);             \
      return GBGPU_EHIP;                                                   \
    }                                                                      \
  } while (0)

// ------------------------------------------------------------------ helpers
// List bytes are reached through pointers kept in the plan, which the
// compiler cannot prove global: it would emit FLAT accesses, and every flat
// load makes the next wait drain vmcnt AND lgkmcnt to zero (in-flight chunk
// prefetches included).  Every list access goes through gl().
typedef const __attribute__((address_space(1))) uint8_t gu8;
__device__ __forceinline__ gu8 *gl(const uint8_t *p) { return (gu8 *)p; }
template <class T>
__device__ __forceinline__ const __attribute__((address_space(1))) T *glc(const uint8_t *p) {
  return (const __attribute__((address_space(1))) T *)p;
}
__device__ __forceinline__ bool unit_is_run_start(gu8 *u) { return (u[1] & 0x02) && !(u[0] & 0x04); }

__device__ __forceinline__ uint64_t unit_docid(const uint8_t *k) {  // Posdb.h:295
  uint64_t d = (uint64_t)k[11];
  d = (d << 32) | ((uint32_t)k[7] | ((uint32_t)k[8] << 8) | ((uint32_t)k[9] << 16) | ((uint32_t)k[10] << 24));
  return d >> 2;
}

// Stage CHUNK_LOAD bytes of a list (16-B aligned, zero padded) into LDS.
__device__ __forceinline__ void load_chunk(const uint8_t *list, uint32_t u0, uint8_t *lds) {
  typedef uint32_t v4 __attribute__((ext_vector_type(4)));
  const auto *src = glc<v4>(list + (size_t)u0 * 6);
  v4 *dst = reinterpret_cast<v4 *>(lds);
  for (int i = threadIdx.x; i < CHUNK_LOAD / 16; i += BLOCK) dst[i] = src[i];
}

// run-start bitmask of this thread's UPT units (Posdb.h:887-889 classifier).
// The thread's 48 bytes are three 16-B LDS reads (byte reads at a 48-byte
// thread stride were 4-way bank conflicts, 16 of them per thread); unit q's
// bytes 0-1 are the low half of word 3(q/2) (q even) or the high half of
// word 3(q/2)+1 (q odd).
__device__ __forceinline__ uint32_t thread_starts(const uint8_t *lds, uint32_t u0, uint32_t units) {
  static_assert(UPT == 8, "three 16-B words per thread");
  typedef uint32_t v4 __attribute__((ext_vector_type(4)));
  const v4 *src = reinterpret_cast<const v4 *>(lds + threadIdx.x * UPT * 6);
  const v4 a = src[0], b = src[1], c = src[2];
  const uint32_t w[12] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x, c.y, c.z, c.w};
  uint32_t m = 0;
#pragma unroll
  for (int q = 0; q < UPT; q++) {
    const uint32_t h = (q & 1) ? (w[3 * (q >> 1) + 1] >> 16) : (w[3 * (q >> 1)] & 0xffffu);
    const uint32_t lu = threadIdx.x * UPT + q;
    if (u0 + lu < units && (h & 0x0200u) && !(h & 0x04u)) m |= 1u << q;
  }
  return m;
}
// the docid of the 12-byte key at LDS unit lu (bytes 7-11; Posdb.h:295) from
// two aligned reads: lu even -> the words at 6lu+4 and 6lu+8, lu odd -> the
// word at 6lu+6 and the half-word at 6lu+10
__device__ __forceinline__ uint64_t lds_unit_docid(const uint8_t *lds, uint32_t lu) {
  const uint32_t b = lu * 6;
  uint64_t v;  // bytes 6..11 of the key in the low 48 bits
  if (lu & 1) {
    const uint32_t lo = *reinterpret_cast<const uint32_t *>(lds + b + 6);
    const uint32_t hi = *reinterpret_cast<const uint16_t *>(lds + b + 10);
    v = (uint64_t)lo | ((uint64_t)hi << 32);
  } else {
    const uint32_t lo = *reinterpret_cast<const uint32_t *>(lds + b + 4);
    const uint32_t hi = *reinterpret_cast<const uint32_t *>(lds + b + 8);
    v = ((uint64_t)lo >> 16) | ((uint64_t)hi << 16);
  }
  // k[7..11] = v bytes 1..5; unit_docid: ((k11 << 32) | k7..k10) >> 2
  return ((v >> 8) & 0xffffffffffull) >> 2;
}

template <int NT = BLOCK>
__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t v, uint32_t *tmp, uint32_t *total) {
  // tmp: NT/64 words of LDS
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) tmp[wid] = x;
  __syncthreads();
  uint32_t base = 0, tot = 0;
  for (int w = 0; w < NT / 64; w++) {
    if (w < wid) base += tmp[w];
    tot += tmp[w];
  }
  __syncthreads();
  *total = tot;
  return base + x - v;
}

// first index in [0,n) with a[i] >= key, cooperatively by the whole block
__device__ uint32_t block_lower_bound(const uint64_t *a, uint32_t n, uint64_t key) {
  uint32_t lo = 0, hi = n;  // answer in [lo, hi]
  while (hi - lo > 0) {
    uint32_t span = hi - lo;
    uint32_t step = (span + BLOCK - 1) / BLOCK;
    uint32_t idx = lo + threadIdx.x * step;
    int below = (idx < hi) && (a[idx] < key);
    int c = __syncthreads_count(below);
    // samples lo, lo+step, ...; c of them are < key
    if (c == 0) return lo;
    uint32_t nlo = lo + (uint32_t)(c - 1) * step + 1;
    uint32_t nhi = lo + (uint32_t)c * step;
    if (nhi > hi) nhi = hi;
    lo = nlo;
    hi = nhi;
    if (step == 1) return lo;
  }
  return lo;
}


// first run start at or after unit e (the end of the run before it); the
// continuation units of a run are the second half of its 12-byte key and
// its 6-byte keys, none of which classify as a run start (Posdb.h:887-889)
__device__ __forceinline__ uint32_t run_end(const DevList &L, uint32_t e) {
  while (e < L.units && !unit_is_run_start(gl(L.p) + (size_t)e * 6)) e++;
  return e;
}

__global__ void k_reset(uint32_t *a, uint32_t na, uint32_t *b, uint32_t nb, uint32_t *c = nullptr, uint32_t nc = 0) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < na + nb + nc; i += gridDim.x * blockDim.x) {
    if (i < na) a[i] = 0;
    else if (i < na + nb) b[i - na] = 0;
    else c[i - na - nb] = 0;
  }
}

// ----------------------------------------------- candidate extraction (G0)
// The page map, RdbMap's role (RdbMap.h:48: a list's pages and where each
// begins) for the GPU: per CHUNK_UNITS-unit page of a swapped list, the run
// starts before it, and their total at [npages].  Built once when a list is
// uploaded (k_page_count, k_page_scan), so a query's candidate slots need no
// counting pass: a run's slot is its page's prefix plus its rank in the page.
__global__ void __launch_bounds__(BLOCK) k_page_count(const uint8_t *__restrict__ list, uint32_t units,
                                                      uint32_t *__restrict__ pm) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[CHUNK_LOAD];
  __shared__ uint32_t tmp[BLOCK / 64];
  const uint32_t u0 = blockIdx.x * (uint32_t)CHUNK_UNITS;
  load_chunk(list, u0, lds);
  __syncthreads();
  uint32_t tot;
  block_exclusive_scan(__popc(thread_starts(lds, u0, units)), tmp, &tot);
  if (threadIdx.x == 0) pm[blockIdx.x] = tot;
}

// exclusive scan of the page counts in place (one block); the total lands
// at pm[npages]
__global__ void __launch_bounds__(1024) k_page_scan(uint32_t npages, uint32_t *pm) {
  __shared__ uint32_t tmp[16];
  __shared__ uint32_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (uint32_t base = 0; base < npages; base += 1024) {
    const uint32_t i = base + threadIdx.x;
    const uint32_t v = i < npages ? pm[i] : 0;
    uint32_t x = v;
    for (int o = 1; o < 64; o <<= 1) {
      uint32_t y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    if (lane == 63) tmp[wid] = x;
    __syncthreads();
    uint32_t pre = 0;
    for (int w = 0; w < wid; w++) pre += tmp[w];
    const uint32_t incl = carry + pre + x;
    __syncthreads();
    if (i < npages) pm[i] = incl - v;
    if (threadIdx.x == 1023) carry = incl;
    __syncthreads();
  }
  if (threadIdx.x == 0) pm[npages] = carry;
}

// Range terms (gbmin:/gbmax:/gbequal:, Posdb.cpp:4948-4999): isInRange on
// one key, the number where the word position is (bytes 2..5 as float or int)
__device__ __forceinline__ bool in_range_key(const DevList &L, gu8 *k) {
  const uint32_t v = (uint32_t)k[2] | ((uint32_t)k[3] << 8) | ((uint32_t)k[4] << 16) | ((uint32_t)k[5] << 24);
  if (L.rint) {
    const int32_t x = (int32_t)v;
    return L.rmode == 1 ? x >= L.ri : L.rmode == 2 ? x <= L.ri : x == L.ri;
  }
  const float x = __uint_as_float(v);
  return L.rmode == 1 ? x >= L.rf : L.rmode == 2 ? x <= L.rf : x == L.rf;
}
// isInRange2 at a run head u, run [u, e): the head, then its 6-byte keys
__device__ bool run_in_range(const DevList &L, uint32_t u, uint32_t e) {
  gu8 *p = gl(L.p);
  if (in_range_key(L, p + (size_t)u * 6)) return true;
  for (uint32_t x = u + 2; x < e; x++)
    if (in_range_key(L, p + (size_t)x * 6)) return true;
  return false;
}
// addDocIdVotes' first-group test (Posdb.cpp:5249-5277): isInRange2 at the
// head and again at every 6-byte key.  From the run's last 6-byte key that
// skips 12 bytes -- onto the next run's second unit -- and goes on over
// units with the 6-byte bit, so the next run's keys can count too.
__device__ bool run_in_range_first(const DevList &L, uint32_t u, uint32_t e) {
  if (run_in_range(L, u, e)) return true;
  if (e - u > 2) {
    gu8 *p = gl(L.p);
    for (uint32_t x = e + 1; x < L.units && (p[(size_t)x * 6] & 0x04); x++)
      if (in_range_key(L, p + (size_t)x * 6)) return true;
  }
  return false;
}

// Writes every candidate slot of every array: its docid, the unit of its run
// start in the array's own list (cunit: array 0's run locations, whose run
// ends where the next candidate's starts), the directory, and the
// whitelist / range-term rejections.  Match state lives in per-list bitmaps
// (k_probe) cleared by k_reset, so no per-slot mask is written here.
__global__ void __launch_bounds__(BLOCK) k_write_runs(const DevPlan *__restrict__ pl, const G0Chunk *__restrict__ chunks,
                                                      uint64_t *__restrict__ cand, uint32_t *__restrict__ cunit,
                                                      Counters *__restrict__ ctr, uint32_t nchunks,
                                                      uint64_t *__restrict__ dir) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[CHUNK_LOAD];
  __shared__ uint32_t tmp[BLOCK / 64];
  __shared__ uint16_t rs_unit[MAX_RUNS];
  const uint32_t me = blockIdx.x;
  const G0Chunk c = chunks[me];
  const int lid = pl->g0list[c.array];
  const DevList &L = pl->lists[lid];
  const uint32_t pos0 = L.pm[c.u0 / CHUNK_UNITS];  // the page's slot offset in its array
  load_chunk(L.p, c.u0, lds);
  __syncthreads();
  const uint32_t m0 = thread_starts(lds, c.u0, L.units);
  uint32_t tot;
  const uint32_t ex = block_exclusive_scan(__popc(m0), tmp, &tot);
  uint32_t m = m0, o = ex;
  while (m) {
    const int q = __ffs(m) - 1;
    m &= m - 1;
    rs_unit[o++] = (uint16_t)(threadIdx.x * UPT + q);
  }
  __syncthreads();
  const uint64_t base = pl->g0base[c.array];
  uint64_t *dir_a = dir + pl->g0dir[c.array];
  const uint64_t dmin = pl->g0dmin[c.array];
  const uint32_t sh = pl->g0sh[c.array];
  const uint64_t tag = (uint64_t)pl->epoch << 32;
  // runs in chunk order, strided over the block: consecutive lanes write
  // consecutive slots (coalesced stores)
  for (uint32_t o2 = threadIdx.x; o2 < tot; o2 += BLOCK) {
    const uint32_t lu = rs_unit[o2];
    const uint32_t p2 = pos0 + o2;
    const uint64_t slot = base + p2;
    const uint64_t d = lds_unit_docid(lds, lu);
    cand[slot] = d;
    cunit[slot] = c.u0 + lu;
    // directory: the first candidate of each bucket within this chunk (a
    // bucket straddling two chunks gets two writers; either names it)
    const uint64_t bkt = (d - dmin) >> sh;
    if (o2 == 0 || ((lds_unit_docid(lds, rs_unit[o2 - 1]) - dmin) >> sh) != bkt) dir_a[bkt] = tag | p2;
    bool rej = false;
    if (pl->use_white) {
      // Posdb.cpp:5294: the 5 bytes at minRecPtr+7 (the run head's docid
      // bytes, siteRank's top bit included) must be in the whitelist table
      const uint8_t *k = lds + lu * 6;
      uint64_t x = 0;
      for (int b = 4; b >= 0; b--) x = (x << 8) | k[7 + b];
      uint32_t lo = 0, hi = pl->nwhite;
      while (lo < hi) {
        const uint32_t mm = (lo + hi) >> 1;
        if (pl->white[mm] < x) lo = mm + 1;
        else hi = mm;
      }
      rej = !(lo < pl->nwhite && pl->white[lo] == x);
    }
    if (c.array == 0 && L.rmode) {
      const uint32_t u = c.u0 + lu;
      const uint32_t e = (o2 + 1 < tot) ? c.u0 + rs_unit[o2 + 1] : run_end(L, u + 2);
      if (!run_in_range_first(L, u, e)) rej = true;  // Posdb.cpp:5249-5277, 5297
    }
    if (pl->use_rej) pl->wrej[slot] = rej;
  }
  // the last chunk of each array publishes the array's count
  const bool last = (me + 1 == nchunks) || (chunks[me + 1].array != c.array);
  if (last && threadIdx.x == 0) ctr->g0count[c.array] = pos0 + tot;
}

// ------------------------------------------------------------- probe scan
// k_probe -- addDocIdVotes for groups g>0 and rmDocIdVotes (Posdb.cpp:5086-
// 5171, 4871-4946), all lists in one launch.  Every WAVE works alone (no
// block barrier anywhere): it owns a contiguous span of one list and walks it
// in 3 KiB chunks (512 six-byte units as three coalesced 1 KiB wave loads),
// loaded straight into registers two chunks ahead of use.  Per chunk:
//   1. each lane classifies its 8 units by the alignment bit (Posdb.h:887-
//      889); the run starts (<= 4 per lane: a run's 12-byte head is 2 units)
//      are compacted into the wave's LDS list with a ballot prefix sum
//      (sorted docids + unit offsets);
//   2. per candidate array k (the smallest group's sublists, in sublist
//      order), the next candidates up to the chunk's last docid -- a
//      contiguous slice continuing where the previous chunk stopped -- each
//      binary-search the run starts.  A run is credited to the first array
//      holding its docid only (claim byte), which is how the k-way union of
//      addDocIdVotes' group 0 keeps each docid once.
//   A hit records the run's (unit, length) in loc[list][slot], adds the
//   length to the slot's arena size and sets the list's bit in the slot's
//   list mask.  The last run of a chunk ends at the next chunk's first run
//   start: its length is patched there (or walked after the span).
// MODE (diagnostic, GBGPU_PROBE_MODE): 0 full, 1 stop after the run-start
// compaction, 2 load chunks only, 3 skip the run-driven lists.
constexpr int PW = 4;                      // waves per probe block
constexpr int WPIECES = 3;                 // 1 KiB wave loads per chunk
constexpr int WCH_BYTES = WPIECES * 1024;  // 3 KiB
constexpr int WCH_UNITS = WCH_BYTES / 6;   // units per wave chunk
static_assert(WCH_BYTES % 6 == 0, "a chunk holds whole units");
constexpr int WMAX_RUNS = WCH_UNITS / 2;
constexpr uint32_t PROBE_WAVES = 256 * 12;  // 3072 spans: measured best with three chunks in flight (4096: 64.1 us, 3072: 62.9)
constexpr uint32_t PROBE_WAVES_WIDE = 256 * 12;  // the wide path: three waves per SIMD (VGPRs)

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
struct WChunk {
  v4u v[WPIECES];  // piece i: bytes i*1024 + 16*lane
  uint2 nb;   // lane 63: the 8 bytes after the chunk (docid of a 12-byte key at unit 511)
};

// The chunk as three fully coalesced 1 KiB wave loads: piece i of lane L is
// bytes i*1024 + 16L .. +16 (a 48-byte-per-lane layout would make each load
// instruction touch the whole 3 KiB; measured 1.5x slower as a pure scan).
__device__ __forceinline__ void wchunk_fetch(const uint8_t *list, uint32_t u0, int lane, WChunk &c) {
  const auto *src = glc<v4u>(list + (size_t)u0 * 6 + lane * 16);
#pragma unroll
  for (int i = 0; i < WPIECES; i++) c.v[i] = __builtin_nontemporal_load(src + i * 64);
  c.nb = make_uint2(0, 0);
  if (lane == 63) {
    typedef uint32_t v2 __attribute__((ext_vector_type(2)));
    const v2 t = *glc<v2>(list + (size_t)u0 * 6 + WCH_BYTES);
    c.nb = make_uint2(t.x, t.y);
  }
}

// The same 3 KiB chunk as four 768-byte wave loads of 12 bytes a lane: lane
// L of piece i holds exactly units 128i + 2L and 128i + 2L + 1, so a unit's
// flag bytes and a run head's docid bytes sit at fixed places in the lane's
// words (no byte realignment), and the two units cannot both start a run (a
// run head's second half has byte 7 & 0x02 clear: posdb_key.h).
constexpr int W12_PIECES = WCH_BYTES / 768;
static_assert(W12_PIECES * 768 == WCH_BYTES, "a chunk is whole 12-byte-lane pieces");
struct U3 {
  uint32_t x, y, z;
};
struct WChunk12 {
  U3 v[W12_PIECES];
  uint2 nb;  // lane 63: the 8 bytes after the chunk (docid of a 12-byte key at unit 511)
};
__device__ __forceinline__ void wchunk12_fetch(const uint8_t *list, uint32_t u0, int lane, WChunk12 &c) {
  const auto *src = glc<uint32_t>(list + (size_t)u0 * 6 + lane * 12);
#pragma unroll
  for (int i = 0; i < W12_PIECES; i++) {
    c.v[i].x = __builtin_nontemporal_load(src + i * 192);
    c.v[i].y = __builtin_nontemporal_load(src + i * 192 + 1);
    c.v[i].z = __builtin_nontemporal_load(src + i * 192 + 2);
  }
  c.nb = make_uint2(0, 0);
  if (lane == 63) {
    typedef uint32_t v2 __attribute__((ext_vector_type(2)));
    const v2 t = *glc<v2>(list + (size_t)u0 * 6 + WCH_BYTES);
    c.nb = make_uint2(t.x, t.y);
  }
}

// first index in [0,n) with a[i] >= key, cooperatively by one wave (64-ary)
__device__ uint32_t wave_lower_bound(const uint64_t *a, uint32_t n, uint64_t key, int lane) {
  uint32_t lo = 0, hi = n;  // answer in [lo, hi]
  while (hi - lo > 64) {
    const uint32_t step = (hi - lo + 63) / 64;
    const uint32_t idx = lo + lane * step;
    const uint64_t m = __ballot(idx < hi && a[idx] < key);
    const uint32_t c = (uint32_t)__popcll(m);
    if (c == 0) return lo;
    const uint32_t nlo = lo + (c - 1) * step + 1;
    const uint32_t nhi = min(hi, lo + c * step);
    lo = nlo;
    hi = nhi;
  }
  const uint32_t idx = lo + lane;
  const uint64_t m = __ballot(idx < hi && a[idx] < key);
  return lo + (uint32_t)__popcll(m);
}

// Candidate lookup for run-driven probing, split so a wave issues every
// lookup's loads before it waits on any: dir_entry() gives the directory
// entry of d's bucket in array k (some candidate of that bucket, or empty);
// cand_resolve() finds d from there -- the four candidates from the entry on
// are loaded together, a walk beyond them (a crowded bucket, or a bucket
// whose entry came from a later chunk) is the rare case.
__device__ __forceinline__ uint64_t dir_entry(const DevPlan *__restrict__ pl, int k, uint32_t n, const uint64_t *dir, uint64_t d) {
  const uint64_t dmin = pl->g0dmin[k];
  if (n == 0 || d < dmin || d > pl->g0dmax[k]) return 0;
  return dir[pl->g0dir[k] + ((d - dmin) >> pl->g0sh[k])];
}
__device__ __forceinline__ int64_t cand_resolve(const DevPlan *__restrict__ pl, uint64_t e, const uint64_t *ck, uint32_t n,
                                                uint64_t d) {
  if ((uint32_t)(e >> 32) != pl->epoch) return -1;  // empty bucket
  uint32_t i = (uint32_t)e;
  uint64_t c4[4];
#pragma unroll
  for (int x = 0; x < 4; x++) c4[x] = i + x < n ? ck[i + x] : ~0ull;
  if (c4[0] > d) {
    while (i > 0) {
      const uint64_t c = ck[--i];
      if (c <= d) return c == d ? (int64_t)i : -1;
    }
    return -1;
  }
#pragma unroll
  for (int x = 0; x < 4; x++)
    if (c4[x] >= d) return c4[x] == d ? (int64_t)(i + x) : -1;
  for (i += 4; i < n; i++) {
    const uint64_t c = ck[i];
    if (c >= d) return c == d ? (int64_t)i : -1;
  }
  return -1;
}

// first index of candidate array k with docid >= key, by one wave: the
// directory entry of key's bucket (or of the next non-empty one of 64) lands
// within a few slots of the answer; a 64-wide window settles it.  Falls back
// to the 64-ary search when the window misses.
__device__ uint32_t wave_lower_bound_dir(const DevPlan *__restrict__ pl, int k, const uint64_t *ck, uint32_t n,
                                         const uint64_t *dir, uint64_t key, int lane) {
  const uint64_t dmin = pl->g0dmin[k];
  if (n == 0 || key <= dmin) return 0;
  if (key > pl->g0dmax[k]) return n;
  const uint32_t sh = pl->g0sh[k];
  const uint64_t h = (key - dmin) >> sh;
  const uint64_t hmax = (pl->g0dmax[k] - dmin) >> sh;
  const uint64_t e = h + lane <= hmax ? dir[pl->g0dir[k] + h + lane] : 0;
  const uint64_t v = __ballot((uint32_t)(e >> 32) == pl->epoch);
  if (v) {
    const int f = __ffsll((unsigned long long)v) - 1;
    const uint32_t i = (uint32_t)__shfl(e, f, 64);
    const uint32_t b0 = i > 32 ? i - 32 : 0;
    const uint32_t idx = b0 + lane;
    const uint32_t c = (uint32_t)__popcll(__ballot(idx < n && ck[idx] < key));
    if (c < 64 && (c > 0 || b0 == 0)) return b0 + c;
  }
  return wave_lower_bound(ck, n, key, lane);
}

__device__ __forceinline__ void wave_lds_sync() {
  // one wave's LDS accesses execute in order; keep the compiler from moving
  // them across this point
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Wave-private probe state: the chunk's run starts and the matches found so
// far (buffered so the scan loop issues no store or atomic: those would share
// the in-order vmcnt counter with the chunk prefetches and force full drains).
constexpr int MBUF = 192;  // with the candidate ring: 4 probe blocks per CU fit in LDS
struct ProbeLds {
  uint64_t doc[WMAX_RUNS];
  uint32_t mslot[MBUF], mu[MBUF], mlen[MBUF];
  uint16_t unit[WMAX_RUNS];
  uint8_t claim[WMAX_RUNS];
};

struct ProbeOut {
  uint32_t *bits;  // list l's match bitmap (bit s of word s >> 5: slot s)
  Loc *loc;        // run locations, [slot][nl]
  uint32_t nl, l;
  int on;          // 0: diagnostic GBGPU_PROBE_MODE=5, matches not published
};

// append up to 64 matches (one per lane), wave-wide
template <class SL>
__device__ __forceinline__ void mbuf_push(SL &S, uint32_t &nbuf, bool hit, uint32_t slot, uint32_t u,
                                          uint32_t len, int lane) {
  const uint64_t m = __ballot(hit);
  if (hit) {
    const uint32_t o = nbuf + (uint32_t)__popcll(m & ((1ull << lane) - 1));
    S.mslot[o] = slot;
    S.mu[o] = u;
    S.mlen[o] = len;
  }
  nbuf += (uint32_t)__popcll(m);
}

// publish buffered matches: each run location, and the list's bit of each
// slot -- the bits of consecutive matches in one bitmap word are OR-ed over
// the wave first (a segmented reduction; buffered slots ascend within each
// candidate array), so one atomicOr goes out per word and batch
// (out of line, with every argument by value: a by-reference counter would
// live in scratch, and scratch loads wait on vmcnt like any global load)
template <class SL>
__device__ __noinline__ void mbuf_flush_n(SL *S, uint32_t nbuf, uint32_t *bits, Loc *loc, uint32_t nl,
                                          uint32_t l, int on, int lane) {
  wave_lds_sync();
  if (!on) nbuf = 0;  // diagnostic (GBGPU_PROBE_MODE=5): matches not published
  for (uint32_t i0 = 0; i0 < nbuf; i0 += 64) {
    const uint32_t i = i0 + lane;
    const bool act = i < nbuf;
    const uint32_t slot = act ? S->mslot[i] : 0xffffffffu;
    if (act) loc[(uint64_t)slot * nl + l] = Loc{S->mu[i], S->mlen[i]};
    const uint32_t word = slot >> 5;
    uint32_t v = act ? 1u << (slot & 31) : 0u;
    const uint32_t wprev = __shfl_up(word, 1, 64);
    const bool head = act && (lane == 0 || wprev != word);
    const uint64_t H = __ballot(head);
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t vv = __shfl_down(v, off, 64);
      // lane + off is in this lane's segment: no head in (lane, lane + off]
      if (lane + off < 64 && !(H & (((1ull << off) - 1) << (lane + 1)))) v |= vv;
    }
    if (head) atomicOr(&bits[word], v);
  }
  wave_lds_sync();
}
template <class SL>
__device__ __forceinline__ void mbuf_flush(SL &S, uint32_t &nbuf, const ProbeOut &o, int lane) {
  mbuf_flush_n(&S, nbuf, o.bits, o.loc, o.nl, o.l, o.on, lane);
  nbuf = 0;
}

// Classify the chunk's units and compact the wave's run starts into S (sorted
// docids + unit offsets within the chunk).  Returns the run count.  Piece by
// piece (wchunk_fetch's layout): lane L's 16 bytes plus the 12 that follow
// (the next lane's, or the next piece's lane 0, or the bytes after the chunk)
// hold every unit starting in its 16 bytes -- 2 or 3 of them, the first at
// byte o0 = (-P) mod 6 in {0, 2, 4} -- whole, docid bytes included; the window
// is realigned to o0 with byte funnel shifts, so every byte is then read at a
// compile-time offset.
__device__ __forceinline__ uint32_t chunk_runs(const WChunk &cur, uint32_t u0, uint32_t u1, int lane, ProbeLds &S) {
  const uint64_t lt = (1ull << lane) - 1;
  uint32_t nrun = 0;
#pragma unroll
  for (int i = 0; i < WPIECES; i++) {
    uint32_t r[7];
    r[0] = cur.v[i].x;
    r[1] = cur.v[i].y;
    r[2] = cur.v[i].z;
    r[3] = cur.v[i].w;
    r[4] = __shfl_down(cur.v[i].x, 1, 64);
    r[5] = __shfl_down(cur.v[i].y, 1, 64);
    r[6] = __shfl_down(cur.v[i].z, 1, 64);
    if (i + 1 < WPIECES) {
      const uint32_t m0 = __shfl(cur.v[i + 1].x, 0, 64), m1 = __shfl(cur.v[i + 1].y, 0, 64),
                     m2 = __shfl(cur.v[i + 1].z, 0, 64);
      if (lane == 63) {
        r[4] = m0;
        r[5] = m1;
        r[6] = m2;
      }
    } else if (lane == 63) {
      r[4] = cur.nb.x;
      r[5] = cur.nb.y;
      r[6] = 0;
    }
    const uint32_t P = (uint32_t)i * 1024 + (uint32_t)lane * 16;
    const uint32_t k0 = (P + 5) / 6;  // first unit starting in [P, P + 16)
    const uint32_t o0 = k0 * 6 - P;
    uint32_t a[6];
#pragma unroll
    for (int j = 0; j < 6; j++)  // v_alignbyte shifts by 0-3 bytes: o0 = 4 is a whole dword
      a[j] = o0 == 4 ? r[j + 1] : __builtin_amdgcn_alignbyte(r[j + 1], r[j], o0);
    auto byte = [&](int b) -> uint32_t { return (a[b >> 2] >> ((b & 3) * 8)) & 0xff; };
    uint32_t starts = 0;
#pragma unroll
    for (int q = 0; q < 3; q++) {
      const bool in = 6 * q + o0 < 16 && u0 + k0 + q < u1;
      if (in && (byte(6 * q + 1) & 0x02) && !(byte(6 * q) & 0x04)) starts |= 1u << q;
    }
    const uint32_t cnt = __popc(starts);  // <= 2: a run head spans two units
    const uint64_t b0 = __ballot(cnt & 1), b1 = __ballot(cnt & 2);
    uint32_t o = nrun + (uint32_t)(__popcll(b0 & lt) + 2 * __popcll(b1 & lt));
#pragma unroll
    for (int q = 0; q < 3; q++) {
      if (!(starts >> q & 1)) continue;
      uint64_t d = 0;
#pragma unroll
      for (int b = 4; b >= 0; b--) d = (d << 8) | byte(6 * q + 7 + b);
      S.doc[o] = d >> 2;
      S.unit[o] = (uint16_t)(k0 + q);
      S.claim[o] = 0;
      o++;
    }
    nrun += (uint32_t)(__popcll(b0) + 2 * __popcll(b1));
  }
  wave_lds_sync();
  return nrun;
}

// docid of the first run start at or after unit u (< u1), ~0 if none
__device__ uint64_t first_run_doc(const DevList &L, uint32_t u, uint32_t u1, int lane) {
  gu8 *p = gl(L.p);
  for (; u < u1; u += 64) {
    const uint32_t x = u + lane;
    const bool st = x < u1 && unit_is_run_start(p + (size_t)x * 6);
    const uint64_t m = __ballot(st);
    if (m) {
      const int f = __ffsll((unsigned long long)m) - 1;
      uint64_t d = 0;
      if (lane == f) {
        gu8 *k = p + (size_t)x * 6;
        for (int i = 11; i >= 7; i--) d = (d << 8) | k[i];
        d >>= 2;
      }
      return __shfl(d, f, 64);
    }
  }
  return ~0ull;
}

#ifdef GBGPU_DIAG  // probe_by_cand and the table path: measured alternatives, diagnostic builds only
// Dense list: candidates search the run starts.  Memory pipelining under the
// in-order vmcnt counter: two chunk buffers with static roles (the loop is
// unrolled by two, so no in-flight register is ever copied -- a copy would
// wait for its load), one chunk in flight while the other is worked on.  Each
// array's candidate window (cur: the 64 candidates from lok, one per lane) is
// followed by the next 64 (nxt), loaded one chunk ahead: the next chunk's
// window is shuffled out of the two, so no candidate load is waited for in
// the loop unless a chunk consumes more than 64 (dense arrays).
template <int MODE, int G0>
__device__ void probe_by_cand(const DevPlan *__restrict__ pl, const ProbeWork &w, const DevList &L, const uint64_t *cand,
                              const Counters *ctr, const uint64_t *dir, ProbeLds &S, const ProbeOut &po, int lane) {
  const int g0n = G0 <= 2 ? G0 : pl->g0n;
  const uint8_t *lp = L.p;
  uint32_t nk[G0], lok[G0];
  uint64_t base[G0], cur[G0], nxt[G0];
  const uint32_t last_u0 = w.u0 + ((w.u1 - w.u0 - 1) / WCH_UNITS) * WCH_UNITS;
  WChunk cA, cB;
  // where each array's candidates meet this span (peeled out of the loop)
  constexpr bool FULL = MODE == 0 || MODE == 5;
  const uint64_t dfirst = FULL ? first_run_doc(L, w.u0, w.u1, lane) : 0;
  auto cload = [&](int k, uint32_t i) -> uint64_t {  // candidate i of array k (clamped; validity at use)
    return cand[base[k] + min(i, max(nk[k], 1u) - 1)];
  };
#pragma unroll
  for (int k = 0; k < G0; k++) {
    nk[k] = k < g0n ? ctr->g0count[k] : 0;
    base[k] = k < g0n ? pl->g0base[k] : 0;
    lok[k] = (FULL && k < g0n) ? wave_lower_bound_dir(pl, k, cand + base[k], nk[k], dir, dfirst, lane) : 0;
    cur[k] = cload(k, lok[k] + lane);
    nxt[k] = cload(k, lok[k] + 64 + lane);
  }
  // the first two chunks after the windows, so the loop header sees the
  // same issue order from here as from its back edge (window, then chunk)
  wchunk_fetch(lp, w.u0, lane, cA);
  wchunk_fetch(lp, min(w.u0 + WCH_UNITS, last_u0), lane, cB);
  uint32_t nbuf = 0;
  uint64_t pend_slot = ~0ull;  // slot whose run length waits for the next run start
  uint32_t pend_u = 0;
  // one chunk at u0 (its bytes in c)
  auto step = [&](const WChunk &c, uint32_t u0) {
    if (MODE == 2) {
      if (c.v[0].x == 0x557713eeu && c.v[1].y == 7u && c.v[2].z == 3u) po.bits[0] = 1;
      return;
    }
    const uint32_t nrun = chunk_runs(c, u0, w.u1, lane, S);
    if (nrun && pend_slot != ~0ull) {
      if (nbuf + 1 > MBUF) mbuf_flush(S, nbuf, po, lane);
      mbuf_push(S, nbuf, lane == 0, (uint32_t)pend_slot, pend_u, u0 + S.unit[0] - pend_u, lane);
      pend_slot = ~0ull;
    }
    if (MODE == 1) {
      if (nrun && S.doc[0] == 0x123456789ull) po.bits[0] = 1;
      wave_lds_sync();
      return;
    }
    const uint64_t dmax = nrun ? S.doc[nrun - 1] : 0;
    // every array's window is searched at once (the arrays' LDS round trips
    // overlap); claims are then settled array by array, in order
    uint64_t dk[G0];
    uint32_t pa[G0];
#pragma unroll
    for (int k = 0; k < G0; k++) {
      dk[k] = (k < g0n && lok[k] + lane < nk[k]) ? cur[k] : ~0ull;
      pa[k] = 0;
    }
    // branchless lower bound (nrun <= WMAX_RUNS): no divergence, no
    // exec-mask bookkeeping, every array's read of a step issued together
#pragma unroll
    for (uint32_t st = WMAX_RUNS; st > 0; st >>= 1) {
#pragma unroll
      for (int k = 0; k < G0; k++) {
        const uint32_t t = pa[k] + st;
        const uint64_t v = S.doc[min(t, max(nrun, 1u)) - 1];
        if (t <= nrun && v < dk[k]) pa[k] = t;
      }
    }
#pragma unroll
    for (int k = 0; k < G0; k++) {
      if (k >= g0n) break;
      uint32_t lo = lok[k];
      // one pass: the 64 candidates from lo (one per lane) against the runs;
      // a is d's lower bound in the runs (searched above)
      auto settle = [&](uint64_t d, uint32_t a) -> uint32_t {
        const bool in = nrun && d <= dmax;
        bool hit = false, last = false;
        uint32_t u = 0, len = 0;
        if (in && a < nrun && S.doc[a] == d && !S.claim[a]) {
          S.claim[a] = 1;
          u = u0 + S.unit[a];
          if (a + 1 < nrun) {
            hit = true;
            len = S.unit[a + 1] - S.unit[a];
          } else {
            last = true;  // ends at the next chunk's first run start
          }
        }
        if (nbuf + 64 > MBUF) mbuf_flush(S, nbuf, po, lane);
        mbuf_push(S, nbuf, hit, (uint32_t)(base[k] + lo + lane), u, len, lane);
        const uint64_t pm = __ballot(last);
        if (pm) {
          pend_slot = base[k] + lo + (uint32_t)(__ffsll((unsigned long long)pm) - 1);
          pend_u = u0 + S.unit[nrun - 1];
        }
        const uint32_t nin = (uint32_t)__popcll(__ballot(in));
        lo += nin;
        return nin;
      };
      const uint32_t used = settle(dk[k], pa[k]);
      if (used < 64u) {
        // the next window: 64 - used candidates left in cur, the rest from nxt
        const int sl = (lane + (int)used) & 63;
        const uint64_t a = __shfl(cur[k], sl, 64), b = __shfl(nxt[k], sl, 64);
        cur[k] = lane + used < 64u ? a : b;
        lok[k] = lo;
        nxt[k] = cload(k, lo + 64 + lane);  // used one chunk later
      } else {
        // a chunk meeting more than 64 candidates (dense arrays) reloads in a
        // loop of its own (its loads are waited for at once)
        for (;;) {
          const uint64_t d = lo + lane < nk[k] ? cand[base[k] + lo + lane] : ~0ull;
          uint32_t a = 0;
#pragma unroll
          for (uint32_t st = WMAX_RUNS; st > 0; st >>= 1) {
            const uint32_t t = a + st;
            const uint64_t v = S.doc[min(t, max(nrun, 1u)) - 1];
            if (t <= nrun && v < d) a = t;
          }
          if (settle(d, a) < 64u) break;
        }
        lok[k] = lo;
        cur[k] = cload(k, lo + lane);
        nxt[k] = cload(k, lo + 64 + lane);
        // both used here, so the merge with the usual path leaves no load of
        // them pending (the waitcnt pass would then wait for everything)
        __asm__ volatile("" ::"v"(cur[k]), "v"(nxt[k]));
      }
    }
    wave_lds_sync();  // the next chunk rewrites the run list
  };
  // static buffer roles: the fetch three chunks ahead goes to the buffer just
  // worked on, after the step's candidate loads (vmcnt is in order: the next
  // step's wait for its chunk then leaves this fetch in flight)
  // Two chunk buffers with static roles (the loop is unrolled by two: no
  // in-flight register is copied), one chunk in flight while the other is
  // worked on; no exit in the loop body's middle (an exit there is an edge
  // into the header between the steps, and the waitcnt pass would wait for
  // the first buffer at once); the odd chunk left over follows it.  The
  // scheduling barriers keep each fetch where it is (sunk to the latch, it
  // would be waited for at once).
  const uint32_t nch = (w.u1 - w.u0 + WCH_UNITS - 1) / WCH_UNITS;
  uint32_t u0 = w.u0;
  for (uint32_t it = 0; it + 2 <= nch; it += 2, u0 += 2 * WCH_UNITS) {
    step(cA, u0);
    wchunk_fetch(lp, min(u0 + 2 * WCH_UNITS, last_u0), lane, cA);
    __builtin_amdgcn_sched_barrier(0);
    step(cB, u0 + WCH_UNITS);
    wchunk_fetch(lp, min(u0 + 3 * WCH_UNITS, last_u0), lane, cB);
    __builtin_amdgcn_sched_barrier(0);
  }
  if (nch & 1) step(cA, u0);
  if (pend_slot != ~0ull) {
    const uint32_t len = lane == 0 ? run_end(L, pend_u + 2) - pend_u : 0;
    if (nbuf + 1 > MBUF) mbuf_flush(S, nbuf, po, lane);
    mbuf_push(S, nbuf, lane == 0, (uint32_t)pend_slot, pend_u, len, lane);
  }
  mbuf_flush(S, nbuf, po, lane);
}

// Dense list, up to four candidate arrays (HPATH): no run list and no
// search.  The run starts stay in the registers that classified them; the
// window of each candidate array (its next 64 candidates, one per lane) goes
// into an LDS table of order-preserving docid buckets over the chunk's docid
// range [dlo, dhi] (bucket = (d - dlo) >> s, fewer than HB buckets), each
// bucket naming its first window lane; a run start then finds a candidate
// with its docid by one table read and one read of the (at most few)
// candidates from that lane -- two LDS round trips where the run-list search
// took nine.  The claim order (a docid goes to the first array holding it,
// addDocIdVotes' k-way union of group 0) is the order the arrays are tried
// in.  A run's length ends at the next run start: the same lane's, the next
// lane's of its piece (one bpermute per piece), a later piece's, or the next
// chunk's (pending).  The span starts at the host-known first run docid
// (ListEntry::gfirst) through the candidate directory (wave_start_dir).
constexpr int HB = 512;     // docid buckets of a chunk's table
constexpr int HPATH_G0 = 4;  // arrays the table path handles (more: probe_by_cand)
template <int G0>
struct HashLds {
  uint16_t tab[G0][HB];  // bucket -> tag << 6 | the bucket's first window lane
  uint64_t win[G0][64];  // each array's window
  uint32_t mslot[MBUF], mu[MBUF], mlen[MBUF];
};

#endif  // GBGPU_DIAG

// first candidate index of array k at or below lower_bound(key) and close to
// it: the directory entry of the last non-empty bucket of the 64 below key's
__device__ uint32_t wave_start_dir(const DevPlan *__restrict__ pl, int k, const uint64_t *ck, uint32_t n, const uint64_t *dir,
                                   uint64_t key, int lane) {
  const uint64_t dmin = pl->g0dmin[k];
  if (n == 0 || key <= dmin) return 0;
  if (key > pl->g0dmax[k]) return n;
  const uint32_t sh = pl->g0sh[k];
  const uint64_t h = (key - dmin) >> sh;  // >= 0; buckets below h hold docids < key
  const int64_t b = (int64_t)h - 64 + lane;
  const uint64_t e = b >= 0 ? dir[pl->g0dir[k] + (uint64_t)b] : 0;
  const uint64_t v = __ballot((uint32_t)(e >> 32) == pl->epoch);
  if (v) {
    const int f = 63 - __builtin_clzll((unsigned long long)v);
    return (uint32_t)__shfl(e, f, 64);
  }
  if (h < 64) return 0;  // every bucket below key's is empty
  return wave_lower_bound(ck, n, key, lane);
}

// DPP whole-wave lane shifts (lane L reads lane L+1 / L-1; the lane with no
// source keeps `edge`): VALU moves, no LDS round trip
__device__ __forceinline__ uint32_t lane_next(uint32_t x, uint32_t edge) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)edge, (int)x, 0x130, 0xf, 0xf, false);  // wave_shl:1
}
__device__ __forceinline__ uint32_t lane_prev(uint32_t x, uint32_t edge) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)edge, (int)x, 0x138, 0xf, 0xf, false);  // wave_shr:1
}

#ifdef GBGPU_DIAG  // the measured alternatives (probe_by_cand_hash / _wide): diagnostic builds only
// piece i of a chunk (wchunk_fetch's layout, as chunk_runs): the run starts
// among the units starting in this lane's 16 bytes (at most two: a run head is
// two units), their docids and chunk-relative units
__device__ __forceinline__ uint32_t piece_starts(const WChunk &cur, int i, uint32_t u0, uint32_t u1, int lane, uint64_t &da,
                                                uint64_t &db, uint32_t &ua, uint32_t &ub) {
  uint32_t r[7];
  r[0] = cur.v[i].x;
  r[1] = cur.v[i].y;
  r[2] = cur.v[i].z;
  r[3] = cur.v[i].w;
  uint32_t e0, e1, e2;  // lane 63: the next piece's first bytes, or the bytes after the chunk
  if (i + 1 < WPIECES) {
    e0 = __builtin_amdgcn_readfirstlane(cur.v[i + 1].x);
    e1 = __builtin_amdgcn_readfirstlane(cur.v[i + 1].y);
    e2 = __builtin_amdgcn_readfirstlane(cur.v[i + 1].z);
  } else {
    e0 = cur.nb.x;
    e1 = cur.nb.y;
    e2 = 0;
  }
  r[4] = lane_next(r[0], e0);
  r[5] = lane_next(r[1], e1);
  r[6] = lane_next(r[2], e2);
  const uint32_t P = (uint32_t)i * 1024 + (uint32_t)lane * 16;
  const uint32_t k0 = (P + 5) / 6;  // first unit starting in [P, P + 16)
  const uint32_t o0 = k0 * 6 - P;
  uint32_t a[6];
#pragma unroll
  for (int j = 0; j < 6; j++) a[j] = o0 == 4 ? r[j + 1] : __builtin_amdgcn_alignbyte(r[j + 1], r[j], o0);
  auto byte = [&](int b) -> uint32_t { return (a[b >> 2] >> ((b & 3) * 8)) & 0xff; };
  auto docid_at = [&](int q) -> uint64_t {
    uint64_t d = 0;
#pragma unroll
    for (int b = 4; b >= 0; b--) d = (d << 8) | byte(6 * q + 7 + b);
    return d >> 2;
  };
  uint32_t starts = 0;
#pragma unroll
  for (int q = 0; q < 3; q++) {
    const bool in = 6 * q + o0 < 16 && u0 + k0 + q < u1;
    if (in && (byte(6 * q + 1) & 0x02) && !(byte(6 * q) & 0x04)) starts |= 1u << q;
  }
  // starts: a subset of {0, 1, 2} with no two adjacent (a head spans 2 units)
  const int qa = starts & 1 ? 0 : starts & 2 ? 1 : 2;
  ua = k0 + (uint32_t)qa;
  ub = k0 + 2;
  const uint64_t dq0 = docid_at(0), dq1 = docid_at(1), dq2 = docid_at(2);
  da = qa == 0 ? dq0 : qa == 1 ? dq1 : dq2;
  db = dq2;
  return (uint32_t)__popc(starts);
}

template <int MODE, int G0>
__device__ void probe_by_cand_hash(const DevPlan *__restrict__ pl, const ProbeWork &w, const DevList &L,
                                   const uint64_t *cand, const Counters *ctr, const uint64_t *dir, HashLds<G0> &S,
                                   const ProbeOut &po, int lane) {
  static_assert(G0 >= 1 && G0 <= HPATH_G0, "table path arrays");
  const uint8_t *lp = L.p;
  const uint32_t last_u0 = w.u0 + ((w.u1 - w.u0 - 1) / WCH_UNITS) * WCH_UNITS;
  WChunk cA, cB;
  constexpr bool FULL = MODE == 0 || MODE >= 5;
  uint32_t nk[G0], lo[G0];
  uint64_t base[G0], cur[G0], nxt[G0];
  const uint64_t dfirst = !FULL ? 0 : w.has_dfirst ? w.dfirst : first_run_doc(L, w.u0, w.u1, lane);
  auto cload = [&](int k, uint32_t i) -> uint64_t {  // candidate i of array k (clamped; validity at use)
    return cand[base[k] + min(i, max(nk[k], 1u) - 1)];
  };
  const int g0n = G0 <= 2 ? G0 : pl->g0n;
#pragma unroll
  for (int k = 0; k < G0; k++) {
    nk[k] = k < g0n ? ctr->g0count[k] : 0;
    base[k] = k < g0n ? pl->g0base[k] : 0;
    lo[k] = FULL && k < g0n ? wave_start_dir(pl, k, cand + base[k], nk[k], dir, dfirst, lane) : 0;
    cur[k] = cload(k, lo[k] + lane);
    nxt[k] = cload(k, lo[k] + 64 + lane);
  }
  wchunk_fetch(lp, w.u0, lane, cA);
  wchunk_fetch(lp, min(w.u0 + WCH_UNITS, last_u0), lane, cB);
  uint32_t nbuf = 0;
  uint64_t pend_slot = ~0ull;  // slot whose run length waits for the next run start
  uint32_t pend_u = 0;
  uint32_t tag = 0;  // table generation (10 bits; tables cleared when it wraps)
  const uint64_t above = ~((2ull << lane) - 1);  // lanes after this one
  auto step = [&](const WChunk &c, uint32_t u0) {
    if (MODE == 2) {
      if (c.v[0].x == 0x557713eeu && c.v[1].y == 7u && c.v[2].z == 3u) po.bits[0] = 1;
      return;
    }
    // 1. run starts, in registers
    uint64_t da[WPIECES], db[WPIECES];
    uint32_t ua[WPIECES], ub[WPIECES], rc[WPIECES];
    uint64_t mk[WPIECES];
#pragma unroll
    for (int i = 0; i < WPIECES; i++) {
      rc[i] = piece_starts(c, i, u0, w.u1, lane, da[i], db[i], ua[i], ub[i]);
      mk[i] = __ballot(rc[i] != 0);
    }
    // the chunk's first and last run start; F[i]: first start unit of pieces >= i
    uint32_t F[WPIECES + 1];
    F[WPIECES] = 0xffffffffu;
    uint64_t dlo = ~0ull, dhi = 0;
#pragma unroll
    for (int i = WPIECES - 1; i >= 0; i--) {
      F[i] = F[i + 1];
      if (mk[i]) {
        const int f = __ffsll((unsigned long long)mk[i]) - 1;
        F[i] = __builtin_amdgcn_readlane(ua[i], f);
        const uint32_t dl = __builtin_amdgcn_readlane((uint32_t)da[i], f);
        const uint32_t dh = __builtin_amdgcn_readlane((uint32_t)(da[i] >> 32), f);
        dlo = ((uint64_t)dh << 32) | dl;
      }
    }
#pragma unroll
    for (int i = 0; i < WPIECES; i++) {
      if (mk[i]) {
        const int h = 63 - __builtin_clzll((unsigned long long)mk[i]);
        const uint64_t x = rc[i] == 2 ? db[i] : da[i];
        const uint32_t dl = __builtin_amdgcn_readlane((uint32_t)x, h);
        const uint32_t dh = __builtin_amdgcn_readlane((uint32_t)(x >> 32), h);
        dhi = ((uint64_t)dh << 32) | dl;
      }
    }
    if (F[0] == 0xffffffffu) return;  // no run starts here: nothing consumed, the pending run goes on
    if (pend_slot != ~0ull) {
      if (nbuf + 1 > MBUF) mbuf_flush(S, nbuf, po, lane);
      mbuf_push(S, nbuf, lane == 0, (uint32_t)pend_slot, pend_u, u0 + F[0] - pend_u, lane);
      pend_slot = ~0ull;
    }
    if (MODE == 1) {
      if (dlo == 0x123456789ull) po.bits[0] = 1;
      return;
    }
    // 2. where each start's run ends (chunk-relative unit; ~0: the next chunk)
    uint32_t ea[WPIECES], eb[WPIECES];
#pragma unroll
    for (int i = 0; i < WPIECES; i++) {
      const uint64_t ab = mk[i] & above;
      const int j = ab ? __ffsll((unsigned long long)ab) - 1 : lane;
      const uint32_t nj = (uint32_t)__builtin_amdgcn_ds_bpermute(j << 2, (int)ua[i]);
      const uint32_t nx = ab ? nj : F[i + 1];
      ea[i] = rc[i] == 2 ? ub[i] : nx;
      eb[i] = nx;
    }
    // 3. the arrays' windows into their tables, then every start looks its
    // docid up, array by array; rounds repeat only while a window is used up
    // inside the chunk (dense arrays), a start staying undecided while its
    // docid lies beyond a used-up window of an array it has not yet matched
    static_assert(HB == 512, "9-bit bucket index");
    const uint64_t span = dhi - dlo;
    const uint32_t sh = span >= (uint64_t)HB ? 64u - (uint32_t)__builtin_clzll(span) - 9u : 0u;  // (dhi-dlo) >> sh < HB
    uint32_t und = 0;  // bit 2i+q: start q of piece i undecided
#pragma unroll
    for (int i = 0; i < WPIECES; i++) und |= (rc[i] >= 1 ? 1u : 0u) << (2 * i) | (rc[i] == 2 ? 2u : 0u) << (2 * i);
    for (;;) {
      if (++tag == 1024) {
        tag = 1;
#pragma unroll
        for (int k = 0; k < G0; k++)
          for (int q = lane; q < HB; q += 64) S.tab[k][q] = 0;
      }
      uint64_t wmax[G0];
      bool full[G0];
#pragma unroll
      for (int k = 0; k < G0; k++) {
        const bool valid = lo[k] + lane < nk[k];
        const uint64_t cd = valid ? cur[k] : ~0ull;
        const bool ins = valid && cd >= dlo && cd <= dhi;
        const uint32_t bk = ins ? (uint32_t)((cd - dlo) >> sh) : 0xffffffffu;
        const uint32_t bp = lane_prev(bk, 0xfffffffeu);
        if (ins && bp != bk) S.tab[k][bk] = (uint16_t)(tag << 6 | (uint32_t)lane);
        S.win[k][lane] = cd;
        // (readlane returns int: each half through uint32_t, no sign extension)
        const uint32_t wlh = (uint32_t)__builtin_amdgcn_readlane((uint32_t)(cur[k] >> 32), 63);
        const uint32_t wll = (uint32_t)__builtin_amdgcn_readlane((uint32_t)cur[k], 63);
        const uint64_t wl = (uint64_t)wlh << 32 | wll;
        full[k] = lo[k] + 64 <= nk[k] && wl <= dhi;  // the whole window lies in the chunk
        wmax[k] = full[k] ? wl : ~0ull;
      }
      wave_lds_sync();
      // lookups: start (i, q) of this lane
      uint32_t hitk[2 * WPIECES], hitl[2 * WPIECES];
#pragma unroll
      for (int x = 0; x < 2 * WPIECES; x++) {
        const int i = x >> 1, q = x & 1;
        hitk[x] = 0xffu;
        hitl[x] = 0;
        if (!(und >> x & 1)) continue;
        const uint64_t d = q ? db[i] : da[i];
        const uint32_t bk = (uint32_t)((d - dlo) >> sh);
        bool decided = true;
#pragma unroll
        for (int k = 0; k < G0; k++) {
          if (k >= G0 || hitk[x] != 0xffu) break;
          if (d > wmax[k]) {
            decided = false;
            break;
          }
          const uint32_t e = S.tab[k][bk];
          if ((e >> 6) != tag) continue;
          uint32_t l = e & 63;
          for (; l < 64; l++) {
            const uint64_t cd = S.win[k][l];
            if (cd >= d) {
              if (cd == d) {
                hitk[x] = (uint32_t)k;
                hitl[x] = l;
              }
              break;
            }
          }
        }
        if (decided) und &= ~(1u << x);
        if (pl->dbg_doc && d == pl->dbg_doc && pl->dbg_buf) {
          // diagnostic (GBGPU_PROBE_DEBUG_DOC): up to 32 records of 16 words
          const uint32_t o = atomicAdd(reinterpret_cast<uint32_t *>(pl->dbg_buf), 1u);
          if (o < 32) {
            unsigned long long *r = pl->dbg_buf + 1 + 16 * o;
            r[0] = po.l, r[1] = u0, r[2] = (uint32_t)x, r[3] = (uint32_t)lane, r[4] = dlo, r[5] = dhi, r[6] = sh;
            r[7] = bk, r[8] = tag, r[9] = bk < HB ? S.tab[0][bk] : 0xdead, r[10] = S.win[0][0], r[11] = S.win[0][63];
            r[12] = lo[0], r[13] = nk[0], r[14] = (uint32_t)full[0] | (decided ? 2u : 0u), r[15] = hitk[x] << 8 | hitl[x];
          }
        }
      }
      // 4. matches into the buffer (a run ending past the chunk waits)
#pragma unroll
      for (int x = 0; x < 2 * WPIECES; x++) {
        const int i = x >> 1, q = x & 1;
        const bool hit = hitk[x] != 0xffu;
        if (!__ballot(hit)) continue;
        uint64_t slot = 0;
#pragma unroll
        for (int k = 0; k < G0; k++)
          if (hitk[x] == (uint32_t)k) slot = base[k] + lo[k] + hitl[x];
        const uint32_t us = q ? ub[i] : ua[i], ue = q ? eb[i] : ea[i];
        const bool last = hit && ue == 0xffffffffu;
        if (nbuf + 64 > MBUF) mbuf_flush(S, nbuf, po, lane);
        mbuf_push(S, nbuf, hit && !last, (uint32_t)slot, u0 + us, ue - us, lane);
        const uint64_t pm = __ballot(last);
        if (pm) {
          const int f = __ffsll((unsigned long long)pm) - 1;
          pend_slot = __shfl(slot, f, 64);
          pend_u = u0 + __shfl(us, f, 64);
        }
      }
      // 5. consumption: a used-up window moves on by 64 and the chunk goes
      // round again; the others wait for the last round
      bool again = false;
#pragma unroll
      for (int k = 0; k < G0; k++) {
        if (full[k]) {
          again = true;
          lo[k] += 64;
          cur[k] = nxt[k];
          nxt[k] = cload(k, lo[k] + 64 + lane);
        }
      }
      if (!again) break;
      wave_lds_sync();  // the next round rewrites the tables
    }
#pragma unroll
    for (int k = 0; k < G0; k++) {
      const bool valid = lo[k] + lane < nk[k];
      const uint32_t used = (uint32_t)__popcll(__ballot(valid && cur[k] <= dhi));
      // the next window: 64 - used candidates left in cur, the rest from nxt
      const int sl = (lane + (int)used) & 63;
      const uint64_t a2 = __shfl(cur[k], sl, 64), b2 = __shfl(nxt[k], sl, 64);
      cur[k] = lane + used < 64u ? a2 : b2;
      lo[k] += used;
      nxt[k] = cload(k, lo[k] + 64 + lane);
    }
    wave_lds_sync();  // the next chunk rewrites the tables
  };
  const uint32_t nch = (w.u1 - w.u0 + WCH_UNITS - 1) / WCH_UNITS;
  uint32_t u0 = w.u0;
  for (uint32_t it = 0; it + 2 <= nch; it += 2, u0 += 2 * WCH_UNITS) {
    step(cA, u0);
    wchunk_fetch(lp, min(u0 + 2 * WCH_UNITS, last_u0), lane, cA);
    __builtin_amdgcn_sched_barrier(0);
    step(cB, u0 + WCH_UNITS);
    wchunk_fetch(lp, min(u0 + 3 * WCH_UNITS, last_u0), lane, cB);
    __builtin_amdgcn_sched_barrier(0);
  }
  if (nch & 1) step(cA, u0);
  if (pend_slot != ~0ull) {
    const uint32_t len = lane == 0 ? run_end(L, pend_u + 2) - pend_u : 0;
    if (nbuf + 1 > MBUF) mbuf_flush(S, nbuf, po, lane);
    mbuf_push(S, nbuf, lane == 0, (uint32_t)pend_slot, pend_u, len, lane);
  }
  mbuf_flush(S, nbuf, po, lane);
}

// Dense list, one or two candidate arrays (the common plan: a word and its
// bigram): probe_by_cand over 6 KiB chunks with 128-candidate windows (two
// per lane).  A wave's dependent chain per chunk -- run-start compaction,
// the run-list search, the settles -- is about as long for 6 KiB as for 3
// KiB (one more search step), so each chain covers twice the bytes; the
// lanes' two candidates search the run list interleaved.  The span starts at
// the host-known first run docid through the directory (wave_start_dir).
constexpr int WP6 = 6;                    // pieces (1 KiB wave loads) of a wide chunk
constexpr int W6_BYTES = WP6 * 1024;
constexpr int W6_UNITS = W6_BYTES / 6;    // 1024 units
constexpr int W6_RUNS = W6_UNITS / 2;     // a run is >= 2 units
static_assert(W6_BYTES % 6 == 0, "a wide chunk holds whole units");
struct WChunk6 {
  v4u v[WP6];
  uint2 nb;
};
struct ProbeLds6 {
  uint64_t doc[W6_RUNS];
  uint32_t mslot[MBUF], mu[MBUF], mlen[MBUF];
  uint16_t unit[W6_RUNS];
  uint8_t claim[W6_RUNS];
};
__device__ __forceinline__ void wchunk6_fetch(const uint8_t *list, uint32_t u0, int lane, WChunk6 &c) {
  const auto *src = glc<v4u>(list + (size_t)u0 * 6 + lane * 16);
#pragma unroll
  for (int i = 0; i < WP6; i++) c.v[i] = __builtin_nontemporal_load(src + i * 64);
  c.nb = make_uint2(0, 0);
  if (lane == 63) {
    typedef uint32_t v2 __attribute__((ext_vector_type(2)));
    const v2 t = *glc<v2>(list + (size_t)u0 * 6 + W6_BYTES);
    c.nb = make_uint2(t.x, t.y);
  }
}
// chunk_runs over WP6 pieces (its comment has the layout): the run starts of
// the chunk into S, sorted; returns their count
__device__ __forceinline__ uint32_t chunk6_runs(const WChunk6 &cur, uint32_t u0, uint32_t u1, int lane, ProbeLds6 &S) {
  const uint64_t lt = (1ull << lane) - 1;
  uint32_t nrun = 0;
#pragma unroll
  for (int i = 0; i < WP6; i++) {
    uint32_t r[7];
    r[0] = cur.v[i].x;
    r[1] = cur.v[i].y;
    r[2] = cur.v[i].z;
    r[3] = cur.v[i].w;
    uint32_t e0, e1, e2;  // lane 63: the next piece's first bytes, or the bytes after the chunk
    if (i + 1 < WP6) {
      e0 = __builtin_amdgcn_readfirstlane(cur.v[i + 1].x);
      e1 = __builtin_amdgcn_readfirstlane(cur.v[i + 1].y);
      e2 = __builtin_amdgcn_readfirstlane(cur.v[i + 1].z);
    } else {
      e0 = cur.nb.x;
      e1 = cur.nb.y;
      e2 = 0;
    }
    r[4] = lane_next(r[0], e0);
    r[5] = lane_next(r[1], e1);
    r[6] = lane_next(r[2], e2);
    const uint32_t P = (uint32_t)i * 1024 + (uint32_t)lane * 16;
    const uint32_t k0 = (P + 5) / 6;  // first unit starting in [P, P + 16)
    const uint32_t o0 = k0 * 6 - P;
    uint32_t a[6];
#pragma unroll
    for (int j = 0; j < 6; j++) a[j] = o0 == 4 ? r[j + 1] : __builtin_amdgcn_alignbyte(r[j + 1], r[j], o0);
    auto byte = [&](int b) -> uint32_t { return (a[b >> 2] >> ((b & 3) * 8)) & 0xff; };
    uint32_t starts = 0;
#pragma unroll
    for (int q = 0; q < 3; q++) {
      const bool in = 6 * q + o0 < 16 && u0 + k0 + q < u1;
      if (in && (byte(6 * q + 1) & 0x02) && !(byte(6 * q) & 0x04)) starts |= 1u << q;
    }
    const uint32_t cnt = __popc(starts);  // <= 2: a run head spans two units
    const uint64_t b0 = __ballot(cnt & 1), b1 = __ballot(cnt & 2);
    uint32_t o = nrun + (uint32_t)(__popcll(b0 & lt) + 2 * __popcll(b1 & lt));
#pragma unroll
    for (int q = 0; q < 3; q++) {
      if (!(starts >> q & 1)) continue;
      uint64_t d = 0;
#pragma unroll
      for (int b = 4; b >= 0; b--) d = (d << 8) | byte(6 * q + 7 + b);
      S.doc[o] = d >> 2;
      S.unit[o] = (uint16_t)(k0 + q);
      S.claim[o] = 0;
      o++;
    }
    nrun += (uint32_t)(__popcll(b0) + 2 * __popcll(b1));
  }
  wave_lds_sync();
  return nrun;
}

template <int MODE, int G0>
__device__ void probe_by_cand_wide(const DevPlan *__restrict__ pl, const ProbeWork &w, const DevList &L, const uint64_t *cand,
                                   const Counters *ctr, const uint64_t *dir, ProbeLds6 &S, const ProbeOut &po, int lane) {
  static_assert(G0 >= 1 && G0 <= 2, "wide path arrays");
  const uint8_t *lp = L.p;
  const uint32_t last_u0 = w.u0 + ((w.u1 - w.u0 - 1) / W6_UNITS) * W6_UNITS;
  constexpr bool FULL = MODE == 0 || MODE == 5;
  uint32_t nk[G0], lo[G0];
  uint64_t base[G0];
  uint64_t ca[G0], cb[G0], na[G0], nb2[G0];  // candidates lo + lane, lo + 64 + lane, then + 128, + 192
  const uint64_t dfirst = !FULL ? 0 : w.has_dfirst ? w.dfirst : first_run_doc(L, w.u0, w.u1, lane);
  auto cload = [&](int k, uint32_t i) -> uint64_t {  // candidate i of array k (clamped; validity at use)
    return cand[base[k] + min(i, max(nk[k], 1u) - 1)];
  };
#pragma unroll
  for (int k = 0; k < G0; k++) {
    nk[k] = ctr->g0count[k];
    base[k] = pl->g0base[k];
    lo[k] = FULL ? wave_start_dir(pl, k, cand + base[k], nk[k], dir, dfirst, lane) : 0;
    ca[k] = cload(k, lo[k] + lane);
    cb[k] = cload(k, lo[k] + 64 + lane);
    na[k] = cload(k, lo[k] + 128 + lane);
    nb2[k] = cload(k, lo[k] + 192 + lane);
  }
  WChunk6 cA, cB;
  wchunk6_fetch(lp, w.u0, lane, cA);
  wchunk6_fetch(lp, min(w.u0 + W6_UNITS, last_u0), lane, cB);
  uint32_t nbuf = 0;
  uint64_t pend_slot = ~0ull;  // slot whose run length waits for the next run start
  uint32_t pend_u = 0;
  auto step = [&](const WChunk6 &c, uint32_t u0) {
    if (MODE == 2) {
      if (c.v[0].x == 0x557713eeu && c.v[1].y == 7u && c.v[2].z == 3u) po.bits[0] = 1;
      return;
    }
    const uint32_t nrun = chunk6_runs(c, u0, w.u1, lane, S);
    if (nrun && pend_slot != ~0ull) {
      if (nbuf + 1 > MBUF) mbuf_flush(S, nbuf, po, lane);
      mbuf_push(S, nbuf, lane == 0, (uint32_t)pend_slot, pend_u, u0 + S.unit[0] - pend_u, lane);
      pend_slot = ~0ull;
    }
    if (MODE == 1) {
      if (nrun && S.doc[0] == 0x123456789ull) po.bits[0] = 1;
      wave_lds_sync();
      return;
    }
    if (!nrun) return;  // nothing consumed; the pending run goes on
    const uint64_t dmax = S.doc[nrun - 1];
    auto search = [&](uint64_t d) -> uint32_t {
      uint32_t a = 0;
#pragma unroll
      for (uint32_t st = W6_RUNS; st > 0; st >>= 1) {
        const uint32_t t = a + st;
        const uint64_t v = S.doc[min(t, nrun) - 1];
        if (t <= nrun && v < d) a = t;
      }
      return a;
    };
    // candidate d (slot `slot`) against the runs; a its lower bound there
    auto settle = [&](uint64_t d, uint32_t a, uint64_t slot) -> bool {
      const bool in = d <= dmax;
      bool hit = false, last = false;
      uint32_t u = 0, len = 0;
      if (in && a < nrun && S.doc[a] == d && !S.claim[a]) {
        S.claim[a] = 1;
        u = u0 + S.unit[a];
        if (a + 1 < nrun) {
          hit = true;
          len = S.unit[a + 1] - S.unit[a];
        } else {
          last = true;  // ends at the next chunk's first run start
        }
      }
      if (nbuf + 64 > MBUF) mbuf_flush(S, nbuf, po, lane);
      mbuf_push(S, nbuf, hit, (uint32_t)slot, u, len, lane);
      const uint64_t pm = __ballot(last);
      if (pm) {
        const int f = __ffsll((unsigned long long)pm) - 1;
        pend_slot = __shfl(slot, f, 64);
        pend_u = u0 + S.unit[nrun - 1];
      }
      return in;
    };
    // every array's two windows searched at once (eight independent LDS
    // round trips a step); claims settled array by array, in order
    uint64_t d0[G0], d1[G0];
    uint32_t a0[G0], a1[G0];
#pragma unroll
    for (int k = 0; k < G0; k++) {
      d0[k] = lo[k] + lane < nk[k] ? ca[k] : ~0ull;
      d1[k] = lo[k] + 64 + lane < nk[k] ? cb[k] : ~0ull;
      a0[k] = a1[k] = 0;
    }
#pragma unroll
    for (uint32_t st = W6_RUNS; st > 0; st >>= 1) {
#pragma unroll
      for (int k = 0; k < G0; k++) {
        const uint32_t t0 = a0[k] + st, t1 = a1[k] + st;
        const uint64_t v0 = S.doc[min(t0, nrun) - 1], v1 = S.doc[min(t1, nrun) - 1];
        if (t0 <= nrun && v0 < d0[k]) a0[k] = t0;
        if (t1 <= nrun && v1 < d1[k]) a1[k] = t1;
      }
    }
#pragma unroll
    for (int k = 0; k < G0; k++) {
      const bool in0 = settle(d0[k], a0[k], base[k] + lo[k] + lane);
      const bool in1 = settle(d1[k], a1[k], base[k] + lo[k] + 64 + lane);
      const uint32_t used = (uint32_t)__popcll(__ballot(in0)) + (uint32_t)__popcll(__ballot(in1));
      if (used < 128u) {
        // the next windows: 128 - used candidates left in ca/cb, then na/nb2
        const uint32_t r0 = used + (uint32_t)lane, r1 = r0 + 64;
        const int s0 = (int)(r0 & 63);
        const uint64_t xa = __shfl(ca[k], s0, 64), xb = __shfl(cb[k], s0, 64), xc = __shfl(na[k], s0, 64),
                       xd = __shfl(nb2[k], s0, 64);
        const uint32_t q0 = r0 >> 6, q1 = r1 >> 6;  // source window of each: 0 ca, 1 cb, 2 na, 3 nb2
        ca[k] = q0 == 0 ? xa : q0 == 1 ? xb : xc;
        cb[k] = q1 == 1 ? xb : q1 == 2 ? xc : xd;
        lo[k] += used;
        na[k] = cload(k, lo[k] + 128 + lane);  // used one chunk later
        nb2[k] = cload(k, lo[k] + 192 + lane);
      } else {
        // a chunk meeting more than 128 candidates (dense arrays): the rest
        // 64 at a time, each window loaded and waited for at once
        lo[k] += 128;
        for (;;) {
          const uint64_t d = lo[k] + lane < nk[k] ? cand[base[k] + lo[k] + lane] : ~0ull;
          const bool in = settle(d, search(d), base[k] + lo[k] + lane);
          const uint32_t u = (uint32_t)__popcll(__ballot(in));
          lo[k] += u;
          if (u < 64u) break;
        }
        ca[k] = cload(k, lo[k] + lane);
        cb[k] = cload(k, lo[k] + 64 + lane);
        na[k] = cload(k, lo[k] + 128 + lane);
        nb2[k] = cload(k, lo[k] + 192 + lane);
        // all used here, so the merge with the usual path leaves no load of
        // them pending (the waitcnt pass would then wait for everything)
        __asm__ volatile("" ::"v"(ca[k]), "v"(cb[k]), "v"(na[k]), "v"(nb2[k]));
      }
    }
    wave_lds_sync();  // the next chunk rewrites the run list
  };
  const uint32_t nch = (w.u1 - w.u0 + W6_UNITS - 1) / W6_UNITS;
  uint32_t u0 = w.u0;
  for (uint32_t it = 0; it + 2 <= nch; it += 2, u0 += 2 * W6_UNITS) {
    step(cA, u0);
    wchunk6_fetch(lp, min(u0 + 2 * W6_UNITS, last_u0), lane, cA);
    __builtin_amdgcn_sched_barrier(0);
    step(cB, u0 + W6_UNITS);
    wchunk6_fetch(lp, min(u0 + 3 * W6_UNITS, last_u0), lane, cB);
    __builtin_amdgcn_sched_barrier(0);
  }
  if (nch & 1) step(cA, u0);
  if (pend_slot != ~0ull) {
    const uint32_t len = lane == 0 ? run_end(L, pend_u + 2) - pend_u : 0;
    if (nbuf + 1 > MBUF) mbuf_flush(S, nbuf, po, lane);
    mbuf_push(S, nbuf, lane == 0, (uint32_t)pend_slot, pend_u, len, lane);
  }
  mbuf_flush(S, nbuf, po, lane);
}

#endif  // GBGPU_DIAG

// Dense list: probe_by_cand with fewer LDS and vector instructions a chunk,
// the measured limit of that path (its LDS pipe and VALU issue, not its HBM
// bytes: a 6 KiB-chunk variant with the same work per byte ran no faster).
//   * a run start is ONE 64-bit LDS word, docid << 16 | unit: the search
//     compares it with d << 16 (the unit bits cannot reorder docids), a hit
//     reads the unit from it and the run's end from the next word (one
//     ds_read2), so classification writes one word a start, not three;
//   * the lane shifts of the classification are DPP moves (lane_next) and
//     the next piece's first bytes scalar reads, not bpermutes;
//   * claims (a docid goes to the first array holding it) are one bit a run,
//     cleared with one store a chunk, and only with several arrays;
//   * the span starts at the host-known first run docid (wave_start_dir).
struct ProbeLdsP {
  uint64_t rk[WMAX_RUNS];             // run starts: docid << 16 | unit in the chunk
  uint32_t cbits[WMAX_RUNS / 32];     // claimed runs
  uint32_t mslot[MBUF], mu[MBUF], mlen[MBUF];
};
__device__ __forceinline__ uint32_t chunk_runs_packed(const WChunk12 &cur, uint32_t u0, uint32_t u1, int lane, ProbeLdsP &S) {
  const uint64_t lt = (1ull << lane) - 1;
  uint32_t nrun = 0;
#pragma unroll
  for (int i = 0; i < W12_PIECES; i++) {
    const uint32_t d0 = cur.v[i].x, d1 = cur.v[i].y, d2 = cur.v[i].z;
    uint32_t e0, e1;  // lane 63: the next piece's first bytes, or the bytes after the chunk
    if (i + 1 < W12_PIECES) {
      e0 = __builtin_amdgcn_readfirstlane(cur.v[i + 1].x);
      e1 = __builtin_amdgcn_readfirstlane(cur.v[i + 1].y);
    } else {
      e0 = cur.nb.x;
      e1 = cur.nb.y;
    }
    const uint32_t n0 = lane_next(d0, e0), n1 = lane_next(d1, e1);  // the next lane's unit
    const uint32_t k0 = (uint32_t)i * 128 + (uint32_t)lane * 2;     // the lane's first unit
    // unit k0: flag bytes 0-1 = d0 bits 0-15; unit k0+1: bytes 6-7 = d1 bits 16-31
    const bool s0 = (u0 + k0 < u1) & ((d0 & 0x200u) != 0) & !(d0 & 0x4u);
    const bool s1 = (u0 + k0 + 1 < u1) & ((d1 & 0x2000000u) != 0) & !(d1 & 0x40000u);
    // the head's docid, key bytes 7..11: d1.3 d2 (unit k0) or the next lane's
    // bytes 1..5 (unit k0+1)
    const uint32_t lo = s0 ? (d1 >> 24) | (d2 << 8) : (n0 >> 8) | (n1 << 24);
    const uint32_t hi = s0 ? d2 >> 24 : (n1 >> 8) & 0xffu;
    const uint64_t w = ((((uint64_t)hi << 32) | lo) >> 2) << 16 | (uint64_t)(k0 + (s0 ? 0u : 1u));
    const bool st = s0 | s1;
    const uint64_t b = __ballot(st);
    if (st) S.rk[nrun + (uint32_t)__popcll(b & lt)] = w;
    nrun += (uint32_t)__popcll(b);
  }
  // keys past the runs read as ~0 (above every candidate key): the search
  // needs no bounds test
  for (uint32_t x = nrun + (uint32_t)lane; x < WMAX_RUNS; x += 64) S.rk[x] = ~0ull;
  if (lane < WMAX_RUNS / 32) S.cbits[lane] = 0;
  wave_lds_sync();
  return nrun;
}

template <int MODE, int G0>
__device__ void probe_by_cand_packed(const DevPlan *__restrict__ pl, const ProbeWork &w, const DevList &L, const uint64_t *cand,
                                     const Counters *ctr, const uint64_t *dir, ProbeLdsP &S, const ProbeOut &po, int lane) {
  const int g0n = G0 <= 2 ? G0 : pl->g0n;
  const uint8_t *lp = L.p;
  uint32_t nk[G0], lok[G0];
  uint64_t base[G0], cur[G0], nxt[G0];
  const uint32_t last_u0 = w.u0 + ((w.u1 - w.u0 - 1) / WCH_UNITS) * WCH_UNITS;
  WChunk12 cA, cB, cC;  // three chunks in flight (9 KiB a wave)
  // a prefetch past the span (issued unconditionally, so every step waits
  // on a fixed load count) reads the list's first chunk, which every wave's
  // tail shares in L2, instead of its own last chunk again from HBM
  auto pre_u = [&](uint32_t u) -> uint32_t { return u <= last_u0 ? u : 0u; };
  constexpr bool FULL = MODE == 0 || MODE == 5;
  const uint64_t dfirst = !FULL ? 0 : w.has_dfirst ? w.dfirst : first_run_doc(L, w.u0, w.u1, lane);
  auto cload = [&](int k, uint32_t i) -> uint64_t {  // candidate i of array k (clamped; validity at use)
    return cand[base[k] + min(i, max(nk[k], 1u) - 1)];
  };
#pragma unroll
  for (int k = 0; k < G0; k++) {
    nk[k] = k < g0n ? ctr->g0count[k] : 0;
    base[k] = k < g0n ? pl->g0base[k] : 0;
    lok[k] = (FULL && k < g0n) ? wave_start_dir(pl, k, cand + base[k], nk[k], dir, dfirst, lane) : 0;
    cur[k] = cload(k, lok[k] + lane);
    nxt[k] = cload(k, lok[k] + 64 + lane);
  }
  wchunk12_fetch(lp, w.u0, lane, cA);
  wchunk12_fetch(lp, pre_u(w.u0 + WCH_UNITS), lane, cB);
  wchunk12_fetch(lp, pre_u(w.u0 + 2 * WCH_UNITS), lane, cC);
  uint32_t nbuf = 0;
  uint64_t pend_slot = ~0ull;  // slot whose run length waits for the next run start
  uint32_t pend_u = 0;
  auto step = [&](const WChunk12 &c, uint32_t u0) {
    if (MODE == 2) {  // every loaded word feeds the (never true) test: no load is dropped
      uint32_t x = 0;
#pragma unroll
      for (int i = 0; i < W12_PIECES; i++) x ^= c.v[i].x ^ (c.v[i].y * 3u) ^ (c.v[i].z * 5u);
      if (x == 0x557713eeu && c.nb.x == 7u) po.bits[0] = 1;
      return;
    }
    const uint32_t nrun = chunk_runs_packed(c, u0, w.u1, lane, S);
    if (nrun && pend_slot != ~0ull) {
      if (nbuf + 1 > MBUF) mbuf_flush(S, nbuf, po, lane);
      mbuf_push(S, nbuf, lane == 0, (uint32_t)pend_slot, pend_u, u0 + (uint32_t)(S.rk[0] & 0xffff) - pend_u, lane);
      pend_slot = ~0ull;
    }
    if (MODE == 1) {
      if (nrun && S.rk[0] == 0x123456789ull) po.bits[0] = 1;
      wave_lds_sync();
      return;
    }
    if (!nrun) return;  // nothing consumed; the pending run goes on
    const uint64_t kmax = S.rk[nrun - 1] | 0xffffull;  // above every key of the chunk's last docid
    uint64_t dk[G0];
    uint32_t pa[G0];
#pragma unroll
    for (int k = 0; k < G0; k++) {
      dk[k] = (k < g0n && lok[k] + lane < nk[k]) ? cur[k] << 16 : ~0ull;
      pa[k] = 0;
    }
    // branchless lower bound of d << 16 among the keys (padded with ~0 to
    // WMAX_RUNS), every array at once
#pragma unroll
    for (uint32_t st = WMAX_RUNS / 2; st > 0; st >>= 1) {
#pragma unroll
      for (int k = 0; k < G0; k++)
        if (S.rk[pa[k] + st - 1] < dk[k]) pa[k] += st;
    }
#pragma unroll
    for (int k = 0; k < G0; k++)
      if (S.rk[pa[k]] < dk[k]) pa[k]++;  // the last position (255 at most)
    auto settle = [&](int k, uint64_t dkey, uint32_t a, uint32_t lo) -> uint32_t {
      const bool in = dkey <= kmax;
      bool hit = false, last = false;
      uint32_t u = 0, len = 0;
      if (in && a < nrun) {
        const uint64_t v = S.rk[a], vn = S.rk[min(a + 1, nrun - 1)];
        const bool claimed = G0 > 1 && k > 0 && ((S.cbits[a >> 5] >> (a & 31)) & 1);
        if ((v >> 16) == (dkey >> 16) && !claimed) {
          if (G0 > 1 && k + 1 < g0n) atomicOr(&S.cbits[a >> 5], 1u << (a & 31));
          u = u0 + (uint32_t)(v & 0xffff);
          if (a + 1 < nrun) {
            hit = true;
            len = (uint32_t)(vn & 0xffff) - (uint32_t)(v & 0xffff);
          } else {
            last = true;  // ends at the next chunk's first run start
          }
        }
      }
      if (nbuf + 64 > MBUF) mbuf_flush(S, nbuf, po, lane);
      mbuf_push(S, nbuf, hit, (uint32_t)(base[k] + lo + lane), u, len, lane);
      const uint64_t pm = __ballot(last);
      if (pm) {
        pend_slot = base[k] + lo + (uint32_t)(__ffsll((unsigned long long)pm) - 1);
        pend_u = u0 + (uint32_t)(S.rk[nrun - 1] & 0xffff);
      }
      return (uint32_t)__popcll(__ballot(in));
    };
#pragma unroll
    for (int k = 0; k < G0; k++) {
      if (k >= g0n) break;
      uint32_t lo = lok[k];
      const uint32_t used = settle(k, dk[k], pa[k], lo);
      lo += used;
      if (used < 64u) {
        const int sl = (lane + (int)used) & 63;
        const uint64_t a2 = __shfl(cur[k], sl, 64), b2 = __shfl(nxt[k], sl, 64);
        cur[k] = lane + used < 64u ? a2 : b2;
        lok[k] = lo;
        nxt[k] = cload(k, lo + 64 + lane);  // used one chunk later
      } else {
        // a chunk meeting more than 64 candidates (dense arrays)
        for (;;) {
          const uint64_t d = lo + lane < nk[k] ? cand[base[k] + lo + lane] << 16 : ~0ull;
          uint32_t a = 0;
#pragma unroll
          for (uint32_t st = WMAX_RUNS / 2; st > 0; st >>= 1)
            if (S.rk[a + st - 1] < d) a += st;
          if (S.rk[a] < d) a++;
          const uint32_t u2 = settle(k, d, a, lo);
          lo += u2;
          if (u2 < 64u) break;
        }
        lok[k] = lo;
        cur[k] = cload(k, lo + lane);
        nxt[k] = cload(k, lo + 64 + lane);
        __asm__ volatile("" ::"v"(cur[k]), "v"(nxt[k]));
      }
    }
    wave_lds_sync();  // the next chunk rewrites the run list
  };
  const uint32_t nch = (w.u1 - w.u0 + WCH_UNITS - 1) / WCH_UNITS;
  uint32_t u0 = w.u0;
  // static buffer roles (the in-order vmcnt then waits exactly for the
  // chunk about to be classified)
  for (uint32_t it = 0; it + 3 <= nch; it += 3, u0 += 3 * WCH_UNITS) {
    step(cA, u0);
    wchunk12_fetch(lp, pre_u(u0 + 3 * WCH_UNITS), lane, cA);
    __builtin_amdgcn_sched_barrier(0);
    step(cB, u0 + WCH_UNITS);
    wchunk12_fetch(lp, pre_u(u0 + 4 * WCH_UNITS), lane, cB);
    __builtin_amdgcn_sched_barrier(0);
    step(cC, u0 + 2 * WCH_UNITS);
    wchunk12_fetch(lp, pre_u(u0 + 5 * WCH_UNITS), lane, cC);
    __builtin_amdgcn_sched_barrier(0);
  }
  const uint32_t rem = nch % 3;
  if (rem >= 1) step(cA, u0);
  if (rem == 2) step(cB, u0 + WCH_UNITS);
  if (pend_slot != ~0ull) {
    const uint32_t len = lane == 0 ? run_end(L, pend_u + 2) - pend_u : 0;
    if (nbuf + 1 > MBUF) mbuf_flush(S, nbuf, po, lane);
    mbuf_push(S, nbuf, lane == 0, (uint32_t)pend_slot, pend_u, len, lane);
  }
  mbuf_flush(S, nbuf, po, lane);
}

// Sparse list: each run start looks its docid up in the arrays, in order;
// the first array holding it takes the run.
template <int G0>
__device__ void probe_by_run(const DevPlan *__restrict__ pl, const ProbeWork &w, const DevList &L, const uint64_t *cand,
                             const Counters *ctr, const uint64_t *dir, ProbeLds &S, const ProbeOut &po, int lane) {
  const int g0n = G0 <= 2 ? G0 : pl->g0n;
  uint32_t nk[G0];
  uint64_t base[G0];
#pragma unroll
  for (int k = 0; k < G0; k++) {
    nk[k] = k < g0n ? ctr->g0count[k] : 0;
    base[k] = k < g0n ? pl->g0base[k] : 0;
  }
  uint32_t nbuf = 0;
  uint64_t pend_slot = ~0ull;
  uint32_t pend_u = 0;
  WChunk cur;
  for (uint32_t u0 = w.u0; u0 < w.u1; u0 += WCH_UNITS) {
    wchunk_fetch(L.p, u0, lane, cur);
    const uint32_t nrun = chunk_runs(cur, u0, w.u1, lane, S);
    if (!nrun) continue;
    if (pend_slot != ~0ull) {
      if (nbuf + 1 > MBUF) mbuf_flush(S, nbuf, po, lane);
      mbuf_push(S, nbuf, lane == 0, (uint32_t)pend_slot, pend_u, u0 + S.unit[0] - pend_u, lane);
      pend_slot = ~0ull;
    }
    for (uint32_t j0 = 0; j0 < nrun; j0 += 64) {
      const uint32_t j = j0 + lane;
      bool hit = false, last = false;
      uint32_t slot = 0, u = 0, len = 0;
      if (j < nrun) {
        const uint64_t d = S.doc[j];
        uint64_t e[G0];
#pragma unroll
        for (int k = 0; k < G0; k++) e[k] = k < g0n ? dir_entry(pl, k, nk[k], dir, d) : 0;
        int64_t i = -1;
        int kh = 0;
#pragma unroll
        for (int k = 0; k < G0; k++) {
          if (i >= 0 || k >= g0n) continue;
          i = cand_resolve(pl, e[k], cand + base[k], nk[k], d);
          kh = k;
        }
        if (i >= 0) {
          slot = (uint32_t)(base[kh] + (uint64_t)i);
          u = u0 + S.unit[j];
          if (j + 1 < nrun) {
            hit = true;
            len = S.unit[j + 1] - S.unit[j];
          } else {
            last = true;
          }
        }
      }
      if (nbuf + 64 > MBUF) mbuf_flush(S, nbuf, po, lane);
      mbuf_push(S, nbuf, hit, slot, u, len, lane);
      const uint64_t pm = __ballot(last);
      if (pm) {
        const int f = __ffsll((unsigned long long)pm) - 1;
        pend_slot = __shfl(slot, f, 64);
        pend_u = u0 + S.unit[nrun - 1];
      }
    }
    wave_lds_sync();
  }
  if (pend_slot != ~0ull) {
    const uint32_t len = lane == 0 ? run_end(L, pend_u + 2) - pend_u : 0;
    if (nbuf + 1 > MBUF) mbuf_flush(S, nbuf, po, lane);
    mbuf_push(S, nbuf, lane == 0, (uint32_t)pend_slot, pend_u, len, lane);
  }
  mbuf_flush(S, nbuf, po, lane);
}

// k_probe -- addDocIdVotes for groups g>0 and rmDocIdVotes (Posdb.cpp:5086-
// 5171, 4871-4946): one wave per work item, each wave alone (no block
// barrier).  The direction is per list (the host's choice, DevList::probe).
// MODE (diagnostic, GBGPU_PROBE_MODE): 0 full, 1 stop after the run-start
// compaction, 2 load chunks only, 3 skip the run-driven lists.
#ifndef GBGPU_PROBE_MINB
#define GBGPU_PROBE_MINB 1
#endif
template <int MODE, int G0>
__global__ void __launch_bounds__(64 * PW, (G0 <= 2 && MODE == 11) ? 3 : (G0 <= 2 ? GBGPU_PROBE_MINB : 1)) k_probe(const DevPlan *__restrict__ pl, const ProbeWork *work, uint32_t nwork,
                                                   const uint64_t *cand, uint32_t *bits, uint32_t nwords, Loc *loc,
                                                   const Counters *ctr, const uint64_t *dir) {
#ifdef GBGPU_DIAG
  // the bucket-table path (probe_by_cand_hash) is a measured alternative,
  // slower than the run-list search at config 2 (188 vs 80 us): diagnostic
  // GBGPU_PROBE_MODE=10 only
  constexpr bool HPATH = G0 <= HPATH_G0 && MODE == 10;
  // a wave runs one of the paths: their LDS overlaps
  constexpr bool WIDE = G0 <= 2 && MODE == 11;  // diagnostic: 6 KiB chunks (slower, see probe_by_cand_wide)
  constexpr bool PACKED = MODE == 0 || MODE == 1 || MODE == 2 || MODE == 5;
  struct None {
    uint8_t x;
  };
  union WaveLds {
    ProbeLds run;
    typename std::conditional<HPATH, HashLds<G0 <= HPATH_G0 ? G0 : 1>, None>::type hash;
    typename std::conditional<WIDE, ProbeLds6, None>::type wide;
    typename std::conditional<PACKED, ProbeLdsP, None>::type packed;
  };
#else
  static_assert(MODE == 0, "the release build has the full probe only");
  union WaveLds {
    ProbeLds run;
    ProbeLdsP packed;
  };
#endif
  __shared__ WaveLds s_w[PW];
  // the wave's index is uniform over the wave: said so, every value derived
  // from it (the work item, the list, the loop bounds) lives in SGPRs and the
  // chunk loop is a uniform one (no exec-mask loop, exact vmcnt waits)
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t wi = blockIdx.x * PW + wid;
  if (wi >= nwork) return;  // the whole wave: no block barrier follows
  ProbeWork w;
  if (wi < pl->nwork_cand) {
    w = work[wi];
  } else {
    const uint32_t i = wi - pl->nwork_cand;
    uint32_t sg = 0;
    while (sg + 1 < pl->nrseg && i >= pl->rseg_wbase[sg + 1]) sg++;
    w.list = pl->rseg_list[sg];
    w.u0 = (i - pl->rseg_wbase[sg]) * pl->run_span;
    w.u1 = min(pl->lists[w.list].units, w.u0 + pl->run_span);
    w.has_dfirst = 0;  // probe_by_run starts from the chunk's own run heads
    w.dfirst = ~0ull;
  }
  const DevList &L = pl->lists[w.list];
  ProbeOut po;
  po.bits = bits + (uint64_t)w.list * nwords;
  po.loc = loc;
  po.nl = (uint32_t)pl->nlists;
  po.l = w.list;
  po.on = MODE == 5 ? 0 : 1;
#ifdef GBGPU_DIAG
  if (L.probe == PROBE_BY_RUN) {
    if (MODE == 0 || MODE >= 10) probe_by_run<G0>(pl, w, L, cand, ctr, dir, s_w[wid].run, po, lane);
  } else {
    if constexpr (HPATH)
      probe_by_cand_hash<MODE, G0>(pl, w, L, cand, ctr, dir, s_w[wid].hash, po, lane);
    else if constexpr (WIDE)
      probe_by_cand_wide<0, G0 <= 2 ? G0 : 2>(pl, w, L, cand, ctr, dir, s_w[wid].wide, po, lane);
    else if constexpr (PACKED)
      probe_by_cand_packed<MODE, G0>(pl, w, L, cand, ctr, dir, s_w[wid].packed, po, lane);
    else
      probe_by_cand<(MODE == 3 || MODE == 12) ? 0 : MODE, G0>(pl, w, L, cand, ctr, dir, s_w[wid].run, po, lane);
  }
#else
  if (L.probe == PROBE_BY_RUN)
    probe_by_run<G0>(pl, w, L, cand, ctr, dir, s_w[wid].run, po, lane);
  else
    probe_by_cand_packed<0, G0>(pl, w, L, cand, ctr, dir, s_w[wid].packed, po, lane);
#endif
}

// A range term's list in a later group votes a docid only if a key of its
// run holds a number in range (Posdb.cpp:5115-5121): k_probe publishes every
// run it matches, and this pass (launched only for such queries) withdraws
// the out-of-range ones from the list's bitmap.  One thread per bitmap word
// (32 slots), so no atomics: the probe is over.
__global__ void k_range_filter(const DevPlan *__restrict__ pl, uint32_t rbits, uint32_t *bits, uint32_t nwords, const Loc *loc) {
  const uint32_t nl = (uint32_t)pl->nlists;
  for (uint32_t w = blockIdx.x * blockDim.x + threadIdx.x; w < nwords; w += gridDim.x * blockDim.x) {
    for (uint32_t rb = rbits; rb; rb &= rb - 1) {
      const int l = __ffs(rb) - 1;
      const DevList &L = pl->lists[l];
      uint32_t *bw = bits + (uint64_t)l * nwords + w;
      const uint32_t v = *bw;
      uint32_t keep = v;
      for (uint32_t x = v; x; x &= x - 1) {
        const uint64_t s = (uint64_t)w * 32 + (uint32_t)(__ffs(x) - 1);
        const Loc lc = loc[s * nl + l];
        if (lc.len < 2 || (uint64_t)lc.unit + lc.len > L.units || !run_in_range(L, lc.unit, lc.unit + lc.len))
          keep &= ~(1u << (s & 31));
      }
      if (keep != v) *bw = keep;
    }
  }
}

// ------------------------------------------------------------- compaction
// Survivors: candidates whose lists cover every positive group and no
// negative one (the final m_docIdVoteBuf, Posdb.cpp:5154-5171), plus the
// shrunk-sublist non-empty flags (shrinkSubLists, Posdb.cpp:5334-5428).
// A slot's list mask is its array's own list (array 0 only: a later array's
// slot is voted by its own list only through the probe, which credits a
// docid to the first array holding it) and its bits in the probe bitmaps.
//
// Two launches, CWORDS bitmap words (CTILE slots) a block of CB threads; the
// survivors are derived once:
//   k_cmp_count  a word a thread for the bit-parallel vote test, then the
//                block's survivors spread over all CB threads (each thread
//                waits on the run locations of about one survivor): their
//                count per size bucket, the lists with a run in some
//                survivor, the re-shrink partials (BlkInfo), and each
//                survivor's (slot, list mask, run units) staged in slot order
//                at the block's CTILE-slot place;
//   k_cmp_place  each block's offset in every bucket (the counts of the
//                blocks before it, 4 B a bucket a block) and the bucket
//                starts, then every staged survivor's record at its final
//                position -- buckets in order, slot order inside a bucket:
//                slot, list mask, run units, docid, and its run locations
//                ([pos][nl]), so k_score reads its survivors' data
//                contiguously.
// Survivors are counted by size (their run units, an upper bound on their
// records) so k_score can give each wave survivors of one size: a wave's
// lanes run the scorers in lockstep, so its time is its largest lane's.
// Bucket 0 holds the largest and is scored first.  Buckets 0, 1 and 2-4
// (more units than a lane's rc records) are scored 8, 16 and 32 to a wave,
// so each survivor gets 8, 4 or 2 lanes' worth of LDS records (size_bucket).  Site clustering
// (the TopTree replay walks survivors in docid order, Posdb.cpp:6137-6140)
// takes the same buckets plus each record's slot-order rank (sv_ord):
// k_bound writes the replay entries in slot order from it.

constexpr int CB = 256;            // compaction threads per block
constexpr int CSPT = 32;           // consecutive slots per bitmap word
#ifndef GBGPU_CWORDS
#define GBGPU_CWORDS 256
#endif
constexpr int CWORDS = GBGPU_CWORDS;  // bitmap words per block (threads 0..CWORDS-1 test them)
static_assert(CWORDS <= CB, "a word a thread");
constexpr int CTILE = CWORDS * CSPT;  // 8192 slots per block (one block scan: <= 2^16 per bucket)
static_assert(CTILE < 65536, "packed 16-bit bucket counts");
constexpr int XR = 4;              // re-shrunk lists reduced per block (more: global atomics)

struct BlkInfo {
  uint32_t cnt[NBKT];  // survivors per bucket
  uint32_t any, pad;   // lists with a run in some survivor of the block
  unsigned long long usum;       // the survivors' run units (their records' upper bound)
  unsigned long long dall;       // largest survivor docid (re-shrink queries)
  unsigned long long xu[XR];     // re-shrunk list r: its runs' units over the block's survivors
  unsigned long long xd[XR];     // ... and the last survivor docid with a run in it
};

// bit l: list l holds the docid of slot s (array a's slot)
__device__ __forceinline__ uint32_t slot_lmask(const DevPlan *__restrict__ pl, const uint32_t *bits, uint32_t nwords, uint64_t s,
                                               int a) {
  uint32_t lm = a == 0 ? 1u << pl->g0list[0] : 0u;
  for (uint32_t pm = pl->probed_mask; pm; pm &= pm - 1) {
    const int l = __ffs(pm) - 1;
    lm |= ((bits[(uint64_t)l * nwords + (s >> 5)] >> (s & 31)) & 1u) << l;
  }
  return lm;
}
// slot s's run in list l (l in its mask): array 0's own list from the
// candidates' run starts (a run ends where the next one starts), the others
// as k_probe recorded them
__device__ __forceinline__ Loc slot_loc(const DevPlan *__restrict__ pl, const Counters *ctr, const uint32_t *cunit, const Loc *loc,
                                        uint64_t s, int l) {
  if (l == pl->g0list[0] && s < pl->g0base[1]) {
    const uint32_t u = cunit[s];
    const uint32_t e = s + 1 < pl->g0base[0] + ctr->g0count[0] ? cunit[s + 1] : pl->lists[l].units;
    return Loc{u, e - u};
  }
  return loc[s * (uint32_t)pl->nlists + l];
}
// a docid survives when a list of every positive group and none of a
// negative group holds it: a loop over the (wave-uniform) groups' list masks
__device__ __forceinline__ bool lm_survives(const DevPlan *__restrict__ pl, uint32_t lm) {
  if (lm & pl->neg_lists) return false;
  for (uint32_t pm = pl->pos_mask; pm; pm &= pm - 1)
    if (!(lm & pl->group_lists[__ffs(pm) - 1])) return false;
  return true;
}
// array of slot s, or -1 past every array's written slots
__device__ __forceinline__ int slot_array(const DevPlan *__restrict__ pl, const Counters *ctr, uint64_t s) {
  int a = 0;
  while (a + 1 < pl->g0n && s >= pl->g0base[a + 1]) a++;
  return s - pl->g0base[a] < ctr->g0count[a] ? a : -1;
}
__device__ bool slot_is_survivor(const DevPlan *__restrict__ pl, const Counters *ctr, const uint32_t *bits, uint32_t nwords,
                                 uint64_t s, uint32_t *lm_out = nullptr) {
  const int a = slot_array(pl, ctr, s);
  if (a < 0) return false;
  if (pl->use_rej && pl->wrej[s]) return false;  // not voted (Posdb.cpp:5294, 5297)
  const uint32_t lm = slot_lmask(pl, bits, nwords, s, a);
  if (lm_out) *lm_out = lm;
  return lm_survives(pl, lm);
}
// arena units of slot s's records: each run once per positive group its
// list belongs to (a shared bigram sublist is merged into both groups); the
// lists are walked in a wave-uniform loop
__device__ uint32_t slot_units(const DevPlan *__restrict__ pl, const Counters *ctr, const uint32_t *cunit, const Loc *loc, uint64_t s,
                               uint32_t lm) {
  uint32_t u = 0;
  for (int l = 0; l < pl->nlists; l++)
    if (lm >> l & 1) u += slot_loc(pl, ctr, cunit, loc, s, l).len * (uint32_t)pl->list_mult[l];
  return u;
}

// bits q of a 32-slot word (first slot s0) with lo <= s0 + q < hi
__device__ __forceinline__ uint32_t range_bits(uint64_t s0, uint64_t lo, uint64_t hi) {
  if (hi <= lo || hi <= s0 || lo >= s0 + 32) return 0u;
  const uint32_t a = lo > s0 ? (uint32_t)(lo - s0) : 0u;
  const uint32_t b = hi < s0 + 32 ? (uint32_t)(hi - s0) : 32u;
  const uint32_t mb = b >= 32 ? 0xffffffffu : ((1u << b) - 1u);
  return mb & ~((1u << a) - 1u);
}

// One bitmap word's 32 slots, bit-parallel: the probed lists' bits, the
// slots of array 0 (whose own list is not probed: its bit is implied), and
// the survivors -- a written, voted slot whose lists hit every positive group
// and no negative one (Posdb.cpp:5154-5171, 4871-4946).
struct CmpWord {
  uint32_t bw[MAXL];
  uint32_t own0;
  uint32_t surv;
};
__device__ __forceinline__ void cmp_word(const DevPlan *__restrict__ pl, const Counters *ctr, const uint32_t *bits, uint32_t nwords,
                                         uint32_t w, CmpWord &c) {
  const uint64_t s0 = (uint64_t)w * 32;
  const uint32_t pm = pl->probed_mask;
#pragma unroll
  for (int l = 0; l < MAXL; l++) c.bw[l] = (pm >> l & 1) ? bits[(uint64_t)l * nwords + w] : 0u;
  uint32_t valid = 0;
  for (int a = 0; a < pl->g0n; a++) valid |= range_bits(s0, pl->g0base[a], pl->g0base[a] + ctr->g0count[a]);
  c.own0 = range_bits(s0, pl->g0base[0], pl->g0base[0] + ctr->g0count[0]);
  uint32_t surv = valid;
  if (pl->boolean) {
    // makeDocIdVoteBufForBoolQuery_r (Posdb.cpp:8026-8231): each slot's
    // QueryTermInfo bit vector from its lists (its canonical slot: any list
    // bit at all), kept where the truth table holds
    uint32_t gw[16];
#pragma unroll
    for (int g = 0; g < 16; g++) gw[g] = 0;
    const int l0 = pl->g0list[0];
    uint32_t any = 0;
#pragma unroll
    for (int l = 0; l < MAXL; l++) {
      const uint32_t lb = c.bw[l] | (l == l0 ? c.own0 : 0u);
      any |= lb;
      const uint32_t gm = l < pl->nlists ? pl->bool_gmask[l] : 0u;
#pragma unroll
      for (int g = 0; g < 16; g++)
        if (gm >> g & 1) gw[g] |= lb;
    }
    uint32_t pass = 0;
    for (uint32_t m = surv & any; m; m &= m - 1) {
      const int q = __ffs(m) - 1;
      uint32_t v = 0;
#pragma unroll
      for (int g = 0; g < 16; g++) v |= ((gw[g] >> q) & 1u) << g;
      if (pl->bool_table[v >> 3] >> (v & 7) & 1) pass |= 1u << q;
    }
    c.surv = pass;
    return;
  }
  if (surv && pl->use_rej) {  // not voted: whitelist / a range term's first group (k_write_runs)
    const v4u *r = reinterpret_cast<const v4u *>(pl->wrej + s0);
    const v4u r0 = r[0], r1 = r[1];
    const uint32_t wd[8] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w};
    uint32_t rej = 0;
#pragma unroll
    for (int i = 0; i < 32; i++) rej |= ((wd[i >> 2] >> ((i & 3) * 8)) & 0xffu) ? 1u << i : 0u;
    surv &= ~rej;
  }
  const uint32_t nm = pl->neg_lists;
#pragma unroll
  for (int l = 0; l < MAXL; l++)
    if (nm >> l & 1) surv &= ~c.bw[l];
  const int l0 = pl->g0list[0];
  for (uint32_t gm = pl->pos_mask; gm; gm &= gm - 1) {
    const uint32_t gl = pl->group_lists[__ffs(gm) - 1];
    uint32_t gh = (gl >> l0 & 1) ? c.own0 : 0u;
#pragma unroll
    for (int l = 0; l < MAXL; l++)
      if (gl >> l & 1) gh |= c.bw[l];
    surv &= gh;
  }
  c.surv = surv;
}
// slot s0 + q's list mask
__device__ __forceinline__ uint32_t cmp_lm(const DevPlan *__restrict__ pl, const CmpWord &c, int q) {
  uint32_t lm = (c.own0 >> q & 1) ? 1u << pl->g0list[0] : 0u;
#pragma unroll
  for (int l = 0; l < MAXL; l++) lm |= ((c.bw[l] >> q) & 1u) << l;
  return lm;
}
// the slot's run in list l (l in its mask): array 0's own list from the
// candidates' run starts (a run ends where the next one starts), the others
// as k_probe recorded them
__device__ __forceinline__ Loc cmp_loc(const DevPlan *__restrict__ pl, const Counters *ctr, const uint32_t *cunit, const Loc *loc,
                                       uint64_t s, int l, bool own) {
  if (own && l == pl->g0list[0]) {
    const uint32_t u = cunit[s];
    const uint32_t e = s + 1 < pl->g0base[0] + ctr->g0count[0] ? cunit[s + 1] : pl->lists[l].units;
    return Loc{u, e - u};
  }
  return loc[s * (uint32_t)pl->nlists + l];
}
// its record units: each run once per positive group its list belongs to
__device__ __forceinline__ uint32_t cmp_units(const DevPlan *__restrict__ pl, const Counters *ctr, const uint32_t *cunit,
                                              const Loc *loc, uint64_t s, uint32_t lm, bool own) {
  uint32_t u = 0;
  const uint32_t nl = (uint32_t)pl->nlists;
  const int l0 = pl->g0list[0];
  if (own) {
    const uint32_t u0 = cunit[s];
    const uint32_t e = s + 1 < pl->g0base[0] + ctr->g0count[0] ? cunit[s + 1] : pl->lists[l0].units;
    u += (e - u0) * (uint32_t)pl->list_mult[l0];
  }
  const uint32_t om = own ? lm & ~(1u << l0) : lm;
#pragma unroll
  for (int l = 0; l < MAXL; l++)
    if (om >> l & 1) u += loc[s * nl + l].len * (uint32_t)pl->list_mult[l];
  return u;
}

// Both passes stage the block's survivors (slot, list mask), in slot order,
// in LDS and then work on them one per thread, so every survivor's loads
// (run locations, docid) go out together instead of one thread walking its
// word's survivors serially.
constexpr int CSV = 2048;  // survivors staged per round
struct CmpStage {
  uint32_t slot[CSV];
  uint32_t lm[CSV];
};
// stage survivors [base, base + CSV) of the block (ex: this thread's first)
__device__ __forceinline__ void cmp_stage(const DevPlan *__restrict__ pl, const CmpWord &c, uint32_t w, uint32_t ex,
                                          uint32_t base, CmpStage &S) {
  const uint32_t n = __popc(c.surv);
  if (!n || ex >= base + CSV || ex + n <= base) return;
  uint32_t idx = ex;
  for (uint32_t sm = c.surv; sm; sm &= sm - 1, idx++) {
    if (idx < base || idx >= base + CSV) continue;
    const int q = __ffs(sm) - 1;
    S.slot[idx - base] = w * 32 + (uint32_t)q;
    S.lm[idx - base] = cmp_lm(pl, c, q);
  }
}

// Pass 1: per block of CTILE slots (one bitmap word a thread), the survivors
// per size bucket, the lists with a run in some survivor, the run units and
// the re-shrink partials.
__global__ void __launch_bounds__(CB) k_cmp_count(const DevPlan *__restrict__ pl, Counters *ctr,
                                                  const uint32_t *__restrict__ cunit, const uint32_t *__restrict__ bits,
                                                  uint32_t nwords, const Loc *__restrict__ loc,
                                                  const uint64_t *__restrict__ cand, uint32_t rc,
                                                  BlkInfo *__restrict__ blk, uint32_t *__restrict__ cnt8,
                                                  uint32_t *__restrict__ st_slot, uint32_t *__restrict__ st_lm,
                                                  uint32_t *__restrict__ st_u) {
  __shared__ CmpStage S;
  __shared__ uint32_t tmp[CB / 64];
  __shared__ uint32_t s_cnt[NBKT];
  __shared__ uint32_t s_any;
  __shared__ unsigned long long s_dall, s_usum, s_xu[XR], s_xd[XR];
  if (threadIdx.x < NBKT) s_cnt[threadIdx.x] = 0;
  if (threadIdx.x < XR) {
    s_xu[threadIdx.x] = 0;
    s_xd[threadIdx.x] = 0;
  }
  if (threadIdx.x == 0) {
    s_any = 0;
    s_dall = 0;
    s_usum = 0;
  }
  const uint32_t w = blockIdx.x * CWORDS + threadIdx.x;
  CmpWord c;
  c.surv = 0;
  if (threadIdx.x < CWORDS && w < nwords) cmp_word(pl, ctr, bits, nwords, w, c);
  uint32_t total;
  const uint32_t ex = block_exclusive_scan<CB>(__popc(c.surv), tmp, &total);
  const uint32_t xmask = pl->reshare_mask;
  uint32_t any = 0, usum = 0;
  unsigned long long tdall = 0, txu[XR] = {0, 0, 0, 0}, txd[XR] = {0, 0, 0, 0};
  for (uint32_t base = 0; base < total; base += CSV) {
    cmp_stage(pl, c, w, ex, base, S);
    __syncthreads();
    const uint32_t nr = min((uint32_t)CSV, total - base);
    for (uint32_t i = threadIdx.x; i < nr; i += CB) {
      const uint64_t s = S.slot[i];
      const uint32_t lm = S.lm[i];
      const bool own = (lm >> pl->g0list[0]) & 1;
      const uint32_t u = cmp_units(pl, ctr, cunit, loc, s, lm, own);
      atomicAdd(&s_cnt[size_bucket(u, rc)], 1u);
      // the block's survivors in slot order for k_cmp_place (block b's at
      // b * CTILE: a block holds at most its CTILE slots' survivors)
      const size_t si = (size_t)blockIdx.x * CTILE + base + i;
      st_slot[si] = (uint32_t)s;
      st_lm[si] = lm;
      st_u[si] = u;
      any |= lm;
      usum += u;
      if (xmask) {
        // re-shrunk lists (k_ext_walk): their survivor run units and last docid
        const unsigned long long d = cand[s];
        tdall = d > tdall ? d : tdall;
        int r = 0;
        for (uint32_t x = xmask; x; x &= x - 1, r++) {
          const int l = __ffs(x) - 1;
          if (!(lm >> l & 1)) continue;
          const uint32_t len = cmp_loc(pl, ctr, cunit, loc, s, l, own).len;
          if (r < XR) {
#pragma unroll
            for (int t = 0; t < XR; t++)
              if (t == r) {
                txu[t] += len;
                txd[t] = d > txd[t] ? d : txd[t];
              }
          } else {
            atomicAdd(&ctr->ext[l].units, (unsigned long long)len);
            atomicMax(&ctr->ext[l].dmax, d);
          }
        }
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    any |= __shfl_xor(any, off, 64);
    usum += __shfl_xor(usum, off, 64);
    if (xmask) {
      const unsigned long long o = __shfl_xor(tdall, off, 64);
      tdall = o > tdall ? o : tdall;
#pragma unroll
      for (int t = 0; t < XR; t++) {
        txu[t] += __shfl_xor(txu[t], off, 64);
        const unsigned long long od = __shfl_xor(txd[t], off, 64);
        txd[t] = od > txd[t] ? od : txd[t];
      }
    }
  }
  if ((threadIdx.x & 63) == 0) {
    if (any) atomicOr(&s_any, any);
    if (usum) atomicAdd(&s_usum, (unsigned long long)usum);
    if (xmask) {
      if (tdall) atomicMax(&s_dall, tdall);
#pragma unroll
      for (int t = 0; t < XR; t++)
        if (txu[t]) {
          atomicAdd(&s_xu[t], txu[t]);
          atomicMax(&s_xd[t], txd[t]);
        }
    }
  }
  __syncthreads();
  BlkInfo &o = blk[blockIdx.x];
  if (threadIdx.x < NBKT) {
    o.cnt[threadIdx.x] = s_cnt[threadIdx.x];
    cnt8[(size_t)blockIdx.x * NBKT + threadIdx.x] = s_cnt[threadIdx.x];
  }
  if (threadIdx.x < XR) {
    o.xu[threadIdx.x] = s_xu[threadIdx.x];
    o.xd[threadIdx.x] = s_xd[threadIdx.x];
  }
  if (threadIdx.x == 0) {
    o.any = s_any;
    o.pad = 0;
    o.usum = s_usum;
    o.dall = s_dall;
  }
}

// One block: each compaction block's offset in every bucket (the counts of
// the blocks before it), the bucket starts, and the totals -- counts, the
// list union, the run units, the re-shrink sums.
// Pass 2: every survivor's record at its final position -- buckets in
// order, slot order inside a bucket: slot, list mask, run units, docid, and
// its run locations ([pos][nl]), so k_score reads its survivors' data
// contiguously.  Each block sums the counts of the blocks before it (its
// offsets) and of all blocks (the bucket starts) from cnt8, 4 B a bucket a block;
// block 0 publishes the totals.  sv_ord (site clustering): each record's
// survivor's rank in slot order, where the replay wants it.
__global__ void __launch_bounds__(CB) k_cmp_place(const DevPlan *__restrict__ pl, Counters *__restrict__ ctr,
                                                  const uint32_t *__restrict__ cunit, const Loc *__restrict__ loc,
                                                  const uint64_t *__restrict__ cand, uint32_t rc,
                                                  const BlkInfo *__restrict__ blk, const uint32_t *__restrict__ cnt8,
                                                  uint32_t nblk, const uint32_t *__restrict__ st_slot,
                                                  const uint32_t *__restrict__ st_lm, const uint32_t *__restrict__ st_u,
                                                  uint32_t *__restrict__ sv_slot,
                                                  uint32_t *__restrict__ sv_lm, uint32_t *__restrict__ sv_u,
                                                  uint64_t *__restrict__ sv_doc, Loc *__restrict__ sv_loc,
                                                  uint32_t *__restrict__ sv_ord) {
  __shared__ uint32_t s_pre[NBKT], s_tot[NBKT], s_carry[NBKT];
  __shared__ uint32_t s_wc[CB / 64][NBKT];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (threadIdx.x < NBKT) {
    s_pre[threadIdx.x] = 0;
    s_tot[threadIdx.x] = 0;
    s_carry[threadIdx.x] = 0;
  }
  __syncthreads();
  {
    typedef uint32_t v4 __attribute__((ext_vector_type(4)));
    const v4 *c4 = reinterpret_cast<const v4 *>(cnt8);
    uint32_t pre[NBKT], tot[NBKT];
#pragma unroll
    for (int b = 0; b < NBKT; b++) pre[b] = tot[b] = 0;
    for (uint32_t i = threadIdx.x; i < nblk; i += CB) {
      uint32_t v[NBKT];
#pragma unroll
      for (int r = 0; r < NBKT / 4; r++) {
        const v4 a = c4[(NBKT / 4) * (size_t)i + r];
        v[4 * r] = a.x;
        v[4 * r + 1] = a.y;
        v[4 * r + 2] = a.z;
        v[4 * r + 3] = a.w;
      }
      const bool before = i < blockIdx.x;
#pragma unroll
      for (int b = 0; b < NBKT; b++) {
        tot[b] += v[b];
        pre[b] += before ? v[b] : 0u;
      }
    }
#pragma unroll
    for (int b = 0; b < NBKT; b++) {
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) {
        pre[b] += __shfl_xor(pre[b], off, 64);
        tot[b] += __shfl_xor(tot[b], off, 64);
      }
    }
    if (lane == 0) {
#pragma unroll
      for (int b = 0; b < NBKT; b++) {
        if (pre[b]) atomicAdd(&s_pre[b], pre[b]);
        if (tot[b]) atomicAdd(&s_tot[b], tot[b]);
      }
    }
  }
  if (blockIdx.x == 0) {
    // the totals: counts, bucket starts, list union, units, re-shrink sums
    uint32_t any = 0;
    unsigned long long usum = 0, dall = 0, xu[XR] = {0, 0, 0, 0}, xd[XR] = {0, 0, 0, 0};
    for (uint32_t i = threadIdx.x; i < nblk; i += CB) {
      const BlkInfo &bi = blk[i];
      any |= bi.any;
      usum += bi.usum;
      dall = bi.dall > dall ? bi.dall : dall;
#pragma unroll
      for (int t = 0; t < XR; t++) {
        xu[t] += bi.xu[t];
        xd[t] = bi.xd[t] > xd[t] ? bi.xd[t] : xd[t];
      }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      any |= __shfl_xor(any, off, 64);
      usum += __shfl_xor(usum, off, 64);
      const unsigned long long o = __shfl_xor(dall, off, 64);
      dall = o > dall ? o : dall;
#pragma unroll
      for (int t = 0; t < XR; t++) {
        xu[t] += __shfl_xor(xu[t], off, 64);
        const unsigned long long od = __shfl_xor(xd[t], off, 64);
        xd[t] = od > xd[t] ? od : xd[t];
      }
    }
    __shared__ uint32_t s_any;
    __shared__ unsigned long long s_usum, s_dall, s_xu[XR], s_xd[XR];
    if (threadIdx.x == 0) {
      s_any = 0;
      s_usum = 0;
      s_dall = 0;
    }
    if (threadIdx.x < XR) {
      s_xu[threadIdx.x] = 0;
      s_xd[threadIdx.x] = 0;
    }
    __syncthreads();
    if (lane == 0) {
      atomicOr(&s_any, any);
      atomicAdd(&s_usum, usum);
      atomicMax(&s_dall, dall);
#pragma unroll
      for (int t = 0; t < XR; t++) {
        atomicAdd(&s_xu[t], xu[t]);
        atomicMax(&s_xd[t], xd[t]);
      }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t acc = 0;
      for (int b = 0; b < NBKT; b++) {
        ctr->bstart[b] = acc;
        ctr->bcnt[b] = s_tot[b];
        acc += s_tot[b];
      }
      ctr->surv_top = ((unsigned long long)acc << 36) | (s_usum & ((1ull << 36) - 1));
      ctr->anysurv = s_any;
      ctr->dmax_all = s_dall;
      int r = 0;
      for (uint32_t x = pl->reshare_mask; x && r < XR; x &= x - 1, r++) {
        const int l = __ffs(x) - 1;
        ctr->ext[l].units += s_xu[r];
        if (s_xd[r] > ctr->ext[l].dmax) ctr->ext[l].dmax = s_xd[r];
      }
    }
  }
  __syncthreads();
  // each bucket's first position for this block: the bucket's start plus
  // the blocks before it
  __shared__ uint32_t s_base[NBKT];
  uint32_t ord0 = 0;  // survivors of the blocks before this one
  {
    uint32_t acc = 0;
#pragma unroll
    for (int b = 0; b < NBKT; b++) {
      if (threadIdx.x == b) s_base[b] = acc + s_pre[b];
      acc += s_tot[b];
      ord0 += s_pre[b];
    }
  }
  // this block's survivors (its row of counts), staged by k_cmp_count
  uint32_t total = 0;
#pragma unroll
  for (int b = 0; b < NBKT; b++) total += cnt8[(size_t)blockIdx.x * NBKT + b];
  const uint32_t nl = (uint32_t)pl->nlists;
  const int l0 = pl->g0list[0];
  const uint64_t lt = (1ull << lane) - 1;
  const size_t sb = (size_t)blockIdx.x * CTILE;
  {
    const uint32_t base = 0;
    const uint32_t nr = total;
    // in steps of CB survivors, in slot order: ranks inside each bucket
    for (uint32_t i0 = 0; i0 < nr; i0 += CB) {
      const uint32_t i = i0 + threadIdx.x;
      const bool act = i < nr;
      const uint64_t s = act ? st_slot[sb + i] : 0;
      const uint32_t lm = act ? st_lm[sb + i] : 0;
      const bool own = (lm >> l0) & 1;
      const uint32_t u = act ? st_u[sb + i] : 0;
      const uint32_t b = (uint32_t)size_bucket(u, rc);
      // the wave's lanes with the same bucket: 4 ballots on its bits; the
      // first of them writes their count
      static_assert(NBKT == 16, "four bucket bits");
      uint64_t peers = __ballot(act);
#pragma unroll
      for (int bit = 0; bit < 4; bit++) {
        const uint64_t m = __ballot((b >> bit) & 1u);
        peers &= ((b >> bit) & 1u) ? m : ~m;
      }
      const uint32_t rk = (uint32_t)__popcll(peers & lt);
      if (lane < NBKT) s_wc[wid][lane] = 0;
      if (act && rk == 0) s_wc[wid][b] = (uint32_t)__popcll(peers);
      __syncthreads();
      if (act) {
        uint32_t pos = s_base[b] + s_carry[b] + rk;
        for (int w2 = 0; w2 < wid; w2++) pos += s_wc[w2][b];
        sv_slot[pos] = (uint32_t)s;
        sv_lm[pos] = lm;
        sv_u[pos] = u;
        sv_doc[pos] = cand[s];
        if (sv_ord) sv_ord[pos] = ord0 + base + i;
        for (uint32_t xm = lm; xm; xm &= xm - 1) {
          const int l = __ffs(xm) - 1;
          sv_loc[(uint64_t)pos * nl + l] = cmp_loc(pl, ctr, cunit, loc, s, l, own);
        }
      }
      __syncthreads();
      if (threadIdx.x < NBKT) {
        uint32_t add = 0;
        for (int w2 = 0; w2 < CB / 64; w2++) add += s_wc[w2][threadIdx.x];
        s_carry[threadIdx.x] += add;
      }
      __syncthreads();
    }
  }
}

// The re-shrink of each list several groups use (ListExt): E = the units
// from |P| on whose byte 0 has the 6-byte bit (stopping at the list end),
// added to the last survivor run's copy for every use but the first -- its
// survivor's records are relocated to the arena's end with room for them.
// The re-shrink then parses on from |P|+E: an aligned parse (a true run head
// there) can match no survivor any more (every survivor run of the list is
// in P); a misaligned one reads garbage docids, and one equal to a later
// survivor would copy a misparsed run -- not emulated, flagged instead
// (GBGPU_EUNSUPPORTED; about 2^-20 per query).  One wave per list.
// slot of candidate docid d in any array, if that slot survived; ~0 if none
__device__ uint64_t survivor_slot(const DevPlan *__restrict__ pl, const Counters *ctr, const uint64_t *cand, const uint32_t *bits,
                                  uint32_t nwords, uint64_t d, int lane) {
  for (int k = 0; k < pl->g0n; k++) {
    const uint64_t *ck = cand + pl->g0base[k];
    const uint32_t n = ctr->g0count[k];
    const uint32_t i = wave_lower_bound(ck, n, d, lane);
    if (i < n && ck[i] == d && slot_is_survivor(pl, ctr, bits, nwords, pl->g0base[k] + i)) return pl->g0base[k] + i;
  }
  return ~0ull;
}

__global__ void __launch_bounds__(64) k_ext_walk(const DevPlan *__restrict__ pl, Counters *ctr, const uint64_t *cand,
                                                 const uint32_t *cunit, const uint32_t *bits, uint32_t nwords,
                                                 const Loc *loc, unsigned long long arena_cap) {
  const int lane = threadIdx.x;
  for (uint32_t xm = pl->reshare_mask; xm; xm &= xm - 1) {
    const int l = __ffs(xm) - 1;
    ListExt &x = ctr->ext[l];
    if (x.units == 0) continue;  // no survivor run in the list
    const DevList &L = pl->lists[l];
    gu8 *p = gl(L.p);
    const uint64_t P = x.units;
    uint64_t u = P;
    for (;;) {  // E: consecutive 6-byte-bit units from |P|
      const uint64_t v = u + lane;
      const bool six = v < L.units && (p[v * 6] & 0x04);
      const uint64_t m = __ballot(!six);
      if (m) {
        u += (uint64_t)(__ffsll((unsigned long long)m) - 1);
        break;
      }
      u += 64;
    }
    const uint64_t s = survivor_slot(pl, ctr, cand, bits, nwords, x.dmax, lane);
    if (lane == 0) {
      x.E = (uint32_t)(u - P);
      x.slot1 = s == ~0ull ? 0u : (uint32_t)(s + 1);
      x.reloc = 0;
    }
    // the parse after the copy: only a misaligned one can match again
    if (x.dmax >= ctr->dmax_all) continue;  // that run was the last survivor: done
    uint64_t h = u;
    bool settled = false;
    for (int step = 0; step < 4096 && !settled; step++) {
      if (h >= L.units) {
        settled = true;
        break;
      }
      gu8 *k = p + h * 6;
      if ((k[1] & 0x02) && !(k[0] & 0x04)) {  // a true run head: aligned
        settled = true;
        break;
      }
      // the docid shrinkSubLists compares: u32 at +8 and byte 7 & 0xfc
      uint64_t g = 0;
      const uint64_t hb = h * 6 + 7;
      for (int b = 4; b >= 0; b--) g = (g << 8) | p[hb + b];
      g = (g & ~3ull) >> 2;
      if (g > ctr->dmax_all) {  // past every survivor: the loop ends
        settled = true;
        break;
      }
      if (g > x.dmax && survivor_slot(pl, ctr, cand, bits, nwords, g, lane) != ~0ull) break;
      h += 2;
      for (;;) {
        const uint64_t v = h + lane;
        const bool six = v < L.units && (p[v * 6] & 0x04);
        const uint64_t m = __ballot(!six);
        if (m) {
          h += (uint64_t)(__ffsll((unsigned long long)m) - 1);
          break;
        }
        h += 64;
      }
    }
    if (!settled && lane == 0) ctr->unsup = 1;  // a misparsed run would be copied
  }
  // the survivors whose re-shrunk copies grow get their records moved to the
  // arena's end, with room for the extra units of every list extending them
  if (lane != 0) return;
  unsigned long long top = ctr->arena_top;
  for (uint32_t xm = pl->reshare_mask; xm; xm &= xm - 1) {
    const int l = __ffs(xm) - 1;
    ListExt &x = ctr->ext[l];
    if (!x.slot1 || !x.E || x.reloc) continue;
    uint32_t lm = 0;
    slot_is_survivor(pl, ctr, bits, nwords, x.slot1 - 1, &lm);
    unsigned long long need = slot_units(pl, ctr, cunit, loc, x.slot1 - 1, lm);
    for (uint32_t ym = pl->reshare_mask; ym; ym &= ym - 1) {
      const int l2 = __ffs(ym) - 1;
      if (ctr->ext[l2].slot1 == x.slot1) need += (unsigned long long)ctr->ext[l2].E * (uint32_t)(pl->lists[l2].uses - 1);
    }
    if (top + need > arena_cap) {
      ctr->unsup = 1;
      return;
    }
    for (uint32_t ym = pl->reshare_mask; ym; ym &= ym - 1) {
      const int l2 = __ffs(ym) - 1;
      if (ctr->ext[l2].slot1 == x.slot1) {
        ctr->ext[l2].reloc = 1;
        ctr->ext[l2].off = top;
      }
    }
    top += need;
  }
  ctr->arena_top = top;
}

// A survivor's run in list lid as group g's sublist x sees it: its own
// units, and -- for a re-shrunk copy of the list's last survivor run
// (ListExt) -- the E units that followed the first shrink's output in the
// buffer, i.e. the list's units [|P|, |P|+E).  Key k of the run is at
// k < len0 ? own + k : ext + (k - len0).
struct SubRun {
  gu8 *own, *ext;
  uint32_t len0, len;
  __device__ __forceinline__ gu8 *key(uint32_t k) const {
    return k < len0 ? own + (size_t)k * 6 : ext + (size_t)(k - len0) * 6;
  }
};
__device__ __forceinline__ SubRun sub_run_at(const DevPlan *__restrict__ pl, const Counters *ctr, Loc lc, int lid, int g, int x,
                                             uint64_t s) {
  gu8 *base = gl(pl->lists[lid].p);
  SubRun r{base + (size_t)lc.unit * 6, base, lc.len, lc.len};
  if ((pl->reshare_mask >> lid & 1) && !(g == pl->lists[lid].owner_group && x == pl->lists[lid].owner_sub) &&
      ctr->ext[lid].slot1 == (uint32_t)(s + 1)) {
    r.ext = base + (size_t)ctr->ext[lid].units * 6;
    r.len += ctr->ext[lid].E;
  }
  return r;
}
// survivor `pos`'s run in list lid (its record's run locations)
__device__ __forceinline__ SubRun sub_run(const DevPlan *__restrict__ pl, const Counters *ctr, const Loc *sv_loc, uint32_t pos,
                                          int lid, int g, int x, uint64_t s) {
  return sub_run_at(pl, ctr, sv_loc[(uint64_t)pos * (uint32_t)pl->nlists + lid], lid, g, x, s);
}

// ------------------------------------------------------------------ score
__constant__ Weights c_weights;

// Per-survivor work, one lane per survivor (Posdb.cpp:6252-7257): for each
// group, mini-merge (Posdb.cpp:6559-6778) its sublist runs into records in
// the survivor's arena range (its run units, handed out from Counters::arena_top), then
// score_doc (scoring.h) over them.
constexpr int SCORE_TPB = 64;
// the two-group variant's LDS records per lane and waves per SIMD it is
// compiled for (A/B builds override them: Makefile `alt`)
#ifndef GBGPU_SCORE_RC2
#define GBGPU_SCORE_RC2 24
#endif
#ifndef GBGPU_SCORE_WAVES2
#define GBGPU_SCORE_WAVES2 4
#endif

// a unit's 6 bytes as one u16 and one u32 load (units are 2-byte aligned;
// which half is 4-byte aligned depends on the unit's parity)
__device__ __forceinline__ uint64_t load6(gu8 *k) {
  const bool odd = ((uintptr_t)k & 2) != 0;
  const auto *h = (const __attribute__((address_space(1))) uint16_t *)(odd ? k : k + 4);
  const auto *w = (const __attribute__((address_space(1))) uint32_t *)(odd ? k + 2 : k);
  const uint64_t hv = *h, wv = *w;
  return odd ? (hv | (wv << 16)) : (wv | (hv << 32));
}

// units b..b+3 of a run (b a multiple of 4) as one dwordx4 and one dwordx3
// load from the 4-byte-aligned address at or below them, instead of eight
// load6 halves: the run's 2-byte phase s (0 or 2) picks which fixed byte
// offsets of the 28 loaded bytes hold each unit.  Reads up to 4 bytes past
// the fourth unit (lists carry LIST_PAD).
__device__ __forceinline__ void load4u(gu8 *src, uint32_t b, uint64_t *v) {
  const uintptr_t a = (uintptr_t)src + (uintptr_t)b * 6;
  const bool s2 = (a & 2) != 0;
  const auto *w = (const __attribute__((address_space(1))) uint32_t *)(a & ~(uintptr_t)3);
  uint32_t x[7];
#pragma unroll
  for (int i = 0; i < 7; i++) x[i] = w[i];
  const uint32_t lo0 = s2 ? (x[0] >> 16) | (x[1] << 16) : x[0], hi0 = s2 ? x[1] >> 16 : x[1] & 0xffff;
  const uint32_t lo1 = s2 ? x[2] : (x[1] >> 16) | (x[2] << 16), hi1 = s2 ? x[3] & 0xffff : x[2] >> 16;
  const uint32_t lo2 = s2 ? (x[3] >> 16) | (x[4] << 16) : x[3], hi2 = s2 ? x[4] >> 16 : x[4] & 0xffff;
  const uint32_t lo3 = s2 ? x[5] : (x[4] >> 16) | (x[5] << 16), hi3 = s2 ? x[6] & 0xffff : x[5] >> 16;
  v[0] = lo0 | ((uint64_t)hi0 << 32);
  v[1] = lo1 | ((uint64_t)hi1 << 32);
  v[2] = lo2 | ((uint64_t)hi2 << 32);
  v[3] = lo3 | ((uint64_t)hi3 << 32);
}

// The stale-mbuf replay (stale_fix): a docid's merges write their keys into
// the reference's function-local mbuf from its start (Posdb.cpp:6007, 6559,
// 6648-6778; a group's first key 12 bytes, later keys 6), so the bytes a later
// docid's trailing empty group reads there are what earlier docids left.  A
// tap keeps the 6 bytes at [lo, lo + 6) of one docid's writes.
struct MbufTap {
  uint32_t lo;
  uint32_t got;  // bit i: b[i] written
  uint8_t b[12];
};
__device__ __forceinline__ void tap_rec(MbufTap *t, uint32_t off, uint64_t lo6, uint64_t hi6, int n) {
  for (int i = 0; i < n; i++) {
    const uint32_t p = off + (uint32_t)i;
    if (p >= t->lo && p < t->lo + 12) {
      const uint64_t src = i < 6 ? lo6 : hi6;
      t->b[p - t->lo] = (uint8_t)(src >> (8 * (i % 6)));
      t->got |= 1u << (p - t->lo);
    }
  }
}

// what the second pass's DocIdScore takes from a scored docid (Posdb.cpp:7555-7563)
struct SurvOut {
  float score;
  int32_t site_rank, doc_lang, ok;
  int32_t ival;  // m_intScore with a gbsortby int term (DocIdScore::m_finalScore is then its double)
  int32_t pad;
};

// MB (the stale-mbuf replay only): count the docid's mbuf bytes (mtot_out),
// tap them (tap: merge only, no scoring), or score with the injected record
template <int NQ, int NS, class RP, class REC = NoRec, bool MB = false>
__device__ __forceinline__ void score_survivor(const DevPlan *__restrict__ pl, const Counters *ctr, uint32_t s, uint32_t lm,
                                               uint32_t anys, const Loc *svloc, RP rec, float *smcol,
                                               uint32_t *key_out, int diag, uint32_t *nrec_out,
                                               bool stamp, uint64_t &tmerge, uint64_t (&tm)[3],
                                               REC *srec = nullptr, SurvOut *so = nullptr,
                                               const uint32_t *kill = nullptr, uint32_t *mtot_out = nullptr,
                                               bool *stale_out = nullptr, const uint64_t *inject = nullptr,
                                               MbufTap *tap = nullptr) {
  const int ng = pl->ngroups;
  DocView<NQ, RP> dv;
  dv.rec = rec;
  dv.present = 0;
  bool empty_pos = false;
  int siteRank = -1, docLang = 0;
  uint64_t sortby_raw = 0;  // gbsortby: the unmerged first key (see below)
  bool sortby_is_raw = false;
  uint32_t nrec = 0;
  uint32_t mtot = 0;  // mbuf bytes the docid's merges wrote (mptr - mbuf)
  // a group's runs: cursor, end, flags (m_bigramFlags of the shrunk sublist
  // index: lists shrunk to empty are not sublists any more)
  struct GrpRuns {
    uint32_t ce[NS], c0[NS];
    uint8_t cfl[NS];
    bool live[NS];
    gu8 *src[NS], *xsrc[NS];
  };
  auto grp_runs = [&](int j, GrpRuns &g) {
    const int gns = pl->gnsub[j];
    int newIdx = 0;
#pragma unroll
    for (int x = 0; x < NS; x++) {
      g.live[x] = false;
      g.ce[x] = 0;
      g.cfl[x] = 0;
      g.src[x] = g.xsrc[x] = nullptr;
      g.c0[x] = 0;
      if (x < gns) {
        const int lid = pl->gsub[j][x];
        if (anys >> lid & 1) {
          g.cfl[x] = pl->gsubflags[j][newIdx];
          newIdx++;
          // kill: sublists the second pass's lookup misses (k_scoreinfo)
          if ((lm >> lid & 1) && !(kill && (kill[j] >> x & 1))) {
            const SubRun sr = sub_run_at(pl, ctr, svloc[lid], lid, j, x, s);
            g.src[x] = sr.own;
            g.xsrc[x] = sr.ext;
            g.c0[x] = sr.len0;
            g.ce[x] = sr.len;
            g.live[x] = true;
          }
        }
      }
    }
  };
  // Two groups (the config-2 variant): both groups' run locations, then both
  // groups' units staged in the lane's LDS column together, one round trip
  // each, when 2 (U0 + U1) <= cap -- the records, at most one per unit, stay
  // below the staged units.  Otherwise each group stages its own (below).
  constexpr bool PRE = NQ <= 2 && std::is_same<RP, LdsRecs>::value && !REC::on;
  GrpRuns pre[PRE ? NQ : 1];
  int preR[PRE ? NQ : 1];
  bool pre_staged = false;
  if constexpr (PRE) {
    uint32_t Ut = 0, cm = 0;
    uint32_t Uj[NQ];
#pragma unroll
    for (int j = 0; j < NQ; j++) {
      Uj[j] = 0;
      if (j < ng && !(pl->gflags0[j] & BF_NEGATIVE)) {
        grp_runs(j, pre[j]);
#pragma unroll
        for (int x = 0; x < NS; x++)
          if (pre[j].live[x]) {
            Uj[j] += pre[j].ce[x];
            cm = pre[j].ce[x] > cm ? pre[j].ce[x] : cm;
          }
      } else {
#pragma unroll
        for (int x = 0; x < NS; x++) pre[j].live[x] = false;
      }
      Ut += Uj[j];
    }
    if (2 * Ut <= (uint32_t)rec.cap && !(diag & 0x200)) {
      pre_staged = true;
      int at = rec.cap - (int)Ut;
#pragma unroll
      for (int j = 0; j < NQ; j++) {
        preR[j] = at;
        at += (int)Uj[j];
      }
      constexpr int SKP = 4;
      for (uint32_t b = 0; b < cm; b += SKP) {
        uint64_t v[NQ][NS][SKP];
#pragma unroll
        for (int j = 0; j < NQ; j++)
#pragma unroll
          for (int x = 0; x < NS; x++) {
            const GrpRuns &g = pre[j];
            if (g.live[x] && b < g.ce[x] && g.c0[x] == g.ce[x] && !(diag & 0x400)) {
              gu8 *sp = g.src[x];
              if (diag & 0x800) {  // diagnostic: every lane reads the first lane's run (no gather, and no divergence)
                const uintptr_t a = (uintptr_t)sp;
                sp = (gu8 *)(((uintptr_t)__builtin_amdgcn_readfirstlane((uint32_t)(a >> 32)) << 32) |
                             (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)a));
              }
              load4u(sp, b, v[j][x]);  // a run of its own list only
            } else {
#pragma unroll
              for (int q = 0; q < SKP; q++) {
                const uint32_t c = b + q;
                v[j][x][q] = (g.live[x] && c < g.ce[x])
                                 ? load6(c < g.c0[x] ? g.src[x] + (size_t)c * 6 : g.xsrc[x] + (size_t)(c - g.c0[x]) * 6)
                                 : 0;
              }
            }
          }
#pragma unroll
        for (int j = 0; j < NQ; j++) {
          uint32_t off = 0;
#pragma unroll
          for (int x = 0; x < NS; x++) {
            const GrpRuns &g = pre[j];
#pragma unroll
            for (int q = 0; q < SKP; q++)
              if (g.live[x] && b + q < g.ce[x]) rec.put(preR[j] + (int)(off + b + q), v[j][x][q]);
            off += g.live[x] ? g.ce[x] : 0;
          }
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < NQ; j++) {
    dv.beg[j] = dv.end[j] = (int)nrec;
    if (j >= ng) continue;
    const uint8_t gf0 = pl->gflags0[j];
    if (gf0 & BF_NEGATIVE) continue;
    uint64_t ta = 0;
    if (stamp) ta = __builtin_amdgcn_s_memtime();
    GrpRuns gr;
    if constexpr (PRE) gr = pre[j];
    else grp_runs(j, gr);
    uint32_t cu[NS], ce[NS], c0[NS];
    uint8_t cfl[NS];
    bool live[NS];
    gu8 *src[NS], *xsrc[NS];
#pragma unroll
    for (int x = 0; x < NS; x++) {
      cu[x] = 0;
      ce[x] = gr.ce[x];
      c0[x] = gr.c0[x];
      cfl[x] = gr.cfl[x];
      live[x] = gr.live[x];
      src[x] = gr.src[x];
      xsrc[x] = gr.xsrc[x];
    }
    // Stage the group's run units in the lane's LDS column at its tail
    // [cap - U, cap), every sublist's next SK units in flight together: the
    // records written meanwhile stay below it when nrec + 2U <= cap, as each
    // record consumes at least one unit.  Otherwise the merge reads the
    // units from global memory one by one.
    constexpr int SK = NS >= 16 ? 1 : NS >= 4 ? 16 / NS : 4;
    if (stamp) {
      __asm__ volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      const uint64_t tb = __builtin_amdgcn_s_memtime();
      tm[0] += tb - ta;
      ta = tb;
    }
    uint32_t offx[NS], U = 0, cmax = 0;
#pragma unroll
    for (int x = 0; x < NS; x++) {
      offx[x] = U;
      U += live[x] ? ce[x] : 0;
      cmax = live[x] && ce[x] > cmax ? ce[x] : cmax;
    }
    bool staged = false;
    int R = 0;
    if constexpr (PRE) {
      if (pre_staged) {
        staged = true;
        R = preR[j];
      }
    }
    if constexpr (std::is_same<RP, LdsRecs>::value) {
      if (!staged && nrec + 2 * U <= (uint32_t)rec.cap && !(diag & 0x200)) {
        staged = true;
        R = rec.cap - (int)U;
        for (uint32_t b = 0; b < cmax; b += SK) {
          uint64_t v[NS][SK];
#pragma unroll
          for (int x = 0; x < NS; x++) {
            bool fast = false;
            if constexpr (SK == 4) fast = live[x] && b < ce[x] && c0[x] == ce[x] && !(diag & 0x400);
            if (fast) {
              if constexpr (SK == 4) load4u(src[x], b, v[x]);  // a run of its own list only
            } else {
#pragma unroll
              for (int q = 0; q < SK; q++) {
                const uint32_t c = b + q;
                v[x][q] = (live[x] && c < ce[x])
                              ? load6(c < c0[x] ? src[x] + (size_t)c * 6 : xsrc[x] + (size_t)(c - c0[x]) * 6)
                              : 0;
              }
            }
          }
#pragma unroll
          for (int x = 0; x < NS; x++)
#pragma unroll
            for (int q = 0; q < SK; q++)
              if (live[x] && b + q < ce[x]) rec.put(R + (int)(offx[x] + b + q), v[x][q]);
        }
      }
    }
    // unit c of sublist x, x a runtime index: one LDS read (staged) or one
    // global unit load, its address picked by select chains
    if (stamp) {
      __asm__ volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      const uint64_t tb = __builtin_amdgcn_s_memtime();
      tm[1] += tb - ta;
      ta = tb;
    }
    auto unit_at = [&](int x, uint32_t c) -> uint64_t {
      uint32_t o = 0, cz = 0;
      gu8 *a = nullptr, *b = nullptr;
#pragma unroll
      for (int y = 0; y < NS; y++)
        if (y == x) {
          o = offx[y];
          cz = c0[y];
          a = src[y];
          b = xsrc[y];
        }
      if (staged) return rec[R + (int)(o + c)];
      return load6(c < cz ? a + (size_t)c * 6 : b + (size_t)(c - cz) * 6);
    };
    uint64_t ck[NS];
    bool cfirst[NS];
#pragma unroll
    for (int x = 0; x < NS; x++) {
      cfirst[x] = live[x];
      ck[x] = 0;
      if (live[x]) {
        if (staged) ck[x] = rec[R + (int)offx[x]];
        else ck[x] = load6(src[x]);  // cu == 0 < c0 (a run has its own units)
      }
    }
    // a numeric (or facet) group with the docid in ONE sublist is not merged:
    // its miniMergedList points into the termlist, keys unrewritten, and
    // nothing of it goes to mbuf (Posdb.cpp:6638-6647) -- so an empty group
    // before it does not read its first key, and the scorers skip it
    // (BF_NUMBER/BF_FACET); only gbsortby reads it (its first key's number)
    {
      int nl = 0;
      uint64_t rk = 0;
      uint8_t f = 0;
#pragma unroll
      for (int x = 0; x < NS; x++)
        if (live[x] && nl++ == 0) {
          rk = ck[x];
          f = cfl[x];
        }
      if (nl == 1 && (f & (BF_FACET | BF_NUMBER)) && !(f & (BF_SYNONYM | BF_HALFSTOPWIKIBIGRAM))) {
        if (j == pl->sortby_group) {
          sortby_raw = rk;
          sortby_is_raw = true;
        }
        dv.beg[j] = dv.end[j] = (int)nrec;
        dv.present |= 1u << j;
        continue;
      }
    }
    const uint32_t start = nrec;
    const uint32_t mg0 = mtot;  // the group's first byte in mbuf
    uint32_t mbytes = 0;  // emulates mptr - mbuf (cap 299000, Posdb.cpp:6007-6008)
    bool isFirstKey = true;
    uint64_t last = 0;
    for (;;) {
      // the smallest current key (6-byte keys compare as 48-bit numbers;
      // ties go to the lowest sublist)
      int mink = -1;
      uint64_t r = 0;
#pragma unroll
      for (int x = 0; x < NS; x++)
        if (live[x] && (mink == -1 || ck[x] < r)) {
          mink = x;
          r = ck[x];
        }
      if (mink == -1) break;
      uint8_t fl = 0;
      uint32_t cx = 0, cex = 0;
      bool cf = false;
#pragma unroll
      for (int x = 0; x < NS; x++)
        if (x == mink) {
          fl = cfl[x];
          cx = cu[x];
          cex = ce[x];
          cf = cfirst[x];
        }
      const bool hack = (fl & BF_BIGRAM) && ((r >> 16) & 0x03);  // Posdb.cpp:6687-6692
      if (!hack) {
        uint64_t b2 = (r >> 16) & 0xfc;
        if (fl & (BF_BIGRAM | BF_SYNONYM)) b2 |= 0x02;
        if (fl & BF_HALFSTOPWIKIBIGRAM) b2 |= 0x01;
        r = (r & ~(0xffull << 16)) | (b2 << 16);
        if (isFirstKey) {
          // siteRank / langId of the key copied as 12 bytes (Posdb.h:308-315):
          // the bytes after the first emitted key
          const uint64_t hi6 = unit_at(mink, cx + 1);
          const uint32_t b0 = (uint32_t)(r & 0xff), b6 = (uint32_t)(hi6 & 0xff), b7 = (uint32_t)((hi6 >> 8) & 0xff);
          const int sr = (int)(((b6 >> 5) | ((b7 & 1) << 3)) & 0x0f);
          const int lg = (int)((b6 & 0x1f) | ((b0 & 0x08) ? 0x20 : 0));
          r = (r & ~0xffull) | (((r & 0xff) & 0xf9) | 0x02);
          if constexpr (MB)
            if (tap) tap_rec(tap, mg0 + mbytes, r, hi6, 12);
          rec.put(nrec++, r);
          last = r;
          mbytes += 12;
          isFirstKey = false;
          if (siteRank < 0 && !(gf0 & (BF_NUMBER | BF_FACET))) {
            siteRank = sr;
            docLang = lg;
          }
        } else {
          const bool dup = (((last >> 32) & 0xffff) == ((r >> 32) & 0xffff)) &&
                           (((last >> 24) & 0xc0) == ((r >> 24) & 0xc0));
          if (!dup) {
            r |= 0x06;
            if constexpr (MB)
              if (tap) tap_rec(tap, mg0 + mbytes, r, 0, 6);
            rec.put(nrec++, r);
            last = r;
            mbytes += 6;
          }
        }
      }
      const uint32_t ncx = cx + (cf ? 2 : 1);
      const bool more = ncx < cex;
      const uint64_t nk = more ? unit_at(mink, ncx) : 0;
#pragma unroll
      for (int x = 0; x < NS; x++)
        if (x == mink) {
          cu[x] = ncx;
          cfirst[x] = false;
          live[x] = more;
          ck[x] = nk;
        }
      if (mbytes >= 299000) break;
    }
    if (stamp) {
      __asm__ volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      tm[2] += __builtin_amdgcn_s_memtime() - ta;
    }
    if constexpr (MB) mtot += mbytes;
    dv.beg[j] = (int)start;
    dv.end[j] = (int)nrec;
    dv.present |= 1u << j;
    // An empty mini-merged list still has one key read by every scorer
    // (do-while loops): what mbuf holds there.  When a later group writes
    // records, that is its first key (groups are merged back to back from
    // the same place), which rec[start] is here too; when none does, it is
    // stale bytes of an earlier docid: the docid is dropped here and
    // stale_fix scores it from those bytes after the pass
    empty_pos = nrec == start;
  }
  if (stale_out) *stale_out = empty_pos;
  if constexpr (MB) {
    if (mtot_out) *mtot_out = mtot;
    if (tap) {  // stale_fix: this docid's mbuf bytes only; key_out 1: no plain group gave a key
      *key_out = siteRank < 0 ? 1u : 0u;
      return;
    }
    if (empty_pos && inject) {
      // stale_fix / k_si_stale: the bytes earlier docids of the call left
      // where the trailing empty group points (the record store has room
      // for one more): inject[0] its bytes 0-5; inject[1] bytes 6-11 with bit
      // 63 set when known.  A docid no plain group gave a key takes siteRank
      // and langId from there too (the group's list pointer, Posdb.cpp:
      // 6984-7003)
      rec.put((int)nrec, inject[0]);
      empty_pos = false;
      if (siteRank < 0 && (inject[1] >> 63)) {
        bool plain = false;
        for (int j = 0; j < ng; j++)
          if (!(pl->gflags0[j] & (BF_NEGATIVE | BF_NUMBER | BF_FACET))) plain = true;
        if (plain) {
          const uint32_t b0 = (uint32_t)(inject[0] & 0xff), b6 = (uint32_t)(inject[1] & 0xff),
                         b7 = (uint32_t)((inject[1] >> 8) & 0xff);
          siteRank = (int)(((b6 >> 5) | ((b7 & 1) << 3)) & 0x0f);
          docLang = (int)((b6 & 0x1f) | ((b0 & 0x08) ? 0x20 : 0));
        }
      }
    }
  }
  float score = 0.0f;
  *nrec_out = nrec;
  if (stamp) {  // diagnostic stamp (GBGPU_SCORE_MODE=2)
    __asm__ volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    tmerge = __builtin_amdgcn_s_memtime();
  }
  if ((diag & 0xff) == 1) {  // diagnostic: mini-merge only
    *key_out = nrec + 1;
    return;
  }
  // (the scorers bound their top-list slot loops by the wave's largest
  // fillable count, wave_max15 in scoring.h)
  bool ok = false;
  if (!empty_pos) {
    const int sr = siteRank < 0 ? 0 : siteRank;
    ok = score_doc<NQ, RP, REC>(&c_weights, pl, dv, sr, docLang, smcol, SCORE_TPB, &score, diag & 0xff, srec);
  }
  // gbsortby: the score is the float of the group's first key, bytes 2..5 as
  // the mini-merge left them (Posdb.cpp:7265-7269)
  uint32_t ival = 0;  // gbsortby int: m_intScore's bits
  if (ok && pl->sortby_group >= 0) {
    const uint32_t v = (uint32_t)((sortby_is_raw ? sortby_raw : dv.rec[rget(dv.beg, pl->sortby_group)]) >> 16);
    if (pl->sortby_int) ival = v;  // getInt (Posdb.cpp:7271-7279)
    else score = __uint_as_float(v);
  }
  if (so) {
    so->score = score;
    so->ival = (int32_t)ival;
    so->site_rank = siteRank < 0 ? 0 : siteRank;
    so->doc_lang = docLang;
    so->ok = empty_pos ? -2 : ok;
    if (siteRank < 0) so->pad = 1;  // no plain group gave a key (a stale docid's siteRank is in mbuf)
  }
  uint32_t key = 0;
  if (ok) {
    const uint32_t b = __float_as_uint(score);
    key = (b & 0x80000000u) ? ~b : (b | 0x80000000u);
    if (pl->sortby_group >= 0 && pl->sortby_int) {
      key = ival ^ 0x80000000u;  // int32 order
      // m_intScore INT32_MIN would travel as key 0 ("not scored"): the query
      // is declined (GBGPU_EUNSUPPORTED), never answered with INT32_MIN + 1
      if (key == 0) const_cast<Counters *>(ctr)->unsup = 1;
    }
    if (key == 0) key = 1;
  }
  *key_out = key;
}

// k_topk's histogram: one atomic per distinct bin of the wave's keys (equal
// scores -- gbsortby values, ties -- would otherwise queue on one address)
__device__ __forceinline__ void hist_add(uint32_t *h, uint32_t key, int lane) {
  uint32_t bin = key ? key >> 16 : 0xffffffffu;
  uint64_t left = __ballot(key != 0);
  while (left) {
    const uint32_t b = __shfl(bin, __ffsll((unsigned long long)left) - 1, 64);
    const uint64_t m = __ballot(bin == b) & left;
    if (lane == __ffsll((unsigned long long)m) - 1) atomicAdd(&h[b], (uint32_t)__popcll(m));
    left &= ~m;
  }
}

// Scored in size-bucket order (k_cmp_place's positions), so a wave's
// survivors have similar work (its lanes run the scorers in lockstep).
// Waves of buckets 3-7 score 64 survivors, one per lane, each keeping its
// records in its lane's column of the wave's LDS record arrays (RC records);
// waves of buckets 0-2 score 8/16/32 larger survivors with 8/4/2 columns
// each.  A survivor that still does not fit (or whose re-shrunk copies grow
// it past that) takes a range of the global record arena.  A survivor's
// data (slot, list mask, units, run locations) is read at its position, so
// a wave's reads are contiguous; its key goes to skey at the same position.
template <int NQ, int NS, int RC>
__global__ void __launch_bounds__(SCORE_TPB, (NQ <= 2 && NS <= 2) ? GBGPU_SCORE_WAVES2 : 1)
    k_score(const DevPlan *__restrict__ pl, const uint64_t *sv_doc, Counters *ctr,
                                                     const uint32_t *sv_slot, const uint32_t *sv_lm,
                                                     const uint32_t *sv_u, const Loc *sv_loc, uint64_t *arena,
                                                     unsigned long long arena_cap, uint32_t *skey, uint8_t *sflag,
                                                     int diag, uint64_t *dbg, uint32_t *khist) {
  static_assert(SCORE_TPB == 64, "LdsRecs columns are one wave wide");
  __shared__ float s_sm[npairs<NQ>() * SCORE_TPB];
  __shared__ uint32_t s_rlo[RC * 64];
  __shared__ uint16_t s_rhi[RC * 64];
  // diagnostic (GBGPU_SCORE_MODE=2): per-wave start/end clock, records
  const uint64_t t0 = dbg ? __builtin_amdgcn_s_memrealtime() : 0;
  uint32_t dmax = 0, dsum = 0, dits = 0;
  uint64_t tseg[3] = {0, 0, 0};  // diagnostic: cycles in setup loads, mini-merge, scorers
  uint64_t tmm[3] = {0, 0, 0};   // ... and in the mini-merge: run locations, staging, merge loop
  stage_weights(&c_weights);
  const uint32_t anys = ctr->anysurv;
  const int lane = threadIdx.x;
  const uint32_t nl = (uint32_t)pl->nlists;
  // waves per bucket: bucket b packs 1 << bucket_shift(b) survivors a wave
  uint32_t wend[NBKT];
  uint32_t nw = 0;
#pragma unroll
  for (int b = 0; b < NBKT; b++) {
    nw += (ctr->bcnt[b] + (1u << bucket_shift(b)) - 1) >> bucket_shift(b);
    wend[b] = nw;
  }
  uint32_t nfilt = 0;
  for (uint32_t w = blockIdx.x; w < nw; w += gridDim.x) {  // uniform over the wave
    int b = 0;
#pragma unroll
    for (int q = 0; q < NBKT - 1; q++) b += w >= wend[q];
    uint32_t st = 0, cnt = 0, wprev = 0;
#pragma unroll
    for (int q = 0; q < NBKT; q++)
      if (q == b) {
        st = ctr->bstart[q];
        cnt = ctr->bcnt[q];
        wprev = q ? wend[q - 1] : 0;
      }
    const int sh = bucket_shift(b);
    const uint32_t j = ((w - wprev) << sh) + (uint32_t)lane;
    bool filt = false;
    if (lane < (1 << sh) && j < cnt) {
      uint64_t ts0 = 0, ts1 = 0, ts2 = 0, ts3 = 0;
      if (dbg) ts0 = __builtin_amdgcn_s_memtime();
      const uint32_t i = st + j;
      const uint32_t s = sv_slot[i];
      const uint32_t lm = sv_lm[i];
      uint32_t units = sv_u[i];
      const Loc *svl = sv_loc + (uint64_t)i * nl;
      unsigned long long off = ~0ull;
      for (uint32_t x = lm & pl->reshare_mask; x; x &= x - 1) {  // re-shrunk copies (k_ext_walk)
        const int l = __ffs(x) - 1;
        const ListExt &e = ctr->ext[l];
        if (e.slot1 == s + 1) {
          units += e.E * (uint32_t)(pl->lists[l].uses - 1);
          if (e.reloc) off = e.off;
        }
      }
      uint32_t key, nr = 0;
      bool st = false;
      if (dbg) {
        __asm__ volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        ts1 = __builtin_amdgcn_s_memtime();
      }
      if (pl->boolean) {
        // a boolean query's score (Posdb.cpp:6514-6534, 7247-7256): the bits of
        // its vector, times (siteRank * 0 + 1.0) and the same-language weight
        // (siteRank and docLang keep their initial 0: the scorers and their
        // siteRank/langId reads are jumped over)
        uint32_t v = 0;
        for (uint32_t xm = lm; xm; xm &= xm - 1) v |= pl->bool_gmask[__ffs(xm) - 1];
        const float minScore = (float)__popc(v);
        float score = (float)((double)minScore * ((double)(0.0f * pl->site_rank_multiplier) + 1.0));
        score *= pl->same_lang_weight;
        const uint32_t b = __float_as_uint(score);
        key = (b & 0x80000000u) ? ~b : (b | 0x80000000u);
        if (key == 0) key = 1;
      } else if (units <= ((uint32_t)RC << (6 - sh))) {
        const LdsRecs lrec{(__attribute__((address_space(3))) uint32_t *)(s_rlo + lane),
                           (__attribute__((address_space(3))) uint16_t *)(s_rhi + lane), sh, RC << (6 - sh)};
        score_survivor<NQ, NS>(pl, ctr, s, lm, anys, svl, lrec, s_sm + lane, &key, diag, &nr,
                               dbg != nullptr, ts2, tmm, (NoRec *)nullptr, nullptr, nullptr, nullptr, &st);
      } else {
        if (off == ~0ull) off = atomicAdd(&ctr->arena_top, (unsigned long long)units);
        if (off + units > arena_cap) {
          ctr->unsup = 1;  // the host sized the arena for every survivor's units: not reached
          key = 0;
        } else {
          const GlobalRecs grec{(__attribute__((address_space(1))) uint64_t *)(arena + off)};
          score_survivor<NQ, NS>(pl, ctr, s, lm, anys, svl, grec, s_sm + lane, &key, diag, &nr,
                                 dbg != nullptr, ts2, tmm, (NoRec *)nullptr, nullptr, nullptr, nullptr, &st);
        }
      }
      if (dbg) {
        __asm__ volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        ts3 = __builtin_amdgcn_s_memtime();
        dmax = nr > dmax ? nr : dmax;
        dsum += nr;
        dits++;
        if (ts2 == 0) ts2 = ts3;
        tseg[0] += ts1 - ts0;
        tseg[1] += ts2 - ts1;
        tseg[2] += ts3 - ts2;
      }
      // the paging filter of a widget's next page (Posdb.cpp:7327-7347):
      // m_filtered counts the scored docids it drops
      if (pl->has_serp && key) {
        const uint64_t d = sv_doc[i];
        if (pl->sortby_group >= 0 && pl->sortby_int) {  // intScore vs (int32_t)m_maxSerpScore
          const int32_t iv = (int32_t)(key ^ 0x80000000u);
          if (iv > pl->max_serp_int) filt = true;
          else if (iv == pl->max_serp_int && (int64_t)d <= pl->min_serp_docid) filt = true;
        } else {
          const uint32_t b2 = (key & 0x80000000u) ? (key & 0x7fffffffu) : ~key;
          const float score = __uint_as_float(b2);
          if (score > (float)pl->max_serp_score) filt = true;
          else if ((double)score == pl->max_serp_score && (int64_t)d <= pl->min_serp_docid) filt = true;
        }
        if (filt) key = 0;
      }
      skey[i] = key;
      if (st) atomicAdd(&ctr->nstale, 1u);  // scored after the pass (stale_fix)
      if (khist) hist_add(khist, key, lane);  // k_topk's first pass
      // site clustering: the replay counts m_filtered, since a docid the
      // prefilters skip never reaches the paging test (Posdb.cpp:6341-6345)
      if (pl->clustering) sflag[i] = filt ? 1 : 0;
    }
    nfilt += (uint32_t)__popcll(__ballot(filt));
  }
  if (!pl->clustering && (threadIdx.x & 63) == 0 && nfilt) atomicAdd((uint32_t *)&ctr->filtered, nfilt);
  if (dbg) {
    for (int o = 32; o > 0; o >>= 1) {
      const uint32_t m = __shfl_xor(dmax, o, 64);
      dmax = m > dmax ? m : dmax;
      dsum += __shfl_xor(dsum, o, 64);
      dits += __shfl_xor(dits, o, 64);
    }
    const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
    for (int o = 32; o > 0; o >>= 1)
      for (int q = 0; q < 3; q++) {
        const uint64_t m = __shfl_xor(tseg[q], o, 64);
        tseg[q] = m > tseg[q] ? m : tseg[q];
        const uint64_t m2 = __shfl_xor(tmm[q], o, 64);
        tmm[q] = m2 > tmm[q] ? m2 : tmm[q];
      }
    if (threadIdx.x == 0) {
      dbg[blockIdx.x * 8 + 0] = t0;
      dbg[blockIdx.x * 8 + 1] = t1;
      dbg[blockIdx.x * 8 + 2] = dmax;
      dbg[blockIdx.x * 8 + 3] = ((uint64_t)dits << 32) | dsum;
      dbg[blockIdx.x * 8 + 4] = tseg[0];
      dbg[blockIdx.x * 8 + 5] = tseg[1];
      dbg[blockIdx.x * 8 + 6] = tseg[2];
      dbg[blockIdx.x * 8 + 7] = (tmm[0] & 0xfffff) | ((tmm[1] & 0xfffff) << 20) | ((tmm[2] & 0xfffff) << 40);
    }
  }
}

// ------------------------------------------- the second pass's score info
// m_getDocIdScoringInfo (Posdb.cpp:6116-6244, 7554-7665, 7752-7770): after
// the first pass, the top min(m_numUsedNodes, m_docsToGet) docids of the tree
// are scored again, high -> low, with the scorers recording their top lists.
// Here the tree's docids find their survivor entry (k_si_find), and
// k_scoreinfo re-runs score_survivor for them -- one lane per docid, the
// records in the survivor's own range of the global arena -- with ScoreRec
// attached; the host lays out DocIdScore and the offsets.

// getSingleTermScore's / getTermPairScoreForAny's recording (Posdb.cpp:
// 3247-3298, 4195-4280) into one docid's slices of the output arrays, in the
// reference's append order.  The host sizes the slices for the worst case.
struct ScoreRec {
  static constexpr bool on = true;
  gbgpu_single_score *ss;
  gbgpu_pair_score *ps;
  int ns, np, scap, pcap;
  __device__ void single(const DevPlan *__restrict__ pl, int i, float best, uint64_t r) {
    if (ns < scap) {
      gbgpu_single_score x;
      __builtin_memset(&x, 0, sizeof x);
      x.is_synonym = (int8_t)r_syn(r);
      x.is_half_stop_wiki_bigram = (int8_t)r_hswb(r);
      x.diversity_rank = (int8_t)r_div(r);
      x.word_spam_rank = (int8_t)r_wsr(r);
      x.hash_group = (int8_t)r_hg(r);
      x.word_pos = (int32_t)r_wordpos(r);
      x.density_rank = (int8_t)r_dens(r);
      float score = best;
      score *= pl->tfw[i];
      score *= pl->tfw[i];
      if (x.is_half_stop_wiki_bigram) {
        score *= GB_WIKI_BIGRAM_WEIGHT;
        score *= GB_WIKI_BIGRAM_WEIGHT;
      }
      x.final_score = score;
      x.tf_weight = pl->tfw[i];
      x.qterm_num = pl->qterm[i];
      x.bflags = (int8_t)pl->gflags0[i];
      __builtin_memcpy(ss + ns, &x, sizeof x);
    }
    ns++;
  }
  __device__ void pair(const DevPlan *__restrict__ pl, int i, int j, float best, float wts, int32_t qdist, uint64_t r1,
                       uint64_t r2, uint8_t fixed) {
    if (np < pcap) {
      gbgpu_pair_score x;
      __builtin_memset(&x, 0, sizeof x);
      float score = best;
      score *= wts;
      score *= pl->tfw[i];
      score *= pl->tfw[j];
      if (r_hswb(r1)) score *= GB_WIKI_BIGRAM_WEIGHT;
      if (r_hswb(r2)) score *= GB_WIKI_BIGRAM_WEIGHT;
      x.final_score = score;
      x.word_pos1 = (int32_t)r_wordpos(r1);
      x.word_pos2 = (int32_t)r_wordpos(r2);
      x.is_synonym1 = (int8_t)r_syn(r1);
      x.is_synonym2 = (int8_t)r_syn(r2);
      x.is_half_stop_wiki_bigram1 = (int8_t)r_hswb(r1);
      x.is_half_stop_wiki_bigram2 = (int8_t)r_hswb(r2);
      x.diversity_rank1 = (int8_t)r_div(r1);
      x.diversity_rank2 = (int8_t)r_div(r2);
      x.word_spam_rank1 = (int8_t)r_wsr(r1);
      x.word_spam_rank2 = (int8_t)r_wsr(r2);
      x.hash_group1 = (int8_t)r_hg(r1);
      x.hash_group2 = (int8_t)r_hg(r2);
      x.qdist = qdist;
      x.density_rank1 = (int8_t)r_dens(r1);
      x.density_rank2 = (int8_t)r_dens(r2);
      x.fixed_distance = (int8_t)fixed;  // 2: the reference reads its uninitialised local here
      x.qterm_num1 = pl->qterm[i];
      x.qterm_num2 = pl->qterm[j];
      x.tf_weight1 = pl->tfw[i];
      x.tf_weight2 = pl->tfw[j];
      x.bflags1 = (int8_t)pl->gflags0[i];
      x.bflags2 = (int8_t)pl->gflags0[j];
      x.in_same_wiki_phrase = (wts == (float)GB_WIKI_WEIGHT) ? 1 : 0;
      __builtin_memcpy(ps + np, &x, sizeof x);
    }
    np++;
  }
};

// The second pass does not walk the vote buffer: it looks each tree docid up
// in every shrunk sublist with getWordPosList (Posdb.h:873-956), a binary
// search that can miss a docid that is there (its step bottoms out at one
// unit after three probes, and a probe landing on a run's first unit
// resolves to the previous run).  A miss drops that sublist from the
// docid's mini merge.  shrinkSubLists (Posdb.cpp:5334-5428) made each
// sublist the survivors' runs in docid order, in place, so the search is
// replayed over a directory: survivors sorted by docid (k_si_keys + sisort),
// and per list the exclusive prefix of their run units (k_si_dir).  Past the
// shrunk end the in-place buffer still holds the list's own bytes.
__global__ void k_si_keys(const uint64_t *sv_doc, uint32_t nsurv, uint64_t *key, uint32_t *val) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nsurv; i += gridDim.x * blockDim.x) {
    key[i] = sv_doc[i];
    val[i] = i;
  }
}

// one block per list: cum[l][k] = units, in list l, of the survivors ranked
// below k (k = 0..nsurv)
__global__ void __launch_bounds__(1024) k_si_dir(const DevPlan *__restrict__ pl, const Loc *sv_loc, const uint32_t *sv_lm,
                                                 const uint32_t *sperm, uint32_t nsurv, uint32_t *cum) {
  __shared__ uint32_t s_w[16];
  const int l = blockIdx.x;
  uint32_t *c = cum + (size_t)l * (nsurv + 1);
  uint32_t carry = 0;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (uint32_t b = 0; b < nsurv; b += 1024) {
    const uint32_t k = b + threadIdx.x;
    uint32_t u = 0;
    if (k < nsurv) {
      const uint32_t i = sperm[k];
      if (sv_lm[i] >> l & 1) u = sv_loc[(uint64_t)i * (uint32_t)pl->nlists + l].len;
    }
    uint32_t x = u;  // inclusive wave scan
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    if (lane == 63) s_w[w] = x;
    __syncthreads();
    uint32_t wb = 0, tot = 0;
    for (int q = 0; q < 16; q++) {
      wb += q < w ? s_w[q] : 0;
      tot += s_w[q];
    }
    if (k < nsurv) c[k] = carry + wb + x - u;
    carry += tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) c[nsurv] = carry;
}

// list lid's in-place buffer as getWordPosList reads it: unit u of the
// shrunk image (u < S), else the list's own unit u (zero past its end)
struct SiList {
  const DevPlan *__restrict__ pl;
  const Loc *sv_loc;
  const uint32_t *sperm, *cum;
  uint32_t nsurv;
  int lid;
  __device__ uint32_t run_of(uint32_t u) const {  // last k with cum[k] <= u
    uint32_t lo = 0, hi = nsurv;
    while (lo < hi) {
      const uint32_t mid = (lo + hi + 1) >> 1;
      if (cum[mid] <= u) lo = mid;
      else hi = mid - 1;
    }
    return lo;
  }
  __device__ uint64_t unit(int64_t u) const {
    gu8 *base = gl(pl->lists[lid].p);
    if (u < (int64_t)cum[nsurv]) {
      const uint32_t k = run_of((uint32_t)u);
      const Loc lc = sv_loc[(uint64_t)sperm[k] * (uint32_t)pl->nlists + lid];
      return load6(base + ((size_t)lc.unit + (size_t)(u - cum[k])) * 6);
    }
    if (u < (int64_t)pl->lists[lid].units) return load6(base + (size_t)u * 6);
    return 0;
  }
};

// getWordPosList(docId) over the shrunk list of U units: 1 found (the
// docid's own run, which starts at unit `own`), 0 NULL, < 0 a path not
// replayed: -1 a match off the list's start, -2 at a negative key, -3
// somewhere else than `own`.  A list shared by several groups is shrunk again in
// place for each later use; that pass re-copies the runs onto themselves and
// then parses the stale bytes after them, extending the last run by E units
// (k_ext_walk) -- the buffer's bytes stay those of SiList::unit, only the
// later uses' U grows.
__device__ int si_word_pos_list(const SiList &L, uint64_t docId, uint32_t own, int64_t U) {
  int64_t step = (6 * U / 12) * 6;  // bytes
  int64_t p = step / 6;              // units
  int count = 0;
  for (int it = 0; it < 256; it++) {
    const int64_t origp = p;
    while (p > 0 && ((L.unit(p) >> 8) & 0x02)) p--;
    p -= 1;
    const uint64_t d = ((L.unit(p + 1) >> 8) & 0xffffffffffull) >> 2;
    if (d == docId) {
      if (p < 0) return -1;
      if (!(L.unit(p) & 0x01)) return -2;
      return p == (int64_t)own ? 1 : -3;
    }
    step >>= 1;
    step -= step % 6;
    if (step <= 0) {
      step = 6;
      if (count++ >= 2) return 0;
    }
    if (d < docId) {
      p = origp + step / 6;
      if (p > U) p = U - 1;
    } else {
      p = origp - step / 6;
      if (p < 0) p = 0;
    }
  }
  return -1;
}

// the sublists getWordPosList finds docid d in (Posdb.cpp:6195-6241): kill
// bit x of group j where it misses; d is the survivor of docid-order rank lo
// with list mask lm.  < 0: a path not replayed (*blid: the list)
__device__ int si_kill(const DevPlan *__restrict__ pl, const Counters *ctr, const Loc *sv_loc, const uint32_t *sperm,
                       const uint32_t *cum, uint32_t nsurv, uint64_t d, uint32_t lo, uint32_t lm, uint32_t *kill,
                       int *blid) {
  for (int j = 0; j < MAXG; j++) kill[j] = 0;
  const uint32_t anys = ctr->anysurv;
  for (int j = 0; j < pl->ngroups; j++) {
    if (pl->gflags0[j] & BF_NEGATIVE) continue;
    for (int x = 0; x < pl->gnsub[j]; x++) {
      const int lid = pl->gsub[j][x];
      if (!(anys >> lid & 1) || !(lm >> lid & 1)) continue;
      const SiList L{pl, sv_loc, sperm, cum + (size_t)lid * (nsurv + 1), nsurv, lid};
      const bool later = (pl->reshare_mask >> lid & 1) &&
                         !(j == pl->lists[lid].owner_group && x == pl->lists[lid].owner_sub);
      const int64_t U = (int64_t)L.cum[nsurv] + ((later && ctr->ext[lid].slot1) ? ctr->ext[lid].E : 0);
      const int f = si_word_pos_list(L, d, L.cum[lo], U);
      if (f < 0) {
        *blid = lid;
        return f;
      }
      if (f == 0) kill[j] |= 1u << x;
    }
  }
  return 0;
}

// docid-order rank of tree docid d among the survivors (sdoc sorted), or nsurv
__device__ __forceinline__ uint32_t si_rank(const uint64_t *sdoc, uint32_t nsurv, uint64_t d) {
  uint32_t lo = 0, hi = nsurv;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (sdoc[mid] < d) lo = mid + 1;
    else hi = mid;
  }
  return lo < nsurv && sdoc[lo] == d ? lo : nsurv;
}

// a survivor's record units, as k_score sizes its store (its re-shrunk copies
// grow by E units each), and the arena offset of a relocated copy (~0: none)
__device__ __forceinline__ uint32_t surv_units_off(const DevPlan *__restrict__ pl, const Counters *ctr, uint32_t s,
                                                   uint32_t lm, uint32_t u, unsigned long long *off) {
  *off = ~0ull;
  for (uint32_t x = lm & pl->reshare_mask; x; x &= x - 1) {
    const int l = __ffs(x) - 1;
    const ListExt &e = ctr->ext[l];
    if (e.slot1 == s + 1) {
      u += e.E * (uint32_t)(pl->lists[l].uses - 1);
      if (e.reloc) *off = e.off;
    }
  }
  return u;
}

// one lane per tree docid: the first pass's score_survivor again, with the
// recorder, over the survivor's arena range (k_score's fallback store); mt:
// the mbuf bytes its merges write (the second pass's stale-byte replay,
// k_si_stale); a docid whose last merged group comes out empty is ok = -4
__global__ void __launch_bounds__(SCORE_TPB) k_scoreinfo(const DevPlan *__restrict__ pl, Counters *ctr, const uint32_t *sv_slot,
                                                         const uint32_t *sv_lm, const uint32_t *sv_u,
                                                         const Loc *sv_loc, uint64_t *arena,
                                                         unsigned long long arena_cap, const uint64_t *tdoc,
                                                         const uint64_t *sdoc, const uint32_t *sperm,
                                                         const uint32_t *cum, uint32_t nsurv,
                                                         uint32_t n, SurvOut *info, int32_t *counts,
                                                         gbgpu_single_score *ss, int scap, gbgpu_pair_score *ps,
                                                         int pcap, uint32_t *mt) {
  __shared__ float s_sm[npairs<MAXG>() * SCORE_TPB];
  stage_weights(&c_weights);
  const uint32_t t = blockIdx.x * SCORE_TPB + threadIdx.x;
  if (t >= n) return;
  SurvOut so{0.0f, 0, 0, -1};
  mt[t] = 0;
  const uint64_t d = tdoc[t];
  const uint32_t lo = si_rank(sdoc, nsurv, d);
  if (lo >= nsurv) {  // not a survivor: reported as ECORRUPT
    info[t] = so;
    return;
  }
  const uint32_t i = sperm[lo];
  const uint32_t s = sv_slot[i];
  const uint32_t lm = sv_lm[i];
  uint32_t kill[MAXG];
  int blid = 0;
  const int f = si_kill(pl, ctr, sv_loc, sperm, cum, nsurv, d, lo, lm, kill, &blid);
  if (f < 0) {
    so.ok = -2;
    so.pad = f * 1000 - blid;  // diagnostic (GBGPU_SI_DEBUG): which path, which list
    info[t] = so;
    return;
  }
  // the records go to a range of the global arena (a re-shrunk copy's
  // relocated range where k_ext_walk gave it one)
  unsigned long long off;
  const uint32_t units = surv_units_off(pl, ctr, s, lm, sv_u[i], &off);
  if (off == ~0ull) off = atomicAdd(&ctr->arena_top, (unsigned long long)units);
  if (off + units > arena_cap) {
    so.ok = -3;  // arena exhausted (not reached: the host sizes it for every survivor)
    info[t] = so;
    return;
  }
  ScoreRec rec{ss + (size_t)t * scap, ps + (size_t)t * pcap, 0, 0, scap, pcap};
  uint32_t key, nr, mtot = 0;
  bool stale = false;
  uint64_t tmerge = 0, tm[3] = {0, 0, 0};
  const GlobalRecs grec{(__attribute__((address_space(1))) uint64_t *)(arena + off)};
  score_survivor<MAXG, MAXSUB, GlobalRecs, ScoreRec, true>(pl, ctr, s, lm, ctr->anysurv,
                                                           sv_loc + (uint64_t)i * (uint32_t)pl->nlists, grec,
                                                           s_sm + threadIdx.x, &key, 0, &nr, false, tmerge, tm, &rec, &so,
                                                           kill, &mtot, &stale);
  if (stale) so.ok = -4;
  mt[t] = mtot;
  info[t] = so;
  counts[2 * t] = rec.ns;
  counts[2 * t + 1] = rec.np;
}

// The second pass's stale-byte docids (ok = -4 above): its docids run in tree
// order after the first pass in the same call (Posdb.cpp:6116-6160), so the 6
// bytes a stale docid's scorers read are those of the latest earlier docid of
// the second pass whose merges (getWordPosList's sublists) reached them, else
// of the first pass's last docid (vote-buffer order) that did.  One lane per
// stale docid: each writer's merge again, tapped for its bytes, then the docid
// scored and recorded with them.
struct SiStale {
  uint32_t t;      // its position in the second pass
  uint32_t O;      // its mbuf bytes (where its empty group points)
  uint32_t nb;     // bytes read there: 6, or 12 when no plain group gave it a key (siteRank, langId)
  uint32_t w[12];  // each byte's writer: a second-pass position, or 0x80000000 | a first-pass survivor index
};
__global__ void __launch_bounds__(SCORE_TPB) k_si_stale(const DevPlan *__restrict__ pl, Counters *ctr,
                                                        const uint32_t *sv_slot, const uint32_t *sv_lm,
                                                        const uint32_t *sv_u, const Loc *sv_loc, uint64_t *arena,
                                                        unsigned long long arena_cap, unsigned long long *fixc,
                                                        const uint64_t *tdoc, const uint64_t *sdoc,
                                                        const uint32_t *sperm, const uint32_t *cum, uint32_t nsurv,
                                                        const SiStale *ent, uint32_t ne, SurvOut *info,
                                                        int32_t *counts, gbgpu_single_score *ss, int scap,
                                                        gbgpu_pair_score *ps, int pcap) {
  __shared__ float s_sm[npairs<MAXG>() * SCORE_TPB];
  stage_weights(&c_weights);
  const uint32_t e = blockIdx.x * SCORE_TPB + threadIdx.x;
  if (e >= ne) return;
  const SiStale E = ent[e];
  const uint32_t anys = ctr->anysurv;
  const uint32_t nl = (uint32_t)pl->nlists;
  SurvOut so{0.0f, 0, 0, -3};  // -3 on a failed replay (capacity / a tap that missed): the host declines
  // survivor index and kill mask of second-pass position t (false: not replayable)
  auto second = [&](uint32_t t, uint32_t &i, uint32_t *kill) -> bool {
    const uint64_t d = tdoc[t];
    const uint32_t lo = si_rank(sdoc, nsurv, d);
    if (lo >= nsurv) return false;
    i = sperm[lo];
    int blid = 0;
    return si_kill(pl, ctr, sv_loc, sperm, cum, nsurv, d, lo, sv_lm[i], kill, &blid) == 0;
  };
  // room for the largest merge this lane runs (plus the injected record)
  uint32_t me = 0;
  uint32_t kill[MAXG];
  if (!second(E.t, me, kill)) {
    info[E.t] = so;
    return;
  }
  unsigned long long roff;
  uint32_t need = surv_units_off(pl, ctr, sv_slot[me], sv_lm[me], sv_u[me], &roff) + 1;
  uint32_t wi[12];
  for (uint32_t p = 0; p < E.nb; p++) {
    uint32_t k2[MAXG];
    wi[p] = E.w[p] & 0x7fffffffu;
    if (!(E.w[p] & 0x80000000u) && !second(E.w[p], wi[p], k2)) {
      info[E.t] = so;
      return;
    }
    const uint32_t u = surv_units_off(pl, ctr, sv_slot[wi[p]], sv_lm[wi[p]], sv_u[wi[p]], &roff);
    need = u > need ? u : need;
  }
  const unsigned long long off = atomicAdd(&fixc[0], (unsigned long long)need);
  if (off + need > arena_cap) {
    info[E.t] = so;
    return;
  }
  const GlobalRecs grec{(__attribute__((address_space(1))) uint64_t *)(arena + off)};
  uint32_t key = 0, nr = 0;
  uint64_t tmerge = 0, tm[3] = {0, 0, 0};
  uint64_t inj[2] = {0, 0};
  uint32_t done = 0;
  for (uint32_t p = 0; p < E.nb; p++) {
    if (done >> p & 1) continue;
    const uint32_t w = wi[p];
    const bool first = (E.w[p] & 0x80000000u) != 0;
    uint32_t k2[MAXG];
    uint32_t wdummy = 0;
    if (!first) (void)second(E.w[p], wdummy, k2);
    MbufTap tap;
    tap.lo = E.O;
    tap.got = 0;
    score_survivor<MAXG, MAXSUB, GlobalRecs, NoRec, true>(pl, ctr, sv_slot[w], sv_lm[w], anys, sv_loc + (uint64_t)w * nl,
                                                          grec, s_sm + threadIdx.x, &key, 0, &nr, false, tmerge, tm,
                                                          nullptr, nullptr, first ? nullptr : k2, nullptr, nullptr,
                                                          nullptr, &tap);
    for (uint32_t q2 = p; q2 < E.nb; q2++) {
      if (E.w[q2] != E.w[p]) continue;
      if (!(tap.got >> q2 & 1)) {
        info[E.t] = so;  // the writer's count said it reached the byte but the tap missed it: not reached
        return;
      }
      inj[q2 / 6] |= (uint64_t)tap.b[q2] << (8 * (q2 % 6));
      done |= 1u << q2;
    }
  }
  if (E.nb == 12) inj[1] |= 1ull << 63;
  ScoreRec rec{ss + (size_t)E.t * scap, ps + (size_t)E.t * pcap, 0, 0, scap, pcap};
  SurvOut so2{0.0f, 0, 0, -1};
  score_survivor<MAXG, MAXSUB, GlobalRecs, ScoreRec, true>(pl, ctr, sv_slot[me], sv_lm[me], anys,
                                                           sv_loc + (uint64_t)me * nl, grec, s_sm + threadIdx.x, &key, 0,
                                                           &nr, false, tmerge, tm, &rec, &so2, kill, nullptr, nullptr,
                                                           inj, nullptr);
  info[E.t] = so2;
  counts[2 * E.t] = rec.ns;
  counts[2 * E.t + 1] = rec.np;
}

// ------------------------------------------------------ stale-mbuf replay
// A survivor whose trailing merged group came out empty (its only keys there
// were BF_BIGRAM keys with syn bits, Posdb.cpp:6687-6692) has every scorer
// read the 6 mbuf bytes at that group's place, which the docid's own merges
// never reach: the reference reads what the docids before it in the pass left
// there (mbuf is a local of intersectLists10_r, Posdb.cpp:6007; each docid's
// merges write it from the start, 6559).  k_score drops such survivors and
// lists them; after the pass (stale_fix), in vote-buffer (docid) order:
//   k_stale_find  each stale survivor's writer of each of the 6 bytes -- the
//                 latest earlier docid whose merges wrote past it -- or none
//                 (the stack's bytes: undefined, the docid stays dropped);
//   k_stale_fix   the writers' merges again, tapped for those bytes, then the
//                 survivor scored with them where its empty group points.
__global__ void k_gather_docs(const uint64_t *doc, const uint32_t *pos, const Counters *ctr, uint64_t *out) {
  for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < ctr->nstale; e += gridDim.x * blockDim.x) out[e] = doc[pos[e] & 0x7fffffffu];
}

__global__ void k_stale_rank(const uint32_t *order, uint32_t n, uint32_t *rank) {
  for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) rank[order[k]] = k;
}

constexpr uint32_t STALE_SCAN = 1u << 20;  // docids a writer search walks back at most (beyond: EUNSUPPORTED)

// skip (site clustering; null: none): survivors the replay's prefilter
// skipped, which run no merges and write no mbuf byte (Posdb.cpp:6341-6345)
__global__ void k_stale_find(Counters *ctr, const uint32_t *stale, const uint32_t *sv_mb, const uint32_t *order,
                             const uint32_t *rank, uint32_t *wr, const uint8_t *skip) {
  const uint32_t ns = ctr->nstale;
  for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < ns; e += gridDim.x * blockDim.x) {
    const uint32_t si = stale[e] & 0x7fffffffu;
    const uint32_t nb = (stale[e] >> 31) ? 12u : 6u;  // 12: its siteRank / langId are read there too
    const uint32_t O = sv_mb[si];
    uint32_t w12[12];
#pragma unroll
    for (int p = 0; p < 12; p++) w12[p] = ~0u;
    uint32_t need = 0, steps = 0;
    for (int64_t j = (int64_t)rank[si] - 1; j >= 0 && need < nb; j--) {
      if (++steps > STALE_SCAN) {
        ctr->unsup = 1;
        break;
      }
      const uint32_t w = order[j];
      if (skip && skip[w]) continue;
      const uint32_t T = sv_mb[w];
      if (T > O + need) {
        const uint32_t upto = min(nb, T - O);
#pragma unroll
        for (int p = 0; p < 12; p++)
          if ((uint32_t)p >= need && (uint32_t)p < upto) w12[p] = w;
        need = upto;
      }
    }
#pragma unroll
    for (int p = 0; p < 12; p++) wr[(size_t)e * 12 + p] = w12[p];
  }
}

// a survivor's record units, as k_score sizes its store (its re-shrunk copies
// grow by E units each)
__device__ __forceinline__ uint32_t surv_units(const DevPlan *__restrict__ pl, const Counters *ctr, uint32_t s, uint32_t lm,
                                               uint32_t u) {
  for (uint32_t x = lm & pl->reshare_mask; x; x &= x - 1) {
    const int l = __ffs(x) - 1;
    const ListExt &e = ctr->ext[l];
    if (e.slot1 == s + 1) u += e.E * (uint32_t)(pl->lists[l].uses - 1);
  }
  return u;
}

// every survivor's mbuf bytes (its merges again, no scoring), one lane each:
// only for a pass with stale survivors
__global__ void __launch_bounds__(SCORE_TPB) k_stale_mb(const DevPlan *__restrict__ pl, Counters *ctr, uint32_t nsurv,
                                                        const uint32_t *sv_slot, const uint32_t *sv_lm, const uint32_t *sv_u,
                                                        const Loc *sv_loc, uint64_t *arena, unsigned long long arena_cap,
                                                        unsigned long long *fixc, uint32_t *sv_mb, uint32_t *stale) {
  __shared__ float s_sm[npairs<MAXG>() * SCORE_TPB];
  stage_weights(&c_weights);
  const uint32_t i = blockIdx.x * SCORE_TPB + threadIdx.x;
  if (i >= nsurv) return;
  const uint32_t nl = (uint32_t)pl->nlists;
  const uint32_t need = surv_units(pl, ctr, sv_slot[i], sv_lm[i], sv_u[i]) + 1;
  const unsigned long long off = atomicAdd(&fixc[0], (unsigned long long)need);
  if (off + need > arena_cap) {
    ctr->unsup = 1;  // the host sized the arena for every survivor: not reached
    return;
  }
  const GlobalRecs grec{(__attribute__((address_space(1))) uint64_t *)(arena + off)};
  uint32_t key = 0, nr = 0, mt = 0;
  bool st = false;
  uint64_t tmerge = 0, tm[3] = {0, 0, 0};
  MbufTap tap;
  tap.lo = ~0u - 8;  // no byte: the count only
  tap.got = 0;
  score_survivor<MAXG, MAXSUB, GlobalRecs, NoRec, true>(pl, ctr, sv_slot[i], sv_lm[i], ctr->anysurv,
                                                        sv_loc + (uint64_t)i * nl, grec, s_sm + threadIdx.x, &key, 0,
                                                        &nr, false, tmerge, tm, nullptr, nullptr, nullptr, &mt, &st,
                                                        nullptr, &tap);
  sv_mb[i] = mt;
  // the list k_stale_find walks (bit 31: no plain group gave a key, so its
  // siteRank / langId come from the stale bytes too)
  if (st) stale[atomicAdd((uint32_t *)&fixc[1], 1u)] = i | (key ? 0x80000000u : 0u);
}

// one lane per stale survivor; okey: its key (0: undefined bytes, not
// scored, or dropped by the paging filter); fixc[0] the fix arena's top,
// fixc[1] the paging filter's count
__global__ void __launch_bounds__(SCORE_TPB) k_stale_fix(const DevPlan *__restrict__ pl, Counters *ctr, const uint32_t *stale,
                                                         const uint32_t *wr, const uint32_t *sv_mb, const uint32_t *sv_slot,
                                                         const uint32_t *sv_lm, const uint32_t *sv_u, const uint64_t *sv_doc,
                                                         const Loc *sv_loc, uint64_t *arena, unsigned long long arena_cap,
                                                         unsigned long long *fixc, uint32_t *skey, uint32_t *okey,
                                                         uint8_t *sflag) {
  __shared__ float s_sm[npairs<MAXG>() * SCORE_TPB];
  stage_weights(&c_weights);
  const uint32_t e = blockIdx.x * SCORE_TPB + threadIdx.x;
  const uint32_t ns = ctr->nstale;
  if (e >= ns) return;
  const uint32_t anys = ctr->anysurv;
  const uint32_t nl = (uint32_t)pl->nlists;
  const uint32_t i = stale[e] & 0x7fffffffu;
  const uint32_t nb = (stale[e] >> 31) ? 12u : 6u;
  uint32_t w6[12];
  bool defined = true;
#pragma unroll
  for (int p = 0; p < 12; p++) {
    w6[p] = wr[(size_t)e * 12 + p];
    defined &= (uint32_t)p >= nb || w6[p] != ~0u;
  }
  okey[e] = 0;
  if (sflag) sflag[i] = 0;
  if (!defined) {  // bytes no docid of the pass wrote: the docid stays dropped
    skey[i] = 0;
    return;
  }
  // room for the largest merge this lane runs (plus the injected record)
  uint32_t need = surv_units(pl, ctr, sv_slot[i], sv_lm[i], sv_u[i]) + 1;
  for (uint32_t p = 0; p < nb; p++) {
    const uint32_t w = w6[p];
    const uint32_t u = surv_units(pl, ctr, sv_slot[w], sv_lm[w], sv_u[w]);
    need = u > need ? u : need;
  }
  const unsigned long long off = atomicAdd(&fixc[0], (unsigned long long)need);
  if (off + need > arena_cap) {
    ctr->unsup = 1;  // the host sized the fix arena for every stale survivor: not reached
    return;
  }
  const GlobalRecs grec{(__attribute__((address_space(1))) uint64_t *)(arena + off)};
  uint32_t key = 0, nr = 0;
  uint64_t tmerge = 0, tm[3] = {0, 0, 0};
  // the writers' bytes at [O, O + 6), each writer's merges once
  const uint32_t O = sv_mb[i];
  uint64_t inj[2] = {0, 0};  // bytes 0-5, 6-11
  uint32_t done = 0;
  for (uint32_t p = 0; p < nb; p++) {
    if (done >> p & 1) continue;
    const uint32_t w = w6[p];
    MbufTap tap;
    tap.lo = O;
    tap.got = 0;
    score_survivor<MAXG, MAXSUB, GlobalRecs, NoRec, true>(pl, ctr, sv_slot[w], sv_lm[w], anys, sv_loc + (uint64_t)w * nl,
                                                          grec, s_sm + threadIdx.x, &key, 0, &nr, false, tmerge, tm,
                                                          nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, &tap);
    for (uint32_t q = p; q < nb; q++) {
      if (w6[q] != w) continue;
      if (!(tap.got >> q & 1)) {
        ctr->unsup = 1;  // the writer wrote past the byte (sv_mb) but the tap missed it: not reached
        return;
      }
      inj[q / 6] |= (uint64_t)tap.b[q] << (8 * (q % 6));
      done |= 1u << q;
    }
  }
  if (nb == 12) inj[1] |= 1ull << 63;
  // the survivor itself, the bytes where its empty group points
  score_survivor<MAXG, MAXSUB, GlobalRecs, NoRec, true>(pl, ctr, sv_slot[i], sv_lm[i], anys, sv_loc + (uint64_t)i * nl,
                                                        grec, s_sm + threadIdx.x, &key, 0, &nr, false, tmerge, tm,
                                                        nullptr, nullptr, nullptr, nullptr, nullptr, inj, nullptr);
  // the paging filter (Posdb.cpp:7327-7347), as k_score applies it
  if (pl->has_serp && key) {
    const uint64_t d = sv_doc[i];
    bool filt = false;
    if (pl->sortby_group >= 0 && pl->sortby_int) {
      const int32_t iv = (int32_t)(key ^ 0x80000000u);
      if (iv > pl->max_serp_int) filt = true;
      else if (iv == pl->max_serp_int && (int64_t)d <= pl->min_serp_docid) filt = true;
    } else {
      const uint32_t b2 = (key & 0x80000000u) ? (key & 0x7fffffffu) : ~key;
      const float score = __uint_as_float(b2);
      if (score > (float)pl->max_serp_score) filt = true;
      else if ((double)score == pl->max_serp_score && (int64_t)d <= pl->min_serp_docid) filt = true;
    }
    if (filt) {
      key = 0;
      atomicAdd(&fixc[1], 1ull);
      if (sflag) sflag[i] = 1;  // site clustering: the replay counts it (m_filtered)
    }
  }
  skey[i] = key;
  okey[e] = key;
}

// site clustering: which survivors the replay's prefilter skipped -- its
// bound B <= minWinningScore at its turn, the value the last add of an
// earlier docid assigned (the replay records each assignment with that
// docid, in docid order; before the first one -1.0, Posdb.cpp:6012)
__global__ void k_stale_skip(uint32_t nsurv, const uint64_t *sv_doc, const uint32_t *sv_ord, const uint4 *rep_slot,
                             const uint4 *mwsl, int ints, uint8_t *skip) {
  const uint32_t nm = mwsl[0].x;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nsurv; i += gridDim.x * blockDim.x) {
    const uint64_t d = sv_doc[i];
    const float B = __uint_as_float(rep_slot[sv_ord[i]].y);
    uint32_t lo = 0, hi = nm;  // assignments from docids below d
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      const uint4 a = mwsl[1 + mid];
      if ((((uint64_t)a.y << 32) | a.x) < d) lo = mid + 1;
      else hi = mid;
    }
    const float mws = lo ? __uint_as_float(mwsl[lo].z) : -1.0f;
    skip[i] = (!ints && B <= mws) ? 1 : 0;
  }
}

// ------------------------------------------------------- site clustering
// With m_doSiteClustering (the Msg39Request default, Msg39.h:41) the TopTree
// keeps per-domain caps (TopTree.cpp:64-186, 312-516), so it holds more than
// docsWanted nodes, minWinningScore becomes live (Posdb.cpp:7699-7704) and
// the two prefilters skip docids whose bound cannot beat it (Posdb.cpp:
// 6322-6504).  The reference decides docid by docid in vote-buffer order.
// Here every survivor is scored in parallel as usual, and additionally
//   k_bound        its prefilter bound B = min of the getMaxPossibleScore
//                  values of both prefilters (-1, "has inlink text", ignored),
//                  one wave per survivor, the 4096-slot ring buffer in LDS;
//   k_rank         (several candidate arrays) its position in docid order;
//   k_tree_replay  ONE wave replays the docid-order loop exactly: a docid is
//                  skipped iff B <= minWinningScore, else offered to the
//                  TopTree with the domain caps.  Offers that cannot change
//                  the tree (skipped, unscored, or not better than the low
//                  node of a full tree) are ruled out 64 at a time with a
//                  ballot; only the others take the sequential path.
constexpr int BND_WAVES = 4;
constexpr int RING = 4096;     // RINGBUFSIZE, Posdb.cpp:6019
constexpr int TC = 10240;      // TopTree nodes the replay keeps in LDS

// getMaxPossibleScore (Posdb.cpp:7811-7960) up to its request- and
// pair-specific tail: the best hash-group weight and density rank over the
// group's runs, scanned backwards (12-byte run head last), and the siteRank /
// langId of its first run.  state: -1 inlink text (returns -1.0), 0 nothing
// found (returns 0.0), 1 a score (base = 100*hgw^2*dw^2*... *tfw_i)
struct BoundCore {
  int state;
  float base;
};

__device__ __forceinline__ float max_score_tail(const DevPlan *__restrict__ pl, BoundCore c, float tfw_m, int32_t bestDist,
                                                int32_t qdist) {
  if (c.state <= 0) return c.state < 0 ? -1.0f : 0.0f;
  float score = c.base;
  if (qdist) {  // Posdb.cpp:7935-7946
    score *= tfw_m;
    bestDist -= qdist;
    if (bestDist < 0) bestDist *= -1;
    if (bestDist > 1) score /= (float)bestDist;
  }
  if (pl->all_same_wiki) score *= GB_WIKI_WEIGHT;
  return score;
}

__device__ BoundCore group_bound_core(const DevPlan *__restrict__ pl, const Counters *ctr, int g, uint32_t s, uint32_t lm,
                                      const Loc *svl) {
  const Weights &W = s_weights;
  float best = -1.0f;
  unsigned bestDR = 0;
  int sr = -1, lang = 0;
  bool hs = false;
  const int gns = pl->gnsub[g];
  for (int x = 0; x < gns; x++) {
    const int lid = pl->gsub[g][x];
    if (!(lm >> lid & 1)) continue;  // m_savedCursor[j] == NULL
    if (pl->gflags0[g] & BF_HALFSTOPWIKIBIGRAM) hs = true;
    const SubRun run = sub_run_at(pl, ctr, svl[lid], lid, g, x, s);
    if (sr == -1) {  // getSiteRank / getLangId of the 12-byte run head
      const uint64_t v0 = load6(run.own), v6 = load6(run.own + 6);  // (two 6-byte loads, not bytes)
      const uint32_t b0 = (uint32_t)v0 & 0xff, b6 = (uint32_t)v6 & 0xff, b7 = (uint32_t)(v6 >> 8) & 0xff;
      sr = (int)(((b6 >> 5) | ((b7 & 1) << 3)) & 0x0f);
      lang = (int)((b6 & 0x1f) | ((b0 & 0x08) ? 0x20 : 0));
    }
    // keys from the last 6-byte key down to the first one, then the head
    // (Posdb.cpp:7851-7897); a body key weaker than the best ends the list
    for (int k = (int)run.len - 1; k >= 0; k--) {
      if (k == 1) continue;  // second half of the 12-byte head
      const uint64_t dv = load6(run.key((uint32_t)k));
      const uint32_t hg = (uint32_t)(dv >> 26) & 0x0f;  // byte 3 >> 2
      if (hg == GB_HG_INLINKTEXT) return BoundCore{-1, 0.0f};
      const float w = W.hashgroup[hg];
      if (w < best) {
        if (hg == GB_HG_BODY) break;
        continue;
      }
      const unsigned dr = (unsigned)(dv >> 11) & 0x1f;  // byte 1 >> 3
      if (w > best) {
        best = w;
        bestDR = dr;
        continue;
      }
      if (dr < bestDR) continue;
      if (dr > bestDR) bestDR = dr;
    }
  }
  if (best < 0) return BoundCore{0, 0.0f};
  float score = 100.0;
  score *= best;
  score *= best;
  score *= W.density[bestDR];
  score *= W.density[bestDR];
  if (hs) {
    score *= GB_WIKI_BIGRAM_WEIGHT;
    score *= GB_WIKI_BIGRAM_WEIGHT;
  }
  score *= (((float)sr) * pl->site_rank_multiplier + 1.0);
  if (pl->language == lang || pl->language == 0 || lang == 0) score *= pl->same_lang_weight;
  score *= pl->tfw[g];
  return BoundCore{1, score};
}

// a key's ring-buffer slot: its word position (bytes 2-5 >> 14) mod RING
__device__ __forceinline__ uint32_t ring_slot(gu8 *kp) {  // bytes 2-5 >> 14: the word position
  return ((uint32_t)(load6(kp) >> 16) >> 14) & (RING - 1);
}
// ring-buffer slots this wave's lanes write for one group's runs (value v);
// returns the slot of the head of the group's last run (ourFirstPos)
__device__ int ring_fill(const DevPlan *__restrict__ pl, const Counters *ctr, int g, uint32_t s, uint32_t lm, const Loc *svl,
                         uint8_t *ring, uint8_t v, int lane) {
  int first = -1;
  const int gns = pl->gnsub[g];
  for (int x = 0; x < gns; x++) {
    const int lid = pl->gsub[g][x];
    if (!(lm >> lid & 1)) continue;
    const SubRun run = sub_run_at(pl, ctr, svl[lid], lid, g, x, s);
    for (uint32_t k = lane; k < run.len; k += 64) {
      if (k == 1) continue;
      ring[ring_slot(run.key(k))] = v;
    }
    first = (int)ring_slot(run.own);
  }
  return first;
}

// ordered summary of a stretch of ring slots holding the min group (type 0)
// or the probed group (type 1): the closest different-type neighbours
struct RingSum {
  int fpos, ftype, lpos, ltype, gap, lastm;  // fpos < 0: nothing
};
__device__ __forceinline__ RingSum ring_join(RingSum a, RingSum b) {
  if (a.fpos < 0) return RingSum{b.fpos, b.ftype, b.lpos, b.ltype, b.gap, b.lastm >= 0 ? b.lastm : a.lastm};
  if (b.fpos < 0) return a;
  RingSum r;
  r.fpos = a.fpos;
  r.ftype = a.ftype;
  r.lpos = b.lpos;
  r.ltype = b.ltype;
  r.gap = min(a.gap, b.gap);
  if (a.ltype != b.ftype) r.gap = min(r.gap, b.fpos - a.lpos);
  r.lastm = b.lastm >= 0 ? b.lastm : a.lastm;
  return r;
}

// Posdb.cpp:6445-6485 for group i: the smallest distance between a slot of
// the min group and a slot of group i (scan order), and the wrap distance
__device__ int32_t ring_best_dist(const uint8_t *ring, uint8_t m, uint8_t i, int ourFirstPos, int lane) {
  RingSum r{-1, 0, -1, 0, 0x7fffffff, -1};
  const uint32_t *w = reinterpret_cast<const uint32_t *>(ring) + lane * 16;
  for (int q = 0; q < 16; q++) {
    const uint32_t v4 = w[q];
    if (v4 == 0xffffffffu) continue;
#pragma unroll
    for (int b = 0; b < 4; b++) {
      const uint8_t v = (uint8_t)(v4 >> (8 * b));
      if (v != m && v != i) continue;
      const int pos = lane * 64 + q * 4 + b;
      const int t = v == m ? 0 : 1;
      if (r.fpos < 0) {
        r.fpos = pos;
        r.ftype = t;
      } else if (t != r.ltype) {
        r.gap = min(r.gap, pos - r.lpos);
      }
      r.lpos = pos;
      r.ltype = t;
      if (t == 0) r.lastm = pos;
    }
  }
  // ordered reduction: lane l joins lane l+off, lane 0 ends with the whole ring
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    RingSum o;
    o.fpos = __shfl_down(r.fpos, off, 64);
    o.ftype = __shfl_down(r.ftype, off, 64);
    o.lpos = __shfl_down(r.lpos, off, 64);
    o.ltype = __shfl_down(r.ltype, off, 64);
    o.gap = __shfl_down(r.gap, off, 64);
    o.lastm = __shfl_down(r.lastm, off, 64);
    if ((lane & (2 * off - 1)) == 0) r = ring_join(r, o);
  }
  int32_t bestDist = __shfl(r.gap, 0, 64);
  const int hisLastPos = __shfl(r.lastm, 0, 64);
  const int32_t wrapDist = ourFirstPos + (RING - hisLastPos);
  if (wrapDist < bestDist) bestDist = wrapDist;
  return bestDist;
}

// one replay entry (16 B, docid order): score key, prefilter bound, docid
// with bit 63 set when the paging test filtered it (k_score's sflag)
__device__ __forceinline__ uint4 rep_entry(uint32_t key, float B, uint64_t d, bool serp) {
  if (serp) d |= 1ull << 63;
  return make_uint4(key, __float_as_uint(B), (uint32_t)d, (uint32_t)(d >> 32));
}

// The ring-buffer filter restated on a survivor's own word positions, one
// lane per survivor: the ring after group m and the groups written before g
// holds, for g's scan, m at the slots (wordPos mod 4096) of m's keys that no
// group written since overwrote, and g at g's slots; the reference's scan
// (Posdb.cpp:6445-6485) then finds the smallest distance between
// neighbouring slots of different types -- the same as between any m slot
// and the last g slot before it or vice versa -- and the wrap distance from
// m's last slot round to ourFirstPos (the head slot of m's last sublist).
// The slots go to per-lane LDS columns; a survivor with more than BL_SLOTS
// keys in a group takes the wave's 4096-slot ring (the reference's own
// buffer) instead.
#ifndef GBGPU_BL_SLOTS
#define GBGPU_BL_SLOTS 32
#endif
constexpr int BL_SLOTS = GBGPU_BL_SLOTS;
// group g's slots into col[0..n) (column layout: entry k of lane at [k][lane]);
// false on overflow.  first: the head slot of the last present sublist.
__device__ bool lane_slots(const DevPlan *__restrict__ pl, const Counters *ctr, int g, uint32_t s, uint32_t lm,
                           const Loc *svl, uint16_t (*col)[64], int lane, int &n, int &first) {
  n = 0;
  const int gns = pl->gnsub[g];
  for (int x = 0; x < gns; x++) {
    const int lid = pl->gsub[g][x];
    if (!(lm >> lid & 1)) continue;
    const SubRun run = sub_run_at(pl, ctr, svl[lid], lid, g, x, s);
    for (uint32_t k = 0; k < run.len; k++) {
      if (k == 1) continue;  // the second half of the 12-byte head
      if (n == BL_SLOTS) return false;
      col[n++][lane] = (uint16_t)ring_slot(run.key(k));
    }
    first = (int)ring_slot(run.own);
  }
  return true;
}
__device__ void lane_sort(uint16_t (*col)[64], int n, int lane) {
  for (int a = 1; a < n; a++) {
    const uint16_t v = col[a][lane];
    int b = a - 1;
    while (b >= 0 && col[b][lane] > v) {
      col[b + 1][lane] = col[b][lane];
      b--;
    }
    col[b + 1][lane] = v;
  }
}

// The replay entry of record i goes to its slot-order rank sv_ord[i]: with
// one candidate array that is docid order (the replay's input), else k_rank
// merges the arrays (oslot: each rank's slot).  A block
// of BND_WAVES waves, one lane per survivor (the ring restated above); the
// survivors whose lists overflow a lane's slot columns then take the wave
// one at a time, over the 4096-slot ring.
__global__ void __launch_bounds__(64 * BND_WAVES) k_bound(const DevPlan *__restrict__ pl, const Counters *ctr,
                                                       const uint32_t *sv_slot, const uint32_t *sv_lm,
                                                       const Loc *sv_loc, const uint32_t *sv_ord, const uint32_t *skey,
                                                       const uint64_t *sdoc, const uint8_t *sflag, uint4 *rep,
                                                       uint32_t *oslot) {
  __shared__ __attribute__((aligned(16))) uint8_t s_ring[BND_WAVES][RING];
  __shared__ uint16_t s_ms[BND_WAVES][BL_SLOTS][64], s_gs[BND_WAVES][BL_SLOTS][64];
  stage_weights(&c_weights);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint8_t *ring = s_ring[wid];
  uint16_t(*ms)[64] = s_ms[wid];
  uint16_t(*gs)[64] = s_gs[wid];
  const uint32_t nsurv = (uint32_t)(ctr->surv_top >> 36);
  const int ng = pl->ngroups, m = pl->min_listi;
  const float INF = __int_as_float(0x7f800000);
  const float tfw_m = pl->tfw[m];
  // gbsortby: both prefilters are skipped (Posdb.cpp:6050-6051, 6350); a
  // boolean query jumps over them (Posdb.cpp:6312-6316)
  const bool sortby = pl->sortby_group >= 0 || pl->boolean;
  for (uint32_t base = (blockIdx.x * BND_WAVES + wid) * 64u; base < nsurv; base += gridDim.x * BND_WAVES * 64u) {
    const uint32_t i = base + lane;
    float B = INF;
    bool over = false;
    if (i < nsurv && !sortby) {
      const uint32_t s = sv_slot[i], lm = sv_lm[i];
      const Loc *svl = sv_loc + (uint64_t)i * (uint32_t)pl->nlists;
      int nm = 0, ourFirstPos = -1;
      over = !lane_slots(pl, ctr, m, s, lm, svl, ms, lane, nm, ourFirstPos);
      if (!over) lane_sort(ms, nm, lane);
      for (int g = 0; g < ng && !over; g++) {
        if (pl->gflags0[g] & (BF_NEGATIVE | BF_FACET)) continue;
        const BoundCore core = group_bound_core(pl, ctr, g, s, lm, svl);
        // filter 1 (m_doMaxScoreAlgo): bestDist 0, qdist 0 (Posdb.cpp:6327-6346)
        if (pl->do_max_score) {
          const float v = max_score_tail(pl, core, 1.0f, 0, 0);
          if (v != -1.0f) B = fminf(B, v);
        }
        if (g == m || pl->has_facet) continue;  // a facet term skips filter 2 (Posdb.cpp:6353-6356)
        // filter 2 (Posdb.cpp:6364-6504): g's keys are written over the ring
        // whatever its bound, then scanned against m's survivors there
        int ngs = 0, dummy = -1;
        if (!lane_slots(pl, ctr, g, s, lm, svl, gs, lane, ngs, dummy)) {
          over = true;
          break;
        }
        lane_sort(gs, ngs, lane);
        // m slots g overwrote (both sorted): gone for this and later groups
        for (int a = 0, b = 0; a < nm && b < ngs;) {
          const uint16_t x = ms[a][lane], y = gs[b][lane];
          if (x == 0xffffu) break;  // removed slots sort last
          if (x < y) a++;
          else if (x > y) b++;
          else ms[a++][lane] = 0xffffu;
        }
        lane_sort(ms, nm, lane);
        if (core.state < 0) continue;  // -1: not applied
        int32_t bestDist = 0x7fffffff, hisLastPos = -1;
        int prev = -1, ptype = -1;
        for (int a = 0, b = 0; a < nm || b < ngs;) {
          const int x = a < nm ? (int)ms[a][lane] : 0xffff, y = b < ngs ? (int)gs[b][lane] : 0xffff;
          if (x == 0xffff && y == 0xffff) break;
          int cur, t;
          if (x < y) {
            cur = x, t = 0, a++;
            hisLastPos = x;
          } else {
            cur = y, t = 1, b++;
          }
          if (prev >= 0 && t != ptype) bestDist = min(bestDist, cur - prev);
          prev = cur, ptype = t;
        }
        const int32_t wrapDist = ourFirstPos + (RING - hisLastPos);
        if (wrapDist < bestDist) bestDist = wrapDist;
        const float v = max_score_tail(pl, core, tfw_m, bestDist, pl->qpos[m] - pl->qpos[g]);
        if (v != -1.0f) B = fminf(B, v);
      }
    }
    // overflowing survivors: the whole wave, one at a time, over the ring
    for (uint64_t om = __ballot(over); om; om &= om - 1) {
      const int j = __ffsll((unsigned long long)om) - 1;
      const uint32_t ij = base + (uint32_t)j;
      const uint32_t s = sv_slot[ij], lm = sv_lm[ij];
      const Loc *svl = sv_loc + (uint64_t)ij * (uint32_t)pl->nlists;
      // lane g: getMaxPossibleScore's scan of group g
      BoundCore core{0, 0.0f};
      if (lane < ng && !(pl->gflags0[lane] & (BF_NEGATIVE | BF_FACET))) core = group_bound_core(pl, ctr, lane, s, lm, svl);
      float Bw = INF;
      if (pl->do_max_score && lane < ng && !(pl->gflags0[lane] & (BF_NEGATIVE | BF_FACET))) {
        const float v = max_score_tail(pl, core, 1.0f, 0, 0);
        if (v != -1.0f) Bw = v;
      }
      uint4 *r4 = reinterpret_cast<uint4 *>(ring);
      for (int q = lane; q < RING / 16; q += 64) r4[q] = make_uint4(~0u, ~0u, ~0u, ~0u);
      wave_lds_sync();
      const int ourFirstPos = ring_fill(pl, ctr, m, s, lm, svl, ring, (uint8_t)m, lane);
      for (int g = 0; g < ng && !pl->has_facet; g++) {
        if (g == m || (pl->gflags0[g] & (BF_NEGATIVE | BF_FACET))) continue;
        wave_lds_sync();
        ring_fill(pl, ctr, g, s, lm, svl, ring, (uint8_t)g, lane);
        wave_lds_sync();
        BoundCore cg;
        cg.state = __shfl(core.state, g, 64);
        cg.base = __shfl(core.base, g, 64);
        if (cg.state < 0) continue;  // -1: not applied
        const int32_t bestDist = ring_best_dist(ring, (uint8_t)m, (uint8_t)g, ourFirstPos, lane);
        const float v = max_score_tail(pl, cg, tfw_m, bestDist, pl->qpos[m] - pl->qpos[g]);
        if (lane == 0 && v != -1.0f) Bw = fminf(Bw, v);
      }
      wave_lds_sync();
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) Bw = fminf(Bw, __shfl_xor(Bw, off, 64));
      if (lane == j) B = Bw;
    }
    if (i < nsurv) {
      const uint32_t o = sv_ord[i];
      rep[o] = rep_entry(skey[i], B, sdoc[i], sflag[i] != 0);
      if (oslot) oslot[o] = sv_slot[i];
    }
  }
}

// position of each survivor in docid order when the smallest group has
// several candidate arrays (each array's survivors are docid-sorted and no
// docid survives in two arrays: the probe credits it to the first)
__device__ __forceinline__ uint32_t lower_bound_u32(const uint32_t *a, uint32_t n, uint32_t v) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (a[mid] < v) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// repo: the entries in slot order (k_bound), oslot their slots
__device__ __forceinline__ uint64_t rep_doc(const uint4 &e) { return ((uint64_t)(e.w & 0x7fffffffu) << 32) | e.z; }
__device__ __forceinline__ uint32_t rep_lower(const uint4 *a, uint32_t lo, uint32_t hi, uint64_t v) {
  const uint32_t b = lo;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (rep_doc(a[mid]) < v) lo = mid + 1;
    else hi = mid;
  }
  return lo - b;
}
__global__ void k_rank(const DevPlan *__restrict__ pl, const Counters *ctr, const uint32_t *oslot, const uint4 *repo,
                       uint4 *rep) {
  const uint32_t nsurv = (uint32_t)(ctr->surv_top >> 36);
  const int g0n = pl->g0n;
  uint32_t sb[MAXG0 + 1];
  for (int k = 0; k <= g0n; k++)
    sb[k] = k == g0n ? nsurv : lower_bound_u32(oslot, nsurv, (uint32_t)pl->g0base[k]);
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nsurv; i += gridDim.x * blockDim.x) {
    int k = 0;
    while (k + 1 < g0n && i >= sb[k + 1]) k++;
    const uint4 e = repo[i];
    const uint64_t d = rep_doc(e);
    uint32_t pos = i - sb[k];
    for (int k2 = 0; k2 < g0n; k2++)
      if (k2 != k) pos += rep_lower(repo, sb[k2], sb[k2 + 1], d);
    rep[pos] = e;
  }
}

// TopTree state carried between the pieces of a docid-split query (Msg39's
// one tree over every piece, Msg39.cpp:345-457)
struct TreeState {
  uint32_t n;
  float vcount;
  int32_t dom[256];
  float score[TC];
  uint64_t docid[TC];
};

struct TreeParams {
  int32_t docs_wanted;  // m_docsWanted
  int32_t cap;          // m_cap
  float partial;        // m_partial
  int32_t emit;         // write the tree out without ending it (the second pass of a docid-split piece)
  int64_t ridiculous;   // m_ridiculousMax
  int64_t num_nodes;    // m_numNodes
  uint32_t init, final; // first / last piece
  int32_t ints;          // m_useIntScores: nodes ordered by m_intScore (TopTree.cpp:216-219, 270-274)
  int32_t on_reg_err;    // run only if k_tree_seq's register tree overflowed (tree_err == TREE_ERR_REG)
  // facet terms with site clustering: every minWinningScore assignment as
  // {docid lo, docid hi, score bits, 0} from [1], the count in [0].x (the
  // facet votes of the docids the prefilter did not skip, k_facet_live)
  uint4 *mwsl;
};

// Node scores: m_score, or with integer tree scores m_intScore kept as the
// float slot's bit pattern (ints): compared as int32, and the domain tree's
// key score cs = (uint32_t)m_intScore (TopTree.cpp:332-335)
__device__ __forceinline__ bool sc_gt(float a, float b, bool ints) {
  return ints ? __float_as_int(a) > __float_as_int(b) : a > b;
}
__device__ __forceinline__ bool sc_eq(float a, float b, bool ints) {
  return ints ? __float_as_int(a) == __float_as_int(b) : a == b;
}
__device__ __forceinline__ uint32_t tree_cs(float s, bool ints) {
  if (ints) return (uint32_t)__float_as_int(s);
  // (uint32_t)m_score as x86-64 converts a float: the low 32 bits of its
  // 64-bit truncation (cvttss2si; 0x8000000000000000 when out of range)
  if (!(s > -9.2233720368547758e18f && s < 9.2233720368547758e18f)) return 0u;
  return (uint32_t)(uint64_t)(int64_t)s;
}
__device__ __forceinline__ bool node_better(float s1, uint64_t d1, float s2, uint64_t d2, bool ints = false) {
  return sc_gt(s1, s2, ints) || (sc_eq(s1, s2, ints) && d1 < d2);
}
__device__ __forceinline__ uint32_t dom_hash8(uint64_t d) { return (uint32_t)((d & 0x3fc0ull) >> 6); }  // Titledb.h:114-115

// index of the first node (best-first order) not better than (s, d)
__device__ uint32_t tree_lower_bound(const float *ts, const uint64_t *td, uint32_t n, float s, uint64_t d, int lane,
                                     bool ints) {
  uint32_t lo = 0, hi = n;
  while (hi - lo > 64) {
    const uint32_t step = (hi - lo + 63) / 64;
    const uint32_t idx = lo + lane * step;
    const uint32_t c = (uint32_t)__popcll(__ballot(idx < hi && node_better(ts[idx], td[idx], s, d, ints)));
    if (c == 0) return lo;
    const uint32_t nlo = lo + (c - 1) * step + 1;
    hi = min(hi, lo + c * step);
    lo = nlo;
  }
  const uint32_t idx = lo + lane;
  return lo + (uint32_t)__popcll(__ballot(idx < hi && node_better(ts[idx], td[idx], s, d, ints)));
}

// deleteNode's count bookkeeping (TopTree.cpp:543-547) and removal of node q
__device__ void tree_delete(float *ts, uint64_t *td, int32_t *dom, uint32_t &n, float &vcount, const TreeParams &tp,
                            uint32_t q, uint32_t dh, int lane) {
  if (dom[dh] < tp.cap) vcount -= 1.0;
  else if (dom[dh] == tp.cap) vcount -= tp.partial;
  wave_lds_sync();
  if (lane == 0) dom[dh]--;
  for (uint32_t b = q; b + 1 < n; b += 64) {
    const uint32_t idx = b + 1 + lane;
    float v = 0.0f;
    uint64_t w = 0;
    if (idx < n) {
      v = ts[idx];
      w = td[idx];
    }
    wave_lds_sync();
    if (idx < n) {
      ts[idx - 1] = v;
      td[idx - 1] = w;
    }
    wave_lds_sync();
  }
  n--;
  wave_lds_sync();
}

// TopTree::addNode (TopTree.cpp:206-516) on the best-first node array; every
// lane runs it (uniform), the array work is spread over the wave
__device__ void tree_add(float *ts, uint64_t *td, int32_t *dom, uint32_t &n, float &vcount, const TreeParams &tp,
                         float s, uint64_t d, uint32_t &err, int lane) {
  const uint32_t dh = dom_hash8(d);
  const bool ints = tp.ints != 0;
  if (vcount >= tp.docs_wanted) {
    if (!node_better(s, d, ts[n - 1], td[n - 1], ints)) return;
  }
  const uint32_t p = tree_lower_bound(ts, td, n, s, d, lane, ints);
  if (p < n && sc_eq(ts[p], s, ints) && td[p] == d) return;  // "if equal do not replace"
  const uint32_t cs = tree_cs(s, ints);
  bool del = false;
  float delS = 0.0f;
  uint64_t delD = 0;
  if (dom[dh] >= tp.ridiculous) {
    // m_domMinNode[domHash]: the domain's minimum m_t2 key (uint32 score, docid)
    uint32_t mc = 0xffffffffu;
    uint64_t md = ~0ull;
    float ms = 0.0f;
    for (uint32_t t = lane; t < n; t += 64) {
      const uint64_t dt = td[t];
      if (dom_hash8(dt) != dh) continue;
      const uint32_t ct = tree_cs(ts[t], ints);
      if (ct < mc || (ct == mc && dt < md)) {
        mc = ct;
        md = dt;
        ms = ts[t];
      }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const uint32_t oc = __shfl_xor(mc, off, 64);
      const uint64_t od = __shfl_xor(md, off, 64);
      const float os = __shfl_xor(ms, off, 64);
      if (oc < mc || (oc == mc && od < md)) {
        mc = oc;
        md = od;
        ms = os;
      }
    }
    if (cs < mc || (cs == mc && d <= md)) return;  // k <= *m_t2.getKey(min)
    del = true;
    delS = ms;
    delD = md;
  }
  if (n >= TC) {
    err = 1;
    return;
  }
  // insert at p
  for (int64_t e = (int64_t)n; e > (int64_t)p; e -= 64) {
    const int64_t idx = e - 64 + lane;
    float v = 0.0f;
    uint64_t w = 0;
    const bool act = idx >= (int64_t)p && idx < (int64_t)n;
    if (act) {
      v = ts[idx];
      w = td[idx];
    }
    wave_lds_sync();
    if (act) {
      ts[idx + 1] = v;
      td[idx + 1] = w;
    }
    wave_lds_sync();
  }
  if (lane == 0) {
    ts[p] = s;
    td[p] = d;
    dom[dh]++;
  }
  n++;
  wave_lds_sync();
  if (dom[dh] < tp.cap) vcount += 1.0;
  else if (dom[dh] == tp.cap) vcount += tp.partial;
  if (del) tree_delete(ts, td, dom, n, vcount, tp, tree_lower_bound(ts, td, n, delS, delD, lane, ints), dh, lane);
  while (n > 0 && (vcount - 1.0 >= tp.docs_wanted || (int64_t)n == tp.num_nodes))
    tree_delete(ts, td, dom, n, vcount, tp, n - 1, dom_hash8(td[n - 1]), lane);
}

__device__ __forceinline__ float key_score(uint32_t key) {
  return __uint_as_float((key & 0x80000000u) ? (key & 0x7fffffffu) : ~key);
}

// one wave: the docid-order loop of intersectLists10_r with the TopTree
// (Posdb.cpp:6137-7706, minWinningScore per pass).  The loop is serial, so
// its input streams through registers: RP_BUF buffers of RP_C chunks (64
// entries each) are in flight while one is staged in LDS and walked chunk by
// chunk; a chunk's lanes are re-tested after every offer that changes the
// tree (the reference's per-docid order).
constexpr int RP_C = 16;
constexpr int RP_BUF = 3;  // 48 loads in flight (vmcnt holds 63)

__global__ void __launch_bounds__(64) k_tree_replay(Counters *ctr, const uint4 *rep, TreeState *T, TreeParams tp,
                                                    uint32_t *out_key, uint64_t *out_doc) {
  __shared__ float ts[TC];
  __shared__ uint64_t td[TC];
  __shared__ int32_t dom[256];
  __shared__ uint4 stage[RP_C * 64];
  const int lane = threadIdx.x;
  if (tp.on_reg_err) {
    // the fallback behind k_tree_seq, on the same stream: nothing to do
    // unless its register tree overflowed (2 = TREE_ERR_REG, defined below)
    const uint32_t te = __builtin_amdgcn_readfirstlane(__atomic_load_n(&ctr->tree_err, __ATOMIC_RELAXED));
    if (te != 2u) return;
    if (lane == 0) ctr->tree_err = 0;
  }
  uint32_t n = 0;
  float vcount = 0.0f;
  if (tp.init) {
    for (int q = lane; q < 256; q += 64) dom[q] = 0;
  } else {
    n = T->n;
    vcount = T->vcount;
    for (int q = lane; q < 256; q += 64) dom[q] = T->dom[q];
    for (uint32_t q = lane; q < n; q += 64) {
      ts[q] = T->score[q];
      td[q] = T->docid[q];
    }
  }
  wave_lds_sync();
  const uint32_t ns = (uint32_t)(ctr->surv_top >> 36);
  const bool ints = tp.ints != 0;
  float mws = -1.0f;  // minWinningScore, Posdb.cpp:6012
  uint32_t nmws = 0;  // its assignments recorded (tp.mwsl)
  bool called = false;
  uint32_t filtered = 0, err = 0;
  uint32_t dbg_adds = 0, dbg_nmax = 0;  // diagnostic (GBGPU_TOPK_DEBUG)
  uint64_t dbg_t = 0;
  const uint64_t dbg_t0 = __builtin_amdgcn_s_memrealtime();
  float bot_s = n ? ts[n - 1] : 0.0f;  // the tree's last node
  uint64_t bot_d = n ? td[n - 1] : 0;
  constexpr uint32_t BATCH = RP_C * 64;
  const uint32_t nbatch = (ns + BATCH - 1) / BATCH;
  // one staged batch, chunk by chunk
  auto walk = [&](uint32_t bt) {
    for (int c = 0; c < RP_C && !err; c++) {
      const uint32_t p = bt * BATCH + (uint32_t)c * 64 + lane;
      if (bt * BATCH + (uint32_t)c * 64 >= ns) break;
      const uint4 e = stage[c * 64 + lane];
      const bool valid = p < ns;
      const uint32_t key = e.x;
      const float B = __uint_as_float(e.y);
      const bool serp = valid && (e.w >> 31);
      const uint64_t d = ((uint64_t)(e.w & 0x7fffffffu) << 32) | e.z;
      const float sc = ints ? __int_as_float((int32_t)(key ^ 0x80000000u)) : key_score(key);
      // (integer scores come from a gbsortby int term: the prefilters are off)
      uint64_t from = ~0ull;  // lanes not yet decided
      for (;;) {
        const bool live = valid && (ints || !(B <= mws));  // not skipped by the prefilters
        const bool ok = live && key != 0;                   // scored, not filtered by paging
        const bool full = vcount >= tp.docs_wanted;
        const bool rej = called && full && n > 0 && !node_better(sc, d, bot_s, bot_d, ints);
        const uint64_t slow = __ballot(ok && !rej) & from;
        const int j = slow ? __ffsll((unsigned long long)slow) - 1 : 64;
        const uint64_t below = j >= 64 ? ~0ull : ((1ull << j) - 1);
        filtered += (uint32_t)__popcll(__ballot(live && serp) & below & from);
        if (!slow) break;
        const float s = __shfl(sc, j, 64);
        const uint64_t dd = __shfl(d, j, 64);
        const uint64_t c0 = __builtin_amdgcn_s_memrealtime();
        tree_add(ts, td, dom, n, vcount, tp, s, dd, err, lane);
        dbg_adds++;
        dbg_t += __builtin_amdgcn_s_memrealtime() - c0;
        dbg_nmax = max(dbg_nmax, n);
        if (err) break;
        called = true;
        if (n) {
          bot_s = ts[n - 1];
          bot_d = td[n - 1];
        }
        if (n > (uint32_t)tp.docs_wanted) {
          mws = ts[n - 1];  // Posdb.cpp:7699-7704
          if (tp.mwsl && lane == 0)
            tp.mwsl[1 + nmws++] = make_uint4((uint32_t)dd, (uint32_t)(dd >> 32), __float_as_uint(mws), 0u);
        }
        if (j == 63) break;
        from = ~0ull << (j + 1);
      }
    }
  };
  // three register buffers of RP_C chunks as named values (an array or a
  // vector would be copied out of the load registers, and wait on them)
#define RP_EACH(M, b) M(b, 0) M(b, 1) M(b, 2) M(b, 3) M(b, 4) M(b, 5) M(b, 6) M(b, 7) \
  M(b, 8) M(b, 9) M(b, 10) M(b, 11) M(b, 12) M(b, 13) M(b, 14) M(b, 15)
#define RP_DECL(b, c) uint4 b##c = make_uint4(0u, 0u, 0u, 0u);
#define RP_LOAD(b, c) b##c = rep[min(bt_ * BATCH + (uint32_t)(c) * 64 + lane, ns - 1)];
#define RP_STAGE(b, c) stage[(c) * 64 + lane] = b##c;
#define RP_FETCH(b, bt)        \
  {                            \
    const uint32_t bt_ = (bt); \
    RP_EACH(RP_LOAD, b)        \
  }
#define RP_CONSUME(b, bt)   \
  RP_EACH(RP_STAGE, b)      \
  wave_lds_sync();          \
  walk(bt);
  static_assert(RP_C == 16 && RP_BUF == 3, "RP_EACH names 16 chunks, three buffers");
  RP_EACH(RP_DECL, x)
  RP_EACH(RP_DECL, y)
  RP_EACH(RP_DECL, z)
  // (fetches are unconditional -- past the end they re-read the last entry --
  // so every path reaches a use with the same loads in flight)
  if (ns) {
  RP_FETCH(x, 0u)
  RP_FETCH(y, 1u)
  RP_FETCH(z, 2u)
  for (uint32_t bt = 0; bt < nbatch && !err; bt += RP_BUF) {
    RP_CONSUME(x, bt)
    RP_FETCH(x, bt + 3)
    if (bt + 1 >= nbatch || err) break;
    RP_CONSUME(y, bt + 1)
    RP_FETCH(y, bt + 4)
    if (bt + 2 >= nbatch || err) break;
    RP_CONSUME(z, bt + 2)
    RP_FETCH(z, bt + 5)
  }
  }
#undef RP_EACH
#undef RP_DECL
#undef RP_LOAD
#undef RP_STAGE
#undef RP_FETCH
#undef RP_CONSUME
  if (lane == 0) {
    ctr->filtered = filtered;
    if (err) ctr->tree_err = 1;
    if (tp.mwsl) tp.mwsl[0] = make_uint4(nmws, 0u, 0u, 0u);
    ctr->pad[0] = dbg_adds;
    ctr->pad[1] = dbg_nmax;
    ctr->rdbg_t = (uint32_t)(dbg_t / 100);
    ctr->rdbg_total = (uint32_t)((__builtin_amdgcn_s_memrealtime() - dbg_t0) / 100);
  }
  if (tp.final || tp.emit) {
    for (uint32_t q = lane; q < n; q += 64) {
      const uint32_t b = __float_as_uint(ts[q]);
      uint32_t k = tp.ints ? (b ^ 0x80000000u) : (b & 0x80000000u) ? ~b : (b | 0x80000000u);
      out_key[q] = k ? k : 1u;
      out_doc[q] = td[q];
    }
    if (lane == 0) {
      if (n < TC) out_key[n] = 0;
      ctr->tree_n = n;
    }
  }
  if (!tp.final) {
    for (uint32_t q = lane; q < n; q += 64) {
      T->score[q] = ts[q];
      T->docid[q] = td[q];
    }
    for (int q = lane; q < 256; q += 64) T->dom[q] = dom[q];
    if (lane == 0) {
      T->n = n;
      T->vcount = vcount;
    }
  }
}

// ------------------------------------- site clustering: the block replay
// k_tree_seq: the same docid-order loop as k_tree_replay for a whole-range
// query (one pass: TREE_INIT | TREE_FINAL), split in two so that one wave's
// serial work is only the offers that can change the tree:
//   * all SQ_W waves of the block rule out, in parallel, the entries of a
//     segment (SQ_SEG entries) that cannot be offered under ANY state the
//     tree can reach from the state at the segment's start, and stage the
//     others (the candidates) in LDS in docid order;
//   * wave 0 (the sequencer) walks the candidates with the exact per-docid
//     test of k_tree_replay, and publishes the new state.
// Why skipping the others is exact: once the tree is full (m_vcount >=
// m_docsWanted after an add), an add keeps it full (every node it deletes
// takes at most 1.0 off m_vcount, and deletes stop below docsWanted + 1:
// TopTree.cpp:446), and its last node never gets worse (a node is only
// inserted above the last one, and deletes only remove nodes); so an entry
// not better than the segment-start last node is never better than the last
// node later, and minWinningScore, reassigned only to the last node's score
// (Posdb.cpp:7699-7704), stays >= L = min(its value, that score).  One
// exception: the m_numNodes delete (TopTree.cpp:446) can take m_vcount
// below docsWanted; the sequencer then walks the rest of the segment raw.
// The tree itself is register-resident in the sequencer: node i (best
// first) at column i >> 6, lane i & 63, K columns; inserts and deletes are
// DPP lane shifts, the lower bound K ballots.  A tree outgrowing 64 K nodes
// sets tree_err = 2 and the host replays the query with k_tree_replay.
constexpr int SQ_W = 8;                              // waves per block
constexpr int SQ_E = 8;                              // entries per lane and segment
constexpr uint32_t SQ_SEG = (uint32_t)SQ_W * 64 * SQ_E;  // 4096: a segment-local index fits 12 bits
constexpr uint32_t TREE_ERR_REG = 2;                 // tree_err: the register tree overflowed

__device__ __forceinline__ uint32_t rl_u32(uint32_t v, uint32_t l) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l);
}
__device__ __forceinline__ float rl_f(float v, uint32_t l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), (int)l));
}
__device__ __forceinline__ uint64_t rl_u64(uint64_t v, uint32_t l) {
  return (uint64_t)rl_u32((uint32_t)(v >> 32), l) << 32 | rl_u32((uint32_t)v, l);
}
// lane L takes lane L-1's value, lane 0 `edge` (wave_shr:1)
__device__ __forceinline__ uint64_t shr_u64(uint64_t x, uint64_t edge) {
  return (uint64_t)lane_prev((uint32_t)(x >> 32), (uint32_t)(edge >> 32)) << 32 | lane_prev((uint32_t)x, (uint32_t)edge);
}
// lane L takes lane L+1's value, lane 63 `edge` (wave_shl:1)
__device__ __forceinline__ uint64_t shl_u64(uint64_t x, uint64_t edge) {
  return (uint64_t)lane_next((uint32_t)(x >> 32), (uint32_t)(edge >> 32)) << 32 | lane_next((uint32_t)x, (uint32_t)edge);
}

// A node's order key: the replay entry's score key (order-preserving uint32
// of the float score, or of the int32 m_intScore) with -0.0 folded onto
// +0.0, so that key order is the TopTree's score order (float compares;
// scores are never NaN).  A -0.0 score is reported as +0.0.
__device__ __forceinline__ uint32_t node_key(uint32_t key, bool ints) {
  return (!ints && key == 0x7fffffffu) ? 0x80000000u : key;
}
__device__ __forceinline__ bool key_better(uint32_t k1, uint64_t d1, uint32_t k2, uint64_t d2) {
  return k1 > k2 || (k1 == k2 && d1 < d2);
}
// tree_cs of a node key
__device__ __forceinline__ uint32_t key_cs(uint32_t k, bool ints) {
  return ints ? (k ^ 0x80000000u) : tree_cs(key_score(k), false);
}

template <int K, bool INTS>
struct RegTree {
  uint32_t kk[K];  // node keys
  uint64_t d[K];
  int32_t dom[4];  // m_domCount: domain h at column h >> 6, lane h & 63
  uint32_t n;
  float vcount;
  uint32_t tk;     // the last node (n > 0), kept in step with the columns
  uint64_t td;

  // node i (uniform): every column read at lane i & 63, then selected -- no
  // branches for up to four columns; a uniform branch ladder beyond
  __device__ __forceinline__ uint32_t nk(uint32_t i) const {
    uint32_t r = rl_u32(kk[0], i & 63);
#pragma unroll
    for (int k = 1; k < K; k++) {
      if (K > 4 && (i >> 6) != (uint32_t)k) continue;
      const uint32_t v = rl_u32(kk[k], i & 63);
      r = (i >> 6) == (uint32_t)k ? v : r;
    }
    return r;
  }
  __device__ __forceinline__ uint64_t nd(uint32_t i) const {
    uint64_t r = rl_u64(d[0], i & 63);
#pragma unroll
    for (int k = 1; k < K; k++) {
      if (K > 4 && (i >> 6) != (uint32_t)k) continue;
      const uint64_t v = rl_u64(d[k], i & 63);
      r = (i >> 6) == (uint32_t)k ? v : r;
    }
    return r;
  }
  __device__ __forceinline__ int32_t domc(uint32_t h) const {
    const uint32_t l = h & 63, c = h >> 6;
    const int32_t c0 = (int32_t)rl_u32((uint32_t)dom[0], l), c1 = (int32_t)rl_u32((uint32_t)dom[1], l);
    const int32_t c2 = (int32_t)rl_u32((uint32_t)dom[2], l), c3 = (int32_t)rl_u32((uint32_t)dom[3], l);
    return c == 0 ? c0 : c == 1 ? c1 : c == 2 ? c2 : c3;
  }
  __device__ __forceinline__ void domadd(uint32_t h, int32_t v, int lane) {
    const bool me = (uint32_t)lane == (h & 63);
#pragma unroll
    for (int c = 0; c < 4; c++) dom[c] += (me & ((h >> 6) == (uint32_t)c)) ? v : 0;
  }
  // nodes better than (k, dd): the insert position (the array is sorted)
  __device__ __forceinline__ uint32_t lower(uint32_t k0, uint64_t dd, int lane) const {
    uint32_t p = 0;
#pragma unroll
    for (int k = 0; k < K; k++) {
      const uint32_t i = (uint32_t)k * 64 + (uint32_t)lane;
      p += (uint32_t)__popcll(__ballot((i < n) & key_better(kk[k], d[k], k0, dd)));
    }
    return p;
  }
  __device__ __forceinline__ void insert(uint32_t p, uint32_t k0, uint64_t dd, int lane) {
#pragma unroll
    for (int k = K - 1; k >= 0; k--) {
      if ((uint32_t)k * 64 > n || (uint32_t)(k + 1) * 64 <= p) continue;  // untouched column
      const uint32_t ek = k > 0 ? rl_u32(kk[k > 0 ? k - 1 : 0], 63) : 0u;  // the previous column's last node
      const uint64_t ed = k > 0 ? rl_u64(d[k > 0 ? k - 1 : 0], 63) : 0ull;
      const uint32_t sk = lane_prev(kk[k], ek);
      const uint64_t sd = shr_u64(d[k], ed);
      const uint32_t i = (uint32_t)k * 64 + (uint32_t)lane;
      kk[k] = i > p ? sk : i == p ? k0 : kk[k];
      d[k] = i > p ? sd : i == p ? dd : d[k];
    }
    n++;
  }
  // deleteNode's count bookkeeping (TopTree.cpp:543-547) for a node of
  // domain h
  __device__ __forceinline__ void uncount(uint32_t h, const TreeParams &tp, int lane) {
    const int32_t c = domc(h);
    if (c < tp.cap) vcount -= 1.0;
    else if (c == tp.cap) vcount -= tp.partial;
    domadd(h, -1, lane);
  }
  __device__ __forceinline__ void retail() {
    if (n) {
      tk = nk(n - 1);
      td = nd(n - 1);
    }
  }
  // node q (not the last) out: the columns from q's shift down one
  __device__ __forceinline__ void remove(uint32_t q, int lane) {
#pragma unroll
    for (int k = 0; k < K; k++) {
      if ((uint32_t)(k + 1) * 64 <= q || (uint32_t)k * 64 >= n) continue;
      const uint32_t ek = k + 1 < K ? rl_u32(kk[k + 1 < K ? k + 1 : k], 0) : 0u;  // the next column's first node
      const uint64_t ed = k + 1 < K ? rl_u64(d[k + 1 < K ? k + 1 : k], 0) : 0ull;
      const uint32_t sk = lane_next(kk[k], ek);
      const uint64_t sd = shl_u64(d[k], ed);
      const uint32_t i = (uint32_t)k * 64 + (uint32_t)lane;
      kk[k] = i >= q ? sk : kk[k];
      d[k] = i >= q ? sd : d[k];
    }
    n--;
  }
  // the domain's minimum m_t2 key (uint32 score, docid) -- m_domMinNode
  // (TopTree.cpp:355-385) -- and that node
  __device__ __forceinline__ void dom_min(uint32_t h, int lane, uint32_t &mc, uint64_t &md, uint32_t &mk) const {
    mc = 0xffffffffu;
    md = ~0ull;
    mk = 0;
#pragma unroll
    for (int k = 0; k < K; k++) {
      const uint32_t i = (uint32_t)k * 64 + (uint32_t)lane;
      if (i >= n || dom_hash8(d[k]) != h) continue;
      const uint32_t ct = key_cs(kk[k], INTS);
      if (ct < mc || (ct == mc && d[k] < md)) {
        mc = ct;
        md = d[k];
        mk = kk[k];
      }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const uint32_t oc = __shfl_xor(mc, off, 64);
      const uint64_t od = __shfl_xor(md, off, 64);
      const uint32_t ok = __shfl_xor(mk, off, 64);
      if (oc < mc || (oc == mc && od < md)) {
        mc = oc;
        md = od;
        mk = ok;
      }
    }
    // (every lane holds the minimum: read as uniform values)
    mc = rl_u32(mc, 0);
    md = rl_u64(md, 0);
    mk = rl_u32(mk, 0);
  }
  // TopTree::addNode (TopTree.cpp:206-516), as tree_add; false: no column left
  __device__ __forceinline__ bool add(const TreeParams &tp, uint32_t k0, uint64_t dd, int lane) {
    const uint32_t dh = dom_hash8(dd);
    if (vcount >= tp.docs_wanted && n > 0 && !key_better(k0, dd, tk, td)) return true;
    // the insert position and "if equal do not replace" in one pass
    uint32_t p = 0;
    uint64_t eqm = 0;
#pragma unroll
    for (int k = 0; k < K; k++) {
      const uint32_t i = (uint32_t)k * 64 + (uint32_t)lane;
      const bool v = i < n;
      p += (uint32_t)__popcll(__ballot(v & key_better(kk[k], d[k], k0, dd)));
      eqm |= __ballot(v & (kk[k] == k0) & (d[k] == dd));
    }
    if (eqm) return true;
    const int32_t c = domc(dh);
    bool del = false;
    uint32_t delK = 0;
    uint64_t delD = 0;
    if (c >= tp.ridiculous) {
      uint32_t mc, mk;
      uint64_t md;
      dom_min(dh, lane, mc, md, mk);
      const uint32_t cs = key_cs(k0, INTS);
      if (cs < mc || (cs == mc && dd <= md)) return true;  // k <= *m_t2.getKey(min)
      del = true;
      delK = mk;
      delD = md;
    }
    if (n >= (uint32_t)K * 64) return false;
    const uint32_t n0 = n;
    insert(p, k0, dd, lane);
    if (p == n0) {
      tk = k0;
      td = dd;
    }
    domadd(dh, 1, lane);
    if (c + 1 < tp.cap) vcount += 1.0;
    else if (c + 1 == tp.cap) vcount += tp.partial;
    if (del) {
      uncount(dh, tp, lane);
      const uint32_t q = lower(delK, delD, lane);
      if (q + 1 < n) remove(q, lane);
      else n--;
      retail();
    }
    // the last node out while the tree holds more than it counts
    // (TopTree.cpp:446): no shift, the new last node read back
    while (n > 0 && (vcount - 1.0 >= tp.docs_wanted || (int64_t)n == tp.num_nodes)) {
      uncount(dom_hash8(td), tp, lane);
      n--;
      retail();
    }
    return true;
  }
};

// the sequencer's state as the filter reads it (published after a segment)
struct SeqState {
  uint32_t pref;   // the tree is full: the filter may rule entries out
  uint32_t stop;   // the register tree overflowed: every wave leaves
  float L;         // lower bound of minWinningScore from here on
  uint32_t bk;     // the last node
  uint64_t bd;
};

template <int K, bool INTS>
__global__ void __launch_bounds__(64 * SQ_W) k_tree_seq(Counters *ctr, const uint4 *rep, TreeParams tp, uint32_t *out_key,
                                                       uint64_t *out_doc) {
  __shared__ uint4 s_cand[SQ_W][64 * SQ_E];
  __shared__ uint32_t s_cnt[SQ_W];
  __shared__ SeqState s_st;
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t lt = (1ull << lane) - 1;
  const uint32_t ns = (uint32_t)(ctr->surv_top >> 36);
  const uint32_t nseg = (ns + SQ_SEG - 1) / SQ_SEG;
  // the sequencer's (wave 0's) state
  RegTree<K, INTS> T;
#pragma unroll
  for (int k = 0; k < K; k++) {
    T.kk[k] = 0;
    T.d[k] = 0;
  }
#pragma unroll
  for (int c = 0; c < 4; c++) T.dom[c] = 0;
  T.n = 0;
  T.vcount = 0.0f;
  T.tk = 0;
  T.td = 0;
  float mws = -1.0f;  // minWinningScore, Posdb.cpp:6012
  uint32_t nmws = 0;  // its assignments recorded (tp.mwsl)
  bool called = false;
  uint32_t filtered = 0, err = 0, adds = 0, nmax = 0, ncand = 0;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint64_t t_add = 0, t_seq = 0, t_filt = 0;  // diagnostic clocks (GBGPU_DIAG)
  if (threadIdx.x == 0) s_st = SeqState{0u, 0u, 0.0f, 0u, 0ull};
  uint4 e[SQ_E];
  auto load = [&](uint32_t sg) {
#pragma unroll
    for (int j = 0; j < SQ_E; j++)
      e[j] = rep[min(sg * SQ_SEG + (uint32_t)wid * 64 * SQ_E + (uint32_t)j * 64 + (uint32_t)lane, ns - 1)];
  };
  // the exact per-docid loop of k_tree_replay over one chunk of 64 entries
  // (prefilters, paging count, offers in docid order); li: each lane's
  // segment-local index.  Returns the local index after the add that broke
  // the filter's premise (the rest of the segment is walked raw), else ~0u.
  auto offer = [&](bool valid, uint4 x, uint32_t li, bool pref) -> uint32_t {
    const uint32_t key = x.x;
    const float B = __uint_as_float(x.y);
    const bool serp = valid && (x.w >> 31);
    const uint64_t d = ((uint64_t)(x.w & 0x3fu) << 32) | x.z;
    const uint32_t k0 = node_key(key, INTS);
    uint64_t from = ~0ull;
    for (;;) {
      // (integer scores come from a gbsortby int term: the prefilters are off)
      const bool live = valid & (INTS || !(B <= mws));
      const bool ok = live & (key != 0);
      const bool rej = called & (T.vcount >= tp.docs_wanted) & (T.n > 0) & !key_better(k0, d, T.tk, T.td);
      const uint64_t slow = __ballot(ok & !rej) & from;
      const int j = slow ? __ffsll((unsigned long long)slow) - 1 : 64;
      const uint64_t below = j >= 64 ? ~0ull : ((1ull << j) - 1);
      filtered += (uint32_t)__popcll(__ballot(live & serp) & below & from);
      if (!slow) return ~0u;
      // the offer as uniform values (readlane, not a shuffle): the add's
      // control flow is then scalar, its node indices SGPRs
#ifdef GBGPU_DIAG
      const uint64_t ta = __builtin_amdgcn_s_memrealtime();
#endif
      const bool added = T.add(tp, rl_u32(k0, (uint32_t)j), rl_u64(d, (uint32_t)j), lane);
#ifdef GBGPU_DIAG
      t_add += __builtin_amdgcn_s_memrealtime() - ta;
#endif
      if (!added) {
        err = TREE_ERR_REG;
        return ~0u;
      }
      adds++;
      nmax = max(nmax, T.n);
      called = true;
      if (T.n > (uint32_t)tp.docs_wanted) {
        mws = key_score(T.tk);  // Posdb.cpp:7699-7704
        if (tp.mwsl) {
          const uint64_t dj = rl_u64(d, (uint32_t)j);
          if (lane == 0) tp.mwsl[1 + nmws] = make_uint4((uint32_t)dj, (uint32_t)(dj >> 32), __float_as_uint(mws), 0u);
          nmws++;
        }
      }
      if (pref && !(T.vcount >= tp.docs_wanted)) return rl_u32(li, (uint32_t)j) + 1;
      if (j == 63) return ~0u;
      from = ~0ull << (j + 1);
    }
  };
  if (ns) load(0);
  for (uint32_t sg = 0; sg < nseg; sg++) {
    __syncthreads();  // s_st published, s_cand free
#ifdef GBGPU_DIAG
    const uint64_t tf = __builtin_amdgcn_s_memrealtime();
#endif
    const SeqState st = s_st;
    if (st.stop) break;  // (uniform over the block)
    // 1. the filter: each wave's 64 SQ_E consecutive entries
    uint32_t cnt = 0;
#pragma unroll
    for (int j = 0; j < SQ_E; j++) {
      const uint32_t li = (uint32_t)wid * 64 * SQ_E + (uint32_t)j * 64 + (uint32_t)lane;
      const uint4 x = e[j];
      const bool serp = x.w >> 31;
      bool c = (sg * SQ_SEG + li < ns) & ((x.x != 0) | serp);
      if (st.pref) {
        const uint64_t d = ((uint64_t)(x.w & 0x3fu) << 32) | x.z;
        c = c && (INTS || !(__uint_as_float(x.y) <= st.L)) && (serp || key_better(node_key(x.x, INTS), d, st.bk, st.bd));
      }
      const uint64_t bm = __ballot(c);
      if (c) s_cand[wid][cnt + (uint32_t)__popcll(bm & lt)] = make_uint4(x.x, x.y, x.z, (x.w & 0x8000003fu) | (li << 8));
      cnt += (uint32_t)__popcll(bm);
    }
    if (lane == 0) s_cnt[wid] = cnt;
    // the next segment's entries go out now and land while the sequencer works
    if (sg + 1 < nseg) load(sg + 1);
    __syncthreads();
    if (wid != 0) continue;
#ifdef GBGPU_DIAG
    const uint64_t ts = __builtin_amdgcn_s_memrealtime();
    t_filt += ts - tf;
#endif
    // 2. the sequencer: the candidates in order, then the state
    uint32_t pre[SQ_W + 1];
    pre[0] = 0;
#pragma unroll
    for (int w = 0; w < SQ_W; w++) pre[w + 1] = pre[w] + __builtin_amdgcn_readfirstlane(s_cnt[w]);
    uint32_t resume = ~0u;
    ncand += pre[SQ_W];
    for (uint32_t c0 = 0; c0 < pre[SQ_W] && resume == ~0u && !err; c0 += 64) {
      const uint32_t t = c0 + (uint32_t)lane;
      uint4 x = make_uint4(0u, 0u, 0u, 0u);
      if (t < pre[SQ_W]) {
        int w = 0;
#pragma unroll
        for (int w2 = 1; w2 < SQ_W; w2++)
          if (t >= pre[w2]) w = w2;
        x = s_cand[w][t - pre[w]];
      }
      resume = offer(t < pre[SQ_W], x, (x.w >> 8) & 0xfffu, st.pref != 0);
    }
    // the filter's premise broke (the m_numNodes delete): the rest raw
    if (resume != ~0u) {
      const uint32_t end = min(ns, (sg + 1) * SQ_SEG);
      for (uint32_t p0 = sg * SQ_SEG + resume; p0 < end && !err; p0 += 64) {
        const uint32_t p = p0 + (uint32_t)lane;
        uint4 x = rep[min(p, ns - 1)];
        x.w = (x.w & 0x8000003fu) | ((p - sg * SQ_SEG) << 8);
        offer(p < end, x, 0u, false);
      }
    }
    if (lane == 0) {
      const bool full = called && T.vcount >= tp.docs_wanted && T.n > 0;
      const float bs = key_score(T.tk);
      s_st = SeqState{full ? 1u : 0u, err ? 1u : 0u, mws < bs ? mws : bs, T.tk, T.td};
    }
#ifdef GBGPU_DIAG
    t_seq += __builtin_amdgcn_s_memrealtime() - ts;
#endif
  }
  if (wid != 0) return;
  if (lane == 0) {
    ctr->filtered = filtered;
    if (err) ctr->tree_err = err;
    if (tp.mwsl) tp.mwsl[0] = make_uint4(nmws, 0u, 0u, 0u);
    ctr->pad[0] = adds;  // diagnostic (GBGPU_TOPK_DEBUG)
    ctr->pad[1] = nmax;
    ctr->rdbg_t = ncand;
    ctr->rdbg_total = (uint32_t)((__builtin_amdgcn_s_memrealtime() - t0) / 100);
    ctr->sq_dbg[0] = (uint32_t)t_add;
    ctr->sq_dbg[1] = (uint32_t)t_seq;
    ctr->sq_dbg[2] = (uint32_t)t_filt;
    ctr->sq_dbg[3] = nseg;
  }
  if (err) return;
#pragma unroll
  for (int k = 0; k < K; k++) {
    const uint32_t i = (uint32_t)k * 64 + (uint32_t)lane;
    if (i < T.n) {
      out_key[i] = T.kk[k];
      out_doc[i] = T.d[k];
    }
  }
  if (lane == 0) {
    if (T.n < TC) out_key[T.n] = 0;
    ctr->tree_n = T.n;
  }
}

// ------------------------------------------------------------------ top-k
// TopTree replacement (TopTree.cpp:195-516 without clustering): the k best
// survivors by (score desc, docid asc).  Scores travel as order-preserving
// uint32 keys (0 = not scored).  k_score counts every key in a 65536-bin
// histogram of its top 16 bits (Select::hist); then ONE launch, k_topk:
//   1. every block scans the histogram from the top to the bin P holding the
//      k-th key;
//   2. the grid gathers keys whose prefix is above P (A, fewer than k) and
//      equal to P (B), one atomic per wave;
//   3. the block that finishes last narrows B in LDS with two 8-bit passes to
//      the k-th key T itself, moves B's keys > T to A and compacts the ties
//      (== T, of which the smallest docids win) in place, then sorts A and
//      merges the ties in LDS.
constexpr int TK_THREADS = 1024;
constexpr int TK_BLOCKS = 32;
// Select::cnt packs |A| (16 bits: < k <= MAX_K), |B| (32 bits) and the
// blocks finished (16 bits) into one 64-bit word
static_assert(MAX_K < 65536 && MAX_K_BIG < 65536 && TK_BLOCKS < 65536, "Select::cnt fields");
constexpr int TK_E = 16;  // keys per thread and gather round

// bitonic sort of sk/sd[0, n) in LDS, n rounded up to a power of two with
// sentinels; "first" = better = key desc, docid asc
__device__ void lds_sort_best_first(uint32_t *sk, uint64_t *sd, uint32_t n) {
  uint32_t S = 1;
  while (S < n) S <<= 1;
  for (uint32_t t = n + threadIdx.x; t < S; t += blockDim.x) {
    sk[t] = 0;
    sd[t] = ~0ull;
  }
  __syncthreads();
  for (uint32_t size = 2; size <= S; size <<= 1) {
    for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
      for (uint32_t t = threadIdx.x; t < S / 2; t += blockDim.x) {
        const uint32_t i = 2 * t - (t & (stride - 1));
        const uint32_t j = i + stride;
        const bool desc = ((i & size) == 0);
        const uint32_t ki = sk[i], kj = sk[j];
        const uint64_t di = sd[i], dj = sd[j];
        const bool jbetter = (kj > ki) || (kj == ki && dj < di);
        if (jbetter == desc) {
          sk[i] = kj; sk[j] = ki;
          sd[i] = dj; sd[j] = di;
        }
      }
      __syncthreads();
    }
  }
}

// the bin (of NB, counts h[]) holding the need-th entry counted from the top
// bin down, and the entries in the bins above it; one block of NT threads,
// each holding NB/NT consecutive counts in registers; tmp: NT/64 words
template <int NT, int NB, class P>
__device__ void top_bin(const P *h, uint32_t need, uint32_t *tmp, uint32_t *s_bin, uint32_t *s_above,
                        uint32_t *s_total) {
  constexpr int BPT = NB >= NT ? NB / NT : 1;
  static_assert(NB < NT || NB % NT == 0, "bins split evenly");
  // thread t: bins [NB - (t+1) BPT, NB - t BPT), walked from the highest
  const int lo = NB - ((int)threadIdx.x + 1) * BPT;
  uint32_t c[BPT], sum = 0;
#pragma unroll
  for (int q = 0; q < BPT; q++) {
    c[q] = lo + q >= 0 ? (uint32_t)h[lo + q] : 0u;
    sum += c[q];
  }
  uint32_t total;
  const uint32_t before = block_exclusive_scan<NT>(sum, tmp, &total);
  if (threadIdx.x == 0) *s_total = total;
  if (need > 0 && before < need && need <= before + sum) {
    uint32_t cum = before;
    bool found = false;
#pragma unroll
    for (int q = BPT - 1; q >= 0; q--) {
      if (!found && cum + c[q] >= need) {
        *s_bin = (uint32_t)(lo + q);
        *s_above = cum;
        found = true;
      }
      cum += c[q];
    }
  }
  __syncthreads();
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
  return x;
}

// top_bin over Select::hist with coalesced 16-B loads (a thread holding 64
// consecutive bins would make every load touch 64 lines): wave w holds bins
// [4096 w, 4096 w + 4096) as 16 rows of 256, lane l bins 4l..4l+3 of a row;
// the wave holding the need-th entry walks its rows, then its lanes, from
// the top.  tmp: 16 words.
__device__ __forceinline__ void top_bin_hist(const uint32_t *h, uint32_t need, uint32_t *tmp, uint32_t *s_bin, uint32_t *s_above,
                             uint32_t *s_total) {
  static_assert(TK_THREADS == 1024 && SEL_HBINS == 16 * 4096, "16 waves of 4096 bins");
  typedef uint32_t v4 __attribute__((ext_vector_type(4)));
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const v4 *src = reinterpret_cast<const v4 *>(h) + w * 1024 + lane;
  v4 v[16];
#pragma unroll
  for (int r = 0; r < 16; r++) v[r] = src[r * 64];
  uint32_t ls[16], lt = 0;
#pragma unroll
  for (int r = 0; r < 16; r++) {
    ls[r] = v[r].x + v[r].y + v[r].z + v[r].w;
    lt += ls[r];
  }
  const uint32_t wt = wave_sum(lt);
  if (lane == 0) tmp[w] = wt;
  __syncthreads();
  uint32_t above = 0, total = 0;  // entries in the waves above (higher bins)
  for (int q = 0; q < 16; q++) {
    const uint32_t c = tmp[q];
    total += c;
    if (q > w) above += c;
  }
  if (threadIdx.x == 0) *s_total = total;
  if (need > 0 && above < need && need <= above + wt) {  // one wave
    uint32_t cum = above;
#pragma unroll
    for (int r = 15; r >= 0; r--) {
      if (__ballot(ls[r] != 0) == 0) continue;
      const uint32_t rs = wave_sum(ls[r]);
      if (cum + rs >= need) {
        uint32_t x = ls[r];  // -> entries of this row in lanes >= lane
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const uint32_t y = __shfl_down(x, o, 64);
          if (lane + o < 64) x += y;
        }
        uint32_t c2 = cum + x - ls[r];
        if (c2 < need && need <= cum + x) {
          const uint32_t e[4] = {v[r].x, v[r].y, v[r].z, v[r].w};
          bool found = false;
#pragma unroll
          for (int c = 3; c >= 0; c--) {
            if (!found && c2 + e[c] >= need) {
              *s_bin = (uint32_t)(w * 4096 + r * 256 + lane * 4 + c);
              *s_above = c2;
              found = true;
            }
            c2 += e[c];
          }
        }
        break;
      }
      cum += rs;
    }
  }
  __syncthreads();
}

// write-through (sc1) stores and L2-served (sc1) loads: the cross-workgroup
// hand-off of MI355X_MICROARCH.md (no buffer_wbl2 / buffer_inv)
template <class T>
__device__ __forceinline__ void st_sc1(T *p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <class T>
__device__ __forceinline__ T ld_sc1(const T *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// append the flagged entries of one block-wide step to dst (block scan, in
// index order); returns the new count (every thread)
__device__ __forceinline__ uint32_t block_append(bool f, uint32_t key, uint64_t doc, uint32_t *dk, uint64_t *dd,
                                                 uint32_t n, uint32_t *tmp) {
  uint32_t tot;
  const uint32_t o = block_exclusive_scan<TK_THREADS>(f ? 1u : 0u, tmp, &tot);
  if (f) {
    st_sc1(dk + n + o, key);
    st_sc1(dd + n + o, doc);
  }
  return n + tot;
}

// TL: the final sort's LDS capacity (k < TL; TILE, or TILE_BIG for a TopTree
// beyond MAX_K nodes)
template <int TL>
__global__ void __launch_bounds__(TK_THREADS) k_topk(const uint32_t *skey, const uint64_t *sdoc, const Counters *ctr,
                                                     Select *sel, uint32_t k, uint32_t *akey, uint64_t *adoc,
                                                     uint32_t *bkey, uint64_t *bdoc, uint32_t *out_key,
                                                     uint64_t *out_doc) {
  __shared__ uint32_t tmp[TK_THREADS / 64];
  __shared__ uint32_t s_bin, s_above, s_total, s_last, s_ba, s_bb;
  __shared__ uint32_t h8[256];
  __shared__ __attribute__((aligned(16))) uint32_t sk[TL];
  __shared__ uint64_t sd[TL];
  const uint32_t n = (uint32_t)(ctr->surv_top >> 36);
  const bool dbg0 = blockIdx.x == 0 && threadIdx.x == 0;
  if (dbg0) sel->tdbg[0] = __builtin_amdgcn_s_memrealtime();
  // 1. the prefix P of the k-th key
  if (threadIdx.x == 0) {
    s_bin = 0;
    s_above = 0;
  }
  __syncthreads();
  top_bin_hist(sel->hist, k, tmp, &s_bin, &s_above, &s_total);
  const bool all = s_total <= k;  // every scored key is taken
  const uint32_t P = s_bin;
  if (dbg0) sel->tdbg[1] = __builtin_amdgcn_s_memrealtime();
  // 2. A: prefix > P (all: every scored key), B: prefix == P.  A block
  // takes TK_E keys a thread per round: flags, one block scan, ONE atomic
  // per list and round, then the writes.
  for (uint32_t r0 = blockIdx.x * TK_THREADS * TK_E; r0 < n; r0 += gridDim.x * TK_THREADS * TK_E) {
    uint32_t keys[TK_E], fa = 0, fb = 0, cnt = 0;
#pragma unroll
    for (int e = 0; e < TK_E; e++) {
      const uint32_t i = r0 + (uint32_t)e * TK_THREADS + threadIdx.x;
      keys[e] = i < n ? skey[i] : 0u;
    }
#pragma unroll
    for (int e = 0; e < TK_E; e++) {
      const uint32_t key = keys[e];
      const bool ga = key != 0 && (all || (key >> 16) > P);
      const bool gb = key != 0 && !all && (key >> 16) == P;
      fa |= (ga ? 1u : 0u) << e;
      fb |= (gb ? 1u : 0u) << e;
    }
    cnt = (uint32_t)__popc(fa) | ((uint32_t)__popc(fb) << 16);  // <= TK_THREADS * TK_E < 2^16 each
    uint32_t tot;
    const uint32_t ex = block_exclusive_scan<TK_THREADS>(cnt, tmp, &tot);
    if (threadIdx.x == 0) {
      unsigned long long old = 0;
      if (tot)
        old = __hip_atomic_fetch_add(&sel->cnt, (unsigned long long)(tot & 0xffff) | ((unsigned long long)(tot >> 16) << 16),
                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_ba = (uint32_t)(old & 0xffff);
      s_bb = (uint32_t)(old >> 16);
    }
    __syncthreads();
    uint32_t oa = s_ba + (ex & 0xffff), ob = s_bb + (ex >> 16);
#pragma unroll
    for (int e = 0; e < TK_E; e++) {
      const uint32_t i = r0 + (uint32_t)e * TK_THREADS + threadIdx.x;
      if (fa >> e & 1) {
        st_sc1(akey + oa, keys[e]);
        st_sc1(adoc + oa++, sdoc[i]);
      }
      if (fb >> e & 1) {
        st_sc1(bkey + ob, keys[e]);
        st_sc1(bdoc + ob++, sdoc[i]);
      }
    }
    __syncthreads();  // s_ba / s_bb are rewritten next round
  }
  if (dbg0) sel->tdbg[2] = __builtin_amdgcn_s_memrealtime();
  // 3. the last block.  Hand-off without L2 write-back (MI355X_MICROARCH.md,
  // hand-offs): every gathered entry was stored write-through (sc1), each
  // wave drains its stores, one lane per block adds to the done counter, and
  // the block whose add came last reads everything with sc1 loads.
  __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // (the same thread made this block's gather adds on the same word before,
  // so the last done-add returns every block's totals)
  __shared__ unsigned long long s_fin;
  if (threadIdx.x == 0) {
    const unsigned long long old =
        __hip_atomic_fetch_add(&sel->cnt, 1ull << 48, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = (old >> 48) == gridDim.x - 1 ? 1u : 0u;
    s_fin = old;
  }
  __syncthreads();
  if (!s_last) return;
  if (threadIdx.x == 0) sel->tdbg[3] = __builtin_amdgcn_s_memrealtime();
  uint32_t na = (uint32_t)(s_fin & 0xffff);
  const uint32_t nb = (uint32_t)((s_fin >> 16) & 0xffffffffu);
  if (threadIdx.x == 0) sel->tdbg[6] = nb;
  if (na + nb <= (uint32_t)TK_THREADS) {
    // the usual case: A and B fit one entry a thread -- the answer is the
    // top k of A u B (everything else ranks below bin P), each entry's
    // output position its rank among them (docids are distinct)
    const uint32_t m = na + nb, t = threadIdx.x;
    uint32_t key = 0;
    uint64_t doc = ~0ull;
    if (t < na) {
      key = ld_sc1(akey + t);
      doc = ld_sc1(adoc + t);
    } else if (t < m) {
      key = ld_sc1(bkey + (t - na));
      doc = ld_sc1(bdoc + (t - na));
    }
    sk[t] = key;  // entries past m: key 0, below every gathered key
    sd[t] = doc;
    __syncthreads();
    if (t < m) {
      typedef uint32_t v4 __attribute__((ext_vector_type(4)));
      uint32_t rank = 0;
      const uint32_t m4 = (m + 3) & ~3u;
#pragma unroll 4
      for (uint32_t j = 0; j < m4; j += 4) {
        const v4 kq = *reinterpret_cast<const v4 *>(sk + j);
        rank += (kq.x > key ? 1u : 0u) + (kq.y > key ? 1u : 0u) + (kq.z > key ? 1u : 0u) + (kq.w > key ? 1u : 0u);
        if (kq.x == key) rank += sd[j] < doc ? 1u : 0u;
        if (kq.y == key) rank += sd[j + 1] < doc ? 1u : 0u;
        if (kq.z == key) rank += sd[j + 2] < doc ? 1u : 0u;
        if (kq.w == key) rank += sd[j + 3] < doc ? 1u : 0u;
      }
      if (rank < k) {
        out_key[rank] = key;
        out_doc[rank] = doc;
      }
    }
    for (uint32_t q = m + t; q < k; q += TK_THREADS) {
      out_key[q] = 0u;
      out_doc[q] = ~0ull;
    }
    if (threadIdx.x == 0) {
      sel->tdbg[4] = sel->tdbg[5] = __builtin_amdgcn_s_memrealtime();
      sel->tdbg[7] = 0;
    }
    return;
  }
  uint32_t nt = 0;  // ties of T, compacted to the front of B
  if (nb) {
    // T inside B: bits 15..8, then 7..0
    const uint32_t need = k - na;  // na < k <= s_above + |B|
    for (int t = threadIdx.x; t < 256; t += TK_THREADS) h8[t] = 0;
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nb; i += TK_THREADS) atomicAdd(&h8[(ld_sc1(bkey + i) >> 8) & 0xff], 1u);
    __syncthreads();
    top_bin<TK_THREADS, 256>(h8, need, tmp, &s_bin, &s_above, &s_total);
    const uint32_t c1 = s_bin, need2 = need - s_above;
    __syncthreads();
    for (int t = threadIdx.x; t < 256; t += TK_THREADS) h8[t] = 0;
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nb; i += TK_THREADS) {
      const uint32_t key = ld_sc1(bkey + i);
      if (((key >> 8) & 0xff) == c1) atomicAdd(&h8[key & 0xff], 1u);
    }
    __syncthreads();
    top_bin<TK_THREADS, 256>(h8, need2, tmp, &s_bin, &s_above, &s_total);
    const uint32_t T = (P << 16) | (c1 << 8) | s_bin;
    // B's keys > T join A; its ties move to B's front (in place: a step
    // writes below the entries it has read)
    const uint32_t lim2 = (nb + TK_THREADS - 1) / TK_THREADS * TK_THREADS;
    for (uint32_t i0 = 0; i0 < lim2; i0 += TK_THREADS) {
      const uint32_t i = i0 + threadIdx.x;
      const uint32_t key = i < nb ? ld_sc1(bkey + i) : 0;
      const uint64_t doc = i < nb ? ld_sc1(bdoc + i) : 0;
      __syncthreads();
      na = block_append(key > T, key, doc, akey, adoc, na, tmp);
      nt = block_append(key == T && i < nb, key, doc, bkey, bdoc, nt, tmp);
    }
  }
  if (threadIdx.x == 0) sel->tdbg[4] = __builtin_amdgcn_s_memrealtime();
  // A (fewer than k entries) plus the ties, merged TILE-k at a time (ties
  // beyond one tile only with huge exact-score ties)
  __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // this block's own appends are in place
  for (uint32_t t = threadIdx.x; t < na; t += TK_THREADS) {
    sk[t] = ld_sc1(akey + t);
    sd[t] = ld_sc1(adoc + t);
  }
  uint32_t kept = na, tb = 0;
  for (;;) {
    const uint32_t take = min(nt - tb, (uint32_t)TL - kept);
    for (uint32_t t = threadIdx.x; t < take; t += TK_THREADS) {
      sk[kept + t] = ld_sc1(bkey + tb + t);
      sd[kept + t] = ld_sc1(bdoc + tb + t);
    }
    tb += take;
    __syncthreads();
    lds_sort_best_first(sk, sd, kept + take);
    kept = min(k, kept + take);
    if (tb >= nt) break;
  }
  for (uint32_t t = threadIdx.x; t < k; t += TK_THREADS) {
    out_key[t] = t < kept ? sk[t] : 0u;
    out_doc[t] = t < kept ? sd[t] : ~0ull;
  }
  if (threadIdx.x == 0) {
    sel->tdbg[5] = __builtin_amdgcn_s_memrealtime();
    sel->tdbg[7] = nt;
  }
}

// ------------------------------------------------- Msg3a exchange (RCCL)
// Every GPU holds one docid range of the index (one Msg39 shard each); its
// reply -- the top of its TopTree and its hit count -- is all-gathered over
// xGMI and every rank merges the replies as Msg3a::mergeLists does
// (Msg3a.cpp:1315-1467): the highest score (as double) first, ties to the
// lower docid, a docid already taken skipped, until docsToGet.
struct XHead {
  int32_t n;
  int32_t pad;
  int64_t hits;
};
constexpr uint32_t XMAX = 4096;  // merged entries (docsToGet) the exchange handles
// one entry of a shard's reply as Msg39 sends it: the double score
// (Msg39.cpp:1661-1664: m_score, or (double)m_intScore with integer tree
// scores) and the docid
struct XRec {
  double score;
  uint64_t docid;
};

// this shard's Msg39Reply: min(nodes, docsToGet) entries of its result block
__global__ void k_xpack(const Counters *ctr, const uint32_t *keys, const uint64_t *docs, uint32_t k, uint32_t kq,
                        int int_scores, uint8_t *send) {
  XHead *h = reinterpret_cast<XHead *>(send);
  XRec *r = reinterpret_cast<XRec *>(send + sizeof(XHead));
  __shared__ uint32_t s_n;
  if (threadIdx.x == 0) s_n = 0;
  __syncthreads();
  const uint32_t lim = min(k, kq);
  for (uint32_t i = threadIdx.x; i < lim; i += blockDim.x) {
    const uint32_t key = keys[i];
    const uint32_t b = (key & 0x80000000u) ? (key & 0x7fffffffu) : ~key;
    r[i].score = int_scores ? (double)(int32_t)(key ^ 0x80000000u) : (double)__uint_as_float(b);
    r[i].docid = docs[i];
    // keys are written best first and end at the first 0 (empty) key
    if (key && (i + 1 == lim || keys[i + 1] == 0)) s_n = i + 1;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    h->n = (int32_t)s_n;
    h->pad = 0;
    h->hits = (int64_t)(ctr->surv_top >> 36);
  }
}

// one wave: Msg3a::mergeLists' loop over the shards' replies (Msg3a.cpp:
// 1315-1467).  Lane r < nranks holds shard r's head; every lane then walks
// the heads in shard order exactly as the reference's scan over j does (a
// later head replaces maxj if its score is greater, or if it is not less and
// not greater -- equal, or NaN on either side -- and its docid is lower), so
// the pick is the reference's even where the comparison is not a total
// order.  A docid already merged is passed over (htable, Msg3a.cpp:1381-
// 1385), and the loop stops at k entries.
__global__ void __launch_bounds__(64) k_xmerge(const uint8_t *recv, int nranks, uint32_t k, size_t stride,
                                               uint8_t *out) {
  const int lane = threadIdx.x;
  XHead *oh = reinterpret_cast<XHead *>(out);
  double *osc = reinterpret_cast<double *>(out + sizeof(XHead));
  int64_t *odoc = reinterpret_cast<int64_t *>(out + sizeof(XHead) + 8 * (size_t)k);
  uint32_t cur = 0, n = 0;
  const XRec *rr = nullptr;
  int64_t hits = 0;
  if (lane < nranks) {
    const XHead *h = reinterpret_cast<const XHead *>(recv + stride * lane);
    n = (uint32_t)h->n;
    hits = h->hits;
    rr = reinterpret_cast<const XRec *>(recv + stride * lane + sizeof(XHead));
  }
  for (int off = 32; off > 0; off >>= 1) hits += __shfl_xor(hits, off, 64);
  __shared__ uint64_t s_doc[XMAX];
  __shared__ double s_sc[XMAX];
  uint32_t taken = 0;
  while (taken < k) {
    const bool has = lane < nranks && cur < n;
    const double hs = has ? rr[cur].score : 0.0;
    const uint64_t hd = has ? rr[cur].docid : ~0ull;
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
    if (bl == 64) break;  // every shard exhausted
    if (lane == bl) cur++;
    bool dup = false;
    for (uint32_t t = lane; t < taken; t += 64) dup |= s_doc[t] == bd;
    if (__ballot(dup)) continue;
    if (lane == 0) {
      s_sc[taken] = bs;
      s_doc[taken] = bd;
    }
    wave_lds_sync();
    taken++;
  }
  for (uint32_t t = lane; t < taken; t += 64) {
    osc[t] = s_sc[t];
    odoc[t] = (int64_t)s_doc[t];
  }
  if (lane == 0) {
    oh->n = (int32_t)taken;
    oh->pad = 0;
    oh->hits = hits;
  }
}

// ------------------------------------------------------------- host side
static Weights host_weights() {  // initWeights, Posdb.cpp:1105-1197
  Weights w;
  std::memset(&w, 0, sizeof w);
  float sum = 0.15;
  for (int i = 0; i <= 15; i++) {
    w.diversity[i] = 1.0;
    sum *= 1.135;
  }
  sum = 0.35;
  for (int i = 0; i <= 31; i++) {
    if (sum > 1.0) sum = 1.0;
    w.density[i] = sum;
    sum *= 1.03445;
  }
  for (int i = 0; i <= 15; i++) w.wordspam[i] = (float)(i + 1) / (15 + 1);
  for (int i = 0; i <= 15; i++) w.linker[i] = std::sqrt(1.0 + i);
  for (int i = 0; i < GB_HG_END; i++) {
    w.in_body[i] = (i == GB_HG_BODY || i == GB_HG_HEADING || i == GB_HG_INLIST || i == GB_HG_INMENU);
  }
  for (int i = 0; i < GB_HG_END; i++)
    for (int j = 0; j < GB_HG_END; j++) w.compatible[i][j] = !w.in_body[i] && !w.in_body[j];
  w.hashgroup[GB_HG_BODY] = 1.0;
  w.hashgroup[GB_HG_TITLE] = 8.0;
  w.hashgroup[GB_HG_HEADING] = 1.5;
  w.hashgroup[GB_HG_INLIST] = 0.3;
  w.hashgroup[GB_HG_INMETATAG] = 0.1;
  w.hashgroup[GB_HG_INLINKTEXT] = 16.0;
  w.hashgroup[GB_HG_INTAG] = 1.0;
  w.hashgroup[GB_HG_NEIGHBORHOOD] = 0.0;
  w.hashgroup[GB_HG_INTERNALINLINKTEXT] = 4.0;
  w.hashgroup[GB_HG_INURL] = 1.0;
  w.hashgroup[GB_HG_INMENU] = 0.2;
  return w;
}

// ---------------------------------------------------------- docid splits
// Msg39::controlLoop's docid-range pieces (Msg39.cpp:345-457) over a
// resident list: the units of the runs whose docid lies in [d0, d1], found
// by binary search over run starts (no serial walk), and the docids of the
// first and last run in that window (directory sizing).
struct SplitWin {
  uint32_t lo, hi;
  uint64_t dmin, dmax;
};

__device__ __forceinline__ uint32_t next_run_start(gu8 *p, uint32_t x, uint32_t n) {
  while (x < n && !unit_is_run_start(p + (size_t)x * 6)) x++;
  return x;
}

// first run start whose docid >= v (n if none): predicate "f(x) == n or
// docid(f(x)) >= v" with f = next_run_start is monotone in x
__device__ uint32_t run_lower_bound(gu8 *p, uint32_t n, uint64_t v) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = lo + (hi - lo) / 2;
    const uint32_t r = next_run_start(p, mid, n);
    uint8_t k[12];
    if (r < n) {
      for (int b = 0; b < 12; b++) k[b] = p[(size_t)r * 6 + b];
    }
    if (r == n || unit_docid(k) >= v) hi = mid;
    else lo = r + 1;
  }
  return next_run_start(p, lo, n);
}

__global__ void k_split_windows(const uint64_t *lp, const uint64_t *units, int nl, const uint64_t *d0,
                                const uint64_t *d1, int ns, SplitWin *out) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nl * ns) return;
  const int i = t / ns, j = t % ns;
  const uint32_t n = (uint32_t)units[i];
  SplitWin w{0, 0, 0, 0};
  if (n) {
    gu8 *p = gl(reinterpret_cast<const uint8_t *>(lp[i]));
    w.lo = run_lower_bound(p, n, d0[j]);
    w.hi = run_lower_bound(p, n, d1[j] + 1);
    if (w.hi < w.lo) w.hi = w.lo;
    if (w.lo < w.hi) {
      uint8_t k[12];
      for (int b = 0; b < 12; b++) k[b] = p[(size_t)w.lo * 6 + b];
      w.dmin = unit_docid(k);
      uint32_t x = w.hi - 1;
      while (x > w.lo && !unit_is_run_start(p + (size_t)x * 6)) x--;
      for (int b = 0; b < 12; b++) k[b] = p[(size_t)x * 6 + b];
      w.dmax = unit_docid(k);
    }
  }
  out[t] = w;
}

// A device buffer that grows on demand.  A query slot's buffers are
// stream-ordered (st: the slot's stream): growing one frees and allocates
// in the stream's order from the device pool, so a query larger than the
// slot has seen does not stall the device (hipFree synchronises it) and
// the other slots' queries run on.
struct DevBuf {
  void *p = nullptr;
  size_t cap = 0;
  hipStream_t st = nullptr;
  hipMemPool_t pool = nullptr;  // the context's own pool (stream-ordered buffers); null: hipMalloc
  // GBGPU_CANARY=1 (debug): a guard of CANARY bytes of 0xA5 after every
  // stream-ordered buffer, checked by canary_ok (collect reports a buffer
  // whose guard a kernel overwrote)
  static constexpr size_t CANARY = 1 << 20;
  static int canary_level() {
    static const int lv = [] {
      const char *s = std::getenv("GBGPU_CANARY");
      return s ? std::atoi(s) : 0;
    }();
    return lv;
  }
  static bool canary_on() { return canary_level() != 0; }
  bool canary_ok() const {
    if (!p || !st || !canary_on()) return true;
    std::vector<uint8_t> h(CANARY);
    if (hipMemcpyAsync(h.data(), static_cast<uint8_t *>(p) + cap, CANARY, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
      return false;
    for (uint8_t b : h)
      if (b != 0xA5) return false;
    return true;
  }
  int ensure(size_t bytes) {
    if (bytes <= cap) return 0;
    const size_t want = std::max<size_t>(bytes + bytes / 4, 1 << 16);
    if (st) {
      if (p) (void)hipFreeAsync(p, st);
      p = nullptr;
      cap = 0;
      const size_t guard = canary_on() ? CANARY : 0;
      if (pool_alloc(&p, want + guard, pool, st)) return ENOMEM;
      if (guard) (void)hipMemsetAsync(static_cast<uint8_t *>(p) + want, 0xA5, guard, st);
    } else {
      if (p) (void)hipFree(p);
      p = nullptr;
      cap = 0;
      if (hipMalloc(&p, want) != hipSuccess) return ENOMEM;
    }
    cap = want;
    return 0;
  }
  // stream-ordered allocation from `pool` (or the device's default pool);
  // on failure the pool's cached free memory goes back to the device and
  // the allocation is tried once more
  static int pool_alloc(void **out, size_t bytes, hipMemPool_t pool, hipStream_t st) {
    for (int t = 0; t < 2; t++) {
      const hipError_t e = pool ? hipMallocFromPoolAsync(out, bytes, pool, st) : hipMallocAsync(out, bytes, st);
      if (e == hipSuccess) return 0;
      (void)hipGetLastError();
      if (!pool || t) break;
      (void)hipStreamSynchronize(st);
      (void)hipMemPoolTrimTo(pool, 0);
    }
    *out = nullptr;
    return ENOMEM;
  }
  template <class T> T *as(size_t off = 0) const { return reinterpret_cast<T *>(static_cast<uint8_t *>(p) + off); }
  void release() {
    if (p) {
      if (st) (void)hipFreeAsync(p, st);
      else (void)hipFree(p);
    }
    p = nullptr;
    cap = 0;
  }
};
// GBGPU_DEFAULT_POOL (A/B knob): the device's default pool instead of the
// context's own
#ifndef GBGPU_DEFAULT_POOL
#define GBGPU_DEFAULT_POOL 0
#endif

// Resident lists and file images live in a context-owned arena of hipMalloc'd
// chunks, carved first-fit on the host.  They came from the stream-ordered
// pool until round 6, where a list freed and re-cut at once (the file-read
// path) was sometimes scanned from stale bytes: the granule table its upload
// read back differed run to run while the image itself compared equal
// afterwards, and the queries over it went astray (wrong top docids, 1-9 s
// probes; scripts/r06_fqbug.py).  hipMalloc'd lists never showed it; the
// arena keeps that memory and reuses it with no allocator call per list.
// A list's memory returns to the arena when its last reference goes: every
// query that read it has been collected (synchronised) by then, and the
// upload stream's own work on it is ordered before the next cut.
struct ListArena {
  static constexpr size_t ALIGN = 256;
  static constexpr size_t CHUNK = 1ull << 30;  // the smallest chunk a growth maps
  struct Chunk {
    uint8_t *base = nullptr;
    size_t size = 0, used = 0;
    std::map<size_t, size_t> free_;  // offset -> bytes, coalesced
  };
  std::mutex mu;
  std::vector<Chunk> chunks;
  int device = 0;
  uint8_t *alloc(size_t bytes) {
    bytes = (std::max<size_t>(bytes, 1) + ALIGN - 1) / ALIGN * ALIGN;
    std::lock_guard<std::mutex> g(mu);
    for (auto &c : chunks)
      for (auto it = c.free_.begin(); it != c.free_.end(); ++it)
        if (it->second >= bytes) {
          const size_t off = it->first, len = it->second;
          c.free_.erase(it);
          if (len > bytes) c.free_[off + bytes] = len - bytes;
          c.used += bytes;
          return c.base + off;
        }
    Chunk c;
    c.size = std::max(bytes, CHUNK);
    (void)hipSetDevice(device);
    if (hipMalloc(reinterpret_cast<void **>(&c.base), c.size) != hipSuccess) {
      (void)hipGetLastError();
      // no room for a new chunk: the wholly free ones go back first
      trim_locked(0);
      if (hipMalloc(reinterpret_cast<void **>(&c.base), c.size) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
      }
    }
    if (c.size > bytes) c.free_[bytes] = c.size - bytes;
    c.used = bytes;
    chunks.push_back(std::move(c));
    return chunks.back().base;
  }
  void free(uint8_t *p, size_t bytes) {
    bytes = (std::max<size_t>(bytes, 1) + ALIGN - 1) / ALIGN * ALIGN;
    std::lock_guard<std::mutex> g(mu);
    for (auto &c : chunks) {
      if (p < c.base || p >= c.base + c.size) continue;
      size_t off = (size_t)(p - c.base), len = bytes;
      auto nx = c.free_.lower_bound(off);
      if (nx != c.free_.end() && nx->first == off + len) {
        len += nx->second;
        nx = c.free_.erase(nx);
      }
      if (nx != c.free_.begin()) {
        auto pv = std::prev(nx);
        if (pv->first + pv->second == off) {
          off = pv->first;
          len += pv->second;
          c.free_.erase(pv);
        }
      }
      c.free_[off] = len;
      c.used -= bytes;
      return;
    }
  }
  // wholly free chunks beyond `keep` bytes of them go back to the device
  void trim_locked(size_t keep) {
    size_t kept = 0;
    for (size_t i = 0; i < chunks.size();) {
      Chunk &c = chunks[i];
      if (c.used == 0 && kept + c.size > keep) {
        (void)hipFree(c.base);
        chunks.erase(chunks.begin() + (long)i);
        continue;
      }
      if (c.used == 0) kept += c.size;
      i++;
    }
  }
  void trim(size_t keep) {
    std::lock_guard<std::mutex> g(mu);
    trim_locked(keep);
  }
  ~ListArena() {
    for (auto &c : chunks) (void)hipFree(c.base);
  }
};

struct ListMem {
  uint8_t *d = nullptr;
  size_t bytes = 0;
  std::shared_ptr<ListArena> arena;  // owner of d
  size_t dbg_len = 0;     // GBGPU_CANARY: bytes hashed (image, pad, page map)
  uint64_t dbg_hash = 0;  // and their hash when the list was finished
  uint64_t hash(hipStream_t s) const {
    std::vector<uint64_t> h((dbg_len + 7) / 8, 0);
    if (hipMemcpyAsync(h.data(), d, dbg_len, hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
      return 0;
    uint64_t x = 1469598103934665603ull;
    for (uint64_t v : h) x = (x ^ v) * 1099511628211ull;
    return x;
  }
  int alloc(const std::shared_ptr<ListArena> &a, size_t n) {
    arena = a;
    bytes = n;
    d = a->alloc(n);
    return d ? 0 : ENOMEM;
  }
  ~ListMem() {
    if (d && arena) arena->free(d, bytes);
  }
};

struct ListEntry {
  uint8_t *d = nullptr;
  uint32_t *pm = nullptr;        // its page map (k_page_count / k_page_scan), in the same allocation
  std::shared_ptr<ListMem> mem;  // owner of d (null for docid-split windows)
  int64_t size = 0;   // original bytes (18-byte first key)
  uint32_t units = 0; // swapped units
  uint64_t dmin = 0, dmax = 0;  // docid of the first and of the last run
  // first run docid at or after each WCH_UNITS-unit granule (k_list_scan; host
  // copy, resident lists only): the probe spans' start docids
  std::shared_ptr<const std::vector<uint64_t>> gfirst;
  bool live = false;
};

// An uploaded (or cut) list's one pass over its bytes, a 2048-unit page a
// block, from the page staged in LDS: the structure check (every unit
// classified alone, Posdb.h:887-889: a unit with the half bit byte1 & 0x02
// starts a key, which must carry a size bit in byte 0, and a 12-byte key's
// second unit must not look like a key start; the list starts with a key), the
// page's run starts (the page map), the first run docid of each of its four
// granules (the granule table: ~0 where the page has none from there on; the
// host carries the next page's first into those), and the last run docid
// (dmax).
struct ListHdr {
  uint32_t bad;
  uint32_t pad;
  unsigned long long dmax;  // unused (the pages' last docids carry it)
};
static_assert(CHUNK_UNITS == 4 * WCH_UNITS, "four granules a page");
// A termlist cut from a resident file (gbgpu_file_list): the swapped list
// image is the map key's first 12 bytes (k, half bit set), then the file's
// bytes [src, src + n).  src is 2-byte aligned (file offsets and key sizes
// are even), so an odd half-dword source is two dword loads joined.
struct CutSrc {
  const uint8_t *file;
  uint64_t fsize, src, n;
  uint32_t k[3];
  uint32_t *dst;  // the list image
};
__device__ __forceinline__ uint32_t cut_dword(const CutSrc &c, uint64_t j) {
  const uint64_t len = 12 + c.n;
  if (4 * j >= len) return 0;  // the zeroed pad
  if (j < 3) return c.k[j];
  const uint32_t *fw = reinterpret_cast<const uint32_t *>(c.file);
  const uint64_t fmax = (c.fsize + 3) / 4 - 1;
  const uint64_t fb = c.src + 4 * j - 12, a = fb >> 2;
  uint32_t v = fw[min(a, fmax)];
  if (fb & 2) v = (v >> 16) | (fw[min(a + 1, fmax)] << 16);
  const uint64_t left = len - 4 * j;
  if (left < 4) v &= (1u << (8 * left)) - 1;
  return v;
}

// CUT: the block builds its page from the file instead of reading the list
// (the dwords staged in LDS and its own page's written to the list image),
// so a cut is one pass over its bytes
template <bool CUT>
__global__ void __launch_bounds__(BLOCK) k_list_scan(const uint8_t *__restrict__ list, uint32_t units,
                                                     uint32_t *__restrict__ pm, uint64_t *__restrict__ gf,
                                                     uint64_t *__restrict__ lastd, ListHdr *hdr, CutSrc cut) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[CHUNK_LOAD];
  __shared__ uint32_t tmp[BLOCK / 64];
  __shared__ uint32_t s_first[4], s_last;
  const uint32_t u0 = blockIdx.x * (uint32_t)CHUNK_UNITS;
  if (threadIdx.x < 4) s_first[threadIdx.x] = ~0u;
  if (threadIdx.x == 0) s_last = 0;
  if constexpr (CUT) {
    static_assert(CHUNK_BYTES % 4 == 0 && CHUNK_LOAD % 4 == 0, "whole dwords a page");
    const uint64_t j0 = (uint64_t)u0 * 6 / 4;
    uint32_t *ld = reinterpret_cast<uint32_t *>(lds);
    uint32_t *img = cut.dst;
    for (int i = threadIdx.x; i < CHUNK_LOAD / 4; i += BLOCK) {
      const uint32_t v = cut_dword(cut, j0 + i);
      ld[i] = v;
      if (i < CHUNK_BYTES / 4) img[j0 + i] = v;
    }
  } else {
    load_chunk(list, u0, lds);
  }
  __syncthreads();
  // the thread's units' bytes 0-1 from three 16-B LDS reads (as thread_starts)
  // and the next thread's first unit's from one aligned word: byte reads at
  // the 48-byte thread stride were 4-way bank conflicts
  uint32_t h[UPT + 1];
  {
    typedef uint32_t v4 __attribute__((ext_vector_type(4)));
    const v4 *src = reinterpret_cast<const v4 *>(lds + threadIdx.x * UPT * 6);
    const v4 a = src[0], b = src[1], c = src[2];
    const uint32_t w[12] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x, c.y, c.z, c.w};
#pragma unroll
    for (int q = 0; q < UPT; q++) h[q] = (q & 1) ? (w[3 * (q >> 1) + 1] >> 16) : (w[3 * (q >> 1)] & 0xffffu);
    h[UPT] = *reinterpret_cast<const uint32_t *>(lds + (threadIdx.x + 1) * UPT * 6) & 0xffffu;  // < CHUNK_LOAD
  }
  uint32_t m = 0, bad = 0;
#pragma unroll
  for (int q = 0; q < UPT; q++) {
    const uint32_t u = u0 + threadIdx.x * UPT + q;
    if (u >= units) break;
    if (!(h[q] & 0x0200u)) {
      if (u == 0) bad = 1;  // the list must start with a key
      continue;
    }
    if (!(h[q] & 0x06u)) bad = 1;
    if (!(h[q] & 0x04u)) {
      m |= 1u << q;  // a 12-byte key: a run start
      if (u + 1 >= units || (h[q + 1] & 0x0200u)) bad = 1;
    }
  }
  if (__ballot(bad) && (threadIdx.x & 63) == 0) atomicOr(&hdr->bad, 1u);
  if (m) {
    const uint32_t f = threadIdx.x * UPT + (uint32_t)(__ffs(m) - 1);
    atomicMin(&s_first[f / WCH_UNITS], f);
    atomicMax(&s_last, threadIdx.x * UPT + (uint32_t)(31 - __clz(m)) + 1);
  }
  uint32_t tot;
  block_exclusive_scan(__popc(m), tmp, &tot);  // its barriers order the LDS atomics
  if (threadIdx.x == 0) pm[blockIdx.x] = tot;
  if (threadIdx.x < 4) {
    uint32_t f = ~0u;  // the first run start at or after the granule, in this page
    for (int g = 3; g >= (int)threadIdx.x; g--) f = s_first[g] != ~0u ? s_first[g] : f;
    gf[(size_t)blockIdx.x * 4 + threadIdx.x] = f == ~0u ? ~0ull : lds_unit_docid(lds, f);
  }
  // the page's last run docid (~0: no run start in the page); the host takes
  // the list's last (one global atomic a page serialised the launch)
  if (threadIdx.x == 0) lastd[blockIdx.x] = s_last ? lds_unit_docid(lds, s_last - 1) : ~0ull;
}

// one block: the page map's exclusive scan (total at pm[npages])
__global__ void __launch_bounds__(1024) k_list_tail(uint32_t npages, uint32_t *pm) {
  __shared__ uint32_t tmp[16];
  __shared__ uint32_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (uint32_t base = 0; base < npages; base += 1024) {
    const uint32_t i = base + threadIdx.x;
    const uint32_t v = i < npages ? pm[i] : 0;
    uint32_t x = v;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    if (lane == 63) tmp[wid] = x;
    __syncthreads();
    uint32_t pre = 0;
    for (int w = 0; w < wid; w++) pre += tmp[w];
    const uint32_t incl = carry + pre + x;
    __syncthreads();
    if (i < npages) pm[i] = incl - v;
    if (threadIdx.x == 1023) carry = incl;
    __syncthreads();
  }
  if (threadIdx.x == 0) pm[npages] = carry;
}

// docid of the key starting at p (Posdb.h:295)
static uint64_t host_docid(const uint8_t *p) {
  uint64_t d = 0;
  for (int i = 11; i >= 7; i--) d = (d << 8) | p[i];
  return d >> 2;
}

static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

}  // namespace gbgpu

using namespace gbgpu;

// One query in flight: its stream, device buffers (grown, then reused),
// pinned staging and result state.  A context owns one or more slots; the
// resident lists are shared by all of them.
constexpr int MAXF = 4;                // facet terms per query
constexpr int MAX_FACET_RANGES = 256;  // QueryWord::m_facetRange{Int,Float}{A,B}

// a facet query term of the slot's query (enqueue_entries)
struct FacetTerm {
  int term;
  int lid;  // its group's list, or -1 (no group: the table holds its ranges only)
  int isfloat;
  std::vector<int32_t> a, b;  // ranges
  uint32_t units;
  const uint8_t *list;
};


// docid splits: each facet query term's table and docid count over the
// pieces (Msg39 runs one Query, whose QueryTerms keep them), by query term
struct FacetAcc {
  std::map<int, std::map<int32_t, gbgpu_facet_entry>> tab;
  std::map<int, uint64_t> docs;
};

struct QuerySlot {
  std::mutex mu;
  hipStream_t stream = nullptr;
  DevBuf tables, chunkcnt, cand, cunit, bits, loc, svslot, svlm, svu, svdoc, svloc, scratch, skey, sel, gath, res, stg;
  DevBuf dir;           // candidate directories, epoch-tagged (never cleared per query)
  DevBuf split, swin;   // docid splits: one piece's list windows; window table
  DevBuf blk, sflag, ord, oslot, rep, tree;  // site clustering: slot-order ranks and slots, replay entries, TopTree state
  DevBuf white, wrej;                       // "&sites=" whitelist: sorted 5-byte values; rejected slots
  DevBuf si;                                // second pass's score info (score_info)
  DevBuf fac;                               // facet tables (facet_pass)
  DevBuf svmb, stale;                       // survivors' mbuf bytes; the stale-mbuf survivors (stale_fix)
  DevBuf si2;                               // the second pass's stale-byte replay (k_si_stale)
  DevBuf mwsl;                              // facets with site clustering: minWinningScore's assignments
  FacetAcc *facc = nullptr;                 // docid splits: the facet tables over the pieces (facet_pass)
  uint64_t rep_off = 0;                     // the replay entries in slot order: q.rep + rep_off (k_bound)
  std::vector<FacetTerm> facets;            // the query's facet terms with a table
  std::vector<uint64_t> h_white;            // its host copy (the upload's source)
  uint32_t epoch = 0;
  uint8_t *h_stage = nullptr;  // pinned: query tables (host -> device, one copy)
  size_t stage_cap = 0;
  uint8_t *h_res = nullptr;    // pinned: counters + top list (device -> host, one copy)
  size_t hres_cap = 0;
  std::vector<G0Chunk> g0c;
  std::vector<ProbeWork> pw;  // the candidate-driven probe waves (DevPlan::nwork_cand)
  uint32_t nwork = 0;         // k_probe waves: pw, then the run-driven segments
  std::vector<uint32_t> afirst;
  std::vector<std::shared_ptr<ListMem>> held;  // lists the in-flight query reads
  // state of the in-flight query
  bool pending = false;
  bool replayed = false;  // site clustering: the pass ran the TopTree replay
  bool seq_replay = false;  // ... as k_tree_seq (a register-tree overflow replays it with k_tree_replay)
  bool whole_range = false; // ... over the whole docid range in one pass (no docid-split pieces)
  uint64_t slot_ub = 0;
  bool early = false;
  int k = 0;
  size_t res_bytes = 0;
  int32_t docs_wanted = 0;
  bool want_info = false;   // m_getDocIdScoringInfo
  bool stale_done = false;  // stale_fix ran for the pending query (before the exchange packed it)
  int32_t stale_filt = 0;   // ... and the paging filter's drops among its survivors
  bool int_scores = false;  // gbsortby int: keys are m_intScore, TopNode::m_score 0
  int info_docs = 0;        // m_docsToGet: the second pass's docid limit
  int info_nterms = 0;      // m_q->m_numTerms and m_realMaxTop (allocTopTree's reservations)
  int info_rmt = 0;
  int info_ng = 0;          // m_numQueryTermInfos
  int info_scap = 0, info_pcap = 0;  // singles / pairs one docid can record
  int64_t scan_bytes = 0;
  int64_t g0_bytes = 0, probe_bytes = 0;  // list bytes of candidate extraction / of the probe scan
  int64_t stats[8] = {};                   // gbgpu_slot_stats of the last collected query
  hipEvent_t ev[7] = {};
  hipEvent_t ev_done = nullptr;  // the query's device work is done (the exchange waits on it)
  float last_ms[6] = {0, 0, 0, 0, 0, 0};

  // site clustering over docid splits: the tree a piece started from
  // (stale_fix_clustered replays the piece from it), the piece's TREE_* phase
  DevBuf tree_bak;
  int tree_phase = 0;
  DevBuf *const bufs[35] = {&tables, &chunkcnt, &cand, &cunit, &bits, &loc, &svslot, &svlm, &svu, &svdoc,
                            &svloc, &scratch, &skey, &sel, &gath, &res, &dir, &split, &swin, &blk,
                            &sflag, &ord, &oslot, &rep, &tree, &white, &wrej, &si, &fac, &svmb, &stale, &si2, &mwsl,
                            &stg, &tree_bak};
  int init(hipMemPool_t pool) {
    if (hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) != hipSuccess) return GBGPU_EHIP;
    for (auto *b : bufs) {
      b->st = stream;
      b->pool = pool;
    }
    for (auto &e : ev)
      if (hipEventCreate(&e) != hipSuccess) return GBGPU_EHIP;
    if (hipEventCreateWithFlags(&ev_done, hipEventDisableTiming) != hipSuccess) return GBGPU_EHIP;
    return 0;
  }
  void release() {
    if (stream) (void)hipStreamSynchronize(stream);
    for (auto *b : bufs) b->release();
    if (stream) (void)hipStreamSynchronize(stream);
    if (h_stage) (void)hipHostFree(h_stage);
    if (h_res) (void)hipHostFree(h_res);
    h_stage = h_res = nullptr;
    for (auto &e : ev)
      if (e) (void)hipEventDestroy(e);
    if (ev_done) (void)hipEventDestroy(ev_done);
    if (stream) (void)hipStreamDestroy(stream);
    stream = nullptr;
  }
};

constexpr int MAX_SLOTS = 64;
constexpr uint64_t POOL_KEEP = 16ull << 30;  // free bytes the context's pool may keep cached

// A Posdb Rdb file image resident in HBM (gbgpu_file_upload): the bytes as
// they lie on disk, termlists back to back.  Termlists are cut from it on the
// device (gbgpu_file_list), the read Msg3/RdbScan makes from disk.
struct FileEntry {
  std::shared_ptr<ListMem> mem;
  int64_t size = 0;
  bool live = false;
};

// Exchange sequencer (gbgpu.h "Exchange ordering"): one caller at a time,
// admitted in increasing sequence number.
struct gbgpu_seq {
  std::mutex mu;
  std::condition_variable cv;
  uint64_t next = 0;  // the number admitted next
  bool busy = false;  // `next` has been admitted and not yet left
};

static int seq_enter(gbgpu_seq *s, uint64_t seq, int timeout_ms) {
  std::unique_lock<std::mutex> g(s->mu);
  if (seq < s->next || (seq == s->next && s->busy)) return EINVAL;
  auto ready = [&] { return s->next == seq && !s->busy; };
  if (timeout_ms < 0) {
    s->cv.wait(g, ready);
  } else if (!s->cv.wait_for(g, std::chrono::milliseconds(timeout_ms), ready)) {
    return ETIMEDOUT;
  }
  s->busy = true;
  return 0;
}

static int seq_leave(gbgpu_seq *s, uint64_t seq) {
  {
    std::lock_guard<std::mutex> g(s->mu);
    if (!s->busy || s->next != seq) return EINVAL;
    s->busy = false;
    s->next++;
  }
  s->cv.notify_all();
  return 0;
}

struct gbgpu_ctx {
  int device = 0;
  hipStream_t upload_stream = nullptr;
  uint32_t *d_flag = nullptr;  // upload validation result (device / pinned host)
  uint32_t *h_flag = nullptr;
  std::mutex free_mu;          // a slot became free (gbgpu_query_resident waits on it)
  std::condition_variable free_cv;
  std::mutex lists_mu;
  std::vector<ListEntry> lists;
  std::vector<FileEntry> files;  // resident Rdb file images (gbgpu_file_upload), under lists_mu
  hipMemPool_t pool = nullptr;  // stream-ordered device memory of the slots, lists and files
  std::mutex slots_mu;  // guards growth of the slot table
  QuerySlot *slots[MAX_SLOTS] = {};
  int nslots = 0;
  bool profiling = false;
  int probe_mode = 0;  // diagnostic only (GBGPU_PROBE_MODE)
  int replay_mode = 0;  // diagnostic only (GBGPU_REPLAY_MODE): 1 the one-wave k_tree_replay always, 3 one register column
  int probe_waves = 0;  // diagnostic: probe spans (GBGPU_PROBE_WAVES; 0 = PROBE_WAVES)
  int probe_runspan = 0;  // diagnostic: chunks per run-driven probe wave (GBGPU_PROBE_RUNSPAN; 0 = 1)
  // candidates a 3 KiB chunk meets above which a list is probed run-driven
  // (GBGPU_PROBE_DIR_T in the diagnostic build): config 3's probe phase at
  // 64 / 128 / 256 / 384 / 768 / 1024: 0.457 / 0.339 / 0.263 / 0.240 / 0.342
  // / 0.394 ms a query (scripts/r06_c3dir.sh); config 2 meets ~36 either way
  double probe_dir_t = 384.0;
  int score_mode = 0;  // diagnostic only (GBGPU_SCORE_MODE): 1 mini-merge without scoring
  int debug_ext = 0;   // diagnostic only (GBGPU_DEBUG_EXT): print the re-shrink table per query
  uint64_t *d_sdbg = nullptr;  // GBGPU_SCORE_MODE=2: per-wave k_score timing (GBGPU_SCORE_DUMP file)
  unsigned long long *d_pdbg = nullptr;  // GBGPU_PROBE_DEBUG_DOC: k_probe's trace of one docid (one slot: the
                                         // buffer is shared, so the trace is meaningful with one query in flight)
  const char *probe_dbg_doc = nullptr;   // its value, read once at gbgpu_open
  bool topk_debug = false;               // GBGPU_TOPK_DEBUG: k_topk / replay phase clocks to stderr
  uint32_t sdbg_grid = 0;
  std::mutex merge_mu;
  gbmerge::MergeState *merge = nullptr;  // created on first use (merge.hip)
  // Msg3a exchange over RCCL (gbgpu_comm_init / gbgpu_allgather_topk)
  std::mutex x_mu;
  ncclComm_t comm = nullptr;
  int nranks = 1, rank = 0;
  gbgpu_seq xseq;  // orders gbgpu_allgather_topk across this rank's threads
  hipStream_t xstream = nullptr;
  DevBuf xsend, xrecv, xout;
  uint8_t *h_xout = nullptr;
  size_t h_xout_cap = 0;
  // the full-reply merge's device scratch and its pinned host stage (the
  // heads, the pack, the merged block): plain allocations the exchange owns,
  // grown between calls, so no copy touches pageable memory
  DevBuf xscratch;
  uint8_t *h_xf = nullptr;
  size_t h_xf_cap = 0;
  // a list upload's readbacks (granule table, pages' last docids, header):
  // pinned, grown between uploads (under lists_mu)
  uint8_t *h_lst = nullptr;
  size_t h_lst_cap = 0;
  DevBuf lscan;                              // and their device side (k_list_scan's outputs)
  DevBuf min_runs, mout;                     // gbgpu_termlist_merge's runs and merged list
  std::shared_ptr<ListArena> arena = std::make_shared<ListArena>();  // lists and file images
  int ensure_h_lst(size_t bytes) {
    if (bytes <= h_lst_cap) return 0;
    if (h_lst) (void)hipHostFree(h_lst);
    h_lst = nullptr;
    h_lst_cap = 0;
    const size_t want = std::max<size_t>(bytes + bytes / 4, 1 << 16);
    if (hipHostMalloc(reinterpret_cast<void **>(&h_lst), want) != hipSuccess) {
      h_lst = nullptr;
      return ENOMEM;
    }
    h_lst_cap = want;
    return 0;
  }
  int ensure_h_xf(size_t bytes) {
    if (bytes <= h_xf_cap) return 0;
    if (h_xf) (void)hipHostFree(h_xf);
    h_xf = nullptr;
    h_xf_cap = 0;
    const size_t want = std::max<size_t>(bytes + bytes / 4, 1 << 18);
    if (hipHostMalloc(reinterpret_cast<void **>(&h_xf), want) != hipSuccess) {
      h_xf = nullptr;
      return ENOMEM;
    }
    h_xf_cap = want;
    return 0;
  }
};

// result block layout: [Counters | keys k | docids k]
static size_t res_keys_off() { return align256(sizeof(Counters)); }
static size_t res_docs_off(int k) { return res_keys_off() + align256(4 * (size_t)std::max(k, 1)); }
static size_t res_size(int k) { return res_docs_off(k) + 8 * (size_t)std::max(k, 1); }

// the page map of a swapped list of `units` units: bytes to reserve, and its
// build (two launches on `st`; an empty list's map is its zeroed total)
static size_t page_map_bytes(uint32_t units) {
  return align256(4 * ((size_t)(units + CHUNK_UNITS - 1) / CHUNK_UNITS + 1));
}
static int build_page_map(const uint8_t *d, uint32_t units, uint32_t *pm, hipStream_t st) {
  const uint32_t np = (units + CHUNK_UNITS - 1) / CHUNK_UNITS;
  if (!np) return 0;
  hipLaunchKernelGGL(k_page_count, dim3(np), dim3(BLOCK), 0, st, d, units, pm);
  hipLaunchKernelGGL(k_page_scan, dim3(1), dim3(1024), 0, st, np, pm);
  HIPCHECK(hipGetLastError());
  return 0;
}

// a list entry of `size` original bytes (18-byte first key), its device
// image and page map allocated and zeroed on the upload stream
static int alloc_list(gbgpu_ctx *ctx, int64_t size, ListEntry &e) {
  if (size < 0 || (size > 0 && size < 18) || (size > 0 && (size - 18) % 6 != 0)) return EINVAL;
  if ((size - 6) / 6 > 0xfffffff0LL) return GBGPU_ECAPACITY;
  e.size = size;
  e.units = size ? (uint32_t)((size - 6) / 6) : 0;
  const size_t lbytes = align256((size_t)(size ? size - 6 : 0) + LIST_PAD);
  const size_t alloc = lbytes + page_map_bytes(e.units);
  e.mem = std::make_shared<ListMem>();
  if (e.mem->alloc(ctx->arena, alloc)) return ENOMEM;
  e.d = e.mem->d;
  e.pm = reinterpret_cast<uint32_t *>(e.d + lbytes);
  // the image's own bytes are written next: zero the pad and the page map
  const size_t img = (size_t)(size ? size - 6 : 0);
  HIPCHECK(hipMemsetAsync(e.d + img, 0, alloc - img, ctx->upload_stream));
  return 0;
}

static int finish_list(gbgpu_ctx *ctx, ListEntry &e, const uint8_t *host_bytes, const uint8_t *first18,
                       int32_t *handle, const CutSrc *cut = nullptr);

static int upload_list(gbgpu_ctx *ctx, const uint8_t *bytes, int64_t size, int32_t *handle) {
  ListEntry e;
  int rc = alloc_list(ctx, size, e);
  if (rc) return rc;
  // the first key must be a whole 18-byte key (Posdb.cpp:5671-5703 swaps it)
  if (size > 0 && (bytes[0] & 0x06)) return GBGPU_ECORRUPT;  // e.mem frees the image
  if (size) {
    // device image = the list after the first-key swap (Posdb.cpp:5689-5698):
    // original bytes 0..11 with the half bit set, then bytes 18..size-1
    uint8_t first[12];
    std::memcpy(first, bytes, 12);
    first[0] |= 0x02;
    HIPCHECK(hipMemcpyAsync(e.d, first, 12, hipMemcpyHostToDevice, ctx->upload_stream));
    if (size > 18)
      HIPCHECK(hipMemcpyAsync(e.d + 12, bytes + 18, (size_t)(size - 18), hipMemcpyHostToDevice, ctx->upload_stream));
  }
  return finish_list(ctx, e, bytes, bytes, handle);
}

// The common tail of a list's upload once its device image is enqueued:
// structure check, page map, granule table; then the docid range, from the
// host bytes when the caller has them, else from the device image's last
// granule that holds a run start.
// the scan's outputs read back (granule table, pages' last docids, header)
// into the entry: the structure check, the granule table, dmin / dmax
static int scan_result(ListEntry &e, const uint8_t *h_gf, const uint8_t *h_last, const uint8_t *h_hdr, uint32_t np,
                       const uint8_t *first18) {
  ListHdr hh;
  std::memcpy(&hh, h_hdr, sizeof hh);
  if (hh.bad) return GBGPU_ECORRUPT;  // e.mem frees the copy
  const size_t ngran = (size_t)np * 4;
  std::vector<uint64_t> gf(ngran);
  std::memcpy(gf.data(), h_gf, 8 * ngran);
  // a granule with no run start after it in its page takes the next
  // page's first (docids ascend; ~0: none); granules past the list's units
  // (the last page's tail) hold ~0
  for (size_t g = ngran - 1; g-- > 0;)
    if (gf[g] == ~0ull) gf[g] = gf[g + 1];
  gf.resize((e.units + WCH_UNITS - 1) / WCH_UNITS);
  e.dmin = host_docid(first18);  // the first key (the list starts with a run)
  e.dmax = 0;
  for (size_t pg = np; pg-- > 0;) {
    uint64_t d;
    std::memcpy(&d, h_last + 8 * pg, 8);
    if (d != ~0ull) {
      e.dmax = d;
      break;
    }
  }
  e.gfirst = std::make_shared<const std::vector<uint64_t>>(std::move(gf));
  return 0;
}

// a checked list into the context's table
static int register_list(gbgpu_ctx *ctx, ListEntry &e, int32_t *handle) {
  if (DevBuf::canary_level() == 5 && e.size) {
    uint64_t x = 1469598103934665603ull;
    for (uint64_t v : *e.gfirst) x = (x ^ v) * 1099511628211ull;
    std::fprintf(stderr, "gbgpu: list %p size %lld units %u dmin %llu dmax %llu gf %zu %016llx\n", (void *)e.d,
                 (long long)e.size, e.units, (unsigned long long)e.dmin, (unsigned long long)e.dmax, e.gfirst->size(),
                 (unsigned long long)x);
  }
  if ((DevBuf::canary_level() == 1 || DevBuf::canary_level() == 2) && e.size) {
    e.mem->dbg_len = (size_t)(reinterpret_cast<uint8_t *>(e.pm) - e.d) + page_map_bytes(e.units);
    e.mem->dbg_hash = e.mem->hash(ctx->upload_stream);
  }
  e.live = true;
  for (size_t i = 0; i < ctx->lists.size(); i++) {
    if (!ctx->lists[i].live) {
      ctx->lists[i] = e;
      *handle = (int32_t)i;
      return 0;
    }
  }
  ctx->lists.push_back(e);
  *handle = (int32_t)ctx->lists.size() - 1;
  return 0;
}

static int finish_list(gbgpu_ctx *ctx, ListEntry &e, const uint8_t *host_bytes, const uint8_t *first18,
                       int32_t *handle, const CutSrc *cut) {
  (void)host_bytes;
  if (e.size) {
    // one pass over the bytes (k_list_scan), the page scan (k_list_tail),
    // then ONE synchronisation for the check, the granule table and the last
    // run docid, read back through the pinned stage
    const uint32_t np = (e.units + CHUNK_UNITS - 1) / CHUNK_UNITS;
    const uint32_t ngran = np * 4;
    DevBuf &dgf = ctx->lscan;  // the context's scan buffer, grown between uploads (under lists_mu)
    const size_t o_last = align256(8 * (size_t)ngran), o_hdr = o_last + align256(8 * (size_t)np);
    const size_t need = o_hdr + sizeof(ListHdr);
    if (dgf.ensure(need) || ctx->ensure_h_lst(need)) return ENOMEM;
    ListHdr *dh = reinterpret_cast<ListHdr *>(dgf.as<uint8_t>(o_hdr));
    HIPCHECK(hipMemsetAsync(dh, 0, sizeof(ListHdr), ctx->upload_stream));
    if (cut)
      hipLaunchKernelGGL(k_list_scan<true>, dim3(np), dim3(BLOCK), 0, ctx->upload_stream, e.d, e.units, e.pm,
                         dgf.as<uint64_t>(), dgf.as<uint64_t>(o_last), dh, *cut);
    else
      hipLaunchKernelGGL(k_list_scan<false>, dim3(np), dim3(BLOCK), 0, ctx->upload_stream, e.d, e.units, e.pm,
                         dgf.as<uint64_t>(), dgf.as<uint64_t>(o_last), dh, CutSrc{});
    hipLaunchKernelGGL(k_list_tail, dim3(1), dim3(1024), 0, ctx->upload_stream, np, e.pm);
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipMemcpyAsync(ctx->h_lst, dgf.p, need, hipMemcpyDeviceToHost, ctx->upload_stream));
    HIPCHECK(hipStreamSynchronize(ctx->upload_stream));
    const int rc = scan_result(e, ctx->h_lst, ctx->h_lst + o_last, ctx->h_lst + o_hdr, np, first18);
    if (rc) return rc;
  }
  return register_list(ctx, e, handle);
}

// Validates a request and copies the list-table entries it names (the table
// may grow under us).
static int snapshot_lists(gbgpu_ctx *ctx, const gbgpu_qterm *terms, int nterms, const int32_t *handles,
                          const gbgpu_params *p, std::vector<ListEntry> &ents) {
  if (!p || nterms < 0 || (nterms && (!terms || !handles))) return EINVAL;
  if (p->docs_to_get <= 0 || p->real_max_top <= 0 || p->num_docid_splits <= 0) return EINVAL;
  if (nterms > 1024) return GBGPU_EUNSUPPORTED;
  ents.resize(nterms);
  std::lock_guard<std::mutex> g(ctx->lists_mu);
  for (int i = 0; i < nterms; i++) {
    int32_t h = handles[i];
    if (h < 0 || h >= (int32_t)ctx->lists.size() || !ctx->lists[h].live) return EINVAL;
    ents[i] = ctx->lists[h];
  }
  return 0;
}

// site clustering: which part of Msg39's one-tree-over-all-pieces a pass is
constexpr int TREE_INIT = 1;   // the pass starts the TopTree
constexpr int TREE_FINAL = 2;  // the pass ends it: the tree is the result
constexpr int TREE_EMIT = 4;   // the pass also writes the tree out (score info over docid splits)

static int enqueue_entries(gbgpu_ctx *ctx, QuerySlot &q, const gbgpu_qterm *terms, int nterms,
                           const ListEntry *ents, const gbgpu_params *p, int32_t dw_override,
                           int tree_phase = TREE_INIT | TREE_FINAL);

// One whole-range query (no docid splits) on slot q's stream.
static int enqueue(gbgpu_ctx *ctx, QuerySlot &q, const gbgpu_qterm *terms, int nterms, const int32_t *handles,
                   const gbgpu_params *p) {
  std::vector<ListEntry> ents;
  int rc = snapshot_lists(ctx, terms, nterms, handles, p, ents);
  if (rc) return rc;
  if (p->num_docid_splits > 1) return GBGPU_EUNSUPPORTED;  // blocking entry points only
  // held before anything is launched: a failed enqueue may have launched
  // kernels that read the lists; the next collect on this slot drains them
  for (auto &e : ents)
    if (e.mem) {
      q.held.push_back(e.mem);
      if (DevBuf::canary_level() == 3) {
        std::vector<uint8_t> one(64);
        (void)hipMemcpyAsync(one.data(), e.mem->d, 64, hipMemcpyDeviceToHost, q.stream);
        (void)hipStreamSynchronize(q.stream);
      }
      if (e.mem->dbg_len && e.mem->hash(q.stream) != e.mem->dbg_hash)
        std::fprintf(stderr, "gbgpu: canary: list %p changed before enqueue\n", (void *)e.mem->d);
    }
  return enqueue_entries(ctx, q, terms, nterms, ents.data(), p, 0);
}

// One PosdbTable pass over the given lists on slot q's stream.  dw_override
// > 0 fixes TopTree::m_docsWanted (docid splits size the tree once, at the
// first piece: Msg39.cpp:938-966).
// TopTree::setNumNodes' sizing (TopTree.cpp:64-101) for the replay
static TreeParams tree_params(int32_t dw, int phase, bool ints) {
  TreeParams tp;
  std::memset(&tp, 0, sizeof tp);
  tp.docs_wanted = dw;
  int64_t rmax = std::max<int64_t>(50, (int64_t)dw * 2);
  tp.ridiculous = rmax;
  tp.num_nodes = tree_nodes(dw, true);
  tp.cap = std::max(2, dw / 50);
  tp.partial = (float)(dw % 50) / 50.0;
  tp.init = (phase & TREE_INIT) ? 1 : 0;
  tp.final = (phase & TREE_FINAL) ? 1 : 0;
  tp.emit = (phase & TREE_EMIT) ? 1 : 0;
  tp.ints = ints ? 1 : 0;
  return tp;
}

// k_tree_seq's register columns (64 nodes each) for docsWanted: room for
// the nodes above docsWanted that capped domains keep in ordinary lists; 0:
// the one-wave replay (LDS tree)
static int seq_columns(int32_t dw) {
  return dw <= 200 ? 4 : dw <= 420 ? 8 : dw <= 880 ? 16 : 0;
}

// result block of a clustering query: up to TC nodes
static int ensure_result(QuerySlot &q) {
  q.res_bytes = res_size(q.k);
  if (q.res.ensure(q.res_bytes)) return ENOMEM;
  if (q.res_bytes > q.hres_cap) {
    if (q.h_res) (void)hipHostFree(q.h_res);
    q.h_res = nullptr;
    q.hres_cap = 0;
    HIPCHECK(hipHostMalloc((void **)&q.h_res, q.res_bytes));
    q.hres_cap = q.res_bytes;
  }
  return 0;
}

// The last piece of a docid-split clustering query scored nothing: the tree
// the earlier pieces left is the result (no survivors to replay).
static int enqueue_tree_emit(QuerySlot &q, int32_t dw) {
  q.k = TC;
  q.docs_wanted = dw;
  q.early = false;
  q.scan_bytes = 0;
  q.slot_ub = 0;
  int rc = ensure_result(q);
  if (rc) return rc;
  hipStream_t st = q.stream;
  Counters *dctr = q.res.as<Counters>();
  hipLaunchKernelGGL(k_reset, dim3(1), dim3(BLOCK), 0, st, reinterpret_cast<uint32_t *>(dctr),
                     (uint32_t)(sizeof(Counters) / 4), reinterpret_cast<uint32_t *>(dctr), 0u);
  hipLaunchKernelGGL(k_tree_replay, dim3(1), dim3(64), 0, st, dctr, (const uint4 *)nullptr, q.tree.as<TreeState>(),
                     tree_params(dw, TREE_FINAL, q.int_scores),
                     q.res.as<uint32_t>(res_keys_off()), q.res.as<uint64_t>(res_docs_off(q.k)));
  HIPCHECK(hipGetLastError());
  HIPCHECK(hipEventRecord(q.ev_done, st));
  HIPCHECK(hipMemcpyAsync(q.h_res, q.res.p, q.res_bytes, hipMemcpyDeviceToHost, st));
  q.pending = true;
  return 0;
}

// The whitelist table of allocWhiteListTable / Posdb.cpp:5544-5572: the 5
// bytes at rec+7 of every record of every whitelist list, records walked with
// RdbList::skipCurrentRecord's posdb sizes (18 first, then 6 / 12 / 18 by the
// compression bits) -- for a 6-byte record rec+7 lies in the next record, as
// in the reference; past the list's end (the reference reads its allocation
// slack, undefined) bytes read as 0.  Membership is exact (HashTableX
// compares the 5 bytes), so a sorted unique array serves.
static int white_set(const gbgpu_params *p, std::vector<uint64_t> &out) {
  out.clear();
  if (p->n_white_lists < 0 || (p->n_white_lists > 0 && !p->white_lists)) return EINVAL;
  for (int i = 0; i < p->n_white_lists; i++) {
    const gbgpu_list &l = p->white_lists[i];
    if (l.size < 0 || (l.size > 0 && !l.bytes)) return EINVAL;
    const uint8_t *b = l.bytes, *end = b + l.size;
    for (const uint8_t *r = b; r < end;) {
      uint64_t x = 0;
      for (int k = 4; k >= 0; k--) x = (x << 8) | (r + 7 + k < end ? r[7 + k] : 0);
      out.push_back(x);
      r += r == b ? 18 : ((r[0] & 0x04) ? 6 : ((r[0] & 0x02) ? 12 : 18));
    }
  }
  std::sort(out.begin(), out.end());
  out.erase(std::unique(out.begin(), out.end()), out.end());
  return 0;
}

static int enqueue_entries(gbgpu_ctx *ctx, QuerySlot &q, const gbgpu_qterm *terms, int nterms,
                           const ListEntry *ents, const gbgpu_params *p, int32_t dw_override, int tree_phase) {
  std::vector<int64_t> sizes(nterms);
  for (int i = 0; i < nterms; i++) sizes[i] = ents[i].size;
  HostPlan hp;
  int rc = build_host_plan(terms, nterms, sizes.data(), p, &hp);
  if (rc) return rc;
  if (dw_override > 0) hp.docs_wanted = dw_override;
  const bool clus = p->site_clustering != 0;
  const bool boolean = p->is_boolean != 0;
  if (boolean) {
    // the truth table is over the plan's QueryTermInfos (m_bitNum = the
    // group index, Posdb.cpp:4485-4721)
    if (!p->bool_table || p->bool_ngroups != hp.ngroups) return EINVAL;
    if (hp.ngroups > 16) return GBGPU_EUNSUPPORTED;
    // a boolean query's gbsortby score reads a mini-merged list that may be
    // another group's or stale (Posdb.cpp:7263-7279); its range terms vote by
    // isInRange over the whole run (8087-8129), not restated on the device;
    if (hp.sortby_group >= 0) return GBGPU_EUNSUPPORTED;
    for (int i = 0; i < nterms; i++) {
      int ri = 0;
      if (terms[i].is_required && range_mode(terms[i].field_code, &ri)) return GBGPU_EUNSUPPORTED;
    }
  }
  q.facets.clear();
  q.stale_done = false;
  q.stale_filt = 0;
  q.docs_wanted = hp.docs_wanted;
  q.k = clus ? TC : hp.docs_wanted;
  // Posdb.cpp:5735: a boolean query goes on with an empty smallest group
  // (allocTopTree gave it no tree only when every list is empty)
  q.early = hp.ngroups == 0 || (boolean ? hp.docs_wanted == 0 : hp.min_list_size == 0);
  q.scan_bytes = 0;
  q.replayed = false;
  q.want_info = p->get_docid_scoring_info != 0;
  q.int_scores = false;
  q.info_docs = p->docs_to_get;
  q.info_nterms = nterms;
  q.info_rmt = hp.real_max_top;
  q.info_ng = hp.ngroups;
  q.info_scap = hp.ngroups * hp.real_max_top;
  q.info_pcap = hp.ngroups * (hp.ngroups - 1) / 2 * hp.real_max_top;
  if (q.want_info) {
    // allocTopTree's reservations (Posdb.cpp:931-975): a call whose records
    // would not fit is dropped there ("CRITICAL ... overflow"); not emulated,
    // so refuse any request whose worst case could reach it
    const int64_t xx = std::max<int64_t>(hp.docs_wanted, 32);
    const int64_t nt = std::min(nterms, 10);
    const int64_t pcap_ref = nt * nt / 2 * hp.real_max_top * xx;
    const int64_t scap_ref = nt * hp.real_max_top * xx;
    if ((int64_t)p->docs_to_get * q.info_pcap > pcap_ref || (int64_t)p->docs_to_get * q.info_scap > scap_ref)
      return GBGPU_EUNSUPPORTED;
  }
  if (q.early) {
    q.pending = true;
    return 0;
  }
  if (hp.ngroups > MAXG) return GBGPU_EUNSUPPORTED;
  if (!clus && q.k > MAX_K_BIG) return GBGPU_EUNSUPPORTED;

  // ---- query tables, built straight into the pinned staging buffer
  // layout: [DevPlan | G0Chunk[] | afirst[MAXG0] | ProbeWork[]]
  DevPlan P;
  std::memset(&P, 0, sizeof P);
  P.ngroups = hp.ngroups;
  P.real_max_top = hp.real_max_top;
  P.language = p->language;
  P.same_lang_weight = p->same_lang_weight;
  P.site_rank_multiplier = boolean ? 0.0f : (float)GB_SITERANKMULTIPLIER;  // Posdb.cpp:774
  P.boolean = boolean ? 1 : 0;
  P.nqt = nterms;
  P.has_serp = p->min_serp_docid != 0;  // Posdb.cpp:4379-4381
  P.max_serp_score = p->max_serp_score;
  P.min_serp_docid = p->min_serp_docid;
  // (int32_t)m_maxSerpScore as the reference's x86-64 build computes it
  // (cvttsd2si): truncation, or INT32_MIN when out of range or NaN
  P.max_serp_int = (p->max_serp_score > -2147483649.0 && p->max_serp_score < 2147483648.0)
                       ? (int32_t)p->max_serp_score
                       : INT32_MIN;
  P.clustering = clus;
  P.use_white = p->use_whitelist != 0 && !boolean;  // the boolean vote never reads the whitelist
  if (P.use_white) {
    rc = white_set(p, q.h_white);
    if (rc) return rc;
    P.nwhite = (uint32_t)q.h_white.size();
  }
  P.do_max_score = p->do_max_score_algo != 0;
  P.sortby_group = hp.sortby_group;
  P.sortby_int = hp.sortby_int;
  q.int_scores = hp.sortby_int != 0;
  P.min_listi = hp.min_listi;
#ifdef GBGPU_DIAG
  if (const char *dd = ctx->probe_dbg_doc) {
    P.dbg_doc = std::strtoull(dd, nullptr, 10);
    if (ctx->d_pdbg) HIPCHECK(hipMemsetAsync(ctx->d_pdbg, 0, 8 * (1 + 16 * 32), q.stream));
    P.dbg_buf = ctx->d_pdbg;
  }
#endif
  P.all_same_wiki = 1;  // m_allInSameWikiPhrase, Posdb.cpp:5764-5778
  for (int j = 0; j < hp.ngroups; j++) {
    if (hp.g[j].flags[0] & (BF_NEGATIVE | BF_NUMBER | BF_FACET)) continue;
    if (hp.g[j].wiki == 1) continue;
    P.all_same_wiki = 0;
    break;
  }
  int dense[1024];
  uint64_t list_dmin[MAXL], list_dmax[MAXL];
  const ListEntry *lent[MAXL] = {};
  for (int i = 0; i < nterms; i++) dense[i] = -1;
  auto dense_id = [&](int term) -> int {
    if (dense[term] >= 0) return dense[term];
    if (P.nlists >= MAXL) return -1;
    int id = P.nlists++;
    dense[term] = id;
    const ListEntry &e = ents[term];
    lent[id] = &e;
    P.lists[id].p = e.d;
    P.lists[id].pm = e.pm;
    P.lists[id].units = e.units;
    list_dmin[id] = e.dmin;
    list_dmax[id] = e.dmax;
    P.lists[id].group_bits = 0;
    P.lists[id].g0_array = -1;
    P.lists[id].probe = 0;
    P.lists[id].owner_group = -1;
    P.lists[id].owner_sub = -1;
    P.lists[id].uses = 0;
    P.lists[id].rmode = 0;
    return id;
  };
  for (int j = 0; j < hp.ngroups; j++) {
    const GroupInfo &g = hp.g[j];
    if (g.nsub > MAXSUB) return GBGPU_EUNSUPPORTED;
    P.gflags0[j] = g.flags[0];
    P.gnsub[j] = (uint8_t)g.nsub;
    P.tfw[j] = g.tfw;
    P.qpos[j] = g.qpos;
    P.wiki[j] = g.wiki;
    P.quote[j] = g.quote;
    P.qterm[j] = g.qterm;
    int rint = 0;
    const int rmode = range_mode(terms[g.qterm].field_code, &rint);
    if (rmode) {
      // a range term's group: its own list only (no synonyms / bigrams), voted
      // by the keys' numbers (Posdb.cpp:5056-5073, 5115-5121, 5242-5298)
      if (g.nsub != 1 || g.sub_term[0] != g.qterm || (g.flags[0] & BF_NEGATIVE)) return GBGPU_EUNSUPPORTED;
    }
    for (int x = 0; x < MAXSUB; x++) P.gsubflags[j][x] = x < 50 ? g.flags[x] : 0;
    const bool neg = (g.flags[0] & BF_NEGATIVE) != 0;
    if (!neg) P.pos_mask |= 1u << j;
    for (int x = 0; x < g.nsub; x++) {
      int id = dense_id(g.sub_term[x]);
      if (id < 0) return GBGPU_EUNSUPPORTED;
      P.gsub[j][x] = (uint8_t)id;
      P.bool_gmask[id] |= (uint16_t)(1u << j);
      if (rmode) {
        if (P.lists[id].uses) return GBGPU_EUNSUPPORTED;  // shared with another group
        P.lists[id].rmode = rmode;
        P.lists[id].rint = rint;
        P.lists[id].rf = terms[g.qterm].number_float;
        P.lists[id].ri = terms[g.qterm].number_int;
      }
      P.lists[id].group_bits |= neg ? NEG_BIT : (1u << j);
      if (neg) P.neg_lists |= 1u << id;
      else P.group_lists[j] |= 1u << id;
      if (!neg) {
        // shrinkSubLists' in-place order: groups in index order, sublists in
        // order (Posdb.cpp:5906-5914); the first use sees the list clean
        if (P.lists[id].uses++ == 0) {
          P.lists[id].owner_group = (int16_t)j;
          P.lists[id].owner_sub = (int16_t)x;
        } else {
          P.reshare_mask |= 1u << id;
        }
      }
    }
  }
  // facet terms with a non-empty list get a table (allocTopTree, Posdb.cpp:
  // 1000-1067); collect() fills it.  Restated without site clustering, a
  // boolean expression or docid splits, for a facet term whose group is its
  // own list alone, used by no other group
  for (int i = 0; i < nterms; i++) {
    const int32_t fc = terms[i].field_code;
    if (fc < FIELD_GBFACETSTR || fc > FIELD_GBFACETFLOAT || ents[i].size == 0) continue;
    if (q.facets.size() >= (size_t)MAXF) return GBGPU_EUNSUPPORTED;
    FacetTerm ft;
    ft.term = i;
    ft.lid = -1;
    ft.isfloat = fc == FIELD_GBFACETFLOAT;
    ft.units = ents[i].units;
    ft.list = ents[i].d;
    for (int j = 0; j < hp.ngroups; j++) {
      if (hp.g[j].qterm != i) continue;
      const GroupInfo &g = hp.g[j];
      const int id = dense[i];
      if (g.nsub != 1 || g.sub_term[0] != i || (g.flags[0] & BF_NEGATIVE) || id < 0 || P.lists[id].uses != 1 ||
          (P.reshare_mask >> id & 1))
        return GBGPU_EUNSUPPORTED;
      ft.lid = id;
    }
    if (p->n_facet_ranges < 0 || (p->n_facet_ranges > 0 && !p->facet_ranges)) return EINVAL;
    for (int r = 0; r < p->n_facet_ranges; r++) {
      const gbgpu_facet_ranges &fr = p->facet_ranges[r];
      if (fr.term != i) continue;
      if (fr.n < 0 || fr.n > MAX_FACET_RANGES || (fr.n > 0 && (!fr.a || !fr.b))) return EINVAL;
      ft.a.assign(fr.a, fr.a + fr.n);
      ft.b.assign(fr.b, fr.b + fr.n);
      break;
    }
    q.facets.push_back(std::move(ft));
  }
  // m_hasFacetTerm: a facet term with a list, or any over docid splits
  // (Posdb.cpp:1013-1023)
  P.has_facet = 0;
  for (int i = 0; i < nterms; i++)
    if (terms[i].field_code >= FIELD_GBFACETSTR && terms[i].field_code <= FIELD_GBFACETFLOAT &&
        (ents[i].size > 0 || p->num_docid_splits > 1))
      P.has_facet = 1;
  // candidate arrays: distinct lists of the smallest group, in sublist order;
  // for a boolean query every distinct list (the docid set is their union:
  // a docid's slot is in the first array holding it, its other arrays'
  // slots get no list bit and die)
  P.g0n = 0;
  uint64_t slot = 0;
  auto add_array = [&](int id) -> int {
    if (P.lists[id].g0_array >= 0) return 0;
    if (P.g0n >= MAXG0) return GBGPU_EUNSUPPORTED;
    P.lists[id].g0_array = P.g0n;
    P.g0list[P.g0n] = id;
    P.g0base[P.g0n] = slot;
    slot += P.lists[id].units / 2 + 1;
    P.g0n++;
    return 0;
  };
  if (boolean) {
    P.reshare_mask = 0;  // no mini merge: no re-shrunk copies
    for (int id = 0; id < P.nlists; id++)
      if ((rc = add_array(id))) return rc;
  } else {
    const GroupInfo &g0 = hp.g[hp.min_listi];
    for (int x = 0; x < g0.nsub; x++)
      if ((rc = add_array(dense[g0.sub_term[x]]))) return rc;
  }
  P.g0base[P.g0n] = slot;
  const uint64_t slot_ub = slot;
  // slots k_write_runs may reject: the whitelist, or a range term in the
  // smallest group (its first-group vote test)
  P.use_rej = P.use_white;
  for (int a = 0; a < P.g0n; a++)
    if (P.lists[P.g0list[a]].rmode) P.use_rej = 1;
  if (slot_ub >= (1ull << 28)) return GBGPU_ECAPACITY;  // 28-bit slot indices (survivor records, replay entries)
  q.slot_ub = slot_ub;
  // directories: about 8 units (2-4 docids) per bucket, power-of-two count
  uint64_t dir_entries = 0;
  for (int a = 0; a < P.g0n; a++) {
    const int id = P.g0list[a];
    const uint32_t units = P.lists[id].units;
    uint64_t nb = 64;
    while (nb < units / 8) nb <<= 1;
    const uint64_t lo = list_dmin[id], hi = list_dmax[id];
    uint32_t sh = 0;
    while (((hi - lo) >> sh) >= nb) sh++;
    P.g0dmin[a] = lo;
    P.g0dmax[a] = hi;
    P.g0sh[a] = sh;
    P.g0dir[a] = dir_entries;
    dir_entries += ((hi - lo) >> sh) + 1;
  }
  // probe direction per list: candidate-driven while a 3 KiB chunk meets at
  // most probe_dir_t candidates (several 64-lane windows a chunk still beat
  // a directory lookup per run), else run-driven
  for (int id = 0; id < P.nlists; id++)
    P.list_mult[id] = (uint8_t)__builtin_popcount(P.lists[id].group_bits & P.pos_mask & ~NEG_BIT);
  P.probed_mask = 0;
  for (int id = 0; id < P.nlists; id++) {
    P.lists[id].probe = 0;
    if (P.lists[id].g0_array == 0) continue;
    const double per_chunk = (double)slot_ub * WCH_UNITS / std::max<uint32_t>(1, P.lists[id].units);
    P.lists[id].probe = per_chunk > ctx->probe_dir_t ? PROBE_BY_RUN : PROBE_BY_CAND;
    P.probed_mask |= 1u << id;
  }

  q.g0c.clear();
  q.afirst.assign(MAXG0, 0);
  for (int a = 0; a < P.g0n; a++) {
    q.afirst[a] = (uint32_t)q.g0c.size();
    const uint32_t units = P.lists[P.g0list[a]].units;
    for (uint32_t u = 0; u < units; u += CHUNK_UNITS) q.g0c.push_back({(uint32_t)a, u});
  }
  if (q.g0c.empty()) {
    // no candidate at all: a boolean query (or docid-split piece) whose every
    // list is empty votes nothing
    q.early = true;
    q.pending = true;
    return 0;
  }
  q.pw.clear();
  int64_t scan = 0;
  uint64_t probe_chunks = 0;
  // candidate-driven lists walk 6 KiB chunks when the smallest group has at
  // most two candidate arrays (probe_by_cand_wide), else 3 KiB
#ifdef GBGPU_DIAG
  const bool wide = P.g0n <= 2 && ctx->probe_mode == 11;
  const uint32_t cunits = wide ? (uint32_t)W6_UNITS : (uint32_t)WCH_UNITS;
#else
  constexpr bool wide = false;
  const uint32_t cunits = (uint32_t)WCH_UNITS;
#endif
  for (int id = 0; id < P.nlists; id++) {
    scan += (int64_t)P.lists[id].units * 6;
    if (P.lists[id].probe == PROBE_BY_CAND) probe_chunks += (P.lists[id].units + cunits - 1) / cunits;
  }
  // one wave per span of S chunks: about PROBE_WAVES spans over all probed
  // lists, so every CU holds ~24 waves and each amortises its initial
  // candidate search over several chunks
  const uint64_t pwaves = ctx->probe_waves ? (uint64_t)ctx->probe_waves : wide ? PROBE_WAVES_WIDE : PROBE_WAVES;
  const uint32_t S = (uint32_t)std::max<uint64_t>(1, (probe_chunks + pwaves - 1) / pwaves);
  // a run-driven chunk costs a few dependent lookups: one chunk per wave,
  // its work computed by the wave itself (DevPlan::rseg_*)
  const uint32_t rspan = ctx->probe_runspan > 0 ? (uint32_t)ctx->probe_runspan : 1u;
  P.run_span = WCH_UNITS * rspan;
  P.nrseg = 0;
  uint64_t rwaves = 0;
  for (int id = 0; id < P.nlists; id++) {
    if (P.lists[id].probe != PROBE_BY_RUN || !P.lists[id].units) continue;
    P.rseg_list[P.nrseg] = (uint32_t)id;
    P.rseg_wbase[P.nrseg++] = (uint32_t)rwaves;
    rwaves += (P.lists[id].units + P.run_span - 1) / P.run_span;
  }
  P.rseg_wbase[P.nrseg] = (uint32_t)rwaves;
  for (int id = 0; id < P.nlists; id++) {
    if (P.lists[id].probe != PROBE_BY_CAND) continue;
    const uint32_t units = P.lists[id].units;
    const uint32_t span = cunits * S;
    const std::vector<uint64_t> *gf = lent[id]->gfirst.get();
    for (uint32_t u = 0; u < units; u += span) {
      ProbeWork pw{(uint32_t)id, u, std::min(units, u + span), 0u, ~0ull};
      if (gf && u / WCH_UNITS < gf->size()) {
        pw.has_dfirst = 1;
        pw.dfirst = (*gf)[u / WCH_UNITS];
      }
      q.pw.push_back(pw);
    }
  }
  P.nwork_cand = (uint32_t)q.pw.size();
  q.nwork = P.nwork_cand + (uint32_t)rwaves;
  q.scan_bytes = scan;
  q.g0_bytes = 0;
  q.probe_bytes = 0;
  for (int id = 0; id < P.nlists; id++) {
    if (P.lists[id].g0_array >= 0) q.g0_bytes += (int64_t)P.lists[id].units * 6;
    if (P.lists[id].probe) q.probe_bytes += (int64_t)P.lists[id].units * 6;
  }
  // scratch upper bound: every group instance can use all of its list once
  uint64_t scratch_ub = 1;
  for (int j = 0; j < hp.ngroups; j++) {
    if (P.gflags0[j] & BF_NEGATIVE) continue;
    for (int x = 0; x < P.gnsub[j]; x++) scratch_ub += P.lists[P.gsub[j][x]].units;
  }
  // re-shrunk lists: one survivor per list has its records relocated to the
  // arena's end with room for the extra units (k_ext_walk checks the fit)
  if (P.reshare_mask) scratch_ub += scratch_ub / 2 + 4096;
  if (scratch_ub >= (1ull << 36)) return GBGPU_ECAPACITY;
  const int k = q.k;
  const size_t o_chunks = align256(sizeof(DevPlan));
  const size_t o_afirst = o_chunks + align256(sizeof(G0Chunk) * q.g0c.size());
  const size_t o_work = o_afirst + align256(4 * MAXG0);
  const size_t o_btab = o_work + align256(sizeof(ProbeWork) * q.pw.size());
  const size_t btab_bytes = boolean ? ((size_t)1 << hp.ngroups) / 8 + 8 : 0;
  const size_t tbytes = o_btab + align256(btab_bytes);
  q.res_bytes = res_size(k);
  int rc2 = 0;
  rc2 |= q.tables.ensure(tbytes);
  const uint32_t nwords = (uint32_t)((slot_ub + 31) / 32);
  const uint32_t cgrid = std::max(1u, (uint32_t)((nwords + CWORDS - 1) / CWORDS));
  rc2 |= q.cand.ensure(8 * slot_ub);
  rc2 |= q.cunit.ensure(4 * slot_ub);
  rc2 |= q.bits.ensure(4 * (size_t)nwords * (uint64_t)P.nlists);
  rc2 |= q.loc.ensure(sizeof(Loc) * slot_ub * (uint64_t)P.nlists);
  // k_score variant: group / sublist capacity and LDS records per lane
  int maxsub = 0;
  for (int j = 0; j < hp.ngroups; j++)
    if (!(P.gflags0[j] & BF_NEGATIVE)) maxsub = std::max(maxsub, (int)P.gnsub[j]);
  const int variant = (boolean || (hp.ngroups <= 2 && maxsub <= 2)) ? 4  // boolean: no records scored
                      : (hp.ngroups <= 2 && maxsub <= 4) ? 0
                      : (hp.ngroups <= 4 && maxsub <= 4) ? 1
                      : (hp.ngroups <= 8 && maxsub <= 4) ? 2
                                                         : 3;
  static constexpr uint32_t kRC[5] = {24, 48, 64, 64, GBGPU_SCORE_RC2};  // LDS records per lane
  const uint32_t rcap = kRC[variant] / 2;  // size buckets: a column holds 2x a bucket-3 survivor's units
  rc2 |= q.svslot.ensure(4 * slot_ub);
  rc2 |= q.svlm.ensure(4 * slot_ub);
  rc2 |= q.svu.ensure(4 * slot_ub);
  rc2 |= q.svdoc.ensure(8 * slot_ub);
  rc2 |= q.svloc.ensure(sizeof(Loc) * slot_ub * (uint64_t)P.nlists);
  rc2 |= q.scratch.ensure(8 * scratch_ub);
  rc2 |= q.skey.ensure(4 * slot_ub);
  rc2 |= q.blk.ensure(align256(sizeof(BlkInfo) * (size_t)cgrid) + 4 * NBKT * (size_t)cgrid);
  rc2 |= q.sel.ensure(sizeof(Select));
  rc2 |= q.gath.ensure(12 * (slot_ub + MAX_K_BIG) + 1024);
  rc2 |= q.stg.ensure(12 * slot_ub + 256);
  rc2 |= q.res.ensure(q.res_bytes);
  if (clus) {
    rc2 |= q.sflag.ensure(slot_ub);
    rc2 |= q.ord.ensure(4 * slot_ub);
    rc2 |= q.oslot.ensure(4 * slot_ub);
    rc2 |= q.rep.ensure((P.g0n > 1 ? 32 : 16) * slot_ub);
    if (!(tree_phase & TREE_FINAL)) rc2 |= q.tree.ensure(sizeof(TreeState));
    // a later docid-split piece keeps the tree it starts from: a stale-mbuf
    // fix replays the piece again from it (stale_fix_clustered)
    if (!(tree_phase & TREE_INIT)) rc2 |= q.tree_bak.ensure(sizeof(TreeState));
    if (!q.facets.empty()) rc2 |= q.mwsl.ensure(16 * (slot_ub + 2));
  }
  if (P.use_white) rc2 |= q.white.ensure(8 * std::max<size_t>(1, q.h_white.size()));
  if (P.use_rej) rc2 |= q.wrej.ensure(align256(slot_ub));  // k_cmp_* read it 32 slots at a time
  const void *dir_before = q.dir.p;
  rc2 |= q.dir.ensure(8 * std::max<uint64_t>(1, dir_entries));
  if (rc2) return ENOMEM;
  if (P.use_rej) P.wrej = q.wrej.as<uint8_t>();
  if (P.use_white) {
    P.white = q.white.as<uint64_t>();
    if (!q.h_white.empty())
      HIPCHECK(hipMemcpyAsync(q.white.p, q.h_white.data(), 8 * q.h_white.size(), hipMemcpyHostToDevice, q.stream));
  }
  if (q.dir.p != dir_before || q.epoch == 0xffffffffu) {
    // fresh directory memory: no entry may carry a live epoch
    HIPCHECK(hipMemsetAsync(q.dir.p, 0, q.dir.cap, q.stream));
    q.epoch = 0;
  }
  P.epoch = ++q.epoch;
  if (boolean) P.bool_table = q.tables.as<uint8_t>(o_btab);
  if (tbytes > q.stage_cap) {
    if (q.h_stage) (void)hipHostFree(q.h_stage);
    q.h_stage = nullptr;
    q.stage_cap = 0;
    HIPCHECK(hipHostMalloc((void **)&q.h_stage, tbytes * 2));
    q.stage_cap = tbytes * 2;
  }
  if (q.res_bytes > q.hres_cap) {
    if (q.h_res) (void)hipHostFree(q.h_res);
    q.h_res = nullptr;
    q.hres_cap = 0;
    HIPCHECK(hipHostMalloc((void **)&q.h_res, q.res_bytes));
    q.hres_cap = q.res_bytes;
  }
  // the staging buffer may still feed the previous query's copy: the stream
  // has been synchronised by collect() (one query in flight per context)
  std::memcpy(q.h_stage, &P, sizeof P);
  std::memcpy(q.h_stage + o_chunks, q.g0c.data(), sizeof(G0Chunk) * q.g0c.size());
  std::memcpy(q.h_stage + o_afirst, q.afirst.data(), 4 * MAXG0);
  std::memcpy(q.h_stage + o_work, q.pw.data(), sizeof(ProbeWork) * q.pw.size());
  if (boolean) {
    std::memset(q.h_stage + o_btab, 0, btab_bytes);
    std::memcpy(q.h_stage + o_btab, p->bool_table, ((size_t)1 << hp.ngroups) / 8 ? ((size_t)1 << hp.ngroups) / 8 : 1);
  }

  hipStream_t st = q.stream;
  if (ctx->profiling) HIPCHECK(hipEventRecord(q.ev[0], st));
  HIPCHECK(hipMemcpyAsync(q.tables.p, q.h_stage, tbytes, hipMemcpyHostToDevice, st));
  const DevPlan *dpl = q.tables.as<DevPlan>();
  const G0Chunk *dchunks = q.tables.as<G0Chunk>(o_chunks);
  const ProbeWork *dwork = q.tables.as<ProbeWork>(o_work);
  Counters *dctr = q.res.as<Counters>();
  Select *dsel = q.sel.as<Select>();
  uint32_t *bits = q.bits.as<uint32_t>();
  Loc *loc = q.loc.as<Loc>();
  {
    const uint32_t nb = nwords * (uint32_t)P.nlists;  // the probe bitmaps
    const uint32_t rg = std::max(16u, std::min(1024u, nb / 2048));
    hipLaunchKernelGGL(k_reset, dim3(rg), dim3(BLOCK), 0, st, reinterpret_cast<uint32_t *>(dctr),
                       (uint32_t)(sizeof(Counters) / 4), reinterpret_cast<uint32_t *>(dsel),
                       (uint32_t)(sizeof(Select) / 4), bits, nb);
  }
  const uint32_t ng0 = (uint32_t)q.g0c.size();
  hipLaunchKernelGGL(k_write_runs, dim3(ng0), dim3(BLOCK), 0, st, dpl, dchunks, q.cand.as<uint64_t>(),
                     q.cunit.as<uint32_t>(), dctr, ng0, q.dir.as<uint64_t>());
  if (ctx->profiling) HIPCHECK(hipEventRecord(q.ev[1], st));
  if (q.nwork) {
#ifdef GBGPU_DIAG
    auto kp = ctx->probe_mode == 11  ? (P.g0n <= 1 ? k_probe<11, 1> : k_probe<11, 2>)  // diagnostic: 6 KiB chunks
              : ctx->probe_mode == 10 ? (P.g0n <= 2 ? k_probe<10, 2> : k_probe<10, 4>)  // diagnostic: bucket tables
              : ctx->probe_mode == 4 ? k_probe<12, MAXG0>  // diagnostic: the unpacked run list
              : ctx->probe_mode == 9 ? k_probe<2, 2>
              : ctx->probe_mode == 8 ? k_probe<1, 2>
              : ctx->probe_mode == 5 ? k_probe<5, 2>
              : ctx->probe_mode == 3 ? k_probe<3, MAXG0>
              : ctx->probe_mode == 2 ? k_probe<2, MAXG0>
              : ctx->probe_mode == 1 ? k_probe<1, MAXG0>
              : P.g0n == 1           ? k_probe<0, 1>
              : P.g0n == 2           ? k_probe<0, 2>
              : P.g0n <= 4           ? k_probe<0, 4>
                                     : k_probe<0, MAXG0>;
#else
    auto kp = P.g0n == 1 ? k_probe<0, 1> : P.g0n == 2 ? k_probe<0, 2> : P.g0n <= 4 ? k_probe<0, 4> : k_probe<0, MAXG0>;
#endif
    const uint32_t nwork = q.nwork;
    hipLaunchKernelGGL(kp, dim3((nwork + PW - 1) / PW), dim3(64 * PW), 0, st, dpl, dwork, nwork,
                       q.cand.as<uint64_t>(), bits, nwords, loc, dctr, q.dir.as<uint64_t>());
  }
  {
    uint32_t rbits = 0;  // range terms' lists outside the smallest group
    for (int l = 0; l < P.nlists; l++)
      if (P.lists[l].rmode && P.lists[l].g0_array < 0) rbits |= 1u << l;
    if (rbits) {
      const uint32_t g = std::max(1u, std::min(4096u, (nwords + 255) / 256));
      hipLaunchKernelGGL(k_range_filter, dim3(g), dim3(256), 0, st, dpl, rbits, bits, nwords, loc);
    }
  }
  if (ctx->profiling) HIPCHECK(hipEventRecord(q.ev[2], st));
  const uint64_t *dcand = q.cand.as<uint64_t>();
  const uint32_t *dcunit = q.cunit.as<uint32_t>();
  BlkInfo *blk = q.blk.as<BlkInfo>();
  uint32_t *svslot = q.svslot.as<uint32_t>(), *svlm = q.svlm.as<uint32_t>(), *svu = q.svu.as<uint32_t>();
  uint64_t *svdoc = q.svdoc.as<uint64_t>();
  Loc *svloc = q.svloc.as<Loc>();
  // site clustering also records each survivor's slot-order rank (the
  // replay walks the survivors in docid order)
  uint32_t *cnt8 = reinterpret_cast<uint32_t *>(q.blk.as<uint8_t>(align256(sizeof(BlkInfo) * (size_t)cgrid)));
  // the staged survivors (slot, list mask, units): 12 bytes a slot
  uint32_t *stslot = q.stg.as<uint32_t>(), *stlm = stslot + slot_ub, *stu = stlm + slot_ub;
  hipLaunchKernelGGL(k_cmp_count, dim3(cgrid), dim3(CB), 0, st, dpl, dctr, dcunit, bits, nwords, loc, dcand, rcap, blk,
                     cnt8, stslot, stlm, stu);
  hipLaunchKernelGGL(k_cmp_place, dim3(cgrid), dim3(CB), 0, st, dpl, dctr, dcunit, loc, dcand, rcap, blk,
                     (const uint32_t *)cnt8, cgrid, stslot, stlm, stu, svslot, svlm, svu, svdoc, svloc,
                     clus ? q.ord.as<uint32_t>() : nullptr);
  const unsigned long long arena_cap = (unsigned long long)(q.scratch.cap / 8);
  if (P.reshare_mask)
    hipLaunchKernelGGL(k_ext_walk, dim3(1), dim3(64), 0, st, dpl, dctr, dcand, dcunit, bits, nwords, loc, arena_cap);
  if (ctx->profiling) HIPCHECK(hipEventRecord(q.ev[3], st));
  {
    const uint32_t grid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((slot_ub + SCORE_TPB - 1) / SCORE_TPB, 8192));
    if (ctx->d_sdbg) {
      ctx->sdbg_grid = grid;
      HIPCHECK(hipMemsetAsync(ctx->d_sdbg, 0, 8192 * 64, st));
    }
    auto launch = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3(grid), dim3(SCORE_TPB), 0, st, dpl, (const uint64_t *)svdoc, dctr,
                         (const uint32_t *)svslot, (const uint32_t *)svlm, (const uint32_t *)svu, (const Loc *)svloc,
                         q.scratch.as<uint64_t>(), arena_cap, q.skey.as<uint32_t>(), q.sflag.as<uint8_t>(),
                         ctx->score_mode, ctx->d_sdbg, clus ? nullptr : dsel->hist);
    };
    if (variant == 4) launch(k_score<2, 2, kRC[4]>);  // two groups of <= 2 sublists (config 2)
    else if (variant == 0) launch(k_score<2, 4, kRC[0]>);
    else if (variant == 1) launch(k_score<4, 4, kRC[1]>);
    else if (variant == 2) launch(k_score<8, 4, kRC[2]>);
    else launch(k_score<MAXG, MAXSUB, kRC[3]>);
  }
  if (ctx->profiling) HIPCHECK(hipEventRecord(q.ev[4], st));
  if (clus) {
    // site clustering: prefilter bounds, docid order, the TopTree replay
    const uint32_t bgrid =
        (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((slot_ub + 64 * BND_WAVES - 1) / (64 * BND_WAVES), 4096));
    // the replay entries in slot order (k_bound): docid order with one
    // candidate array, else merged by k_rank from the second half of rep
    const bool ranked = P.g0n > 1;
    uint4 *rep_slot = q.rep.as<uint4>() + (ranked ? slot_ub : 0);
    hipLaunchKernelGGL(k_bound, dim3(bgrid), dim3(64 * BND_WAVES), 0, st, dpl, dctr, (const uint32_t *)svslot,
                       (const uint32_t *)svlm, (const Loc *)svloc, (const uint32_t *)q.ord.as<uint32_t>(),
                       (const uint32_t *)q.skey.as<uint32_t>(), (const uint64_t *)svdoc, (const uint8_t *)q.sflag.as<uint8_t>(),
                       rep_slot, ranked ? q.oslot.as<uint32_t>() : nullptr);
    if (ranked) {
      const uint32_t rgrid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((slot_ub + 255) / 256, 4096));
      hipLaunchKernelGGL(k_rank, dim3(rgrid), dim3(256), 0, st, dpl, dctr, (const uint32_t *)q.oslot.as<uint32_t>(),
                         (const uint4 *)rep_slot, q.rep.as<uint4>());
    }
    // a whole-range pass: the block replay with the tree in registers
    // (columns for the nodes docsWanted and the domain caps normally keep);
    // a docid-split piece carries its tree in TreeState: the one-wave replay
    const int kcol = ctx->replay_mode == 3 ? 1 : seq_columns(q.docs_wanted);  // 3: diagnostic, 64 nodes (overflows)
    TreeParams tp = tree_params(q.docs_wanted, tree_phase, q.int_scores);
    if (!q.facets.empty()) tp.mwsl = q.mwsl.as<uint4>();
    q.rep_off = ranked ? slot_ub : 0;
    q.whole_range = tree_phase == (TREE_INIT | TREE_FINAL);
    q.tree_phase = tree_phase;
    if (!(tree_phase & TREE_INIT))
      HIPCHECK(hipMemcpyAsync(q.tree_bak.p, q.tree.p, sizeof(TreeState), hipMemcpyDeviceToDevice, st));
    q.seq_replay = q.whole_range && kcol > 0 && ctx->replay_mode != 1;
    if (q.seq_replay) {
      auto ks = q.int_scores ? (kcol == 1 ? k_tree_seq<1, true> : kcol == 4 ? k_tree_seq<4, true>
                                : kcol == 8 ? k_tree_seq<8, true> : k_tree_seq<16, true>)
                             : (kcol == 1 ? k_tree_seq<1, false> : kcol == 4 ? k_tree_seq<4, false>
                                : kcol == 8 ? k_tree_seq<8, false> : k_tree_seq<16, false>);
      hipLaunchKernelGGL(ks, dim3(1), dim3(64 * SQ_W), 0, st, dctr, (const uint4 *)q.rep.as<uint4>(), tp,
                         q.res.as<uint32_t>(res_keys_off()), q.res.as<uint64_t>(res_docs_off(k)));
      // a tree that outgrew the register columns replays the same entries
      // through the LDS tree right behind it, before ev_done: the result
      // block is final when the exchange (k_xpack) or collect reads it
      TreeParams tf = tp;
      tf.on_reg_err = 1;
      hipLaunchKernelGGL(k_tree_replay, dim3(1), dim3(64), 0, st, dctr, (const uint4 *)q.rep.as<uint4>(),
                         (TreeState *)nullptr, tf, q.res.as<uint32_t>(res_keys_off()),
                         q.res.as<uint64_t>(res_docs_off(k)));
    } else {
      hipLaunchKernelGGL(k_tree_replay, dim3(1), dim3(64), 0, st, dctr, (const uint4 *)q.rep.as<uint4>(),
                         (tree_phase & TREE_FINAL) ? (TreeState *)q.tree.p : q.tree.as<TreeState>(), tp,
                         q.res.as<uint32_t>(res_keys_off()), q.res.as<uint64_t>(res_docs_off(k)));
    }
    q.replayed = true;
    HIPCHECK(hipGetLastError());  // a launch refused above
    if (ctx->profiling) HIPCHECK(hipEventRecord(q.ev[5], st));
    HIPCHECK(hipEventRecord(q.ev_done, st));
    HIPCHECK(hipMemcpyAsync(q.h_res, q.res.p, q.res_bytes, hipMemcpyDeviceToHost, st));
    if (ctx->profiling) HIPCHECK(hipEventRecord(q.ev[6], st));
    q.pending = true;
    return 0;
  }
  // top-k: radix select over the survivors' keys, then one LDS sort
  const uint32_t *skey = q.skey.as<uint32_t>();
  uint32_t *akey = q.gath.as<uint32_t>();
  uint64_t *adoc = q.gath.as<uint64_t>(align256(4 * (size_t)MAX_K_BIG));
  uint32_t *bkey = q.gath.as<uint32_t>(align256(4 * (size_t)MAX_K_BIG) + align256(8 * (size_t)MAX_K_BIG));
  uint64_t *bdoc = q.gath.as<uint64_t>(align256(4 * (size_t)MAX_K_BIG) + align256(8 * (size_t)MAX_K_BIG) +
                                          align256(4 * slot_ub));
  const uint32_t tgrid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(TK_BLOCKS, (slot_ub + TK_THREADS - 1) / TK_THREADS));
  hipLaunchKernelGGL(k <= MAX_K ? k_topk<TILE> : k_topk<TILE_BIG>, dim3(tgrid), dim3(TK_THREADS), 0, st, skey,
                     (const uint64_t *)svdoc, dctr, dsel,
                     (uint32_t)k, akey, adoc, bkey, bdoc, q.res.as<uint32_t>(res_keys_off()),
                     q.res.as<uint64_t>(res_docs_off(k)));
  HIPCHECK(hipGetLastError());  // a launch refused above
  if (ctx->profiling) HIPCHECK(hipEventRecord(q.ev[5], st));
  HIPCHECK(hipEventRecord(q.ev_done, st));
  HIPCHECK(hipMemcpyAsync(q.h_res, q.res.p, q.res_bytes, hipMemcpyDeviceToHost, st));
  if (ctx->profiling) HIPCHECK(hipEventRecord(q.ev[6], st));
  q.pending = true;
  return 0;
}

// the sorted intersected docid set of the slot's last query (its vote buffer)
static int fetch_hits(QuerySlot &q, uint32_t nsurv, std::vector<int64_t> &out) {
  const size_t base = out.size();
  if (!nsurv) return 0;
  out.resize(base + nsurv);
  HIPCHECK(hipMemcpyAsync(out.data() + base, q.svdoc.p, 8 * (size_t)nsurv, hipMemcpyDeviceToHost, q.stream));
  HIPCHECK(hipStreamSynchronize(q.stream));
  std::sort(out.begin() + base, out.end());
  return 0;
}

static void write_hits(const std::vector<int64_t> &h, gbgpu_result *out) {
  out->n_hit_docids = 0;
  if (!out->hit_docids) return;
  const int64_t n = std::min<int64_t>((int64_t)h.size(), std::max<int64_t>(0, out->hit_capacity));
  if (n) std::memcpy(out->hit_docids, h.data(), 8 * (size_t)n);
  out->n_hit_docids = n;
}

static void slot_released(gbgpu_ctx *ctx) {
  { std::lock_guard<std::mutex> g(ctx->free_mu); }
  ctx->free_cv.notify_all();
}

// The second pass (see k_scoreinfo) for the first min(tree size, docs_to_get)
// docids of the collected tree, and the three buffers' host layout: one
// DocIdScore per docid in tree order, its PairScores / SingleScores appended
// in scoring order, m_pairsOffset / m_singlesOffset the byte offsets where
// its first record went (-1: none).  A docid the scorer rejects (minScore <=
// 0, never a tree member) would append records without a DocIdScore, as
// Posdb.cpp:7228-7230 jumps past the bookkeeping.
// padding bytes of the three records, zeroed after the copy (struct stores
// may leave them unspecified)
static void zero_gap(void *rec, size_t from, size_t to) {
  if (to > from) std::memset(static_cast<char *>(rec) + from, 0, to - from);
}
static void zero_pads(gbgpu_docid_score *d) {
  zero_gap(d, offsetof(gbgpu_docid_score, site_rank) + 1, offsetof(gbgpu_docid_score, doc_lang));
  zero_gap(d, offsetof(gbgpu_docid_score, singles_offset) + 4, offsetof(gbgpu_docid_score, pair_scores));
}
static void zero_pads(gbgpu_pair_score *p) {
  zero_gap(p, offsetof(gbgpu_pair_score, fixed_distance) + 1, offsetof(gbgpu_pair_score, word_pos1));
  zero_gap(p, offsetof(gbgpu_pair_score, word_pos2) + 4, offsetof(gbgpu_pair_score, term_freq1));
  zero_gap(p, offsetof(gbgpu_pair_score, bflags2) + 1, offsetof(gbgpu_pair_score, qdist));
}
static void zero_pads(gbgpu_single_score *s) {
  zero_gap(s, offsetof(gbgpu_single_score, hash_group) + 1, offsetof(gbgpu_single_score, word_pos));
  zero_gap(s, offsetof(gbgpu_single_score, bflags) + 1, sizeof(gbgpu_single_score));
}

// the score info records of several second passes, appended in order (the
// reference's buffers persist over docid-split pieces)
struct InfoAcc {
  int nd = 0, np = 0, ns = 0;
  bool room = true;
};
// Appends each scored docid's records straight to the caller's arrays (one
// second pass: no buffer limit is reached, enqueue checked the worst case).
struct OutSink {
  gbgpu_result *out;
  InfoAcc &acc;
  int ng;
  bool ints;
  int operator()(uint64_t docid, const SurvOut &inf, int cs, int cp, const gbgpu_single_score *ss,
                 const gbgpu_pair_score *ps) {
    gbgpu_docid_score d;
    std::memset(&d, 0, sizeof d);
    d.docid = (int64_t)docid;
    d.final_score = ints ? (double)inf.ival : (double)inf.score;  // Posdb.cpp:7557-7560
    d.site_rank = (int8_t)inf.site_rank;
    d.doc_lang = inf.doc_lang;
    d.num_required_terms = ng;
    d.num_pairs = cp;
    d.num_singles = cs;
    d.pairs_offset = cp ? acc.np * (int32_t)sizeof(gbgpu_pair_score) : -1;
    d.singles_offset = cs ? acc.ns * (int32_t)sizeof(gbgpu_single_score) : -1;
    if (acc.ns + cs > out->single_scores_cap || acc.np + cp > out->pair_scores_cap ||
        (inf.ok && acc.nd + 1 > out->docid_scores_cap))
      acc.room = false;
    if (acc.room) {
      if (cs) std::memcpy(out->single_scores + acc.ns, ss, sizeof(gbgpu_single_score) * cs);
      if (cp) std::memcpy(out->pair_scores + acc.np, ps, sizeof(gbgpu_pair_score) * cp);
      for (int k = 0; k < cs; k++) zero_pads(out->single_scores + acc.ns + k);
      for (int k = 0; k < cp; k++) zero_pads(out->pair_scores + acc.np + k);
      if (inf.ok) {
        std::memcpy(out->docid_scores + acc.nd, &d, sizeof d);
        zero_pads(out->docid_scores + acc.nd);
      }
    }
    acc.ns += cs;
    acc.np += cp;
    acc.nd += inf.ok ? 1 : 0;
    return 0;
  }
};
// The buffers as they stand over the docid-split pieces, in the reference's
// SafeBufs' capacities (allocTopTree, Posdb.cpp:931-975): m_scoreInfoBuf
// keeps at most what fits, and once it is full each new DocIdScore pushes out
// the first one whose docid the tree no longer holds, with that docid's
// pair / single chunks and the offsets after them (Posdb.cpp:7562-7665).
struct SplitSink {
  std::vector<gbgpu_docid_score> dinfo;
  std::vector<gbgpu_pair_score> dp;
  std::vector<gbgpu_single_score> ds;
  int64_t cap_d = 0, cap_p = 0, cap_s = 0;  // bytes
  int ng = 0;
  bool ints = false;
  std::vector<uint64_t> tree;  // the tree's docids after this piece, sorted (hasDocId)
  int operator()(uint64_t docid, const SurvOut &inf, int cs, int cp, const gbgpu_single_score *ss,
                 const gbgpu_pair_score *ps) {
    constexpr int64_t DS = sizeof(gbgpu_docid_score), PS = sizeof(gbgpu_pair_score), SS = sizeof(gbgpu_single_score);
    // a scorer whose records do not fit drops them (Posdb.cpp:3258-3264,
    // 4213-4219): not emulated
    if ((int64_t)(ds.size() + cs) * SS > cap_s || (int64_t)(dp.size() + cp) * PS > cap_p) return GBGPU_EUNSUPPORTED;
    gbgpu_docid_score d;
    std::memset(&d, 0, sizeof d);
    d.docid = (int64_t)docid;
    d.final_score = ints ? (double)inf.ival : (double)inf.score;  // Posdb.cpp:7557-7560
    d.site_rank = (int8_t)inf.site_rank;
    d.doc_lang = inf.doc_lang;
    d.num_required_terms = ng;
    d.num_pairs = cp;
    d.num_singles = cs;
    d.pairs_offset = cp ? (int32_t)(dp.size() * PS) : -1;
    d.singles_offset = cs ? (int32_t)(ds.size() * SS) : -1;
    for (int k = 0; k < cs; k++) {
      ds.push_back(ss[k]);
      zero_pads(&ds.back());
    }
    for (int k = 0; k < cp; k++) {
      dp.push_back(ps[k]);
      zero_pads(&dp.back());
    }
    if (!inf.ok) return 0;
    int64_t avail = cap_d - (int64_t)dinfo.size() * DS;
    if (avail < DS + 1) return 0;  // no room: its pair / single records stay, unreferenced
    zero_pads(&d);
    dinfo.push_back(d);
    avail -= DS;
    if (avail >= DS) return 0;
    size_t v = 0;
    for (; v < dinfo.size(); v++)
      if (!std::binary_search(tree.begin(), tree.end(), (uint64_t)dinfo[v].docid)) break;
    if (v == dinfo.size()) return 0;
    const gbgpu_docid_score x = dinfo[v];
    const int32_t po = x.pairs_offset, pz = x.num_pairs * (int32_t)PS;
    const int32_t so = x.singles_offset, sz = x.num_singles * (int32_t)SS;
    dinfo.erase(dinfo.begin() + (long)v);
    if (pz) dp.erase(dp.begin() + po / PS, dp.begin() + (po + pz) / PS);
    if (sz) ds.erase(ds.begin() + so / SS, ds.begin() + (so + sz) / SS);
    for (auto &e : dinfo) {
      if (e.pairs_offset > po) e.pairs_offset -= pz;
      if (e.singles_offset > so) e.singles_offset -= sz;
    }
    return 0;
  }
};
// the second pass over docs[0, n) (tree docids, high -> low) against the
// slot's last query: each docid's records to `sink`
template <class Sink>
static int score_info_docs(QuerySlot &q, const uint64_t *docs, int n, uint32_t nsurv, Sink &sink) {
  if (!n) return 0;
  const DevPlan *hpl = reinterpret_cast<const DevPlan *>(q.h_stage);  // this query's plan (enqueue's staging copy)
  const int scap = std::max(q.info_scap, 1), pcap = std::max(q.info_pcap, 1);
  const int nl = std::max(hpl->nlists, 1);
  size_t sort_tmp = 0;
  HIPCHECK(si_sort_pairs(nullptr, sort_tmp, nullptr, nullptr, nullptr, nullptr, nsurv, q.stream));
  const size_t o_key = 0;
  const size_t o_val = o_key + align256(8 * (size_t)nsurv);
  const size_t o_skey = o_val + align256(4 * (size_t)nsurv);
  const size_t o_sval = o_skey + align256(8 * (size_t)nsurv);
  const size_t o_cum = o_sval + align256(4 * (size_t)nsurv);
  const size_t o_tmp = o_cum + align256(4 * (size_t)nl * (nsurv + 1));
  const size_t o_tdoc = o_tmp + align256(sort_tmp);
  const size_t o_info = o_tdoc + align256(8 * (size_t)n);
  const size_t o_cnt = o_info + align256(sizeof(SurvOut) * (size_t)n);
  const size_t o_ss = o_cnt + align256(8 * (size_t)n);
  const size_t o_ps = o_ss + align256(sizeof(gbgpu_single_score) * (size_t)n * scap);
  const size_t o_mt = o_ps + align256(sizeof(gbgpu_pair_score) * (size_t)n * pcap);
  const size_t total = o_mt + 4 * (size_t)n;
  if (q.si.ensure(total)) return ENOMEM;
  hipStream_t st = q.stream;
  const uint32_t g = std::max(1u, std::min<uint32_t>(1024, (nsurv + 255) / 256));
  hipLaunchKernelGGL(k_si_keys, dim3(g), dim3(256), 0, st, q.svdoc.as<uint64_t>(), nsurv,
                     q.si.as<uint64_t>(o_key), q.si.as<uint32_t>(o_val));
  HIPCHECK(si_sort_pairs(q.si.as<uint8_t>(o_tmp), sort_tmp, q.si.as<uint64_t>(o_key), q.si.as<uint64_t>(o_skey),
                         q.si.as<uint32_t>(o_val), q.si.as<uint32_t>(o_sval), nsurv, st));
  hipLaunchKernelGGL(k_si_dir, dim3(nl), dim3(1024), 0, st, q.tables.as<DevPlan>(), q.svloc.as<Loc>(),
                     q.svlm.as<uint32_t>(), q.si.as<uint32_t>(o_sval), nsurv, q.si.as<uint32_t>(o_cum));
  HIPCHECK(hipMemcpyAsync(q.si.as<uint8_t>(o_tdoc), docs, 8 * (size_t)n, hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(k_scoreinfo, dim3((n + SCORE_TPB - 1) / SCORE_TPB), dim3(SCORE_TPB), 0, st,
                     q.tables.as<DevPlan>(), q.res.as<Counters>(), q.svslot.as<uint32_t>(), q.svlm.as<uint32_t>(),
                     q.svu.as<uint32_t>(), q.svloc.as<Loc>(), q.scratch.as<uint64_t>(),
                     (unsigned long long)(q.scratch.cap / 8), q.si.as<uint64_t>(o_tdoc), q.si.as<uint64_t>(o_skey), q.si.as<uint32_t>(o_sval),
                     q.si.as<uint32_t>(o_cum), nsurv, (uint32_t)n, q.si.as<SurvOut>(o_info),
                     q.si.as<int32_t>(o_cnt), q.si.as<gbgpu_single_score>(o_ss), scap,
                     q.si.as<gbgpu_pair_score>(o_ps), pcap, q.si.as<uint32_t>(o_mt));
  HIPCHECK(hipGetLastError());
  std::vector<SurvOut> info((size_t)n);
  std::vector<int32_t> cnt(2 * (size_t)n);
  std::vector<uint32_t> mt((size_t)n);
  std::vector<gbgpu_single_score> hs((size_t)n * scap);
  std::vector<gbgpu_pair_score> hp((size_t)n * pcap);
  auto fetch = [&]() -> int {
    HIPCHECK(hipMemcpyAsync(info.data(), q.si.as<uint8_t>(o_info), sizeof(SurvOut) * (size_t)n, hipMemcpyDeviceToHost, st));
    HIPCHECK(hipMemcpyAsync(cnt.data(), q.si.as<uint8_t>(o_cnt), 8 * (size_t)n, hipMemcpyDeviceToHost, st));
    HIPCHECK(hipMemcpyAsync(hs.data(), q.si.as<uint8_t>(o_ss), sizeof(gbgpu_single_score) * hs.size(),
                            hipMemcpyDeviceToHost, st));
    HIPCHECK(hipMemcpyAsync(hp.data(), q.si.as<uint8_t>(o_ps), sizeof(gbgpu_pair_score) * hp.size(),
                            hipMemcpyDeviceToHost, st));
    HIPCHECK(hipStreamSynchronize(st));
    return 0;
  };
  HIPCHECK(hipMemcpyAsync(mt.data(), q.si.as<uint8_t>(o_mt), 4 * (size_t)n, hipMemcpyDeviceToHost, st));
  if (int rc = fetch()) return rc;
  // docids whose last merged group comes out empty read the mbuf bytes
  // earlier docids left (k_si_stale): their writers, the second pass's first
  std::vector<SiStale> ents;
  bool need_first = false;
  for (int t = 0; t < n; t++) {
    if (info[t].ok != -4) continue;
    SiStale E;
    E.t = (uint32_t)t;
    E.O = mt[t];
    E.nb = info[t].pad == 1 ? 12 : 6;
    uint32_t need = 0;
    for (int p = 0; p < 12; p++) E.w[p] = ~0u;
    for (int t2 = t - 1; t2 >= 0 && need < E.nb; t2--) {
      const uint32_t T = mt[t2];
      if (T > E.O + need) {
        const uint32_t upto = std::min<uint32_t>(E.nb, T - E.O);
        for (uint32_t p = need; p < upto; p++) E.w[p] = (uint32_t)t2;
        need = upto;
      }
    }
    if (need < E.nb) need_first = true;
    ents.push_back(E);
  }
  if (!ents.empty()) {
    for (int t = 0; t < n; t++) {
      if (info[t].ok == -1) return GBGPU_ECORRUPT;
      if (info[t].ok == -2) return GBGPU_EUNSUPPORTED;
      if (info[t].ok == -3) return GBGPU_ECAPACITY;
    }
    const Counters *hc = reinterpret_cast<const Counters *>(q.h_res);
    const unsigned long long usum = hc->surv_top & ((1ull << 36) - 1);
    const size_t ne = ents.size();
    const unsigned long long mcap = need_first ? usum + 64ull * nsurv + 4096 : 0;
    const unsigned long long fcap = (unsigned long long)ne * (usum + 4096) + 4096;
    size_t o = 0;
    auto take = [&](size_t bytes) {
      const size_t at = o;
      o += align256(bytes);
      return at;
    };
    const size_t o_fixc = take(16), o_ent = take(sizeof(SiStale) * ne), o_lst = take(4 * (size_t)nsurv + 4),
                 o_marena = take(8 * (size_t)mcap), o_farena = take(8 * (size_t)fcap);
    if (q.si2.ensure(o) || q.svmb.ensure(4 * (size_t)nsurv + 4)) return ENOMEM;
    Counters *dctr = q.res.as<Counters>();
    if (need_first) {
      // the first pass's residue: every survivor's mbuf bytes (its merges
      // again), and its writers in vote-buffer (docid) order.  With site
      // clustering the prefilter's skips decide which docids wrote: declined
      if (q.replayed) return GBGPU_EUNSUPPORTED;
      HIPCHECK(hipMemsetAsync(q.si2.as<uint8_t>(o_fixc), 0, 16, st));
      hipLaunchKernelGGL(k_stale_mb, dim3((nsurv + SCORE_TPB - 1) / SCORE_TPB), dim3(SCORE_TPB), 0, st,
                         q.tables.as<DevPlan>(), dctr, nsurv, (const uint32_t *)q.svslot.as<uint32_t>(),
                         (const uint32_t *)q.svlm.as<uint32_t>(), (const uint32_t *)q.svu.as<uint32_t>(),
                         (const Loc *)q.svloc.as<Loc>(), q.si2.as<uint64_t>(o_marena), mcap,
                         q.si2.as<unsigned long long>(o_fixc), q.svmb.as<uint32_t>(), q.si2.as<uint32_t>(o_lst));
      HIPCHECK(hipGetLastError());
      std::vector<uint32_t> mb(nsurv), perm(nsurv);
      uint32_t unsup = 0;
      HIPCHECK(hipMemcpyAsync(mb.data(), q.svmb.p, 4 * (size_t)nsurv, hipMemcpyDeviceToHost, st));
      HIPCHECK(hipMemcpyAsync(perm.data(), q.si.as<uint8_t>(o_sval), 4 * (size_t)nsurv, hipMemcpyDeviceToHost, st));
      HIPCHECK(hipMemcpyAsync(&unsup, reinterpret_cast<uint8_t *>(dctr) + offsetof(Counters, unsup), 4,
                              hipMemcpyDeviceToHost, st));
      HIPCHECK(hipStreamSynchronize(st));
      if (unsup) return GBGPU_EUNSUPPORTED;
      for (auto &E : ents) {
        uint32_t need = 0;
        while (need < E.nb && E.w[need] != ~0u) need++;
        for (int64_t k = (int64_t)nsurv - 1; k >= 0 && need < E.nb; k--) {
          const uint32_t i = perm[(size_t)k];
          const uint32_t T = mb[i];
          if (T > E.O + need) {
            const uint32_t upto = std::min<uint32_t>(E.nb, T - E.O);
            for (uint32_t p = need; p < upto; p++) E.w[p] = 0x80000000u | i;
            need = upto;
          }
        }
        if (need < E.nb) return GBGPU_EUNSUPPORTED;  // bytes no docid of the call wrote: the stack's
      }
    }
#ifdef GBGPU_DIAG
    if (std::getenv("GBGPU_SI_DEBUG")) {
      for (const auto &E : ents)
        std::fprintf(stderr, "gbgpu si stale: t %u docid %llu O %u nb %u writers %x %x %x %x %x %x %x %x\n", E.t,
                     (unsigned long long)docs[E.t], E.O, E.nb, E.w[0], E.w[1], E.w[5], E.w[6], E.w[7], E.w[8], E.w[10],
                     E.w[11]);
      for (int t = 0; t < n; t++)
        std::fprintf(stderr, "gbgpu si mt: t %d docid %llu mt %u ok %d\n", t, (unsigned long long)docs[t], mt[t],
                     info[t].ok);
    }
#endif
    HIPCHECK(hipMemcpyAsync(q.si2.as<uint8_t>(o_ent), ents.data(), sizeof(SiStale) * ne, hipMemcpyHostToDevice, st));
    HIPCHECK(hipMemsetAsync(q.si2.as<uint8_t>(o_fixc), 0, 16, st));
    hipLaunchKernelGGL(k_si_stale, dim3((uint32_t)((ne + SCORE_TPB - 1) / SCORE_TPB)), dim3(SCORE_TPB), 0, st,
                       q.tables.as<DevPlan>(), dctr, (const uint32_t *)q.svslot.as<uint32_t>(),
                       (const uint32_t *)q.svlm.as<uint32_t>(), (const uint32_t *)q.svu.as<uint32_t>(),
                       (const Loc *)q.svloc.as<Loc>(), q.si2.as<uint64_t>(o_farena), fcap,
                       q.si2.as<unsigned long long>(o_fixc), (const uint64_t *)q.si.as<uint64_t>(o_tdoc),
                       (const uint64_t *)q.si.as<uint64_t>(o_skey), (const uint32_t *)q.si.as<uint32_t>(o_sval),
                       (const uint32_t *)q.si.as<uint32_t>(o_cum), nsurv, (const SiStale *)q.si2.as<SiStale>(o_ent),
                       (uint32_t)ne, q.si.as<SurvOut>(o_info), q.si.as<int32_t>(o_cnt),
                       q.si.as<gbgpu_single_score>(o_ss), scap, q.si.as<gbgpu_pair_score>(o_ps), pcap);
    HIPCHECK(hipGetLastError());
    if (int rc = fetch()) return rc;
    for (const auto &E : ents)
      if (info[E.t].ok == -3 || info[E.t].ok == -4) return GBGPU_EUNSUPPORTED;  // a replay that failed
  }
  for (int t = 0; t < n; t++) {
    if (info[t].ok == -1) return GBGPU_ECORRUPT;      // a tree docid with no survivor entry
    if (info[t].ok == -2) {  // a getWordPosList path not replayed
#ifdef GBGPU_DIAG
      if (std::getenv("GBGPU_SI_DEBUG"))
        std::fprintf(stderr, "gbgpu si decline: docid %llu path %d list %d\n", (unsigned long long)docs[t],
                     -((-info[t].pad) / 1000), (-info[t].pad) % 1000);
#endif
      return GBGPU_EUNSUPPORTED;
    }
    if (info[t].ok == -3) return GBGPU_ECAPACITY;     // record arena exhausted
    const int cs = cnt[2 * t], cp = cnt[2 * t + 1];
    if (cs > scap || cp > pcap) return GBGPU_ECAPACITY;
    const int rc = sink(docs[t], info[t], cs, cp, &hs[(size_t)t * scap], &hp[(size_t)t * pcap]);
    if (rc) return rc;
  }
  return 0;
}
// A boolean query's second pass (Posdb.cpp:6116-6244 with m_isBoolean): the
// loop still walks the tree's nodes (numProcessed, the docid-range skips),
// but the boolean block at boolJump1 (6514-6534) sets m_docId again from
// docIdPtr, which the second pass restarted at the vote buffer's start
// (6119) and advances once a docid (7732); the scorers are jumped over
// (6833), so the t-th DocIdScore is the t-th vote-buffer docid (ascending)
// with its boolean score -- unless the paging filter drops it -- with
// siteRank and docLang 0 and no pair or single records.  m: the docids the
// pass processes (at most the vote buffer's).
template <class Sink>
static int bool_info_docs(QuerySlot &q, int m, uint32_t nsurv, Sink &sink) {
  m = std::min<int>(m, (int)nsurv);
  if (m <= 0) return 0;
  size_t sort_tmp = 0;
  HIPCHECK(si_sort_pairs(nullptr, sort_tmp, nullptr, nullptr, nullptr, nullptr, nsurv, q.stream));
  const size_t o_key = 0;
  const size_t o_val = o_key + align256(8 * (size_t)nsurv);
  const size_t o_skey = o_val + align256(4 * (size_t)nsurv);
  const size_t o_sval = o_skey + align256(8 * (size_t)nsurv);
  const size_t o_tmp = o_sval + align256(4 * (size_t)nsurv);
  if (q.si.ensure(o_tmp + align256(sort_tmp))) return ENOMEM;
  hipStream_t st = q.stream;
  const uint32_t g = std::max(1u, std::min<uint32_t>(1024, (nsurv + 255) / 256));
  hipLaunchKernelGGL(k_si_keys, dim3(g), dim3(256), 0, st, q.svdoc.as<uint64_t>(), nsurv,
                     q.si.as<uint64_t>(o_key), q.si.as<uint32_t>(o_val));
  HIPCHECK(si_sort_pairs(q.si.as<uint8_t>(o_tmp), sort_tmp, q.si.as<uint64_t>(o_key), q.si.as<uint64_t>(o_skey),
                         q.si.as<uint32_t>(o_val), q.si.as<uint32_t>(o_sval), nsurv, st));
  std::vector<uint64_t> doc((size_t)m);
  std::vector<uint32_t> pos((size_t)m), key((size_t)nsurv);
  HIPCHECK(hipMemcpyAsync(doc.data(), q.si.as<uint8_t>(o_skey), 8 * (size_t)m, hipMemcpyDeviceToHost, st));
  HIPCHECK(hipMemcpyAsync(pos.data(), q.si.as<uint8_t>(o_sval), 4 * (size_t)m, hipMemcpyDeviceToHost, st));
  HIPCHECK(hipMemcpyAsync(key.data(), q.skey.p, 4 * (size_t)nsurv, hipMemcpyDeviceToHost, st));
  HIPCHECK(hipStreamSynchronize(st));
  for (int t = 0; t < m; t++) {
    const uint32_t k = key[pos[(size_t)t]];
    SurvOut inf;
    std::memset(&inf, 0, sizeof inf);
    const uint32_t b = (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k;
    std::memcpy(&inf.score, &b, 4);
    inf.ok = k != 0;  // 0: the paging filter dropped it (7327-7347)
    const int rc = sink(doc[(size_t)t], inf, 0, 0, nullptr, nullptr);
    if (rc) return rc;
  }
  return 0;
}

static int score_info(QuerySlot &q, const uint32_t *keys, const uint64_t *docs, uint32_t nsurv, gbgpu_result *out) {
  int n = 0;
  while (n < q.k && n < q.info_docs && keys[n]) n++;
  InfoAcc acc;
  OutSink sink{out, acc, q.info_ng, q.int_scores};
  const int rc = reinterpret_cast<const DevPlan *>(q.h_stage)->boolean ? bool_info_docs(q, n, nsurv, sink)
                                                                       : score_info_docs(q, docs, n, nsurv, sink);
  out->n_docid_scores = acc.nd;
  out->n_pair_scores = acc.np;
  out->n_single_scores = acc.ns;
  return rc ? rc : (acc.room ? 0 : ENOSPC);
}

// ------------------------------------------------------------------ facets
// Each facet query term's QueryTerm::m_facetHashTable (Posdb.h:401-413) and
// m_numDocsThatHaveFacet, after the scoring pass.  The reference builds them
// inside intersectLists10_r: every docid that reaches the TopTree (after the
// paging filter) walks its run in the facet list and votes once per entry
// (Posdb.cpp:7362-7542), then countUniqueDocids (5002-5038, called at
// 7786-7796) walks the facet list's whole buffer -- the survivors' runs that
// shrinkSubLists wrote over its start, then the list's own bytes past them --
// counting each record's value in an existing entry and each record longer
// than 6 bytes.  Here: the votes are emitted per survivor, sorted by (facet,
// key, docid) -- the reference's docid order, which a gbfacetfloat sum (a
// double accumulated in that order) needs -- and reduced one wave per entry;
// the buffer walk is the survivors' runs in parallel, the unaligned start of
// the list's tail walked by one lane until it meets a key start, and the rest
// of the tail in parallel (a walk that is aligned visits exactly the units
// whose byte 1 has the 0x02 bit).
constexpr int FAC_LDS = 4096;          // table entries counted in LDS per block

struct FacetPlan {
  int nf;
  int lid[MAXF];      // the facet group's only list (dense id); -1: no group
  int isfloat[MAXF];  // gbfacetfloat: ranges and stats compare as floats
  int nr[MAXF];       // ranges
  const int32_t *ra[MAXF], *rb[MAXF];
  const int32_t *tkey[MAXF];  // the table's keys, ascending (k_facet_outside / k_facet_tail)
  int tn[MAXF];
  uint32_t tbase[MAXF];  // the table's first counter in `outside`
  uint32_t units[MAXF];
  const uint8_t *list[MAXF];
  // docid splits: the tables as the pieces before left them (the Query's
  // QueryTerms keep them over the pieces), facet f's entries by key at
  // prev[prev_off[f], prev_off[f + 1]); null: the first piece or no splits
  const gbgpu_facet_entry *prev;
  uint32_t prev_off[MAXF + 1];
};

struct FacetCtr {
  uint32_t nrec, nseg;
  uint32_t pad[2];
  unsigned long long B[MAXF];     // units the survivors' runs take (the shrunk buffer's size)
  unsigned long long docs[MAXF];  // m_numDocsThatHaveFacet
  unsigned long long heads[MAXF]; // survivors with a run in the facet list (the shrunk buffer's 12-byte keys)
};

__device__ __forceinline__ int32_t fac_val(gu8 *k) {  // Posdb::getFacetVal32: bytes 2..5
  return (int32_t)((uint32_t)k[2] | ((uint32_t)k[3] << 8) | ((uint32_t)k[4] << 16) | ((uint32_t)k[5] << 24));
}

// the entry value v votes for (Posdb.cpp:7380-7430): the first range holding
// it (keyed by its A value), or v itself without ranges; false: no range
__device__ __forceinline__ bool fac_bucket(const FacetPlan &fp, int f, int32_t v, int32_t *key) {
  const int nr = fp.nr[f];
  if (nr == 0) {
    *key = v;
    return true;
  }
  const int32_t *ra = fp.ra[f], *rb = fp.rb[f];
  for (int k = 0; k < nr; k++) {
    const int32_t a = ra[k], b = rb[k];
    if (fp.isfloat[f]) {
      const float x = __int_as_float(v);
      if (x < __int_as_float(a)) continue;
      if (x >= __int_as_float(b)) continue;
    } else {
      if (v < a) continue;
      if (v >= b) continue;
    }
    *key = a;
    return true;
  }
  return false;
}

// key k of a run: its 12-byte head is units 0-1, its 6-byte keys follow
__device__ __forceinline__ gu8 *run_key(gu8 *list, Loc lc, uint32_t k) {
  return list + ((size_t)lc.unit + (k ? k + 1 : 0)) * 6;
}

// the survivors' votes: one record (facet, entry key, docid, value) per
// entry a docid's run touches first (FacetEntry::m_docId == docId skips the
// rest, 7440-7445); and each facet list's shrunk size B
// Site clustering: only the docids the prefilter did not skip reach the
// facet votes (Posdb.cpp:6341-6345 jump back to docIdLoop).  A docid is skipped
// when its bound B <= minWinningScore as the replay had it on reaching the
// docid: the last assignment (tp.mwsl, docid order) of a lower docid.  fkey:
// skey with the skipped docids' keys cleared.
__global__ void k_facet_live(uint32_t nsurv, const uint64_t *sdoc, const uint32_t *sv_ord, const uint4 *rep_slot,
                             const uint4 *mwsl, int ints, const uint32_t *skey, uint32_t *fkey) {
  const uint32_t nm = mwsl[0].x;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nsurv; i += gridDim.x * blockDim.x) {
    const uint64_t d = sdoc[i];
    const float B = __uint_as_float(rep_slot[sv_ord[i]].y);
    uint32_t lo = 0, hi = nm;  // assignments at docids < d: [1, 1 + lo)
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      const uint4 e = mwsl[1 + mid];
      if ((((uint64_t)e.y << 32) | e.x) < d) lo = mid + 1;
      else hi = mid;
    }
    const float mws = lo ? __uint_as_float(mwsl[lo].z) : -1.0f;
    const bool live = ints || !(B <= mws);
    fkey[i] = live ? skey[i] : 0u;
  }
}

__global__ void __launch_bounds__(256) k_facet_emit(FacetPlan fp, const Counters *ctr, FacetCtr *fc, const uint32_t *skey,
                                                    const uint64_t *sv_doc, const uint32_t *sv_lm, const Loc *sv_loc,
                                                    uint32_t nl,
                                                    uint64_t *rdoc, uint64_t *rkey, int32_t *rval, uint32_t cap) {
  const uint32_t nsurv = (uint32_t)(ctr->surv_top >> 36);
  const int lane = threadIdx.x & 63;
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t base = blockIdx.x * blockDim.x + (threadIdx.x & ~63u); base < nsurv; base += stride) {
    const uint32_t i = base + lane;
    const bool act = i < nsurv;
    const bool vote = act && skey[i] != 0;
    for (int f = 0; f < fp.nf; f++) {
      if (fp.lid[f] < 0) continue;
      gu8 *list = gl(fp.list[f]);
      // (a boolean expression may admit a docid the facet list does not hold)
      const Loc lc = act && (sv_lm[i] >> fp.lid[f] & 1) ? sv_loc[(uint64_t)i * nl + (uint32_t)fp.lid[f]] : Loc{0, 0};
      unsigned long long lsum = lc.len;
      for (int o = 32; o > 0; o >>= 1) lsum += __shfl_xor(lsum, o, 64);
      const unsigned long long nh = (unsigned long long)__popcll(__ballot(lc.len > 0));
      if (lane == 0) {
        atomicAdd(&fc->B[f], lsum);
        atomicAdd(&fc->heads[f], nh);
      }
      const uint32_t nk = vote && lc.len >= 2 ? lc.len - 1 : 0;
      // pass 0 counts this lane's records, pass 1 writes them
      uint32_t n = 0, at = 0;
      for (int pass = 0; pass < 2; pass++) {
        if (pass == 1) {
          uint32_t inc = n;  // inclusive scan over the wave
          for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(inc, o, 64);
            if (lane >= o) inc += y;
          }
          uint32_t wbase = 0;
          if (lane == 63 && inc) wbase = atomicAdd(&fc->nrec, inc);
          wbase = __shfl(wbase, 63, 64);
          at = wbase + inc - n;
        }
        for (uint32_t k = 0; k < nk; k++) {
          const int32_t v = fac_val(run_key(list, lc, k));
          int32_t key;
          if (!fac_bucket(fp, f, v, &key)) continue;
          bool seen = false;
          for (uint32_t j = 0; j < k && !seen; j++) {
            int32_t k2;
            seen = fac_bucket(fp, f, fac_val(run_key(list, lc, j)), &k2) && k2 == key;
          }
          if (seen) continue;
          if (pass == 0) {
            n++;
          } else if (at < cap) {
            rdoc[at] = sv_doc[i];
            rkey[at] = ((uint64_t)f << 32) | (uint32_t)(key ^ (int32_t)0x80000000);
            rval[at] = v;
            at++;
          }
        }
      }
    }
  }
}

__global__ void k_facet_gather(const uint32_t *idx, const uint64_t *rkey, uint32_t n, uint64_t *k2) {
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < n; j += gridDim.x * blockDim.x) k2[j] = rkey[idx[j]];
}

// the first record of each (facet, key) run of the sorted records
__global__ void __launch_bounds__(256) k_facet_heads(const uint64_t *k2s, uint32_t n, FacetCtr *fc, uint32_t *segs) {
  const int lane = threadIdx.x & 63;
  for (uint32_t base = blockIdx.x * blockDim.x + (threadIdx.x & ~63u); base < n; base += gridDim.x * blockDim.x) {
    const uint32_t j = base + lane;
    const bool head = j < n && (j == 0 || k2s[j] != k2s[j - 1]);
    const uint64_t m = __ballot(head);
    if (!m) continue;
    uint32_t w = 0;
    if (lane == 0) w = atomicAdd(&fc->nseg, (uint32_t)__popcll(m));
    w = __shfl(w, 0, 64);
    if (head) segs[w + (uint32_t)__popcll(m & ((1ull << lane) - 1))] = j;
  }
}

// one wave per entry: FacetEntry's count, last docid (the records are in
// docid order), and the sum / max / min of its votes -- a gbfacetfloat
// entry's in vote order (Posdb.cpp:7450-7540: the double sum and the float
// compares as the reference runs them)
__global__ void __launch_bounds__(256) k_facet_reduce(FacetPlan fp, const FacetCtr *fc, const uint64_t *k2s,
                                                      const uint32_t *idx, uint32_t n, const uint32_t *segs,
                                                      const uint64_t *rdoc, const int32_t *rval, gbgpu_facet_entry *out) {
  const int lane = threadIdx.x & 63;
  const uint32_t nseg = fc->nseg;
  const uint32_t nw = gridDim.x * (blockDim.x / 64);
  for (uint32_t s = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); s < nseg; s += nw) {
    const uint32_t st = segs[s];
    const uint64_t key = k2s[st];
    const int f = (int)(key >> 32);
    const bool fl = fp.isfloat[f] != 0;
    uint32_t cnt = 0;
    uint64_t last = 0;
    long long isum = 0;
    int32_t imin = INT32_MAX, imax = INT32_MIN;
    double fsum = 0.0;
    float fmin = 0.0f, fmax = 0.0f;
    uint32_t from = st;
    if (fp.prev) {
      // the entry as the earlier pieces left it: its votes go on from there,
      // and the docid that voted last there (pieces overlap by two docids)
      // is not counted again (Posdb.cpp:7509: fe->m_docId == m_docId)
      const int32_t k32 = (int32_t)((uint32_t)key ^ 0x80000000u);
      uint32_t lo = fp.prev_off[f], hi = fp.prev_off[f + 1];
      while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (fp.prev[mid].key < k32) lo = mid + 1;
        else hi = mid;
      }
      if (lo < fp.prev_off[f + 1] && fp.prev[lo].key == k32) {
        const gbgpu_facet_entry pv = fp.prev[lo];
        cnt = (uint32_t)pv.count;
        last = (uint64_t)pv.docid;
        if (cnt) {
          if (fl) {
            fsum = __longlong_as_double(pv.sum);
            fmin = __int_as_float(pv.min);
            fmax = __int_as_float(pv.max);
          } else {
            isum = pv.sum;
            imin = pv.min;
            imax = pv.max;
          }
          if (rdoc[idx[st]] == last) from = st + 1;
        }
      }
    }
    for (uint32_t j0 = from;; j0 += 64) {
      const uint32_t j = j0 + lane;
      const bool in = j < n && k2s[j] == key;
      const uint64_t m = __ballot(in);  // a prefix of the lanes: the run is contiguous
      const int c = __popcll(m);
      if (c == 0) break;
      const uint32_t id = in ? idx[j] : 0;
      const int32_t v = in ? rval[id] : 0;
      const uint64_t d = in ? rdoc[id] : 0;
      last = __shfl(d, c - 1, 64);
      if (fl) {
        for (int l = 0; l < c; l++) {  // every lane runs the same sequence
          const float x = __int_as_float(__shfl(v, l, 64));
          if (cnt == 0 && l == 0) {
            fmin = fmax = x;
          }
          fsum += (double)x;
          if (x < fmin) fmin = x;
          if (x > fmax) fmax = x;
        }
      } else {
        long long s2 = in ? (long long)v : 0;
        int32_t mn = in ? v : INT32_MAX, mx = in ? v : INT32_MIN;
        for (int o = 32; o > 0; o >>= 1) {
          s2 += __shfl_xor(s2, o, 64);
          const int32_t a = __shfl_xor(mn, o, 64), b = __shfl_xor(mx, o, 64);
          mn = a < mn ? a : mn;
          mx = b > mx ? b : mx;
        }
        isum += s2;
        imin = mn < imin ? mn : imin;
        imax = mx > imax ? mx : imax;
      }
      cnt += (uint32_t)c;
      if (c < 64) break;
    }
    if (lane == 0) {
      gbgpu_facet_entry e;
      e.term = f;  // the facet's index here; the host names the query term
      e.key = (int32_t)((uint32_t)key ^ 0x80000000u);
      e.count = (int32_t)cnt;
      e.outside = 0;
      e.docid = (int64_t)last;
      if (fl) {
        e.sum = __double_as_longlong(fsum);
        e.max = __float_as_int(fmax);
        e.min = __float_as_int(fmin);
      } else {
        e.sum = isum;
        e.max = imax;
        e.min = imin;
      }
      out[s] = e;
    }
  }
}

// the entry of value v in facet f's table (-1: none)
__device__ __forceinline__ int fac_find(const FacetPlan &fp, int f, int32_t v) {
  const int32_t *t = fp.tkey[f];
  int lo = 0, hi = fp.tn[f];
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (t[mid] < v) lo = mid + 1;
    else hi = mid;
  }
  return lo < fp.tn[f] && t[lo] == v ? lo : -1;
}

__device__ __forceinline__ void fac_count(uint32_t *lds, uint32_t *outside, bool use_lds, uint32_t e) {
  if (use_lds) atomicAdd(lds + e, 1u);
  else atomicAdd(outside + e, 1u);
}
__device__ __forceinline__ void fac_lds_init(uint32_t *lds, uint32_t et) {
  for (uint32_t e = threadIdx.x; e < et; e += blockDim.x) lds[e] = 0;
  __syncthreads();
}
__device__ __forceinline__ void fac_lds_flush(const uint32_t *lds, uint32_t et, uint32_t *outside) {
  __syncthreads();
  for (uint32_t e = threadIdx.x; e < et; e += blockDim.x)
    if (lds[e]) atomicAdd(outside + e, lds[e]);
}

// countUniqueDocids over the shrunk part of the buffer: every key of every
// survivor's run (voting or not) in an existing entry
__global__ void __launch_bounds__(256) k_facet_outside(FacetPlan fp, const Counters *ctr, const uint32_t *sv_lm,
                                                       const Loc *sv_loc, uint32_t nl, uint32_t et, uint32_t *outside) {
  __shared__ uint32_t s_cnt[FAC_LDS];
  const bool use_lds = et <= (uint32_t)FAC_LDS;
  if (use_lds) fac_lds_init(s_cnt, et);
  const uint32_t nsurv = (uint32_t)(ctr->surv_top >> 36);
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nsurv; i += gridDim.x * blockDim.x) {
    for (int f = 0; f < fp.nf; f++) {
      if (fp.lid[f] < 0 || fp.tn[f] == 0 || !(sv_lm[i] >> fp.lid[f] & 1)) continue;
      gu8 *list = gl(fp.list[f]);
      const Loc lc = sv_loc[(uint64_t)i * nl + (uint32_t)fp.lid[f]];
      const uint32_t nk = lc.len >= 2 ? lc.len - 1 : 0;
      for (uint32_t k = 0; k < nk; k++) {
        const int e = fac_find(fp, f, fac_val(run_key(list, lc, k)));
        if (e >= 0) fac_count(s_cnt, outside, use_lds, fp.tbase[f] + (uint32_t)e);
      }
    }
  }
  if (use_lds) fac_lds_flush(s_cnt, et, outside);
}

// the tail's start: the walk resumes at unit B, where the list's own bytes
// follow the shrunk runs -- possibly the second unit of a 12-byte key, read
// as a record of the size its byte 0 claims (RdbList::getRecSize) until the
// walk lands on a key start; one lane per facet.  tail0[f] = that start.
__global__ void k_facet_tailhead(FacetPlan fp, const Counters *ctr, FacetCtr *fc, uint32_t *outside,
                                 unsigned long long *tail0) {
  const int f = threadIdx.x;
  if (f >= fp.nf || fp.lid[f] < 0) return;
  gu8 *list = gl(fp.list[f]);
  const uint64_t units = fp.units[f];
  uint64_t u = fc->B[f];
  unsigned long long docs = fc->heads[f];  // every survivor run's head (12 bytes)
  while (u < units && !(list[u * 6 + 1] & 0x02)) {
    gu8 *k = list + u * 6;
    if (fp.tn[f]) {
      const int e = fac_find(fp, f, fac_val(k));
      if (e >= 0) atomicAdd(outside + fp.tbase[f] + (uint32_t)e, 1u);
    }
    const uint32_t rs = (k[0] & 0x04) ? 6u : (k[0] & 0x02) ? 12u : 18u;  // RdbList::getRecSize
    if (rs > 6) docs++;
    u += rs / 6;
  }
  tail0[f] = u;
  fc->docs[f] = docs;
}

// the aligned tail: each key start from tail0 on is one record
__global__ void __launch_bounds__(256) k_facet_tail(FacetPlan fp, FacetCtr *fc, const unsigned long long *tail0,
                                                    uint32_t et, uint32_t *outside) {
  __shared__ uint32_t s_cnt[FAC_LDS];
  const bool use_lds = et <= (uint32_t)FAC_LDS;
  if (use_lds) fac_lds_init(s_cnt, et);
  const int lane = threadIdx.x & 63;
  for (int f = 0; f < fp.nf; f++) {
    if (fp.lid[f] < 0) continue;
    gu8 *list = gl(fp.list[f]);
    const uint64_t u0 = tail0[f], units = fp.units[f];
    uint32_t heads = 0;
    for (uint64_t u = u0 + blockIdx.x * blockDim.x + threadIdx.x; u < units; u += (uint64_t)gridDim.x * blockDim.x) {
      gu8 *k = list + u * 6;
      const uint32_t b01 = (uint32_t)k[0] | ((uint32_t)k[1] << 8);
      if (!(b01 & 0x0200u)) continue;
      if (!(b01 & 0x04u)) heads++;  // a 12-byte record: a new docid
      if (fp.tn[f]) {
        const int e = fac_find(fp, f, fac_val(k));
        if (e >= 0) fac_count(s_cnt, outside, use_lds, fp.tbase[f] + (uint32_t)e);
      }
    }
    unsigned long long h = heads;
    for (int o = 32; o > 0; o >>= 1) h += __shfl_xor(h, o, 64);
    if (lane == 0 && h) atomicAdd(&fc->docs[f], h);
  }
  if (use_lds) fac_lds_flush(s_cnt, et, outside);
}

// The facet tables of the slot's collected query (see k_facet_emit): into
// out->facets (term then key ascending) and out->facet_docs.
static int facet_pass(QuerySlot &q, uint32_t nsurv, gbgpu_result *out) {
  const int nf = (int)q.facets.size();
  hipStream_t st = q.stream;
  FacetPlan fp;
  std::memset(&fp, 0, sizeof fp);
  fp.nf = nf;
  uint64_t cap = 0;
  size_t nranges = 0;
  for (int f = 0; f < nf; f++) {
    const FacetTerm &t = q.facets[f];
    fp.lid[f] = t.lid;
    fp.isfloat[f] = t.isfloat;
    fp.nr[f] = (int)t.a.size();
    fp.units[f] = t.units;
    fp.list[f] = t.list;
    if (t.lid >= 0) cap += t.units;
    nranges += t.a.size();
  }
  // docid splits: the tables the pieces before left (the entries' votes go
  // on from there, and this piece's records count in every entry they hold)
  std::vector<gbgpu_facet_entry> prev;
  if (q.facc) {
    for (int f = 0; f < nf; f++) {
      fp.prev_off[f] = (uint32_t)prev.size();
      auto it = q.facc->tab.find(q.facets[f].term);
      if (it != q.facc->tab.end())
        for (const auto &kv : it->second) prev.push_back(kv.second);
    }
    fp.prev_off[nf] = (uint32_t)prev.size();
  }
  const bool dev = cap > 0;
  // entries: the votes' and the ranges' (the ranges' A values stand as
  // entries from allocTopTree on, Posdb.cpp:5575-5631)
  std::vector<std::vector<gbgpu_facet_entry>> tab((size_t)nf);
  uint32_t nrec = 0, nseg = 0;
  const DevPlan *hpl = reinterpret_cast<const DevPlan *>(q.h_stage);
  const uint32_t nl = (uint32_t)std::max(hpl->nlists, 1);
  size_t o_ctr = 0, o_rng = 0, o_rdoc = 0, o_rkey = 0, o_rval = 0, o_k1 = 0, o_k1s = 0, o_i0 = 0, o_i1 = 0, o_k2 = 0,
         o_k2s = 0, o_i2 = 0, o_seg = 0, o_ent = 0, o_tkey = 0, o_out = 0, o_t0 = 0, o_tmp = 0, o_fkey = 0, o_prev = 0;
  const uint64_t ecap = cap + nranges + prev.size() + 1;  // table entries: voted keys + ranges (+ earlier pieces')
  if (dev) {
    if (cap >= (1ull << 31)) return GBGPU_ECAPACITY;
    size_t tmp1 = 0, tmp2 = 0;
    HIPCHECK(si_sort_pairs(nullptr, tmp1, nullptr, nullptr, nullptr, nullptr, (uint32_t)cap, st, 38));
    HIPCHECK(si_sort_pairs(nullptr, tmp2, nullptr, nullptr, nullptr, nullptr, (uint32_t)cap, st, 34));
    size_t o = 0;
    auto take = [&](size_t bytes) {
      const size_t at = o;
      o += align256(bytes);
      return at;
    };
    o_ctr = take(sizeof(FacetCtr));
    o_fkey = take(4 * (size_t)nsurv + 4);
    o_prev = take(sizeof(gbgpu_facet_entry) * std::max<size_t>(prev.size(), 1));
    o_rng = take(8 * std::max<size_t>(nranges, 1));
    o_rdoc = take(8 * cap);
    o_rkey = take(8 * cap);
    o_rval = take(4 * cap);
    o_k1 = take(8 * cap);
    o_k1s = take(8 * cap);
    o_i0 = take(4 * cap);
    o_i1 = take(4 * cap);
    o_k2 = take(8 * cap);
    o_k2s = take(8 * cap);
    o_i2 = take(4 * cap);
    o_seg = take(4 * cap);
    o_ent = take(sizeof(gbgpu_facet_entry) * cap);
    o_tkey = take(4 * ecap);
    o_out = take(4 * ecap);
    o_t0 = take(8 * MAXF);
    o_tmp = take(std::max(tmp1, tmp2));
    if (q.fac.ensure(o)) return ENOMEM;
    std::vector<int32_t> rng;
    size_t r = 0;
    for (int f = 0; f < nf; f++) {
      const FacetTerm &t = q.facets[f];
      fp.ra[f] = q.fac.as<int32_t>(o_rng) + r;
      rng.insert(rng.end(), t.a.begin(), t.a.end());
      r += t.a.size();
    }
    for (int f = 0; f < nf; f++) {
      const FacetTerm &t = q.facets[f];
      fp.rb[f] = q.fac.as<int32_t>(o_rng) + r;
      rng.insert(rng.end(), t.b.begin(), t.b.end());
      r += t.b.size();
    }
    if (!prev.empty()) {
      HIPCHECK(hipMemcpyAsync(q.fac.as<uint8_t>(o_prev), prev.data(), sizeof(gbgpu_facet_entry) * prev.size(),
                              hipMemcpyHostToDevice, st));
      fp.prev = q.fac.as<gbgpu_facet_entry>(o_prev);
    }
    HIPCHECK(hipMemsetAsync(q.fac.as<uint8_t>(o_ctr), 0, sizeof(FacetCtr), st));
    if (!rng.empty())
      HIPCHECK(hipMemcpyAsync(q.fac.as<uint8_t>(o_rng), rng.data(), 4 * rng.size(), hipMemcpyHostToDevice, st));
    FacetCtr *dfc = q.fac.as<FacetCtr>(o_ctr);
    if (nsurv) {
      const uint32_t g = std::max(1u, std::min<uint32_t>(2048, (nsurv + 255) / 256));
      // the votes' keys: the scores (0: not scored or dropped by the paging
      // filter), with site clustering also 0 where the prefilter skipped
      const uint32_t *vkey = q.skey.as<uint32_t>();
      if (q.replayed) {
        hipLaunchKernelGGL(k_facet_live, dim3(g), dim3(256), 0, st, nsurv, (const uint64_t *)q.svdoc.as<uint64_t>(),
                           (const uint32_t *)q.ord.as<uint32_t>(), (const uint4 *)(q.rep.as<uint4>() + q.rep_off),
                           (const uint4 *)q.mwsl.as<uint4>(), q.int_scores ? 1 : 0, vkey, q.fac.as<uint32_t>(o_fkey));
        vkey = q.fac.as<uint32_t>(o_fkey);
      }
      hipLaunchKernelGGL(k_facet_emit, dim3(g), dim3(256), 0, st, fp, (const Counters *)q.res.as<Counters>(), dfc,
                         vkey, (const uint64_t *)q.svdoc.as<uint64_t>(), (const uint32_t *)q.svlm.as<uint32_t>(),
                         (const Loc *)q.svloc.as<Loc>(), nl, q.fac.as<uint64_t>(o_rdoc), q.fac.as<uint64_t>(o_rkey),
                         q.fac.as<int32_t>(o_rval), (uint32_t)cap);
      HIPCHECK(hipGetLastError());
      HIPCHECK(hipMemcpyAsync(&nrec, &dfc->nrec, 4, hipMemcpyDeviceToHost, st));
      HIPCHECK(hipStreamSynchronize(st));
    }
    if (nrec > cap) return GBGPU_ECORRUPT;  // runs are disjoint parts of the lists: not reached
    if (nrec) {
      const uint32_t g = std::max(1u, std::min<uint32_t>(2048, (nrec + 255) / 256));
      // docid order, then (facet, key) order, stable: each entry's votes as the reference casts them
      hipLaunchKernelGGL(k_si_keys, dim3(g), dim3(256), 0, st, (const uint64_t *)q.fac.as<uint64_t>(o_rdoc), nrec,
                         q.fac.as<uint64_t>(o_k1), q.fac.as<uint32_t>(o_i0));
      size_t tb = std::max(tmp1, tmp2);
      HIPCHECK(si_sort_pairs(q.fac.as<uint8_t>(o_tmp), tb, q.fac.as<uint64_t>(o_k1), q.fac.as<uint64_t>(o_k1s),
                             q.fac.as<uint32_t>(o_i0), q.fac.as<uint32_t>(o_i1), nrec, st, 38));
      hipLaunchKernelGGL(k_facet_gather, dim3(g), dim3(256), 0, st, (const uint32_t *)q.fac.as<uint32_t>(o_i1),
                         (const uint64_t *)q.fac.as<uint64_t>(o_rkey), nrec, q.fac.as<uint64_t>(o_k2));
      tb = std::max(tmp1, tmp2);
      HIPCHECK(si_sort_pairs(q.fac.as<uint8_t>(o_tmp), tb, q.fac.as<uint64_t>(o_k2), q.fac.as<uint64_t>(o_k2s),
                             q.fac.as<uint32_t>(o_i1), q.fac.as<uint32_t>(o_i2), nrec, st, 34));
      hipLaunchKernelGGL(k_facet_heads, dim3(g), dim3(256), 0, st, (const uint64_t *)q.fac.as<uint64_t>(o_k2s), nrec,
                         dfc, q.fac.as<uint32_t>(o_seg));
      hipLaunchKernelGGL(k_facet_reduce, dim3(std::max(1u, std::min<uint32_t>(4096, (nrec + 3) / 4))), dim3(256), 0, st,
                         fp, (const FacetCtr *)dfc, (const uint64_t *)q.fac.as<uint64_t>(o_k2s),
                         (const uint32_t *)q.fac.as<uint32_t>(o_i2), nrec, (const uint32_t *)q.fac.as<uint32_t>(o_seg),
                         (const uint64_t *)q.fac.as<uint64_t>(o_rdoc), (const int32_t *)q.fac.as<int32_t>(o_rval),
                         q.fac.as<gbgpu_facet_entry>(o_ent));
      HIPCHECK(hipGetLastError());
      HIPCHECK(hipMemcpyAsync(&nseg, &dfc->nseg, 4, hipMemcpyDeviceToHost, st));
      HIPCHECK(hipStreamSynchronize(st));
      if (nseg > nrec) return GBGPU_ECORRUPT;
      std::vector<gbgpu_facet_entry> ents(nseg);
      if (nseg) {
        HIPCHECK(hipMemcpyAsync(ents.data(), q.fac.as<uint8_t>(o_ent), sizeof(gbgpu_facet_entry) * nseg,
                                hipMemcpyDeviceToHost, st));
        HIPCHECK(hipStreamSynchronize(st));
      }
      for (const gbgpu_facet_entry &e : ents) tab[(size_t)e.term].push_back(e);
    }
  }
  // the tables: votes and ranges, by key
  uint32_t et = 0;
  std::vector<int32_t> tkeys;
  for (int f = 0; f < nf; f++) {
    auto &t = tab[(size_t)f];
    std::sort(t.begin(), t.end(), [](const gbgpu_facet_entry &x, const gbgpu_facet_entry &y) { return x.key < y.key; });
    for (int32_t a : q.facets[f].a) {
      auto it = std::lower_bound(t.begin(), t.end(), a,
                                 [](const gbgpu_facet_entry &x, int32_t k) { return x.key < k; });
      if (it != t.end() && it->key == a) continue;
      gbgpu_facet_entry z;
      std::memset(&z, 0, sizeof z);
      z.key = a;
      t.insert(it, z);
    }
    for (auto &e : t) e.term = q.facets[f].term;
    if (q.facc) {
      // this piece's entries over the earlier pieces' (a voted entry came
      // back merged; a range entry nobody voted keeps what it had), then the
      // whole table, by key, for this piece's record counts
      auto &A = q.facc->tab[q.facets[f].term];
      for (const auto &e : t) {
        auto it = A.find(e.key);
        if (it == A.end()) {
          A[e.key] = e;
        } else if (e.count) {
          const int32_t o = it->second.outside;
          it->second = e;
          it->second.outside = o;
        }
      }
      t.clear();
      for (const auto &kv : A) t.push_back(kv.second);
    }
    fp.tbase[f] = et;
    fp.tn[f] = (int)t.size();
    for (auto &e : t) tkeys.push_back(e.key);
    et += (uint32_t)t.size();
  }
  std::vector<uint32_t> outside(et, 0);
  std::vector<uint64_t> docs((size_t)nf, 0);
  if (dev) {
    if (et > ecap) return GBGPU_ECORRUPT;
    for (int f = 0; f < nf; f++) fp.tkey[f] = q.fac.as<int32_t>(o_tkey) + fp.tbase[f];
    FacetCtr *dfc = q.fac.as<FacetCtr>(o_ctr);
    uint32_t *dout = q.fac.as<uint32_t>(o_out);
    if (et) {
      HIPCHECK(hipMemcpyAsync(q.fac.as<uint8_t>(o_tkey), tkeys.data(), 4 * (size_t)et, hipMemcpyHostToDevice, st));
      HIPCHECK(hipMemsetAsync(dout, 0, 4 * (size_t)et, st));
    }
    if (nsurv && et) {
      const uint32_t g = std::max(1u, std::min<uint32_t>(1024, (nsurv + 255) / 256));
      hipLaunchKernelGGL(k_facet_outside, dim3(g), dim3(256), 0, st, fp, (const Counters *)q.res.as<Counters>(),
                         (const uint32_t *)q.svlm.as<uint32_t>(), (const Loc *)q.svloc.as<Loc>(), nl, et, dout);
    }
    hipLaunchKernelGGL(k_facet_tailhead, dim3(1), dim3(64), 0, st, fp, (const Counters *)q.res.as<Counters>(), dfc,
                       dout, q.fac.as<unsigned long long>(o_t0));
    uint64_t tu = 0;
    for (int f = 0; f < nf; f++) tu = std::max<uint64_t>(tu, fp.units[f]);
    const uint32_t g = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(2048, (tu + 255) / 256));
    hipLaunchKernelGGL(k_facet_tail, dim3(g), dim3(256), 0, st, fp, dfc,
                       (const unsigned long long *)q.fac.as<unsigned long long>(o_t0), et, dout);
    HIPCHECK(hipGetLastError());
    FacetCtr hc;
    if (et) HIPCHECK(hipMemcpyAsync(outside.data(), dout, 4 * (size_t)et, hipMemcpyDeviceToHost, st));
    HIPCHECK(hipMemcpyAsync(&hc, dfc, sizeof hc, hipMemcpyDeviceToHost, st));
    HIPCHECK(hipStreamSynchronize(st));
    for (int f = 0; f < nf; f++) docs[(size_t)f] = q.facets[f].lid >= 0 ? hc.docs[f] : 0;
  }
  if (q.facc) {  // a docid-split piece: the counts go on over the pieces
    for (int f = 0; f < nf; f++) {
      auto &A = q.facc->tab[q.facets[f].term];
      const auto &t = tab[(size_t)f];
      for (size_t k = 0; k < t.size(); k++) A[t[k].key].outside += (int32_t)outside[fp.tbase[f] + k];
      q.facc->docs[q.facets[f].term] += docs[(size_t)f];
    }
    return 0;
  }
  int n = 0;
  std::vector<int> order((size_t)nf);
  for (int f = 0; f < nf; f++) order[(size_t)f] = f;
  std::sort(order.begin(), order.end(), [&](int x, int y) { return q.facets[x].term < q.facets[y].term; });
  for (int f : order) {
    auto &t = tab[(size_t)f];
    for (size_t k = 0; k < t.size(); k++) {
      t[k].outside = (int32_t)outside[fp.tbase[f] + k];
      if (out->facets && n < out->facets_cap) out->facets[n] = t[k];
      n++;
    }
    if (out->facet_docs) out->facet_docs[q.facets[f].term] = docs[(size_t)f];
  }
  out->n_facets = n;
  return out->facets && n > out->facets_cap ? ENOSPC : 0;
}

// The stale-mbuf survivors of the slot's pass (k_stale_find / k_stale_fix):
// scored from the bytes earlier docids left, then merged into the top list in
// the pinned result block (the best k by key, then docid) and in the device
// one (the exchange packs from it), their paging-filter drops kept in
// q.stale_filt.  Site clustering (the replay's prefilter skips decide which
// docids write mbuf) and the second pass decline.  The slot's stream is idle.
static int stale_fix(QuerySlot &q, uint32_t nsurv, uint32_t nstale) {
  if (q.replayed || q.want_info) return GBGPU_EUNSUPPORTED;
  const Counters *hc = reinterpret_cast<const Counters *>(q.h_res);
  hipStream_t st = q.stream;
  size_t sort_tmp = 0;
  HIPCHECK(si_sort_pairs(nullptr, sort_tmp, nullptr, nullptr, nullptr, nullptr, nsurv, st));
  size_t o = 0;
  auto take = [&](size_t bytes) {
    const size_t at = o;
    o += align256(bytes);
    return at;
  };
  const size_t o_key = take(8 * (size_t)nsurv), o_val = take(4 * (size_t)nsurv), o_skey = take(8 * (size_t)nsurv),
               o_ord = take(4 * (size_t)nsurv), o_rank = take(4 * (size_t)nsurv), o_wr = take(48 * (size_t)nstale),
               o_okey = take(4 * (size_t)nstale), o_sdoc = take(8 * (size_t)nstale), o_fixc = take(16),
               o_tmp = take(sort_tmp);
  // the fix arena: every survivor's merges once (k_stale_mb), then every
  // stale survivor's largest merge (its own records or a writer's)
  const unsigned long long usum = hc->surv_top & ((1ull << 36) - 1);
  const unsigned long long fcap = 2 * usum + 64ull * nsurv + 4096;
  const size_t o_arena = take(8 * (size_t)fcap);
  if (q.si.ensure(o)) return ENOMEM;
  const uint32_t g = std::max(1u, std::min<uint32_t>(1024, (nsurv + 255) / 256));
  hipLaunchKernelGGL(k_si_keys, dim3(g), dim3(256), 0, st, (const uint64_t *)q.svdoc.as<uint64_t>(), nsurv,
                     q.si.as<uint64_t>(o_key), q.si.as<uint32_t>(o_val));
  HIPCHECK(si_sort_pairs(q.si.as<uint8_t>(o_tmp), sort_tmp, q.si.as<uint64_t>(o_key), q.si.as<uint64_t>(o_skey),
                         q.si.as<uint32_t>(o_val), q.si.as<uint32_t>(o_ord), nsurv, st));
  hipLaunchKernelGGL(k_stale_rank, dim3(g), dim3(256), 0, st, (const uint32_t *)q.si.as<uint32_t>(o_ord), nsurv,
                     q.si.as<uint32_t>(o_rank));
  Counters *dctr = q.res.as<Counters>();
  if (q.svmb.ensure(4 * (size_t)nsurv) || q.stale.ensure(4 * (size_t)nstale)) return ENOMEM;
  HIPCHECK(hipMemsetAsync(q.si.as<uint8_t>(o_fixc), 0, 16, st));
  hipLaunchKernelGGL(k_stale_mb, dim3((nsurv + SCORE_TPB - 1) / SCORE_TPB), dim3(SCORE_TPB), 0, st,
                     q.tables.as<DevPlan>(), dctr, nsurv, (const uint32_t *)q.svslot.as<uint32_t>(),
                     (const uint32_t *)q.svlm.as<uint32_t>(), (const uint32_t *)q.svu.as<uint32_t>(),
                     (const Loc *)q.svloc.as<Loc>(), q.si.as<uint64_t>(o_arena), fcap,
                     q.si.as<unsigned long long>(o_fixc), q.svmb.as<uint32_t>(), q.stale.as<uint32_t>());
  HIPCHECK(hipMemsetAsync(q.si.as<uint8_t>(o_fixc), 0, 16, st));
  const uint32_t gs = std::max(1u, std::min<uint32_t>(1024, (nstale + 255) / 256));
  hipLaunchKernelGGL(k_stale_find, dim3(gs), dim3(256), 0, st, dctr, (const uint32_t *)q.stale.as<uint32_t>(),
                     (const uint32_t *)q.svmb.as<uint32_t>(), (const uint32_t *)q.si.as<uint32_t>(o_ord),
                     (const uint32_t *)q.si.as<uint32_t>(o_rank), q.si.as<uint32_t>(o_wr), (const uint8_t *)nullptr);
  hipLaunchKernelGGL(k_stale_fix, dim3((nstale + SCORE_TPB - 1) / SCORE_TPB), dim3(SCORE_TPB), 0, st,
                     q.tables.as<DevPlan>(), dctr, (const uint32_t *)q.stale.as<uint32_t>(),
                     (const uint32_t *)q.si.as<uint32_t>(o_wr), (const uint32_t *)q.svmb.as<uint32_t>(),
                     (const uint32_t *)q.svslot.as<uint32_t>(), (const uint32_t *)q.svlm.as<uint32_t>(),
                     (const uint32_t *)q.svu.as<uint32_t>(), (const uint64_t *)q.svdoc.as<uint64_t>(),
                     (const Loc *)q.svloc.as<Loc>(), q.si.as<uint64_t>(o_arena), fcap,
                     q.si.as<unsigned long long>(o_fixc), q.skey.as<uint32_t>(), q.si.as<uint32_t>(o_okey),
                     (uint8_t *)nullptr);
  hipLaunchKernelGGL(k_gather_docs, dim3(gs), dim3(256), 0, st, (const uint64_t *)q.svdoc.as<uint64_t>(),
                     (const uint32_t *)q.stale.as<uint32_t>(), (const Counters *)dctr, q.si.as<uint64_t>(o_sdoc));
  HIPCHECK(hipGetLastError());
  std::vector<uint32_t> okey(nstale);
  std::vector<uint64_t> sdoc(nstale);
  unsigned long long fixc[2] = {0, 0};
  uint32_t unsup = 0;
  HIPCHECK(hipMemcpyAsync(sdoc.data(), q.si.as<uint8_t>(o_sdoc), 8 * (size_t)nstale, hipMemcpyDeviceToHost, st));
  HIPCHECK(hipMemcpyAsync(okey.data(), q.si.as<uint8_t>(o_okey), 4 * (size_t)nstale, hipMemcpyDeviceToHost, st));
  HIPCHECK(hipMemcpyAsync(fixc, q.si.as<uint8_t>(o_fixc), 16, hipMemcpyDeviceToHost, st));
  HIPCHECK(hipMemcpyAsync(&unsup, &dctr->unsup, 4, hipMemcpyDeviceToHost, st));
  HIPCHECK(hipStreamSynchronize(st));
  if (unsup) return GBGPU_EUNSUPPORTED;
  q.stale_filt = (int32_t)fixc[1];
  // the docids of the scored ones, then the top list merged
  std::vector<std::pair<uint32_t, uint64_t>> all;
  for (uint32_t e = 0; e < nstale; e++)
    if (okey[e]) all.push_back({okey[e], sdoc[e]});
  if (all.empty()) return 0;
  uint32_t *keys = reinterpret_cast<uint32_t *>(q.h_res + res_keys_off());
  uint64_t *docs = reinterpret_cast<uint64_t *>(q.h_res + res_docs_off(q.k));
  for (int x = 0; x < q.k && keys[x]; x++) all.push_back({keys[x], docs[x]});
  std::sort(all.begin(), all.end(), [](const std::pair<uint32_t, uint64_t> &a, const std::pair<uint32_t, uint64_t> &b) {
    return a.first > b.first || (a.first == b.first && a.second < b.second);
  });
  for (int x = 0; x < q.k; x++) {
    keys[x] = x < (int)all.size() ? all[x].first : 0u;
    docs[x] = x < (int)all.size() ? all[x].second : ~0ull;
  }
  HIPCHECK(hipMemcpyAsync(q.res.as<uint8_t>(res_keys_off()), keys, 4 * (size_t)q.k, hipMemcpyHostToDevice, st));
  HIPCHECK(hipMemcpyAsync(q.res.as<uint8_t>(res_docs_off(q.k)), docs, 8 * (size_t)q.k, hipMemcpyHostToDevice, st));
  HIPCHECK(hipStreamSynchronize(st));
  return 0;
}

// Site clustering (a whole-range pass through k_tree_seq): the stale
// survivors' bytes come from the latest earlier docid that the replay's
// prefilter did not skip, and which docids it skips depends on the tree the
// stale survivors' own scores feed.  So: score them with the writers of an
// unskipped pass, replay (recording minWinningScore's assignments), derive
// the skips, find the writers again among the unskipped docids and score
// again -- until the scores the replay used are the ones its skips give
// (usually at once; at most STALE_ROUNDS replays, else EUNSUPPORTED).
constexpr int STALE_ROUNDS = 4;
static int stale_fix_clustered(QuerySlot &q, uint32_t nsurv, uint32_t nstale) {
  if (q.want_info || !q.facets.empty() || (q.tree_phase & TREE_EMIT)) return GBGPU_EUNSUPPORTED;
  const Counters *hc = reinterpret_cast<const Counters *>(q.h_res);
  hipStream_t st = q.stream;
  const uint64_t slot_ub = q.slot_ub;
  size_t sort_tmp = 0;
  HIPCHECK(si_sort_pairs(nullptr, sort_tmp, nullptr, nullptr, nullptr, nullptr, nsurv, st));
  size_t o = 0;
  auto take = [&](size_t bytes) {
    const size_t at = o;
    o += align256(bytes);
    return at;
  };
  const size_t o_key = take(8 * (size_t)nsurv), o_val = take(4 * (size_t)nsurv), o_skey = take(8 * (size_t)nsurv),
               o_ord = take(4 * (size_t)nsurv), o_rank = take(4 * (size_t)nsurv), o_wr = take(48 * (size_t)nstale),
               o_okey = take(4 * (size_t)nstale), o_fixc = take(16), o_skip = take((size_t)nsurv),
               o_tmp = take(sort_tmp);
  const unsigned long long usum = hc->surv_top & ((1ull << 36) - 1);
  const unsigned long long fcap = 2 * usum + 64ull * nsurv + 4096;
  const size_t o_arena = take(8 * (size_t)fcap);
  if (q.si.ensure(o) || q.svmb.ensure(4 * (size_t)nsurv) || q.stale.ensure(4 * (size_t)nstale) ||
      q.mwsl.ensure(16 * (slot_ub + 2)))
    return ENOMEM;
  const DevPlan *dpl = q.tables.as<DevPlan>();
  Counters *dctr = q.res.as<Counters>();
  const uint32_t g = std::max(1u, std::min<uint32_t>(1024, (nsurv + 255) / 256));
  // the survivors in docid order, every survivor's mbuf length, the stale list
  hipLaunchKernelGGL(k_si_keys, dim3(g), dim3(256), 0, st, (const uint64_t *)q.svdoc.as<uint64_t>(), nsurv,
                     q.si.as<uint64_t>(o_key), q.si.as<uint32_t>(o_val));
  HIPCHECK(si_sort_pairs(q.si.as<uint8_t>(o_tmp), sort_tmp, q.si.as<uint64_t>(o_key), q.si.as<uint64_t>(o_skey),
                         q.si.as<uint32_t>(o_val), q.si.as<uint32_t>(o_ord), nsurv, st));
  hipLaunchKernelGGL(k_stale_rank, dim3(g), dim3(256), 0, st, (const uint32_t *)q.si.as<uint32_t>(o_ord), nsurv,
                     q.si.as<uint32_t>(o_rank));
  HIPCHECK(hipMemsetAsync(q.si.as<uint8_t>(o_fixc), 0, 16, st));
  hipLaunchKernelGGL(k_stale_mb, dim3((nsurv + SCORE_TPB - 1) / SCORE_TPB), dim3(SCORE_TPB), 0, st, dpl, dctr, nsurv,
                     (const uint32_t *)q.svslot.as<uint32_t>(), (const uint32_t *)q.svlm.as<uint32_t>(),
                     (const uint32_t *)q.svu.as<uint32_t>(), (const Loc *)q.svloc.as<Loc>(), q.si.as<uint64_t>(o_arena),
                     fcap, q.si.as<unsigned long long>(o_fixc), q.svmb.as<uint32_t>(), q.stale.as<uint32_t>());
  // the replay as enqueue() launched it
  const bool ranked = q.rep_off != 0;
  uint4 *rep_slot = q.rep.as<uint4>() + q.rep_off;
  const uint32_t bgrid =
      (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((slot_ub + 64 * BND_WAVES - 1) / (64 * BND_WAVES), 4096));
  const int kcol = seq_columns(q.docs_wanted);
  TreeParams tp = tree_params(q.docs_wanted, q.tree_phase, q.int_scores);
  tp.mwsl = q.mwsl.as<uint4>();
  auto ks = q.int_scores ? (kcol == 1 ? k_tree_seq<1, true> : kcol == 4 ? k_tree_seq<4, true>
                            : kcol == 8 ? k_tree_seq<8, true> : k_tree_seq<16, true>)
                         : (kcol == 1 ? k_tree_seq<1, false> : kcol == 4 ? k_tree_seq<4, false>
                            : kcol == 8 ? k_tree_seq<8, false> : k_tree_seq<16, false>);
  const int k = q.k;
  uint8_t *skip = q.si.as<uint8_t>(o_skip);
  const uint32_t gs = std::max(1u, std::min<uint32_t>(1024, (nstale + 255) / 256));
  std::vector<uint32_t> okey(nstale), prev;
  for (int round = 0; round <= STALE_ROUNDS; round++) {
    // the stale survivors' writers (none skipped in the first round) and scores
    HIPCHECK(hipMemsetAsync(q.si.as<uint8_t>(o_fixc), 0, 16, st));
    hipLaunchKernelGGL(k_stale_find, dim3(gs), dim3(256), 0, st, dctr, (const uint32_t *)q.stale.as<uint32_t>(),
                       (const uint32_t *)q.svmb.as<uint32_t>(), (const uint32_t *)q.si.as<uint32_t>(o_ord),
                       (const uint32_t *)q.si.as<uint32_t>(o_rank), q.si.as<uint32_t>(o_wr),
                       round ? (const uint8_t *)skip : (const uint8_t *)nullptr);
    hipLaunchKernelGGL(k_stale_fix, dim3((nstale + SCORE_TPB - 1) / SCORE_TPB), dim3(SCORE_TPB), 0, st, dpl, dctr,
                       (const uint32_t *)q.stale.as<uint32_t>(), (const uint32_t *)q.si.as<uint32_t>(o_wr),
                       (const uint32_t *)q.svmb.as<uint32_t>(), (const uint32_t *)q.svslot.as<uint32_t>(),
                       (const uint32_t *)q.svlm.as<uint32_t>(), (const uint32_t *)q.svu.as<uint32_t>(),
                       (const uint64_t *)q.svdoc.as<uint64_t>(), (const Loc *)q.svloc.as<Loc>(),
                       q.si.as<uint64_t>(o_arena), fcap, q.si.as<unsigned long long>(o_fixc), q.skey.as<uint32_t>(),
                       q.si.as<uint32_t>(o_okey), q.sflag.as<uint8_t>());
    HIPCHECK(hipGetLastError());
    uint32_t unsup = 0;
    HIPCHECK(hipMemcpyAsync(okey.data(), q.si.as<uint8_t>(o_okey), 4 * (size_t)nstale, hipMemcpyDeviceToHost, st));
    HIPCHECK(hipMemcpyAsync(&unsup, &dctr->unsup, 4, hipMemcpyDeviceToHost, st));
    HIPCHECK(hipStreamSynchronize(st));
    if (unsup) return GBGPU_EUNSUPPORTED;
    if (round > 0 && okey == prev) {
      // the replay ran with these scores: its skips give them back
      HIPCHECK(hipMemcpyAsync(q.h_res, q.res.p, q.res_bytes, hipMemcpyDeviceToHost, st));
      HIPCHECK(hipStreamSynchronize(st));
      q.stale_filt = 0;  // the replay counted the paging filter's drops
      return hc->tree_err ? GBGPU_ECAPACITY : 0;
    }
    if (round == STALE_ROUNDS) break;
    prev = okey;
    // the replay again with these scores, recording minWinningScore
    HIPCHECK(hipMemsetAsync(&dctr->tree_err, 0, 4, st));
    hipLaunchKernelGGL(k_bound, dim3(bgrid), dim3(64 * BND_WAVES), 0, st, dpl, dctr, (const uint32_t *)q.svslot.as<uint32_t>(),
                       (const uint32_t *)q.svlm.as<uint32_t>(), (const Loc *)q.svloc.as<Loc>(),
                       (const uint32_t *)q.ord.as<uint32_t>(), (const uint32_t *)q.skey.as<uint32_t>(),
                       (const uint64_t *)q.svdoc.as<uint64_t>(), (const uint8_t *)q.sflag.as<uint8_t>(), rep_slot,
                       ranked ? q.oslot.as<uint32_t>() : nullptr);
    if (ranked) {
      const uint32_t rgrid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((slot_ub + 255) / 256, 4096));
      hipLaunchKernelGGL(k_rank, dim3(rgrid), dim3(256), 0, st, dpl, dctr, (const uint32_t *)q.oslot.as<uint32_t>(),
                         (const uint4 *)rep_slot, q.rep.as<uint4>());
    }
    if (q.seq_replay) {
      hipLaunchKernelGGL(ks, dim3(1), dim3(64 * SQ_W), 0, st, dctr, (const uint4 *)q.rep.as<uint4>(), tp,
                         q.res.as<uint32_t>(res_keys_off()), q.res.as<uint64_t>(res_docs_off(k)));
      TreeParams tf = tp;
      tf.on_reg_err = 1;
      hipLaunchKernelGGL(k_tree_replay, dim3(1), dim3(64), 0, st, dctr, (const uint4 *)q.rep.as<uint4>(),
                         (TreeState *)nullptr, tf, q.res.as<uint32_t>(res_keys_off()),
                         q.res.as<uint64_t>(res_docs_off(k)));
    } else {
      // the one-wave replay: a docid-split piece (from the tree the piece
      // started with), a tree past the register columns, or the diagnostic
      // GBGPU_REPLAY_MODE=1
      if (!(q.tree_phase & TREE_INIT))
        HIPCHECK(hipMemcpyAsync(q.tree.p, q.tree_bak.p, sizeof(TreeState), hipMemcpyDeviceToDevice, st));
      hipLaunchKernelGGL(k_tree_replay, dim3(1), dim3(64), 0, st, dctr, (const uint4 *)q.rep.as<uint4>(),
                         (q.tree_phase & TREE_FINAL) ? (TreeState *)q.tree.p : q.tree.as<TreeState>(), tp,
                         q.res.as<uint32_t>(res_keys_off()), q.res.as<uint64_t>(res_docs_off(k)));
    }
    hipLaunchKernelGGL(k_stale_skip, dim3(g), dim3(256), 0, st, nsurv, (const uint64_t *)q.svdoc.as<uint64_t>(),
                       (const uint32_t *)q.ord.as<uint32_t>(), (const uint4 *)rep_slot, (const uint4 *)q.mwsl.as<uint4>(),
                       q.int_scores ? 1 : 0, skip);
    HIPCHECK(hipGetLastError());
  }
  return GBGPU_EUNSUPPORTED;  // the scores did not settle
}

// hits_acc: when non-null, the query's intersected docids are appended to it
// (docid splits gather them over the pieces) instead of being written to out
static int collect(gbgpu_ctx *ctx, QuerySlot &q, gbgpu_result *out, std::vector<int64_t> *hits_acc = nullptr) {
  if (!q.pending) return EINVAL;
  q.pending = false;
  out->n = 0;
  out->hits = 0;
  out->filtered = 0;
  out->n_hit_docids = 0;
  out->n_docid_scores = out->n_pair_scores = out->n_single_scores = 0;
  out->docs_wanted = q.docs_wanted;
  out->n_facets = 0;
  if (out->facet_docs)  // the facet pass sets the terms with a table
    for (int t = 0; t < q.info_nterms; t++) out->facet_docs[t] = 0;
  if (q.early) {
    (void)hipStreamSynchronize(q.stream);  // nothing of this query; a failed one's kernels
    q.held.clear();
    return 0;
  }
  const hipError_t se = hipStreamSynchronize(q.stream);
  // the lists may go once this returns (gbgpu_list_free while in flight);
  // the facet pass still reads them
  std::vector<std::shared_ptr<ListMem>> held;
  held.swap(q.held);
  if (se != hipSuccess) {
    std::fprintf(stderr, "gbgpu: query stream failed: %s\n", hipGetErrorString(se));
    return GBGPU_EHIP;
  }
  if (DevBuf::canary_on())
    for (size_t i = 0; i < sizeof q.bufs / sizeof q.bufs[0]; i++)
      if (!q.bufs[i]->canary_ok())
        std::fprintf(stderr, "gbgpu: canary: slot buffer #%zu (cap %zu) overrun\n", i, q.bufs[i]->cap);
  if (DevBuf::canary_on())
    for (auto &m : held)
      if (m->dbg_len && m->hash(q.stream) != m->dbg_hash)
        std::fprintf(stderr, "gbgpu: canary: list %p changed during the query\n", (void *)m->d);
  if (ctx->profiling) {
    float t;
    (void)hipEventElapsedTime(&t, q.ev[0], q.ev[6]);
    q.last_ms[0] = t;
    for (int i = 1; i < 6; i++) {
      (void)hipEventElapsedTime(&t, q.ev[i - 1], q.ev[i]);
      q.last_ms[i] = t;
    }
  }
  const Counters *c = reinterpret_cast<const Counters *>(q.h_res);
  const uint32_t *keys = reinterpret_cast<const uint32_t *>(q.h_res + res_keys_off());
  const uint64_t *docs = reinterpret_cast<const uint64_t *>(q.h_res + res_docs_off(q.k));
  out->hits = (int64_t)(c->surv_top >> 36);
  out->filtered = (int32_t)c->filtered;
  {
    int64_t ncand = 0;
    for (int a = 0; a < MAXG0; a++) ncand += c->g0count[a];
    const int64_t st[8] = {q.scan_bytes, q.g0_bytes, q.probe_bytes, ncand, out->hits,
                           (int64_t)(c->surv_top & ((1ull << 36) - 1)) * 6, (int64_t)c->tree_n, 0};
    std::memcpy(q.stats, st, sizeof st);
  }
  if (c->corrupt) return GBGPU_ECORRUPT;
  if (c->tree_err) return GBGPU_ECAPACITY;
  if (c->unsup) return GBGPU_EUNSUPPORTED;
  if (c->nstale) {
    if (!q.stale_done) {
      const int rc = q.replayed ? stale_fix_clustered(q, (uint32_t)out->hits, c->nstale)
                                : stale_fix(q, (uint32_t)out->hits, c->nstale);
      if (rc) return rc;
      out->filtered = (int32_t)c->filtered;  // (a clustered replay counted them again)
    }
    out->filtered += q.stale_filt;
  }
#ifdef GBGPU_DIAG
  if (ctx->d_sdbg && ctx->sdbg_grid) {
    std::vector<uint64_t> h((size_t)ctx->sdbg_grid * 8);
    if (hipMemcpy(h.data(), ctx->d_sdbg, h.size() * 8, hipMemcpyDeviceToHost) == hipSuccess)
      if (const char *fn = std::getenv("GBGPU_SCORE_DUMP"))
        if (FILE *f = std::fopen(fn, "ab")) {
          std::fwrite(h.data(), 8, h.size(), f);
          std::fclose(f);
        }
  }
  if (ctx->d_pdbg) {
    std::vector<unsigned long long> h(1 + 16 * 32);
    if (hipMemcpy(h.data(), ctx->d_pdbg, 8 * h.size(), hipMemcpyDeviceToHost) == hipSuccess)
      for (unsigned long long o = 0; o < std::min<unsigned long long>(h[0] & 0xffffffffull, 32); o++) {
        const unsigned long long *r = &h[1 + 16 * o];
        std::fprintf(stderr,
                     "probe dbg: list %llu u0 %llu slot %llu lane %llu dlo %llu dhi %llu sh %llu bk %llu tag %llu "
                     "e %llx win0 %llu win63 %llu lo %llu nk %llu full|dec %llu hit %llx\n",
                     r[0], r[1], r[2], r[3], r[4], r[5], r[6], r[7], r[8], r[9], r[10], r[11], r[12], r[13], r[14], r[15]);
      }
  }
  if (ctx->topk_debug && q.sel.p) {
    unsigned long long td[8];
    if (hipMemcpy(td, q.sel.as<uint8_t>(offsetof(Select, tdbg)), sizeof td, hipMemcpyDeviceToHost) == hipSuccess)
      std::fprintf(stderr, "topk us: hist %.2f gather %.2f wait %.2f refine %.2f sort %.2f nb %llu nt %llu\n",
                   (td[1] - td[0]) / 100.0, (td[2] - td[1]) / 100.0, (td[3] - td[2]) / 100.0, (td[4] - td[3]) / 100.0,
                   (td[5] - td[4]) / 100.0, td[6], td[7]);
  }
  if (ctx->topk_debug && q.replayed)
    std::fprintf(stderr, "replay: adds %u nmax %u tree_n %u us_add|cand %u us_total %u nsurv %u "
                 "seq: us_in_add %.1f us_seq %.1f us_filt %.1f nseg %u\n", c->pad[0], c->pad[1],
                 c->tree_n, c->rdbg_t, c->rdbg_total, (uint32_t)(c->surv_top >> 36), c->sq_dbg[0] / 100.0,
                 c->sq_dbg[1] / 100.0, c->sq_dbg[2] / 100.0, c->sq_dbg[3]);
  if (ctx->debug_ext) {
    for (int l = 0; l < MAXL; l++)
      if (c->ext[l].units || c->ext[l].E)
        std::fprintf(stderr, "gbgpu ext list %d units %llu dmax %llu E %u slot1 %u\n", l, c->ext[l].units,
                     c->ext[l].dmax, c->ext[l].E, c->ext[l].slot1);
  }
#endif
  if (hits_acc || out->hit_docids) {
    std::vector<int64_t> local;
    std::vector<int64_t> &h = hits_acc ? *hits_acc : local;
    int rc = fetch_hits(q, (uint32_t)out->hits, h);
    if (rc) return rc;
    if (!hits_acc) write_hits(h, out);
  }
  int n = 0;
  for (int i = 0; i < q.k && n < out->capacity; i++) {
    const uint32_t key = keys[i];
    if (key == 0) break;
    const uint32_t b = (key & 0x80000000u) ? (key & 0x7fffffffu) : ~key;
    float f;
    std::memcpy(&f, &b, 4);
    if (q.int_scores) f = 0.0f;  // TopNode::m_score with integer scores (Posdb.cpp:7680-7683)
    if (out->docids) out->docids[n] = (int64_t)docs[i];
    if (out->scores) out->scores[n] = f;
    if (out->int_scores) out->int_scores[n] = q.int_scores ? (int32_t)(key ^ 0x80000000u) : 0;
    n++;
  }
  out->n = n;
  if (!q.facets.empty() && (out->facets || out->facet_docs || q.facc)) {
    const int rc = facet_pass(q, (uint32_t)out->hits, out);
    if (rc) return rc;
  }
  if (q.want_info) return score_info(q, keys, docs, (uint32_t)out->hits, out);
  return 0;
}

constexpr uint64_t GB_MAX_DOCID = 0x3fffffffffULL;  // MAX_DOCID = DOCID_MASK (Titledb.h:10-11)

// Msg39::controlLoop's docid-split loop (Msg39.cpp:345-457) on one slot: piece
// j reads docids [d0, d1+2] (getLists, Msg39.cpp:573-615, one stripe), so
// neighbouring pieces overlap; each piece is one PosdbTable pass over its
// windows of the resident lists (copied to 16-B aligned, zero-padded device
// buffers), into ONE TopTree sized at the first piece (allocTopTree's split
// branch, Posdb.cpp:859-877) and never reset; hits and m_filtered add up.
// Without site clustering the tree is the best docs_wanted by (score desc,
// docid asc), each docid once, whatever the insertion order -- so the pieces'
// top lists merge exactly on the host.
// One docid-split piece's second pass: the tree's nodes (tree[0, n), high ->
// low) whose docid lies in the piece's [lo, hi), walked under the
// m_docsToGet limit below, are scored again against the piece's survivors
// into the buffers `sink` keeps over the pieces.
static int split_info(QuerySlot &q, const int64_t *tree, int n, uint64_t lo, uint64_t hi, uint32_t nsurv,
                      SplitSink &sink, std::vector<uint64_t> &sel) {
  // numProcessed counts every node walked, but the docsToGet test runs only
  // before a docid is looked for: out-of-range nodes are skipped by `goto
  // nextNode` past it, so the first in-range node after the limit is still
  // scored (Posdb.cpp:6163-6193)
  sel.clear();
  int walked = 0, x = 0;
  while (walked < q.info_docs) {
    bool found = false;
    while (x < n) {
      const uint64_t d = (uint64_t)tree[x++];
      walked++;
      if (d >= lo && d < hi) {
        sel.push_back(d);
        found = true;
        break;
      }
    }
    if (!found) break;
  }
  if (sel.empty()) return 0;
  if (!sink.cap_d) {
    // allocTopTree's reservations, xx = max(the tree's nodes, 32)
    const int64_t xx = std::max<int64_t>(q.docs_wanted, 32);
    const int64_t nt = std::min<int64_t>(q.info_nterms, 10);
    sink.cap_d = xx * (int64_t)sizeof(gbgpu_docid_score) + 100;
    sink.cap_p = nt * nt / 2 * q.info_rmt * xx * (int64_t)sizeof(gbgpu_pair_score);
    sink.cap_s = nt * q.info_rmt * xx * (int64_t)sizeof(gbgpu_single_score);
    sink.ng = q.info_ng;
    sink.ints = q.int_scores;
  }
  sink.tree.assign(tree, tree + n);
  std::sort(sink.tree.begin(), sink.tree.end());
  if (reinterpret_cast<const DevPlan *>(q.h_stage)->boolean) return bool_info_docs(q, (int)sel.size(), nsurv, sink);
  return score_info_docs(q, sel.data(), (int)sel.size(), nsurv, sink);
}

static int query_splits(gbgpu_ctx *ctx, QuerySlot &q, const gbgpu_qterm *terms, int nterms,
                        const std::vector<ListEntry> &ents, const gbgpu_params *p, gbgpu_result *out) {
  std::vector<uint64_t> d0, d1, dmx;  // dmx: the piece's m_maxDocId (its second pass's range end)
  {
    const uint64_t delta = GB_MAX_DOCID / (uint64_t)p->num_docid_splits;
    uint64_t ddd = 0;
    do {
      const uint64_t a = ddd;
      ddd += delta;
      uint64_t b = ddd;
      if (b + 20 > GB_MAX_DOCID) {
        b = GB_MAX_DOCID;
        ddd = GB_MAX_DOCID;
      }
      d0.push_back(a);
      d1.push_back(std::min(b + 2, GB_MAX_DOCID));
      dmx.push_back(b);
    } while (ddd < GB_MAX_DOCID);
  }
  const int ns = (int)d0.size(), nl = nterms;
  if ((int64_t)ns * std::max(nl, 1) > (1 << 22)) return GBGPU_EUNSUPPORTED;
  // window search: in [list ptr nl | units nl | d0 ns | d1 ns], out SplitWin[nl][ns]
  std::vector<uint64_t> hin(2 * (size_t)nl + 2 * (size_t)ns);
  for (int i = 0; i < nl; i++) {
    hin[i] = (uint64_t)(uintptr_t)ents[i].d;
    hin[nl + i] = ents[i].units;
  }
  for (int j = 0; j < ns; j++) {
    hin[2 * nl + j] = d0[j];
    hin[2 * nl + ns + j] = d1[j];
  }
  const size_t in_bytes = 8 * hin.size();
  const size_t out_off = align256(in_bytes);
  const int nt = nl * ns;
  if (q.swin.ensure(out_off + sizeof(SplitWin) * (size_t)std::max(nt, 1))) return ENOMEM;
  std::vector<SplitWin> win((size_t)std::max(nt, 1));
  if (nt) {
    HIPCHECK(hipMemcpyAsync(q.swin.p, hin.data(), in_bytes, hipMemcpyHostToDevice, q.stream));
    const uint64_t *b = q.swin.as<uint64_t>();
    hipLaunchKernelGGL(k_split_windows, dim3((nt + 255) / 256), dim3(256), 0, q.stream, b, b + nl, nl, b + 2 * nl,
                       b + 2 * nl + ns, ns, q.swin.as<SplitWin>(out_off));
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipMemcpyAsync(win.data(), q.swin.as<uint8_t>(out_off), sizeof(SplitWin) * nt, hipMemcpyDeviceToHost,
                            q.stream));
    HIPCHECK(hipStreamSynchronize(q.stream));
  }
  // the tree's (score, docid): m_score, or m_intScore with a gbsortby int
  // term, as a double (exact for both)
  std::vector<std::pair<double, int64_t>> top;
  int32_t dw = 0;
  int64_t hits = 0;
  int32_t filtered = 0;
  std::vector<ListEntry> we(nl);
  std::vector<size_t> off(nl);
  std::vector<int64_t> td;
  std::vector<float> ts;
  std::vector<int32_t> ti;
  std::vector<int64_t> hit_ids;
  const bool clus = p->site_clustering != 0;
  bool tree_started = false, emitted = false;
  // m_getDocIdScoringInfo over the pieces: after each piece's first pass,
  // the reference walks the tree from its best node, counting at most
  // m_docsToGet nodes, and scores again the ones inside the piece's range
  // [m_minDocId, m_maxDocId) (Posdb.cpp:6160-6193); the records of every
  // piece append to the same buffers (they persist over pieces).  The pieces
  // run without the pass (pq), which this loop adds.
  const bool want_info = p->get_docid_scoring_info != 0;
  gbgpu_params pq = *p;
  pq.get_docid_scoring_info = 0;
  SplitSink sink;
  // facet terms: their tables and docid counts go on over the pieces
  // (facet_pass with q.facc); written out after the last
  FacetAcc facc;
  struct FaccGuard {
    QuerySlot &q;
    ~FaccGuard() { q.facc = nullptr; }
  } facc_guard{q};
  bool any_facet = false;
  for (int i = 0; i < nterms; i++)
    if (terms[i].field_code >= FIELD_GBFACETSTR && terms[i].field_code <= FIELD_GBFACETFLOAT) any_facet = true;
  if (any_facet && (out->facets || out->facet_docs)) q.facc = &facc;
  std::vector<uint64_t> sel;
  for (int j = 0; j < ns; j++) {
    size_t total = 0;
    for (int i = 0; i < nl; i++) {
      const SplitWin &w = win[(size_t)i * ns + j];
      off[i] = total;
      total += align256((size_t)(w.hi - w.lo) * 6 + LIST_PAD) + page_map_bytes(w.hi - w.lo);
    }
    if (q.split.ensure(std::max<size_t>(total, 256))) return ENOMEM;
    if (total) HIPCHECK(hipMemsetAsync(q.split.p, 0, total, q.stream));
    for (int i = 0; i < nl; i++) {
      const SplitWin &w = win[(size_t)i * ns + j];
      const uint32_t n = w.hi - w.lo;
      ListEntry e;
      e.d = q.split.as<uint8_t>(off[i]);
      e.pm = reinterpret_cast<uint32_t *>(e.d + align256((size_t)n * 6 + LIST_PAD));
      e.units = n;
      e.size = n ? (int64_t)n * 6 + 6 : 0;  // as Msg2 holds it: first key 18 bytes
      e.dmin = w.dmin;
      e.dmax = w.dmax;
      e.live = true;
      if (n) {
        HIPCHECK(hipMemcpyAsync(e.d, ents[i].d + (size_t)w.lo * 6, (size_t)n * 6, hipMemcpyDeviceToDevice, q.stream));
        int rc = build_page_map(e.d, n, e.pm, q.stream);
        if (rc) return rc;
      }
      we[i] = e;
    }
    if (dw == 0) {
      // allocTopTree at the first piece whose lists are not all empty; until
      // then Msg39 skips the pieces (Msg39.cpp:938-948, Posdb.cpp:890-891)
      std::vector<int64_t> sz(nl);
      for (int i = 0; i < nl; i++) sz[i] = we[i].size;
      dw = docs_wanted(p, sz.data(), nl);
      if (dw == 0) continue;
    }
    const int phase = clus ? ((tree_started ? 0 : TREE_INIT) | (j == ns - 1 ? TREE_FINAL : 0) | (want_info ? TREE_EMIT : 0))
                           : (TREE_INIT | TREE_FINAL);
    int rc = enqueue_entries(ctx, q, terms, nterms, we.data(), &pq, dw, phase);
    if (rc) {
      q.pending = false;
      return rc;
    }
    const bool replayed = q.replayed;
    if (replayed) tree_started = true;
    const int cap = clus ? TC : dw;
    td.assign(std::max(cap, 1), 0);
    ts.assign(std::max(cap, 1), 0.f);
    ti.assign(std::max(cap, 1), 0);
    gbgpu_result r;
    std::memset(&r, 0, sizeof r);
    r.docids = td.data();
    r.scores = ts.data();
    r.int_scores = ti.data();
    r.capacity = cap;
    rc = collect(ctx, q, &r, out->hit_docids ? &hit_ids : nullptr);
    auto node_key = [&](int x) -> double { return q.int_scores ? (double)ti[x] : (double)ts[x]; };
    if (rc) return rc;
    hits += r.hits;
    filtered += r.filtered;
    if (clus) {
      // one TopTree over every piece, carried on the device between them
      if (replayed && (phase & TREE_FINAL)) {
        emitted = true;
        for (int x = 0; x < r.n; x++) top.push_back({node_key(x), td[x]});
      }
      if (want_info && replayed) {
        rc = split_info(q, td.data(), r.n, d0[j], dmx[j], (uint32_t)r.hits, sink, sel);
        if (rc) return rc;
      }
      continue;
    }
    for (int x = 0; x < r.n; x++) top.push_back({node_key(x), td[x]});
    std::sort(top.begin(), top.end(), [](const std::pair<double, int64_t> &a, const std::pair<double, int64_t> &b) {
      return a.first > b.first || (a.first == b.first && a.second < b.second);
    });
    // a docid read by two overlapping pieces scores the same in both
    top.erase(std::unique(top.begin(), top.end(),
                          [](const std::pair<double, int64_t> &a, const std::pair<double, int64_t> &b) {
                            return a.second == b.second;
                          }),
              top.end());
    if ((int32_t)top.size() > dw) top.resize(dw);
    if (want_info && !q.early) {
      td.resize(top.size());
      for (size_t x = 0; x < top.size(); x++) td[x] = top[x].second;
      rc = split_info(q, td.data(), (int)top.size(), d0[j], dmx[j], (uint32_t)r.hits, sink, sel);
      if (rc) return rc;
    }
  }
  if (clus && tree_started && !emitted) {
    // the last piece scored nothing: the tree as the earlier pieces left it
    int rc = enqueue_tree_emit(q, dw);
    if (rc) {
      q.pending = false;
      return rc;
    }
    td.assign(TC, 0);
    ts.assign(TC, 0.f);
    ti.assign(TC, 0);
    gbgpu_result r;
    std::memset(&r, 0, sizeof r);
    r.docids = td.data();
    r.scores = ts.data();
    r.int_scores = ti.data();
    r.capacity = TC;
    rc = collect(ctx, q, &r);
    if (rc) return rc;
    for (int x = 0; x < r.n; x++) top.push_back({q.int_scores ? (double)ti[x] : (double)ts[x], td[x]});
  }
  out->hits = hits;
  out->filtered = filtered;
  out->docs_wanted = dw;
  out->n_facets = 0;
  if (q.facc) {
    if (out->facet_docs)
      for (int i = 0; i < nterms; i++) out->facet_docs[i] = 0;
    // every facet term has its table (allocTopTree over docid splits makes
    // one even for an empty list, its ranges as zeroed entries, Posdb.cpp:
    // 1013-1067), by term, then key
    for (int i = 0; i < nterms; i++) {
      if (terms[i].field_code < FIELD_GBFACETSTR || terms[i].field_code > FIELD_GBFACETFLOAT) continue;
      auto &A = facc.tab[i];
      for (int r = 0; r < p->n_facet_ranges; r++) {
        const gbgpu_facet_ranges &fr = p->facet_ranges[r];
        if (fr.term != i) continue;
        for (int k = 0; k < fr.n; k++)
          if (!A.count(fr.a[k])) {
            gbgpu_facet_entry z;
            std::memset(&z, 0, sizeof z);
            z.term = i;
            z.key = fr.a[k];
            A[fr.a[k]] = z;
          }
      }
    }
    int nfe = 0;
    for (const auto &tv : facc.tab) {
      for (const auto &kv : tv.second) {
        if (out->facets && nfe < out->facets_cap) {
          out->facets[nfe] = kv.second;
          out->facets[nfe].term = tv.first;
        }
        nfe++;
      }
      if (out->facet_docs) out->facet_docs[tv.first] = facc.docs[tv.first];
    }
    out->n_facets = nfe;
    if (out->facets && nfe > out->facets_cap) return ENOSPC;
  }
  bool room = true;
  if (want_info) {
    out->n_docid_scores = (int32_t)sink.dinfo.size();
    out->n_pair_scores = (int32_t)sink.dp.size();
    out->n_single_scores = (int32_t)sink.ds.size();
    room = out->n_docid_scores <= out->docid_scores_cap && out->n_pair_scores <= out->pair_scores_cap &&
           out->n_single_scores <= out->single_scores_cap;
    if (room) {
      std::copy(sink.dinfo.begin(), sink.dinfo.end(), out->docid_scores);
      std::copy(sink.dp.begin(), sink.dp.end(), out->pair_scores);
      std::copy(sink.ds.begin(), sink.ds.end(), out->single_scores);
    }
  }
  if (out->hit_docids) {
    // pieces overlap by two docids (getLists' [d0, d1+2]): the set has each once
    std::sort(hit_ids.begin(), hit_ids.end());
    hit_ids.erase(std::unique(hit_ids.begin(), hit_ids.end()), hit_ids.end());
    write_hits(hit_ids, out);
  }
  int n = 0;
  for (const auto &t : top) {
    if (n >= out->capacity) break;
    if (out->docids) out->docids[n] = t.second;
    if (out->scores) out->scores[n] = q.int_scores ? 0.0f : (float)t.first;
    if (out->int_scores) out->int_scores[n] = q.int_scores ? (int32_t)t.first : 0;
    n++;
  }
  out->n = n;
  return room ? 0 : ENOSPC;
}

// ------------------------------------------------------------------ C ABI
extern "C" {

int gbgpu_abi_version(void) { return GBGPU_ABI_VERSION; }

const char *gbgpu_strerror(int code) {
  switch (code) {
    case 0: return "ok";
    case GBGPU_ENODEVICE: return "no usable HIP device";
    case GBGPU_EUNSUPPORTED: return "request mode not supported by the GPU path";
    case GBGPU_ECORRUPT: return "corrupt posdb list";
    case GBGPU_EHIP: return "HIP runtime error";
    case GBGPU_ECAPACITY: return "device capacity exceeded";
    default: return std::strerror(code);
  }
}

static QuerySlot *slot_of(gbgpu_ctx *ctx, int slot) {
  if (!ctx || slot < 0) return nullptr;
  std::lock_guard<std::mutex> g(ctx->slots_mu);
  return slot < ctx->nslots ? ctx->slots[slot] : nullptr;
}

static int grow_slots(gbgpu_ctx *ctx, int n) {
  std::lock_guard<std::mutex> g(ctx->slots_mu);
  if (n > MAX_SLOTS) return EINVAL;
  while (ctx->nslots < n) {
    QuerySlot *q = new QuerySlot();
    int rc = q->init(ctx->pool);
    if (rc) {
      q->release();
      delete q;
      return rc;
    }
    ctx->slots[ctx->nslots++] = q;
  }
  return 0;
}

int gbgpu_open(int device, gbgpu_ctx **out) {
  if (!out) return EINVAL;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= device || device < 0) return GBGPU_ENODEVICE;
  if (hipSetDevice(device) != hipSuccess) return GBGPU_ENODEVICE;
  gbgpu_ctx *ctx = new gbgpu_ctx();
  ctx->device = device;
  if (!GBGPU_DEFAULT_POOL) {
    // the slots' stream-ordered buffers, resident lists and file images come
    // from the context's own pool (the device's default pool and its
    // process-wide settings are left alone): up to POOL_KEEP of what they
    // free stays cached there (a regrown buffer reuses it with no device
    // sync); beyond that the pool releases memory at the next sync, and a
    // freed list or file image is trimmed back to the device at once
    hipMemPoolProps pp;
    std::memset(&pp, 0, sizeof pp);
    pp.allocType = hipMemAllocationTypePinned;
    pp.handleTypes = hipMemHandleTypeNone;
    pp.location.type = hipMemLocationTypeDevice;
    pp.location.id = device;
    if (hipMemPoolCreate(&ctx->pool, &pp) != hipSuccess) {
      ctx->pool = nullptr;
      delete ctx;
      return GBGPU_EHIP;
    }
    uint64_t keep = POOL_KEEP;
    (void)hipMemPoolSetAttribute(ctx->pool, hipMemPoolAttrReleaseThreshold, &keep);
    if (const char *s = std::getenv("GBGPU_POOL_STRICT"); s && *s == '1') {
      // A/B: memory a stream freed is reused by that stream only
      int off = 0;
      (void)hipMemPoolSetAttribute(ctx->pool, hipMemPoolReuseAllowOpportunistic, &off);
      (void)hipMemPoolSetAttribute(ctx->pool, hipMemPoolReuseAllowInternalDependencies, &off);
      (void)hipMemPoolSetAttribute(ctx->pool, hipMemPoolReuseFollowEventDependencies, &off);
    }
  }
  Weights w = host_weights();
  ctx->arena->device = device;
  // the upload stream at the device's greatest priority (GBGPU_UPLOAD_PRIO=0:
  // the default): a cut's scan, which the host waits on, is dispatched ahead
  // of the queries in flight
  int prio_lo = 0, prio_hi = 0;
  (void)hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi);
  if (const char *s = std::getenv("GBGPU_UPLOAD_PRIO"); s && *s == '0') prio_hi = prio_lo;
  if (hipStreamCreateWithPriority(&ctx->upload_stream, hipStreamNonBlocking, prio_hi) != hipSuccess ||
      hipMalloc((void **)&ctx->d_flag, 4) != hipSuccess ||
      hipHostMalloc((void **)&ctx->h_flag, 4) != hipSuccess ||
      hipMemcpyToSymbol(HIP_SYMBOL(c_weights), &w, sizeof w) != hipSuccess || grow_slots(ctx, 1) != 0) {
    gbgpu_close(ctx);
    return GBGPU_EHIP;
  }
  for (DevBuf *b : {&ctx->lscan, &ctx->min_runs, &ctx->mout}) {
    b->st = ctx->upload_stream;
    b->pool = ctx->pool;
  }
#ifdef GBGPU_DIAG
  // diagnostic builds only (make diag: lib/libgbgpu_diag.so); the release
  // library reads no environment and runs the one production path
  if (const char *pm = std::getenv("GBGPU_PROBE_MODE")) ctx->probe_mode = std::atoi(pm);
  if (const char *rm = std::getenv("GBGPU_REPLAY_MODE")) ctx->replay_mode = std::atoi(rm);
  if (const char *pw = std::getenv("GBGPU_PROBE_WAVES")) ctx->probe_waves = std::atoi(pw);
  if (const char *rs = std::getenv("GBGPU_PROBE_RUNSPAN")) ctx->probe_runspan = std::atoi(rs);
  if (const char *dt = std::getenv("GBGPU_PROBE_DIR_T")) ctx->probe_dir_t = std::atof(dt);
  if (const char *sm = std::getenv("GBGPU_SCORE_MODE")) ctx->score_mode = std::atoi(sm);
  if (ctx->score_mode == 2) HIPCHECK(hipMalloc(&ctx->d_sdbg, 8192 * 64));
  if (const char *de = std::getenv("GBGPU_DEBUG_EXT")) ctx->debug_ext = std::atoi(de);
  ctx->probe_dbg_doc = std::getenv("GBGPU_PROBE_DEBUG_DOC");
  ctx->topk_debug = std::getenv("GBGPU_TOPK_DEBUG") != nullptr;
  if (ctx->probe_dbg_doc && hipMalloc((void **)&ctx->d_pdbg, 8 * (1 + 16 * 32)) != hipSuccess) ctx->d_pdbg = nullptr;
#endif
  *out = ctx;
  return 0;
}

void gbgpu_close(gbgpu_ctx *ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  for (int i = 0; i < ctx->nslots; i++) {
    ctx->slots[i]->release();
    delete ctx->slots[i];
  }
  if (ctx->comm) (void)ncclCommDestroy(ctx->comm);
  if (ctx->xstream) (void)hipStreamDestroy(ctx->xstream);
  ctx->xsend.release();
  ctx->xrecv.release();
  ctx->xout.release();
  ctx->xscratch.release();
  ctx->lscan.release();
  ctx->min_runs.release();
  ctx->mout.release();
  if (ctx->h_xout) (void)hipHostFree(ctx->h_xout);
  if (ctx->h_xf) (void)hipHostFree(ctx->h_xf);
  if (ctx->h_lst) (void)hipHostFree(ctx->h_lst);
  ctx->lists.clear();  // the last references: ListMem frees the device copies
  ctx->files.clear();
  if (ctx->upload_stream) (void)hipStreamSynchronize(ctx->upload_stream);
  gbmerge::state_free(ctx->merge);
  if (ctx->d_flag) (void)hipFree(ctx->d_flag);
  if (ctx->d_sdbg) (void)hipFree(ctx->d_sdbg);
  if (ctx->d_pdbg) (void)hipFree(ctx->d_pdbg);
  if (ctx->h_flag) (void)hipHostFree(ctx->h_flag);
  if (ctx->upload_stream) (void)hipStreamDestroy(ctx->upload_stream);
  if (ctx->pool) {
    (void)hipDeviceSynchronize();  // every stream-ordered free has run
    (void)hipMemPoolTrimTo(ctx->pool, 0);
    (void)hipMemPoolDestroy(ctx->pool);
  }
  delete ctx;
}

int gbgpu_set_query_slots(gbgpu_ctx *ctx, int n) {
  if (!ctx || n < 1) return EINVAL;
  (void)hipSetDevice(ctx->device);
  return grow_slots(ctx, n);
}

int gbgpu_query_slots(gbgpu_ctx *ctx) {
  if (!ctx) return 0;
  std::lock_guard<std::mutex> g(ctx->slots_mu);
  return ctx->nslots;
}

int32_t gbgpu_docs_wanted(const gbgpu_params *p, const int64_t *sizes, int nterms) {
  if (!p || (nterms && !sizes)) return 0;
  return docs_wanted(p, sizes, nterms);
}

int32_t gbgpu_tree_capacity(const gbgpu_params *p, const int64_t *sizes, int nterms) {
  if (!p || (nterms && !sizes)) return 0;
  const int32_t dw = docs_wanted(p, sizes, nterms);
  if (!p->site_clustering) return dw;
  return (int32_t)std::min<int64_t>(tree_nodes(dw, true), TREE_CAP);
}

// a freed list or file image goes back to the device once its stream-ordered
// free has run (TrimTo releases only memory no stream can still use); the
// slots' cached buffers up to POOL_KEEP stay
static void pool_trim(gbgpu_ctx *ctx) {
  if (ctx->pool) (void)hipMemPoolTrimTo(ctx->pool, POOL_KEEP);
  ctx->arena->trim(POOL_KEEP);
}

int gbgpu_list_upload(gbgpu_ctx *ctx, const uint8_t *bytes, int64_t size, int32_t *handle) {
  if (!ctx || !handle || (size > 0 && !bytes)) return EINVAL;
  std::lock_guard<std::mutex> g(ctx->lists_mu);
  (void)hipSetDevice(ctx->device);
  return upload_list(ctx, bytes, size, handle);
}

int gbgpu_file_upload(gbgpu_ctx *ctx, const uint8_t *bytes, int64_t size, int32_t *fh) {
  if (!ctx || !fh || size < 0 || (size > 0 && !bytes) || size % 6 != 0) return EINVAL;
  std::lock_guard<std::mutex> g(ctx->lists_mu);
  (void)hipSetDevice(ctx->device);
  FileEntry f;
  f.size = size;
  f.mem = std::make_shared<ListMem>();
  if (f.mem->alloc(ctx->arena, std::max<size_t>((size_t)size, 256))) return ENOMEM;
  if (size) HIPCHECK(hipMemcpyAsync(f.mem->d, bytes, (size_t)size, hipMemcpyHostToDevice, ctx->upload_stream));
  HIPCHECK(hipStreamSynchronize(ctx->upload_stream));
  f.live = true;
  for (size_t i = 0; i < ctx->files.size(); i++) {
    if (!ctx->files[i].live) {
      ctx->files[i] = f;
      *fh = (int32_t)i;
      return 0;
    }
  }
  ctx->files.push_back(f);
  *fh = (int32_t)ctx->files.size() - 1;
  return 0;
}

int gbgpu_file_free(gbgpu_ctx *ctx, int32_t fh) {
  if (!ctx) return EINVAL;
  std::shared_ptr<ListMem> last;  // lists cut from it are copies: nothing else holds it
  {
    std::lock_guard<std::mutex> g(ctx->lists_mu);
    if (fh < 0 || fh >= (int32_t)ctx->files.size() || !ctx->files[fh].live) return EINVAL;
    last = std::move(ctx->files[fh].mem);
    ctx->files[fh] = FileEntry();
  }
  (void)hipSetDevice(ctx->device);
  last.reset();
  pool_trim(ctx);
  return 0;
}

// RdbScan's read (RdbScan.cpp:319-361) on the device: bytes [offset,
// offset+size) of a resident file; a compressed first key (12 or 6 bytes) is
// replaced by the full key the caller's RdbMap gives for it (m_startKey), then
// the first-key swap of Posdb.cpp:5671-5703; the image goes through the same
// checks as gbgpu_list_upload.  A query's termlists are cut together (Msg2
// asks Msg3 for all of them at once): one round trip for the cuts' heads, one
// for their scans' outputs, whatever their number.
int gbgpu_file_lists(gbgpu_ctx *ctx, int32_t fh, int n, const int64_t *offsets, const int64_t *sizes,
                     const uint8_t *const *key18s, int32_t *handles) {
  if (!ctx || !handles || n < 0 || (n && (!offsets || !sizes)) || n > 4096) return EINVAL;
  for (int i = 0; i < n; i++) handles[i] = -1;
  std::lock_guard<std::mutex> g(ctx->lists_mu);
  (void)hipSetDevice(ctx->device);
  if (fh < 0 || fh >= (int32_t)ctx->files.size() || !ctx->files[fh].live) return EINVAL;
  const FileEntry &f = ctx->files[fh];
  for (int i = 0; i < n; i++)
    if (offsets[i] < 0 || sizes[i] < 0 || offsets[i] > f.size || sizes[i] > f.size - offsets[i] || offsets[i] % 6 ||
        sizes[i] % 6)
      return EINVAL;
  struct Cut {
    int ks = 18;
    uint8_t full[18];
    ListEntry e;
    CutSrc cs;
    uint32_t np = 0, ngran = 0;
    size_t o = 0, o_last = 0, o_hdr = 0;
  };
  std::vector<Cut> cut((size_t)n);
  // the heads, one round trip
  if (n && ctx->ensure_h_lst(32 * (size_t)n)) return ENOMEM;
  for (int i = 0; i < n; i++)
    if (sizes[i])
      HIPCHECK(hipMemcpyAsync(ctx->h_lst + 32 * (size_t)i, f.mem->d + offsets[i], (size_t)std::min<int64_t>(18, sizes[i]),
                              hipMemcpyDeviceToHost, ctx->upload_stream));
  HIPCHECK(hipStreamSynchronize(ctx->upload_stream));
  for (int i = 0; i < n; i++) {
    if (!sizes[i]) continue;
    const uint8_t *head = ctx->h_lst + 32 * (size_t)i;
    if (!(head[1] & 0x02)) return GBGPU_ECORRUPT;  // not a key start (Posdb.cpp:410-412)
    Cut &c = cut[(size_t)i];
    c.ks = (head[0] & 0x04) ? 6 : (head[0] & 0x02) ? 12 : 18;
    if (sizes[i] < c.ks) return GBGPU_ECORRUPT;
    const uint8_t *key18 = key18s ? key18s[i] : nullptr;
    if (key18) {
      // the map's key must be this key: its stored bytes, compression bits aside
      std::memcpy(c.full, key18, 18);
      if (c.full[0] & 0x06) return EINVAL;
      uint8_t a[18], b[18];
      std::memcpy(a, head, c.ks);
      std::memcpy(b, c.full, c.ks);
      a[0] &= 0xf9;
      if (std::memcmp(a, b, c.ks)) return EINVAL;
    } else {
      if (c.ks != 18) return EINVAL;  // a compressed first key needs the map's key
      std::memcpy(c.full, head, 18);
    }
  }
  // the images and their scans (k_list_scan<true> builds each image as it
  // scans it: one pass), the outputs side by side in the context's buffer
  size_t total = 0;
  for (int i = 0; i < n; i++) {
    if (!sizes[i]) continue;
    Cut &c = cut[(size_t)i];
    int rc = alloc_list(ctx, sizes[i] - c.ks + 18, c.e);
    if (rc) return rc;  // the cuts' entries free their images
    c.np = (c.e.units + CHUNK_UNITS - 1) / CHUNK_UNITS;
    c.ngran = c.np * 4;
    c.o = total;
    c.o_last = c.o + align256(8 * (size_t)c.ngran);
    c.o_hdr = c.o_last + align256(8 * (size_t)c.np);
    total = c.o_hdr + align256(sizeof(ListHdr));
    uint8_t first[12];
    std::memcpy(first, c.full, 12);
    first[0] |= 0x02;
    c.cs.file = f.mem->d;
    c.cs.fsize = (uint64_t)f.size;
    c.cs.src = (uint64_t)(offsets[i] + c.ks);
    c.cs.n = (uint64_t)(sizes[i] - c.ks);
    std::memcpy(c.cs.k, first, 12);
    c.cs.dst = reinterpret_cast<uint32_t *>(c.e.d);
  }
  if (total) {
    DevBuf &dgf = ctx->lscan;
    if (dgf.ensure(total) || ctx->ensure_h_lst(total)) return ENOMEM;
    for (int i = 0; i < n; i++) {
      if (!sizes[i]) continue;
      Cut &c = cut[(size_t)i];
      ListHdr *dh = reinterpret_cast<ListHdr *>(dgf.as<uint8_t>(c.o_hdr));
      HIPCHECK(hipMemsetAsync(dh, 0, sizeof(ListHdr), ctx->upload_stream));
      hipLaunchKernelGGL(k_list_scan<true>, dim3(c.np), dim3(BLOCK), 0, ctx->upload_stream, c.e.d, c.e.units, c.e.pm,
                         dgf.as<uint64_t>(c.o), dgf.as<uint64_t>(c.o_last), dh, c.cs);
      hipLaunchKernelGGL(k_list_tail, dim3(1), dim3(1024), 0, ctx->upload_stream, c.np, c.e.pm);
      HIPCHECK(hipGetLastError());
    }
    HIPCHECK(hipMemcpyAsync(ctx->h_lst, dgf.p, total, hipMemcpyDeviceToHost, ctx->upload_stream));
    HIPCHECK(hipStreamSynchronize(ctx->upload_stream));
    for (int i = 0; i < n; i++) {
      if (!sizes[i]) continue;
      Cut &c = cut[(size_t)i];
      int rc = scan_result(c.e, ctx->h_lst + c.o, ctx->h_lst + c.o_last, ctx->h_lst + c.o_hdr, c.np, c.full);
      if (rc) return rc;
    }
  }
  if (DevBuf::canary_level() == 1)
    for (int i = 0; i < n; i++) {
      if (sizes[i] <= cut[(size_t)i].ks) continue;
      const Cut &c = cut[(size_t)i];
      std::vector<uint8_t> a((size_t)c.cs.n), b((size_t)c.cs.n);
      HIPCHECK(hipMemcpy(a.data(), c.e.d + 12, a.size(), hipMemcpyDeviceToHost));
      HIPCHECK(hipMemcpy(b.data(), f.mem->d + c.cs.src, b.size(), hipMemcpyDeviceToHost));
      if (a != b)
        std::fprintf(stderr, "gbgpu: canary: cut %lld+%lld differs from the file\n", (long long)offsets[i],
                     (long long)sizes[i]);
    }
  // every cut checked: the handles
  for (int i = 0; i < n; i++) {
    int rc = sizes[i] ? register_list(ctx, cut[(size_t)i].e, &handles[i]) : upload_list(ctx, nullptr, 0, &handles[i]);
    if (rc) {
      for (int j = 0; j < i; j++) {
        ctx->lists[handles[j]] = ListEntry();
        handles[j] = -1;
      }
      return rc;
    }
  }
  return 0;
}

int gbgpu_file_list(gbgpu_ctx *ctx, int32_t fh, int64_t offset, int64_t size, const uint8_t *key18,
                    int32_t *handle) {
  if (!ctx || !handle || offset < 0 || size < 0) return EINVAL;
  return gbgpu_file_lists(ctx, fh, 1, &offset, &size, &key18, handle);
}

static gbmerge::MergeState *merge_state(gbgpu_ctx *ctx);

// Msg5::mergeLists_r over resident files (Msg5.cpp:1415-1471, 1621-1795):
// each piece becomes a merge input run in HBM starting with an 18-byte key
// (a file cut's compressed head replaced by the map key, as RdbScan does;
// RdbScan.cpp:319-361), the runs are merged on the device (merge.hip), and
// the merged list becomes a resident list (first-key swap, checks, page map)
// with device-to-device copies only.
int gbgpu_termlist_merge(gbgpu_ctx *ctx, const gbgpu_piece *pieces, int n, int remove_neg_keys,
                         int64_t min_rec_sizes, int32_t *handle, uint8_t *merged_out, int64_t merged_cap,
                         int64_t *merged_size) {
  if (!ctx || !handle || n < 0 || n > 256 || (n && !pieces)) return EINVAL;
  if (merged_size) *merged_size = 0;
  (void)hipSetDevice(ctx->device);
  gbmerge::MergeState *m = merge_state(ctx);
  if (!m) return GBGPU_EHIP;
  std::lock_guard<std::mutex> g(ctx->lists_mu);
  // the runs: one 16-B aligned segment each (the merge reads whole 16-byte
  // words), in piece order (oldest first)
  std::vector<int64_t> rsz(n), roff(n);
  std::vector<std::array<uint8_t, 18>> head(n);
  std::vector<const uint8_t *> src(n);  // device bytes after the first key (file pieces)
  std::vector<int> hks(n, 18);          // bytes the piece's first key takes in its source
  int64_t total = 0, in_bytes = 0;
  for (int i = 0; i < n; i++) {
    const gbgpu_piece &pc = pieces[i];
    if (pc.offset < 0 || pc.size < 0 || pc.size % 6) return EINVAL;
    rsz[i] = 0;
    roff[i] = in_bytes;
    if (!pc.size) continue;
    if (pc.file < 0) {
      if (!pc.bytes || pc.size < 18) return EINVAL;
      if (pc.bytes[pc.offset] & 0x06) return EINVAL;  // merge_r: every run starts with an 18-byte key
      std::memcpy(head[i].data(), pc.bytes + pc.offset, 18);
      rsz[i] = pc.size;
    } else {
      if (pc.file >= (int32_t)ctx->files.size() || !ctx->files[pc.file].live) return EINVAL;
      const FileEntry &f = ctx->files[pc.file];
      if (pc.offset > f.size || pc.size > f.size - pc.offset) return EINVAL;
      const uint8_t *d = f.mem->d + pc.offset;
      uint8_t h[18] = {};
      HIPCHECK(hipMemcpy(h, d, (size_t)std::min<int64_t>(18, pc.size), hipMemcpyDeviceToHost));
      if (!(h[1] & 0x02)) return GBGPU_ECORRUPT;  // not a key start
      const int ks = (h[0] & 0x04) ? 6 : (h[0] & 0x02) ? 12 : 18;
      if (pc.size < ks) return GBGPU_ECORRUPT;
      if (pc.key18) {
        uint8_t a[18], b[18];
        std::memcpy(a, h, ks);
        std::memcpy(b, pc.key18, ks);
        a[0] &= 0xf9;
        if ((pc.key18[0] & 0x06) || std::memcmp(a, b, ks)) return EINVAL;
        std::memcpy(head[i].data(), pc.key18, 18);
      } else {
        if (ks != 18) return EINVAL;
        std::memcpy(head[i].data(), h, 18);
      }
      hks[i] = ks;
      src[i] = d + ks;
      rsz[i] = pc.size - ks + 18;
    }
    total += rsz[i];
    in_bytes += (int64_t)align256((size_t)rsz[i] + 16);
  }
  if (total == 0) return upload_list(ctx, nullptr, 0, handle);
  // the context's merge buffers, grown between calls (under lists_mu)
  DevBuf &in = ctx->min_runs, &out = ctx->mout;
  if (in.ensure((size_t)in_bytes + 256) || out.ensure((size_t)total + 256)) return ENOMEM;
  std::vector<const uint8_t *> ptrs(n);
  for (int i = 0; i < n; i++) {
    uint8_t *dst = in.as<uint8_t>(roff[i]);
    ptrs[i] = dst;
    if (!rsz[i]) continue;
    const gbgpu_piece &pc = pieces[i];
    if (pc.file < 0) {
      HIPCHECK(hipMemcpyAsync(dst, pc.bytes + pc.offset, (size_t)rsz[i], hipMemcpyHostToDevice, ctx->upload_stream));
    } else {
      HIPCHECK(hipMemcpyAsync(dst, head[i].data(), 18, hipMemcpyHostToDevice, ctx->upload_stream));
      if (rsz[i] > 18)
        HIPCHECK(hipMemcpyAsync(dst + 18, src[i], (size_t)(rsz[i] - 18), hipMemcpyDeviceToDevice, ctx->upload_stream));
    }
    // zero the run's tail to its 16-byte word (the merge reads whole words)
    const size_t tail = align256((size_t)rsz[i] + 16) - (size_t)rsz[i];
    HIPCHECK(hipMemsetAsync(dst + rsz[i], 0, tail, ctx->upload_stream));
  }
  HIPCHECK(hipStreamSynchronize(ctx->upload_stream));  // the merge runs on its own stream
  int64_t osz = 0;
  int rc = gbmerge::merge_device(m, ptrs.data(), rsz.data(), n, remove_neg_keys, min_rec_sizes, out.as<uint8_t>(),
                                 (int64_t)out.cap, &osz);
  if (rc) return rc;
  if (merged_out || merged_size) {
    if (merged_size) *merged_size = osz;
    if (merged_out) {
      if (osz > merged_cap) return ENOSPC;
      if (osz) HIPCHECK(hipMemcpy(merged_out, out.p, (size_t)osz, hipMemcpyDeviceToHost));
    }
  }
  if (!osz) return upload_list(ctx, nullptr, 0, handle);
  uint8_t first[18];
  HIPCHECK(hipMemcpy(first, out.p, 18, hipMemcpyDeviceToHost));
  if (first[0] & 0x06) return GBGPU_ECORRUPT;
  ListEntry e;
  rc = alloc_list(ctx, osz, e);
  if (rc) return rc;
  uint8_t sw[12];
  std::memcpy(sw, first, 12);
  sw[0] |= 0x02;  // the first-key swap (Posdb.cpp:5689-5698)
  HIPCHECK(hipMemcpyAsync(e.d, sw, 12, hipMemcpyHostToDevice, ctx->upload_stream));
  if (osz > 18)
    HIPCHECK(hipMemcpyAsync(e.d + 12, out.as<uint8_t>(18), (size_t)(osz - 18), hipMemcpyDeviceToDevice,
                            ctx->upload_stream));
  return finish_list(ctx, e, nullptr, first, handle);
}

int gbgpu_list_free(gbgpu_ctx *ctx, int32_t h) {
  if (!ctx) return EINVAL;
  std::shared_ptr<ListMem> last;  // released outside the lock
  {
    std::lock_guard<std::mutex> g(ctx->lists_mu);
    if (h < 0 || h >= (int32_t)ctx->lists.size() || !ctx->lists[h].live) return EINVAL;
    // queries in flight hold their own references (QuerySlot::held), so the
    // memory outlives them; nothing is drained here
    last = std::move(ctx->lists[h].mem);
    ctx->lists[h] = ListEntry();
  }
  (void)hipSetDevice(ctx->device);
  last.reset();
  pool_trim(ctx);
  return 0;
}

int gbgpu_query_slot_enqueue(gbgpu_ctx *ctx, int slot, const gbgpu_qterm *terms, int nterms,
                             const int32_t *handles, const gbgpu_params *p) {
  QuerySlot *q = slot_of(ctx, slot);
  if (!q) return EINVAL;
  std::lock_guard<std::mutex> g(q->mu);
  (void)hipSetDevice(ctx->device);
  if (q->pending) return EBUSY;
  int rc = enqueue(ctx, *q, terms, nterms, handles, p);
  if (rc) q->pending = false;
  return rc;
}

int gbgpu_query_slot_collect(gbgpu_ctx *ctx, int slot, gbgpu_result *out) {
  QuerySlot *q = slot_of(ctx, slot);
  if (!q || !out) return EINVAL;
  int rc;
  {
    std::lock_guard<std::mutex> g(q->mu);
    (void)hipSetDevice(ctx->device);
    rc = collect(ctx, *q, out);
  }
  slot_released(ctx);
  return rc;
}

int gbgpu_query_resident_enqueue(gbgpu_ctx *ctx, const gbgpu_qterm *terms, int nterms, const int32_t *handles,
                                 const gbgpu_params *p) {
  return gbgpu_query_slot_enqueue(ctx, 0, terms, nterms, handles, p);
}

int gbgpu_query_collect(gbgpu_ctx *ctx, gbgpu_result *out) { return gbgpu_query_slot_collect(ctx, 0, out); }

// Blocking query on whichever slot is free (re-entrant: Msg39 runs several
// intersect threads); waits on one slot when all are busy.
static int query_resident_on(gbgpu_ctx *ctx, QuerySlot *q, const gbgpu_qterm *terms, int nterms,
                             const int32_t *handles, const gbgpu_params *p, gbgpu_result *out);

int gbgpu_query_resident(gbgpu_ctx *ctx, const gbgpu_qterm *terms, int nterms, const int32_t *handles,
                         const gbgpu_params *p, gbgpu_result *out) {
  if (!ctx || !out) return EINVAL;
  // take a free slot; when every slot is busy (other intersect threads, or
  // an enqueue/collect caller's uncollected query) wait until one is released
  for (;;) {
    const int n = gbgpu_query_slots(ctx);
    for (int i = 0; i < n; i++) {
      QuerySlot *c = slot_of(ctx, i);
      std::unique_lock<std::mutex> t(c->mu, std::try_to_lock);
      if (t.owns_lock() && !c->pending) {
        const int rc = query_resident_on(ctx, c, terms, nterms, handles, p, out);
        t.unlock();
        slot_released(ctx);
        return rc;
      }
    }
    std::unique_lock<std::mutex> w(ctx->free_mu);
    ctx->free_cv.wait_for(w, std::chrono::milliseconds(1));
  }
}

static int query_resident_on(gbgpu_ctx *ctx, QuerySlot *q, const gbgpu_qterm *terms, int nterms,
                             const int32_t *handles, const gbgpu_params *p, gbgpu_result *out) {
  (void)hipSetDevice(ctx->device);
  if (p && p->num_docid_splits > 1) {
    std::vector<ListEntry> ents;
    int rc = snapshot_lists(ctx, terms, nterms, handles, p, ents);
    if (!rc) rc = query_splits(ctx, *q, terms, nterms, ents, p, out);
    q->pending = false;
    // on an error, launched window copies may still read the lists `ents` holds
    if (rc) (void)hipStreamSynchronize(q->stream);
    return rc;
  }
  int rc = enqueue(ctx, *q, terms, nterms, handles, p);
  if (rc) {
    q->pending = false;
    (void)hipStreamSynchronize(q->stream);
    q->held.clear();
    return rc;
  }
  return collect(ctx, *q, out);
}

int gbgpu_query(gbgpu_ctx *ctx, const gbgpu_qterm *terms, int nterms, const gbgpu_list *lists,
                const gbgpu_params *p, gbgpu_result *out) {
  if (!ctx || !out || (nterms && !lists)) return EINVAL;
  std::vector<int32_t> h(nterms, -1);
  int rc = 0;
  for (int i = 0; i < nterms && !rc; i++) rc = gbgpu_list_upload(ctx, lists[i].bytes, lists[i].size, &h[i]);
  if (!rc) rc = gbgpu_query_resident(ctx, terms, nterms, h.data(), p, out);
  for (int i = 0; i < nterms; i++)
    if (h[i] >= 0) gbgpu_list_free(ctx, h[i]);
  return rc;
}

void *gbgpu_stream(gbgpu_ctx *ctx) { return gbgpu_slot_stream(ctx, 0); }

void *gbgpu_slot_stream(gbgpu_ctx *ctx, int slot) {
  QuerySlot *q = slot_of(ctx, slot);
  return q ? (void *)q->stream : nullptr;
}

int gbgpu_last_topk_device(gbgpu_ctx *ctx, void **dev_ptr, int32_t *n) {
  QuerySlot *q = slot_of(ctx, 0);
  if (!q || !dev_ptr || !n) return EINVAL;
  *dev_ptr = q->res.p ? q->res.as<uint8_t>(res_keys_off()) : nullptr;
  *n = q->k;
  return 0;
}

int gbgpu_set_profiling(gbgpu_ctx *ctx, int enable) {
  if (!ctx) return EINVAL;
  ctx->profiling = enable != 0;
  return 0;
}

int gbgpu_slot_timings(gbgpu_ctx *ctx, int slot, float *ms6, int64_t *scan_bytes) {
  QuerySlot *q = slot_of(ctx, slot);
  if (!q) return EINVAL;
  if (ms6) std::memcpy(ms6, q->last_ms, sizeof q->last_ms);
  if (scan_bytes) *scan_bytes = q->scan_bytes;
  return 0;
}

int gbgpu_slot_stats(gbgpu_ctx *ctx, int slot, int64_t *stats8) {
  QuerySlot *q = slot_of(ctx, slot);
  if (!q || !stats8) return EINVAL;
  std::memcpy(stats8, q->stats, sizeof q->stats);
  return 0;
}

// ------------------------------------------------ bandwidth ceiling (§8(d))
// The achievable-HBM reference the roofline is reported against beside the
// 8 TB/s spec: 16-byte-per-lane streaming kernels over buffers far larger
// than the 256 MiB Infinity Cache.
__global__ void __launch_bounds__(256) k_stream_read(const v4u *a, size_t n, uint32_t *sink) {
  uint32_t x = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const v4u v = __builtin_nontemporal_load(a + i);
    x ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (x == 0x9e3779b9u) sink[0] = x;  // keeps the loads; practically never stores
}
__global__ void __launch_bounds__(256) k_stream_copy(const v4u *a, v4u *b, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    __builtin_nontemporal_store(__builtin_nontemporal_load(a + i), b + i);
}

int gbgpu_bandwidth_ceiling(gbgpu_ctx *ctx, int64_t bytes, int iters, double *read_gbps, double *copy_gbps) {
  if (!ctx || bytes < (1 << 20) || iters < 1) return EINVAL;
  (void)hipSetDevice(ctx->device);
  const size_t n = (size_t)bytes / 16;
  v4u *a = nullptr, *b = nullptr;
  uint32_t *sink = nullptr;
  hipStream_t st = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  int rc = 0;
  float ms = 0.0f;
  if (hipMalloc(&a, n * 16) != hipSuccess || hipMalloc(&b, n * 16) != hipSuccess || hipMalloc(&sink, 4) != hipSuccess) {
    rc = ENOMEM;
    goto out;
  }
  if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess || hipEventCreate(&e0) != hipSuccess ||
      hipEventCreate(&e1) != hipSuccess) {
    rc = GBGPU_EHIP;
    goto out;
  }
  (void)hipMemsetAsync(a, 1, n * 16, st);
  (void)hipMemsetAsync(b, 0, n * 16, st);
  {
    const uint32_t grid = 256 * 8;  // 8 blocks of 256 per CU
    hipLaunchKernelGGL(k_stream_read, dim3(grid), dim3(256), 0, st, a, n, sink);
    (void)hipEventRecord(e0, st);
    for (int i = 0; i < iters; i++) hipLaunchKernelGGL(k_stream_read, dim3(grid), dim3(256), 0, st, a, n, sink);
    (void)hipEventRecord(e1, st);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (read_gbps) *read_gbps = (double)n * 16 * iters / (ms * 1e-3) / 1e9;
    hipLaunchKernelGGL(k_stream_copy, dim3(grid), dim3(256), 0, st, a, b, n);
    (void)hipEventRecord(e0, st);
    for (int i = 0; i < iters; i++) hipLaunchKernelGGL(k_stream_copy, dim3(grid), dim3(256), 0, st, a, b, n);
    (void)hipEventRecord(e1, st);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (copy_gbps) *copy_gbps = 2.0 * (double)n * 16 * iters / (ms * 1e-3) / 1e9;
    if (hipGetLastError() != hipSuccess) rc = GBGPU_EHIP;
  }
out:
  if (e0) (void)hipEventDestroy(e0);
  if (e1) (void)hipEventDestroy(e1);
  if (st) (void)hipStreamDestroy(st);
  if (a) (void)hipFree(a);
  if (b) (void)hipFree(b);
  if (sink) (void)hipFree(sink);
  return rc;
}

int gbgpu_last_timings(gbgpu_ctx *ctx, float *ms6, int64_t *scan_bytes) {
  return gbgpu_slot_timings(ctx, 0, ms6, scan_bytes);
}

int gbgpu_comm_unique_id(uint8_t *id) {
  if (!id) return EINVAL;
  ncclUniqueId u;
  if (ncclGetUniqueId(&u) != ncclSuccess) return GBGPU_EHIP;
  static_assert(sizeof(u) == GBGPU_COMM_ID_BYTES, "ncclUniqueId size");
  std::memcpy(id, &u, sizeof u);
  return 0;
}

int gbgpu_comm_init(gbgpu_ctx *ctx, int nranks, int rank, const uint8_t *id) {
  if (!ctx || !id || nranks < 1 || rank < 0 || rank >= nranks || nranks > 64) return EINVAL;
  std::lock_guard<std::mutex> g(ctx->x_mu);
  if (ctx->comm) return EBUSY;
  (void)hipSetDevice(ctx->device);
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof u);
  if (!ctx->xstream && hipStreamCreateWithFlags(&ctx->xstream, hipStreamNonBlocking) != hipSuccess) return GBGPU_EHIP;
  if (ncclCommInitRank(&ctx->comm, nranks, u, rank) != ncclSuccess) {
    ctx->comm = nullptr;
    return GBGPU_EHIP;
  }
  ctx->nranks = nranks;
  ctx->rank = rank;
  // the exchange buffers at their largest (XMAX entries), so no call can fail
  // to allocate once admitted: a failure there would skip the collective
  const size_t stride = align256(sizeof(XHead) + sizeof(XRec) * (size_t)XMAX);
  const size_t out_bytes = sizeof(XHead) + 16 * (size_t)XMAX;
  if (ctx->xsend.ensure(stride) || ctx->xrecv.ensure(stride * nranks) || ctx->xout.ensure(out_bytes) ||
      (out_bytes > ctx->h_xout_cap && (ctx->h_xout ? (void)hipHostFree(ctx->h_xout) : (void)0,
                                       ctx->h_xout = nullptr, ctx->h_xout_cap = 0,
                                       hipHostMalloc((void **)&ctx->h_xout, out_bytes) != hipSuccess))) {
    (void)ncclCommDestroy(ctx->comm);
    ctx->comm = nullptr;
    return ENOMEM;
  }
  ctx->h_xout_cap = std::max(ctx->h_xout_cap, out_bytes);
  {
    std::lock_guard<std::mutex> sg(ctx->xseq.mu);
    ctx->xseq.next = 0;
    ctx->xseq.busy = false;
  }
  return 0;
}

// One exchange, admitted by the context's sequencer: the collectives of
// every rank run in sequence-number order whichever thread gets here first.
// Once admitted, this rank takes part in the all-gather whatever happens: a
// failure before it (`err`: an invalid or idle slot, a failed pack) sends an
// empty reply, so the other ranks' exchange stays paired with theirs, and is
// returned after the collective.  Buffers were sized at gbgpu_comm_init.
static int allgather_admitted(gbgpu_ctx *ctx, QuerySlot *q, int err, int32_t k, int64_t *docids, double *scores,
                              int32_t *n, int64_t *hits, gbgpu_result *local) {
  std::lock_guard<std::mutex> xg(ctx->x_mu);
  if (!ctx->comm) return EINVAL;  // no communicator: no collective to pair
  std::unique_lock<std::mutex> lk;
  if (q) {
    lk = std::unique_lock<std::mutex>(q->mu);
    if (!q->pending) {
      if (!err) err = EINVAL;
      lk.unlock();
      q = nullptr;
    }
  }
  (void)hipSetDevice(ctx->device);
  const size_t stride = align256(sizeof(XHead) + sizeof(XRec) * (size_t)k);
  const size_t out_bytes = sizeof(XHead) + 16 * (size_t)k;
  hipStream_t xs = ctx->xstream;
  bool packed = false;
  if (q && !q->early && !err) {
    // stale-mbuf survivors are scored on the host's word after the pass: the
    // reply waits for them (the pass done, its result block read)
    if (hipStreamSynchronize(q->stream) != hipSuccess) err = GBGPU_EHIP;
    const Counters *hc = reinterpret_cast<const Counters *>(q->h_res);
    if (!err && hc->nstale && !hc->corrupt && !hc->tree_err && !hc->unsup) {
      err = q->replayed ? stale_fix_clustered(*q, (uint32_t)(hc->surv_top >> 36), hc->nstale)
                        : stale_fix(*q, (uint32_t)(hc->surv_top >> 36), hc->nstale);
      if (!err) q->stale_done = true;
    }
  }
  if (q && !q->early && !err) {
    if (hipStreamWaitEvent(xs, q->ev_done, 0) == hipSuccess) {
      hipLaunchKernelGGL(k_xpack, dim3(1), dim3(256), 0, xs, q->res.as<Counters>(), q->res.as<uint32_t>(res_keys_off()),
                         q->res.as<uint64_t>(res_docs_off(q->k)), (uint32_t)k, (uint32_t)q->k, q->int_scores ? 1 : 0,
                         ctx->xsend.as<uint8_t>());
      packed = hipGetLastError() == hipSuccess;
    }
    if (!packed) err = GBGPU_EHIP;
  }
  // an empty reply (n = 0, no hits): an early-out query, no slot, or a failure
  if (!packed && hipMemsetAsync(ctx->xsend.p, 0, sizeof(XHead), xs) != hipSuccess && !err) err = GBGPU_EHIP;
  if (ncclAllGather(ctx->xsend.p, ctx->xrecv.p, stride, ncclUint8, ctx->comm, xs) != ncclSuccess) err = GBGPU_EHIP;
  hipLaunchKernelGGL(k_xmerge, dim3(1), dim3(64), 0, xs, ctx->xrecv.as<uint8_t>(), ctx->nranks, (uint32_t)k, stride,
                     ctx->xout.as<uint8_t>());
  if (hipMemcpyAsync(ctx->h_xout, ctx->xout.p, out_bytes, hipMemcpyDeviceToHost, xs) != hipSuccess ||
      hipStreamSynchronize(xs) != hipSuccess)
    err = err ? err : GBGPU_EHIP;
  if (q) {
    // finish the slot's own query (its result block was read on the device);
    // collected even after a failure, so the slot is free again
    gbgpu_result tmp;
    std::memset(&tmp, 0, sizeof tmp);
    const int rc = collect(ctx, *q, local ? local : &tmp);
    lk.unlock();
    slot_released(ctx);
    if (!err) err = rc;
  }
  if (err) return err;
  const XHead *h = reinterpret_cast<const XHead *>(ctx->h_xout);
  const double *sc = reinterpret_cast<const double *>(ctx->h_xout + sizeof(XHead));
  const int64_t *dc = reinterpret_cast<const int64_t *>(ctx->h_xout + sizeof(XHead) + 8 * (size_t)k);
  *n = h->n;
  *hits = h->hits;
  for (int i = 0; i < h->n; i++) {
    if (docids) docids[i] = dc[i];
    if (scores) scores[i] = sc[i];
  }
  return 0;
}

// The sequence number is used up by every call that is admitted, whatever
// its outcome; only ETIMEDOUT (not admitted) leaves it to be retried.  k must
// be the same on every rank (it sizes the collective): a k out of range is
// refused before admission, as a protocol error of the caller.
int gbgpu_allgather_topk(gbgpu_ctx *ctx, int slot, uint64_t seq, int timeout_ms, int32_t k, int64_t *docids,
                         double *scores, int32_t *n, int64_t *hits, gbgpu_result *local) {
  if (!ctx || k < 1 || (uint32_t)k > XMAX || !n || !hits) return EINVAL;
  QuerySlot *q = nullptr;
  int err = 0;
  if (slot >= 0) {
    q = slot_of(ctx, slot);
    if (!q) err = EINVAL;  // still takes part, with an empty reply
  }
  int rc = seq_enter(&ctx->xseq, seq, timeout_ms);
  if (rc) return rc;
  rc = allgather_admitted(ctx, q, err, k, docids, scores, n, hits, local);
  seq_leave(&ctx->xseq, seq);
  return rc;
}

uint64_t gbgpu_exchange_next(gbgpu_ctx *ctx) { return ctx ? gbgpu_seq_next(&ctx->xseq) : 0; }

int gbgpu_seq_open(uint64_t first, gbgpu_seq **out) {
  if (!out) return EINVAL;
  gbgpu_seq *s = new gbgpu_seq();
  s->next = first;
  *out = s;
  return 0;
}
int gbgpu_seq_enter(gbgpu_seq *s, uint64_t seq, int timeout_ms) { return s ? seq_enter(s, seq, timeout_ms) : EINVAL; }
int gbgpu_seq_leave(gbgpu_seq *s, uint64_t seq) { return s ? seq_leave(s, seq) : EINVAL; }
uint64_t gbgpu_seq_next(const gbgpu_seq *s) {
  if (!s) return 0;
  std::lock_guard<std::mutex> g(const_cast<gbgpu_seq *>(s)->mu);
  return s->next;
}
void gbgpu_seq_close(gbgpu_seq *s) { delete s; }

int gbgpu_merge_topk_device(gbgpu_ctx *ctx, int nranks, int32_t k, const int32_t *counts, const int64_t *shard_hits,
                            const int64_t *const *shard_docids, const double *const *shard_scores,
                            int64_t *docids, double *scores, int32_t *n, int64_t *hits) {
  if (!ctx || nranks < 1 || nranks > 64 || k < 1 || (uint32_t)k > XMAX || !counts || !n || !hits) return EINVAL;
  (void)hipSetDevice(ctx->device);
  const size_t stride = align256(sizeof(XHead) + sizeof(XRec) * (size_t)k);
  std::vector<uint8_t> recv(stride * nranks, 0);
  for (int r = 0; r < nranks; r++) {
    XHead *h = reinterpret_cast<XHead *>(recv.data() + stride * r);
    XRec *rec = reinterpret_cast<XRec *>(recv.data() + stride * r + sizeof(XHead));
    const int m = std::min(counts[r], k);
    h->n = m;
    h->hits = shard_hits ? shard_hits[r] : 0;
    for (int i = 0; i < m; i++) {
      rec[i].score = shard_scores[r][i];
      rec[i].docid = (uint64_t)shard_docids[r][i];
    }
  }
  const size_t out_bytes = sizeof(XHead) + 16 * (size_t)k;
  DevBuf din, dout;
  if (din.ensure(recv.size()) || dout.ensure(out_bytes)) {
    din.release();
    dout.release();
    return ENOMEM;
  }
  std::vector<uint8_t> out(out_bytes);
  int rc = 0;
  if (hipMemcpy(din.p, recv.data(), recv.size(), hipMemcpyHostToDevice) != hipSuccess) rc = GBGPU_EHIP;
  if (!rc) {
    hipLaunchKernelGGL(k_xmerge, dim3(1), dim3(64), 0, 0, din.as<uint8_t>(), nranks, (uint32_t)k, stride,
                       dout.as<uint8_t>());
    if (hipGetLastError() != hipSuccess || hipMemcpy(out.data(), dout.p, out_bytes, hipMemcpyDeviceToHost) != hipSuccess)
      rc = GBGPU_EHIP;
  }
  din.release();
  dout.release();
  if (rc) return rc;
  const XHead *h = reinterpret_cast<const XHead *>(out.data());
  const double *sc = reinterpret_cast<const double *>(out.data() + sizeof(XHead));
  const int64_t *dc = reinterpret_cast<const int64_t *>(out.data() + sizeof(XHead) + 8 * (size_t)k);
  *n = h->n;
  *hits = h->hits;
  for (int i = 0; i < h->n; i++) {
    if (docids) docids[i] = dc[i];
    if (scores) scores[i] = sc[i];
  }
  return 0;
}

int gbgpu_merge_topk(const int64_t *const *sd, const double *const *ss, const int32_t *cnt, int nshards, int32_t k,
                     int64_t *od, double *os, int32_t *on) {
  // Msg3a::mergeLists, Msg3a.cpp:1315-1467: scanning the shards in order,
  // a later head replaces the best one only with a higher (double) score,
  // or an equal score and a lower docid; a docid already merged is skipped
  if (!on || nshards < 0 || k < 0) return EINVAL;
  std::vector<int32_t> cur(nshards, 0);
  std::vector<int64_t> seen;
  int32_t n = 0;
  while (n < k) {
    int best = -1;
    for (int s = 0; s < nshards; s++) {
      if (cur[s] >= cnt[s]) continue;
      if (best < 0) { best = s; continue; }
      const double sc = ss[s][cur[s]], bs = ss[best][cur[best]];
      if (sc < bs) continue;
      if (sc > bs || sd[s][cur[s]] < sd[best][cur[best]]) best = s;
    }
    if (best < 0) break;
    const int64_t bd = sd[best][cur[best]];
    const double bsc = ss[best][cur[best]];
    cur[best]++;
    if (std::find(seen.begin(), seen.end(), bd) != seen.end()) continue;
    seen.push_back(bd);
    od[n] = bd;
    os[n] = bsc;
    n++;
  }
  *on = n;
  return 0;
}

// ---- Msg3a::mergeLists whole over full replies (exchange.hip)
int gbgpu_merge_replies(const gbgpu_merge_req *req, const gbgpu_reply *replies, int nshards, gbgpu_merged *out) {
  return gbx::merge_host(req, replies, nshards, out);
}

// the replies' packs, `stride` apart (the layout the all-gather leaves)
static int pack_all(const gbgpu_merge_req *req, const gbgpu_reply *replies, int nshards, std::vector<uint8_t> &buf,
                    size_t &stride, std::vector<int32_t> &fbytes) {
  stride = 256;
  for (int j = 0; j < nshards; j++) {
    const gbgpu_reply &r = replies[j];
    const size_t b = gbx::pack_bytes(&r);
    if (!b || r.nqt != req->nqt || (req->site_clustering && r.n > 0 && !r.cluster_recs) ||
        (r.n > 0 && (!r.docids || !r.scores)))
      return EINVAL;
    stride = std::max(stride, align256(b));
  }
  buf.assign(stride * nshards, 0);
  fbytes.assign(nshards, 0);
  for (int j = 0; j < nshards; j++) {
    gbx::pack_reply(&replies[j], req->nqt, buf.data() + stride * j);
    fbytes[j] = replies[j].facet_list ? replies[j].facet_list_size : 0;
  }
  return 0;
}

int gbgpu_merge_replies_device(gbgpu_ctx *ctx, const gbgpu_merge_req *req, const gbgpu_reply *replies, int nshards,
                               gbgpu_merged *out) {
  gbx::XFReq rq;
  if (!ctx || !out || nshards < 1 || nshards > 64 || !replies) return EINVAL;
  int rc = gbx::make_req(req, &rq);
  if (rc) return rc;
  if ((uint32_t)req->docs_to_get > gbx::XFMAX) return EINVAL;
  std::vector<uint8_t> buf;
  std::vector<int32_t> fb;
  size_t stride = 0;
  if ((rc = pack_all(req, replies, nshards, buf, stride, fb))) return rc;
  const size_t sb = gbx::merge_scratch_bytes(nshards, fb.data());
  if (!sb) return GBGPU_ECAPACITY;
  std::lock_guard<std::mutex> xg(ctx->x_mu);
  (void)hipSetDevice(ctx->device);
  if (!ctx->xstream && hipStreamCreateWithFlags(&ctx->xstream, hipStreamNonBlocking) != hipSuccess) return GBGPU_EHIP;
  hipStream_t xs = ctx->xstream;
  // the packs go where an all-gather would leave them (the receive buffer),
  // staged through pinned memory
  if (ctx->xrecv.ensure(buf.size()) || ctx->xscratch.ensure(sb) ||
      ctx->ensure_h_xf(std::max(buf.size(), gbx::merge_stage_bytes())))
    return ENOMEM;
  std::memcpy(ctx->h_xf, buf.data(), buf.size());
  if (hipMemcpyAsync(ctx->xrecv.p, ctx->h_xf, buf.size(), hipMemcpyHostToDevice, xs) != hipSuccess ||
      hipStreamSynchronize(xs) != hipSuccess)
    return GBGPU_EHIP;
  rc = gbx::merge_device(xs, ctx->xrecv.as<uint8_t>(), nshards, stride, rq, fb.data(), ctx->xscratch.as<uint8_t>(),
                         ctx->xscratch.cap, ctx->h_xf, out);
  if (hipStreamSynchronize(xs) != hipSuccess && !rc) rc = GBGPU_EHIP;
  return rc;
}

// One exchange of full replies, admitted by the sequencer.  Three
// collectives, so no rank is left waiting whatever fails: the heads (fixed
// size), then every rank's verdict on the buffers the largest pack needs
// (a min all-reduce), then the packs at that size.
static int allgather_replies_admitted(gbgpu_ctx *ctx, const gbx::XFReq &rq, const gbgpu_reply *mine, int err,
                                      gbgpu_merged *out) {
  std::lock_guard<std::mutex> xg(ctx->x_mu);
  if (!ctx->comm) return EINVAL;
  (void)hipSetDevice(ctx->device);
  hipStream_t xs = ctx->xstream;
  const int nr = ctx->nranks;
  const size_t mb = std::max(err ? sizeof(gbx::XFHead) : gbx::pack_bytes(mine), sizeof(gbx::XFHead));
  std::vector<uint8_t> pk(mb, 0);
  gbx::pack_reply(err ? nullptr : mine, rq.nqt, pk.data());
  int rc = 0;
  int32_t ok = 1;
  size_t stride = 256;
  std::vector<int32_t> fb(nr, 0);
  // the flags go through the small result buffer (xout, sized at
  // gbgpu_comm_init and never reallocated): a rank whose pack buffers
  // could not grow still takes part in every collective
  uint8_t *dflag = ctx->xout.as<uint8_t>();
  uint8_t *dflags = dflag + 256;
  static_assert(256 + 4 * 64 <= sizeof(XHead) + 16 * (size_t)XMAX, "flags fit xout");
  // 1: the heads (the send and receive buffers hold at least XMAX records
  // since gbgpu_comm_init, so this never allocates), staged through the
  // pinned result buffer
  uint8_t *hx = ctx->h_xout;
  std::memcpy(hx, pk.data(), sizeof(gbx::XFHead));
  if (hipMemcpyAsync(ctx->xsend.p, hx, sizeof(gbx::XFHead), hipMemcpyHostToDevice, xs) != hipSuccess) rc = GBGPU_EHIP;
  if (ncclAllGather(ctx->xsend.p, ctx->xrecv.p, sizeof(gbx::XFHead), ncclUint8, ctx->comm, xs) != ncclSuccess) rc = GBGPU_EHIP;
  if (hipMemcpyAsync(hx, ctx->xrecv.p, sizeof(gbx::XFHead) * nr, hipMemcpyDeviceToHost, xs) != hipSuccess ||
      hipStreamSynchronize(xs) != hipSuccess)
    rc = GBGPU_EHIP;
  if (!rc) {
    for (int r = 0; r < nr; r++) {
      gbx::XFHead h;
      std::memcpy(&h, hx + sizeof h * r, sizeof h);
      if (h.empty) continue;
      gbgpu_reply x;
      std::memset(&x, 0, sizeof x);
      x.n = h.n;
      x.nqt = h.nqt;
      x.facet_list_size = h.facet_bytes;
      const size_t b = gbx::pack_bytes(&x);
      if (!b) {
        rc = GBGPU_ECORRUPT;
        break;
      }
      stride = std::max(stride, align256(b));
      fb[r] = h.facet_bytes;
    }
  }
  // 2: every rank can hold the packs and the merge's scratch (an all-gather
  // of the verdicts)
  const size_t sb = rc ? 0 : gbx::merge_scratch_bytes(nr, fb.data());
  if (rc || !sb || pk.size() > stride || ctx->xsend.ensure(stride) || ctx->xrecv.ensure(stride * nr) ||
      ctx->xscratch.ensure(sb) || ctx->ensure_h_xf(std::max(stride, gbx::merge_stage_bytes())))
    ok = 0;
  std::memcpy(hx, &ok, 4);
  if (hipMemcpyAsync(dflag, hx, 4, hipMemcpyHostToDevice, xs) != hipSuccess) rc = rc ? rc : GBGPU_EHIP;
  if (ncclAllGather(dflag, dflags, 4, ncclUint8, ctx->comm, xs) != ncclSuccess) rc = rc ? rc : GBGPU_EHIP;
  if (hipMemcpyAsync(hx, dflags, 4 * (size_t)nr, hipMemcpyDeviceToHost, xs) != hipSuccess ||
      hipStreamSynchronize(xs) != hipSuccess)
    rc = rc ? rc : GBGPU_EHIP;
  if (rc) return rc;
  for (int r = 0; r < nr; r++) {
    int32_t f;
    std::memcpy(&f, hx + 4 * r, 4);
    if (!f) return ENOMEM;
  }
  // 3: the packs
  std::memcpy(ctx->h_xf, pk.data(), pk.size());
  if (hipMemcpyAsync(ctx->xsend.p, ctx->h_xf, pk.size(), hipMemcpyHostToDevice, xs) != hipSuccess) rc = GBGPU_EHIP;
  if (ncclAllGather(ctx->xsend.p, ctx->xrecv.p, stride, ncclUint8, ctx->comm, xs) != ncclSuccess) rc = GBGPU_EHIP;
  if (hipStreamSynchronize(xs) != hipSuccess) rc = GBGPU_EHIP;
  if (!rc)
    rc = gbx::merge_device(xs, ctx->xrecv.as<uint8_t>(), nr, stride, rq, fb.data(), ctx->xscratch.as<uint8_t>(),
                           ctx->xscratch.cap, ctx->h_xf, out);
  if (hipStreamSynchronize(xs) != hipSuccess && !rc) rc = GBGPU_EHIP;
  if (err) return err;
  return rc;
}

int gbgpu_allgather_replies(gbgpu_ctx *ctx, uint64_t seq, int timeout_ms, const gbgpu_merge_req *req,
                            const gbgpu_reply *mine, gbgpu_merged *out) {
  gbx::XFReq rq;
  if (!ctx || !out || gbx::make_req(req, &rq) || (uint32_t)req->docs_to_get > gbx::XFMAX) return EINVAL;
  // a reply this rank cannot pack still takes part, as an empty one
  int err = 0;
  if (mine && (!gbx::pack_bytes(mine) || mine->nqt != req->nqt ||
               (req->site_clustering && mine->n > 0 && !mine->cluster_recs) ||
               (mine->n > 0 && (!mine->docids || !mine->scores))))
    err = EINVAL;
  int rc = seq_enter(&ctx->xseq, seq, timeout_ms);
  if (rc) return rc;
  rc = allgather_replies_admitted(ctx, rq, mine, err, out);
  seq_leave(&ctx->xseq, seq);
  return rc;
}

static gbmerge::MergeState *merge_state(gbgpu_ctx *ctx) {
  std::lock_guard<std::mutex> g(ctx->merge_mu);
  if (!ctx->merge && gbmerge::state_new(&ctx->merge) != 0) ctx->merge = nullptr;
  return ctx->merge;
}

int gbgpu_merge_posdb(gbgpu_ctx *ctx, const gbgpu_list *lists, int n, int remove_neg_keys, int64_t min_rec_sizes,
                      uint8_t *out, int64_t out_cap, int64_t *out_size) {
  if (!ctx || !out_size || n < 0 || (n > 0 && !lists) || (out_cap > 0 && !out)) return EINVAL;
  *out_size = 0;
  (void)hipSetDevice(ctx->device);
  gbmerge::MergeState *m = merge_state(ctx);
  if (!m) return GBGPU_EHIP;
  std::vector<const uint8_t *> p(n);
  std::vector<int64_t> sz(n);
  for (int i = 0; i < n; i++) {
    p[i] = lists[i].bytes;
    sz[i] = lists[i].bytes ? lists[i].size : 0;
  }
  return gbmerge::merge_host(m, p.data(), sz.data(), n, remove_neg_keys, min_rec_sizes, out, out_cap, out_size);
}

int gbgpu_merge_posdb_device(gbgpu_ctx *ctx, const uint8_t *const *dev_lists, const int64_t *sizes, int n,
                             int remove_neg_keys, int64_t min_rec_sizes, uint8_t *dev_out, int64_t out_cap,
                             int64_t *out_size) {
  if (!ctx || !out_size) return EINVAL;
  *out_size = 0;
  (void)hipSetDevice(ctx->device);
  gbmerge::MergeState *m = merge_state(ctx);
  if (!m) return GBGPU_EHIP;
  return gbmerge::merge_device(m, dev_lists, sizes, n, remove_neg_keys, min_rec_sizes, dev_out, out_cap, out_size);
}

int gbgpu_merge_last_key(gbgpu_ctx *ctx, uint8_t *key18) {
  if (!ctx || !key18) return EINVAL;
  gbmerge::MergeState *m = merge_state(ctx);
  if (!m) return GBGPU_EHIP;
  return gbmerge::last_key(m, key18);
}

int gbgpu_merge_input_left(gbgpu_ctx *ctx, int32_t *left) {
  if (!ctx || !left) return EINVAL;
  gbmerge::MergeState *m = merge_state(ctx);
  if (!m) return GBGPU_EHIP;
  *left = 0;
  const int rc = gbmerge::last_key(m, nullptr, left);
  return rc == ENOENT ? 0 : rc;
}

int gbgpu_merge_timings(gbgpu_ctx *ctx, float *ms6, int64_t *nkeys, int64_t *ntiles) {
  if (!ctx) return EINVAL;
  gbmerge::MergeState *m = merge_state(ctx);
  if (!m) return GBGPU_EHIP;
  gbmerge::last_timings(m, ms6, nkeys, ntiles);
  return 0;
}

int gbgpu_merge_path(gbgpu_ctx *ctx) {
  if (!ctx) return -EINVAL;
  gbmerge::MergeState *m = merge_state(ctx);
  if (!m) return -GBGPU_EHIP;
  return gbmerge::last_path(m);
}

}  // extern "C"
