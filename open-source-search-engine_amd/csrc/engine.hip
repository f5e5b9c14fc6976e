// gbgpu engine: MI355X (gfx950) kernels for PosdbTable::intersectLists10_r
// and the C-ABI around them (include/gbgpu.h).
//
// Per query, with every list resident in HBM (first key swapped to 12 bytes
// at upload, Posdb.cpp:5671-5703), the stream runs:
//
//   k_count_runs / k_scan_runs / k_write_runs
//        candidate docids = run starts of the sublists of the smallest group
//        (addDocIdVotes group 0, Posdb.cpp:5178-5332), one sorted array per
//        sublist; sublist 0's own locations and group bits are recorded here.
//   k_probe
//        merge-path scan of every other list (and the remaining smallest-group
//        sublists): each block owns a contiguous span of one list, stages
//        12 KiB chunks in LDS, classifies every 6-byte unit by the alignment
//        bit, and matches each docid run against a sliding LDS window of the
//        candidate array (addDocIdVotes g>0 / rmDocIdVotes, Posdb.cpp:5086-
//        5171, 4871-4946).  Matches OR the list's group bits into the
//        candidate's mask and record the run location.
//   k_compact
//        survivors = candidates holding every positive group bit and no
//        negative bit (the final m_docIdVoteBuf); per-list "shrunk sublist is
//        non-empty" flags (shrinkSubLists, Posdb.cpp:5334-5428).
//   k_score
//        one lane per survivor: mini-merge (Posdb.cpp:6559-6778) into scratch
//        records, then the scorers of scoring.h.
//   k_topk_tile (x stages)
//        LDS bitonic selection replacing TopTree (score desc, docid asc).
//
// No host synchronisation happens between kernels: counts live in device
// memory and grids are sized from host-known upper bounds.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "../../include/gbgpu.h"
#include "plan.h"
#include "posdb_key.h"
#include "scoring.h"

namespace gbgpu {

constexpr int BLOCK = 256;
constexpr int UPT = 8;                           // units per thread
constexpr int CHUNK_UNITS = BLOCK * UPT;         // 2048 units = 12 KiB per chunk
constexpr int CHUNK_BYTES = CHUNK_UNITS * 6;
constexpr int CHUNK_LOAD = CHUNK_BYTES + 16;     // + the tail of a 12-byte key
constexpr int CHUNKS_PER_PROBE_BLOCK = 8;        // merge-path span of one block
constexpr int WIN = 256;                         // candidate window (LDS)
constexpr int TILE = 2048;                       // top-k tile
constexpr int LIST_PAD = CHUNK_LOAD + 128;

struct Counters {
  uint32_t nsurv;
  uint32_t corrupt;
  unsigned long long scratch_top;
  uint32_t g0count[MAXG0];
  uint32_t anysurv[MAXL];
  uint32_t topk_n[8];
};

struct G0Chunk {
  uint32_t array;  // candidate array index
  uint32_t u0;     // first unit
};
struct ProbeWork {
  uint32_t list;
  uint32_t u0, u1;
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
__device__ __forceinline__ uint64_t unit_docid(const uint8_t *k) {  // Posdb.h:295
  uint64_t d = (uint64_t)k[11];
  d = (d << 32) | ((uint32_t)k[7] | ((uint32_t)k[8] << 8) | ((uint32_t)k[9] << 16) | ((uint32_t)k[10] << 24));
  return d >> 2;
}

// Stage CHUNK_LOAD bytes of a list (16-B aligned, zero padded) into LDS.
__device__ __forceinline__ void load_chunk(const uint8_t *list, uint32_t u0, uint8_t *lds) {
  const uint4 *src = reinterpret_cast<const uint4 *>(list + (size_t)u0 * 6);
  uint4 *dst = reinterpret_cast<uint4 *>(lds);
  for (int i = threadIdx.x; i < CHUNK_LOAD / 16; i += BLOCK) dst[i] = src[i];
}

// run-start bitmask of this thread's UPT units (Posdb.h:887-889 classifier)
__device__ __forceinline__ uint32_t thread_starts(const uint8_t *lds, uint32_t u0, uint32_t units) {
  uint32_t m = 0;
#pragma unroll
  for (int q = 0; q < UPT; q++) {
    uint32_t lu = threadIdx.x * UPT + q;
    const uint8_t *k = lds + lu * 6;
    if (u0 + lu < units && (k[1] & 0x02) && !(k[0] & 0x04)) m |= 1u << q;
  }
  return m;
}

__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t v, uint32_t *tmp, uint32_t *total) {
  // tmp: BLOCK/64 words of LDS
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
  for (int w = 0; w < BLOCK / 64; w++) {
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

// ----------------------------------------------- candidate extraction (G0)
__global__ void __launch_bounds__(BLOCK) k_count_runs(const DevPlan *pl, const G0Chunk *chunks,
                                                      uint32_t *chunk_count) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[CHUNK_LOAD];
  __shared__ uint32_t tmp[BLOCK / 64];
  const G0Chunk c = chunks[blockIdx.x];
  const DevList &L = pl->lists[pl->g0list[c.array]];
  load_chunk(L.p, c.u0, lds);
  __syncthreads();
  uint32_t m = thread_starts(lds, c.u0, L.units);
  uint32_t tot;
  block_exclusive_scan(__popc(m), tmp, &tot);
  if (threadIdx.x == 0) chunk_count[blockIdx.x] = tot;
}

// exclusive scan of per-chunk counts, per candidate array (single block)
__global__ void __launch_bounds__(1024) k_scan_runs(const G0Chunk *chunks, uint32_t nchunks,
                                                    uint32_t *chunk_count, Counters *ctr) {
  __shared__ uint32_t tmp[16];
  __shared__ uint32_t carry;
  __shared__ uint32_t carry_array;
  if (threadIdx.x == 0) { carry = 0; carry_array = 0; }
  __syncthreads();
  for (uint32_t base = 0; base < nchunks; base += 1024) {
    uint32_t i = base + threadIdx.x;
    uint32_t v = i < nchunks ? chunk_count[i] : 0;
    uint32_t arr = i < nchunks ? chunks[i].array : 0xffffffffu;
    // segmented by array: chunks are grouped by array in order; handle the
    // segment start by subtracting the array's running base on the host side
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint32_t x = v;
    for (int o = 1; o < 64; o <<= 1) {
      uint32_t y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    if (lane == 63) tmp[wid] = x;
    __syncthreads();
    uint32_t pre = 0;
    for (int w = 0; w < wid; w++) pre += tmp[w];
    uint32_t incl = carry + pre + x;
    __syncthreads();
    if (i < nchunks) chunk_count[i] = incl - v;  // global exclusive prefix
    if (threadIdx.x == 1023) carry = incl;
    (void)arr;
    __syncthreads();
  }
  (void)carry_array;
  (void)ctr;
}

__global__ void __launch_bounds__(BLOCK) k_write_runs(const DevPlan *pl, const G0Chunk *chunks,
                                                      const uint32_t *chunk_off,
                                                      const uint32_t *array_first_chunk,
                                                      uint64_t *cand, uint32_t *mask, uint32_t *loc,
                                                      uint64_t slot_ub, Counters *ctr,
                                                      uint32_t nchunks) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[CHUNK_LOAD];
  __shared__ uint32_t tmp[BLOCK / 64];
  const G0Chunk c = chunks[blockIdx.x];
  const int lid = pl->g0list[c.array];
  const DevList &L = pl->lists[lid];
  load_chunk(L.p, c.u0, lds);
  __syncthreads();
  uint32_t m = thread_starts(lds, c.u0, L.units);
  uint32_t tot;
  uint32_t ex = block_exclusive_scan(__popc(m), tmp, &tot);
  // offset inside this array = global prefix - prefix at the array's first chunk
  const uint32_t arr_base_off = chunk_off[array_first_chunk[c.array]];
  uint32_t pos = chunk_off[blockIdx.x] - arr_base_off + ex;
  const uint64_t base = pl->g0base[c.array];
  const bool own = (c.array == 0);  // array 0 is never probed: record it here
  while (m) {
    int q = __ffs(m) - 1;
    m &= m - 1;
    uint32_t lu = threadIdx.x * UPT + q;
    uint64_t d = unit_docid(lds + lu * 6);
    uint64_t slot = base + pos;
    cand[slot] = d;
    if (own) {
      loc[(uint64_t)lid * slot_ub + slot] = c.u0 + lu;
      mask[slot] = L.group_bits;
    }
    pos++;
  }
  // the last chunk of each array publishes the array's count
  bool last = (blockIdx.x + 1 == nchunks) || (chunks[blockIdx.x + 1].array != c.array);
  if (last && threadIdx.x == 0) ctr->g0count[c.array] = chunk_off[blockIdx.x] - arr_base_off + tot;
}

// ------------------------------------------------------------- probe scan
// Per-thread view of its UPT=8 units: 64 bytes read from the LDS chunk with
// four conflict-free ds_read_b128 (thread t at byte 48t: dword 12t mod 64
// tiles all 64 banks over 16 lanes), so classification and docid extraction
// run from registers.  Bytes 48..63 belong to the next thread and supply the
// docid bytes of a 12-byte key starting at the last unit.
struct UnitRegs {
  uint32_t w[16];
  __device__ __forceinline__ uint32_t byte(int i) const { return (w[i >> 2] >> ((i & 3) * 8)) & 0xff; }
};

__device__ __forceinline__ void load_units(const uint8_t *lds, UnitRegs &r) {
  const uint4 *p = reinterpret_cast<const uint4 *>(lds + threadIdx.x * 48);
#pragma unroll
  for (int i = 0; i < 4; i++) {
    uint4 v = p[i];
    r.w[4 * i] = v.x;
    r.w[4 * i + 1] = v.y;
    r.w[4 * i + 2] = v.z;
    r.w[4 * i + 3] = v.w;
  }
}

// docid of a key starting at unit q of this thread (bytes 6q+7 .. 6q+11)
__device__ __forceinline__ uint64_t regs_docid(const UnitRegs &r, int q) {
  const int b = 6 * q + 7;
  uint64_t d = 0;
#pragma unroll
  for (int i = 4; i >= 0; i--) d = (d << 8) | r.byte(b + i);
  return d >> 2;
}

__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    uint64_t y = __shfl_xor(v, o, 64);
    v = y < v ? y : v;
  }
  return v;
}
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    uint64_t y = __shfl_xor(v, o, 64);
    v = y > v ? y : v;
  }
  return v;
}

// MODE (diagnostic builds only, GBGPU_PROBE_MODE): 0 full, 1 stop after the
// unit classification, 2 stop after staging the chunk in LDS.
template <int MODE>
__global__ void __launch_bounds__(BLOCK) k_probe(const DevPlan *pl, const ProbeWork *work,
                                                 const uint64_t *cand, uint32_t *mask, uint32_t *loc,
                                                 uint64_t slot_ub, const Counters *ctr) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[CHUNK_LOAD + 32];
  __shared__ uint64_t win[WIN];
  __shared__ uint32_t s_lo[MAXG0];
  __shared__ uint64_t s_red[2][BLOCK / 64];
  const ProbeWork w = work[blockIdx.x];
  const DevList &L = pl->lists[w.list];
  const uint32_t bits = L.group_bits;
  const int g0n = pl->g0n;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  bool first_chunk = true;
  for (uint32_t u0 = w.u0; u0 < w.u1; u0 += CHUNK_UNITS) {
    load_chunk(L.p, u0, lds);
    __syncthreads();
    if (MODE == 2) {
      if (lds[threadIdx.x * 48] == 0xee && lds[threadIdx.x * 48 + 1] == 0x77) mask[0] = 1;
      __syncthreads();
      continue;
    }
    UnitRegs r;
    load_units(lds, r);
    uint32_t starts = 0;
    uint64_t dk[UPT];
    uint64_t tmin = ~0ull, tmax = 0;
#pragma unroll
    for (int q = 0; q < UPT; q++) {
      const uint32_t gu = u0 + threadIdx.x * UPT + q;
      const bool st = gu < w.u1 && (r.byte(6 * q + 1) & 0x02) && !(r.byte(6 * q) & 0x04);
      dk[q] = st ? regs_docid(r, q) : 0;
      if (st) {
        starts |= 1u << q;
        tmin = dk[q] < tmin ? dk[q] : tmin;
        tmax = dk[q] > tmax ? dk[q] : tmax;
      }
    }
    tmin = wave_min_u64(tmin);
    tmax = wave_max_u64(tmax);
    if (lane == 0) {
      s_red[0][wid] = tmin;
      s_red[1][wid] = tmax;
    }
    __syncthreads();
    uint64_t dmin = s_red[0][0], dmax = s_red[1][0];
#pragma unroll
    for (int i = 1; i < BLOCK / 64; i++) {
      dmin = s_red[0][i] < dmin ? s_red[0][i] : dmin;
      dmax = s_red[1][i] > dmax ? s_red[1][i] : dmax;
    }
    if (dmin == ~0ull || MODE == 1) {  // no run starts in this chunk
      if (MODE == 1 && dk[0] == 0x123456789ull) mask[0] = 1;
      __syncthreads();
      continue;
    }
    uint32_t found = 0;
    for (int k = 0; k < g0n; k++) {
      const uint32_t nk = ctr->g0count[k];
      const uint64_t *ck = cand + pl->g0base[k];
      if (first_chunk) {
        uint32_t lo0 = block_lower_bound(ck, nk, dmin);
        if (threadIdx.x == 0) s_lo[k] = lo0;
        __syncthreads();
      }
      const uint32_t lo = s_lo[k];
      const uint32_t wc = (nk > lo) ? min((uint32_t)WIN, nk - lo) : 0u;
      if (threadIdx.x < wc) win[threadIdx.x] = ck[lo + threadIdx.x];
      __syncthreads();
      const bool covered = (lo + wc >= nk) || (win[wc - 1] >= dmax);
      uint32_t hi;  // one past the last candidate <= dmax
      if (covered) {
        uint32_t a = 0, b = wc;
        while (a < b) {
          uint32_t mid = (a + b) >> 1;
          if (win[mid] <= dmax) a = mid + 1;
          else b = mid;
        }
        hi = lo + a;
      } else {
        hi = lo + block_lower_bound(ck + lo, nk - lo, dmax + 1);
      }
#pragma unroll
      for (int q = 0; q < UPT; q++) {
        if (!((starts & ~found) >> q & 1)) continue;
        const uint64_t d = dk[q];
        uint32_t a, b;
        bool hit;
        if (covered) {
          a = 0;
          b = hi - lo;
          while (a < b) {
            uint32_t mid = (a + b) >> 1;
            if (win[mid] < d) a = mid + 1;
            else b = mid;
          }
          hit = (a < hi - lo) && win[a] == d;
        } else {
          a = lo;
          b = hi;
          while (a < b) {
            uint32_t mid = (a + b) >> 1;
            if (ck[mid] < d) a = mid + 1;
            else b = mid;
          }
          hit = (a < hi) && ck[a] == d;
          a -= lo;
        }
        if (hit) {
          const uint64_t slot = pl->g0base[k] + lo + a;
          found |= 1u << q;
          loc[(uint64_t)w.list * slot_ub + slot] = u0 + threadIdx.x * UPT + q;
          atomicOr(&mask[slot], bits);
        }
      }
      __syncthreads();
      if (threadIdx.x == 0) s_lo[k] = hi;  // next chunk's docids are > dmax
      __syncthreads();
    }
    first_chunk = false;
  }
}

// ------------------------------------------------------------- compaction
__device__ __forceinline__ uint32_t run_units(const uint8_t *p, uint32_t units, uint32_t u) {
  // a docid run: 12-byte key (2 units) then 6-byte keys (Posdb.cpp:5141-5145)
  uint32_t e = u + 2;
  while (e < units && (p[(size_t)e * 6] & 0x04)) e++;
  return e - u;
}

__device__ __forceinline__ bool valid_run(const DevList &L, uint32_t u, uint64_t docid) {
  if (u >= L.units) return false;
  const uint8_t *k = L.p + (size_t)u * 6;
  if (!((k[1] & 0x02) && !(k[0] & 0x04))) return false;
  if (u + 1 >= L.units) return false;
  return unit_docid(k) == docid;
}

constexpr int CSPT = 16;                        // compaction slots per thread
constexpr int CTILE = BLOCK * CSPT;              // 4096 slots per block

// Survivors of one contiguous tile of candidate slots, appended with ONE
// pair of atomics per block (a single device counter cannot take one atomic
// per wave: MI355X_MICROARCH.md "dequeue" row, ~88 per us per word).
__global__ void __launch_bounds__(BLOCK) k_compact(const DevPlan *pl, const uint64_t *cand,
                                                   const uint32_t *mask, const uint32_t *loc,
                                                   uint64_t slot_ub, Counters *ctr, uint32_t *surv,
                                                   unsigned long long *surv_off) {
  __shared__ uint32_t tmp[BLOCK / 64];
  __shared__ uint32_t s_base_i;
  __shared__ unsigned long long s_base_u;
  const uint32_t pos = pl->pos_mask;
  const uint64_t s0 = (uint64_t)blockIdx.x * CTILE + (uint64_t)threadIdx.x * CSPT;
  uint32_t okm = 0, nok = 0, utot = 0;
  uint32_t units[CSPT];
#pragma unroll
  for (int q = 0; q < CSPT; q++) {
    const uint64_t s = s0 + q;
    units[q] = 0;
    if (s >= slot_ub) continue;
    int k = 0;
    while (k + 1 < pl->g0n && s >= pl->g0base[k + 1]) k++;
    if (s - pl->g0base[k] >= ctr->g0count[k]) continue;
    const uint32_t m = mask[s];
    if (!(((m & pos) == pos) && !(m & NEG_BIT))) continue;
    const uint64_t d = cand[s];
    uint32_t u_s = 0;
    for (int j = 0; j < pl->ngroups; j++) {
      if (pl->gflags0[j] & BF_NEGATIVE) continue;
      for (int x = 0; x < pl->gnsub[j]; x++) {
        const int lid = pl->gsub[j][x];
        const DevList &L = pl->lists[lid];
        const uint32_t u = loc[(uint64_t)lid * slot_ub + s];
        if (!valid_run(L, u, d)) continue;
        u_s += run_units(L.p, L.units, u);
        if (!ctr->anysurv[lid]) atomicOr((uint32_t *)&ctr->anysurv[lid], 1u);
      }
    }
    units[q] = u_s;
    okm |= 1u << q;
    nok++;
    utot += u_s;
  }
  uint32_t tot_n, tot_u;
  const uint32_t ex_n = block_exclusive_scan(nok, tmp, &tot_n);
  const uint32_t ex_u = block_exclusive_scan(utot, tmp, &tot_u);
  if (threadIdx.x == 0) {
    s_base_i = tot_n ? atomicAdd(&ctr->nsurv, tot_n) : 0;
    s_base_u = tot_n ? atomicAdd(&ctr->scratch_top, (unsigned long long)tot_u) : 0;
  }
  __syncthreads();
  uint32_t i = s_base_i + ex_n;
  unsigned long long off = s_base_u + ex_u;
#pragma unroll
  for (int q = 0; q < CSPT; q++) {
    if (!(okm >> q & 1)) continue;
    surv[i] = (uint32_t)(s0 + q);
    surv_off[i] = off;
    i++;
    off += units[q];
  }
}

// ------------------------------------------------------------------ score
__constant__ Weights c_weights;

struct MCur {
  const uint8_t *p;
  uint32_t u, end;
  uint8_t flags;
  bool first;
  bool live;
};

__device__ __forceinline__ uint64_t load6(const uint8_t *k) {
  const uint16_t *h = reinterpret_cast<const uint16_t *>(k);
  return (uint64_t)h[0] | ((uint64_t)h[1] << 16) | ((uint64_t)h[2] << 32);
}

__global__ void __launch_bounds__(BLOCK) k_score(const DevPlan *pl, const uint64_t *cand,
                                                 const uint32_t *loc, uint64_t slot_ub,
                                                 const Counters *ctr, const uint32_t *surv,
                                                 const unsigned long long *surv_off,
                                                 uint64_t *scratch, uint32_t *skey,
                                                 uint64_t *sdoc) {
  const uint32_t nsurv = ctr->nsurv;
  for (uint32_t i = blockIdx.x * BLOCK + threadIdx.x; i < nsurv; i += gridDim.x * BLOCK) {
    const uint32_t s = surv[i];
    const uint64_t docid = cand[s];
    uint64_t *rec = scratch + surv_off[i];
    DocView dv;
    dv.rec = rec;
    int nrec = 0;
    uint32_t mbytes = 0;  // emulates mptr - mbuf (cap 299000, Posdb.cpp:6007-6008)
    bool empty_pos = false;
    int siteRank = -1, docLang = 0;
    for (int j = 0; j < pl->ngroups; j++) {
      dv.beg[j] = dv.end[j] = nrec;
      if (pl->gflags0[j] & BF_NEGATIVE) {
        dv.present[j] = false;
        continue;
      }
      dv.present[j] = true;
      MCur cur[MAXSUB];
      int nsub = 0, newIdx = 0;
      for (int x = 0; x < pl->gnsub[j]; x++) {
        const int lid = pl->gsub[j][x];
        if (!ctr->anysurv[lid]) continue;  // shrunk to empty: not a new sublist
        const uint8_t fl = pl->gsubflags[j][newIdx];  // m_bigramFlags[new index]
        newIdx++;
        const DevList &L = pl->lists[lid];
        const uint32_t u = loc[(uint64_t)lid * slot_ub + s];
        if (!valid_run(L, u, docid)) continue;
        MCur &c = cur[nsub++];
        c.p = L.p;
        c.u = u;
        c.end = u + run_units(L.p, L.units, u);
        c.flags = fl;
        c.first = true;
        c.live = true;
      }
      bool isFirstKey = true;
      uint64_t last = 0;
      const uint8_t *firstSrc = nullptr;
      for (;;) {
        int mink = -1;
        uint32_t mhi = 0, mlo = 0;
        for (int k = 0; k < nsub; k++) {
          if (!cur[k].live) continue;
          const uint8_t *kp = cur[k].p + (size_t)cur[k].u * 6;
          const uint32_t hi = gb_u32(kp + 2), lo = gb_u16(kp);
          if (mink == -1) { mink = k; mhi = hi; mlo = lo; continue; }
          if (hi > mhi) continue;
          if (hi == mhi && lo >= mlo) continue;
          mink = k; mhi = hi; mlo = lo;
        }
        if (mink == -1) break;
        MCur &c = cur[mink];
        const uint8_t *src = c.p + (size_t)c.u * 6;
        const bool hack = (c.flags & BF_BIGRAM) && (src[2] & 0x03);  // Posdb.cpp:6687-6692
        if (!hack) {
          uint64_t r = load6(src);
          uint64_t b2 = (r >> 16) & 0xfc;
          if (c.flags & (BF_BIGRAM | BF_SYNONYM)) b2 |= 0x02;
          if (c.flags & BF_HALFSTOPWIKIBIGRAM) b2 |= 0x01;
          r = (r & ~(0xffull << 16)) | (b2 << 16);
          if (isFirstKey) {
            r = (r & ~0xffull) | (((r & 0xff) & 0xf9) | 0x02);
            rec[nrec++] = r;
            last = r;
            mbytes += 12;
            isFirstKey = false;
            firstSrc = src;
          } else {
            const bool dup = (((last >> 32) & 0xffff) == ((r >> 32) & 0xffff)) &&
                             (((last >> 24) & 0xc0) == ((r >> 24) & 0xc0));
            if (!dup) {
              r |= 0x06;
              rec[nrec++] = r;
              last = r;
              mbytes += 6;
            }
          }
        }
        c.u += c.first ? 2 : 1;
        c.first = false;
        if (c.u >= c.end) c.live = false;
        if (mbytes >= 299000) break;
      }
      dv.end[j] = nrec;
      if (nrec == dv.beg[j]) empty_pos = true;  // reference reads stale mbuf here (UB)
      if (siteRank < 0 && firstSrc && !(pl->gflags0[j] & (BF_NUMBER | BF_FACET))) {
        // Posdb.cpp:6985-7003: group 0 if present, else first present k >= 1
        siteRank = gb_siterank(firstSrc);
        docLang = (int)gb_langid(firstSrc);
      }
    }
    float score = 0.0f;
    bool ok = !empty_pos && score_doc(&c_weights, pl, dv, siteRank < 0 ? 0 : siteRank, docLang, &score);
    uint32_t key = 0;
    if (ok) {
      const uint32_t b = __float_as_uint(score);
      key = (b & 0x80000000u) ? ~b : (b | 0x80000000u);
      if (key == 0) key = 1;
    }
    skey[i] = key;
    sdoc[i] = docid;
  }
}

// ------------------------------------------------------------------ top-k
// Each block sorts one tile of up to TILE (key, docid) pairs in LDS by
// (key desc, docid asc) and writes its best k.  Invalid entries have key 0.
__global__ void __launch_bounds__(1024) k_topk_tile(const uint32_t *in_key, const uint64_t *in_doc,
                                                    const uint32_t *n_in_ptr, uint32_t n_in_const,
                                                    uint32_t *out_key, uint64_t *out_doc,
                                                    uint32_t *n_out_ptr, int k) {
  __shared__ uint32_t sk[TILE];
  __shared__ uint64_t sd[TILE];
  const uint32_t n_in = n_in_ptr ? *n_in_ptr : n_in_const;
  const uint64_t base = (uint64_t)blockIdx.x * TILE;
  if (blockIdx.x == 0 && threadIdx.x == 0 && n_out_ptr) {
    const uint32_t tiles = (n_in + TILE - 1) / TILE;
    *n_out_ptr = tiles * (uint32_t)k;
  }
  // tiles past the live count exit (grid sized by an upper bound); tile 0
  // always runs so an empty input still yields an all-invalid output
  if (base >= n_in && blockIdx.x != 0) return;
  for (int t = threadIdx.x; t < TILE; t += blockDim.x) {
    const uint64_t g = base + t;
    if (g < n_in) {
      sk[t] = in_key[g];
      sd[t] = in_doc[g];
    } else {
      sk[t] = 0;
      sd[t] = ~0ull;
    }
  }
  __syncthreads();
  // bitonic sort, "greater" = better rank
  for (int size = 2; size <= TILE; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = threadIdx.x; t < TILE / 2; t += blockDim.x) {
        const int i = 2 * t - (t & (stride - 1));
        const int j = i + stride;
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
  const uint64_t obase = (uint64_t)blockIdx.x * k;
  for (int t = threadIdx.x; t < k; t += blockDim.x) {
    out_key[obase + t] = sk[t];
    out_doc[obase + t] = sd[t];
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

struct DevBuf {
  void *p = nullptr;
  size_t cap = 0;
  int ensure(size_t bytes) {
    if (bytes <= cap) return 0;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    size_t want = std::max<size_t>(bytes + bytes / 4, 1 << 16);
    if (hipMalloc(&p, want) != hipSuccess) return ENOMEM;
    cap = want;
    return 0;
  }
  template <class T> T *as() const { return reinterpret_cast<T *>(p); }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

struct ListEntry {
  uint8_t *d = nullptr;
  int64_t size = 0;   // original bytes (18-byte first key)
  uint32_t units = 0; // swapped units
  bool live = false;
};

}  // namespace gbgpu

using namespace gbgpu;

struct gbgpu_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  std::mutex mu;
  std::vector<ListEntry> lists;
  DevBuf plan, counters, g0chunks, chunkcnt, arrfirst, work, cand, mask, loc, surv, survoff, scratch,
      skey, sdoc, tk_key[2], tk_doc[2];
  DevPlan *h_plan = nullptr;   // pinned
  Counters *h_ctr = nullptr;   // pinned
  uint32_t *h_out_key = nullptr;
  uint64_t *h_out_doc = nullptr;
  int out_cap = 0;
  std::vector<G0Chunk> g0c;
  std::vector<ProbeWork> pw;
  std::vector<uint32_t> afirst;
  uint8_t *h_stage = nullptr;  // pinned staging for the per-query tables
  size_t stage_cap = 0;
  // state of the in-flight query
  bool pending = false;
  bool early = false;
  int k = 0;
  int final_buf = 0;
  int32_t docs_wanted = 0;
  int64_t scan_bytes = 0;
  bool profiling = false;
  int probe_mode = 0;  // diagnostic only (GBGPU_PROBE_MODE)
  hipEvent_t ev[7] = {};
  float last_ms[6] = {0, 0, 0, 0, 0, 0};
  // per-query temporary lists (gbgpu_query with host lists)
  std::vector<int32_t> temp_handles;
};

static int upload_list(gbgpu_ctx *ctx, const uint8_t *bytes, int64_t size, int32_t *handle) {
  if (size < 0 || (size > 0 && size < 18) || (size > 0 && (size - 18) % 6 != 0)) return EINVAL;
  if ((size - 6) / 6 > 0xfffffff0LL) return GBGPU_ECAPACITY;
  ListEntry e;
  e.size = size;
  e.units = size ? (uint32_t)((size - 6) / 6) : 0;
  size_t alloc = (size_t)(size ? size - 6 : 0) + LIST_PAD;
  alloc = (alloc + 255) & ~(size_t)255;
  if (hipMalloc(&e.d, alloc) != hipSuccess) return ENOMEM;
  HIPCHECK(hipMemsetAsync(e.d, 0, alloc, ctx->stream));
  if (size) {
    // device image = the list after the first-key swap (Posdb.cpp:5689-5698):
    // original bytes 0..11 with the half bit set, then bytes 18..size-1
    uint8_t first[12];
    std::memcpy(first, bytes, 12);
    first[0] |= 0x02;
    HIPCHECK(hipMemcpyAsync(e.d, first, 12, hipMemcpyHostToDevice, ctx->stream));
    if (size > 18)
      HIPCHECK(hipMemcpyAsync(e.d + 12, bytes + 18, (size_t)(size - 18), hipMemcpyHostToDevice, ctx->stream));
  }
  HIPCHECK(hipStreamSynchronize(ctx->stream));
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

static int enqueue(gbgpu_ctx *ctx, const gbgpu_qterm *terms, int nterms, const int32_t *handles,
                   const gbgpu_params *p) {
  if (!p || nterms < 0 || (nterms && (!terms || !handles))) return EINVAL;
  if (p->site_clustering || p->num_docid_splits > 1) return GBGPU_EUNSUPPORTED;
  if (p->docs_to_get <= 0 || p->real_max_top <= 0) return EINVAL;
  std::vector<int64_t> sizes(nterms);
  for (int i = 0; i < nterms; i++) {
    if (terms[i].field_code) return GBGPU_EUNSUPPORTED;
    int32_t h = handles[i];
    if (h < 0 || h >= (int32_t)ctx->lists.size() || !ctx->lists[h].live) return EINVAL;
    sizes[i] = ctx->lists[h].size;
  }
  HostPlan hp;
  int rc = build_host_plan(terms, nterms, sizes.data(), p, &hp);
  if (rc) return rc;
  ctx->docs_wanted = hp.docs_wanted;
  ctx->k = hp.docs_wanted;
  ctx->pending = true;
  ctx->early = (hp.ngroups == 0 || hp.min_list_size == 0);
  ctx->scan_bytes = 0;
  if (ctx->early) return 0;
  if (hp.ngroups > MAXG) { ctx->pending = false; return GBGPU_EUNSUPPORTED; }
  if (ctx->k > TILE) { ctx->pending = false; return GBGPU_EUNSUPPORTED; }

  DevPlan &P = *ctx->h_plan;
  std::memset(&P, 0, sizeof P);
  P.ngroups = hp.ngroups;
  P.real_max_top = hp.real_max_top;
  P.language = p->language;
  P.same_lang_weight = p->same_lang_weight;
  P.site_rank_multiplier = GB_SITERANKMULTIPLIER;
  P.nqt = nterms;
  int dense[1024];
  std::vector<int> term_of(0);
  if (nterms > 1024) { ctx->pending = false; return GBGPU_EUNSUPPORTED; }
  for (int i = 0; i < nterms; i++) dense[i] = -1;
  auto dense_id = [&](int term) -> int {
    if (dense[term] >= 0) return dense[term];
    if (P.nlists >= MAXL) return -1;
    int id = P.nlists++;
    dense[term] = id;
    term_of.push_back(term);
    const ListEntry &e = ctx->lists[handles[term]];
    P.lists[id].p = e.d;
    P.lists[id].units = e.units;
    P.lists[id].group_bits = 0;
    P.lists[id].g0_array = -1;
    P.lists[id].probe = 0;
    return id;
  };
  for (int j = 0; j < hp.ngroups; j++) {
    const GroupInfo &g = hp.g[j];
    if (g.nsub > MAXSUB) { ctx->pending = false; return GBGPU_EUNSUPPORTED; }
    P.gflags0[j] = g.flags[0];
    P.gnsub[j] = (uint8_t)g.nsub;
    P.tfw[j] = g.tfw;
    P.qpos[j] = g.qpos;
    P.wiki[j] = g.wiki;
    P.quote[j] = g.quote;
    for (int x = 0; x < MAXSUB; x++) P.gsubflags[j][x] = x < 50 ? g.flags[x] : 0;
    const bool neg = (g.flags[0] & BF_NEGATIVE) != 0;
    if (!neg) P.pos_mask |= 1u << j;
    for (int x = 0; x < g.nsub; x++) {
      int id = dense_id(g.sub_term[x]);
      if (id < 0) { ctx->pending = false; return GBGPU_EUNSUPPORTED; }
      P.gsub[j][x] = (uint8_t)id;
      P.lists[id].group_bits |= neg ? NEG_BIT : (1u << j);
    }
  }
  // candidate arrays: distinct lists of the smallest group, in sublist order
  const GroupInfo &g0 = hp.g[hp.min_listi];
  P.g0n = 0;
  uint64_t slot = 0;
  for (int x = 0; x < g0.nsub; x++) {
    int id = dense[g0.sub_term[x]];
    if (P.lists[id].g0_array >= 0) continue;
    if (P.g0n >= MAXG0) { ctx->pending = false; return GBGPU_EUNSUPPORTED; }
    P.lists[id].g0_array = P.g0n;
    P.g0list[P.g0n] = id;
    P.g0base[P.g0n] = slot;
    slot += P.lists[id].units / 2 + 1;
    P.g0n++;
  }
  P.g0base[P.g0n] = slot;
  const uint64_t slot_ub = slot;
  for (int id = 0; id < P.nlists; id++) P.lists[id].probe = (P.lists[id].g0_array != 0);

  // work tables
  ctx->g0c.clear();
  ctx->afirst.assign(MAXG0, 0);
  for (int a = 0; a < P.g0n; a++) {
    ctx->afirst[a] = (uint32_t)ctx->g0c.size();
    const uint32_t units = P.lists[P.g0list[a]].units;
    for (uint32_t u = 0; u < units; u += CHUNK_UNITS) ctx->g0c.push_back({(uint32_t)a, u});
  }
  ctx->pw.clear();
  int64_t scan = 0;
  for (int id = 0; id < P.nlists; id++) {
    const uint32_t units = P.lists[id].units;
    scan += (int64_t)units * 6;
    if (!P.lists[id].probe) continue;
    // long lists: 8 chunks per block amortise the candidate search; short
    // lists: 1 chunk per block so they do not form the kernel's tail
    const uint32_t nch = (units + CHUNK_UNITS - 1) / CHUNK_UNITS;
    const uint32_t cpb = std::max(1u, std::min<uint32_t>(CHUNKS_PER_PROBE_BLOCK, nch / 1024));
    const uint32_t span = CHUNK_UNITS * cpb;
    for (uint32_t u = 0; u < units; u += span) ctx->pw.push_back({(uint32_t)id, u, std::min(units, u + span)});
  }
  ctx->scan_bytes = scan;
  // scratch upper bound: every group instance can use all of its list once
  uint64_t scratch_ub = 1;
  for (int j = 0; j < hp.ngroups; j++) {
    if (P.gflags0[j] & BF_NEGATIVE) continue;
    for (int x = 0; x < P.gnsub[j]; x++) scratch_ub += P.lists[P.gsub[j][x]].units;
  }
  const int k = ctx->k;
  const uint64_t tiles0 = (slot_ub + TILE - 1) / TILE;
  int rc2 = 0;
  rc2 |= ctx->plan.ensure(sizeof(DevPlan));
  rc2 |= ctx->counters.ensure(sizeof(Counters));
  rc2 |= ctx->g0chunks.ensure(sizeof(G0Chunk) * std::max<size_t>(1, ctx->g0c.size()));
  rc2 |= ctx->chunkcnt.ensure(4 * std::max<size_t>(1, ctx->g0c.size()));
  rc2 |= ctx->arrfirst.ensure(4 * MAXG0);
  rc2 |= ctx->work.ensure(sizeof(ProbeWork) * std::max<size_t>(1, ctx->pw.size()));
  rc2 |= ctx->cand.ensure(8 * slot_ub);
  rc2 |= ctx->mask.ensure(4 * slot_ub);
  rc2 |= ctx->loc.ensure(4 * slot_ub * (uint64_t)P.nlists);
  rc2 |= ctx->surv.ensure(4 * slot_ub);
  rc2 |= ctx->survoff.ensure(8 * slot_ub);
  rc2 |= ctx->scratch.ensure(8 * scratch_ub);
  rc2 |= ctx->skey.ensure(4 * slot_ub);
  rc2 |= ctx->sdoc.ensure(8 * slot_ub);
  rc2 |= ctx->tk_key[0].ensure(4 * (tiles0 * k + TILE));
  rc2 |= ctx->tk_doc[0].ensure(8 * (tiles0 * k + TILE));
  rc2 |= ctx->tk_key[1].ensure(4 * (tiles0 * k + TILE));
  rc2 |= ctx->tk_doc[1].ensure(8 * (tiles0 * k + TILE));
  if (rc2) { ctx->pending = false; return ENOMEM; }
  if (ctx->out_cap < k) {
    if (ctx->h_out_key) (void)hipHostFree(ctx->h_out_key);
    if (ctx->h_out_doc) (void)hipHostFree(ctx->h_out_doc);
    HIPCHECK(hipHostMalloc((void **)&ctx->h_out_key, 4 * (size_t)std::max(k, 1)));
    HIPCHECK(hipHostMalloc((void **)&ctx->h_out_doc, 8 * (size_t)std::max(k, 1)));
    ctx->out_cap = std::max(k, 1);
  }
  hipStream_t st = ctx->stream;
  if (ctx->profiling) HIPCHECK(hipEventRecord(ctx->ev[0], st));
  HIPCHECK(hipMemcpyAsync(ctx->plan.p, ctx->h_plan, sizeof(DevPlan), hipMemcpyHostToDevice, st));
  {
    // the tables go through pinned memory: a pageable source makes the copy
    // synchronous with the host and stalls the stream
    const size_t b1 = sizeof(G0Chunk) * ctx->g0c.size(), b2 = 4 * MAXG0, b3 = sizeof(ProbeWork) * ctx->pw.size();
    const size_t need = b1 + b2 + b3 + 64;
    if (need > ctx->stage_cap) {
      if (ctx->h_stage) (void)hipHostFree(ctx->h_stage);
      ctx->h_stage = nullptr;
      ctx->stage_cap = 0;
      HIPCHECK(hipHostMalloc((void **)&ctx->h_stage, need * 2));
      ctx->stage_cap = need * 2;
    }
    std::memcpy(ctx->h_stage, ctx->g0c.data(), b1);
    std::memcpy(ctx->h_stage + b1, ctx->afirst.data(), b2);
    std::memcpy(ctx->h_stage + b1 + b2, ctx->pw.data(), b3);
    if (b1) HIPCHECK(hipMemcpyAsync(ctx->g0chunks.p, ctx->h_stage, b1, hipMemcpyHostToDevice, st));
    HIPCHECK(hipMemcpyAsync(ctx->arrfirst.p, ctx->h_stage + b1, b2, hipMemcpyHostToDevice, st));
    if (b3) HIPCHECK(hipMemcpyAsync(ctx->work.p, ctx->h_stage + b1 + b2, b3, hipMemcpyHostToDevice, st));
  }
  HIPCHECK(hipMemsetAsync(ctx->counters.p, 0, sizeof(Counters), st));
  HIPCHECK(hipMemsetAsync(ctx->mask.p, 0, 4 * slot_ub, st));
  const DevPlan *dpl = ctx->plan.as<DevPlan>();
  Counters *dctr = ctx->counters.as<Counters>();
  const uint32_t ng0 = (uint32_t)ctx->g0c.size();
  if (ng0) {
    hipLaunchKernelGGL(k_count_runs, dim3(ng0), dim3(BLOCK), 0, st, dpl, ctx->g0chunks.as<G0Chunk>(),
                       ctx->chunkcnt.as<uint32_t>());
    hipLaunchKernelGGL(k_scan_runs, dim3(1), dim3(1024), 0, st, ctx->g0chunks.as<G0Chunk>(), ng0,
                       ctx->chunkcnt.as<uint32_t>(), dctr);
    hipLaunchKernelGGL(k_write_runs, dim3(ng0), dim3(BLOCK), 0, st, dpl, ctx->g0chunks.as<G0Chunk>(),
                       ctx->chunkcnt.as<uint32_t>(), ctx->arrfirst.as<uint32_t>(), ctx->cand.as<uint64_t>(),
                       ctx->mask.as<uint32_t>(), ctx->loc.as<uint32_t>(), slot_ub, dctr, ng0);
  }
  if (ctx->profiling) HIPCHECK(hipEventRecord(ctx->ev[1], st));
  if (!ctx->pw.empty()) {
    auto kp = ctx->probe_mode == 1 ? k_probe<1> : (ctx->probe_mode == 2 ? k_probe<2> : k_probe<0>);
    hipLaunchKernelGGL(kp, dim3((uint32_t)ctx->pw.size()), dim3(BLOCK), 0, st, dpl,
                       ctx->work.as<ProbeWork>(), ctx->cand.as<uint64_t>(), ctx->mask.as<uint32_t>(),
                       ctx->loc.as<uint32_t>(), slot_ub, dctr);
  }
  if (ctx->profiling) HIPCHECK(hipEventRecord(ctx->ev[2], st));
  const uint32_t cgrid = (uint32_t)((slot_ub + CTILE - 1) / CTILE);
  hipLaunchKernelGGL(k_compact, dim3(std::max(cgrid, 1u)), dim3(BLOCK), 0, st, dpl, ctx->cand.as<uint64_t>(),
                     ctx->mask.as<uint32_t>(), ctx->loc.as<uint32_t>(), slot_ub, dctr, ctx->surv.as<uint32_t>(),
                     ctx->survoff.as<unsigned long long>());
  if (ctx->profiling) HIPCHECK(hipEventRecord(ctx->ev[3], st));
  const uint32_t sgrid = (uint32_t)std::min<uint64_t>((slot_ub + BLOCK - 1) / BLOCK, 2048);
  hipLaunchKernelGGL(k_score, dim3(std::max(sgrid, 1u)), dim3(BLOCK), 0, st, dpl, ctx->cand.as<uint64_t>(),
                     ctx->loc.as<uint32_t>(), slot_ub, dctr, ctx->surv.as<uint32_t>(),
                     ctx->survoff.as<unsigned long long>(), ctx->scratch.as<uint64_t>(), ctx->skey.as<uint32_t>(),
                     ctx->sdoc.as<uint64_t>());
  if (ctx->profiling) HIPCHECK(hipEventRecord(ctx->ev[4], st));
  // top-k stages: survivors -> tiles -> ... -> one tile
  uint64_t n_ub = slot_ub;
  const uint32_t *in_key = ctx->skey.as<uint32_t>();
  const uint64_t *in_doc = ctx->sdoc.as<uint64_t>();
  const uint32_t *in_n = &dctr->nsurv;
  int buf = 0, stage = 0;
  for (;;) {
    uint64_t tiles = (n_ub + TILE - 1) / TILE;
    if (tiles == 0) tiles = 1;
    uint32_t *ok = ctx->tk_key[buf].as<uint32_t>();
    uint64_t *od = ctx->tk_doc[buf].as<uint64_t>();
    uint32_t *on = &dctr->topk_n[stage & 7];
    hipLaunchKernelGGL(k_topk_tile, dim3((uint32_t)tiles), dim3(1024), 0, st, in_key, in_doc, in_n, 0u, ok, od,
                       on, k);
    ctx->final_buf = buf;
    if (tiles == 1) break;
    n_ub = tiles * (uint64_t)k;
    in_key = ok;
    in_doc = od;
    in_n = on;
    buf ^= 1;
    stage++;
  }
  if (ctx->profiling) HIPCHECK(hipEventRecord(ctx->ev[5], st));
  HIPCHECK(hipMemcpyAsync(ctx->h_out_key, ctx->tk_key[ctx->final_buf].p, 4 * (size_t)k, hipMemcpyDeviceToHost, st));
  HIPCHECK(hipMemcpyAsync(ctx->h_out_doc, ctx->tk_doc[ctx->final_buf].p, 8 * (size_t)k, hipMemcpyDeviceToHost, st));
  HIPCHECK(hipMemcpyAsync(ctx->h_ctr, ctx->counters.p, sizeof(Counters), hipMemcpyDeviceToHost, st));
  if (ctx->profiling) HIPCHECK(hipEventRecord(ctx->ev[6], st));
  return 0;
}

static int collect(gbgpu_ctx *ctx, gbgpu_result *out) {
  if (!ctx->pending) return EINVAL;
  ctx->pending = false;
  out->n = 0;
  out->hits = 0;
  out->filtered = 0;
  out->docs_wanted = ctx->docs_wanted;
  if (ctx->early) return 0;
  HIPCHECK(hipStreamSynchronize(ctx->stream));
  if (ctx->profiling) {
    float t;
    (void)hipEventElapsedTime(&t, ctx->ev[0], ctx->ev[6]);
    ctx->last_ms[0] = t;
    for (int i = 1; i < 6; i++) {
      (void)hipEventElapsedTime(&t, ctx->ev[i - 1], ctx->ev[i]);
      ctx->last_ms[i] = t;
    }
  }
  out->hits = ctx->h_ctr->nsurv;
  int n = 0;
  for (int i = 0; i < ctx->k && n < out->capacity; i++) {
    uint32_t key = ctx->h_out_key[i];
    if (key == 0) break;
    uint32_t b = (key & 0x80000000u) ? (key & 0x7fffffffu) : ~key;
    float f;
    std::memcpy(&f, &b, 4);
    if (out->docids) out->docids[n] = (int64_t)ctx->h_out_doc[i];
    if (out->scores) out->scores[n] = f;
    n++;
  }
  out->n = n;
  return 0;
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

int gbgpu_open(int device, gbgpu_ctx **out) {
  if (!out) return EINVAL;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= device || device < 0) return GBGPU_ENODEVICE;
  if (hipSetDevice(device) != hipSuccess) return GBGPU_ENODEVICE;
  gbgpu_ctx *ctx = new gbgpu_ctx();
  ctx->device = device;
  if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
    delete ctx;
    return GBGPU_EHIP;
  }
  Weights w = host_weights();
  if (hipMemcpyToSymbol(HIP_SYMBOL(c_weights), &w, sizeof w) != hipSuccess) {
    delete ctx;
    return GBGPU_EHIP;
  }
  if (hipHostMalloc((void **)&ctx->h_plan, sizeof(DevPlan)) != hipSuccess ||
      hipHostMalloc((void **)&ctx->h_ctr, sizeof(Counters)) != hipSuccess) {
    delete ctx;
    return ENOMEM;
  }
  for (auto &e : ctx->ev) (void)hipEventCreate(&e);
  if (const char *pm = std::getenv("GBGPU_PROBE_MODE")) ctx->probe_mode = std::atoi(pm);
  *out = ctx;
  return 0;
}

void gbgpu_close(gbgpu_ctx *ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  (void)hipStreamSynchronize(ctx->stream);
  for (auto &e : ctx->lists)
    if (e.live) (void)hipFree(e.d);
  DevBuf *bufs[] = {&ctx->plan, &ctx->counters, &ctx->g0chunks, &ctx->chunkcnt, &ctx->arrfirst, &ctx->work,
                    &ctx->cand, &ctx->mask, &ctx->loc, &ctx->surv, &ctx->survoff, &ctx->scratch, &ctx->skey,
                    &ctx->sdoc, &ctx->tk_key[0], &ctx->tk_doc[0], &ctx->tk_key[1], &ctx->tk_doc[1]};
  for (auto *b : bufs) b->release();
  if (ctx->h_plan) (void)hipHostFree(ctx->h_plan);
  if (ctx->h_ctr) (void)hipHostFree(ctx->h_ctr);
  if (ctx->h_out_key) (void)hipHostFree(ctx->h_out_key);
  if (ctx->h_out_doc) (void)hipHostFree(ctx->h_out_doc);
  if (ctx->h_stage) (void)hipHostFree(ctx->h_stage);
  for (auto &e : ctx->ev)
    if (e) (void)hipEventDestroy(e);
  (void)hipStreamDestroy(ctx->stream);
  delete ctx;
}

int32_t gbgpu_docs_wanted(const gbgpu_params *p, const int64_t *sizes, int nterms) {
  if (!p || (nterms && !sizes)) return 0;
  return docs_wanted(p, sizes, nterms);
}

int gbgpu_list_upload(gbgpu_ctx *ctx, const uint8_t *bytes, int64_t size, int32_t *handle) {
  if (!ctx || !handle || (size > 0 && !bytes)) return EINVAL;
  std::lock_guard<std::mutex> g(ctx->mu);
  (void)hipSetDevice(ctx->device);
  return upload_list(ctx, bytes, size, handle);
}

int gbgpu_list_free(gbgpu_ctx *ctx, int32_t h) {
  if (!ctx) return EINVAL;
  std::lock_guard<std::mutex> g(ctx->mu);
  if (h < 0 || h >= (int32_t)ctx->lists.size() || !ctx->lists[h].live) return EINVAL;
  (void)hipStreamSynchronize(ctx->stream);
  (void)hipFree(ctx->lists[h].d);
  ctx->lists[h] = ListEntry();
  return 0;
}

int gbgpu_query_resident_enqueue(gbgpu_ctx *ctx, const gbgpu_qterm *terms, int nterms, const int32_t *handles,
                                 const gbgpu_params *p) {
  if (!ctx) return EINVAL;
  std::lock_guard<std::mutex> g(ctx->mu);
  (void)hipSetDevice(ctx->device);
  if (ctx->pending) return EBUSY;
  int rc = enqueue(ctx, terms, nterms, handles, p);
  if (rc) ctx->pending = false;
  return rc;
}

int gbgpu_query_collect(gbgpu_ctx *ctx, gbgpu_result *out) {
  if (!ctx || !out) return EINVAL;
  std::lock_guard<std::mutex> g(ctx->mu);
  (void)hipSetDevice(ctx->device);
  return collect(ctx, out);
}

int gbgpu_query_resident(gbgpu_ctx *ctx, const gbgpu_qterm *terms, int nterms, const int32_t *handles,
                         const gbgpu_params *p, gbgpu_result *out) {
  if (!ctx || !out) return EINVAL;
  std::lock_guard<std::mutex> g(ctx->mu);
  (void)hipSetDevice(ctx->device);
  if (ctx->pending) return EBUSY;
  int rc = enqueue(ctx, terms, nterms, handles, p);
  if (rc) {
    ctx->pending = false;
    return rc;
  }
  return collect(ctx, out);
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

void *gbgpu_stream(gbgpu_ctx *ctx) { return ctx ? (void *)ctx->stream : nullptr; }

int gbgpu_last_topk_device(gbgpu_ctx *ctx, void **dev_ptr, int32_t *n) {
  if (!ctx || !dev_ptr || !n) return EINVAL;
  *dev_ptr = ctx->tk_key[ctx->final_buf].p;
  *n = ctx->k;
  return 0;
}

int gbgpu_set_profiling(gbgpu_ctx *ctx, int enable) {
  if (!ctx) return EINVAL;
  ctx->profiling = enable != 0;
  return 0;
}

int gbgpu_last_timings(gbgpu_ctx *ctx, float *ms6, int64_t *scan_bytes) {
  if (!ctx) return EINVAL;
  if (ms6) std::memcpy(ms6, ctx->last_ms, sizeof ctx->last_ms);
  if (scan_bytes) *scan_bytes = ctx->scan_bytes;
  return 0;
}

int gbgpu_merge_topk(const int64_t *const *sd, const float *const *ss, const int32_t *cnt, int nshards, int32_t k,
                     int64_t *od, double *os, int32_t *on) {
  // Msg3a::mergeLists, Msg3a.cpp:1315-1467: repeatedly take the shard head
  // with the max (double) score, ties -> lower docid, skip duplicate docids
  if (!on || nshards < 0 || k < 0) return EINVAL;
  std::vector<int32_t> cur(nshards, 0);
  std::vector<int64_t> seen;
  int32_t n = 0;
  while (n < k) {
    int best = -1;
    double bs = 0;
    int64_t bd = 0;
    for (int s = 0; s < nshards; s++) {
      if (cur[s] >= cnt[s]) continue;
      double sc = (double)ss[s][cur[s]];
      int64_t d = sd[s][cur[s]];
      if (best < 0 || sc > bs || (sc == bs && d < bd)) {
        best = s;
        bs = sc;
        bd = d;
      }
    }
    if (best < 0) break;
    cur[best]++;
    if (std::find(seen.begin(), seen.end(), bd) != seen.end()) continue;
    seen.push_back(bd);
    od[n] = bd;
    os[n] = bs;
    n++;
  }
  *on = n;
  return 0;
}

int gbgpu_merge_posdb(gbgpu_ctx *ctx, const gbgpu_list *lists, int n, int remove_neg_keys, int64_t min_rec_sizes,
                      uint8_t *out, int64_t out_cap, int64_t *out_size) {
  (void)ctx; (void)lists; (void)n; (void)remove_neg_keys; (void)min_rec_sizes; (void)out; (void)out_cap;
  if (out_size) *out_size = 0;
  return GBGPU_EUNSUPPORTED;  // next milestone
}

}  // extern "C"
