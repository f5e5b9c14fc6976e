// gbgpu merge: MI355X kernels for RdbList::posdbMerge_r (RdbList.cpp:3065-3568),
// the k-way merge of posdb runs ("tiered files", oldest first) that Msg5 and
// RdbMerge run on the CPU, one key at a time.
//
// The reference's loop has three observable rules (oracle/posdb_merge_oracle.c):
//   order   keys leave in bfcmpPosdb order (RdbList.h:620-641): the 18-byte key
//           as a 144-bit integer (hi6, lo6, base6) with the base's low 3 bits
//           (delete + compression bits) ignored;
//   dedup   on a tie the older list's key is dropped and the scan restarts
//           (RdbList.cpp:3254-3274), so a key survives iff no NEWER list holds
//           an equal key; removeNegKeys then drops surviving delete keys;
//   output  each survivor is re-compressed against the previously written key
//           (18/12/6 bytes, RdbList.cpp:3308-3385) and the loop stops after the
//           first key that takes the output to >= maxPtr (3419, 3443).
// None of that needs the serial loop.  Pipeline (one stream, two host syncs):
//
//   k_mcount / k_mscan / k_mdecode
//       every 6-byte unit of every run is classified in parallel -- base (key
//       start: byte1 & 0x02 set, Posdb.h:887-889 / posdb_key.h), lo (byte 7's
//       0 bit) or hi (termid bytes, ambiguous alone, resolved from the two
//       units before it) -- and each key is decoded to (hi48, lo48, base48)
//       SoA with the hi/lo it inherits found by a max-scan of unit indices.
//   k_msample / k_mrank / k_moff
//       every S-th key of every run is a splitter; the splitters are ranked
//       into one sorted sequence (binary searches in the other runs' samples)
//       and every n-th one becomes a tile boundary, whose lower bound in every
//       run is found in the S keys between two samples.  A tile then holds at
//       most 2nS = TCAP keys, all keys equal to one another in the same tile.
//   k_mtile  per tile, in LDS: survivor flags (equal key in a newer run?),
//       merged rank of each survivor (lower bounds in the other runs'
//       segments over an exclusive survivor count), survivors 2..n
//       re-compressed against their predecessor into a byte arena; a tile
//       summary (count, arena bytes, first/last key)
//   k_tscan1/2/3  tile byte offsets: the first key of a tile is compressed
//       against the last survivor of the closest non-empty tile before it
//   k_mcut   the key at which the reference loop stops (maxPtr)
//   k_mcopy  each tile's first key + its arena bytes to the output.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "../../include/gbgpu.h"
#include "merge.h"

namespace gbmerge {

constexpr int MB = 256;                          // threads per block
constexpr int MUPT = 8;                          // units per thread (decode)
constexpr int MCH = MB * MUPT;                   // 2048 units = 12 KiB per decode chunk
constexpr int WIN_LO = 16;                       // bytes staged before a chunk (2 units + pad)
constexpr int WIN_BYTES = WIN_LO + MCH * 6 + 16; // + 2 units after it
#ifndef GBGPU_TCAP
#define GBGPU_TCAP 512
#endif
constexpr int TCAP = GBGPU_TCAP;                 // keys per merge tile
#ifndef GBGPU_TB
#define GBGPU_TB 256
#endif
constexpr int TB = GBGPU_TB;                     // threads per merge-tile block
constexpr int MAXN = 256;                        // runs per merge (oracle MAXL)
constexpr int SCAN_TPB = MB * 4;                 // tiles per scan block

enum : uint32_t { F_CORRUPT = 1, F_FIRST = 2, F_CAPACITY = 4, F_MORE = 8 };

struct MList {
  const uint8_t *p;
  uint64_t size;   // bytes
  uint32_t units;  // size / 6
  uint32_t c0;     // first decode chunk of this run
  uint64_t koff;   // first key slot in the decoded arrays
  uint32_t nkeys;  // k_mscan
  uint32_t soff;   // first sample
  uint32_t ns;     // samples
  uint32_t pad;
};

// per decode chunk: keys, last lo unit + 1, last hi unit + 1 (0: none);
// k_mscan turns them into the exclusive carries of the chunk
struct DSum {
  uint32_t nkeys, lastlo, lasthi, pad;
};

struct Keys {
  uint64_t *hi, *lo, *b;
};

struct TileSum {
  uint32_t n, inner;  // survivors; bytes of survivors 2..n (compressed in the tile)
  uint64_t fhi, flo, fb, lhi, llo;  // first survivor (hi, lo, base), last (hi, lo)
  uint64_t arena;     // where survivors 2..n's bytes sit in the arena
};
struct TileOff {
  uint64_t off;    // output offset of the tile's first byte
  uint32_t fsize;  // its first key's re-compressed size (0: empty tile)
  int32_t prev;    // closest non-empty tile before this one, -1 none
};
struct BlkSum {
  uint64_t bytes;  // bytes of the block's tiles, less its first non-empty tile's first key
  int32_t first, last;
};
struct MCtl {
  uint32_t flags, pad;
  unsigned long long out_end;     // end of the last key written (the list size)
  unsigned long long last_start;  // start of that key (ENOSPC check)
  uint64_t lk_hi, lk_lo, lk_b;    // that key, decompressed (RdbList::m_lastKey)
};

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
template <class T>
__device__ __forceinline__ const __attribute__((address_space(1))) T *gptr(const void *p) {
  return (const __attribute__((address_space(1))) T *)p;
}

// ---------------------------------------------------------------- helpers
template <int NT, class T, class Op>
__device__ __forceinline__ T block_scan(T v, T id, Op op, T *tmp, T *total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  T x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    T y = __shfl_up(x, o, 64);
    if (lane >= o) x = op(x, y);
  }
  if (lane == 63) tmp[wid] = x;
  __syncthreads();
  T base = id, tot = id;
#pragma unroll
  for (int w = 0; w < NT / 64; w++) {
    if (w < wid) base = op(base, tmp[w]);
    tot = op(tot, tmp[w]);
  }
  T ex = __shfl_up(x, 1, 64);
  if (lane == 0) ex = id;
  __syncthreads();
  *total = tot;
  return op(base, ex);
}
struct OpAdd {
  template <class T> __device__ T operator()(T a, T b) const { return a + b; }
};
struct OpMax {
  template <class T> __device__ T operator()(T a, T b) const { return a > b ? a : b; }
};

// bfcmpPosdb (RdbList.h:620-641): hi, lo, then base with bits 0-2 ignored
__device__ __forceinline__ bool key_lt(uint64_t h1, uint64_t l1, uint64_t b1, uint64_t h2, uint64_t l2, uint64_t b2) {
  if (h1 != h2) return h1 < h2;
  if (l1 != l2) return l1 < l2;
  return (b1 | 7) < (b2 | 7);
}
// the same order without short-circuits: all three words are loaded up front
__device__ __forceinline__ bool key_lt_bl(uint64_t h1, uint64_t l1, uint64_t b1, uint64_t h2, uint64_t l2,
                                          uint64_t b2) {
  return (h1 < h2) | ((h1 == h2) & ((l1 < l2) | ((l1 == l2) & ((b1 | 7) < (b2 | 7)))));
}
__device__ __forceinline__ bool key_eq(uint64_t h1, uint64_t l1, uint64_t b1, uint64_t h2, uint64_t l2, uint64_t b2) {
  return h1 == h2 && l1 == l2 && (b1 | 7) == (b2 | 7);
}
// re-compressed size against the previously written key (RdbList.cpp:3308-3385)
__device__ __forceinline__ uint32_t ksize(uint64_t h, uint64_t l, uint64_t ph, uint64_t pl) {
  return h != ph ? 18u : (l != pl ? 12u : 6u);
}

// run index of decode chunk c / of sample g (runs ordered by c0 / soff)
__device__ __forceinline__ int list_of_chunk(const MList *L, int n, uint32_t c) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    int mid = (lo + hi + 1) >> 1;
    if (L[mid].c0 <= c) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}
__device__ __forceinline__ int list_of_sample(const MList *L, int n, uint32_t g) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    int mid = (lo + hi + 1) >> 1;
    if (L[mid].soff <= g) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// Stage bytes [u0*6 - 16, u0*6 + 12 KiB + 16) of a run into LDS.  Bytes
// before the run read as zero; the run is readable up to size rounded to 16.
__device__ __forceinline__ void stage(const MList &L, uint32_t u0, uint8_t *lds) {
  const int64_t g0 = (int64_t)u0 * 6 - WIN_LO;
  const uint64_t lim = (L.size + 15) & ~(uint64_t)15;
  for (int i = threadIdx.x; i < WIN_BYTES / 16; i += MB) {
    const int64_t g = g0 + 16 * (int64_t)i;
    v4u v = {0, 0, 0, 0};
    if (g >= 0 && (uint64_t)g + 16 <= lim) v = *gptr<v4u>(L.p + g);
    reinterpret_cast<v4u *>(lds)[i] = v;
  }
}
__device__ __forceinline__ const uint8_t *lunit(const uint8_t *lds, uint32_t u0, int64_t u) {
  return lds + WIN_LO + (int)(u - (int64_t)u0) * 6;
}
// the alignment bit of unit u; units before the run count as set
__device__ __forceinline__ uint32_t sbit(const uint8_t *lds, uint32_t u0, int64_t u) {
  return u < 0 ? 1u : ((lunit(lds, u0, u)[1] >> 1) & 1u);
}
// 0: key start (base), 1: lo unit (bytes 6-11), 2: hi unit (bytes 12-17).
// A base always has byte1 & 0x02 set and a lo unit never does (posdb_key.h);
// a hi unit (termid bytes) may have either, but always follows a lo unit, and
// a lo unit always follows a base.  So: clear bit -> lo after a set unit, hi
// after a clear one; set bit after a clear one -> hi iff that clear unit is a
// lo whose base (two back) is an uncompressed 18-byte key.
__device__ __forceinline__ int utype(const uint8_t *lds, uint32_t u0, int64_t u) {
  if (!sbit(lds, u0, u)) return sbit(lds, u0, u - 1) ? 1 : 2;
  if (sbit(lds, u0, u - 1)) return 0;
  if (u >= 2 && sbit(lds, u0, u - 2) && (lunit(lds, u0, u - 2)[0] & 0x06) == 0) return 2;
  return 0;
}
// key size in units from byte 0 (getKeySize, Posdb.h:271-275)
__device__ __forceinline__ uint32_t kunits(uint8_t b0) { return (b0 & 0x04) ? 1u : ((b0 & 0x02) ? 2u : 3u); }

__device__ __forceinline__ uint64_t rd48(const uint8_t *p) {
  return (uint64_t)p[0] | ((uint64_t)p[1] << 8) | ((uint64_t)p[2] << 16) | ((uint64_t)p[3] << 24) |
         ((uint64_t)p[4] << 32) | ((uint64_t)p[5] << 40);
}
__device__ __forceinline__ uint64_t rd48g(const uint8_t *p) {  // 2-B aligned global
  const auto *q = gptr<uint16_t>(p);
  return (uint64_t)q[0] | ((uint64_t)q[1] << 16) | ((uint64_t)q[2] << 32);
}

// ------------------------------------------------------------- decoding
__global__ void __launch_bounds__(MB) k_mcount(const MList *lists, int n, DSum *sum, MCtl *ctl) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[WIN_BYTES];
  __shared__ uint32_t t0[MB / 64], t1[MB / 64], t2[MB / 64];
  const int li = list_of_chunk(lists, n, blockIdx.x);
  const MList L = lists[li];
  const uint32_t u0 = (blockIdx.x - L.c0) * MCH;
  stage(L, u0, lds);
  __syncthreads();
  uint32_t cnt = 0, llo = 0, lhi = 0, bad = 0;
#pragma unroll
  for (int q = 0; q < MUPT; q++) {
    const uint32_t u = u0 + threadIdx.x * MUPT + q;
    if (u >= L.units) break;
    const int t = utype(lds, u0, u);
    if (t == 0) {
      cnt++;
      const uint32_t ku = kunits(lunit(lds, u0, u)[0]);
      if ((uint64_t)u + ku > L.units) bad |= F_CORRUPT;
      if (u == 0 && ku != 3) bad |= F_FIRST;
    } else if (t == 1) {
      llo = u + 1;
    } else {
      lhi = u + 1;
    }
    if (u == 0 && t != 0) bad |= F_FIRST;
  }
  if (bad) atomicOr(&ctl->flags, bad);
  uint32_t a, b, c;
  (void)block_scan<MB>(cnt, 0u, OpAdd(), t0, &a);
  (void)block_scan<MB>(llo, 0u, OpMax(), t1, &b);
  (void)block_scan<MB>(lhi, 0u, OpMax(), t2, &c);
  if (threadIdx.x == 0) sum[blockIdx.x] = DSum{a, b, c, 0};
}

// per run (one block each): exclusive key count and lo/hi carries per chunk;
// each thread takes SCH consecutive chunks per pass
constexpr int SCH = 8;
__global__ void __launch_bounds__(1024) k_mscan(MList *lists, DSum *sum) {
  __shared__ uint32_t t0[16], t1[16], t2[16];
  __shared__ uint32_t carry[3];
  MList &L = lists[blockIdx.x];
  const uint32_t nch = (L.units + MCH - 1) / MCH;
  if (threadIdx.x == 0) carry[0] = carry[1] = carry[2] = 0;
  __syncthreads();
  for (uint32_t base = 0; base < nch; base += 1024 * SCH) {
    const uint32_t i0 = base + threadIdx.x * SCH;
    DSum v[SCH];
    uint32_t x0 = 0, x1 = 0, x2 = 0;
#pragma unroll
    for (int q = 0; q < SCH; q++) {
      v[q] = i0 + q < nch ? sum[L.c0 + i0 + q] : DSum{0, 0, 0, 0};
      x0 += v[q].nkeys;
      x1 = v[q].lastlo > x1 ? v[q].lastlo : x1;
      x2 = v[q].lasthi > x2 ? v[q].lasthi : x2;
    }
    uint32_t a, b, c;
    const uint32_t c0 = carry[0], c1 = carry[1], c2 = carry[2];
    const uint32_t e0 = block_scan<1024>(x0, 0u, OpAdd(), t0, &a);
    const uint32_t e1 = block_scan<1024>(x1, 0u, OpMax(), t1, &b);
    const uint32_t e2 = block_scan<1024>(x2, 0u, OpMax(), t2, &c);
    uint32_t r0 = c0 + e0, r1 = e1 > c1 ? e1 : c1, r2 = e2 > c2 ? e2 : c2;
#pragma unroll
    for (int q = 0; q < SCH; q++) {
      if (i0 + q < nch) sum[L.c0 + i0 + q] = DSum{r0, r1, r2, 0};
      r0 += v[q].nkeys;
      r1 = v[q].lastlo > r1 ? v[q].lastlo : r1;
      r2 = v[q].lasthi > r2 ? v[q].lasthi : r2;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      carry[0] = c0 + a;
      carry[1] = b > c1 ? b : c1;
      carry[2] = c > c2 ? c : c2;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) L.nkeys = carry[0];
}

// Units are taken in 8 rounds of 256 consecutive units (lane i of wave w
// holds unit u0 + 256q + 64w + i), so the keys a round decodes are written to
// consecutive slots by consecutive lanes.  Within a wave, key ranks and the
// last lo / hi unit before a lane come from ballots; across waves and rounds
// from per-wave totals in LDS and the chunk carries of k_mscan.
__global__ void __launch_bounds__(MB) k_mdecode(const MList *lists, int n, const DSum *sum, Keys K, MCtl *ctl) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[WIN_BYTES];
  __shared__ uint32_t wk[MUPT][MB / 64], wlo[MUPT][MB / 64], whi[MUPT][MB / 64];
  const int li = list_of_chunk(lists, n, blockIdx.x);
  const MList L = lists[li];
  const uint32_t u0 = (blockIdx.x - L.c0) * MCH;
  stage(L, u0, lds);
  __syncthreads();
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const uint64_t below = (1ull << lane) - 1;
  uint32_t types = 0;
#pragma unroll
  for (int q = 0; q < MUPT; q++) {
    const uint32_t u = u0 + q * MB + threadIdx.x;
    const int t = u < L.units ? utype(lds, u0, u) : 3;
    types |= (uint32_t)t << (2 * q);
    const uint64_t bk = __ballot(t == 0), bl = __ballot(t == 1), bh = __ballot(t == 2);
    if (lane == 0) {
      const uint32_t w0 = u0 + q * MB + wid * 64;
      wk[q][wid] = (uint32_t)__popcll(bk);
      wlo[q][wid] = bl ? w0 + (63 - __clzll(bl)) + 1 : 0;
      whi[q][wid] = bh ? w0 + (63 - __clzll(bh)) + 1 : 0;
    }
  }
  __syncthreads();
  const DSum c = sum[blockIdx.x];
  uint64_t kbase = L.koff + c.nkeys;
  uint32_t clo = c.lastlo, chi = c.lasthi;
  bool bad = false;
  const int64_t wlo_u = (int64_t)u0 - 2, whi_u = (int64_t)u0 + MCH + 2;
#pragma unroll
  for (int q = 0; q < MUPT; q++) {
    const uint32_t u = u0 + q * MB + threadIdx.x;
    const int t = (types >> (2 * q)) & 3;
    const uint64_t bk = __ballot(t == 0), bl = __ballot(t == 1), bh = __ballot(t == 2);
    uint64_t kb = kbase;
    uint32_t lo = clo, hi = chi;
    for (int w = 0; w < MB / 64; w++) {
      if (w < wid) {
        kb += wk[q][w];
        lo = lo > wlo[q][w] ? lo : wlo[q][w];
        hi = hi > whi[q][w] ? hi : whi[q][w];
      }
      kbase += wk[q][w];
      clo = clo > wlo[q][w] ? clo : wlo[q][w];
      chi = chi > whi[q][w] ? chi : whi[q][w];
    }
    if (t == 0) {
      const uint32_t w0 = u0 + q * MB + wid * 64;
      const uint64_t ml = bl & below, mh = bh & below;
      if (ml) lo = w0 + (63 - __clzll(ml)) + 1;
      if (mh) hi = w0 + (63 - __clzll(mh)) + 1;
      const uint64_t kidx = kb + __popcll(bk & below);
      const uint8_t *bp = lunit(lds, u0, u);
      const uint32_t ku = kunits(bp[0]);
      const int64_t lu = ku >= 2 ? (int64_t)u + 1 : (int64_t)lo - 1;
      const int64_t hu = ku == 3 ? (int64_t)u + 2 : (int64_t)hi - 1;
      uint64_t lov = 0, hiv = 0;
      if (lu < 0 || hu < 0 || (uint64_t)u + ku > L.units) {
        bad = true;
      } else {
        lov = (lu >= wlo_u && lu < whi_u) ? rd48(lunit(lds, u0, lu)) : rd48g(L.p + (size_t)lu * 6);
        hiv = (hu >= wlo_u && hu < whi_u) ? rd48(lunit(lds, u0, hu)) : rd48g(L.p + (size_t)hu * 6);
      }
      K.hi[kidx] = hiv;
      K.lo[kidx] = lov;
      K.b[kidx] = rd48(bp);
    }
  }
  if (bad) atomicOr(&ctl->flags, (uint32_t)F_CORRUPT);
}

// ------------------------------------------------------------ partition
// a splitter: the three key words side by side, so one step of a search over
// splitters touches one 32-byte sector instead of three cache lines
struct __attribute__((aligned(32))) SKey {
  uint64_t h, l, b, pad;
};

__global__ void __launch_bounds__(MB) k_msample(const MList *lists, int n, uint32_t S, Keys K, SKey *Sm,
                                                uint32_t nsamples) {
  const uint32_t g = blockIdx.x * MB + threadIdx.x;
  if (g >= nsamples) return;
  const MList &L = lists[list_of_sample(lists, n, g)];
  const uint64_t idx = L.koff + (uint64_t)(g - L.soff) * S;
  Sm[g] = SKey{K.hi[idx], K.lo[idx], K.b[idx], 0};
}

// first index in [a, z) of K whose key is >= v (UB: > v)
template <bool UB>
__device__ __forceinline__ uint64_t gbound(const Keys &K, uint64_t a, uint64_t z, uint64_t vh, uint64_t vl,
                                           uint64_t vb) {
  while (a < z) {
    const uint64_t m = (a + z) >> 1;
    const bool go = UB ? !key_lt(vh, vl, vb, K.hi[m], K.lo[m], K.b[m]) : key_lt(K.hi[m], K.lo[m], K.b[m], vh, vl, vb);
    if (go) a = m + 1;
    else z = m;
  }
  return a;
}

template <bool UB>
__device__ __forceinline__ uint64_t sbound(const SKey *Sm, uint64_t a, uint64_t z, uint64_t vh, uint64_t vl,
                                           uint64_t vb) {
  while (a < z) {
    const uint64_t m = (a + z) >> 1;
    const SKey x = Sm[m];
    const bool go = UB ? !key_lt(vh, vl, vb, x.h, x.l, x.b) : key_lt(x.h, x.l, x.b, vh, vl, vb);
    if (go) a = m + 1;
    else z = m;
  }
  return a;
}

// sorted order of all samples by (key, run, index): scatter sample ids
__global__ void __launch_bounds__(MB) k_mrank(const MList *lists, int n, const SKey *Sm, uint32_t nsamples, uint32_t *tiles) {
  const uint32_t g = blockIdx.x * MB + threadIdx.x;
  if (g >= nsamples) return;
  const int l = list_of_sample(lists, n, g);
  const SKey v = Sm[g];
  const uint64_t vh = v.h, vl = v.l, vb = v.b;
  uint64_t pos = g - lists[l].soff;
  for (int l2 = 0; l2 < n; l2++) {
    if (l2 == l) continue;
    const uint64_t a = lists[l2].soff, z = a + lists[l2].ns;
    pos += (l2 < l ? sbound<true>(Sm, a, z, vh, vl, vb) : sbound<false>(Sm, a, z, vh, vl, vb)) - a;
  }
  tiles[pos] = g;
}

// off[t*n + l2] = lower bound in run l2 (key index in the run) of tile t's
// boundary, the sorted sample at position t*J; row T holds the run lengths.
// Run l2's segment then holds at most (samples of l2 among the J + 1)*S keys,
// so a tile holds at most (J + n)*S keys -- TCAP for J = n, S = TCAP/2n.
__global__ void __launch_bounds__(MB) k_moff(const MList *lists, int n, uint32_t S, uint32_t J, Keys K, const SKey *Sm,
                                             const uint32_t *tiles, uint32_t T, uint32_t *off) {
  const uint64_t i = (uint64_t)blockIdx.x * MB + threadIdx.x;
  if (i >= (uint64_t)(T + 1) * n) return;
  const uint32_t t = (uint32_t)(i / n);
  const int l2 = (int)(i % n);
  const MList &L = lists[l2];
  if (t == T) {
    off[i] = L.nkeys;
    return;
  }
  const uint32_t g = tiles[(size_t)t * J];
  const SKey v = Sm[g];
  const uint64_t vh = v.h, vl = v.l, vb = v.b;
  const uint64_t q = sbound<false>(Sm, L.soff, (uint64_t)L.soff + L.ns, vh, vl, vb) - L.soff;
  uint64_t r = 0;
  if (q > 0) {
    // samples q-1 < v <= sample q: the bound is in ((q-1)S, qS]
    const uint64_t a = L.koff + (q - 1) * S + 1;
    const uint64_t z = L.koff + (q * S < L.nkeys ? q * S : (uint64_t)L.nkeys);
    r = gbound<false>(K, a, z, vh, vl, vb) - L.koff;
  }
  off[i] = (uint32_t)r;
}

// ------------------------------------------------------------ tile merge
template <int TBt, int TCAPt>
struct TileLdsT {
  uint64_t h[TCAPt], l[TCAPt], b[TCAPt];
  uint16_t ord[TCAPt];    // entry of merged rank r
  uint8_t run[TCAPt];
  uint8_t keep[TCAPt];
  uint32_t seg[MAXN + 1];
  uint32_t beg[MAXN];
  uint64_t koff[MAXN];
  uint32_t tmp[TBt / 64];
  uint64_t tmp64[TBt / 64];
};
typedef TileLdsT<TB, TCAP> TileLds;

__device__ __forceinline__ void put48(uint16_t *o, uint64_t v) {
  o[0] = (uint16_t)v;
  o[1] = (uint16_t)(v >> 16);
  o[2] = (uint16_t)(v >> 32);
}
// the output bytes of a key of re-compressed size sz (RdbList.cpp:3308-3385:
// byte 0's compression bits rewritten, then lo and hi as needed)
__device__ __forceinline__ void put_key(uint16_t *o, uint32_t sz, uint64_t h, uint64_t l, uint64_t b) {
  const uint64_t cbits = sz == 6 ? 0x06 : (sz == 12 ? 0x02 : 0x00);
  put48(o, (b & ~(uint64_t)0x06) | cbits);
  if (sz >= 12) put48(o + 3, l);
  if (sz == 18) put48(o + 6, h);
}

// The tile's n sorted run segments are in s (seg[] = their starts, seg[n] =
// tot, run[] = each entry's run): merge them, find the survivors (no equal
// key in a newer run, RdbList.cpp:3254-3274; not a delete key under
// removeNegKeys, 3276-3279), and append the bytes of survivors 2..n
// compressed against their predecessor to the arena at 18 x kbefore (the
// keys of all runs before this tile); publish the tile summary.
// Merge-path split: in the pair of segment groups [g0, g0+w) (A) and
// [g0+w, g0+2w) (B), the A and B entries (LDS indices i, j) at which output
// p of the pair's merge starts; am / a1 = ends of A / B.  An A key goes
// before an equal B key.
template <class S>
__device__ __forceinline__ void mp_split(const S &s, int n, int w, int g0, uint32_t p, uint32_t &am, uint32_t &a1,
                                         uint32_t &i, uint32_t &j) {
  const int gm = g0 + w < n ? g0 + w : n, g1 = g0 + 2 * w < n ? g0 + 2 * w : n;
  const uint32_t a0 = s.seg[g0];
  am = s.seg[gm];
  a1 = s.seg[g1];
  const uint32_t d = p - a0, la = am - a0, lb = a1 - am;
  uint32_t x = d > lb ? d - lb : 0, y = d < la ? d : la;
  while (x < y) {
    const uint32_t mid = (x + y) >> 1, ea = a0 + mid, eb = am + d - mid - 1;
    // A[mid] goes first iff A[mid] <= B[d-mid-1]
    if (!key_lt_bl(s.h[eb], s.l[eb], s.b[eb], s.h[ea], s.l[ea], s.b[ea])) x = mid + 1;
    else y = mid;
  }
  i = a0 + x;
  j = am + (d - x);
}

template <int TBt, int TCAPt, int MODE = 0>
__device__ void tile_merge_emit(TileLdsT<TBt, TCAPt> &s, int n, uint32_t tot, uint64_t kbefore, uint32_t t,
                                TileSum *ts, int rm, uint8_t *arena) {
  constexpr int KPTt = TCAPt / TBt;
  // Merge the n sorted segments in place, pairwise: the round with width w
  // merges each group of w segments (A, older runs) with the next w (B), so
  // keys equal under bfcmpPosdb stay in run order (older first).  Merge
  // path: thread i produces outputs [i*VT, i*VT + VT) of the round; its
  // start in its pair (A, B) is one diagonal search (how many of the first
  // d outputs come from A, an A key going first on a tie), then it merges
  // VT keys serially with both heads in registers.  Outputs are written back
  // in place after a barrier.
  constexpr int VT = KPTt;
  for (int w = 1; w < n; w <<= 1) {
    uint64_t oh[VT], ol[VT], ob[VT];
    uint8_t orr[VT];
    const uint32_t p0 = threadIdx.x * VT;
    if (p0 < tot) {
      int lo = 0, hi = n - 1;  // last segment starting at or before p0
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (s.seg[mid] <= p0) lo = mid;
        else hi = mid - 1;
      }
      int g0 = lo & ~(2 * w - 1);
      uint32_t am, a1, i, j;
      mp_split(s, n, w, g0, p0, am, a1, i, j);
      uint64_t ah = 0, al = 0, ab = 0, bh = 0, bl = 0, bb = 0;
      if (i < am) { ah = s.h[i]; al = s.l[i]; ab = s.b[i]; }
      if (j < a1) { bh = s.h[j]; bl = s.l[j]; bb = s.b[j]; }
#pragma unroll
      for (int v = 0; v < VT; v++) {
        const uint32_t p = p0 + v;
        if (p >= tot) break;
        if (p == a1) {  // the next pair starts here (empty pairs skipped)
          do {
            g0 += 2 * w;
          } while (s.seg[g0 + 2 * w < n ? g0 + 2 * w : n] <= p);
          mp_split(s, n, w, g0, p, am, a1, i, j);
          if (i < am) { ah = s.h[i]; al = s.l[i]; ab = s.b[i]; }
          if (j < a1) { bh = s.h[j]; bl = s.l[j]; bb = s.b[j]; }
        }
        const bool ta = i < am && (j >= a1 || !key_lt_bl(bh, bl, bb, ah, al, ab));
        if (ta) {
          oh[v] = ah; ol[v] = al; ob[v] = ab; orr[v] = s.run[i];
          i++;
          if (i < am) { ah = s.h[i]; al = s.l[i]; ab = s.b[i]; }
        } else {
          oh[v] = bh; ol[v] = bl; ob[v] = bb; orr[v] = s.run[j];
          j++;
          if (j < a1) { bh = s.h[j]; bl = s.l[j]; bb = s.b[j]; }
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int v = 0; v < VT; v++) {
      const uint32_t p = p0 + v;
      if (p >= tot) break;
      s.h[p] = oh[v];
      s.l[p] = ol[v];
      s.b[p] = ob[v];
      s.run[p] = orr[v];
    }
    __syncthreads();
  }
  if (MODE == 3) {  // diagnostic: stop after the merge rounds
    if (threadIdx.x == 0) ts[t] = TileSum{0, 0, s.h[0], 0, 0, 0, 0, 0};
    return;
  }
  // a survivor has no equal key in a newer run (RdbList.cpp:3254-3274): the
  // equal keys after it are in run order, so look for one from another run
  for (uint32_t e = threadIdx.x; e < tot; e += TBt) {
    const uint64_t vh = s.h[e], vl = s.l[e], vb = s.b[e];
    bool drop = rm && !(vb & 1);
    for (uint32_t f = e + 1; !drop && f < tot && key_eq(s.h[f], s.l[f], s.b[f], vh, vl, vb); f++)
      drop = s.run[f] != s.run[e];
    s.keep[e] = !drop;
  }
  __syncthreads();
  uint32_t em = 0;
#pragma unroll
  for (int j = 0; j < KPTt; j++) {
    const uint32_t e = threadIdx.x * KPTt + j;
    if (e < tot && s.keep[e]) em |= 1u << j;
  }
  uint32_t nemit;
  const uint32_t eb = block_scan<TBt>((uint32_t)__popc(em), 0u, OpAdd(), s.tmp, &nemit);
  // entries are in merged order: a survivor's rank is the survivors before it
#pragma unroll
  for (int j = 0; j < KPTt; j++) {
    const uint32_t e = threadIdx.x * KPTt + j;
    if (e < tot && (em >> j & 1)) s.ord[eb + __popc(em & ((1u << j) - 1))] = (uint16_t)e;
  }
  if (nemit == 0) {
    if (threadIdx.x == 0) ts[t] = TileSum{0, 0, 0, 0, 0, 0, 0, 0};
    return;
  }
  __syncthreads();
  // sizes of ranks 1..n-1 against their predecessor, their tile offsets
  uint32_t sz[KPTt], mine = 0;
#pragma unroll
  for (int j = 0; j < KPTt; j++) {
    const uint32_t r = threadIdx.x * KPTt + j;
    sz[j] = 0;
    if (r == 0 || r >= nemit) continue;
    const uint32_t e = s.ord[r], p = s.ord[r - 1];
    sz[j] = ksize(s.h[e], s.l[e], s.h[p], s.l[p]);
    mine += sz[j];
  }
  uint32_t inner;
  uint32_t o = block_scan<TBt>(mine, 0u, OpAdd(), s.tmp, &inner);
  const uint64_t at = 18 * kbefore;
  if (threadIdx.x == 0) {
    const uint32_t f = s.ord[0], z = s.ord[nemit - 1];
    ts[t] = TileSum{nemit, inner, s.h[f], s.l[f], s.b[f], s.h[z], s.l[z], at};
  }
  uint8_t *dst = arena + at;
#pragma unroll
  for (int j = 0; j < KPTt; j++) {
    const uint32_t r = threadIdx.x * KPTt + j;
    if (!sz[j]) continue;
    const uint32_t e = s.ord[r];
    put_key(reinterpret_cast<uint16_t *>(dst + o), sz[j], s.h[e], s.l[e], s.b[e]);
    o += sz[j];
  }
}

// One tile (legacy path): the segment of every run between two boundary keys,
// gathered from the decoded keys into LDS, then merged and emitted.
__global__ void __launch_bounds__(TB) k_mtile(const MList *lists, int n, const uint32_t *off, Keys K, TileSum *ts,
                                              int rm, uint8_t *arena, MCtl *ctl) {
  __shared__ TileLds s;
  const uint32_t t = blockIdx.x;
  uint32_t len = 0;
  uint64_t before = 0;
  if (threadIdx.x < n) {
    const uint32_t b = off[(size_t)t * n + threadIdx.x], e = off[(size_t)(t + 1) * n + threadIdx.x];
    s.beg[threadIdx.x] = b;
    s.koff[threadIdx.x] = lists[threadIdx.x].koff;
    len = e - b;
    before = b;
  }
  uint32_t tot;
  const uint32_t ex = block_scan<TB>(len, 0u, OpAdd(), s.tmp, &tot);
  // keys of all runs before this tile: the tile's arena bytes start at 18x that
  uint64_t kbefore;
  block_scan<TB>(before, (uint64_t)0, OpAdd(), s.tmp64, &kbefore);
  if (threadIdx.x < n) s.seg[threadIdx.x] = ex;
  if (threadIdx.x == 0) s.seg[n] = tot;
  if (tot > TCAP || tot == 0) {
    if (threadIdx.x == 0) {
      ts[t] = TileSum{0, 0, 0, 0, 0, 0, 0, 0};
      if (tot > TCAP) atomicOr(&ctl->flags, (uint32_t)F_CAPACITY);
    }
    return;
  }
  __syncthreads();
  for (uint32_t e = threadIdx.x; e < tot; e += TB) {
    int lo = 0, hi = n - 1;  // last run whose segment starts at or before e
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (s.seg[mid] <= e) lo = mid;
      else hi = mid - 1;
    }
    const uint64_t idx = s.koff[lo] + s.beg[lo] + (e - s.seg[lo]);
    s.h[e] = K.hi[idx];
    s.l[e] = K.lo[idx];
    s.b[e] = K.b[idx];
    s.run[e] = (uint8_t)lo;
  }
  __syncthreads();
  tile_merge_emit<TB, TCAP>(s, n, tot, kbefore, t, ts, rm, arena);
}

// --------------------------------------------------------- tile offsets
// Walk a thread's SCAN_TPB/MB tiles: bytes of its non-empty tiles, the first
// key of the first one compressed against (ph, pl) when `has`, else skipped.
__device__ __forceinline__ void walk(const TileSum *ts, uint32_t T, uint32_t i0, bool has, uint64_t ph, uint64_t pl,
                                     uint64_t *bytes, int32_t *first, int32_t *last) {
  uint64_t by = 0;
  int32_t f = -1, z = -1;
  for (int j = 0; j < SCAN_TPB / MB; j++) {
    const uint32_t i = i0 + j;
    if (i >= T) break;
    const TileSum &s = ts[i];
    if (s.n == 0) continue;
    if (z >= 0 || has) by += ksize(s.fhi, s.flo, ph, pl);
    else f = (int32_t)i;
    by += s.inner;
    ph = s.lhi;
    pl = s.llo;
    z = (int32_t)i;
  }
  *bytes = by;
  *first = f;
  *last = z;
}

__global__ void __launch_bounds__(MB) k_tscan1(const TileSum *ts, uint32_t T, BlkSum *bs) {
  __shared__ int32_t ti[MB / 64];
  __shared__ uint64_t tb[MB / 64];
  const uint32_t i0 = blockIdx.x * SCAN_TPB + threadIdx.x * (SCAN_TPB / MB);
  uint64_t by;
  int32_t f, z;
  walk(ts, T, i0, false, 0, 0, &by, &f, &z);
  int32_t zall;
  const int32_t prev = block_scan<MB>(z, -1, OpMax(), ti, &zall);
  // the thread's first tile follows the block's previous non-empty tile
  if (f >= 0 && prev >= 0) by += ksize(ts[f].fhi, ts[f].flo, ts[prev].lhi, ts[prev].llo);
  uint64_t btot;
  block_scan<MB>(by, (uint64_t)0, OpAdd(), tb, &btot);
  // the block's first non-empty tile: the f of the first thread with one
  int32_t fm = (f >= 0 && prev < 0) ? f : 0x7fffffff;
  int32_t fall;
  block_scan<MB>(-fm, (int32_t)-0x7fffffff, OpMax(), ti, &fall);
  if (threadIdx.x == 0) bs[blockIdx.x] = BlkSum{btot, -fall == 0x7fffffff ? -1 : -fall, zall};
}

// single block: block offsets and each block's previous non-empty tile
__global__ void __launch_bounds__(1024) k_tscan2(const TileSum *ts, const BlkSum *bs, uint32_t nblk, TileOff *bo) {
  __shared__ int32_t ti[16];
  __shared__ uint64_t tb[16];
  __shared__ int32_t cprev;
  __shared__ uint64_t coff;
  if (threadIdx.x == 0) {
    cprev = -1;
    coff = 0;
  }
  __syncthreads();
  for (uint32_t base = 0; base < nblk; base += 1024) {
    const uint32_t i = base + threadIdx.x;
    const BlkSum v = i < nblk ? bs[i] : BlkSum{0, -1, -1};
    const int32_t p0 = cprev;
    const uint64_t o0 = coff;
    int32_t zall;
    int32_t prev = block_scan<1024>(v.last, -1, OpMax(), ti, &zall);
    prev = prev > p0 ? prev : p0;
    uint64_t by = v.bytes;
    if (v.first >= 0)
      by += prev >= 0 ? ksize(ts[v.first].fhi, ts[v.first].flo, ts[prev].lhi, ts[prev].llo) : 18u;
    uint64_t btot;
    const uint64_t eo = block_scan<1024>(by, (uint64_t)0, OpAdd(), tb, &btot);
    if (i < nblk) bo[i] = TileOff{o0 + eo, 0, prev};
    __syncthreads();
    if (threadIdx.x == 0) {
      cprev = zall > p0 ? zall : p0;
      coff = o0 + btot;
    }
    __syncthreads();
  }
}

__global__ void __launch_bounds__(MB) k_tscan3(const TileSum *ts, uint32_t T, const TileOff *bo, TileOff *to) {
  __shared__ int32_t ti[MB / 64];
  __shared__ uint64_t tb[MB / 64];
  const uint32_t i0 = blockIdx.x * SCAN_TPB + threadIdx.x * (SCAN_TPB / MB);
  const TileOff B = bo[blockIdx.x];
  uint64_t by;
  int32_t f, z;
  walk(ts, T, i0, false, 0, 0, &by, &f, &z);
  int32_t zall;
  int32_t prev = block_scan<MB>(z, -1, OpMax(), ti, &zall);
  prev = prev > B.prev ? prev : B.prev;
  if (f >= 0) by += prev >= 0 ? ksize(ts[f].fhi, ts[f].flo, ts[prev].lhi, ts[prev].llo) : 18u;
  uint64_t btot;
  uint64_t o = B.off + block_scan<MB>(by, (uint64_t)0, OpAdd(), tb, &btot);
  for (int j = 0; j < SCAN_TPB / MB; j++) {
    const uint32_t i = i0 + j;
    if (i >= T) break;
    const TileSum &s = ts[i];
    uint32_t fs = 0;
    if (s.n) fs = prev >= 0 ? ksize(s.fhi, s.flo, ts[prev].lhi, ts[prev].llo) : 18u;
    to[i] = TileOff{o, fs, prev};
    if (s.n == 0) continue;
    o += fs + s.inner;
    prev = (int32_t)i;
  }
}

// The loop stops after the first key that takes the output to >= maxPtr
// (RdbList.cpp:3419,3443): find that key's end (one thread; binary search
// over the tiles, then a walk over the compressed keys of one tile).
__global__ void k_mcut(const TileSum *ts, const TileOff *to, uint32_t T, const uint8_t *arena, uint64_t maxoff,
                       MCtl *ctl) {
  if (threadIdx.x != 0 || blockIdx.x != 0 || T == 0) return;
  // last tile whose offset is < maxoff (tile offsets are non-decreasing)
  uint32_t lo = 0, hi = T - 1;
  while (lo < hi) {
    const uint32_t m = (lo + hi + 1) >> 1;
    if (to[m].off < maxoff) lo = m;
    else hi = m - 1;
  }
  // the non-empty tile holding the last key that starts below maxoff
  int64_t t = lo;
  while (t >= 0 && ts[t].n == 0) t--;
  if (t < 0) return;  // no survivor at all
  const TileSum &S = ts[t];
  uint64_t pos = to[t].off, start = pos;
  pos += to[t].fsize;
  uint64_t kh = S.fhi, kl = S.flo, kb = S.fb;
  const uint8_t *p = arena + S.arena;
  for (uint32_t k = 1; k < S.n && pos < maxoff; k++) {
    start = pos;
    const uint32_t sz = (p[0] & 0x04) ? 6u : ((p[0] & 0x02) ? 12u : 18u);
    kb = rd48(p);
    if (sz >= 12) kl = rd48(p + 6);
    if (sz == 18) kh = rd48(p + 12);
    pos += sz;
    p += sz;
  }
  ctl->out_end = pos;
  ctl->last_start = start;
  // m_lastKey: base with the compression bits cleared (RdbList.cpp:3526-3535)
  ctl->lk_hi = kh;
  ctl->lk_lo = kl;
  ctl->lk_b = kb & ~(uint64_t)0x06;
}

// posdbMerge_r's numLists after its loop (RdbList.cpp:3541-3542): the loop
// stops right after writing the cut key W, so a run still holds keys iff it
// has one ordered after W (bfcmpPosdb; keys equal to W in older runs were
// dropped before it, and W's own run is past it).  One thread per run.
__global__ void __launch_bounds__(256) k_mrest(const MList *lists, int n, Keys K, MCtl *ctl) {
  const int i = threadIdx.x;
  if (i >= n || ctl->out_end == 0) return;
  const MList L = lists[i];
  const uint64_t end = L.koff + L.nkeys;
  if (gbound<true>(K, L.koff, end, ctl->lk_hi, ctl->lk_lo, ctl->lk_b) < end) atomicOr(&ctl->flags, (uint32_t)F_MORE);
}

// out[off, off + bytes) of every tile, below the cut: its first key, then its
// arena bytes.  Byte offsets are even (keys are 6-byte multiples).
__global__ void __launch_bounds__(MB) k_mcopy(const TileSum *ts, const TileOff *to, const uint8_t *arena,
                                              const MCtl *ctl, uint64_t cap, uint8_t *out, uint32_t T) {
  // one wave per tile
  const uint32_t t = blockIdx.x * (MB / 64) + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (t >= T) return;
  const TileSum S = ts[t];
  if (S.n == 0) return;
  const TileOff o = to[t];
  uint64_t lim = ctl->out_end;
  if (lim > cap) lim = cap;
  if (o.off >= lim) return;
  if (lane == 0 && o.off + o.fsize <= lim)
    put_key(reinterpret_cast<uint16_t *>(out + o.off), o.fsize, S.fhi, S.flo, S.fb);
  const uint64_t d0 = o.off + o.fsize;
  if (d0 >= lim) return;
  const uint32_t nb = (uint32_t)((d0 + S.inner <= lim ? d0 + S.inner : lim) - d0);
  // 2-byte stores up to an 8-byte aligned destination and after the last
  // whole word (the bytes either side belong to the neighbouring tiles), 8-byte
  // stores in between, each assembled from two aligned source words (the
  // arena has slack past its last tile, so reading one word beyond is safe)
  const uint8_t *sp = arena + S.arena;
  uint8_t *dp = out + d0;
  uint32_t head = (uint32_t)((8 - ((uintptr_t)dp & 7)) & 7);
  if (head > nb) head = nb;
  if (lane < head / 2)
    reinterpret_cast<uint16_t *>(dp)[lane] = reinterpret_cast<const uint16_t *>(sp)[lane];
  const uint32_t nw = (nb - head) >> 3, tail = (nb - head) & 7;
  const uintptr_t sa = (uintptr_t)(sp + head);
  const uint64_t *sw = reinterpret_cast<const uint64_t *>(sa & ~(uintptr_t)7);
  const uint32_t sh = (uint32_t)(sa & 7) * 8;
  uint64_t *dw = reinterpret_cast<uint64_t *>(dp + head);
  if (sh == 0) {
    for (uint32_t w = lane; w < nw; w += 64) dw[w] = sw[w];
  } else {
    for (uint32_t w = lane; w < nw; w += 64) dw[w] = (sw[w] >> sh) | (sw[w + 1] << (64 - sh));
  }
  const uint32_t t0 = head + nw * 8;
  if (lane < tail / 2)
    reinterpret_cast<uint16_t *>(dp + t0)[lane] = reinterpret_cast<const uint16_t *>(sp + t0)[lane];
}

// ------------------------------------------------------------------ host
#define MCHECK(x)                                                                                   \
  do {                                                                                              \
    hipError_t e_ = (x);                                                                            \
    if (e_ != hipSuccess) {                                                                         \
      std::fprintf(stderr, "gbgpu merge: %s failed: %s (%s:%d)\n", #x, hipGetErrorString(e_), __FILE__, \
                   __LINE__);                                                                       \
      return GBGPU_EHIP;                                                                            \
    }                                                                                               \
  } while (0)

struct Buf {
  void *p = nullptr;
  size_t cap = 0;
  int ensure(size_t bytes) {
    if (bytes <= cap) return 0;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    const size_t want = std::max<size_t>(bytes + bytes / 8, 1 << 16);
    if (hipMalloc(&p, want) != hipSuccess) return ENOMEM;
    cap = want;
    return 0;
  }
  template <class T> T *as(size_t off = 0) const { return reinterpret_cast<T *>(static_cast<uint8_t *>(p) + off); }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

struct MergeState {
  std::mutex mu;
  hipStream_t st = nullptr;
  hipEvent_t ev[6] = {};
  Buf mlist, dsum, khi, klo, kb, shi, slo, sb, tiles, off, ts, to, bs, bo, ctl, arena, in, out;
  MList *h_lists = nullptr;  // pinned
  MCtl *h_ctl = nullptr;     // pinned
  float ms[6] = {0, 0, 0, 0, 0, 0};
  int64_t nkeys = 0, ntiles = 0;
  int path = 0;  // last merge: 2 (the decoded-key pipeline; 1 was the retired tile path)
  bool has_last = false;
  bool more = false;  // input keys were left unmerged (posdbMerge_r's numLists > 0 at its end)
  uint8_t last_key[18] = {};
};

int state_new(MergeState **out) {
  MergeState *s = new MergeState();
  bool ok = hipStreamCreateWithFlags(&s->st, hipStreamNonBlocking) == hipSuccess &&
            hipHostMalloc((void **)&s->h_lists, sizeof(MList) * MAXN, 0) == hipSuccess &&
            hipHostMalloc((void **)&s->h_ctl, sizeof(MCtl), 0) == hipSuccess;
  for (auto &e : s->ev) ok = ok && hipEventCreate(&e) == hipSuccess;
  if (!ok) {
    state_free(s);
    return GBGPU_EHIP;
  }
  *out = s;
  return 0;
}

void state_free(MergeState *s) {
  if (!s) return;
  if (s->st) (void)hipStreamSynchronize(s->st);
  Buf *bufs[] = {&s->mlist, &s->dsum, &s->khi, &s->klo, &s->kb, &s->shi, &s->slo, &s->sb, &s->tiles, &s->off,
                 &s->ts, &s->to, &s->bs, &s->bo, &s->ctl, &s->arena, &s->in, &s->out};
  for (auto *b : bufs) b->release();
  if (s->h_lists) (void)hipHostFree(s->h_lists);
  if (s->h_ctl) (void)hipHostFree(s->h_ctl);
  for (auto &e : s->ev)
    if (e) (void)hipEventDestroy(e);
  if (s->st) (void)hipStreamDestroy(s->st);
  delete s;
}

static inline uint32_t cdiv(uint64_t a, uint64_t b) { return (uint32_t)((a + b - 1) / b); }

// prepareForMerge + merge_r's bound on the output (oracle/posdb_merge_oracle.c)
static int64_t max_offset(int64_t total, int64_t mrs, int64_t cap) {
  int64_t m = total;
  if (mrs > 0) {
    int64_t nm = (int64_t)(int32_t)((uint32_t)mrs + 36u);
    if (nm < mrs) nm = 0x7fffffff;
    if (m > nm) m = nm;
  }
  return m > cap ? cap : m;
}

// the tile-offset scans, the cut and the copy, shared by both paths; then
// the result flags.  Returns 0, or RETRY when a tile overflowed.
constexpr int RETRY = -1;
static int finish_tiles(MergeState *s, uint32_t T32, uint64_t maxoff, int64_t cap, uint8_t *out, MCtl *dctl, int n,
                        const Keys &K) {
  hipStream_t st = s->st;
  const uint32_t nblk = cdiv(T32, SCAN_TPB);
  TileSum *ts = s->ts.as<TileSum>();
  TileOff *to = s->to.as<TileOff>();
  uint8_t *arena = s->arena.as<uint8_t>();
  k_tscan1<<<nblk, MB, 0, st>>>(ts, T32, s->bs.as<BlkSum>());
  k_tscan2<<<1, 1024, 0, st>>>(ts, s->bs.as<BlkSum>(), nblk, s->bo.as<TileOff>());
  k_tscan3<<<nblk, MB, 0, st>>>(ts, T32, s->bo.as<TileOff>(), to);
  k_mcut<<<1, 64, 0, st>>>(ts, to, T32, arena, maxoff, dctl);
  k_mrest<<<1, 256, 0, st>>>(s->mlist.as<MList>(), n, K, dctl);
  MCHECK(hipEventRecord(s->ev[4], st));
  k_mcopy<<<cdiv(T32, MB / 64), MB, 0, st>>>(ts, to, arena, dctl, (uint64_t)cap, out, T32);
  MCHECK(hipGetLastError());
  MCHECK(hipEventRecord(s->ev[5], st));
  MCHECK(hipMemcpyAsync(s->h_ctl, dctl, sizeof(MCtl), hipMemcpyDeviceToHost, st));
  MCHECK(hipStreamSynchronize(st));
  // [0] total, [1] decode, [2] partition, [3] tile merge, [4] offsets + cut, [5] copy
  (void)hipEventElapsedTime(&s->ms[0], s->ev[0], s->ev[5]);
  for (int i = 1; i <= 5; i++) (void)hipEventElapsedTime(&s->ms[i], s->ev[i - 1], s->ev[i]);
  return (s->h_ctl->flags & F_CAPACITY) ? RETRY : 0;
}

static int ensure_tile_bufs(MergeState *s, uint64_t NS, uint64_t T, int n) {
  const uint32_t nblk = cdiv(T, SCAN_TPB);
  if (s->shi.ensure(sizeof(SKey) * NS) || s->tiles.ensure(4 * NS) || s->off.ensure(4 * (T + 1) * n) ||
      s->ts.ensure(sizeof(TileSum) * T) || s->to.ensure(sizeof(TileOff) * T) || s->bs.ensure(sizeof(BlkSum) * nblk) ||
      s->bo.ensure(sizeof(TileOff) * nblk))
    return ENOMEM;
  return 0;
}

// Every key decoded to 24-byte SoA in HBM, samples every S keys.
static int run_legacy(MergeState *s, int n, uint32_t nch, uint64_t units, int rm, uint64_t maxoff, uint8_t *out,
                      int64_t cap) {
  hipStream_t st = s->st;
  if (s->khi.ensure(8 * units) || s->klo.ensure(8 * units) || s->kb.ensure(8 * units)) return ENOMEM;
  MList *dl = s->mlist.as<MList>();
  MCtl *dctl = s->ctl.as<MCtl>();
  Keys K{s->khi.as<uint64_t>(), s->klo.as<uint64_t>(), s->kb.as<uint64_t>()};
  MCHECK(hipEventRecord(s->ev[0], st));
  MCHECK(hipMemcpyAsync(dl, s->h_lists, sizeof(MList) * n, hipMemcpyHostToDevice, st));
  MCHECK(hipMemsetAsync(dctl, 0, sizeof(MCtl), st));
  k_mcount<<<nch, MB, 0, st>>>(dl, n, s->dsum.as<DSum>(), dctl);
  k_mscan<<<n, 1024, 0, st>>>(dl, s->dsum.as<DSum>());
  k_mdecode<<<nch, MB, 0, st>>>(dl, n, s->dsum.as<DSum>(), K, dctl);
  MCHECK(hipGetLastError());
  MCHECK(hipEventRecord(s->ev[1], st));
  MCHECK(hipMemcpyAsync(s->h_lists, dl, sizeof(MList) * n, hipMemcpyDeviceToHost, st));
  MCHECK(hipMemcpyAsync(s->h_ctl, dctl, sizeof(MCtl), hipMemcpyDeviceToHost, st));
  MCHECK(hipStreamSynchronize(st));
  if (s->h_ctl->flags & F_FIRST) return EINVAL;  // first key must be 18 bytes
  if (s->h_ctl->flags & F_CORRUPT) return GBGPU_ECORRUPT;

  // partition: every S-th key of every run is a splitter and every n-th
  // splitter (in key order) a tile boundary.  A run's segment exceeds its
  // bound only when keys repeat inside the run (never in a canonical Rdb
  // list); the tile pass then flags F_CAPACITY and the partition is redone
  // with a smaller S.
  const uint32_t J = (uint32_t)n;
  if (s->arena.ensure(18 * (size_t)std::max<uint64_t>(units, 1) + 16)) return ENOMEM;  // + k_mcopy read slack
  for (uint32_t S = (uint32_t)std::max(1, TCAP / (2 * n));; S /= 2) {
    uint64_t NS = 0;
    s->nkeys = 0;
    for (int i = 0; i < n; i++) {
      MList &L = s->h_lists[i];
      L.soff = (uint32_t)NS;
      L.ns = cdiv(L.nkeys, S);
      NS += L.ns;
      s->nkeys += L.nkeys;
    }
    const uint64_t T = (NS + J - 1) / J;
    if (NS >= 0x7fffffffULL || (T + 1) * (uint64_t)n >= 0xffffffffULL) return GBGPU_ECAPACITY;
    s->ntiles = (int64_t)T;
    if (ensure_tile_bufs(s, NS, T, n)) return ENOMEM;
    SKey *Sm = s->shi.as<SKey>();
    const uint32_t T32 = (uint32_t)T, NS32 = (uint32_t)NS;
    MCHECK(hipMemcpyAsync(dl, s->h_lists, sizeof(MList) * n, hipMemcpyHostToDevice, st));
    k_msample<<<cdiv(NS, MB), MB, 0, st>>>(dl, n, S, K, Sm, NS32);
    k_mrank<<<cdiv(NS, MB), MB, 0, st>>>(dl, n, Sm, NS32, s->tiles.as<uint32_t>());
    k_moff<<<cdiv((T + 1) * n, MB), MB, 0, st>>>(dl, n, S, J, K, Sm, s->tiles.as<uint32_t>(), T32,
                                                 s->off.as<uint32_t>());
    MCHECK(hipGetLastError());
    MCHECK(hipEventRecord(s->ev[2], st));
    k_mtile<<<T32, TB, 0, st>>>(dl, n, s->off.as<uint32_t>(), K, s->ts.as<TileSum>(), rm, s->arena.as<uint8_t>(),
                                dctl);
    MCHECK(hipEventRecord(s->ev[3], st));
    const int rc = finish_tiles(s, T32, maxoff, cap, out, dctl, n, K);
    if (rc != RETRY) return rc;
    if (S == 1) return GBGPU_ECAPACITY;  // > S equal keys in one run
    MCHECK(hipMemsetAsync(dctl, 0, sizeof(MCtl), st));
  }
}

static int run(MergeState *s, const uint8_t *const *lists, const int64_t *sizes, int nin, int rm, int64_t mrs,
               uint8_t *out, int64_t cap, int64_t *out_size) {
  *out_size = 0;
  s->nkeys = s->ntiles = 0;
  s->has_last = false;
  s->more = false;
  s->path = 0;
  std::fill(s->ms, s->ms + 6, 0.f);
  if (nin < 0 || nin > MAXN || cap < 0) return EINVAL;
  if (mrs == 0) return 0;
  if (((uintptr_t)out & 1) != 0) return EINVAL;
  int64_t total = 0;
  int n = 0;
  uint64_t units = 0;
  uint32_t nch = 0;
  for (int i = 0; i < nin; i++) {
    if (sizes[i] < 0) return EINVAL;
    if (sizes[i] == 0) continue;
    if (sizes[i] % 6 != 0) return GBGPU_ECORRUPT;
    if (sizes[i] / 6 > 0xffffffffLL) return GBGPU_ECAPACITY;
    if (((uintptr_t)lists[i] & 15) != 0) return EINVAL;
    MList &L = s->h_lists[n++];
    L = MList{};
    L.p = lists[i];
    L.size = (uint64_t)sizes[i];
    L.units = (uint32_t)(sizes[i] / 6);
    L.c0 = nch;
    L.koff = units;
    units += L.units;
    const uint64_t c = cdiv(L.units, MCH);
    if ((uint64_t)nch + c > 0x7fffffffULL) return GBGPU_ECAPACITY;
    nch += (uint32_t)c;
    total += sizes[i];
  }
  if (n == 0) return 0;
  const int64_t maxoff = std::max<int64_t>(max_offset(total, mrs, cap), 1);
  if (s->mlist.ensure(sizeof(MList) * MAXN) || s->dsum.ensure(sizeof(DSum) * nch) || s->ctl.ensure(sizeof(MCtl)))
    return ENOMEM;
  s->path = 2;
  const int rc = run_legacy(s, n, nch, units, rm, (uint64_t)maxoff, out, cap);
  if (rc) return rc;
  const uint32_t fl = s->h_ctl->flags;
  if (fl & F_CORRUPT) return GBGPU_ECORRUPT;
  // the reference loop refuses a key that would start within 18 bytes of the
  // end of the buffer (oracle/posdb_merge_oracle.c)
  if (s->h_ctl->out_end && s->h_ctl->last_start + 18 > (uint64_t)cap) return ENOSPC;
  *out_size = (int64_t)s->h_ctl->out_end;
  if (*out_size) {
    const uint64_t v[3] = {s->h_ctl->lk_b, s->h_ctl->lk_lo, s->h_ctl->lk_hi};
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 6; j++) s->last_key[6 * i + j] = (uint8_t)(v[i] >> (8 * j));
    s->has_last = true;
    s->more = (s->h_ctl->flags & F_MORE) != 0;
  }
  return 0;
}

int merge_device(MergeState *s, const uint8_t *const *lists, const int64_t *sizes, int n, int rm, int64_t mrs,
                 uint8_t *out, int64_t cap, int64_t *out_size) {
  if (!s || !out_size || (n > 0 && (!lists || !sizes))) return EINVAL;
  std::lock_guard<std::mutex> g(s->mu);
  return run(s, lists, sizes, n, rm, mrs, out, cap, out_size);
}

int merge_host(MergeState *s, const uint8_t *const *lists, const int64_t *sizes, int n, int rm, int64_t mrs,
               uint8_t *out, int64_t cap, int64_t *out_size) {
  if (!s || !out_size || (n > 0 && (!lists || !sizes)) || n < 0 || n > MAXN || cap < 0) return EINVAL;
  *out_size = 0;
  if (mrs == 0) return 0;
  std::lock_guard<std::mutex> g(s->mu);
  // the reference rejects a run whose first key is not 18 bytes
  int64_t total = 0;
  std::vector<size_t> at(n);
  size_t inb = 0;
  for (int i = 0; i < n; i++) {
    if (sizes[i] < 0) return EINVAL;
    if (sizes[i] > 0 && (lists[i][0] & 0x06)) return EINVAL;
    at[i] = inb;
    inb += ((size_t)sizes[i] + 255) & ~(size_t)255;
    total += sizes[i];
  }
  if (total == 0) return 0;
  const int64_t maxoff = std::max<int64_t>(max_offset(total, mrs, cap), 1);
  const size_t outb = (size_t)std::min<int64_t>(cap, maxoff + 18);
  if (s->in.ensure(inb + 256) || s->out.ensure(outb + 256)) return ENOMEM;
  std::vector<const uint8_t *> dptr(n);
  for (int i = 0; i < n; i++) {
    dptr[i] = s->in.as<uint8_t>(at[i]);
    if (sizes[i]) MCHECK(hipMemcpyAsync(s->in.as<uint8_t>(at[i]), lists[i], (size_t)sizes[i], hipMemcpyHostToDevice, s->st));
  }
  int rc = run(s, dptr.data(), sizes, n, rm, mrs, s->out.as<uint8_t>(), cap, out_size);
  if (rc) return rc;
  if (*out_size) MCHECK(hipMemcpy(out, s->out.p, (size_t)*out_size, hipMemcpyDeviceToHost));
  return 0;
}

int last_key(MergeState *s, uint8_t *key18, int32_t *more) {
  std::lock_guard<std::mutex> g(s->mu);
  if (more) *more = s->more ? 1 : 0;
  if (!s->has_last) return ENOENT;
  if (key18) std::memcpy(key18, s->last_key, 18);
  return 0;
}

void last_timings(MergeState *s, float *ms6, int64_t *nkeys, int64_t *ntiles) {
  std::lock_guard<std::mutex> g(s->mu);
  if (ms6) std::copy(s->ms, s->ms + 6, ms6);
  if (nkeys) *nkeys = s->nkeys;
  if (ntiles) *ntiles = s->ntiles;
}

int last_path(MergeState *s) {
  std::lock_guard<std::mutex> g(s->mu);
  return s->path;
}

}  // namespace gbmerge
