// Stable LSD radix sort (sisort.h), 8-bit digits, one pass per digit:
//   k_rs_hist    each block counts its tile's digits (LDS atomics) into a
//                digit-major table hist[digit][block];
//   k_rs_scan    one block turns the table into exclusive offsets: digit d of
//                block b starts after every smaller digit and after digit d
//                of blocks < b, which is what makes the pass stable;
//   k_rs_scatter each block walks its tile in rounds of 256 items; a wave
//                ranks its lanes among the lanes with the same digit with
//                8 ballots (no LDS atomics, so the order is the lane order),
//                the four waves' counts are prefix-summed in LDS, and every
//                item goes to its digit's running offset plus its rank.
// Keys and values ping-pong between (kout, vout) and the scratch pair, so
// the last pass lands in (kout, vout).
#include "sisort.h"

namespace gbgpu {
namespace {
constexpr int RS_T = 256;            // threads a block (four waves)
constexpr int RS_R = 16;             // rounds a tile
constexpr int RS_TILE = RS_T * RS_R; // items a block

__global__ void __launch_bounds__(RS_T) k_rs_hist(const uint64_t *k, uint32_t n, int shift, uint32_t nb,
                                                  uint32_t *hist) {
  __shared__ uint32_t c[256];
  c[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t base = blockIdx.x * RS_TILE;
  for (int r = 0; r < RS_R; r++) {
    const uint32_t i = base + r * RS_T + threadIdx.x;
    if (i < n) atomicAdd(&c[(uint32_t)(k[i] >> shift) & 255u], 1u);
  }
  __syncthreads();
  hist[(size_t)threadIdx.x * nb + blockIdx.x] = c[threadIdx.x];
}

// exclusive scan of `total` counts in place by one block of 1024 threads
__global__ void __launch_bounds__(1024) k_rs_scan(uint32_t *h, uint32_t total) {
  __shared__ uint32_t ws[16];
  const uint32_t per = (total + 1023) / 1024;
  const uint32_t b = threadIdx.x * per, e = min(total, b + per);
  uint32_t s = 0;
  for (uint32_t i = b; i < e; i++) s += h[i];
  // block exclusive scan of s
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
  }
  __syncthreads();
  uint32_t run = ws[w] + x - s;
  for (uint32_t i = b; i < e; i++) {
    const uint32_t t = h[i];
    h[i] = run;
    run += t;
  }
}

__global__ void __launch_bounds__(RS_T) k_rs_scatter(const uint64_t *kin, const uint32_t *vin, uint64_t *kout,
                                                     uint32_t *vout, uint32_t n, int shift, uint32_t nb,
                                                     const uint32_t *off) {
  __shared__ uint32_t run[256];
  __shared__ uint32_t cnt[4][256];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  run[t] = off[(size_t)t * nb + blockIdx.x];
  for (int x = 0; x < 4; x++) cnt[x][t] = 0;
  __syncthreads();
  const uint32_t base = blockIdx.x * RS_TILE;
  const uint64_t lt = (1ull << lane) - 1;
  for (int r = 0; r < RS_R; r++) {
    if (base + r * RS_T >= n) break;  // uniform over the block
    const uint32_t i = base + r * RS_T + t;
    const bool has = i < n;
    uint64_t key = has ? kin[i] : 0;
    const uint32_t val = has ? vin[i] : 0;
    const uint32_t d = (uint32_t)(key >> shift) & 255u;
    // the lanes holding the same digit: 8 ballots
    uint64_t peers = __ballot(has);
    for (int bit = 0; bit < 8; bit++) {
      const uint64_t b = __ballot((d >> bit) & 1u);
      peers &= ((d >> bit) & 1u) ? b : ~b;
    }
    const uint32_t rank = __popcll(peers & lt);
    if (has && rank == 0) cnt[w][d] = __popcll(peers);
    __syncthreads();
    if (has) {
      uint32_t pos = run[d] + rank;
      for (int x = 0; x < w; x++) pos += cnt[x][d];
      kout[pos] = key;
      vout[pos] = val;
    }
    __syncthreads();
    run[t] += cnt[0][t] + cnt[1][t] + cnt[2][t] + cnt[3][t];
    for (int x = 0; x < 4; x++) cnt[x][t] = 0;
    __syncthreads();
  }
}

size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }
}  // namespace

hipError_t si_sort_pairs(void *tmp, size_t &tmp_bytes, const uint64_t *kin, uint64_t *kout, const uint32_t *vin,
                         uint32_t *vout, uint32_t n, hipStream_t st, int end_bit) {
  const uint32_t nb = n ? (n + RS_TILE - 1) / RS_TILE : 1;
  const size_t need = al256(8 * (size_t)n) + al256(4 * (size_t)n) + al256(4 * 256 * (size_t)nb) + 256;
  if (!tmp) {
    tmp_bytes = need;
    return hipSuccess;
  }
  if (tmp_bytes < need) return hipErrorInvalidValue;
  if (n == 0) return hipSuccess;
  uint8_t *p = static_cast<uint8_t *>(tmp);
  uint64_t *k2 = reinterpret_cast<uint64_t *>(p);
  uint32_t *v2 = reinterpret_cast<uint32_t *>(p + al256(8 * (size_t)n));
  uint32_t *hist = reinterpret_cast<uint32_t *>(p + al256(8 * (size_t)n) + al256(4 * (size_t)n));
  const int passes = end_bit <= 0 ? 0 : (end_bit + 7) / 8;
  // the pass count decides where the ping-pong starts so the last lands in
  // (kout, vout); a single pass reads the input directly
  const uint64_t *ks = kin;
  const uint32_t *vs = vin;
  for (int ps = 0; ps < passes; ps++) {
    const bool to_out = ((passes - 1 - ps) % 2) == 0;
    uint64_t *kd = to_out ? kout : k2;
    uint32_t *vd = to_out ? vout : v2;
    hipLaunchKernelGGL(k_rs_hist, dim3(nb), dim3(RS_T), 0, st, ks, n, 8 * ps, nb, hist);
    hipLaunchKernelGGL(k_rs_scan, dim3(1), dim3(1024), 0, st, hist, 256u * nb);
    hipLaunchKernelGGL(k_rs_scatter, dim3(nb), dim3(RS_T), 0, st, ks, vs, kd, vd, n, 8 * ps, nb, hist);
    ks = kd;
    vs = vd;
  }
  if (passes == 0 && n) {
    hipError_t e = hipMemcpyAsync(kout, kin, 8 * (size_t)n, hipMemcpyDeviceToDevice, st);
    if (e == hipSuccess) e = hipMemcpyAsync(vout, vin, 4 * (size_t)n, hipMemcpyDeviceToDevice, st);
    return e;
  }
  return hipGetLastError();
}
}  // namespace gbgpu
