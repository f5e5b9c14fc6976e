// Per-docid scoring of PosdbTable::intersectLists10_r, device side.
//
// A docid's mini-merged lists (Posdb.cpp:6559-6778) are held as 8-byte
// records: the low 6 bytes are the rewritten posdb key bytes 0..5 (density,
// word position, hash group, spam rank, diversity, F bits).  Every scorer
// below restates its reference function over record indices instead of
// char pointers; expression shapes (float vs double promotion, operand
// order) follow the reference exactly so results round identically
// (compiled with -ffp-contract=off).
//
// Register residency: the per-docid state of the reference (top-10 score
// slots, window cursors, per-term best positions) is kept in fixed-size
// register arrays -- every loop over them is unrolled to a compile-time bound
// and runtime indices go through rget/rset select chains -- so nothing spills
// to scratch.  NQ (the kernel's group capacity) is a template parameter; the
// term-pair score matrix lives in LDS, one column per lane.
#ifndef GBGPU_SCORING_H
#define GBGPU_SCORING_H

#include <stdint.h>

#include "plan.h"

namespace gbgpu {

constexpr int MAX_TOP = 10;          // Posdb.h:817
constexpr int FIXED_DISTANCE = 400;  // Posdb.h:765
#define GB_SYNONYM_WEIGHT 0.90       /* Posdb.h:94 */
#define GB_WIKI_WEIGHT 0.10          /* Posdb.h:95 */
#define GB_WIKI_BIGRAM_WEIGHT 1.40   /* Posdb.h:115 */
#define GB_SITERANKMULTIPLIER 0.33333333 /* Posdb.h:97 */

// initWeights tables (Posdb.cpp:1094-1197), filled on the host
struct Weights {
  float diversity[16];
  float density[32];
  float wordspam[16];
  float linker[16];
  float hashgroup[16];
  uint8_t in_body[16];
  uint8_t compatible[16][16];
};

// The tables as every scoring kernel reads them: staged into LDS at kernel
// start (stage_weights), so a lookup by a per-lane index is one ds_read
// instead of a dependent global load.
__shared__ Weights s_weights;

__device__ __forceinline__ void stage_weights(const Weights *src) {
  static_assert(sizeof(Weights) % 4 == 0, "Weights is copied as words");
  for (int i = threadIdx.x; i < (int)(sizeof(Weights) / 4); i += blockDim.x)
    reinterpret_cast<uint32_t *>(&s_weights)[i] = reinterpret_cast<const uint32_t *>(src)[i];
  __syncthreads();
}

// record field accessors (Posdb.h:319-361 on key bytes 0..5)
__host__ __device__ __forceinline__ uint32_t r_wordpos(uint64_t r) { return (uint32_t)(r >> 30) & 0x3ffff; }
__host__ __device__ __forceinline__ uint32_t r_hg(uint64_t r) { return (uint32_t)(r >> 26) & 0xf; }
__host__ __device__ __forceinline__ uint32_t r_wsr(uint64_t r) { return (uint32_t)(r >> 22) & 0xf; }
__host__ __device__ __forceinline__ uint32_t r_div(uint64_t r) { return (uint32_t)(r >> 18) & 0xf; }
__host__ __device__ __forceinline__ uint32_t r_syn(uint64_t r) { return (uint32_t)(r >> 16) & 0x3; }
__host__ __device__ __forceinline__ uint32_t r_hswb(uint64_t r) { return (uint32_t)(r >> 16) & 0x1; }
__host__ __device__ __forceinline__ uint32_t r_dens(uint64_t r) { return (uint32_t)(r >> 11) & 0x1f; }

// score /= (dist + 1.0) of the reference: a float promoted to double,
// divided, rounded back to float.  dist + 1 is an integer below 2^24, exact
// in either precision, and rounding a double quotient of two floats to float
// gives the correctly rounded float quotient (53 >= 2 * 24 + 2: double
// rounding is innocuous for division), so one IEEE float division yields the
// same bits without the f64 divide sequence.
template <class D>
__device__ __forceinline__ float div_dist(float score, D dist) {
  return score / (float)(dist + 1);
}

// register-array access with a runtime index (unrolled select chains)
template <int N, class T>
__device__ __forceinline__ T rget(const T (&a)[N], int i) {
  T v = a[0];
#pragma unroll
  for (int q = 1; q < N; q++) v = (q == i) ? a[q] : v;
  return v;
}
template <int N, class T>
__device__ __forceinline__ void rset(T (&a)[N], int i, T v) {
#pragma unroll
  for (int q = 0; q < N; q++)
    if (q == i) a[q] = v;
}

// The largest v (0..15) among the wave's active lanes, as a wave-uniform
// value (four ballots).  The scorers' top lists bound their unrolled slot
// loops with it: a lane fills at most min(m_realMaxTop, steps) slots, so the
// slots past the wave's largest such count are never touched and their
// iterations are skipped with one scalar branch each.
__device__ __forceinline__ int wave_max15(int v) {
  int m = 0;
#pragma unroll
  for (int s = 8; s >= 1; s >>= 1)
    if (__ballot(v >= m + s)) m += s;
  return m;
}

// The top lists' modified hash groups, packed 4 bits a slot (hash groups are
// 4-bit fields): the lowest slot below n whose nibble equals v is found with
// the zero-nibble test on pm ^ v*0x11..1 -- a borrow can only flag nibbles
// ABOVE a zero one, so the lowest flag is exact -- instead of a per-slot loop.
constexpr uint64_t NIB1 = 0x1111111111111111ull, NIB8 = 0x8888888888888888ull;
__device__ __forceinline__ uint64_t nib_match(uint64_t pm, uint32_t v, int n) {
  const uint64_t x = pm ^ ((uint64_t)v * NIB1);
  const uint64_t z = (x - NIB1) & ~x & NIB8;
  return n >= 16 ? z : z & ((1ull << (4 * n)) - 1);
}
__device__ __forceinline__ uint64_t nib_set(uint64_t pm, int q, uint32_t v) {
  return (pm & ~(0xfull << (4 * q))) | ((uint64_t)v << (4 * q));
}

// index of pair (i, j), i < j, in the upper triangle of an NQ x NQ matrix
template <int NQ>
__device__ __forceinline__ int pair_index(int i, int j) {
  return i * (2 * NQ - i - 1) / 2 + (j - i - 1);
}
template <int NQ>
constexpr int npairs() {
  return NQ * (NQ - 1) / 2;
}

// Where one docid's records live.  RP is one of these two record stores, so
// every record access compiles to a ds_read/ds_write or a global load/store,
// never a flat one.
//  LdsRecs:    the lane's column of the wave's LDS record arrays, [cap][S]
//              for S survivors per wave (48-bit records split 32 + 16 bits;
//              consecutive lanes hit consecutive banks, so a wave's record
//              reads are conflict-free);
//  GlobalRecs: a contiguous range of the global record arena.
struct LdsRecs {
  __attribute__((address_space(3))) uint32_t *lo;
  __attribute__((address_space(3))) uint16_t *hi;
  int sh;   // log2 of the column stride (the survivors sharing the wave's arrays)
  int cap;  // records the column holds
  __device__ __forceinline__ uint64_t operator[](int r) const {
    return (uint64_t)lo[r << sh] | ((uint64_t)hi[r << sh] << 32);
  }
  __device__ __forceinline__ void put(int r, uint64_t v) const {
    lo[r << sh] = (uint32_t)v;
    hi[r << sh] = (uint16_t)(v >> 32);
  }
};
struct GlobalRecs {
  __attribute__((address_space(1))) uint64_t *p;
  __device__ __forceinline__ uint64_t operator[](int r) const { return p[r]; }
  __device__ __forceinline__ void put(int r, uint64_t v) const { p[r] = v; }
};

// What one docid's scorer sees: nq groups, each a record range in rec.
template <int NQ, class RP>
struct DocView {
  RP rec;  // records (ranges are indices into rec)
  int beg[NQ], end[NQ];
  uint32_t present;     // bit i: miniMergedList[i] != NULL (positive group)
};

template <int NQ>
struct ScoreCtx {
  const Weights *w;
  const DevPlan *pl;
  int nq;
  int realMaxTop;
  int qdist;             // PosdbTable::m_qdist (set by evalSlidingWindow)
  float bestWindowScore; // m_bestWindowScore
  int window[NQ];        // m_windowTermPtrs (record index, -1 = NULL)
  float *sm;             // score matrix column of this lane (LDS), stride smStride
  int smStride;
  uint32_t excl;         // bit i: group i is piped/negative/number/facet (BF_EXCLUDE)
};

// The second pass's score info (pdcs != NULL, Posdb.cpp:3247-3298,
// 4195-4280): a recorder receives each scorer's top list.  NoRec (the first
// pass) compiles away; ScoreRec writes the reference's SingleScore /
// PairScore records (include/gbgpu.h mirrors) for one docid.
struct NoRec {
  static constexpr bool on = false;
  __device__ void single(const DevPlan *, int, float, uint64_t) {}
  __device__ void pair(const DevPlan *, int, int, float, float, int32_t, uint64_t, uint64_t, uint8_t) {}
};

// getSingleTermScore, Posdb.cpp:3087-3301.  bestPos = record index of the
// best non-body occurrence or -1; REC receives the top list (pdcs path).
// T: the top list's register capacity, a bound the caller guarantees on the
// slots it can fill -- min(m_realMaxTop, the group's records) -- so the
// unrolled bookkeeping below costs T steps per record, not MAX_TOP.
template <int NQ, class RP, class REC = NoRec, int T = MAX_TOP>
__device__ __forceinline__ float single_term_score(const ScoreCtx<NQ> &c, const DocView<NQ, RP> &d, int i, int *bestPos,
                                                  REC *rec = nullptr, int tw = T) {
  const Weights &W = s_weights;
  float nonBodyMax = -1.0;
  int minx = 0;
  float minv = 0.0f;  // bestScores[minx]
  float bestScores[T];
  int bestwpi[REC::on ? T : 1];
  uint64_t bestmhg = 0;  // slot q's modified hash group: nibble q (slots < numTop)
  uint32_t besths = 0;  // bit q: slot q's key is a half-stop wiki bigram (r_hswb)
#pragma unroll
  for (int q = 0; q < T; q++) {
    bestScores[q] = 0.0f;
    if constexpr (REC::on) bestwpi[q] = 0;
  }
  int numTop = 0;
  int bp = -1;
  const int rmt = c.realMaxTop;
  // a do-while, as the reference's loop (Posdb.cpp:3117-3206): an empty
  // mini-merged list still has its first key read -- the next group's
  // first key, written at the same place (see score_survivor)
  const int e = rget(d.end, i);
  int r = rget(d.beg, i);
  do {
    const uint64_t k = d.rec[r];
    float score = 100.0;
    const uint32_t div = r_div(k);
    score *= W.diversity[div];
    score *= W.diversity[div];
    const uint32_t hg = r_hg(k);
    uint32_t mhg = hg;
    if (W.in_body[mhg]) mhg = GB_HG_BODY;
    score *= W.hashgroup[hg];
    score *= W.hashgroup[hg];
    const uint32_t dens = r_dens(k);
    score *= W.density[dens];
    score *= W.density[dens];
    const uint32_t wspam = r_wsr(k);
    if (hg == GB_HG_INLINKTEXT) {
      score *= W.linker[wspam];
      score *= W.linker[wspam];
    } else {
      score *= W.wordspam[wspam];
      score *= W.wordspam[wspam];
    }
    if (r_syn(k)) {
      score *= GB_SYNONYM_WEIGHT;
      score *= GB_SYNONYM_WEIGHT;
    }
    // same modified hash group already in the top list (not inlink text)
    int bro = -1;
    float broScore = 0.0f;
    if (hg != GB_HG_INLINKTEXT) {
      const uint64_t z = nib_match(bestmhg, mhg, numTop);  // lowest matching slot
      if (z) {
        bro = (int)(__builtin_ctzll(z) >> 2);
#pragma unroll
        for (int q = 0; q < T; q++) {
          if (q >= tw) break;  // wave-uniform: no lane holds slot q
          if (q == bro) broScore = bestScores[q];
        }
      }
    }
    int slot = -1;
    if (bro >= 0) {
      if (score > broScore) slot = bro;
    } else if (numTop < rmt) {
      slot = numTop;
      numTop++;
    } else if (score > minv) {
      slot = minx;
    }
#pragma unroll
    for (int q = 0; q < T; q++) {
      if (q == slot) {
        bestScores[q] = score;
        if constexpr (REC::on) bestwpi[q] = r;
      }
    }
    if (slot >= 0) {
      besths = (besths & ~(1u << slot)) | (r_hswb(k) << slot);
      bestmhg = nib_set(bestmhg, slot, mhg);
    }
    if (numTop >= rmt) {
      minx = 0;
      minv = bestScores[0];
#pragma unroll
      for (int q = 1; q < T; q++) {
        if (q >= tw) break;  // rmt <= numTop <= tw here
        if (q < rmt && !(bestScores[q] > minv)) {
          minx = q;
          minv = bestScores[q];
        }
      }
    }
    if (score > nonBodyMax && !W.in_body[hg]) {
      nonBodyMax = score;
      bp = r;
    }
  } while (++r < e);
  *bestPos = bp;
  float sum = 0.0;
#pragma unroll
  for (int q = 0; q < T; q++) {
    if (q >= tw) break;
    if (q < numTop) {
      if (besths >> q & 1)
        sum += (bestScores[q] * GB_WIKI_BIGRAM_WEIGHT * GB_WIKI_BIGRAM_WEIGHT);
      else
        sum += bestScores[q];
    }
  }
  sum *= c.pl->tfw[i];
  sum *= c.pl->tfw[i];
  if constexpr (REC::on) {
    for (int q = 0; q < T; q++)
      if (q < numTop) rec->single(c.pl, i, bestScores[q], d.rec[rget(bestwpi, q)]);
  }
  return sum;
}

// getTermPairScoreForNonBody, Posdb.cpp:3305-3555
template <int NQ, class RP>
__device__ __forceinline__ float pair_score_nonbody(const ScoreCtx<NQ> &c, const DocView<NQ, RP> &d, int i, int j, int qdist) {
  const Weights &W = s_weights;
  int wi = rget(d.beg, i), wj = rget(d.beg, j);
  const int endi = rget(d.end, i), endj = rget(d.end, j);
  uint64_t ki = d.rec[wi], kj = d.rec[wj];
  int32_t p1 = (int32_t)r_wordpos(ki), p2 = (int32_t)r_wordpos(kj);
  uint32_t hg1 = r_hg(ki), hg2 = r_hg(kj);
  float spamw1 = (hg1 == GB_HG_INLINKTEXT) ? W.linker[r_wsr(ki)] : W.wordspam[r_wsr(ki)];
  float spamw2 = (hg2 == GB_HG_INLINKTEXT) ? W.linker[r_wsr(kj)] : W.wordspam[r_wsr(kj)];
  float denw1 = W.density[r_dens(ki)];
  float denw2 = W.density[r_dens(kj)];
  float max = -1.0;
  float score;
  int32_t dist;
  for (;;) {
    if (p1 <= p2) {
      if (W.compatible[hg1][hg2]) {
        dist = p2 - p1;
        if (dist < 2) dist = 2;
        if (dist > 50) dist = FIXED_DISTANCE;
        if (dist >= qdist) dist = dist - qdist;
        score = 100 * denw1 * denw2;
        score *= W.hashgroup[hg1];
        score *= W.hashgroup[hg2];
        if (r_syn(ki)) score *= GB_SYNONYM_WEIGHT;
        if (r_syn(kj)) score *= GB_SYNONYM_WEIGHT;
        score *= spamw1 * spamw2;
        score = div_dist(score, dist);
        if (score > max) max = score;
      }
      if (++wi >= endi) break;
      ki = d.rec[wi];
      p1 = (int32_t)r_wordpos(ki);
      hg1 = r_hg(ki);
      denw1 = W.density[r_dens(ki)];
      spamw1 = (hg1 == GB_HG_INLINKTEXT) ? W.linker[r_wsr(ki)] : W.wordspam[r_wsr(ki)];
    } else {
      if (W.compatible[hg1][hg2]) {
        dist = p1 - p2;
        if (dist < 2) dist = 2;
        if (dist > 50) dist = FIXED_DISTANCE;
        if (dist >= qdist) {
          dist = dist - qdist;
          dist += qdist - 1;
        } else {
          dist += 1;
        }
        score = 100 * denw1 * denw2;
        score *= W.hashgroup[hg1];
        score *= W.hashgroup[hg2];
        if (r_syn(ki)) score *= GB_SYNONYM_WEIGHT;
        if (r_syn(kj)) score *= GB_SYNONYM_WEIGHT;
        score *= spamw1 * spamw2;
        score = div_dist(score, dist);
        if (score > max) max = score;
      }
      if (++wj >= endj) break;
      kj = d.rec[wj];
      p2 = (int32_t)r_wordpos(kj);
      hg2 = r_hg(kj);
      denw2 = W.density[r_dens(kj)];
      spamw2 = (hg2 == GB_HG_INLINKTEXT) ? W.linker[r_wsr(kj)] : W.wordspam[r_wsr(kj)];
    }
  }
  return max;
}

// getTermPairScoreForWindow, Posdb.cpp:3557-3625 (record index -1 = NULL)
template <class RP>
__device__ __forceinline__ float pair_score_window(const Weights &W, int cqdist, RP rec, int wpi, int wpj,
                                          int32_t fixedDistance) {
  if (wpi < 0) return -1.00;
  if (wpj < 0) return -1.00;
  const uint64_t ki = rec[wpi], kj = rec[wpj];
  const int32_t p1 = (int32_t)r_wordpos(ki), p2 = (int32_t)r_wordpos(kj);
  const uint32_t hg1 = r_hg(ki), hg2 = r_hg(kj);
  const float spamw1 = (hg1 == GB_HG_INLINKTEXT) ? W.linker[r_wsr(ki)] : W.wordspam[r_wsr(ki)];
  const float spamw2 = (hg2 == GB_HG_INLINKTEXT) ? W.linker[r_wsr(kj)] : W.wordspam[r_wsr(kj)];
  const float denw1 = W.density[r_dens(ki)];
  const float denw2 = W.density[r_dens(kj)];
  float dist, score;
  if (fixedDistance != 0) {
    dist = fixedDistance;
  } else {
    if (p2 < p1) dist = p1 - p2;
    else dist = p2 - p1;
    if (dist < 2) dist = 2;
    if (dist >= cqdist) dist = dist - cqdist;
    if (p2 < p1) dist += 1;
  }
  score = 100 * denw1 * denw2;
  score *= W.hashgroup[hg1];
  score *= W.hashgroup[hg2];
  if (r_syn(ki)) score *= GB_SYNONYM_WEIGHT;
  if (r_syn(kj)) score *= GB_SYNONYM_WEIGHT;
  score *= spamw1 * spamw2;
  score = div_dist(score, dist);
  return score;
}

// One occurrence as getTermPairScoreForWindow reads it: its word position
// and weight factors, looked up once per record instead of per pair call.
struct WinRec {
  int32_t p;
  float spamw, denw, hgw;
  bool syn, valid;
};
__device__ __forceinline__ WinRec win_rec(const Weights &W, uint64_t k) {
  WinRec r;
  const uint32_t hg = r_hg(k);
  r.p = (int32_t)r_wordpos(k);
  r.spamw = (hg == GB_HG_INLINKTEXT) ? W.linker[r_wsr(k)] : W.wordspam[r_wsr(k)];
  r.denw = W.density[r_dens(k)];
  r.hgw = W.hashgroup[hg];
  r.syn = r_syn(k) != 0;
  r.valid = true;
  return r;
}
// pair_score_window on WinRecs (same expression order, so the same bits)
__device__ __forceinline__ float pair_score_window_rec(int cqdist, const WinRec &a, const WinRec &b,
                                                      int32_t fixedDistance) {
  if (!a.valid) return -1.00;
  if (!b.valid) return -1.00;
  float dist, score;
  if (fixedDistance != 0) {
    dist = fixedDistance;
  } else {
    if (b.p < a.p) dist = a.p - b.p;
    else dist = b.p - a.p;
    if (dist < 2) dist = 2;
    if (dist >= cqdist) dist = dist - cqdist;
    if (b.p < a.p) dist += 1;
  }
  score = 100 * a.denw * b.denw;
  score *= a.hgw;
  score *= b.hgw;
  if (a.syn) score *= GB_SYNONYM_WEIGHT;
  if (b.syn) score *= GB_SYNONYM_WEIGHT;
  score *= a.spamw * b.spamw;
  score = div_dist(score, dist);
  return score;
}

// evalSlidingWindow, Posdb.cpp:1275-1511
template <int NQ, class RP>
__device__ __forceinline__ void eval_window(ScoreCtx<NQ> &c, const DocView<NQ, RP> &d, const int (&ptrs)[NQ],
                                   const int (&bestPos)[NQ]) {
  const Weights &W = s_weights;
  const DevPlan *pl = c.pl;
  float minTermPairScoreInWindow = 999999999.0;
  const int nr = c.nq;
  for (int i = 0; i < nr; i++) {
    if ((c.excl >> i & 1)) continue;
    const int wpi = rget(ptrs, i);
    const int bpi = rget(bestPos, i);
    for (int j = i + 1; j < nr; j++) {
      if ((c.excl >> j & 1)) continue;
      const int wpj = rget(ptrs, j);
      const int bpj = rget(bestPos, j);
      float wikiWeight;
      if (pl->wiki[j] == pl->wiki[i] && pl->wiki[j]) {
        c.qdist = pl->qpos[j] - pl->qpos[i];
        wikiWeight = GB_WIKI_WEIGHT;
      } else {
        c.qdist = 2;
        wikiWeight = 1.0;
      }
      float max = pair_score_window(W, c.qdist, d.rec, wpi, wpj, 0);
      float score = pair_score_window(W, c.qdist, d.rec, bpi, wpj, FIXED_DISTANCE);
      if (score > max) max = score;
      score = pair_score_window(W, c.qdist, d.rec, bpi, bpj, FIXED_DISTANCE);
      if (score > max) max = score;
      score = pair_score_window(W, c.qdist, d.rec, wpi, bpj, FIXED_DISTANCE);
      if (score > max) max = score;
      if (wikiWeight != 1.0) max *= wikiWeight;
      max *= pl->tfw[i] * pl->tfw[j];
      const float smv = c.sm[pair_index<NQ>(i, j) * c.smStride];
      if (smv > max) max = smv;
      if (pl->quote[j] >= 0 && pl->quote[j] == pl->quote[i]) {
        if (wpi < 0) {
          max = -1.0;
        } else if (wpj < 0) {
          max = -1.0;
        } else {
          const int32_t qd = pl->qpos[j] - pl->qpos[i];
          const int32_t p1 = (int32_t)r_wordpos(d.rec[wpi]);
          const int32_t p2 = (int32_t)r_wordpos(d.rec[wpj]);
          const int32_t dist = p2 - p1;
          if (dist < 0) max = -1.0;
          else if (dist > qd && dist - qd > 1) max = -1.0;
          else if (dist < qd && qd - dist > 1) max = -1.0;
        }
      }
      if (max < minTermPairScoreInWindow) minTermPairScoreInWindow = max;
    }
  }
  if (minTermPairScoreInWindow <= c.bestWindowScore) return;
  c.bestWindowScore = minTermPairScoreInWindow;
#pragma unroll
  for (int q = 0; q < NQ; q++) c.window[q] = ptrs[q];
}

// getTermPairScoreForAny, Posdb.cpp:3631-4344 (T as in single_term_score:
// a bound on the slots the pair's records can fill); REC receives the top pairs
// (pdcs path, 4195-4280) with their record indices and fixedDistance flag --
// which the reference only assigns when dist < 50 or the distance is fixed,
// so it carries over from the previous scored pair of the call otherwise; a
// pair scored before any assignment in the call reads the reference's
// uninitialised local (Posdb.cpp:3730), recorded here as 2
template <int NQ, class RP, class REC = NoRec, int T = MAX_TOP>
__device__ __forceinline__ float pair_score_any(const ScoreCtx<NQ> &c, const DocView<NQ, RP> &d, int i, int j,
                                               REC *rec = nullptr, int tw = T) {
  const Weights &W = s_weights;
  const DevPlan *pl = c.pl;
  float wts;
  int32_t qdist;
  if (pl->wiki[j] == pl->wiki[i] && pl->wiki[j]) {
    qdist = pl->qpos[j] - pl->qpos[i];
    wts = (float)GB_WIKI_WEIGHT;
  } else {
    qdist = 2;
    wts = 1.0;
  }
  const bool inSameQuotedPhrase = (pl->quote[i] == pl->quote[j] && pl->quote[i] >= 0);
  if (inSameQuotedPhrase) qdist = pl->qpos[j] - pl->qpos[i];
  const int wini = rget(c.window, i), winj = rget(c.window, j);
  int wi = rget(d.beg, i), wj = rget(d.beg, j);
  const int endi = rget(d.end, i), endj = rget(d.end, j);
  uint64_t ki = d.rec[wi], kj = d.rec[wj];
  int32_t p1 = (int32_t)r_wordpos(ki), p2 = (int32_t)r_wordpos(kj);
  uint32_t hg1 = r_hg(ki), hg2 = r_hg(kj);
  uint32_t mhg1 = W.in_body[hg1] ? GB_HG_BODY : hg1;
  uint32_t mhg2 = W.in_body[hg2] ? GB_HG_BODY : hg2;
  float spamw1 = (hg1 == GB_HG_INLINKTEXT) ? W.linker[r_wsr(ki)] : W.wordspam[r_wsr(ki)];
  float spamw2 = (hg2 == GB_HG_INLINKTEXT) ? W.linker[r_wsr(kj)] : W.wordspam[r_wsr(kj)];
  float denw1 = W.density[r_dens(ki)];
  float denw2 = W.density[r_dens(kj)];
  float score = 0.0f;
  int minx = -1;
  float minv = 0.0f;  // bestScores[minx]
  float bestScores[T];
  uint64_t bestmhg1 = 0, bestmhg2 = 0;  // nibble q: slot q's modified hash groups
  int bestwpi[REC::on ? T : 1], bestwpj[REC::on ? T : 1];
  uint8_t bestFixed[REC::on ? T : 1];
  bool fixedDistance = false;
  bool fixedSet = false;  // fixedDistance assigned in this call
#pragma unroll
  for (int q = 0; q < T; q++) {
    bestScores[q] = 0.0f;
    if constexpr (REC::on) {
      bestwpi[q] = bestwpj[q] = 0;
      bestFixed[q] = 0;
    }
  }
  int numTop = 0;
  const int rmt = c.realMaxTop;
  int32_t dist;
  for (;;) {
    bool adv1;
    bool scored = false;
    if (W.in_body[hg1] && wi != wini) {
      adv1 = true;
    } else if (W.in_body[hg2] && wj != winj) {
      adv1 = false;
    } else if (p1 <= p2) {
      adv1 = true;
      dist = p2 - p1;
      bool skip = false;
      if (inSameQuotedPhrase) {
        if (dist > qdist && dist - qdist >= 2) skip = true;
        if (dist < qdist && qdist - dist >= 2) skip = true;
      }
      if (!skip) {
        const uint32_t syn1 = r_syn(ki), syn2 = r_syn(kj);
        if (dist < 2) dist = 2;
        if (dist < 50) {
          fixedDistance = false;
          fixedSet = true;
        } else if (mhg1 != mhg2) {
          dist = FIXED_DISTANCE;
          fixedDistance = true;
          fixedSet = true;
        } else if (mhg1 == GB_HG_INLINKTEXT) {
          dist = FIXED_DISTANCE;
          fixedDistance = true;
          fixedSet = true;
        }
        if (dist >= qdist) dist = dist - qdist;
        score = 100 * denw1 * denw2;
        score *= W.hashgroup[hg1];
        score *= W.hashgroup[hg2];
        if (syn1) score *= GB_SYNONYM_WEIGHT;
        if (syn2) score *= GB_SYNONYM_WEIGHT;
        if (r_hswb(ki)) score *= GB_WIKI_BIGRAM_WEIGHT;
        if (r_hswb(kj)) score *= GB_WIKI_BIGRAM_WEIGHT;
        score *= spamw1 * spamw2;
        score = div_dist(score, dist);
        scored = true;
      }
    } else {
      adv1 = false;
      dist = p1 - p2;
      if (!inSameQuotedPhrase) {
        if (dist < 2) dist = 2;
        if (dist < 50) {
          fixedDistance = false;
          fixedSet = true;
        } else if (mhg1 != mhg2) {
          dist = FIXED_DISTANCE;
          fixedDistance = true;
          fixedSet = true;
        } else if (mhg1 == GB_HG_INLINKTEXT) {
          dist = FIXED_DISTANCE;
          fixedDistance = true;
          fixedSet = true;
        }
        if (dist >= qdist) {
          dist = dist - qdist;
          dist += qdist - 1;
        } else {
          dist += 1;
        }
        score = 100 * denw1 * denw2;
        score *= W.hashgroup[hg1];
        score *= W.hashgroup[hg2];
        if (r_syn(ki)) score *= GB_SYNONYM_WEIGHT;
        if (r_syn(kj)) score *= GB_SYNONYM_WEIGHT;
        score *= spamw1 * spamw2;
        score = div_dist(score, dist);
        scored = true;
      }
    }
    if (scored) {  // the topScores block, Posdb.cpp:3875-3922
      int bro = -1;
      float broScore = 0.0f;
      // the lowest slot matching either modified hash group (not inlink text)
      uint64_t z = 0;
      if (hg1 != GB_HG_INLINKTEXT) z |= nib_match(bestmhg1, mhg1, numTop);
      if (hg2 != GB_HG_INLINKTEXT) z |= nib_match(bestmhg2, mhg2, numTop);
      if (z) {
        bro = (int)(__builtin_ctzll(z) >> 2);
#pragma unroll
        for (int q = 0; q < T; q++) {
          if (q >= tw) break;  // wave-uniform: no lane holds slot q
          if (q == bro) broScore = bestScores[q];
        }
      }
      int slot = -1;
      if (bro >= 0) {
        if (score > broScore) slot = bro;
      } else if (numTop < rmt) {
        slot = numTop;
        numTop++;
      } else if (score > minv) {
        slot = minx;
      }
#pragma unroll
      for (int q = 0; q < T; q++) {
        if (q == slot) {
          bestScores[q] = score;
          if constexpr (REC::on) {
            bestwpi[q] = wi;
            bestwpj[q] = wj;
            bestFixed[q] = fixedSet ? (fixedDistance ? 1 : 0) : 2;
          }
        }
      }
      if (slot >= 0) {
        bestmhg1 = nib_set(bestmhg1, slot, mhg1);
        bestmhg2 = nib_set(bestmhg2, slot, mhg2);
      }
      if (numTop >= rmt) {
        minx = 0;
        minv = bestScores[0];
#pragma unroll
        for (int q = 1; q < T; q++) {
          if (q >= tw) break;  // rmt <= numTop <= tw here
          if (q < rmt && !(bestScores[q] > minv)) {
            minx = q;
            minv = bestScores[q];
          }
        }
      }
    }
    if (adv1) {
      if (++wi >= endi) break;
      ki = d.rec[wi];
      p1 = (int32_t)r_wordpos(ki);
      hg1 = r_hg(ki);
      mhg1 = W.in_body[hg1] ? GB_HG_BODY : hg1;
      denw1 = W.density[r_dens(ki)];
      spamw1 = (hg1 == GB_HG_INLINKTEXT) ? W.linker[r_wsr(ki)] : W.wordspam[r_wsr(ki)];
    } else {
      if (++wj >= endj) break;
      kj = d.rec[wj];
      p2 = (int32_t)r_wordpos(kj);
      hg2 = r_hg(kj);
      mhg2 = W.in_body[hg2] ? GB_HG_BODY : hg2;
      denw2 = W.density[r_dens(kj)];
      spamw2 = (hg2 == GB_HG_INLINKTEXT) ? W.linker[r_wsr(kj)] : W.wordspam[r_wsr(kj)];
    }
  }
  float sum = 0.0;
#pragma unroll
  for (int q = 0; q < T; q++) {
    if (q >= tw) break;
    if (q < numTop) sum += bestScores[q];
  }
  sum *= wts;
  sum *= pl->tfw[i];
  sum *= pl->tfw[j];
  if constexpr (REC::on) {
    for (int q = 0; q < T; q++)
      if (q < numTop)
        rec->pair(pl, i, j, bestScores[q], wts, qdist, d.rec[rget(bestwpi, q)], d.rec[rget(bestwpj, q)],
                  rget(bestFixed, q));
  }
  return sum;
}

// The per-docid body of intersectLists10_r after the mini merges
// (Posdb.cpp:6847-7257).  Returns false when the docid is not scored
// (minScore <= 0); siteRank/docLang come from the first key of the first
// present group (Posdb.cpp:6985-7003).  sm: this lane's score-matrix column
// (npairs<NQ>() floats at stride smStride).
template <int NQ, class RP, class REC = NoRec, int T = MAX_TOP>
__device__ __forceinline__ bool score_doc(const Weights *w, const DevPlan *pl, const DocView<NQ, RP> &d, int siteRank, int docLang,
                                 float *sm, int smStride, float *outScore, int stop = 0, REC *rec = nullptr) {
  ScoreCtx<NQ> c;
  c.w = w;
  c.pl = pl;
  c.nq = pl->ngroups;
  c.realMaxTop = pl->real_max_top;
  c.qdist = 2;
  c.sm = sm;
  c.smStride = smStride;
  c.excl = 0;
  for (int i = 0; i < c.nq; i++)
    if (pl->gflags0[i] & BF_EXCLUDE) c.excl |= 1u << i;
  int bestPos[NQ];
  // non-body pair scores, Posdb.cpp:6847-6926
  for (int i = 0; i < c.nq; i++) {
    if ((c.excl >> i & 1)) continue;
    for (int j = i + 1; j < c.nq; j++) {
      if ((c.excl >> j & 1)) continue;
      int32_t qdist;
      float wts;
      if (pl->wiki[j] == pl->wiki[i] && pl->wiki[j]) {
        qdist = pl->qpos[j] - pl->qpos[i];
        wts = (float)GB_WIKI_WEIGHT;
      } else {
        qdist = 2;
        wts = 1.0;
      }
      float pss = 0.0;
      if ((d.present >> i & 1) && (d.present >> j & 1)) pss = pair_score_nonbody(c, d, i, j, qdist);
      float v;
      if (pss < 0) {
        v = -1.00;
      } else {
        wts *= pss;
        wts *= pl->tfw[i];
        wts *= pl->tfw[j];
        v = wts;
      }
      sm[pair_index<NQ>(i, j) * smStride] = v;
    }
  }
  if (stop == 3) {  // diagnostic (GBGPU_SCORE_MODE=3): stop after the non-body pairs
    *outScore = sm[0];
    return true;
  }
  // single term scores, Posdb.cpp:6933-6978
  float minSingleScore = 999999999.0;
#pragma unroll
  for (int i = 0; i < NQ; i++) bestPos[i] = -1;
  for (int i = 0; i < c.nq; i++) {
    if ((c.excl >> i & 1)) continue;
    int bp;
    // the do-while reads at least one record, and fills a slot a record at most
    const int ni = rget(d.end, i) - rget(d.beg, i);
    const int tw = wave_max15(min(c.realMaxTop, max(ni, 1)));
    const float sts = single_term_score<NQ, RP, REC, T>(c, d, i, &bp, rec, tw);
    rset(bestPos, i, bp);
    if (sts < minSingleScore) minSingleScore = sts;
  }
  if (stop == 4) {  // diagnostic: stop after the single-term scores
    *outScore = minSingleScore + (float)bestPos[0];
    return true;
  }
  // sliding window, Posdb.cpp:7013-7150
  c.bestWindowScore = -2.0;
  int xpos[NQ];
#pragma unroll
  for (int i = 0; i < NQ; i++) {
    xpos[i] = (i < c.nq && (d.present >> i & 1)) ? d.beg[i] : -1;
    c.window[i] = -1;
  }
  bool allNull = true;
#pragma unroll
  for (int i = 0; i < NQ; i++) {
    if (i < c.nq && !(c.excl >> i & 1)) {
      int xp = xpos[i];
      while (xp >= 0 && !s_weights.in_body[r_hg(d.rec[xp])]) {
        xp++;
        if (xp >= d.end[i]) xp = -1;
      }
      xpos[i] = xp;
      if (xp >= 0) allNull = false;
    }
  }
  bool fast2 = false;
  if constexpr (NQ == 2) fast2 = c.nq == 2 && c.excl == 0;
  if (!allNull && fast2) {
    // Two groups, one pair: the same walk with the pair's four window terms
    // kept in registers.  (best, best) never changes and (best, window) /
    // (window, best) only when that window pointer moves, so a step scores
    // two of the four; each pointer's record fields are read once.
    const Weights &W = s_weights;
    float wikiWeight;
    int cq;
    if (pl->wiki[1] == pl->wiki[0] && pl->wiki[1]) {
      cq = pl->qpos[1] - pl->qpos[0];
      wikiWeight = GB_WIKI_WEIGHT;
    } else {
      cq = 2;
      wikiWeight = 1.0;
    }
    const float tf = pl->tfw[0] * pl->tfw[1];
    const float smv = sm[0];
    const bool quoted = pl->quote[1] >= 0 && pl->quote[1] == pl->quote[0];
    const int32_t qd = pl->qpos[1] - pl->qpos[0];
    WinRec b0{0, 0, 0, 0, false, false}, b1{0, 0, 0, 0, false, false};
    if (bestPos[0] >= 0) b0 = win_rec(W, d.rec[bestPos[0]]);
    if (bestPos[1] >= 0) b1 = win_rec(W, d.rec[bestPos[1]]);
    WinRec w0{0, 0, 0, 0, false, false}, w1{0, 0, 0, 0, false, false};
    int x0 = xpos[0], x1 = xpos[1];
    if (x0 >= 0) w0 = win_rec(W, d.rec[x0]);
    if (x1 >= 0) w1 = win_rec(W, d.rec[x1]);
    const float sbb = pair_score_window_rec(cq, b0, b1, FIXED_DISTANCE);
    float sbw = pair_score_window_rec(cq, b0, w1, FIXED_DISTANCE);
    float swb = pair_score_window_rec(cq, w0, b1, FIXED_DISTANCE);
    const int e0 = d.end[0], e1 = d.end[1];
    for (;;) {
      float mx = pair_score_window_rec(cq, w0, w1, 0);
      if (sbw > mx) mx = sbw;
      if (sbb > mx) mx = sbb;
      if (swb > mx) mx = swb;
      if (wikiWeight != 1.0) mx *= wikiWeight;
      mx *= tf;
      if (smv > mx) mx = smv;
      if (quoted) {
        if (x0 < 0) {
          mx = -1.0;
        } else if (x1 < 0) {
          mx = -1.0;
        } else {
          const int32_t dist = w1.p - w0.p;
          if (dist < 0) mx = -1.0;
          else if (dist > qd && dist - qd > 1) mx = -1.0;
          else if (dist < qd && qd - dist > 1) mx = -1.0;
        }
      }
      float minTPS = 999999999.0;
      if (mx < minTPS) minTPS = mx;
      if (!(minTPS <= c.bestWindowScore)) {
        c.bestWindowScore = minTPS;
        c.window[0] = x0;
        c.window[1] = x1;
      }
      bool done = false;
      for (;;) {  // advanceMin: the lower position moves (term 0 on ties)
        const bool m0 = x0 >= 0 && (x1 < 0 || (uint32_t)w0.p <= (uint32_t)w1.p);
        int xp = m0 ? x0 : x1;
        const int xe = m0 ? e0 : e1;
        bool exhausted = false;
        uint64_t k = 0;
        for (;;) {  // advanceAgain
          xp++;
          if (xp >= xe) {
            xp = -1;
            exhausted = true;
            break;
          }
          k = d.rec[xp];
          if (W.in_body[r_hg(k)]) break;
        }
        WinRec nr{0, 0, 0, 0, false, false};
        if (!exhausted) nr = win_rec(W, k);
        if (m0) {
          x0 = xp;
          w0 = nr;
          swb = pair_score_window_rec(cq, w0, b1, FIXED_DISTANCE);
        } else {
          x1 = xp;
          w1 = nr;
          sbw = pair_score_window_rec(cq, b0, w1, FIXED_DISTANCE);
        }
        if (!exhausted) break;  // -> slideMore
        if (x0 < 0 && x1 < 0) {
          done = true;
          break;
        }
      }
      if (done) break;
    }
  }
  if (!allNull && !fast2) {
    for (;;) {
      eval_window(c, d, xpos, bestPos);
      bool done = false;
      for (;;) {  // advanceMin
        int minx = -1;
        uint32_t minPos = 0;
#pragma unroll
        for (int x = 0; x < NQ; x++) {
          if (x < c.nq && !(c.excl >> x & 1) && xpos[x] >= 0) {
            const uint32_t wp = r_wordpos(d.rec[xpos[x]]);
            if (minx == -1 || wp < minPos) {
              minx = x;
              minPos = wp;
            }
          }
        }
        int xp = rget(xpos, minx);
        const int xe = rget(d.end, minx);
        bool exhausted = false;
        for (;;) {  // advanceAgain
          xp++;
          if (xp >= xe) {
            xp = -1;
            exhausted = true;
            break;
          }
          if (s_weights.in_body[r_hg(d.rec[xp])]) break;
        }
        rset(xpos, minx, xp);
        if (!exhausted) break;  // -> slideMore
        bool any = false;
#pragma unroll
        for (int k = 0; k < NQ; k++)
          if (k < c.nq && !(c.excl >> k & 1) && xpos[k] >= 0) any = true;
        if (!any) { done = true; break; }
      }
      if (done) break;
    }
  }
  if (stop == 5) {  // diagnostic: stop after the sliding window
    *outScore = c.bestWindowScore + (float)c.window[0];
    return true;
  }
  // window-restricted pair scores, Posdb.cpp:7159-7219
  float minPairScore = -1.0;
  for (int i = 0; i < c.nq; i++) {
    if ((c.excl >> i & 1)) continue;
    for (int j = i + 1; j < c.nq; j++) {
      if ((c.excl >> j & 1)) continue;
      if (!(d.present >> i & 1)) continue;
      if (!(d.present >> j & 1)) continue;
      // each step advances one cursor and fills a slot at most: n_i + n_j - 1 steps
      const int nij = (rget(d.end, i) - rget(d.beg, i)) + (rget(d.end, j) - rget(d.beg, j)) - 1;
      const int tw = wave_max15(min(c.realMaxTop, max(nij, 1)));
      const float score = pair_score_any<NQ, RP, REC, T>(c, d, i, j, rec, tw);
      if (score >= minPairScore && minPairScore >= 0.0) continue;
      minPairScore = score;
    }
  }
  // final score, Posdb.cpp:7228-7257
  float minScore = 999999999.0;
  if (minPairScore < minScore && minPairScore >= 0.0) minScore = minPairScore;
  if (minSingleScore < minScore) minScore = minSingleScore;
  if (minScore <= 0.0) return false;
  float score = minScore * (((float)siteRank) * pl->site_rank_multiplier + 1.0);
  if (pl->language == 0 || docLang == 0 || pl->language == docLang) score *= pl->same_lang_weight;
  *outScore = score;
  return true;
}

}  // namespace gbgpu

#endif
