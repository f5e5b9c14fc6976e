// Per-docid scoring of PosdbTable::intersectLists10_r, device side.
//
// A docid's mini-merged lists (Posdb.cpp:6559-6778) are held as 8-byte
// records: the low 6 bytes are the rewritten posdb key bytes 0..5 (density,
// word position, hash group, spam rank, diversity, F bits).  Every scorer
// below restates its reference function over record indices instead of
// char pointers; expression shapes (float vs double promotion, operand
// order) follow the reference exactly so results round identically
// (compiled with -ffp-contract=off).
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

// record field accessors (Posdb.h:319-361 on key bytes 0..5)
__host__ __device__ __forceinline__ uint32_t r_wordpos(uint64_t r) { return (uint32_t)(r >> 30) & 0x3ffff; }
__host__ __device__ __forceinline__ uint32_t r_hg(uint64_t r) { return (uint32_t)(r >> 26) & 0xf; }
__host__ __device__ __forceinline__ uint32_t r_wsr(uint64_t r) { return (uint32_t)(r >> 22) & 0xf; }
__host__ __device__ __forceinline__ uint32_t r_div(uint64_t r) { return (uint32_t)(r >> 18) & 0xf; }
__host__ __device__ __forceinline__ uint32_t r_syn(uint64_t r) { return (uint32_t)(r >> 16) & 0x3; }
__host__ __device__ __forceinline__ uint32_t r_hswb(uint64_t r) { return (uint32_t)(r >> 16) & 0x1; }
__host__ __device__ __forceinline__ uint32_t r_dens(uint64_t r) { return (uint32_t)(r >> 11) & 0x1f; }

// What one docid's scorer sees: nq groups, each a record range.
struct DocView {
  const uint64_t *rec;  // records of this docid (all groups back to back)
  int beg[MAXG], end[MAXG];
  bool present[MAXG];   // miniMergedList[j] != NULL (positive group)
};

struct ScoreCtx {
  const Weights *w;
  const DevPlan *pl;
  int nq;
  uint8_t bflags[MAXG];
  int realMaxTop;
  int qdist;             // PosdbTable::m_qdist (set by evalSlidingWindow)
  float bestWindowScore; // m_bestWindowScore
  int window[MAXG];      // m_windowTermPtrs (record index, -1 = NULL)
};

// getSingleTermScore, Posdb.cpp:3087-3301 (pdcs == NULL).  bestPos = record
// index of the best non-body occurrence or -1.
__device__ inline float single_term_score(const ScoreCtx &c, const DocView &d, int i, int *bestPos) {
  const Weights &W = *c.w;
  float nonBodyMax = -1.0;
  int minx = 0;
  float bestScores[MAX_TOP];
  int bestwpi[MAX_TOP];
  uint8_t bestmhg[MAX_TOP];
  int numTop = 0;
  *bestPos = -1;
  for (int r = d.beg[i]; r < d.end[i]; r++) {
    uint64_t k = d.rec[r];
    float score = 100.0;
    uint32_t div = r_div(k);
    score *= W.diversity[div];
    score *= W.diversity[div];
    uint32_t hg = r_hg(k);
    uint32_t mhg = hg;
    if (W.in_body[mhg]) mhg = GB_HG_BODY;
    score *= W.hashgroup[hg];
    score *= W.hashgroup[hg];
    uint32_t dens = r_dens(k);
    score *= W.density[dens];
    score *= W.density[dens];
    uint32_t wspam = r_wsr(k);
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
    int bro = -1;
    for (int q = 0; q < numTop; q++) {
      if (bestmhg[q] == mhg && hg != GB_HG_INLINKTEXT) { bro = q; break; }
    }
    if (bro >= 0) {
      if (score > bestScores[bro]) {
        bestScores[bro] = score;
        bestwpi[bro] = r;
        bestmhg[bro] = (uint8_t)mhg;
      }
    } else if (numTop < c.realMaxTop) {
      bestScores[numTop] = score;
      bestwpi[numTop] = r;
      bestmhg[numTop] = (uint8_t)mhg;
      numTop++;
    } else if (score > bestScores[minx]) {
      bestScores[minx] = score;
      bestwpi[minx] = r;
      bestmhg[minx] = (uint8_t)mhg;
    }
    if (numTop >= c.realMaxTop) {
      minx = 0;
      for (int q = 1; q < c.realMaxTop; q++) {
        if (bestScores[q] > bestScores[minx]) continue;
        minx = q;
      }
    }
    if (score > nonBodyMax && !W.in_body[hg]) {
      nonBodyMax = score;
      *bestPos = r;
    }
  }
  float sum = 0.0;
  for (int q = 0; q < numTop; q++) {
    if (r_hswb(d.rec[bestwpi[q]]))
      sum += (bestScores[q] * GB_WIKI_BIGRAM_WEIGHT * GB_WIKI_BIGRAM_WEIGHT);
    else
      sum += bestScores[q];
  }
  sum *= c.pl->tfw[i];
  sum *= c.pl->tfw[i];
  return sum;
}

// getTermPairScoreForNonBody, Posdb.cpp:3305-3555
__device__ inline float pair_score_nonbody(const ScoreCtx &c, const DocView &d, int i, int j, int qdist) {
  const Weights &W = *c.w;
  int wi = d.beg[i], wj = d.beg[j];
  const int endi = d.end[i], endj = d.end[j];
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
        score /= (dist + 1.0);
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
        score /= (dist + 1.0);
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
__device__ inline float pair_score_window(const ScoreCtx &c, const DocView &d, int wpi, int wpj,
                                          int32_t fixedDistance) {
  if (wpi < 0) return -1.00;
  if (wpj < 0) return -1.00;
  const Weights &W = *c.w;
  uint64_t ki = d.rec[wpi], kj = d.rec[wpj];
  int32_t p1 = (int32_t)r_wordpos(ki), p2 = (int32_t)r_wordpos(kj);
  uint32_t hg1 = r_hg(ki), hg2 = r_hg(kj);
  float spamw1 = (hg1 == GB_HG_INLINKTEXT) ? W.linker[r_wsr(ki)] : W.wordspam[r_wsr(ki)];
  float spamw2 = (hg2 == GB_HG_INLINKTEXT) ? W.linker[r_wsr(kj)] : W.wordspam[r_wsr(kj)];
  float denw1 = W.density[r_dens(ki)];
  float denw2 = W.density[r_dens(kj)];
  float dist, score;
  if (fixedDistance != 0) {
    dist = fixedDistance;
  } else {
    if (p2 < p1) dist = p1 - p2;
    else dist = p2 - p1;
    if (dist < 2) dist = 2;
    if (dist >= c.qdist) dist = dist - c.qdist;
    if (p2 < p1) dist += 1;
  }
  score = 100 * denw1 * denw2;
  score *= W.hashgroup[hg1];
  score *= W.hashgroup[hg2];
  if (r_syn(ki)) score *= GB_SYNONYM_WEIGHT;
  if (r_syn(kj)) score *= GB_SYNONYM_WEIGHT;
  score *= spamw1 * spamw2;
  score /= (dist + 1.0);
  return score;
}

// evalSlidingWindow, Posdb.cpp:1275-1511
__device__ inline void eval_window(ScoreCtx &c, const DocView &d, const int *ptrs, const int *bestPos,
                                   const float *scoreMatrix) {
  float minTermPairScoreInWindow = 999999999.0;
  const int nr = c.nq;
  for (int i = 0; i < nr; i++) {
    if (c.bflags[i] & BF_EXCLUDE) continue;
    int wpi = ptrs[i];
    for (int j = i + 1; j < nr; j++) {
      if (c.bflags[j] & BF_EXCLUDE) continue;
      int wpj = ptrs[j];
      float wikiWeight;
      if (c.pl->wiki[j] == c.pl->wiki[i] && c.pl->wiki[j]) {
        c.qdist = c.pl->qpos[j] - c.pl->qpos[i];
        wikiWeight = GB_WIKI_WEIGHT;
      } else {
        c.qdist = 2;
        wikiWeight = 1.0;
      }
      float max = pair_score_window(c, d, wpi, wpj, 0);
      float score = pair_score_window(c, d, bestPos[i], wpj, FIXED_DISTANCE);
      if (score > max) max = score;
      score = pair_score_window(c, d, bestPos[i], bestPos[j], FIXED_DISTANCE);
      if (score > max) max = score;
      score = pair_score_window(c, d, wpi, bestPos[j], FIXED_DISTANCE);
      if (score > max) max = score;
      if (wikiWeight != 1.0) max *= wikiWeight;
      max *= c.pl->tfw[i] * c.pl->tfw[j];
      if (scoreMatrix[i * MAXG + j] > max) max = scoreMatrix[i * MAXG + j];
      if (c.pl->quote[j] >= 0 && c.pl->quote[j] == c.pl->quote[i]) {
        if (wpi < 0) {
          max = -1.0;
        } else if (wpj < 0) {
          max = -1.0;
        } else {
          int32_t qd = c.pl->qpos[j] - c.pl->qpos[i];
          int32_t p1 = (int32_t)r_wordpos(d.rec[wpi]);
          int32_t p2 = (int32_t)r_wordpos(d.rec[wpj]);
          int32_t dist = p2 - p1;
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
  for (int i = 0; i < nr; i++) c.window[i] = ptrs[i];
}

// getTermPairScoreForAny, Posdb.cpp:3631-4344 (pdcs == NULL)
__device__ inline float pair_score_any(const ScoreCtx &c, const DocView &d, int i, int j) {
  const Weights &W = *c.w;
  float wts;
  int32_t qdist;
  if (c.pl->wiki[j] == c.pl->wiki[i] && c.pl->wiki[j]) {
    qdist = c.pl->qpos[j] - c.pl->qpos[i];
    wts = (float)GB_WIKI_WEIGHT;
  } else {
    qdist = 2;
    wts = 1.0;
  }
  const bool inSameQuotedPhrase = (c.pl->quote[i] == c.pl->quote[j] && c.pl->quote[i] >= 0);
  if (inSameQuotedPhrase) qdist = c.pl->qpos[j] - c.pl->qpos[i];
  int wi = d.beg[i], wj = d.beg[j];
  const int endi = d.end[i], endj = d.end[j];
  uint64_t ki = d.rec[wi], kj = d.rec[wj];
  int32_t p1 = (int32_t)r_wordpos(ki), p2 = (int32_t)r_wordpos(kj);
  uint32_t hg1 = r_hg(ki), hg2 = r_hg(kj);
  uint32_t mhg1 = W.in_body[hg1] ? GB_HG_BODY : hg1;
  uint32_t mhg2 = W.in_body[hg2] ? GB_HG_BODY : hg2;
  float spamw1 = (hg1 == GB_HG_INLINKTEXT) ? W.linker[r_wsr(ki)] : W.wordspam[r_wsr(ki)];
  float spamw2 = (hg2 == GB_HG_INLINKTEXT) ? W.linker[r_wsr(kj)] : W.wordspam[r_wsr(kj)];
  float denw1 = W.density[r_dens(ki)];
  float denw2 = W.density[r_dens(kj)];
  float score;
  int minx = -1;
  float bestScores[MAX_TOP];
  uint8_t bestmhg1[MAX_TOP], bestmhg2[MAX_TOP];
  int numTop = 0;
  int32_t dist;
  for (;;) {
    bool adv1;
    if (W.in_body[hg1] && wi != c.window[i]) {
      adv1 = true;
    } else if (W.in_body[hg2] && wj != c.window[j]) {
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
        uint32_t syn1 = r_syn(ki), syn2 = r_syn(kj);
        if (dist < 2) dist = 2;
        if (dist < 50) {
        } else if (mhg1 != mhg2) {
          dist = FIXED_DISTANCE;
        } else if (mhg1 == GB_HG_INLINKTEXT) {
          dist = FIXED_DISTANCE;
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
        score /= (dist + 1.0);
        goto topScores;
      }
    } else {
      adv1 = false;
      dist = p1 - p2;
      if (!inSameQuotedPhrase) {
        if (dist < 2) dist = 2;
        if (dist < 50) {
        } else if (mhg1 != mhg2) {
          dist = FIXED_DISTANCE;
        } else if (mhg1 == GB_HG_INLINKTEXT) {
          dist = FIXED_DISTANCE;
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
        score /= (dist + 1.0);
        goto topScores;
      }
    }
    goto advance;
  topScores : {
    int bro = -1;
    for (int q = 0; q < numTop; q++) {
      if (bestmhg1[q] == mhg1 && hg1 != GB_HG_INLINKTEXT) { bro = q; break; }
      if (bestmhg2[q] == mhg2 && hg2 != GB_HG_INLINKTEXT) { bro = q; break; }
    }
    if (bro >= 0) {
      if (score > bestScores[bro]) {
        bestScores[bro] = score;
        bestmhg1[bro] = (uint8_t)mhg1;
        bestmhg2[bro] = (uint8_t)mhg2;
      }
    } else if (numTop < c.realMaxTop) {
      bestScores[numTop] = score;
      bestmhg1[numTop] = (uint8_t)mhg1;
      bestmhg2[numTop] = (uint8_t)mhg2;
      numTop++;
    } else if (score > bestScores[minx]) {
      bestScores[minx] = score;
      bestmhg1[minx] = (uint8_t)mhg1;
      bestmhg2[minx] = (uint8_t)mhg2;
    }
    if (numTop >= c.realMaxTop) {
      minx = 0;
      for (int q = 1; q < c.realMaxTop; q++) {
        if (bestScores[q] > bestScores[minx]) continue;
        minx = q;
      }
    }
  }
  advance:
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
  for (int q = 0; q < numTop; q++) sum += bestScores[q];
  sum *= wts;
  sum *= c.pl->tfw[i];
  sum *= c.pl->tfw[j];
  return sum;
}

// The per-docid body of intersectLists10_r after the mini merges
// (Posdb.cpp:6847-7257).  Returns false when the docid is not scored
// (minScore <= 0); siteRank/docLang come from the first key of the first
// present group (Posdb.cpp:6985-7003).
__device__ inline bool score_doc(const Weights *w, const DevPlan *pl, const DocView &d, int siteRank,
                                 int docLang, float *outScore) {
  ScoreCtx c;
  c.w = w;
  c.pl = pl;
  c.nq = pl->ngroups;
  c.realMaxTop = pl->real_max_top;
  c.qdist = 2;
  for (int i = 0; i < c.nq; i++) c.bflags[i] = pl->gflags0[i];
  float scoreMatrix[MAXG * MAXG];
  int bestPos[MAXG];
  // non-body pair scores, Posdb.cpp:6847-6926
  for (int i = 0; i < c.nq; i++) {
    if (c.bflags[i] & BF_EXCLUDE) continue;
    for (int j = i + 1; j < c.nq; j++) {
      if (c.bflags[j] & BF_EXCLUDE) continue;
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
      if (d.present[i] && d.present[j]) pss = pair_score_nonbody(c, d, i, j, qdist);
      if (pss < 0) {
        scoreMatrix[i * MAXG + j] = -1.00;
      } else {
        wts *= pss;
        wts *= pl->tfw[i];
        wts *= pl->tfw[j];
        scoreMatrix[i * MAXG + j] = wts;
      }
    }
  }
  // single term scores, Posdb.cpp:6933-6978
  float minSingleScore = 999999999.0;
  for (int i = 0; i < c.nq; i++) {
    bestPos[i] = -1;
    if (c.bflags[i] & BF_EXCLUDE) continue;
    float sts = single_term_score(c, d, i, &bestPos[i]);
    if (sts < minSingleScore) minSingleScore = sts;
  }
  // sliding window, Posdb.cpp:7013-7150
  c.bestWindowScore = -2.0;
  int xpos[MAXG];
  for (int i = 0; i < c.nq; i++) {
    xpos[i] = d.present[i] ? d.beg[i] : -1;
    c.window[i] = -1;
  }
  bool allNull = true;
  for (int i = 0; i < c.nq; i++) {
    if (c.bflags[i] & BF_EXCLUDE) continue;
    while (xpos[i] >= 0 && !w->in_body[r_hg(d.rec[xpos[i]])]) {
      xpos[i]++;
      if (xpos[i] < d.end[i]) continue;
      xpos[i] = -1;
    }
    if (xpos[i] >= 0) allNull = false;
  }
  if (!allNull) {
    for (;;) {
      eval_window(c, d, xpos, bestPos, scoreMatrix);
      bool done = false;
      for (;;) {  // advanceMin
        int minx = -1;
        uint32_t minPos = 0;
        for (int x = 0; x < c.nq; x++) {
          if (c.bflags[x] & BF_EXCLUDE) continue;
          if (xpos[x] < 0) continue;
          uint32_t wp = r_wordpos(d.rec[xpos[x]]);
          if (minx == -1) { minx = x; minPos = wp; continue; }
          if (wp >= minPos) continue;
          minx = x;
          minPos = wp;
        }
        bool again = true;
        bool exhausted = false;
        while (again) {  // advanceAgain
          xpos[minx]++;
          if (xpos[minx] >= d.end[minx]) {
            xpos[minx] = -1;
            exhausted = true;
            break;
          }
          again = !w->in_body[r_hg(d.rec[xpos[minx]])];
        }
        if (!exhausted) break;  // -> slideMore
        int k;
        for (k = 0; k < c.nq; k++) {
          if (c.bflags[k] & BF_EXCLUDE) continue;
          if (xpos[k] >= 0) break;
        }
        if (k >= c.nq) { done = true; break; }
      }
      if (done) break;
    }
  }
  // window-restricted pair scores, Posdb.cpp:7159-7219
  float minPairScore = -1.0;
  for (int i = 0; i < c.nq; i++) {
    if (c.bflags[i] & BF_EXCLUDE) continue;
    for (int j = i + 1; j < c.nq; j++) {
      if (c.bflags[j] & BF_EXCLUDE) continue;
      if (!d.present[i]) continue;
      if (!d.present[j]) continue;
      float score = pair_score_any(c, d, i, j);
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
