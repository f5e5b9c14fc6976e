/* TEST INFRASTRUCTURE ONLY (see posdb_oracle.h).
 *
 * CPU restatement of the reference's Posdb query path, written against the
 * reference's own byte-level algorithm so that it inherits its exact
 * behaviour, quirks included.  Compile with -ffp-contract=off: the reference
 * is x86-64 SSE -O2 (Makefile:101), FLT_EVAL_METHOD 0, no FMA, so every float
 * expression below is written with the same operand types and order as the
 * reference expression it restates and rounds the same way.
 *
 * Pinned bit-exact against the reference's own PosdbTable (oracle/ref.mk,
 * tests/golden/, tests/test_reference.py).
 */
#include "posdb_oracle.h"

#include <errno.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

/* Posdb.h:102-108 */
#define BF_HALFSTOPWIKIBIGRAM 0x01
#define BF_PIPED              0x02
#define BF_SYNONYM            0x04
#define BF_NEGATIVE           0x08
#define BF_BIGRAM             0x10
#define BF_NUMBER             0x20
#define BF_FACET              0x40
#define BF_EXCLUDE (BF_PIPED | BF_NEGATIVE | BF_NUMBER | BF_FACET)

#define MAX_SUBLISTS 50        /* Posdb.h:417 */
#define MAX_TOP 10             /* Posdb.h:817 */
#define FIXED_DISTANCE 400     /* Posdb.h:765 */
#define SYNONYM_WEIGHT 0.90    /* Posdb.h:94  */
#define WIKI_WEIGHT 0.10       /* Posdb.h:95  */
#define SITERANKMULTIPLIER 0.33333333 /* Posdb.h:97 */
#define WIKI_BIGRAM_WEIGHT 1.40       /* Posdb.h:115 */

#define HASHGROUP_BODY 0
#define HASHGROUP_TITLE 1
#define HASHGROUP_HEADING 2
#define HASHGROUP_INLIST 3
#define HASHGROUP_INMETATAG 4
#define HASHGROUP_INLINKTEXT 5
#define HASHGROUP_INTAG 6
#define HASHGROUP_NEIGHBORHOOD 7
#define HASHGROUP_INTERNALINLINKTEXT 8
#define HASHGROUP_INURL 9
#define HASHGROUP_INMENU 10
#define HASHGROUP_END 11

/* ---------------------------------------------------------------- weights */
/* initWeights, Posdb.cpp:1094-1197 */
static int s_init = 0;
static float s_diversityWeights[16];
static float s_densityWeights[32];
static float s_wordSpamWeights[16];
static float s_linkerWeights[16];
static float s_hashGroupWeights[HASHGROUP_END];
static char s_isCompatible[HASHGROUP_END][HASHGROUP_END];
static char s_inBody[HASHGROUP_END];

static void initWeights(void) {
  if (s_init) return;
  s_init = 1;
  float sum = 0.15;
  for (int i = 0; i <= 15; i++) {
    s_diversityWeights[i] = 1.0;
    sum *= 1.135;
  }
  sum = 0.35;
  for (int i = 0; i <= 31; i++) {
    if (sum > 1.0) sum = 1.0;
    s_densityWeights[i] = sum;
    sum *= 1.03445;
  }
  for (int i = 0; i <= 15; i++) s_wordSpamWeights[i] = (float)(i + 1) / (15 + 1);
  for (int i = 0; i <= 15; i++) s_linkerWeights[i] = sqrt(1.0 + i);
  for (int i = 0; i < HASHGROUP_END; i++) {
    s_inBody[i] = 0;
    if (i == HASHGROUP_BODY || i == HASHGROUP_HEADING || i == HASHGROUP_INLIST ||
        i == HASHGROUP_INMENU)
      s_inBody[i] = 1;
    for (int j = 0; j < HASHGROUP_END; j++) {
      s_isCompatible[i][j] = 0;
      int inBody1 = 1, inBody2 = 1;
      if (i != HASHGROUP_BODY && i != HASHGROUP_HEADING && i != HASHGROUP_INLIST &&
          i != HASHGROUP_INMENU)
        inBody1 = 0;
      if (j != HASHGROUP_BODY && j != HASHGROUP_HEADING && j != HASHGROUP_INLIST &&
          j != HASHGROUP_INMENU)
        inBody2 = 0;
      if (inBody1 || inBody2) continue;
      s_isCompatible[i][j] = 1;
    }
  }
  s_hashGroupWeights[HASHGROUP_BODY] = 1.0;
  s_hashGroupWeights[HASHGROUP_TITLE] = 8.0;
  s_hashGroupWeights[HASHGROUP_HEADING] = 1.5;
  s_hashGroupWeights[HASHGROUP_INLIST] = 0.3;
  s_hashGroupWeights[HASHGROUP_INMETATAG] = 0.1;
  s_hashGroupWeights[HASHGROUP_INLINKTEXT] = 16.0;
  s_hashGroupWeights[HASHGROUP_INTAG] = 1.0;
  s_hashGroupWeights[HASHGROUP_NEIGHBORHOOD] = 0.0;
  s_hashGroupWeights[HASHGROUP_INTERNALINLINKTEXT] = 4.0;
  s_hashGroupWeights[HASHGROUP_INURL] = 1.0;
  s_hashGroupWeights[HASHGROUP_INMENU] = 0.2;
}

void orc_weights(float *d32, float *w16, float *l16, float *h11, float *v16) {
  initWeights();
  if (d32) memcpy(d32, s_densityWeights, sizeof s_densityWeights);
  if (w16) memcpy(w16, s_wordSpamWeights, sizeof s_wordSpamWeights);
  if (l16) memcpy(l16, s_linkerWeights, sizeof s_linkerWeights);
  if (h11) memcpy(h11, s_hashGroupWeights, sizeof s_hashGroupWeights);
  if (v16) memcpy(v16, s_diversityWeights, sizeof s_diversityWeights);
}

/* ------------------------------------------------------------ key getters */
/* Posdb.h:271-380 */
static inline uint32_t U32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }
static inline uint16_t U16(const uint8_t *p) { uint16_t v; memcpy(&v, p, 2); return v; }
static inline int keySize(const uint8_t *k) { return (k[0] & 0x04) ? 6 : ((k[0] & 0x02) ? 12 : 18); }
static inline uint64_t getDocId(const uint8_t *k) {
  uint64_t d = k[11];
  d <<= 32;
  d |= U32(k + 7);
  return d >> 2;
}
static inline unsigned char getSiteRank(const uint8_t *k) {
  uint64_t n1;
  memcpy(&n1, k + 2, 8);
  return (n1 >> 37) & 0x0f;
}
static inline unsigned char getLangId(const uint8_t *k) {
  uint64_t n1;
  memcpy(&n1, k + 2, 8);
  if (k[0] & 0x08) return ((n1 >> 32) & 0x1f) | 0x20;
  return (n1 >> 32) & 0x1f;
}
static inline unsigned char getHashGroup(const uint8_t *k) { return (k[3] >> 2) & 0x0f; }
static inline int32_t getWordPos(const uint8_t *k) { return U32(k + 2) >> (8 + 6); }
static inline unsigned char getWordSpamRank(const uint8_t *k) { return (U16(k + 2) >> 6) & 0x0f; }
static inline unsigned char getDiversityRank(const uint8_t *k) { return (k[2] >> 2) & 0x0f; }
static inline unsigned char getIsSynonym(const uint8_t *k) { return k[2] & 0x03; }
static inline unsigned char getIsHalfStopWikiBigram(const uint8_t *k) { return k[2] & 0x01; }
static inline unsigned char getDensityRank(const uint8_t *k) { return (U16(k) >> 11) & 0x1f; }

/* ------------------------------------------------------------ structures */
typedef struct {
  uint8_t *list; /* RdbList::m_list (mutated by the first-key swap) */
  int64_t size;  /* RdbList::m_listSize                              */
} OList;

/* QueryTermInfo, Posdb.h:421-451 (sublists refer to query-term lists) */
typedef struct {
  int subList[MAX_SUBLISTS];
  char bigramFlags[MAX_SUBLISTS];
  int64_t newSubListSize[MAX_SUBLISTS];
  uint8_t *newSubListStart[MAX_SUBLISTS];
  uint8_t *newSubListEnd[MAX_SUBLISTS];
  uint8_t *cursor[MAX_SUBLISTS];
  uint8_t *savedCursor[MAX_SUBLISTS];
  int numNewSubLists;
  int numSubLists;
  int64_t totalSubListsSize;
  float termFreqWeight;
  int qtermNum, qpos, wikiPhraseId, quotedStartId;
  int fieldCode;     /* m_qt->m_fieldCode                                   */
  float qwFloat;     /* m_qt->m_qword->m_float (range terms)                */
  int32_t qwInt;     /* m_qt->m_qword->m_int                                */
} QTI;

/* Query::m_fieldCode values PosdbTable treats specially (Query.h:118-132) */
enum { F_SORTBYFLOAT = 54, F_REVSORTBYFLOAT = 55, F_NUMBERMIN = 56, F_NUMBERMAX = 57, F_SORTBYINT = 59,
       F_REVSORTBYINT = 60, F_NUMBERMININT = 61, F_NUMBERMAXINT = 62, F_FACETSTR = 63, F_FACETINT = 64,
       F_FACETFLOAT = 65, F_NUMBEREQUALINT = 66, F_NUMBEREQUALFLOAT = 67 };
static int isNumberField(int fc) { /* Posdb.cpp:4572-4594 */
  return fc == F_SORTBYFLOAT || fc == F_REVSORTBYFLOAT || fc == F_NUMBERMIN || fc == F_NUMBERMAX ||
         fc == F_NUMBEREQUALFLOAT || fc == F_SORTBYINT || fc == F_REVSORTBYINT || fc == F_NUMBERMININT ||
         fc == F_NUMBERMAXINT || fc == F_NUMBEREQUALINT;
}
static int isRangeField(int fc) { /* Posdb.cpp:5056-5073 */
  return fc == F_NUMBERMIN || fc == F_NUMBERMAX || fc == F_NUMBEREQUALFLOAT || fc == F_NUMBERMININT ||
         fc == F_NUMBERMAXINT || fc == F_NUMBEREQUALINT;
}

typedef struct {
  /* PosdbTable state used by the scorers */
  int realMaxTop;
  float *freqWeights;
  int32_t *qpos, *wikiPhraseIds, *quotedStartIds;
  char *bflags;
  int32_t qdist;
  float bestWindowScore;
  uint8_t **windowTermPtrs;
  uint64_t docId;
  int nqt;
} PT;

/* TopTree (TopTree.h:65-154, TopTree.cpp:64-516).  Its readout (getHighNode /
 * getPrev) and low node only depend on the SET of nodes, ordered by (score
 * asc, docid desc) -- the AVL shape does not show -- so the nodes are kept as
 * an array sorted best first (score desc, docid asc).  The embedded m_t2
 * RdbTree holds exactly the same nodes (every add to one is an add to the
 * other, every delete likewise), keyed per domain by (uint32 score, docid)
 * (TopTree.cpp:337-342), so m_domMinNode[] is the minimum of that key over the
 * domain's nodes and is found by a scan here. */
typedef struct {
  int64_t numNodes;      /* m_numNodes                                   */
  int32_t docsWanted;    /* m_docsWanted                                 */
  int clustering;        /* m_doSiteClustering                           */
  int64_t ridiculousMax; /* m_ridiculousMax                              */
  int32_t cap;           /* m_cap                                        */
  float partial;         /* m_partial                                    */
  float vcount;          /* m_vcount                                     */
  int32_t domCount[256]; /* m_domCount                                   */
  int64_t n;             /* m_numUsedNodes                               */
  double *score;         /* sorted best first (an int score is exact)     */
  int64_t *docid;
  int ints;              /* m_useIntScores: score holds m_intScore        */
} TTree;

/* TopTree::setNumNodes, TopTree.cpp:64-101 */
static int tt_init(TTree *t, int32_t docsWanted, int clustering) {
  memset(t, 0, sizeof *t);
  t->docsWanted = docsWanted;
  t->clustering = clustering;
  t->ridiculousMax = (int64_t)docsWanted * 2;
  if (t->ridiculousMax < 50) t->ridiculousMax = 50;
  int64_t numNodes = t->ridiculousMax * 256;
  if (numNodes > 2000000000LL) numNodes = 2000000000LL; /* MAXDOCIDSTOCOMPUTE, Msg40.h:25 */
  if (!clustering) t->ridiculousMax = 0x7fffffff;
  if (!clustering) numNodes = t->docsWanted + 1;
  t->vcount = 0.0;
  t->cap = t->docsWanted / 50;
  if (t->cap < 2) t->cap = 2;
  if (!clustering) t->cap = 0x7fffffff;
  t->partial = (float)(t->docsWanted % 50) / 50.0;
  t->numNodes = numNodes;
  /* the array grows on demand (numNodes can be 2 * docsWanted * 256) */
  return 0;
}

static void tt_free(TTree *t) {
  free(t->score);
  free(t->docid);
  t->score = NULL;
  t->docid = NULL;
}

static inline uint8_t domHash8(int64_t d) { return (uint8_t)((d & ~0xffffffffffffc03fULL) >> 6); } /* Titledb.h:114-115 */

/* deleteNode's count bookkeeping (TopTree.cpp:543-547) + removal of node i */
static void tt_delete(TTree *t, int64_t i, uint8_t domHash) {
  if (t->domCount[domHash] < t->cap) t->vcount -= 1.0;
  else if (t->domCount[domHash] == t->cap) t->vcount -= t->partial;
  t->domCount[domHash]--;
  memmove(t->score + i, t->score + i + 1, sizeof(double) * (size_t)(t->n - i - 1));
  memmove(t->docid + i, t->docid + i + 1, sizeof(int64_t) * (size_t)(t->n - i - 1));
  t->n--;
}

/* the domain tree's key score cs (TopTree.cpp:332-335): (uint32_t)m_intScore,
   or (uint32_t)m_score as x86-64 converts a float (the low 32 bits of its
   64-bit truncation, cvttss2si) -- spelled out, the C casts being undefined
   for negative values */
static inline uint32_t tt_cs(const TTree *t, double score) {
  if (t->ints) return (uint32_t)(int32_t)score;
  const float f = (float)score;
  if (!(f > -9.2233720368547758e18f && f < 9.2233720368547758e18f)) return 0; /* 0x8000000000000000 */
  return (uint32_t)(uint64_t)(int64_t)f;
}

/* TopTree::addNode, TopTree.cpp:206-516; returns 1 if the node was added */
static int tt_add(TTree *t, double score, int64_t docid) {
  const uint8_t domHash = domHash8(docid);
  if (t->vcount >= t->docsWanted) {
    const double ls = t->score[t->n - 1];
    const int64_t ld = t->docid[t->n - 1];
    if (score < ls) return 0;
    if (score > ls) goto addIt;
    if (docid >= ld) return 0;
  }
addIt:;
  /* position: after every node that ranks above (score desc, docid asc) */
  int64_t pos = 0;
  {
    int64_t lo = 0, hi = t->n;
    while (lo < hi) {
      int64_t mid = (lo + hi) / 2;
      if (t->score[mid] > score || (t->score[mid] == score && t->docid[mid] < docid)) lo = mid + 1;
      else hi = mid;
    }
    pos = lo;
    if (pos < t->n && t->score[pos] == score && t->docid[pos] == docid) return 0; /* equal: not replaced */
  }
  const uint32_t cs = tt_cs(t, score);
  int64_t deleteMe = -1; /* docid of the domain's m_t2 minimum to delete */
  if (t->domCount[domHash] >= t->ridiculousMax) {
    /* m_domMinNode[domHash]: minimum (uint32 score, docid) of the domain */
    int64_t m = -1;
    uint32_t mcs = 0;
    for (int64_t i = 0; i < t->n; i++) {
      if (domHash8(t->docid[i]) != domHash) continue;
      const uint32_t c = tt_cs(t, t->score[i]);
      if (m < 0 || c < mcs || (c == mcs && t->docid[i] < t->docid[m])) {
        m = i;
        mcs = c;
      }
    }
    if (cs < mcs || (cs == mcs && docid <= t->docid[m])) return 0; /* k <= key(min) */
    deleteMe = t->docid[m];
  }
  if (t->n % 4096 == 0) {
    t->score = (double *)realloc(t->score, sizeof(double) * (size_t)(t->n + 4096));
    t->docid = (int64_t *)realloc(t->docid, sizeof(int64_t) * (size_t)(t->n + 4096));
  }
  memmove(t->score + pos + 1, t->score + pos, sizeof(double) * (size_t)(t->n - pos));
  memmove(t->docid + pos + 1, t->docid + pos, sizeof(int64_t) * (size_t)(t->n - pos));
  t->score[pos] = score;
  t->docid[pos] = docid;
  t->n++;
  t->domCount[domHash]++;
  if (t->domCount[domHash] < t->cap) t->vcount += 1.0;
  else if (t->domCount[domHash] == t->cap) t->vcount += t->partial;
  if (deleteMe >= 0) {
    int64_t i = 0;
    while (t->docid[i] != deleteMe) i++;
    tt_delete(t, i, domHash);
  }
  while (t->vcount - 1.0 >= t->docsWanted || t->n == t->numNodes) {
    const int64_t tn = t->n - 1; /* m_lowNode */
    tt_delete(t, tn, domHash8(t->docid[tn]));
  }
  return 1;
}

/* --------------------------------------------------------------- scorers */
/* getSingleTermScore, Posdb.cpp:3087-3301 (pdcs == NULL) */
static float getSingleTermScore(PT *pt, int i, uint8_t *wpi, uint8_t *endi, uint8_t **bestPos) {
  float nonBodyMax = -1.0;
  int first = 1;
  int32_t minx = 0;
  float bestScores[MAX_TOP];
  uint8_t *bestwpi[MAX_TOP];
  char bestmhg[MAX_TOP];
  int32_t numTop = 0;
  *bestPos = NULL;
  if (!wpi) goto done;
  for (;;) {
    float score = 100.0;
    unsigned char div = getDiversityRank(wpi);
    score *= s_diversityWeights[div];
    score *= s_diversityWeights[div];
    unsigned char hg = getHashGroup(wpi);
    unsigned char mhg = hg;
    if (s_inBody[mhg]) mhg = HASHGROUP_BODY;
    score *= s_hashGroupWeights[hg];
    score *= s_hashGroupWeights[hg];
    unsigned char dens = getDensityRank(wpi);
    score *= s_densityWeights[dens];
    score *= s_densityWeights[dens];
    unsigned char wspam = getWordSpamRank(wpi);
    if (hg == HASHGROUP_INLINKTEXT) {
      score *= s_linkerWeights[wspam];
      score *= s_linkerWeights[wspam];
    } else {
      score *= s_wordSpamWeights[wspam];
      score *= s_wordSpamWeights[wspam];
    }
    if (getIsSynonym(wpi)) {
      score *= SYNONYM_WEIGHT;
      score *= SYNONYM_WEIGHT;
    }
    int32_t bro = -1;
    for (int32_t k = 0; k < numTop; k++) {
      if (bestmhg[k] == mhg && hg != HASHGROUP_INLINKTEXT) {
        bro = k;
        break;
      }
    }
    if (bro >= 0) {
      if (score > bestScores[bro]) {
        bestScores[bro] = score;
        bestwpi[bro] = wpi;
        bestmhg[bro] = mhg;
      }
    } else if (numTop < pt->realMaxTop) {
      bestScores[numTop] = score;
      bestwpi[numTop] = wpi;
      bestmhg[numTop] = mhg;
      numTop++;
    } else if (score > bestScores[minx]) {
      bestScores[minx] = score;
      bestwpi[minx] = wpi;
      bestmhg[minx] = mhg;
    }
    if (numTop >= pt->realMaxTop) {
      minx = 0;
      for (int32_t k = 1; k < pt->realMaxTop; k++) {
        if (bestScores[k] > bestScores[minx]) continue;
        minx = k;
      }
    }
    if (score > nonBodyMax && !s_inBody[hg]) {
      nonBodyMax = score;
      *bestPos = wpi;
    }
    if (first) { wpi += 6; first = 0; }
    wpi += 6;
    if (wpi < endi && keySize(wpi) == 6) continue;
    break;
  }
done:;
  float sum = 0.0;
  for (int32_t k = 0; k < numTop; k++) {
    if (getIsHalfStopWikiBigram(bestwpi[k]))
      sum += (bestScores[k] * WIKI_BIGRAM_WEIGHT * WIKI_BIGRAM_WEIGHT);
    else
      sum += bestScores[k];
  }
  sum *= pt->freqWeights[i];
  sum *= pt->freqWeights[i];
  return sum;
}

/* getTermPairScoreForNonBody, Posdb.cpp:3305-3555 (m_msg2 != NULL) */
static void getTermPairScoreForNonBody(PT *pt, int i, int j, uint8_t *wpi, uint8_t *wpj,
                                       uint8_t *endi, uint8_t *endj, int32_t qdist, float *retMax) {
  (void)pt; (void)i; (void)j;
  int32_t p1 = getWordPos(wpi);
  int32_t p2 = getWordPos(wpj);
  unsigned char hg1 = getHashGroup(wpi);
  unsigned char hg2 = getHashGroup(wpj);
  unsigned char wsr1 = getWordSpamRank(wpi);
  unsigned char wsr2 = getWordSpamRank(wpj);
  float spamw1, spamw2;
  if (hg1 == HASHGROUP_INLINKTEXT) spamw1 = s_linkerWeights[wsr1];
  else spamw1 = s_wordSpamWeights[wsr1];
  if (hg2 == HASHGROUP_INLINKTEXT) spamw2 = s_linkerWeights[wsr2];
  else spamw2 = s_wordSpamWeights[wsr2];
  float denw1 = s_densityWeights[getDensityRank(wpi)];
  float denw2 = s_densityWeights[getDensityRank(wpj)];
  int firsti = 1, firstj = 1;
  float score;
  float max = -1.0;
  int32_t dist;
  for (;;) {
    if (p1 <= p2) {
      if (!s_isCompatible[hg1][hg2]) goto skip1;
      dist = p2 - p1;
      if (dist < 2) dist = 2;
      if (dist > 50) dist = FIXED_DISTANCE;
      if (dist >= qdist) dist = dist - qdist;
      score = 100 * denw1 * denw2;
      score *= s_hashGroupWeights[hg1];
      score *= s_hashGroupWeights[hg2];
      if (getIsSynonym(wpi)) score *= SYNONYM_WEIGHT;
      if (getIsSynonym(wpj)) score *= SYNONYM_WEIGHT;
      score *= spamw1 * spamw2;
      score /= (dist + 1.0);
      if (score > max) max = score;
    skip1:
      if (firsti) { wpi += 6; firsti = 0; }
      wpi += 6;
      if (wpi >= endi) break;
      if (keySize(wpi) != 6) break;
      p1 = getWordPos(wpi);
      hg1 = getHashGroup(wpi);
      denw1 = s_densityWeights[getDensityRank(wpi)];
      if (hg1 == HASHGROUP_INLINKTEXT) spamw1 = s_linkerWeights[getWordSpamRank(wpi)];
      else spamw1 = s_wordSpamWeights[getWordSpamRank(wpi)];
    } else {
      if (!s_isCompatible[hg1][hg2]) goto skip2;
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
      score *= s_hashGroupWeights[hg1];
      score *= s_hashGroupWeights[hg2];
      if (getIsSynonym(wpi)) score *= SYNONYM_WEIGHT;
      if (getIsSynonym(wpj)) score *= SYNONYM_WEIGHT;
      score *= spamw1 * spamw2;
      score /= (dist + 1.0);
      if (score > max) max = score;
    skip2:
      if (firstj) { wpj += 6; firstj = 0; }
      wpj += 6;
      if (wpj >= endj) break;
      if (keySize(wpj) != 6) break;
      p2 = getWordPos(wpj);
      hg2 = getHashGroup(wpj);
      denw2 = s_densityWeights[getDensityRank(wpj)];
      if (hg2 == HASHGROUP_INLINKTEXT) spamw2 = s_linkerWeights[getWordSpamRank(wpj)];
      else spamw2 = s_wordSpamWeights[getWordSpamRank(wpj)];
    }
  }
  *retMax = max;
}

/* getTermPairScoreForWindow, Posdb.cpp:3557-3625 */
static float getTermPairScoreForWindow(PT *pt, uint8_t *wpi, uint8_t *wpj, int32_t fixedDistance) {
  if (!wpi) return -1.00;
  if (!wpj) return -1.00;
  int32_t p1 = getWordPos(wpi);
  int32_t p2 = getWordPos(wpj);
  unsigned char hg1 = getHashGroup(wpi);
  unsigned char hg2 = getHashGroup(wpj);
  unsigned char wsr1 = getWordSpamRank(wpi);
  unsigned char wsr2 = getWordSpamRank(wpj);
  float spamw1, spamw2, denw1, denw2, dist, score;
  if (hg1 == HASHGROUP_INLINKTEXT) spamw1 = s_linkerWeights[wsr1];
  else spamw1 = s_wordSpamWeights[wsr1];
  if (hg2 == HASHGROUP_INLINKTEXT) spamw2 = s_linkerWeights[wsr2];
  else spamw2 = s_wordSpamWeights[wsr2];
  denw1 = s_densityWeights[getDensityRank(wpi)];
  denw2 = s_densityWeights[getDensityRank(wpj)];
  if (fixedDistance != 0) {
    dist = fixedDistance;
  } else {
    if (p2 < p1) dist = p1 - p2;
    else dist = p2 - p1;
    if (dist < 2) dist = 2;
    if (dist >= pt->qdist) dist = dist - pt->qdist;
    if (p2 < p1) dist += 1;
  }
  score = 100 * denw1 * denw2;
  score *= s_hashGroupWeights[hg1];
  score *= s_hashGroupWeights[hg2];
  if (getIsSynonym(wpi)) score *= SYNONYM_WEIGHT;
  if (getIsSynonym(wpj)) score *= SYNONYM_WEIGHT;
  score *= spamw1 * spamw2;
  score /= (dist + 1.0);
  return score;
}

/* evalSlidingWindow, Posdb.cpp:1275-1511 */
static void evalSlidingWindow(PT *pt, uint8_t **ptrs, int32_t nr, uint8_t **bestPos,
                              float *scoreMatrix) {
  float wikiWeight;
  float minTermPairScoreInWindow = 999999999.0;
  int32_t maxi = nr;
  for (int32_t i = 0; i < maxi; i++) {
    if (pt->bflags[i] & BF_EXCLUDE) continue;
    uint8_t *wpi = ptrs[i];
    for (int32_t j = i + 1; j < nr; j++) {
      if (pt->bflags[j] & BF_EXCLUDE) continue;
      uint8_t *wpj = ptrs[j];
      if (pt->wikiPhraseIds[j] == pt->wikiPhraseIds[i] && pt->wikiPhraseIds[j]) {
        pt->qdist = pt->qpos[j] - pt->qpos[i];
        wikiWeight = WIKI_WEIGHT;
      } else {
        pt->qdist = 2;
        wikiWeight = 1.0;
      }
      float max = getTermPairScoreForWindow(pt, wpi, wpj, 0);
      float score = getTermPairScoreForWindow(pt, bestPos[i], wpj, FIXED_DISTANCE);
      if (score > max) max = score;
      score = getTermPairScoreForWindow(pt, bestPos[i], bestPos[j], FIXED_DISTANCE);
      if (score > max) max = score;
      score = getTermPairScoreForWindow(pt, wpi, bestPos[j], FIXED_DISTANCE);
      if (score > max) max = score;
      if (wikiWeight != 1.0) max *= wikiWeight;
      max *= pt->freqWeights[i] * pt->freqWeights[j];
      if (scoreMatrix[pt->nqt * i + j] > max) max = scoreMatrix[pt->nqt * i + j];
      if (pt->quotedStartIds[j] >= 0 && pt->quotedStartIds[j] == pt->quotedStartIds[i]) {
        if (!wpi) {
          max = -1.0;
        } else if (!wpj) {
          max = -1.0;
        } else {
          int32_t qdist = pt->qpos[j] - pt->qpos[i];
          int32_t p1 = getWordPos(wpi);
          int32_t p2 = getWordPos(wpj);
          int32_t dist = p2 - p1;
          if (dist < 0) max = -1.0;
          else if (dist > qdist && dist - qdist > 1) max = -1.0;
          else if (dist < qdist && qdist - dist > 1) max = -1.0;
        }
      }
      if (max < minTermPairScoreInWindow) minTermPairScoreInWindow = max;
    }
  }
  if (minTermPairScoreInWindow <= pt->bestWindowScore) return;
  pt->bestWindowScore = minTermPairScoreInWindow;
  for (int32_t i = 0; i < maxi; i++) pt->windowTermPtrs[i] = ptrs[i];
}

/* getTermPairScoreForAny, Posdb.cpp:3631-4344 (pdcs == NULL) */
static float getTermPairScoreForAny(PT *pt, int32_t i, int32_t j, uint8_t *wpi, uint8_t *wpj,
                                    uint8_t *endi, uint8_t *endj, int *corrupt) {
  float wts;
  int32_t qdist;
  if (pt->wikiPhraseIds[j] == pt->wikiPhraseIds[i] && pt->wikiPhraseIds[j]) {
    qdist = pt->qpos[j] - pt->qpos[i];
    wts = (float)WIKI_WEIGHT;
  } else {
    qdist = 2;
    wts = 1.0;
  }
  int inSameQuotedPhrase = 0;
  if (pt->quotedStartIds[i] == pt->quotedStartIds[j] && pt->quotedStartIds[i] >= 0)
    inSameQuotedPhrase = 1;
  if (inSameQuotedPhrase) qdist = pt->qpos[j] - pt->qpos[i];
  int32_t p1 = getWordPos(wpi);
  int32_t p2 = getWordPos(wpj);
  unsigned char hg1 = getHashGroup(wpi);
  unsigned char hg2 = getHashGroup(wpj);
  unsigned char mhg1 = hg1, mhg2 = hg2;
  if (s_inBody[mhg1]) mhg1 = HASHGROUP_BODY;
  if (s_inBody[mhg2]) mhg2 = HASHGROUP_BODY;
  unsigned char wsr1 = getWordSpamRank(wpi);
  unsigned char wsr2 = getWordSpamRank(wpj);
  float spamw1, spamw2;
  if (hg1 == HASHGROUP_INLINKTEXT) spamw1 = s_linkerWeights[wsr1];
  else spamw1 = s_wordSpamWeights[wsr1];
  if (hg2 == HASHGROUP_INLINKTEXT) spamw2 = s_linkerWeights[wsr2];
  else spamw2 = s_wordSpamWeights[wsr2];
  float denw1 = s_densityWeights[getDensityRank(wpi)];
  float denw2 = s_densityWeights[getDensityRank(wpj)];
  int firsti = 1, firstj = 1;
  float score;
  int32_t minx = -1;
  float bestScores[MAX_TOP];
  char bestmhg1[MAX_TOP];
  char bestmhg2[MAX_TOP];
  int32_t numTop = 0;
  int32_t dist;
  int32_t bro;
  char syn1, syn2;
  for (;;) {
    if (s_inBody[hg1] && wpi != pt->windowTermPtrs[i]) goto skip1;
    if (s_inBody[hg2] && wpj != pt->windowTermPtrs[j]) goto skip2;
    if (p1 <= p2) {
      dist = p2 - p1;
      if (inSameQuotedPhrase) {
        if (dist > qdist && dist - qdist >= 2) goto skip1;
        if (dist < qdist && qdist - dist >= 2) goto skip1;
      }
      syn1 = getIsSynonym(wpi);
      syn2 = getIsSynonym(wpj);
      if (dist < 2) dist = 2;
      if (dist < 50) {
      } else if (mhg1 != mhg2) {
        dist = FIXED_DISTANCE;
      } else if (mhg1 == HASHGROUP_INLINKTEXT) {
        dist = FIXED_DISTANCE;
      }
      if (dist >= qdist) dist = dist - qdist;
      score = 100 * denw1 * denw2;
      score *= s_hashGroupWeights[hg1];
      score *= s_hashGroupWeights[hg2];
      if (syn1) score *= SYNONYM_WEIGHT;
      if (syn2) score *= SYNONYM_WEIGHT;
      if (getIsHalfStopWikiBigram(wpi)) score *= WIKI_BIGRAM_WEIGHT;
      if (getIsHalfStopWikiBigram(wpj)) score *= WIKI_BIGRAM_WEIGHT;
      score *= spamw1 * spamw2;
      score /= (dist + 1.0);
      bro = -1;
      for (int32_t k = 0; k < numTop; k++) {
        if (bestmhg1[k] == mhg1 && hg1 != HASHGROUP_INLINKTEXT) { bro = k; break; }
        if (bestmhg2[k] == mhg2 && hg2 != HASHGROUP_INLINKTEXT) { bro = k; break; }
      }
      if (bro >= 0) {
        if (score > bestScores[bro]) {
          bestScores[bro] = score;
          bestmhg1[bro] = mhg1;
          bestmhg2[bro] = mhg2;
        }
      } else if (numTop < pt->realMaxTop) {
        bestScores[numTop] = score;
        bestmhg1[numTop] = mhg1;
        bestmhg2[numTop] = mhg2;
        numTop++;
      } else if (score > bestScores[minx]) {
        bestScores[minx] = score;
        bestmhg1[minx] = mhg1;
        bestmhg2[minx] = mhg2;
      }
      if (numTop >= pt->realMaxTop) {
        minx = 0;
        for (int32_t k = 1; k < pt->realMaxTop; k++) {
          if (bestScores[k] > bestScores[minx]) continue;
          minx = k;
        }
      }
    skip1:
      if (firsti) { wpi += 6; firsti = 0; }
      wpi += 6;
      if (wpi >= endi) break;
      if (keySize(wpi) != 6) {
        if (getDocId(wpi) != pt->docId) { *corrupt = 1; break; }
        firsti = 1;
      }
      p1 = getWordPos(wpi);
      hg1 = getHashGroup(wpi);
      mhg1 = hg1;
      if (s_inBody[mhg1]) mhg1 = HASHGROUP_BODY;
      denw1 = s_densityWeights[getDensityRank(wpi)];
      if (hg1 == HASHGROUP_INLINKTEXT) spamw1 = s_linkerWeights[getWordSpamRank(wpi)];
      else spamw1 = s_wordSpamWeights[getWordSpamRank(wpi)];
      continue;
    } else {
      dist = p1 - p2;
      if (inSameQuotedPhrase) goto skip2;
      if (dist < 2) dist = 2;
      if (dist < 50) {
      } else if (mhg1 != mhg2) {
        dist = FIXED_DISTANCE;
      } else if (mhg1 == HASHGROUP_INLINKTEXT) {
        dist = FIXED_DISTANCE;
      }
      if (dist >= qdist) {
        dist = dist - qdist;
        dist += qdist - 1;
      } else {
        dist += 1;
      }
      score = 100 * denw1 * denw2;
      score *= s_hashGroupWeights[hg1];
      score *= s_hashGroupWeights[hg2];
      if (getIsSynonym(wpi)) score *= SYNONYM_WEIGHT;
      if (getIsSynonym(wpj)) score *= SYNONYM_WEIGHT;
      score *= spamw1 * spamw2;
      score /= (dist + 1.0);
      bro = -1;
      for (int32_t k = 0; k < numTop; k++) {
        if (bestmhg1[k] == mhg1 && hg1 != HASHGROUP_INLINKTEXT) { bro = k; break; }
        if (bestmhg2[k] == mhg2 && hg2 != HASHGROUP_INLINKTEXT) { bro = k; break; }
      }
      if (bro >= 0) {
        if (score > bestScores[bro]) {
          bestScores[bro] = score;
          bestmhg1[bro] = mhg1;
          bestmhg2[bro] = mhg2;
        }
      } else if (numTop < pt->realMaxTop) {
        bestScores[numTop] = score;
        bestmhg1[numTop] = mhg1;
        bestmhg2[numTop] = mhg2;
        numTop++;
      } else if (score > bestScores[minx]) {
        bestScores[minx] = score;
        bestmhg1[minx] = mhg1;
        bestmhg2[minx] = mhg2;
      }
      if (numTop >= pt->realMaxTop) {
        minx = 0;
        for (int32_t k = 1; k < pt->realMaxTop; k++) {
          if (bestScores[k] > bestScores[minx]) continue;
          minx = k;
        }
      }
    skip2:
      if (firstj) { wpj += 6; firstj = 0; }
      wpj += 6;
      if (wpj >= endj) break;
      if (keySize(wpj) != 6) {
        if (getDocId(wpj) != pt->docId) { *corrupt = 1; break; }
        firstj = 1;
      }
      p2 = getWordPos(wpj);
      hg2 = getHashGroup(wpj);
      mhg2 = hg2;
      if (s_inBody[mhg2]) mhg2 = HASHGROUP_BODY;
      denw2 = s_densityWeights[getDensityRank(wpj)];
      if (hg2 == HASHGROUP_INLINKTEXT) spamw2 = s_linkerWeights[getWordSpamRank(wpj)];
      else spamw2 = s_wordSpamWeights[getWordSpamRank(wpj)];
      continue;
    }
  }
  float sum = 0.0;
  for (int32_t k = 0; k < numTop; k++) sum += bestScores[k];
  sum *= wts;
  sum *= pt->freqWeights[i];
  sum *= pt->freqWeights[j];
  return sum;
}

/* ------------------------------------------------- setQueryTermInfo etc. */
/* PosdbTable::setQueryTermInfo, Posdb.cpp:4354-4869 */
static int setQueryTermInfo(const orc_qterm *qt, int nqt, OList *lists, QTI *qip, int *nrgOut,
                            int64_t *minListSize, int *minListi) {
  int nrg = 0;
  for (int i = 0; i < nqt; i++) {
    if (!qt[i].is_required) continue;
    QTI *qti = &qip[nrg];
    memset(qti, 0, sizeof *qti);
    qti->qtermNum = i;
    qti->qpos = qt[i].qpos;
    qti->wikiPhraseId = qt[i].wiki_phrase_id;
    qti->quotedStartId = qt[i].quote_start;
    int nn = 0;
    int left = qt[i].left_phrase_term, right = qt[i].right_phrase_term;
    int leftTerm = left, rightTerm = right; /* m_leftPhraseTerm (NULL iff num < 0) */
    int leftAlreadyAdded = 0, rightAlreadyAdded = 0;
    char piped = qt[i].piped ? BF_PIPED : 0;
#define ADD(listIdx, flags)                                   \
    do {                                                      \
      if (nn >= MAX_SUBLISTS) return E2BIG;                   \
      qti->subList[nn] = (listIdx);                           \
      qti->bigramFlags[nn] = (char)(flags);                   \
      if (lists[(listIdx)].size) nn++;                        \
    } while (0)
    if (left >= 0 && leftTerm >= 0 && qt[leftTerm].is_wiki_half_stop_bigram) {
      leftAlreadyAdded = 1;
      ADD(left, BF_HALFSTOPWIKIBIGRAM | piped);
      for (int k = 0; k < nqt; k++)
        if (qt[k].synonym_of == leftTerm) ADD(k, BF_HALFSTOPWIKIBIGRAM | BF_SYNONYM | piped);
    }
    if (right >= 0 && rightTerm >= 0 && qt[rightTerm].is_wiki_half_stop_bigram) {
      rightAlreadyAdded = 1;
      ADD(right, BF_HALFSTOPWIKIBIGRAM | piped);
      for (int k = 0; k < nqt; k++)
        if (qt[k].synonym_of == rightTerm) ADD(k, BF_HALFSTOPWIKIBIGRAM | BF_SYNONYM | piped);
    }
    {
      int fl = piped;
      if (qt[i].term_sign == '-') fl |= BF_NEGATIVE;
      if (isNumberField(qt[i].field_code)) fl |= BF_NUMBER; /* Posdb.cpp:4572-4594 */
      if (qt[i].field_code == F_FACETSTR || qt[i].field_code == F_FACETINT || qt[i].field_code == F_FACETFLOAT)
        fl |= BF_FACET; /* Posdb.cpp:4597-4602 */
      ADD(i, fl);
    }
    qti->fieldCode = qt[i].field_code;
    qti->qwFloat = qt[i].number_float;
    qti->qwInt = qt[i].number_int;
    if (left >= 0 && !leftAlreadyAdded) {
      ADD(left, piped | BF_BIGRAM);
      for (int k = 0; k < nqt; k++)
        if (leftTerm >= 0 ? qt[k].synonym_of == leftTerm : qt[k].synonym_of < 0)
          ADD(k, BF_SYNONYM | piped);
    }
    if (right >= 0 && !rightAlreadyAdded) {
      ADD(right, BF_BIGRAM | piped);
      for (int k = 0; k < nqt; k++)
        if (rightTerm >= 0 ? qt[k].synonym_of == rightTerm : qt[k].synonym_of < 0)
          ADD(k, BF_SYNONYM | piped);
    }
    for (int k = 0; k < nqt; k++)
      if (qt[k].synonym_of == i) ADD(k, BF_SYNONYM | piped);
#undef ADD
    qti->numSubLists = nn;
    qti->termFreqWeight = qt[i].tf_weight;
    if (nn >= MAX_SUBLISTS) return E2BIG; /* "too many sublists" */
    qti->totalSubListsSize = 0;
    for (int q = 0; q < nn; q++) qti->totalSubListsSize += lists[qti->subList[q]].size;
    nrg++;
  }
  *minListSize = 0;
  *minListi = -1;
  for (int i = 0; i < nrg; i++) {
    QTI *qti = &qip[i];
    if (qti->bigramFlags[0] & BF_NEGATIVE) continue;
    int64_t total = qti->totalSubListsSize;
    if (total < *minListSize || *minListi == -1) {
      *minListSize = total;
      *minListi = i;
    }
  }
  *nrgOut = nrg;
  return 0;
}

/* docid-record compare helpers (Posdb.cpp:5100-5113) */
static inline int vcmp(const uint8_t *dp, const uint8_t *rec) {
  uint32_t a = U32(dp + 1), b = U32(rec + 8);
  if (a > b) return 1;
  if (a < b) return -1;
  unsigned char x = dp[0], y = rec[7] & 0xfc;
  if (x > y) return 1;
  if (x < y) return -1;
  return 0;
}

typedef struct {
  uint8_t *buf;
  int64_t len;
} VoteBuf;

/* The whitelist table (allocWhiteListTable + the fill of Posdb.cpp:5544-
 * 5572): the 5 bytes at rec+7 of every record of every whitelist list,
 * walked with RdbList::skipCurrentRecord's posdb record sizes (18 first, then
 * 6 if byte0&0x04, 12 if byte0&0x02, else 18).  For a 6-byte record rec+7
 * lies in the record after it, as in the reference; bytes past the list end
 * (read from the reference's allocation slack: undefined) read as 0 here.
 * Membership is exact (HashTableX compares the 5 key bytes), so a sorted
 * array stands in for the hash table. */
typedef struct {
  uint64_t *v;
  int64_t n;
} WhiteSet;

static uint64_t five_at(const uint8_t *p, const uint8_t *end) {
  uint64_t x = 0;
  for (int b = 4; b >= 0; b--) x = (x << 8) | (p + b < end ? p[b] : 0);
  return x;
}
static int cmp_u64(const void *a, const void *b) {
  const uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
  return x < y ? -1 : x > y;
}
static int white_build(const orc_params *prm, WhiteSet *ws) {
  ws->v = NULL;
  ws->n = 0;
  int64_t cap = 0;
  for (int i = 0; i < prm->n_white_lists; i++) cap += prm->white_lists[i].size / 6 + 1;
  ws->v = (uint64_t *)malloc(8 * (size_t)(cap > 0 ? cap : 1));
  if (!ws->v) return ENOMEM;
  for (int i = 0; i < prm->n_white_lists; i++) {
    const uint8_t *p = prm->white_lists[i].bytes, *end = p + prm->white_lists[i].size;
    for (int first = 1; p < end; first = 0) {
      ws->v[ws->n++] = five_at(p + 7, end);
      p += first ? 18 : ((p[0] & 0x04) ? 6 : ((p[0] & 0x02) ? 12 : 18));
    }
  }
  qsort(ws->v, (size_t)ws->n, 8, cmp_u64);
  return 0;
}
static int white_has(const WhiteSet *ws, const uint8_t *p) {
  uint64_t x = 0;
  for (int b = 4; b >= 0; b--) x = (x << 8) | p[b];
  int64_t lo = 0, hi = ws->n;
  while (lo < hi) {
    const int64_t m = (lo + hi) >> 1;
    if (ws->v[m] < x) lo = m + 1;
    else hi = m;
  }
  return lo < ws->n && ws->v[lo] == x;
}

/* isInRange / isInRange2, Posdb.cpp:4948-4999 */
static int isInRange(const uint8_t *p, const QTI *qti) {
  float f;
  int32_t v;
  memcpy(&f, p + 2, 4);
  memcpy(&v, p + 2, 4);
  switch (qti->fieldCode) {
    case F_NUMBERMIN: return f >= qti->qwFloat;
    case F_NUMBERMAX: return f <= qti->qwFloat;
    case F_NUMBEREQUALFLOAT: return f == qti->qwFloat;
    case F_NUMBERMININT: return v >= qti->qwInt;
    case F_NUMBERMAXINT: return v <= qti->qwInt;
    case F_NUMBEREQUALINT: return v == qti->qwInt;
  }
  return 1;
}
static int isInRange2(const uint8_t *recPtr, const uint8_t *subListEnd, const QTI *qti) {
  if (isInRange(recPtr, qti)) return 1;
  recPtr += 12;
  for (; recPtr < subListEnd && ((*recPtr) & 0x04); recPtr += 6)
    if (isInRange(recPtr, qti)) return 1;
  return 0;
}

/* addDocIdVotes, Posdb.cpp:5043-5332; ws: the whitelist table when the
 * request has one (Posdb.cpp:5294), else NULL */
static void addDocIdVotes(QTI *qti, int listGroupNum, OList *lists, VoteBuf *vb, const WhiteSet *ws) {
  const int isRangeTerm = isRangeField(qti->fieldCode);
  uint8_t *dp, *dpEnd, *recPtr, *subListEnd;
  for (int i = 0; i < qti->numSubLists && listGroupNum > 0; i++) {
    recPtr = lists[qti->subList[i]].list;
    subListEnd = recPtr + lists[qti->subList[i]].size;
    dp = vb->buf;
    dpEnd = dp + vb->len;
  subLoop:
    for (; dp < dpEnd; dp += 6) {
      int c = vcmp(dp, recPtr);
      if (c > 0) break;
      if (c < 0) continue;
      if (isRangeTerm && !isInRange2(recPtr, subListEnd, qti)) break; /* 5120-5121 */
      dp[5] = (uint8_t)listGroupNum;
      dp += 6;
      break;
    }
    if (dp >= dpEnd) continue;
    recPtr += 12;
    for (; recPtr < subListEnd && ((*recPtr) & 0x04); recPtr += 6);
    if (recPtr < subListEnd) goto subLoop;
  }
  if (listGroupNum > 0) {
    dp = vb->buf;
    dpEnd = dp + vb->len;
    uint8_t *dst = dp;
    for (; dp < dpEnd; dp += 6) {
      if ((signed char)dp[5] != listGroupNum) continue;
      memmove(dst, dp, 6);
      dst += 6;
    }
    vb->len = dst - vb->buf;
    return;
  }
  uint8_t *cursor[MAX_SUBLISTS], *cursorEnd[MAX_SUBLISTS];
  for (int i = 0; i < qti->numSubLists; i++) {
    cursor[i] = lists[qti->subList[i]].list;
    cursorEnd[i] = cursor[i] + lists[qti->subList[i]].size;
  }
  dp = vb->buf;
  uint8_t *minRecPtr, *lastMinRecPtr = NULL;
  int mini = -1;
  for (;;) {
    minRecPtr = NULL;
    for (int i = 0; i < qti->numSubLists; i++) {
      if (!cursor[i]) continue;
      recPtr = cursor[i];
      if (!minRecPtr) { minRecPtr = recPtr; mini = i; continue; }
      if (U32(recPtr + 8) > U32(minRecPtr + 8)) continue;
      if (U32(recPtr + 8) < U32(minRecPtr + 8)) { minRecPtr = recPtr; mini = i; continue; }
      if ((recPtr[7] & 0xfc) > (minRecPtr[7] & 0xfc)) continue;
      if ((recPtr[7] & 0xfc) < (minRecPtr[7] & 0xfc)) { minRecPtr = recPtr; mini = i; continue; }
    }
    if (!minRecPtr) {
      vb->len = dp - vb->buf;
      return;
    }
    int inRange = 0; /* Posdb.cpp:5242-5277 */
    if (isRangeTerm && isInRange2(cursor[mini], cursorEnd[mini], qti)) inRange = 1;
    cursor[mini] += 12;
    for (;;) {
      if (cursor[mini] >= cursorEnd[mini]) { cursor[mini] = NULL; break; }
      if (!(cursor[mini][0] & 0x04)) break;
      if (isRangeTerm && isInRange2(cursor[mini], cursorEnd[mini], qti)) inRange = 1;
      cursor[mini] += 6;
    }
    if (lastMinRecPtr && U32(lastMinRecPtr + 8) == U32(minRecPtr + 8) &&
        (lastMinRecPtr[7] & 0xfc) == (minRecPtr[7] & 0xfc))
      continue;
    /* not in the whitelist: not stored, lastMinRecPtr unchanged (5294) */
    if (ws && !white_has(ws, minRecPtr + 7)) continue;
    if (isRangeTerm && !inRange) continue; /* 5297-5298 */
    lastMinRecPtr = minRecPtr;
    memcpy(dp + 1, minRecPtr + 8, 4);
    dp[0] = minRecPtr[7] & 0xfc;
    dp[5] = 0;
    dp += 6;
  }
}

/* rmDocIdVotes, Posdb.cpp:4871-4946 */
static void rmDocIdVotes(QTI *qti, OList *lists, VoteBuf *vb) {
  uint8_t *dp = NULL, *dpEnd, *recPtr, *subListEnd;
  for (int i = 0; i < qti->numSubLists; i++) {
    recPtr = lists[qti->subList[i]].list;
    subListEnd = recPtr + lists[qti->subList[i]].size;
    dp = vb->buf;
    dpEnd = dp + vb->len;
  subLoop:
    for (; dp < dpEnd; dp += 6) {
      int c = vcmp(dp, recPtr);
      if (c > 0) break;
      if (c < 0) continue;
      dp[5] = 0xff;
      dp += 6;
      break;
    }
    if (dp >= dpEnd) continue;
    recPtr += 12;
    for (; recPtr < subListEnd && ((*recPtr) & 0x04); recPtr += 6);
    if (recPtr < subListEnd) goto subLoop;
  }
  dp = vb->buf;
  dpEnd = dp + vb->len;
  uint8_t *dst = dp;
  for (; dp < dpEnd; dp += 6) {
    if (dp[5] == 0xff) continue;
    memmove(dst, dp, 6);
    dst += 6;
  }
  vb->len = dst - vb->buf;
}

/* shrinkSubLists, Posdb.cpp:5334-5428 (in place, like the reference) */
static void shrinkSubLists(QTI *qti, OList *lists, VoteBuf *vb) {
  qti->numNewSubLists = 0;
  for (int i = 0; i < qti->numSubLists; i++) {
    uint8_t *recPtr = lists[qti->subList[i]].list;
    uint8_t *subListEnd = recPtr + lists[qti->subList[i]].size;
    uint8_t *dp = vb->buf;
    uint8_t *dpEnd = dp + vb->len;
    uint8_t *dst = recPtr;
    uint8_t *savedDst = dst;
  subLoop:
    for (;; dp += 6) {
      if (dp >= dpEnd) goto doneWithSubList;
      int c = vcmp(dp, recPtr);
      if (c > 0) break;
      if (c < 0) continue;
      memmove(dst, recPtr, 12);
      dst += 12;
      recPtr += 12;
      for (;;) {
        if (recPtr >= subListEnd) goto doneWithSubList;
        if (!(recPtr[0] & 0x04)) break;
        memmove(dst, recPtr, 6);
        dst += 6;
        recPtr += 6;
      }
    }
    recPtr += 12;
    for (;;) {
      if (recPtr >= subListEnd) goto doneWithSubList;
      if (!(recPtr[0] & 0x04)) break;
      recPtr += 6;
    }
    goto subLoop;
  doneWithSubList:;
    int x = qti->numNewSubLists;
    qti->newSubListSize[x] = dst - savedDst;
    qti->newSubListStart[x] = savedDst;
    qti->newSubListEnd[x] = dst;
    qti->cursor[x] = savedDst;
    qti->savedCursor[x] = savedDst;
    if (qti->newSubListSize[x]) qti->numNewSubLists++;
  }
}

/* --------------------------------------------------- pruning (clustering) */
typedef struct {
  float siteRankMultiplier;
  int language;
  float sameLangWeight;
  int allInSameWikiPhrase; /* m_allInSameWikiPhrase, Posdb.cpp:5764-5778 */
} MaxCtx;

/* getMaxPossibleScore, Posdb.cpp:7811-7960 (over the docid's shrunk-sublist
 * runs [m_savedCursor, m_cursor)) */
static float getMaxPossibleScore(const MaxCtx *c, QTI *qti, int32_t bestDist, int32_t qdist, QTI *qtm) {
  float bestHashGroupWeight = -1.0;
  unsigned char bestDensityRank = 0;
  char siteRank = -1;
  char docLang = 0;
  unsigned char hgrp;
  int hadHalfStopWikiBigram = 0;
  for (int j = 0; j < qti->numNewSubLists; j++) {
    uint8_t *start = qti->savedCursor[j];
    if (!start) continue;
    if (qti->bigramFlags[0] & BF_HALFSTOPWIKIBIGRAM) hadHalfStopWikiBigram = 1;
    if (start >= qti->newSubListEnd[j]) continue;
    if (siteRank == -1) {
      siteRank = (char)getSiteRank(start);
      docLang = (char)getLangId(start);
    }
    start += 12;
    uint8_t *dc = qti->cursor[j];
    dc -= 6;
    int retried = 0;
    for (; dc >= start; dc -= 6) {
    retry:
      hgrp = getHashGroup(dc);
      if (hgrp == HASHGROUP_INLINKTEXT) return -1.0;
      if (s_hashGroupWeights[hgrp] < bestHashGroupWeight) {
        if (hgrp == HASHGROUP_BODY) goto nextTermList;
        continue;
      }
      {
        char dr = (char)getDensityRank(dc);
        if (s_hashGroupWeights[hgrp] > bestHashGroupWeight) {
          if (hgrp == HASHGROUP_INLINKTEXT) return -1.0;
          bestHashGroupWeight = s_hashGroupWeights[hgrp];
          bestDensityRank = dr;
          continue;
        }
        if (dr < bestDensityRank) continue;
        if (dr > bestDensityRank) bestDensityRank = dr;
      }
    }
    /* the run's 12-byte key last (Posdb.cpp:7893-7897) */
    if (!retried) {
      retried = 1;
      dc = qti->savedCursor[j];
      goto retry;
    }
  nextTermList:
    continue;
  }
  if (bestHashGroupWeight < 0) return 0.0;
  float score = 100.0;
  score *= bestHashGroupWeight;
  score *= bestHashGroupWeight;
  score *= s_densityWeights[bestDensityRank];
  score *= s_densityWeights[bestDensityRank];
  if (hadHalfStopWikiBigram) {
    score *= WIKI_BIGRAM_WEIGHT;
    score *= WIKI_BIGRAM_WEIGHT;
  }
  score *= (((float)siteRank) * c->siteRankMultiplier + 1.0);
  if (c->language == (unsigned char)docLang || c->language == 0 || docLang == 0) score *= c->sameLangWeight;
  score *= qti->termFreqWeight;
  if (qdist) {
    score *= qtm->termFreqWeight;
    bestDist -= qdist;
    if (qdist < 0) qdist *= -1;
    if (bestDist < 0) bestDist *= -1;
    if (bestDist > 1) score /= (float)bestDist;
  }
  if (c->allInSameWikiPhrase) score *= WIKI_WEIGHT;
  return score;
}

#define RINGBUFSIZE 4096

/* The two prefilters of the per-docid loop, Posdb.cpp:6322-6504: 1 if the
 * docid is skipped (its bound cannot beat minWinningScore). */
static int prefilter_skip(const MaxCtx *c, QTI *qip, int nqti, int minListi, int doMaxScoreAlgo,
                          float minWinningScore, unsigned char *ringBuf, int32_t *ourFirstPos, int hasFacet) {
  const int nnn = doMaxScoreAlgo ? nqti : 0;
  for (int i = 0; i < nnn; i++) {
    if (qip[i].bigramFlags[0] & (BF_NEGATIVE | BF_FACET)) continue;
    float maxScore = getMaxPossibleScore(c, &qip[i], 0, 0, NULL);
    if (maxScore == -1.0) continue;
    if (maxScore <= minWinningScore) return 1;
  }
  /* a query with a facet term skips the scoring filter: facet stats are over
     every result (Posdb.cpp:6353-6356) */
  if (hasFacet) return 0;
  memset(ringBuf, 0xff, RINGBUFSIZE);
  QTI *qtx = &qip[minListi];
  for (int k = 0; k < qtx->numNewSubLists; k++) {
    uint8_t *sub = qtx->savedCursor[k];
    if (!sub) continue;
    uint8_t *end = qtx->cursor[k];
    uint32_t wx = U32(sub + 3) >> 6;
    wx &= (RINGBUFSIZE - 1);
    ringBuf[wx] = (unsigned char)minListi;
    *ourFirstPos = (int32_t)wx;
    sub += 12;
    for (; sub < end; sub += 6) {
      wx = U32(sub + 3) >> 6;
      wx &= (RINGBUFSIZE - 1);
      ringBuf[wx] = (unsigned char)minListi;
    }
  }
  for (int i = 0; i < nqti; i++) {
    if (i == minListi) continue;
    QTI *qti = &qip[i];
    if (qti->bigramFlags[0] & (BF_NEGATIVE | BF_FACET)) continue;
    for (int k = 0; k < qti->numNewSubLists; k++) {
      uint8_t *sub = qti->savedCursor[k];
      if (!sub) continue;
      uint8_t *end = qti->cursor[k];
      uint32_t wx = U32(sub + 3) >> 6;
      wx &= (RINGBUFSIZE - 1);
      ringBuf[wx] = (unsigned char)i;
      sub += 12;
      for (; sub < end; sub += 6) {
        wx = U32(sub + 3) >> 6;
        wx &= (RINGBUFSIZE - 1);
        ringBuf[wx] = (unsigned char)i;
      }
    }
    int32_t ourLastPos = -1;
    int32_t hisLastPos = -1;
    int32_t bestDist = 0x7fffffff;
    for (int32_t x = 0; x < (int32_t)RINGBUFSIZE;) {
      if (U32(ringBuf + x) == 0xffffffff) {
        x += 4;
        continue;
      }
      if (ringBuf[x] == 0xff) {
        x++;
        continue;
      }
      unsigned char qt = ringBuf[x];
      if (qt == minListi) {
        hisLastPos = x;
        if (ourLastPos == -1) {
          x++;
          continue;
        }
        if (x - ourLastPos < bestDist) bestDist = x - ourLastPos;
      } else if (qt == i) {
        ourLastPos = x;
        if (hisLastPos == -1) {
          x++;
          continue;
        }
        ourLastPos = x;
        if (x - hisLastPos < bestDist) bestDist = x - hisLastPos;
      }
      x++;
    }
    int32_t wrapDist = *ourFirstPos + ((int32_t)RINGBUFSIZE - hisLastPos);
    if (wrapDist < bestDist) bestDist = wrapDist;
    int32_t qdist = qip[minListi].qpos - qip[i].qpos;
    float maxScore2 = getMaxPossibleScore(c, &qip[i], bestDist, qdist, &qip[minListi]);
    if (maxScore2 == -1.0) continue;
    if (maxScore2 <= minWinningScore) return 1;
  }
  return 0;
}

/* ----------------------------------------------------------------- facets */
/* QueryTerm::m_facetHashTable (key = the facet value's 32 bits, or a range's
 * A value) of FacetEntry (Posdb.h:401-413), per facet query term; kept over
 * the docid-range pieces of one query (Posdb.cpp:1040, 5593) */
typedef struct {
  int32_t key, count, outside;
  int64_t docid, sum;
  int32_t max, min;
} FEnt;
typedef struct {
  int live;
  int term;
  uint64_t docs; /* m_numDocsThatHaveFacet */
  FEnt *e;
  int n, cap;
} FTable;
#define ORC_MAXF 16
static FTable s_ft[ORC_MAXF];
static int s_nft = 0;

static FEnt *ft_get(FTable *t, int32_t key) {
  for (int i = 0; i < t->n; i++)
    if (t->e[i].key == key) return &t->e[i];
  return NULL;
}
static FEnt *ft_add(FTable *t, int32_t key) {
  if (t->n == t->cap) {
    t->cap = t->cap ? 2 * t->cap : 64;
    t->e = (FEnt *)realloc(t->e, sizeof(FEnt) * (size_t)t->cap);
  }
  FEnt *f = &t->e[t->n++];
  memset(f, 0, sizeof *f);
  f->key = key;
  return f;
}
static void ft_reset(void) {
  for (int i = 0; i < ORC_MAXF; i++) {
    free(s_ft[i].e);
    memset(&s_ft[i], 0, sizeof s_ft[i]);
  }
  s_nft = 0;
}
static const orc_facet_ranges *facet_ranges_of(const orc_params *prm, int term) {
  for (int i = 0; i < prm->n_facet_ranges; i++)
    if (prm->facet_ranges[i].term == term) return &prm->facet_ranges[i];
  return NULL;
}
static int isFacetField(int fc) { return fc == F_FACETSTR || fc == F_FACETINT || fc == F_FACETFLOAT; }
static int cmp_fent(const void *a, const void *b) {
  const int32_t x = ((const FEnt *)a)->key, y = ((const FEnt *)b)->key;
  return x < y ? -1 : x > y;
}
/* stale-mbuf docids of the last orc_query (see run_range): scored from the
 * bytes earlier docids left, and skipped (never written in the pass) */
static int s_stale_def = 0, s_stale_undef = 0;
void orc_last_stale(int32_t *defined, int32_t *undefined) {
  *defined = s_stale_def;
  *undefined = s_stale_undef;
}

int orc_last_facets(int32_t *w, int cap) {
  int k = 0;
  if (cap < 1) return -1;
  w[k++] = s_nft;
  for (int i = 0; i < s_nft; i++) {
    FTable *t = &s_ft[i];
    qsort(t->e, (size_t)t->n, sizeof(FEnt), cmp_fent);
    if (k + 4 + 9 * t->n > cap) return -1;
    w[k++] = t->term;
    memcpy(&w[k], &t->docs, 8);
    k += 2;
    w[k++] = t->n;
    for (int j = 0; j < t->n; j++) {
      const FEnt *f = &t->e[j];
      w[k++] = f->key;
      w[k++] = f->count;
      w[k++] = f->outside;
      memcpy(&w[k], &f->docid, 8);
      k += 2;
      memcpy(&w[k], &f->sum, 8);
      k += 2;
      w[k++] = f->max;
      w[k++] = f->min;
    }
  }
  return k;
}

/* ---------------------------------------------------------------- driver */
#define LIST_PAD 64

static void free_lists(OList *L, uint8_t **alloc, int n) {
  for (int i = 0; i < n; i++) free(alloc[i]);
  free(alloc);
  free(L);
}

/* copies + Msg39 early outs; returns 0 and fills everything up to the votes */
typedef struct {
  OList *lists;
  uint8_t **alloc;
  QTI *qip;
  int nrg;
  int64_t minListSize;
  int minListi;
  VoteBuf vb;
  int64_t grand;      /* the positive groups' list bytes (m_docIdVoteBuf's boolean size) */
  uint32_t *bvec;     /* boolean: each vote-buffer docid's QueryTermInfo bit vector (m_bt) */
} Prep;

static int prepare(const orc_qterm *qt, const uint8_t *const *lists, const int64_t *sizes, int nqt,
                   Prep *P, int boolean) {
  memset(P, 0, sizeof *P);
  P->lists = (OList *)calloc(nqt > 0 ? nqt : 1, sizeof(OList));
  P->alloc = (uint8_t **)calloc(nqt > 0 ? nqt : 1, sizeof(uint8_t *));
  P->qip = (QTI *)calloc(nqt > 0 ? nqt : 1, sizeof(QTI));
  if (!P->lists || !P->alloc || !P->qip) return ENOMEM;
  for (int i = 0; i < nqt; i++) {
    int64_t sz = sizes[i];
    if (sz < 0 || (sz && !lists[i])) return EINVAL;
    /* zero padding guards the reference's reads just past a list end */
    P->alloc[i] = (uint8_t *)calloc(1, (size_t)sz + 2 * LIST_PAD);
    if (!P->alloc[i]) return ENOMEM;
    if (sz) memcpy(P->alloc[i] + LIST_PAD, lists[i], (size_t)sz);
    P->lists[i].list = P->alloc[i] + LIST_PAD;
    P->lists[i].size = sz;
  }
  int rc = setQueryTermInfo(qt, nqt, P->lists, P->qip, &P->nrg, &P->minListSize, &P->minListi);
  if (rc) return rc;
  /* Posdb.cpp:4813-4826: grand = the positive groups' sizes; a boolean
   * query's vote buffer may hold every one of their docids */
  for (int i = 0; i < P->nrg; i++)
    if (!(P->qip[i].bigramFlags[0] & BF_NEGATIVE)) P->grand += P->qip[i].totalSubListsSize;
  /* first-key swap, Posdb.cpp:5671-5703 */
  for (int k = 0; k < nqt; k++) {
    OList *l = &P->lists[k];
    if (!l->size) continue;
    uint8_t ttt[12];
    uint8_t *p = l->list;
    memcpy(ttt, p, 12);
    memcpy(p, p + 12, 6);
    memcpy(p + 6, ttt, 12);
    p += 6;
    *p |= 0x02;
    l->size -= 6;
    l->list = p;
  }
  int64_t need = (P->minListSize / 12) * 6 + 8;
  if (boolean) {
    /* Posdb.cpp:4826: grand -- but the union runs over every group, negative
     * ones included (Posdb.cpp:8026-8153), so size for all lists here */
    need = 8;
    for (int i = 0; i < nqt; i++) need += P->lists[i].size + 6;
  }
  P->vb.buf = (uint8_t *)calloc(1, (size_t)need + 16);
  if (!P->vb.buf) return ENOMEM;
  return 0;
}

static void unprepare(Prep *P, int nqt) {
  free(P->vb.buf);
  free(P->bvec);
  free(P->qip);
  if (P->lists) free_lists(P->lists, P->alloc, nqt);
}

/* phases 3-4 of intersectLists10_r, Posdb.cpp:5808-5860 */
static void votes(Prep *P, const WhiteSet *ws) {
  QTI *qip = P->qip;
  int listGroupNum = 0;
  addDocIdVotes(&qip[P->minListi], listGroupNum, P->lists, &P->vb, ws);
  for (int i = 0; i < P->nrg; i++) {
    if (i == P->minListi) continue;
    if (qip[i].bigramFlags[0] & BF_NEGATIVE) continue;
    listGroupNum++;
    if (listGroupNum >= 256) listGroupNum = 1;
    addDocIdVotes(&qip[i], listGroupNum, P->lists, &P->vb, NULL);
  }
  for (int i = 0; i < P->nrg; i++) {
    if (i == P->minListi) continue;
    if (!(qip[i].bigramFlags[0] & BF_NEGATIVE)) continue;
    rmDocIdVotes(&qip[i], P->lists, &P->vb);
  }
}

/* makeDocIdVoteBufForBoolQuery_r, Posdb.cpp:8006-8249: every group's
 * sublists (negative groups too) are walked run by run; a docid takes the bit
 * of each QueryTermInfo it occurs in (QueryTerm::m_bitNum = the group index,
 * Posdb.cpp:4485-4721) -- a range term's run only if one of its keys is in
 * range (isInRange, 8087-8129) -- and is voted if the expression holds for
 * its bit vector (the truth table stands for m_ct / Query::matchesBoolQuery,
 * 8164-8231).  The vote buffer is sorted by docid (dcmp6, 8237-8244); bvec
 * keeps each voted docid's vector (m_bt) for the score (Posdb.cpp:6514-6534). */
typedef struct {
  uint64_t d;
  uint32_t bits;
} BEnt;
static int bent_cmp(const void *a, const void *b) {
  const uint64_t x = ((const BEnt *)a)->d, y = ((const BEnt *)b)->d;
  return x < y ? -1 : x > y ? 1 : 0;
}
static int boolVotes(Prep *P, const orc_params *prm) {
  QTI *qip = P->qip;
  int64_t cap = 16, n = 0;
  BEnt *e = (BEnt *)malloc(sizeof(BEnt) * cap);
  if (!e) return ENOMEM;
  for (int i = 0; i < P->nrg; i++) {
    QTI *qti = &qip[i];
    const int isRange = isRangeField(qti->fieldCode);
    const uint32_t mask = 1u << i;
    for (int j = 0; j < qti->numSubLists; j++) {
      const OList *L = &P->lists[qti->subList[j]];
      const uint8_t *p = L->list, *pend = L->list + L->size;
      while (p < pend) {
        const uint64_t d = getDocId(p);
        int inRange = 0;
        if (isRange && isInRange(p, qti)) inRange = 1;
        if (p[0] & 0x02) p += 12;
        else p += 18;
        while (p < pend && (p[0] & 0x04)) {
          if (isRange && isInRange(p, qti)) inRange = 1;
          p += 6;
        }
        if (isRange && !inRange) continue;
        if (n == cap) {
          cap *= 2;
          BEnt *ne = (BEnt *)realloc(e, sizeof(BEnt) * cap);
          if (!ne) { free(e); return ENOMEM; }
          e = ne;
        }
        e[n].d = d;
        e[n].bits = mask;
        n++;
      }
    }
  }
  qsort(e, (size_t)n, sizeof(BEnt), bent_cmp);
  P->bvec = (uint32_t *)malloc(sizeof(uint32_t) * (size_t)(n ? n : 1));
  if (!P->bvec) { free(e); return ENOMEM; }
  int64_t nv = 0;
  uint8_t *dst = P->vb.buf;
  for (int64_t a = 0; a < n;) {
    int64_t b = a;
    uint32_t v = 0;
    while (b < n && e[b].d == e[a].d) v |= e[b++].bits;
    if (prm->bool_table[v >> 3] >> (v & 7) & 1) {
      const uint64_t x = e[a].d << 2; /* a 6-byte record: docid << 2 (Posdb.cpp:8196-8209) */
      for (int k = 0; k < 6; k++) dst[k] = (uint8_t)(x >> (8 * k));
      dst += 6;
      P->bvec[nv++] = v;
    }
    a = b;
  }
  P->vb.len = dst - P->vb.buf;
  free(e);
  return 0;
}

int64_t orc_intersect(const orc_qterm *qt, const uint8_t *const *lists, const int64_t *sizes,
                      int nqt, int64_t *docids, int64_t cap, const orc_params *prm) {
  initWeights();
  WhiteSet ws = {NULL, 0};
  if (prm && prm->use_whitelist && white_build(prm, &ws)) return -ENOMEM;
  Prep P;
  const int boolean = prm && prm->is_boolean;
  int rc = prepare(qt, lists, sizes, nqt, &P, boolean);
  if (rc) { unprepare(&P, nqt); free(ws.v); return -rc; }
  int64_t n = 0;
  if (boolean && P.nrg > 0) {
    if (prm->bool_ngroups != P.nrg || !prm->bool_table) { unprepare(&P, nqt); free(ws.v); return -EINVAL; }
    rc = boolVotes(&P, prm);
    if (rc) { unprepare(&P, nqt); free(ws.v); return -rc; }
    n = P.vb.len / 6;
    for (int64_t i = 0; i < n && i < cap; i++) {
      const uint8_t *d = P.vb.buf + 6 * i;
      uint64_t id = U32(d + 1);
      id <<= 8;
      id |= d[0];
      docids[i] = (int64_t)(id >> 2);
    }
  } else if (P.nrg > 0 && P.minListSize != 0) {
    votes(&P, (prm && prm->use_whitelist) ? &ws : NULL);
    n = P.vb.len / 6;
    for (int64_t i = 0; i < n && i < cap; i++) {
      const uint8_t *d = P.vb.buf + 6 * i;
      uint64_t id = U32(d + 1);
      id <<= 8;
      id |= d[0];
      docids[i] = (int64_t)(id >> 2);
    }
  }
  unprepare(&P, nqt);
  free(ws.v);
  return n;
}

/* allocTopTree sizing, Posdb.cpp:838-930 + TopTree::setNumNodes */
static int64_t docs_wanted(const orc_params *p, const int64_t *sizes, int nqt) {
  int64_t nn1 = p->docs_to_get, nn2 = 0;
  for (int k = 0; k < nqt; k++) {
    if (!sizes[k]) continue;
    nn2 += (int32_t)sizes[k] / (18 - 6);
  }
  if (p->num_docid_splits > 1) { /* Posdb.cpp:859-877 */
    if (nn2 < 100) nn2 = 100;
    nn2 *= p->num_docid_splits;
    nn2 *= 2;
    if (nn1 < 100) nn1 = 100;
    nn1 *= p->num_docid_splits;
    nn1 *= 2;
  }
  int64_t nn = nn2;
  if (nn1 < nn2) nn = nn1;
  if (nn == 0) return 0;
  if (nn < 30) nn = 30;
  if (p->site_clustering) nn *= 2; /* Posdb.cpp:900 */
  if (nn > 2000000000) nn = 2000000000;
  if (nn > (int64_t)p->docs_to_get * 2 && nn > 60) nn = (int64_t)p->docs_to_get * 2;
  return nn;
}

/* One PosdbTable pass (init .. intersectLists10_r, Posdb.cpp:5437-7806) over
 * one docid range's lists, adding its winners to the caller's TopTree. */
static int run_range(const orc_qterm *qt, const uint8_t *const *lists, const int64_t *sizes, int nqt,
                     const orc_params *prm, const WhiteSet *ws, TTree *tree, orc_result *out) {
  Prep P;
  const int boolean = prm->is_boolean != 0;
  int rc = prepare(qt, lists, sizes, nqt, &P, boolean);
  if (rc) {
    unprepare(&P, nqt);
    return rc;
  }
  QTI *qip = P.qip;
  int nqti = P.nrg;
  /* Posdb.cpp:5728-5735: a boolean query goes on with an empty smallest group */
  if (nqti == 0 || (P.minListSize == 0 && !boolean)) goto finish;

  if (boolean) {
    if (prm->bool_ngroups != nqti || !prm->bool_table) {
      unprepare(&P, nqt);
      return EINVAL;
    }
    rc = boolVotes(&P, prm);
    if (rc) {
      unprepare(&P, nqt);
      return rc;
    }
  } else {
    votes(&P, ws);
  }
  out->hits = P.vb.len / 6;
  for (int i = 0; i < nqti; i++) {
    if (qip[i].bigramFlags[0] & BF_NEGATIVE) continue;
    shrinkSubLists(&qip[i], P.lists, &P.vb);
  }

  {
    int32_t *wikiPhraseIds = (int32_t *)calloc(nqt, 4);
    int32_t *quotedStartIds = (int32_t *)calloc(nqt, 4);
    int32_t *qpos = (int32_t *)calloc(nqt, 4);
    float *freqWeights = (float *)calloc(nqt, 4);
    uint8_t **mml = (uint8_t **)calloc(nqt, sizeof(uint8_t *));
    uint8_t **mme = (uint8_t **)calloc(nqt, sizeof(uint8_t *));
    uint8_t **bestPos = (uint8_t **)calloc(nqt, sizeof(uint8_t *));
    uint8_t **winnerStack = (uint8_t **)calloc(nqt, sizeof(uint8_t *));
    uint8_t **xpos = (uint8_t **)calloc(nqt, sizeof(uint8_t *));
    char *bflags = (char *)calloc(nqt, 1);
    char *rawg = (char *)calloc(nqt, 1); /* group not mini-merged (one numeric sublist) */
    float *scoreMatrix = (float *)calloc((size_t)nqt * nqt, 4);
    uint8_t *mbuf = (uint8_t *)calloc(1, 300000 + 64);
    uint8_t *mptrEnd = mbuf + 299000;
    size_t mhwm = 0; /* mbuf bytes any docid of this pass has written */
    for (int i = 0; i < nqti; i++) {
      wikiPhraseIds[i] = qip[i].wikiPhraseId;
      quotedStartIds[i] = qip[i].quotedStartId;
      qpos[i] = qip[i].qpos;
      freqWeights[i] = qip[i].termFreqWeight;
    }
    PT pt;
    memset(&pt, 0, sizeof pt);
    pt.realMaxTop = prm->real_max_top > MAX_TOP ? MAX_TOP : prm->real_max_top;
    pt.freqWeights = freqWeights;
    pt.qpos = qpos;
    pt.wikiPhraseIds = wikiPhraseIds;
    pt.quotedStartIds = quotedStartIds;
    pt.bflags = bflags;
    pt.windowTermPtrs = winnerStack;
    pt.nqt = nqt;
    float siteRankMultiplier = boolean ? 0.0f : SITERANKMULTIPLIER; /* Posdb.cpp:774 */
    char siteRank = 0, docLang = 0;
    float minWinningScore = -1.0; /* Posdb.cpp:6012: per pass */
    int sortByF = -1, sortByI = -1; /* m_sortByTermInfoNum(Int), Posdb.cpp:4413-4425 */
    for (int i = 0; i < nqti; i++) {
      if (qip[i].fieldCode == F_SORTBYFLOAT || qip[i].fieldCode == F_REVSORTBYFLOAT) sortByF = i;
      if (qip[i].fieldCode == F_SORTBYINT || qip[i].fieldCode == F_REVSORTBYINT) sortByI = i;
    }
    int32_t ourFirstPos = -1;
    unsigned char ringBuf[RINGBUFSIZE + 10];
    MaxCtx mc;
    mc.siteRankMultiplier = siteRankMultiplier;
    mc.language = prm->language;
    mc.sameLangWeight = prm->same_lang_weight;
    mc.allInSameWikiPhrase = 1;
    for (int i = 0; i < nqti; i++) {
      if (qip[i].bigramFlags[0] & (BF_NEGATIVE | BF_NUMBER | BF_FACET)) continue;
      if (qip[i].wikiPhraseId == 1) continue;
      mc.allInSameWikiPhrase = 0;
      break;
    }
    uint8_t *nwp[MAX_SUBLISTS], *nwpEnd[MAX_SUBLISTS];
    char nwpFlags[MAX_SUBLISTS];
    uint8_t *docIdEnd = P.vb.buf + P.vb.len;
    /* facet terms (allocTopTree, Posdb.cpp:1000-1067; the range buckets,
     * 5575-5631): a table per facet query term with a non-empty list (any,
     * over docid splits), its ranges as zeroed entries once */
    int fgroup[ORC_MAXF], fterm[ORC_MAXF], nf = 0, hasFacet = 0;
    for (int i = 0; i < nqt && nf < ORC_MAXF; i++) {
      if (!isFacetField(qt[i].field_code)) continue;
      if (sizes[i] == 0 && prm->num_docid_splits <= 1) continue;
      int g = -1;
      for (int k = 0; k < nqti; k++)
        if (qip[k].qtermNum == i) g = k;
      FTable *t = NULL;
      for (int k = 0; k < s_nft; k++)
        if (s_ft[k].term == i) t = &s_ft[k];
      if (!t) {
        t = &s_ft[s_nft++];
        t->live = 1;
        t->term = i;
      }
      hasFacet = 1;
      if (t->n == 0) {
        const orc_facet_ranges *fr = facet_ranges_of(prm, i);
        for (int k = 0; fr && k < fr->n; k++)
          if (!ft_get(t, fr->a[k])) ft_add(t, fr->a[k]);
      }
      fgroup[nf] = g;
      fterm[nf] = i;
      nf++;
    }

    for (uint8_t *docIdPtr = P.vb.buf; docIdPtr < docIdEnd; docIdPtr += 6) {
      float minScore = 999999999.0;
      /* cursor pre-advance, Posdb.cpp:6252-6310 */
      for (int i = 0; i < nqti; i++) {
        QTI *qti = &qip[i];
        if (qti->bigramFlags[0] & BF_NEGATIVE) continue;
        for (int j = 0; j < qti->numNewSubLists; j++) {
          uint8_t *xc = qti->cursor[j];
          uint8_t *xcEnd = qti->newSubListEnd[j];
          if (xc >= xcEnd || U32(xc + 8) != U32(docIdPtr + 1) ||
              (xc[7] & 0xfc) != (docIdPtr[0] & 0xfc)) {
            qti->savedCursor[j] = NULL;
            continue;
          }
          qti->savedCursor[j] = xc;
          xc += 12;
          for (;; xc += 6) {
            if (xc >= xcEnd) break;
            if ((*xc & 0x06) == 0x00) { out->corrupt = 1; goto doneAll; }
            if (!(*xc & 0x04)) break;
          }
          qti->cursor[j] = xc;
        }
      }
      /* the max-score and ring-buffer prefilters, Posdb.cpp:6322-6504 (live
       * only once the TopTree holds more than docsWanted nodes, i.e. with
       * site clustering: minWinningScore is -1 until then) */
      /* a boolean query: no prefilter, no mini merge that shows, no scorers --
       * minScore is the number of bits of the docid's vector and siteRank /
       * docLang keep their initial 0 (Posdb.cpp:5984-5985, 6312-6316,
       * 6514-6534, 6833-6834 -> boolJump2 at 7247) */
      if (boolean) {
        uint64_t d = U32(docIdPtr + 1);
        d <<= 8;
        d |= docIdPtr[0];
        pt.docId = d >> 2;
        minScore = (float)__builtin_popcount(P.bvec[(docIdPtr - P.vb.buf) / 6]);
        siteRank = 0;
        docLang = 0;
        /* the mini merge runs in a boolean query too (Posdb.cpp:6512-6778);
         * only the facet votes read its lists there: a facet group's one
         * sublist is the termlist's run itself (6638-6647), and a group the
         * docid is not in (the expression did not need it) is empty */
        for (int j = 0; hasFacet && j < nqti; j++) {
          QTI *qti = &qip[j];
          if (!(qti->bigramFlags[0] & BF_FACET)) continue;
          int nsub = 0;
          uint8_t *a = NULL, *e = NULL;
          char fl = 0;
          for (int k = 0; k < qti->numNewSubLists; k++) {
            if (!qti->savedCursor[k]) continue;
            a = qti->savedCursor[k];
            e = qti->cursor[k];
            fl = qti->bigramFlags[k];
            nsub++;
          }
          mml[j] = NULL;
          if (nsub == 1 && !(fl & (BF_SYNONYM | BF_HALFSTOPWIKIBIGRAM))) {
            mml[j] = a;
            mme[j] = e;
          }
        }
        goto boolJump2;
      }
      /* gbsortby: both prefilters off (Posdb.cpp:6050-6051, 6350-6351) */
      if (sortByF < 0 && sortByI < 0 &&
          prefilter_skip(&mc, qip, nqti, P.minListi, prm->do_max_score_algo, minWinningScore, ringBuf,
                         &ourFirstPos, hasFacet))
        continue;

      /* mini merges, Posdb.cpp:6559-6778 */
      {
        uint8_t *mptr = mbuf, *lastMptr = NULL;
        for (int j = 0; j < nqti; j++) {
          QTI *qti = &qip[j];
          bflags[j] = qti->bigramFlags[0];
          rawg[j] = 0;
          if (qti->bigramFlags[0] & BF_NEGATIVE) { mml[j] = NULL; continue; }
          mml[j] = mptr;
          int isFirstKey = 1;
          int nsub = 0;
          for (int k = 0; k < qti->numNewSubLists; k++) {
            if (!qti->savedCursor[k]) continue;
            nwp[nsub] = qti->savedCursor[k];
            nwpEnd[nsub] = qti->cursor[k];
            nwpFlags[nsub] = qti->bigramFlags[k];
            nsub++;
          }
          /* one sublist of a numeric/facet group: not merged, the list
           * itself (Posdb.cpp:6638-6647) */
          if (nsub == 1 && (nwpFlags[0] & (BF_FACET | BF_NUMBER)) && !(nwpFlags[0] & BF_SYNONYM) &&
              !(nwpFlags[0] & BF_HALFSTOPWIKIBIGRAM)) {
            mml[j] = nwp[0];
            mme[j] = nwpEnd[0];
            bflags[j] = nwpFlags[0];
            rawg[j] = 1; /* writes nothing to mbuf */
            continue;
          }
          for (;;) {
            int mink = -1;
            for (int k = 0; k < nsub; k++) {
              if (!nwp[k]) continue;
              if (mink == -1) { mink = k; continue; }
              if (U32(nwp[k] + 2) > U32(nwp[mink] + 2)) continue;
              if (U32(nwp[k] + 2) == U32(nwp[mink] + 2) && U16(nwp[k]) >= U16(nwp[mink])) continue;
              mink = k;
            }
            if (mink == -1) { mme[j] = mptr; break; }
            int ks = keySize(nwp[mink]);
            if ((nwpFlags[mink] & BF_BIGRAM) && (nwp[mink][2] & 0x03)) goto skipOver;
            if (isFirstKey) {
              memcpy(mptr, nwp[mink], 12);
              mptr[2] &= 0xfc;
              if (nwpFlags[mink] & (BF_BIGRAM | BF_SYNONYM)) mptr[2] |= 0x02;
              if (nwpFlags[mink] & BF_HALFSTOPWIKIBIGRAM) mptr[2] |= 0x01;
              mptr[0] &= 0xf9;
              mptr[0] |= 0x02;
              lastMptr = mptr;
              mptr += 12;
              isFirstKey = 0;
            } else {
              if (lastMptr[4] == nwp[mink][4] && lastMptr[5] == nwp[mink][5] &&
                  (lastMptr[3] & 0xc0) == (nwp[mink][3] & 0xc0))
                goto skipOver;
              memcpy(mptr, nwp[mink], 6);
              mptr[2] &= 0xfc;
              if (nwpFlags[mink] & (BF_BIGRAM | BF_SYNONYM)) mptr[2] |= 0x02;
              if (nwpFlags[mink] & BF_HALFSTOPWIKIBIGRAM) mptr[2] |= 0x01;
              mptr[0] |= 0x06;
              lastMptr = mptr;
              mptr += 6;
            }
          skipOver:
            nwp[mink] += ks;
            if (nwp[mink] >= nwpEnd[mink]) nwp[mink] = NULL;
            else if (keySize(nwp[mink]) != 6) nwp[mink] = NULL;
            if (mptr < mptrEnd) continue;
            mme[j] = mptr;
            break;
          }
        }
      }

      {
        uint64_t d = U32(docIdPtr + 1);
        d <<= 8;
        d |= docIdPtr[0];
        pt.docId = d >> 2;
      }
      /* A positive group whose mini-merged list came out empty (all of its
       * keys for this docid were BF_BIGRAM keys with syn bits, skipped at
       * Posdb.cpp:6687-6692) still has its first key read by every scorer
       * (their loops test the end after a key).  When a later group wrote
       * records, that key is the later group's first (groups are merged back
       * to back), scored here as there.  When none did, the scorers read the
       * mbuf bytes at that place as earlier docids of this pass left them
       * (the function-local mbuf, Posdb.cpp:6007) -- mbuf here persists over
       * the pass the same way, so they are scored from it; where no earlier
       * docid of the pass wrote those 6 bytes they are the stack's (undefined):
       * the docid is skipped. */
      {
        int trailingEmpty = 0;
        size_t at = 0, end = 0;
        for (int j = 0; j < nqti; j++) {
          if (!mml[j] || rawg[j]) continue; /* an unmerged numeric group writes no records */
          trailingEmpty = (mml[j] == mme[j]);
          at = (size_t)(mml[j] - mbuf);
          end = (size_t)(mme[j] - mbuf);
        }
        if (end > mhwm) mhwm = end;
        if (trailingEmpty) {
          if (at + 6 > mhwm) {
            s_stale_undef++;
            continue;
          }
          s_stale_def++;
        }
      }

      /* non-body pair scores, Posdb.cpp:6847-6926 */
      for (int i = 0; i < nqti; i++) {
        if (bflags[i] & BF_EXCLUDE) continue;
        for (int j = i + 1; j < nqti; j++) {
          if (bflags[j] & BF_EXCLUDE) continue;
          int32_t qdist;
          float wts;
          if (wikiPhraseIds[j] == wikiPhraseIds[i] && wikiPhraseIds[j]) {
            qdist = qpos[j] - qpos[i];
            wts = (float)WIKI_WEIGHT;
          } else {
            qdist = 2;
            wts = 1.0;
          }
          float pss = 0.0;
          if (mml[i] && mml[j])
            getTermPairScoreForNonBody(&pt, i, j, mml[i], mml[j], mme[i], mme[j], qdist, &pss);
          if (pss < 0) {
            scoreMatrix[i * nqt + j] = -1.00;
            wts = -1.0;
          } else {
            wts *= pss;
            wts *= freqWeights[i];
            wts *= freqWeights[j];
            scoreMatrix[i * nqt + j] = wts;
          }
        }
      }

      /* single term scores, Posdb.cpp:6933-6978 */
      float minSingleScore = 999999999.0;
      for (int i = 0; i < nqti; i++) {
        if (bflags[i] & BF_EXCLUDE) continue;
        float sts = getSingleTermScore(&pt, i, mml[i], mme[i], &bestPos[i]);
        if (sts < minSingleScore) minSingleScore = sts;
      }

      /* siterank / langid, Posdb.cpp:6985-7003 */
      if (mml[0] && !(qip[0].bigramFlags[0] & (BF_NUMBER | BF_FACET))) {
        siteRank = getSiteRank(mml[0]);
        docLang = getLangId(mml[0]);
      } else {
        for (int k = 1; k < nqti; k++) {
          if (!mml[k]) continue;
          if (qip[k].bigramFlags[0] & (BF_NUMBER | BF_FACET)) continue;
          siteRank = getSiteRank(mml[k]);
          docLang = getLangId(mml[k]);
          break;
        }
      }

      /* sliding window, Posdb.cpp:7013-7150 */
      pt.bestWindowScore = -2.0;
      for (int i = 0; i < nqti; i++) xpos[i] = mml[i];
      {
        int allNull = 1;
        for (int i = 0; i < nqti; i++) {
          if (bflags[i] & BF_EXCLUDE) continue;
          while (xpos[i] && !s_inBody[getHashGroup(xpos[i])]) {
            if (!(xpos[i][0] & 0x04)) xpos[i] += 12;
            else xpos[i] += 6;
            if (xpos[i] < mme[i] && (xpos[i][0] & 0x04)) continue;
            xpos[i] = NULL;
          }
          if (xpos[i]) allNull = 0;
        }
        if (!allNull) {
          int32_t minx, minPos = 0;
          for (;;) {
            evalSlidingWindow(&pt, xpos, nqti, bestPos, scoreMatrix);
          advanceMin:
            minx = -1;
            for (int x = 0; x < nqti; x++) {
              if (bflags[x] & BF_EXCLUDE) continue;
              if (!xpos[x]) continue;
              if (minx == -1) {
                minx = x;
                minPos = getWordPos(xpos[x]);
                continue;
              }
              if (getWordPos(xpos[x]) >= minPos) continue;
              minx = x;
              minPos = getWordPos(xpos[x]);
            }
          advanceAgain:
            if (!(xpos[minx][0] & 0x04)) xpos[minx] += 12;
            else xpos[minx] += 6;
            if (xpos[minx] >= mme[minx] || !(xpos[minx][0] & 0x04)) {
              xpos[minx] = NULL;
              int k;
              for (k = 0; k < nqti; k++) {
                if (bflags[k] & BF_EXCLUDE) continue;
                if (xpos[k]) break;
              }
              if (k >= nqti) break;
              goto advanceMin;
            }
            if (!s_inBody[getHashGroup(xpos[minx])]) goto advanceAgain;
          }
        }
      }

      /* window-restricted pair scores, Posdb.cpp:7159-7219 */
      float minPairScore = -1.0;
      for (int i = 0; i < nqti; i++) {
        if (bflags[i] & BF_EXCLUDE) continue;
        for (int j = i + 1; j < nqti; j++) {
          if (bflags[j] & BF_EXCLUDE) continue;
          if (!mml[i]) continue;
          if (!mml[j]) continue;
          float score = getTermPairScoreForAny(&pt, i, j, mml[i], mml[j], mme[i], mme[j],
                                               &out->corrupt);
          if (score >= minPairScore && minPairScore >= 0.0) continue;
          minPairScore = score;
        }
      }

      /* final score, Posdb.cpp:7228-7257 */
      if (minPairScore < minScore && minPairScore >= 0.0) minScore = minPairScore;
      if (minSingleScore < minScore) minScore = minSingleScore;
      if (minScore <= 0.0) continue;
    boolJump2:;
      float score = minScore * (((float)siteRank) * siteRankMultiplier + 1.0);
      if (prm->language == 0 || docLang == 0 || prm->language == docLang)
        score *= prm->same_lang_weight;
      out->filtered++;
      int32_t intScore = 0;
      if (sortByF >= 0) { /* Posdb.cpp:7265-7269 */
        if (!mml[sortByF]) continue;
        memcpy(&score, mml[sortByF] + 2, 4);
      }
      if (sortByI >= 0) { /* 7271-7279 */
        if (!mml[sortByI]) continue;
        memcpy(&intScore, mml[sortByI] + 2, 4);
      }
      if (prm->min_serp_docid) { /* m_hasMaxSerpScore, Posdb.cpp:4379-4381, 7327-7347 */
        if (sortByI >= 0) {
          /* (int32_t)m_maxSerpScore as x86-64 compiles it (cvttsd2si): the
             truncation, or INT32_MIN when out of range or NaN (in C that
             cast is undefined, so it is spelled out) */
          const double ms = prm->max_serp_score;
          const int32_t m = (ms > -2147483649.0 && ms < 2147483648.0) ? (int32_t)ms : INT32_MIN;
          if (intScore > m) continue;
          if (intScore == m && (int64_t)pt.docId <= prm->min_serp_docid) continue;
        } else {
          if (score > (float)prm->max_serp_score) continue;
          if (score == prm->max_serp_score && (int64_t)pt.docId <= prm->min_serp_docid) continue;
        }
      }
      out->filtered--;
      /* facet stats of every docid in the search results (Posdb.cpp:7362-7542):
       * each key of its facet list's run, bucketed into a range with ranges,
       * one vote per docid per entry */
      for (int f = 0; hasFacet && f < nf; f++) {
        const int g = fgroup[f];
        if (g < 0 || !mml[g]) continue;
        FTable *t = NULL;
        for (int k = 0; k < s_nft; k++)
          if (s_ft[k].term == fterm[f]) t = &s_ft[k];
        const orc_facet_ranges *fr = facet_ranges_of(prm, fterm[f]);
        const int isFloat = qt[fterm[f]].field_code == F_FACETFLOAT;
        uint8_t *p2 = mml[g];
        int firstTime = 1;
        for (;;) {
          if (p2 >= mme[g]) break;
          if (!firstTime && !(p2[0] & 0x04)) break;
          int32_t val32;
          memcpy(&val32, p2 + 2, 4);
          p2 += firstTime ? 12 : 6;
          firstTime = 0;
          float fv;
          memcpy(&fv, &val32, 4);
          FEnt *fe = NULL;
          if (fr && fr->n > 0) {
            for (int k = 0; k < fr->n; k++) {
              if (isFloat) {
                float A, B;
                memcpy(&A, &fr->a[k], 4);
                memcpy(&B, &fr->b[k], 4);
                if (fv < A) continue;
                if (fv >= B) continue;
              } else {
                if (val32 < fr->a[k]) continue;
                if (val32 >= fr->b[k]) continue;
              }
              fe = ft_get(t, fr->a[k]);
              break;
            }
          } else {
            fe = ft_get(t, val32);
            if (!fe) fe = ft_add(t, val32);
          }
          if (!fe) continue;
          if (fe->docid == (int64_t)pt.docId) continue;
          fe->docid = (int64_t)pt.docId;
          fe->count++;
          if (fe->count == 1) {
            if (isFloat) {
              const double z = 0.0;
              memcpy(&fe->sum, &z, 8);
              memcpy(&fe->min, &fv, 4);
              memcpy(&fe->max, &fv, 4);
            } else {
              fe->sum = 0;
              fe->min = val32;
              fe->max = val32;
            }
          }
          if (isFloat) {
            double sum;
            memcpy(&sum, &fe->sum, 8);
            sum += fv;
            memcpy(&fe->sum, &sum, 8);
            float mn, mx;
            memcpy(&mn, &fe->min, 4);
            memcpy(&mx, &fe->max, 4);
            if (fv < mn) memcpy(&fe->min, &fv, 4);
            if (fv > mx) memcpy(&fe->max, &fv, 4);
          } else {
            fe->sum += val32;
            if (val32 < fe->min) fe->min = val32;
            if (val32 > fe->max) fe->max = val32;
          }
        }
      }
      /* with m_useIntScores the tree orders by m_intScore (TopTree.cpp:216-219, 270-274) */
      tt_add(tree, sortByI >= 0 ? (double)intScore : (double)score, (int64_t)pt.docId);
      if (tree->n > tree->docsWanted) minWinningScore = tree->score[tree->n - 1]; /* 7699-7704 */
    }
    /* countUniqueDocids (Posdb.cpp:5002-5038, called at 7786-7796): the
     * facet group's first sublist walked record by record over its whole
     * buffer -- the shrunk runs, then the list's own bytes past them -- every
     * record's value counted in an existing entry, the records longer than 6
     * bytes into m_numDocsThatHaveFacet */
    for (int f = 0; hasFacet && f < nf; f++) {
      const int g = fgroup[f];
      if (g < 0) continue;
      FTable *t = NULL;
      for (int k = 0; k < s_nft; k++)
        if (s_ft[k].term == fterm[f]) t = &s_ft[k];
      const OList *L = &P.lists[qip[g].subList[0]];
      const uint8_t *rp = L->list, *end = L->list + L->size;
      uint64_t count = 0;
      while (rp < end) {
        int32_t val32;
        memcpy(&val32, rp + 2, 4);
        FEnt *fe = ft_get(t, val32);
        if (fe) fe->outside++;
        const int rs = keySize(rp);
        rp += rs;
        if (rs > 6) count++;
      }
      t->docs += count;
    }
  doneAll:
    free(wikiPhraseIds); free(quotedStartIds); free(qpos); free(freqWeights);
    free(mml); free(mme); free(bestPos); free(winnerStack); free(xpos); free(bflags); free(rawg);
    free(scoreMatrix); free(mbuf);
  }

finish:
  unprepare(&P, nqt);
  return 0;
}

/* RdbList::constrain (RdbList.cpp:1328-1560) of a posdb list to the keys with
 * docid in [d0, d1]: the first kept key is written out whole (18 bytes), the
 * rest keep their compressed form.  Returns the restricted size. */
static int64_t constrain_docids(const uint8_t *l, int64_t n, uint64_t d0, uint64_t d1, uint8_t *out) {
  uint8_t hi[6] = {0}, lo[6] = {0};
  int64_t o = 0;
  for (int64_t p = 0; p < n;) {
    const int ks = keySize(l + p);
    if (ks == 18) memcpy(hi, l + p + 12, 6);
    if (ks >= 12) memcpy(lo, l + p + 6, 6);
    uint8_t k[18];
    memcpy(k, l + p, 6);
    memcpy(k + 6, lo, 6);
    memcpy(k + 12, hi, 6);
    const uint64_t d = getDocId(k);
    if (d > d1) break;
    if (d >= d0) {
      if (o == 0) {
        memcpy(out, k, 18);
        out[0] &= 0xf9;
        o = 18;
      } else {
        memcpy(out + o, l + p, ks);
        o += ks;
      }
    }
    p += ks;
  }
  return o;
}

#define ORC_MAX_DOCID 0x3fffffffffULL /* MAX_DOCID = DOCID_MASK, Titledb.h:10-11 */

/* Msg39::controlLoop (Msg39.cpp:345-457) + getLists' range (573-615): the
 * docid range is cut into m_numDocIdSplits pieces; each piece's lists are
 * read constrained to it and intersected into ONE TopTree, allocated once at
 * the first piece with allocTopTree's split sizing (Posdb.cpp:859-877) and
 * never reset; hit counts and m_filtered add up over the pieces.  A piece
 * reads docids [d0, d1+2] (getLists adds 1 twice), so neighbours overlap. */
int orc_query(const orc_qterm *qt, const uint8_t *const *lists, const int64_t *sizes, int nqt,
              const orc_params *prm, int64_t *docids, float *scores, int cap, orc_result *out) {
  memset(out, 0, sizeof *out);
  ft_reset();
  s_stale_def = s_stale_undef = 0;
  if (nqt < 0 || !prm) return EINVAL;
  if (prm->real_max_top <= 0 || prm->docs_to_get <= 0 || prm->num_docid_splits <= 0) return EINVAL;
  int intMode = 0;
  for (int i = 0; i < nqt; i++) {
    const int fc = qt[i].field_code;
    if ((fc == F_SORTBYINT || fc == F_REVSORTBYINT) && qt[i].is_required) intMode = 1;
    /* facets in a boolean query: restated for a facet term without synonyms
     * (its group one sublist, the run itself) */
    if ((fc == F_FACETSTR || fc == F_FACETINT || fc == F_FACETFLOAT) && prm->is_boolean)
      for (int k = 0; k < nqt; k++)
        if (qt[k].synonym_of == i) return ENOTSUP;
    /* a boolean query's gbsortby score reads a mini-merged list that may be
       the next group's or stale bytes (Posdb.cpp:7263-7279): not restated */
    if (prm->is_boolean && (fc == F_SORTBYFLOAT || fc == F_REVSORTBYFLOAT || fc == F_SORTBYINT ||
                            fc == F_REVSORTBYINT))
      return ENOTSUP;
  }
  initWeights();

  const int splits = prm->num_docid_splits;
  WhiteSet ws = {NULL, 0};
  if (prm->use_whitelist && white_build(prm, &ws)) return ENOMEM;
  TTree tk;
  memset(&tk, 0, sizeof tk);
  int alloced = 0, rc = 0;
  const uint8_t **pl = (const uint8_t **)calloc(nqt > 0 ? nqt : 1, sizeof(uint8_t *));
  int64_t *ps = (int64_t *)calloc(nqt > 0 ? nqt : 1, sizeof(int64_t));
  uint8_t **own = (uint8_t **)calloc(nqt > 0 ? nqt : 1, sizeof(uint8_t *));
  const uint64_t delta = ORC_MAX_DOCID / (uint64_t)splits;
  uint64_t ddd = 0;
  do {
    const uint64_t d0 = ddd;
    ddd += delta;
    uint64_t d1 = ddd;
    if (d1 + 20 > ORC_MAX_DOCID) {
      d1 = ORC_MAX_DOCID;
      ddd = ORC_MAX_DOCID;
    }
    uint64_t dend = d1 + 2;
    if (dend > ORC_MAX_DOCID) dend = ORC_MAX_DOCID;
    for (int i = 0; i < nqt; i++) {
      if (splits == 1) {
        pl[i] = lists[i];
        ps[i] = sizes[i];
        continue;
      }
      free(own[i]);
      own[i] = (uint8_t *)malloc(sizes[i] + 24);
      ps[i] = constrain_docids(lists[i], sizes[i], d0, dend, own[i]);
      pl[i] = own[i];
    }
    if (!alloced) {
      /* Msg39::intersectLists: no tree while it would have no nodes (938-947) */
      int64_t dw = docs_wanted(prm, ps, nqt);
      if (dw == 0) continue;
      alloced = 1;
      out->docs_wanted = (int32_t)dw;
      tt_init(&tk, (int32_t)dw, prm->site_clustering != 0);
      tk.ints = intMode;
    }
    orc_result r;
    memset(&r, 0, sizeof r);
    rc = run_range(qt, pl, ps, nqt, prm, prm->use_whitelist ? &ws : NULL, &tk, &r);
    if (rc) break;
    out->hits += r.hits;
    out->filtered += r.filtered;
    if (r.corrupt) out->corrupt = r.corrupt;
  } while (ddd < ORC_MAX_DOCID);
  for (int i = 0; i < nqt; i++) free(own[i]);
  free(own); free(pl); free(ps);
  free(ws.v);
  out->n = tk.n < cap ? (int32_t)tk.n : cap;
  for (int i = 0; i < out->n; i++) {
    docids[i] = tk.docid[i];
    scores[i] = intMode ? 0.0f : (float)tk.score[i]; /* TopNode::m_score is 0 with int scores */
  }
  tt_free(&tk);
  return rc;
}

/* posdbMerge_r restatement lives in posdb_merge_oracle.c */
