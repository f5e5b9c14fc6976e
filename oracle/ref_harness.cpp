// TEST INFRASTRUCTURE ONLY -- drives the REFERENCE's own PosdbTable,
// TopTree and RdbList::merge_r, compiled unmodified from /root/reference by
// oracle/ref.mk into oracle/_ref/gbref.  Tests use it to pin the
// restatement (posdb_oracle.c) and to generate tests/golden/ fixtures; the
// product never loads it, and it is built only where /root/reference exists.
//
// The harness plays the part of main.cpp + Msg39 for one query: it fills a
// Query/QueryTerm/QueryWord array the way Query::set2 leaves it (the fields
// PosdbTable reads, Posdb.cpp:4354-4869), wraps the caller's lists in a Msg2,
// and runs the same sequence as Msg39::intersectLists (Msg39.cpp:884-1053):
//   PosdbTable::init -> allocTopTree -> allocWhiteListTable ->
//   setQueryTermInfo -> intersectLists10_r
// then reads TopTree high -> low (Msg39.cpp:1346-1420 readout order).
//
// Lists are copied before every run because intersectLists10_r mutates them
// (first-key swap Posdb.cpp:5671-5703, shrinkSubLists Posdb.cpp:5334-5428).
#include "gb-include.h"

#include "Collectiondb.h"
#include "Mem.h"
#include "Msg2.h"
#include "Msg39.h"
#include "Posdb.h"
#include "Query.h"
#include "RdbList.h"
#include "TopTree.h"

#include <stdint.h>
#include <string.h>

#include <vector>

#include "posdb_oracle.h"  // orc_qterm / orc_params / orc_result

// Symbols main.cpp defines for the gb binary (main.cpp:155,197,199); the
// harness is this program's main module.
int g_inMemcpy = 0;
bool g_recoveryMode = false;
int32_t g_recoveryLevel = 0;

extern bool hashinit();

// A fault inside the reference (or a call into a unit ref.mk did not link)
// prints a backtrace instead of dying silently.  Installed before any static
// initialiser of the reference units runs.
#include <execinfo.h>
#include <signal.h>
#include <unistd.h>
#include <stdio.h>
#include <ucontext.h>
static void on_fault(int sig, siginfo_t *si, void *uc) {
  void *bt[64];
  int n = backtrace(bt, 64);
  const ucontext_t *u = (const ucontext_t *)uc;
  const unsigned long pc = u->uc_mcontext.gregs[REG_RIP];
  const unsigned long sp = u->uc_mcontext.gregs[REG_RSP];
  char msg[160];
  // pc 0 = a call into a unit ref.mk does not link: [sp] is its caller
  int m = snprintf(msg, sizeof msg, "gbref: fatal signal %d at pc=%#lx addr=%p caller=%#lx; backtrace:\n", sig,
                   pc, si->si_addr, pc == 0 ? *(const unsigned long *)sp : 0ul);
  write(2, msg, m);
  backtrace_symbols_fd(bt, n, 2);
  _exit(128 + sig);
}
__attribute__((constructor(101))) static void install_fault_handler() {
  struct sigaction sa;
  memset(&sa, 0, sizeof sa);
  sa.sa_sigaction = on_fault;
  sa.sa_flags = SA_SIGINFO;
  sigaction(SIGSEGV, &sa, NULL);
  sigaction(SIGBUS, &sa, NULL);
  sigaction(SIGFPE, &sa, NULL);
}

static bool s_inited = false;
// INTEGRATION.md's adapter (gbgpuIntersectLists), linked only into the GPU
// build of this harness (oracle/ref.mk: gbref_gpu); op 4 runs it in place of
// intersectLists10_r, in the same Msg39 sequence, and falls back to the
// unmodified CPU body where it declines -- as the adapter's caller does
extern bool gbref_adapter_intersect(PosdbTable *pt) __attribute__((weak));
// the docid-split loop replaced at the Msg39 level
// (gbgpuDocIdSplits) with the whole-range lists resident; op 4 mode 2
extern bool gbref_adapter_splits(Msg39 *m, const uint8_t *const *lists, const int64_t *sizes)
    __attribute__((weak));
// gbgpuShardQuery as shard 0 of a one-rank exchange; op 7
extern int gbref_adapter_shard(PosdbTable *pt, const uint8_t *const *lists, const int64_t *sizes, int32_t k,
                               int64_t *docids, double *scores, int32_t *n, int64_t *hits) __attribute__((weak));
// gbgpuMergePosdb in place of merge_r's posdbMerge_r call; op 6
extern bool gbref_adapter_merge(RdbList *self, RdbList **lists, int32_t numLists, char *startKey, char *endKey,
                                int32_t minRecSizes, bool removeNegRecs) __attribute__((weak));
static int s_adapter = 0;   // op 4 mode: 1 = the adapter body, 2 = and the Msg39 split adapter
static int s_answered = 0;  // passes the adapter answered
// the second pass's score info (Posdb.cpp:6116-6244, 7554-7665): the last
// query's m_scoreInfoBuf / m_pairScoreBuf / m_singleScoreBuf bytes
static std::vector<char> s_info[3];
static double s_isect_s = 0;  // seconds inside intersectLists10_r (list copies excluded)
static double s_merge_s = 0;  // seconds inside RdbList::merge_r
static double now_s();
static CollectionRec *s_crPtr[1];

static void ref_init() {
  if (s_inited) return;
  // gb.conf "maxmem" (Conf.h m_maxMem, read by Mem's operator new): no
  // gb.conf is loaded here, so give the allocator the whole box
  g_conf.m_maxMem = (int64_t)1 << 40;
  g_mem.init();
  hashinit();
  // one collection, collnum 0 (PosdbTable::init requires getRec(collnum))
  static CollectionRec *cr = new CollectionRec();
  s_crPtr[0] = cr;
  g_collectiondb.m_recs = s_crPtr;
  g_collectiondb.m_numRecs = 1;
  s_inited = true;
}

enum { MAXT = 64 };

static PosdbTable *s_tab = NULL;       // the last query's PosdbTable
// a boolean query's expression (Query::m_qwords as Query::set2 leaves them
// for Expression::addExpression, Query.cpp:5424-5514): tokens >= 0 are
// operand words naming query term t (QueryWord::m_queryWordTerm), negative
// ones the opcodes OP_OR -1, OP_AND -2, OP_NOT -3, OP_LEFTPAREN -4,
// OP_RIGHTPAREN -5; none = not boolean
static std::vector<int32_t> s_btok;
// the last query's truth table over its QueryTermInfo bit vectors:
// Query::matchesBoolQuery for every vector (bit v at byte v >> 3, bit v & 7)
static std::vector<uint8_t> s_btable;
static int32_t s_bgroups = -1;
// gbfacetint:/gbfacetfloat: ranges (QueryWord::m_numFacetRanges and
// m_facetRange{Int,Float}{A,B}, Query.h:389-393) per query term, and the
// facet tables the last query left (QueryTerm::m_facetHashTable, its
// m_numDocsThatHaveFacet; Posdb.cpp:1000-1067, 5575-5631, 7362-7542, 7786-7796)
struct FacetRanges {
  int32_t term, n;
  std::vector<int32_t> a, b;
};
static std::vector<FacetRanges> s_franges;
static std::vector<char> s_facets;  // i32 nterms; per facet term: i32 term, u64 docs, i32 n, n x (i32 key, FacetEntry)
static std::vector<int32_t> s_plan;    // the last query's QueryTermInfos (op 4)
static int32_t s_used_nodes = 0;       // the last query's TopTree::m_numUsedNodes
static std::vector<int32_t> s_ints;    // its nodes' m_intScore, high -> low
static int ref_query(const orc_qterm *terms, const uint8_t *const *lists, const int64_t *sizes, int nterms,
                         const orc_params *p, int64_t *docids, float *scores, int cap, orc_result *out,
                         int64_t *vote_docids, int64_t vote_cap) {
  ref_init();
  if (nterms < 0 || nterms > MAXT) return EINVAL;
  static Query q;
  static QueryTerm qts[MAXT];
  static QueryWord qws[MAXT];
  static RdbList rl[MAXT];
  static Msg2 msg2;
  static Msg39Request req;
  static TopTree s_tree;
  static float tfw[MAXT];
  // mode 2 plays Msg39 itself: its m_tt is the tree, its m_posdbTable the
  // table (Msg39.h:252,278), which gbgpuDocIdSplits fills
  static Msg39 *s_m39 = NULL;
  const bool msg39 = s_adapter == 2 && p->num_docid_splits > 1;
  if (msg39 && !s_m39) s_m39 = new Msg39();
  TopTree &tree = msg39 ? s_m39->m_tt : s_tree;
  PosdbTable *&tab = s_tab;

  memset((void *)qts, 0, sizeof(qts));
  memset((void *)qws, 0, sizeof(qws));
  // QueryTerm's facet table as Query constructs it (HashTableX::HashTableX:
  // writable, no buffer) -- a zeroed one refuses every addKey
  for (int i = 0; i < MAXT; i++) new (&qts[i].m_facetHashTable) HashTableX();
  for (int i = 0; i < nterms; i++) {
    const orc_qterm &t = terms[i];
    QueryTerm *qt = &qts[i];
    QueryWord *qw = &qws[i];
    qw->m_posNum = t.qpos;
    qw->m_wikiPhraseId = t.wiki_phrase_id;
    qw->m_quoteStart = t.quote_start;
    qw->m_float = t.number_float;  // gbmin:/gbmax:/gbequal: bounds (Posdb.cpp:4948-4979)
    qw->m_int = t.number_int;
    qt->m_qword = qw;
    qt->m_isRequired = t.is_required != 0;
    qt->m_termSign = (char)t.term_sign;
    qt->m_fieldCode = (char)t.field_code;
    qt->m_piped = t.piped != 0;
    qt->m_synonymOf = t.synonym_of >= 0 ? &qts[t.synonym_of] : NULL;
    qt->m_leftPhraseTermNum = t.left_phrase_term;
    qt->m_rightPhraseTermNum = t.right_phrase_term;
    qt->m_leftPhraseTerm = t.left_phrase_term >= 0 ? &qts[t.left_phrase_term] : NULL;
    qt->m_rightPhraseTerm = t.right_phrase_term >= 0 ? &qts[t.right_phrase_term] : NULL;
    qt->m_isWikiHalfStopBigram = t.is_wiki_half_stop_bigram != 0;
    tfw[i] = t.tf_weight;
  }
  q.m_qterms = qts;
  q.m_numTerms = nterms;
  q.m_isBoolean = !s_btok.empty();
  static QueryWord bws[256];
  static char s_alpha[] = "x", s_op[] = "(";
  if (q.m_isBoolean) {
    const int nw = (int)s_btok.size();
    if (nw > 256) return EINVAL;
    memset((void *)bws, 0, sizeof(bws));
    for (int i = 0; i < nw; i++) {
      const int32_t t = s_btok[i];
      QueryWord *w = &bws[i];
      if (t >= 0) {
        if (t >= nterms) return EINVAL;
        w->m_word = s_alpha;  // isAlphaWord() (Query.h:269)
        w->m_wordLen = 1;
        w->m_queryWordTerm = &qts[t];
      } else {
        w->m_word = s_op;
        w->m_wordLen = 1;
        w->m_opcode = (char)(t == -1 ? OP_OR : t == -2 ? OP_AND : t == -3 ? OP_NOT : t == -4 ? OP_LEFTPAREN
                                                                                           : OP_RIGHTPAREN);
      }
    }
    q.m_qwords = bws;
    q.m_numWords = nw;
    q.m_numExpressions = 1;
    if (!q.m_expressions[0].addExpression(0, nw, &q, 0)) return EINVAL;
  }
  for (size_t i = 0; i < s_franges.size(); i++) {
    const FacetRanges &fr = s_franges[i];
    if (fr.term < 0 || fr.term >= nterms || fr.n < 0 || fr.n > MAX_FACET_RANGES) return EINVAL;
    QueryWord *qw = &qws[fr.term];
    qw->m_numFacetRanges = fr.n;
    for (int k = 0; k < fr.n; k++) {
      qw->m_facetRangeIntA[k] = fr.a[k];
      qw->m_facetRangeIntB[k] = fr.b[k];
      memcpy(&qw->m_facetRangeFloatA[k], &fr.a[k], 4);
      memcpy(&qw->m_facetRangeFloatB[k], &fr.b[k], 4);
    }
  }
  for (int i = 0; i < nterms; i++) qws[i].m_fieldCode = qts[i].m_fieldCode;  // QueryWord's copy (Posdb.cpp:7439-7441)

  msg2.m_query = &q;
  msg2.m_lists = rl;
  msg2.m_numLists = nterms;  // Msg2::getLists sets it (Msg2.cpp:121-347)
  msg2.m_w = 0;

  req.reset();
  req.m_docsToGet = p->docs_to_get;
  req.m_realMaxTop = p->real_max_top;
  req.m_language = (uint8_t)p->language;
  req.m_sameLangWeight = p->same_lang_weight;
  req.m_doSiteClustering = p->site_clustering != 0;
  req.m_numDocIdSplits = p->num_docid_splits;
  req.m_doMaxScoreAlgo = p->do_max_score_algo != 0;
  req.m_maxSerpScore = p->max_serp_score;
  req.m_minSerpDocId = p->min_serp_docid;
  req.m_getDocIdScoringInfo = p->get_docid_scoring_info != 0;
  req.m_collnum = 0;
  req.ptr_termFreqWeights = (char *)tfw;
  req.size_termFreqWeights = 4 * nterms;
  // the "&sites=" whitelist: allocWhiteListTable only tests size_whiteList > 1
  // (Posdb.cpp:800-801); the lists are Msg2::m_whiteLists[0..m_w)
  static char s_sites[] = "x";
  req.ptr_whiteList = p->use_whitelist ? s_sites : NULL;
  req.size_whiteList = p->use_whitelist ? 2 : 0;
  const int nw = p->use_whitelist ? p->n_white_lists : 0;
  if (nw < 0 || nw > MAX_WHITELISTS) return EINVAL;

  tree.~TopTree();
  memset((void *)&tree, 0, sizeof tree);  // m_docsWanted is only set by setNumNodes
  new (&tree) TopTree();
  out->hits = 0;
  out->filtered = 0;
  out->corrupt = 0;

  // Msg39::controlLoop's docid-split loop (Msg39.cpp:345-457): one TopTree
  // (reset once, Msg39.cpp:263) filled by one PosdbTable pass per docid range;
  // each pass gets its lists as Msg2 reads them for getLists' range
  // (Msg39.cpp:573-647: [d0, d1+2] with one stripe), here by the reference's
  // own RdbList::constrain on a fresh copy of the whole list.
  bool alloced = false;
  int64_t ddd = 0;
  const int64_t dddEnd = MAX_DOCID;
  const int32_t splits = p->num_docid_splits;
  do {
    const int64_t d0 = ddd;
    const int64_t delta = MAX_DOCID / (int64_t)splits;
    ddd += delta;
    int64_t d1 = ddd;
    if (d1 + 20LL > MAX_DOCID) {
      d1 = MAX_DOCID;
      ddd = MAX_DOCID;
    }
    // Msg39::controlLoop hands each piece its range (Msg39.cpp:376-377): the
    // second pass rescores only the tree's docids inside it (Posdb.cpp:6189)
    req.m_minDocId = d0;
    req.m_maxDocId = d1;
    int64_t docIdEnd = d1 + 1 + 1;
    if (docIdEnd > MAX_DOCID) docIdEnd = MAX_DOCID;
    for (int i = 0; i < nterms; i++) {
      rl[i].freeList();
      // RdbList::set(list, size, alloc, allocSize, fixedDataSize, ownData,
      // useHalfKeys, keySize=18): a fresh mutable copy per pass
      char *buf = NULL;
      int32_t sz = (int32_t)sizes[i];
      if (sz > 0) {
        buf = (char *)mmalloc(sz + 64, "refharness");
        memcpy(buf, lists[i], sz);
      }
      rl[i].set(buf, sz, buf, sz ? sz + 64 : 0, 0, true, true, 18);
      if (splits > 1 && sz > 0) {
        char first[18], sk[18], ek[18];
        memcpy(first, lists[i], 18);
        const int64_t tid = g_posdb.getTermId(first);
        g_posdb.makeStartKey(sk, tid, d0);
        g_posdb.makeEndKey(ek, tid, docIdEnd);
        if (!rl[i].constrain(sk, ek, -1, 0, first, (char *)"refharness", 0)) return EIO;
      }
    }
    // whitelist lists as Msg2 reads them for each piece: fresh (their cursor
    // is walked by the table fill, Posdb.cpp:5550-5571)
    for (int i = 0; i < MAX_WHITELISTS && i < (nw > msg2.m_w ? nw : msg2.m_w); i++) msg2.m_whiteLists[i].freeList();
    for (int i = 0; i < nw; i++) {
      char *buf = NULL;
      const int32_t sz = (int32_t)p->white_lists[i].size;
      if (sz > 0) {
        buf = (char *)mmalloc(sz + 64, "refharness");
        memcpy(buf, p->white_lists[i].bytes, sz);
        memset(buf + sz, 0, 64);
      }
      msg2.m_whiteLists[i].set(buf, sz, buf, sz ? sz + 64 : 0, 0, true, true, 18);
    }
    msg2.m_w = nw;
    // one PosdbTable over all pieces: reset per piece (Msg39::reset2,
    // Msg39.cpp:51-69), its allocTopTree buffers (m_stackBuf) kept
    if (d0 == 0) {
      if (tab && tab != (s_m39 ? &s_m39->m_posdbTable : NULL)) {
        tab->~PosdbTable();
        mfree(tab, sizeof(PosdbTable), "refharness");
      }
      if (msg39) {
        tab = &s_m39->m_posdbTable;
        tab->~PosdbTable();
        new (tab) PosdbTable();
        s_m39->m_r = &req;
        s_m39->m_numTotalHits = 0;
      } else {
        tab = (PosdbTable *)mmalloc(sizeof(PosdbTable), "refharness");
        new (tab) PosdbTable();
      }
    }
    tab->reset();
    // Msg39::intersectLists sequence (Msg39.cpp:922-1027)
    tab->init(&q, 0, NULL, &tree, 0, &msg2, &req);
    if (!alloced && !tab->allocTopTree()) return ENOMEM;
    if (tree.m_numNodes == 0) continue;  // all lists empty: no pass (Msg39.cpp:945-948)
    alloced = true;
    if (!tab->allocWhiteListTable()) return ENOMEM;
    if (!tab->setQueryTermInfo()) return ENOMEM;
    if (getenv("GBREF_TRACE"))
      for (int i = 0; i < nterms; i++)
        fprintf(stderr, "gbref: term %d fc %d slots %d used %d qti %d hasFacet %d\n", i, (int)qts[i].m_fieldCode,
                (int)qts[i].m_facetHashTable.m_numSlots, (int)qts[i].m_facetHashTable.m_numSlotsUsed,
                qts[i].m_queryTermInfoNum, (int)tab->m_hasFacetTerm);
    const double t0 = now_s();
    if (msg39 && d0 == 0 && gbref_adapter_splits && gbref_adapter_splits(s_m39, lists, sizes)) {
      // every piece answered at once (Msg39's loop skipped to phase 3):
      // m_numTotalHits is the hits less m_filtered (Msg39.cpp:409-414)
      s_isect_s += now_s() - t0;
      s_answered++;
      out->hits = s_m39->m_numTotalHits;
      out->filtered = 0;
      break;
    }
    if (s_adapter && gbref_adapter_intersect && gbref_adapter_intersect(tab)) s_answered++;
    else tab->intersectLists10_r();
    s_isect_s += now_s() - t0;
    out->hits += tab->m_docIdVoteBuf.length() / 6;
    out->filtered += tab->m_filtered;
    if (tab->m_errno) out->corrupt = tab->m_errno;
  } while (ddd < dddEnd);
  // the facet tables (Msg39.cpp:1453-1545 serializes the same)
  s_facets.clear();
  {
    int32_t nf = 0;
    std::vector<char> body;
    for (int i = 0; i < nterms; i++) {
      QueryTerm *qt = &qts[i];
      if (qt->m_fieldCode != FIELD_GBFACETSTR && qt->m_fieldCode != FIELD_GBFACETINT &&
          qt->m_fieldCode != FIELD_GBFACETFLOAT)
        continue;
      HashTableX *ft = &qt->m_facetHashTable;
      int32_t used = ft->m_numSlots ? ft->m_numSlotsUsed : 0;
      const uint64_t docs = qt->m_numDocsThatHaveFacet;
      const size_t at = body.size();
      body.resize(at + 16 + (size_t)used * (4 + sizeof(FacetEntry)));
      char *p = &body[at];
      memcpy(p, &i, 4);
      memcpy(p + 4, &docs, 8);
      int32_t k2 = 0;
      char *e = p + 16;
      for (int32_t k = 0; k < ft->m_numSlots; k++) {
        if (!ft->m_flags[k]) continue;
        const int32_t key = ft->getKey32FromSlot(k);
        memcpy(e, &key, 4);
        memcpy(e + 4, ft->getValFromSlot(k), sizeof(FacetEntry));
        e += 4 + sizeof(FacetEntry);
        k2++;
      }
      memcpy(p + 12, &k2, 4);
      nf++;
    }
    s_facets.resize(4);
    memcpy(&s_facets[0], &nf, 4);
    s_facets.insert(s_facets.end(), body.begin(), body.end());
  }
  // a boolean query's truth table, by the reference's own evaluator over
  // every bit vector of its QueryTermInfos (m_bitNum, Posdb.cpp:4485-4721)
  s_btable.clear();
  s_bgroups = -1;
  if (q.m_isBoolean && tab) {
    const int32_t ng = tab->m_numQueryTermInfos;
    if (ng >= 0 && ng <= 16) {
      s_bgroups = ng;
      const int32_t nv = 1 << ng;
      s_btable.assign((nv + 7) / 8, 0);
      const int32_t vs = ng / 8 + (ng % 8 ? 1 : 0);
      for (int32_t v = 0; v < nv; v++) {
        unsigned char vec[4] = {(unsigned char)v, (unsigned char)(v >> 8), 0, 0};
        if (q.matchesBoolQuery(vec, vs > 0 ? vs : 1)) s_btable[v >> 3] |= (uint8_t)(1u << (v & 7));
      }
    }
  }
  // allocTopTree returns before setNumNodes when every list is empty
  // (Posdb.cpp:889-890): no tree, reported as 0 like the oracle
  out->docs_wanted = tree.m_numNodes > 0 ? tree.m_docsWanted : 0;
  // setQueryTermInfo's groups (Posdb.cpp:4354-4869): per QueryTermInfo its
  // m_bigramFlags[0], m_numSubLists and each sublist's term index and flags
  s_plan.clear();
  if (tab) {
    const QueryTermInfo *qip = (const QueryTermInfo *)tab->m_qiBuf.getBufStart();
    const int32_t ng = qip ? tab->m_numQueryTermInfos : 0;
    s_plan.push_back(ng);
    for (int32_t g = 0; g < ng; g++) {
      s_plan.push_back((unsigned char)qip[g].m_bigramFlags[0]);
      s_plan.push_back(qip[g].m_numSubLists);
      for (int32_t j = 0; j < qip[g].m_numSubLists; j++) {
        s_plan.push_back((int32_t)(qip[g].m_subLists[j] - rl));
        s_plan.push_back((unsigned char)qip[g].m_bigramFlags[j]);
      }
    }
  } else {
    s_plan.push_back(0);
  }
  int n = 0;
  s_ints.clear();
  s_used_nodes = tree.m_numNodes > 0 ? tree.m_numUsedNodes : 0;
  if (tree.m_numNodes > 0) {
    for (int32_t ti = tree.getHighNode(); ti >= 0 && n < cap; ti = tree.getPrev(ti)) {
      TopNode *t = tree.getNode(ti);
      docids[n] = t->m_docId;
      scores[n] = t->m_score;
      s_ints.push_back(t->m_intScore);
      n++;
    }
  }
  out->n = n;
  for (int b = 0; b < 3; b++) s_info[b].clear();
  if (p->get_docid_scoring_info && tab) {
    SafeBuf *sb[3] = {&tab->m_scoreInfoBuf, &tab->m_pairScoreBuf, &tab->m_singleScoreBuf};
    for (int b = 0; b < 3; b++) s_info[b].assign(sb[b]->getBufStart(), sb[b]->getBufStart() + sb[b]->length());
  }
  if (vote_docids) {
    // m_docIdVoteBuf records: [b7&0xfc, b8..b11, vote] (Posdb.cpp:5281-5290)
    const uint8_t *v = (const uint8_t *)tab->m_docIdVoteBuf.getBufStart();
    int64_t nv = tab->m_docIdVoteBuf.length() / 6;
    for (int64_t i = 0; i < nv && i < vote_cap; i++) {
      const uint8_t *r = v + 6 * i;
      uint64_t d = (uint64_t)r[0] | ((uint64_t)r[1] << 8) | ((uint64_t)r[2] << 16) |
                   ((uint64_t)r[3] << 24) | ((uint64_t)r[4] << 32);
      vote_docids[i] = (int64_t)(d >> 2);
    }
  }
  return 0;
}

// RdbList::merge_r -> posdbMerge_r (RdbList.cpp:1658,1745-1756,3065) on
// copies of n posdb lists (oldest first), as Msg5::mergeLists_r calls it.
static int64_t ref_posdb_merge(const uint8_t *const *lists, const int64_t *sizes, int n, int remove_neg_keys,
                                   int64_t min_rec_sizes, uint8_t *out, int64_t cap) {
  ref_init();
  if (n < 0 || n > 256) return -EINVAL;
  static RdbList in[256];
  RdbList *ptrs[256];
  for (int i = 0; i < n; i++) {
    in[i].freeList();
    int32_t sz = (int32_t)sizes[i];
    char *buf = NULL;
    if (sz > 0) {
      buf = (char *)mmalloc(sz, "refharness");
      memcpy(buf, lists[i], sz);
    }
    in[i].set(buf, sz, buf, sz, 0, true, true, 18);
    ptrs[i] = &in[i];
  }
  RdbList dst;
  dst.set(NULL, 0, NULL, 0, 0, true, true, 18);
  char startKey[18], endKey[18];
  memset(startKey, 0, 18);
  memset(endKey, 0xff, 18);
  int32_t mrs = min_rec_sizes < 0 ? -1 : (int32_t)min_rec_sizes;
  if (!dst.prepareForMerge(ptrs, n, mrs)) return -ENOMEM;
  int32_t filtered = 0;
  const double t0 = now_s();
  dst.merge_r(ptrs, n, startKey, endKey, mrs, remove_neg_keys != 0, RDB_POSDB, &filtered, NULL, NULL, false, 0);
  s_merge_s = now_s() - t0;
  int64_t sz = dst.m_listSize;
  if (sz > cap) return -ENOSPC;
  memcpy(out, dst.m_list, sz);
  dst.freeList();
  return sz;
}

// op 6: RdbList::merge_r for posdb as Msg5::mergeLists_r / RdbMerge call it
// (prepareForMerge, then merge_r with a start and end key), either unchanged
// (mode 0) or with INTEGRATION.md 5's gbgpuMergePosdb where merge_r calls
// posdbMerge_r (mode 1).  The reference is not edited, so mode 1 runs
// merge_r's own steps before that call here (RdbList.cpp:1658-1741 for
// RDB_POSDB: the early returns, the key range with its dangling-negative
// fix, the key size) and then the adapter, falling back to posdbMerge_r
// where it declines -- the body merge_r would have with the adapter in it.
// Returns the list and what merge_r's caller reads after it: m_lastKey (and
// whether it is valid) and m_endKey.
static int64_t ref_posdb_merge_r(int mode, const uint8_t *const *lists, const int64_t *sizes, int n,
                                 int remove_neg_keys, int64_t min_rec_sizes, const char *sk, const char *ek,
                                 uint8_t *out, int64_t cap, char *last_key, int32_t *last_valid, char *end_key,
                                 int32_t *answered) {
  ref_init();
  if (n < 0 || n > 256) return -EINVAL;
  static RdbList in[256];
  RdbList *ptrs[256];
  for (int i = 0; i < n; i++) {
    in[i].freeList();
    int32_t sz = (int32_t)sizes[i];
    char *buf = NULL;
    if (sz > 0) {
      buf = (char *)mmalloc(sz, "refharness");
      memcpy(buf, lists[i], sz);
    }
    in[i].set(buf, sz, buf, sz, 0, true, true, 18);
    ptrs[i] = &in[i];
  }
  RdbList dst;
  dst.set(NULL, 0, NULL, 0, 0, true, true, 18);
  char startKey[18], endKey[18];
  memcpy(startKey, sk, 18);
  memcpy(endKey, ek, 18);
  const int32_t mrs = min_rec_sizes < 0 ? -1 : (int32_t)min_rec_sizes;
  if (!dst.prepareForMerge(ptrs, n, mrs)) return -ENOMEM;
  int32_t filtered = 0;
  *answered = 0;
  const double t0 = now_s();
  bool done = false;
  if (mode == 1 && gbref_adapter_merge) {
    // merge_r's steps before its posdbMerge_r call (RdbList.cpp:1681-1741)
    if (n == 0 || dst.m_mergeMinListSize == -1 || (mrs >= 0 && dst.m_listSize >= mrs)) {
      done = true;
    } else {
      KEYSET(dst.m_startKey, startKey, dst.m_ks);
      KEYSET(dst.m_endKey, endKey, dst.m_ks);
      if (KEYCMP(dst.m_startKey, dst.m_endKey, dst.m_ks) != 0 && KEYNEG(dst.m_endKey)) KEYSUB(dst.m_endKey, 1, dst.m_ks);
      dst.m_ks = ptrs[0]->m_ks;
      if (mrs == 0) done = true;
      else if (gbref_adapter_merge(&dst, ptrs, n, startKey, endKey, mrs, remove_neg_keys != 0)) {
        *answered = 1;
        done = true;
      } else {
        dst.posdbMerge_r(ptrs, n, startKey, endKey, dst.m_mergeMinListSize, remove_neg_keys != 0, &filtered,
                         false, false, 0);
        done = true;
      }
    }
  }
  if (!done)
    dst.merge_r(ptrs, n, startKey, endKey, mrs, remove_neg_keys != 0, RDB_POSDB, &filtered, NULL, NULL, false, 0);
  s_merge_s = now_s() - t0;
  int64_t sz = dst.m_listSize;
  if (sz > cap) return -ENOSPC;
  memcpy(out, dst.m_list, sz);
  memcpy(last_key, dst.m_lastKey, 18);
  *last_valid = dst.m_lastKeyIsValid ? 1 : 0;
  memcpy(end_key, dst.m_endKey, 18);
  dst.freeList();
  return sz;
}

// Msg3a::mergeLists (Msg3a.cpp:971-1503) over n fake shard replies, as
// Msg3a::gotAllShardReplies calls it: each reply is a Msg39Reply whose
// ptr_docIds / ptr_scores (double, Msg39.cpp:1661-1664) are the caller's
// arrays; no cluster recs (m_doSiteClustering off: the clusterdb site caps
// need Msg51 recs, out of scope), no facets (a query with no terms), no
// score info.  Output: the merged m_docIds / m_scores.
#include "Msg3a.h"
static int ref_msg3a_merge(int nshards, int32_t docs_to_get, const int32_t *counts,
                           const int64_t *const *docids, const double *const *scores,
                           std::vector<int64_t> &od, std::vector<double> &os) {
  ref_init();
  if (nshards < 0 || nshards > MAX_SHARDS || docs_to_get <= 0) return EINVAL;
  static Msg3a *m = NULL;
  static Msg39Request req;
  static Query q;
  static Msg39Reply rep[MAX_SHARDS];
  if (!m) m = new Msg3a();
  req.reset();
  req.m_doSiteClustering = false;
  req.m_getDocIdScoringInfo = false;
  q.m_numTerms = 0;
  m->m_q = &q;
  m->m_r = &req;
  m->m_debug = 0;
  m->m_docsToGet = docs_to_get;
  m->m_numHosts = nshards;
  for (int j = 0; j < nshards; j++) {
    Msg39Reply &r = rep[j];
    memset((void *)&r, 0, sizeof r);
    r.m_numDocIds = counts[j];
    r.ptr_docIds = (char *)docids[j];
    r.ptr_scores = (char *)scores[j];
    r.size_docIds = 8 * counts[j];
    r.size_scores = 8 * counts[j];
    m->m_reply[j] = &r;
  }
  m->mergeLists();
  od.assign(m->m_docIds, m->m_docIds + m->m_numDocIds);
  os.assign(m->m_scores, m->m_scores + m->m_numDocIds);
  for (int j = 0; j < nshards; j++) m->m_reply[j] = NULL;  // not Msg3a's to free
  return 0;
}

// ---- a24 whole: Msg39's reply with cluster records and facet lists, and
// Msg3a::mergeLists over such replies -- the ≤2-per-site cap
// (Msg3a.cpp:1342-1379), the facet-table merge (1089-1240) and the facet
// doc counts gotAllShardReplies sums (794-802).
#include <algorithm>
#include <stdlib.h>
#include "Clusterdb.h"
#include "Msg51.h"

// one shard's Msg39Reply (Msg39.h:169-208): its fixed fields and the
// variable parts serializeMsg lays out
struct ShardReply {
  std::vector<int64_t> docids;   // ptr_docIds
  std::vector<double> scores;    // ptr_scores
  std::vector<char> recs;        // ptr_clusterRecs: n x 12-byte key_t; empty = size_clusterRecs 0
  int32_t hits;                  // m_estimatedHits (int32 on the wire)
  std::vector<char> facets;      // ptr_facetHashList (Msg39.cpp:1457-1555 layout)
  std::vector<int64_t> fcounts;  // ptr_numDocsThatHaveFacetList, one per query term
};
// what Msg3a leaves: m_docIds / m_scores / m_clusterRecs, the summed hits,
// each QueryTerm's m_numDocsThatHaveFacet and m_facetHashTable
struct MergedOut {
  int32_t rc;
  std::vector<int64_t> docids;
  std::vector<double> scores;
  std::vector<char> recs;
  int64_t hits;
  std::vector<int64_t> fdocs;
  std::vector<std::vector<char> > tables;  // per query term: (i32 key, FacetEntry) by key
};

// a query term table read out in key order (its slot order is the hash's)
static std::vector<char> table_by_key(HashTableX *ft) {
  std::vector<std::pair<int32_t, int32_t> > slots;
  for (int32_t k = 0; ft->m_numSlots && k < ft->m_numSlots; k++)
    if (ft->m_flags[k]) slots.push_back(std::make_pair(ft->getKey32FromSlot(k), k));
  std::sort(slots.begin(), slots.end());
  std::vector<char> t(slots.size() * (4 + sizeof(FacetEntry)));
  for (size_t i = 0; i < slots.size(); i++) {
    memcpy(&t[i * 36], &slots[i].first, 4);
    memcpy(&t[i * 36 + 4], ft->getValFromSlot(slots[i].second), sizeof(FacetEntry));
  }
  return t;
}

// INTEGRATION.md §4's Msg3a-side block (gbgpuFillMsg3a over the exchange's
// merged result) -- linked only into gbref_gpu
extern int gbref_adapter_exchange(Msg3a *m, const Msg39Reply *mine) __attribute__((weak));

static Msg3a *s_m3a = NULL;
static Msg39Request s_m3req;
static Query s_m3q;
static QueryTerm s_m3qt[MAXT];

// Msg3a set up as Msg3a::getDocIds leaves it for mergeLists: the query's
// terms (m_termId, m_fieldCode: what the facet merge reads), the request's
// clustering flags
static void msg3a_setup(int32_t docs_to_get, bool clus, bool hide_all, bool family,
                        const std::vector<int64_t> &tids, const std::vector<int32_t> &fcs) {
  ref_init();
  if (!s_m3a) {
    s_m3a = new Msg3a();
    for (int i = 0; i < MAXT; i++) new (&s_m3qt[i].m_facetHashTable) HashTableX();
  }
  s_m3req.reset();
  s_m3req.m_doSiteClustering = clus;
  s_m3req.m_hideAllClustered = hide_all;
  s_m3req.m_familyFilter = family;
  s_m3req.m_getDocIdScoringInfo = false;
  // sortFacetEntries truncates each term's index to m_maxFacets (reset(): -1)
  s_m3req.m_maxFacets = 1 << 20;
  const int nqt = (int)tids.size();
  for (int i = 0; i < nqt; i++) {
    s_m3qt[i].m_termId = tids[i];
    s_m3qt[i].m_fieldCode = (char)fcs[i];
    s_m3qt[i].m_numDocsThatHaveFacet = 0;
  }
  s_m3q.m_qterms = s_m3qt;
  s_m3q.m_numTerms = nqt;
  s_m3a->m_q = &s_m3q;
  s_m3a->m_r = &s_m3req;
  s_m3a->m_debug = 0;
  s_m3a->m_docsToGet = docs_to_get;
  s_m3a->m_numTotalEstimatedHits = 0;
}

static void msg3a_read(MergedOut &o) {
  Msg3a *m = s_m3a;
  o.docids.assign(m->m_docIds, m->m_docIds + m->m_numDocIds);
  o.scores.assign(m->m_scores, m->m_scores + m->m_numDocIds);
  o.recs.clear();
  if (m->m_r->m_doSiteClustering)
    o.recs.assign((char *)m->m_clusterRecs, (char *)m->m_clusterRecs + 12 * (size_t)m->m_numDocIds);
  o.fdocs.clear();
  o.tables.clear();
  for (int i = 0; i < m->m_q->m_numTerms; i++) {
    o.fdocs.push_back(m->m_q->m_qterms[i].m_numDocsThatHaveFacet);
    o.tables.push_back(table_by_key(&m->m_q->m_qterms[i].m_facetHashTable));
  }
}

// mode 0: the reference's Msg3a::mergeLists over the replies; mode 1 (one
// reply, gbref_gpu): INTEGRATION.md's exchange of it as a one-rank RCCL
// collective and its fill of Msg3a
static int ref_msg3a_full(int mode, std::vector<ShardReply> &sh, int32_t docs_to_get, bool clus, bool hide_all,
                          bool family, const std::vector<int64_t> &tids, const std::vector<int32_t> &fcs,
                          MergedOut &o) {
  const int ns = (int)sh.size();
  const int nqt = (int)tids.size();
  if (ns < 0 || ns > MAX_SHARDS || docs_to_get <= 0 || nqt > MAXT || (mode == 1 && ns != 1)) return EINVAL;
  msg3a_setup(docs_to_get, clus, hide_all, family, tids, fcs);
  Msg3a *m = s_m3a;
  static Msg39Reply rep[MAX_SHARDS];
  m->m_numHosts = ns;
  o.hits = 0;
  for (int j = 0; j < ns; j++) {
    ShardReply &s = sh[j];
    Msg39Reply &r = rep[j];
    memset((void *)&r, 0, sizeof r);
    const int32_t n = (int32_t)s.docids.size();
    r.m_numDocIds = n;
    r.m_nqt = nqt;
    r.m_estimatedHits = s.hits;
    r.ptr_docIds = (char *)s.docids.data();
    r.size_docIds = 8 * n;
    r.ptr_scores = (char *)s.scores.data();
    r.size_scores = 8 * n;
    r.ptr_clusterRecs = s.recs.empty() ? NULL : (char *)s.recs.data();
    r.size_clusterRecs = (int32_t)s.recs.size();
    r.ptr_facetHashList = s.facets.empty() ? NULL : (char *)s.facets.data();
    r.size_facetHashList = (int32_t)s.facets.size();
    s.fcounts.resize(nqt, 0);
    r.ptr_numDocsThatHaveFacetList = (char *)s.fcounts.data();
    r.size_numDocsThatHaveFacetList = 8 * nqt;
    m->m_reply[j] = &r;
  }
  if (mode == 0) {
    // Msg3a::gotAllShardReplies (Msg3a.cpp:792-802): the hits and each
    // term's facet doc count summed over the replies, then mergeLists
    for (int j = 0; j < ns; j++) {
      o.hits += rep[j].m_estimatedHits;
      const int64_t *fc = (const int64_t *)rep[j].ptr_numDocsThatHaveFacetList;
      for (int k = 0; k < rep[j].m_nqt && k < s_m3q.m_numTerms; k++) s_m3qt[k].m_numDocsThatHaveFacet += fc[k];
    }
    srand(1);  // the facet merge picks m_docId with rand() (Msg3a.cpp:1232-1233)
    m->mergeLists();
  } else {
    if (!gbref_adapter_exchange) return ENOSYS;
    int rc = gbref_adapter_exchange(m, &rep[0]);
    if (rc) {
      for (int j = 0; j < ns; j++) m->m_reply[j] = NULL;
      return rc;
    }
    o.hits = m->m_numTotalEstimatedHits;
  }
  msg3a_read(o);
  for (int j = 0; j < ns; j++) m->m_reply[j] = NULL;  // not Msg3a's to free
  return 0;
}

// Msg51's clusterdb lookup (Msg51.cpp:380-416) over a synthetic clusterdb:
// the record of docid d has site hash d mod nsites (0 included), docids with
// d % 11 == 3 have none (CR_ERROR_CLUSTERDB, the record left 0), d % 13 == 5
// is adult, and d % 17 == 7 has the record of another docid (the mismatch
// keeps CR_ERROR_CLUSTERDB but the record is stored, Msg51.cpp:400-413)
static void fake_clusterdb(int64_t d, int32_t nsites, key_t *rec, char *level) {
  rec->n0 = 0;
  rec->n1 = 0;
  *level = CR_ERROR_CLUSTERDB;
  if (d % 11 == 3) return;
  const int64_t owner = d % 17 == 7 ? d ^ 0x40 : d;
  const int32_t sh = (int32_t)((uint64_t)(d * 2654435761ULL >> 7) % (uint64_t)(nsites > 0 ? nsites : 1));
  *rec = g_clusterdb.makeClusterRecKey(owner, d % 13 == 5, (uint8_t)(d % 5), sh, false);
  if (g_clusterdb.getDocId(rec) != d) return;
  *level = CR_OK;
}

// Msg39 after the intersection, as Msg39::setClusterRecs / gotClusterRecs
// (Msg39.cpp:1201-1344: Msg51's records, then the reference's own
// setClusterLevels with 2 docids per site) and estimateHitsAndSendReply
// (1346-1684: CR_OK nodes only, at most docsToGet, double scores or
// (double)m_intScore; the facet lists of every facet term; each term's
// m_numDocsThatHaveFacet; m_estimatedHits = hits less filtered, 409-414)
// build the reply, from the tree read high -> low
static void ref_msg39_reply(const int64_t *docids, const float *scores, int n, const orc_params *p, bool family,
                            int32_t nsites, int64_t hits, ShardReply &s) {
  const bool clus = p->site_clustering != 0;
  const bool ints = s_tab && s_tab->m_sortByTermNumInt >= 0;
  std::vector<key_t> recs(n > 0 ? n : 1);
  std::vector<char> levels(n > 0 ? n : 1, CR_OK);
  int32_t visible = n;
  if (clus && n > 0) {
    std::vector<int64_t> d(docids, docids + n);
    for (int i = 0; i < n; i++) fake_clusterdb(docids[i], nsites, &recs[i], &levels[i]);
    setClusterLevels(&recs[0], &d[0], n, 2, true, family, 0, false, &levels[0]);
    visible = 0;
    for (int i = 0; i < n; i++) visible += levels[i] == CR_OK;
  }
  int32_t nd = visible < p->docs_to_get ? visible : p->docs_to_get;
  s.docids.clear();
  s.scores.clear();
  s.recs.clear();
  for (int i = 0; i < n && (int32_t)s.docids.size() < nd; i++) {
    if (clus && levels[i] != CR_OK) continue;
    s.docids.push_back(docids[i]);
    s.scores.push_back(ints ? (double)s_ints[i] : (double)scores[i]);
    if (clus) s.recs.insert(s.recs.end(), (char *)&recs[i], (char *)&recs[i] + 12);
  }
  s.hits = (int32_t)hits;
  s.facets.clear();
  s.fcounts.clear();
  Query *q = s_tab ? s_tab->m_q : NULL;
  const int nqt = q ? q->m_numTerms : 0;
  for (int i = 0; i < nqt; i++) {
    QueryTerm *qt = &q->m_qterms[i];
    s.fcounts.push_back(qt->m_numDocsThatHaveFacet);
    if (qt->m_fieldCode != FIELD_GBFACETSTR && qt->m_fieldCode != FIELD_GBFACETINT &&
        qt->m_fieldCode != FIELD_GBFACETFLOAT)
      continue;
    HashTableX *ft = &qt->m_facetHashTable;
    if (!ft->m_numSlots || ft->m_numSlotsUsed == 0) continue;
    int32_t used = ft->getNumSlotsUsed();
    if (used > 20000) used = 20000;  // MAX_FACETS, Msg39.cpp:1449, 1518-1519
    const size_t at = s.facets.size();
    s.facets.resize(at + 12 + (size_t)used * 36);
    char *w = &s.facets[at];
    memcpy(w, &qt->m_termId, 8);
    memcpy(w + 8, &used, 4);
    w += 12;
    int32_t count = 0;
    for (int32_t k = 0; k < ft->m_numSlots; k++) {
      if (!ft->m_flags[k]) continue;
      const int32_t key = ft->getKey32FromSlot(k);
      memcpy(w, &key, 4);
      memcpy(w + 4, ft->getValFromSlot(k), sizeof(FacetEntry));
      w += 36;
      if (++count >= 20000) break;
    }
  }
}

static void write_merged(const MergedOut &o);

// ------------------------------------------------------------------ driver
// Binary request on stdin, response on stdout (little-endian, host layout):
//   op=1 query: i32 nterms, orc_params (its white_lists pointer ignored), nterms x orc_qterm,
//               nterms x (i64 size, bytes), i32 cap, i32 want_votes, i32 reps
//        ->     orc_result, n x i64 docid, n x f32 score,
//               i64 nvotes, nvotes x i64 docid, f64 seconds per run (median of
//               the time inside intersectLists10_r: the per-run list copies,
//               which the reference mutates, are not timed)
//   op=2 merge: i32 n, i32 remove_neg, i64 min_rec_sizes, n x (i64 size, bytes)
//        ->     i64 size (or -errno), bytes, f64 seconds inside merge_r
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

#include <algorithm>
#include <vector>

// the response stream: the process's original stdout, kept private; fd 1
// itself is pointed at stderr, so anything a linked library prints (RCCL /
// HIP banners and debug logs) cannot corrupt the protocol
static FILE *s_proto = NULL;

static void rd(void *p, size_t n) {
  if (n && fread(p, 1, n, stdin) != n) {
    fprintf(stderr, "gbref: short read\n");
    exit(2);
  }
}
static void wr(const void *p, size_t n) {
  if (n && fwrite(p, 1, n, s_proto) != n) exit(3);
}
// op 8 / 9 response: i32 n (or -errno), n x i64 docid, n x f64 score,
// i32 recs (0/1) then n x 12-byte cluster rec, i64 hits, i32 nqt, nqt x i64
// m_numDocsThatHaveFacet, per term i32 entries then (i32 key, FacetEntry) by key
static void write_merged(const MergedOut &o) {
  int32_t n = o.rc ? -o.rc : (int32_t)o.docids.size();
  wr(&n, 4);
  if (o.rc) return;
  wr(o.docids.data(), 8 * (size_t)n);
  wr(o.scores.data(), 8 * (size_t)n);
  const int32_t hr = o.recs.empty() ? 0 : 1;
  wr(&hr, 4);
  if (hr) wr(o.recs.data(), o.recs.size());
  wr(&o.hits, 8);
  const int32_t nqt = (int32_t)o.fdocs.size();
  wr(&nqt, 4);
  wr(o.fdocs.data(), 8 * (size_t)nqt);
  for (int i = 0; i < nqt; i++) {
    const int32_t ne = (int32_t)(o.tables[i].size() / 36);
    wr(&ne, 4);
    wr(o.tables[i].data(), o.tables[i].size());
  }
}
static double now_s() {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

int main(int argc, char **argv) {
  ref_init();  // Mem's global operator new needs g_mem before any allocation
  {
    const int pfd = dup(1);
    if (pfd < 0 || dup2(2, 1) < 0) return 6;
    s_proto = fdopen(pfd, "wb");
    if (!s_proto) return 6;
  }
  int32_t op;
  while (fread(&op, 4, 1, stdin) == 1) {
    if (op == 1 || op == 4 || op == 7 || op == 9) {
      // op 4: i32 mode first (0 the CPU body, 1 the GPU adapter), then op 1's
      // request; the response adds i32 passes the adapter answered, i32
      // m_numUsedNodes and n x i32 m_intScore.
      // op 9: i32 mode, i32 familyFilter, i32 hideAllClustered, i32 nsites,
      // then op 1's request: the query (mode 0 the CPU body, 1 the adapter),
      // Msg39's reply from its tree over the synthetic clusterdb
      // (fake_clusterdb), and that one reply merged (mode 0 the reference's
      // Msg3a::mergeLists, 1 INTEGRATION.md's exchange): op 1's response,
      // then write_merged's
      int32_t mode = 0, o9[3] = {0, 0, 0};
      if (op == 4 || op == 9) rd(&mode, 4);
      if (op == 9) rd(o9, 12);
      s_adapter = mode;
      s_answered = 0;
      int32_t nt;
      rd(&nt, 4);
      if (nt < 0 || nt > MAXT) return 4;
      orc_params p;
      rd(&p, sizeof p);
      std::vector<orc_qterm> t(nt);
      rd(t.data(), sizeof(orc_qterm) * nt);
      std::vector<std::vector<uint8_t> > bufs(nt);
      std::vector<const uint8_t *> ptrs(nt);
      std::vector<int64_t> sizes(nt);
      for (int i = 0; i < nt; i++) {
        rd(&sizes[i], 8);
        bufs[i].resize(sizes[i] + 1);
        rd(bufs[i].data(), sizes[i]);
        ptrs[i] = bufs[i].data();
      }
      int32_t cap, want_votes, reps, nw;
      rd(&cap, 4);
      rd(&want_votes, 4);
      rd(&reps, 4);
      rd(&nw, 4);  // whitelist lists follow
      if (nw < 0 || nw > MAX_WHITELISTS) return 4;
      std::vector<std::vector<uint8_t> > wbufs(nw);
      std::vector<orc_list> wl(nw);
      for (int i = 0; i < nw; i++) {
        int64_t sz;
        rd(&sz, 8);
        wbufs[i].resize(sz + 1);
        rd(wbufs[i].data(), sz);
        wl[i].bytes = wbufs[i].data();
        wl[i].size = sz;
      }
      p.n_white_lists = nw;
      p.white_lists = nw ? wl.data() : NULL;
      int32_t ntok;
      rd(&ntok, 4);  // the boolean expression (s_btok), 0: not boolean
      if (ntok < 0 || ntok > 256) return 4;
      s_btok.resize(ntok);
      rd(s_btok.data(), 4 * (size_t)ntok);
      int32_t nfr;
      rd(&nfr, 4);  // facet ranges: per term i32 term, i32 n, n x i32 a, n x i32 b
      if (nfr < 0 || nfr > MAXT) return 4;
      s_franges.assign(nfr, FacetRanges());
      for (int i = 0; i < nfr; i++) {
        rd(&s_franges[i].term, 4);
        rd(&s_franges[i].n, 4);
        if (s_franges[i].n < 0 || s_franges[i].n > MAX_FACET_RANGES) return 4;
        s_franges[i].a.resize(s_franges[i].n);
        s_franges[i].b.resize(s_franges[i].n);
        rd(s_franges[i].a.data(), 4 * (size_t)s_franges[i].n);
        rd(s_franges[i].b.data(), 4 * (size_t)s_franges[i].n);
      }
      std::vector<int64_t> d(cap > 0 ? cap : 1);
      std::vector<float> s(cap > 0 ? cap : 1);
      int64_t vcap = 0;
      for (int i = 0; i < nt; i++) vcap += sizes[i] / 12 + 1;
      std::vector<int64_t> votes(want_votes ? vcap : 1);
      orc_result r;
      memset(&r, 0, sizeof r);
      std::vector<double> times;
      if (reps < 1) reps = 1;
      int rc = 0;
      for (int k = 0; k < reps; k++) {
        s_isect_s = 0;
        rc = ref_query(t.data(), ptrs.data(), sizes.data(), nt, &p, d.data(), s.data(), cap, &r,
                       want_votes ? votes.data() : NULL, vcap);
        times.push_back(s_isect_s);
        if (rc) break;
      }
      if (rc) r.corrupt = -rc;
      std::sort(times.begin(), times.end());
      double med = times[times.size() / 2];
      wr(&r, sizeof r);
      wr(d.data(), 8 * (size_t)r.n);
      wr(s.data(), 4 * (size_t)r.n);
      int64_t nv = want_votes ? std::min<int64_t>(r.hits, vcap) : 0;
      wr(&nv, 8);
      wr(votes.data(), 8 * (size_t)nv);
      wr(&med, 8);
      // score info buffers: DocIdScore[], PairScore[], SingleScore[] bytes
      for (int b = 0; b < 3; b++) {
        const int64_t nb = (int64_t)s_info[b].size();
        wr(&nb, 8);
        wr(s_info[b].data(), (size_t)nb);
      }
      // the boolean truth table (i32 groups, -1 none; then its bytes)
      wr(&s_bgroups, 4);
      if (s_bgroups >= 0) wr(s_btable.data(), s_btable.size());
      if (s_facets.size() < 4) s_facets.assign(4, 0);
      wr(s_facets.data(), s_facets.size());  // the facet tables
      s_facets.clear();
      if (op == 7) {
        // the shard's reply merged by the reference's own Msg3a::mergeLists
        // (one shard: the TopTree's first docsToGet as Msg39 sends them,
        // double scores), then the same query through gbgpuShardQuery
        std::vector<double> sd(r.n > 0 ? r.n : 1);
        // Msg39.cpp:1661-1664: m_score, or (double)m_intScore with integer tree scores
        const bool ints = s_tab && s_tab->m_sortByTermNumInt >= 0;
        for (int i = 0; i < r.n; i++) sd[i] = ints ? (double)s_ints[i] : (double)s[i];
        const int64_t *dp = d.data();
        const double *sp = sd.data();
        const int32_t cnt = std::min<int32_t>(r.n, p.docs_to_get);
        std::vector<int64_t> od;
        std::vector<double> os;
        int mrc = ref_msg3a_merge(1, p.docs_to_get, &cnt, &dp, &sp, od, os);
        int32_t no = mrc ? -mrc : (int32_t)od.size();
        wr(&no, 4);
        if (no > 0) {
          wr(od.data(), 8 * (size_t)no);
          wr(os.data(), 8 * (size_t)no);
        }
        const int32_t k = p.docs_to_get;
        std::vector<int64_t> gd(k > 0 ? k : 1);
        std::vector<double> gs(k > 0 ? k : 1);
        int32_t gn = 0;
        int64_t gh = 0;
        int32_t grc = gbref_adapter_shard ? gbref_adapter_shard(s_tab, ptrs.data(), sizes.data(), k, gd.data(),
                                                                gs.data(), &gn, &gh)
                                          : -1;
        if (grc) gn = 0;
        wr(&grc, 4);
        wr(&gn, 4);
        wr(&gh, 8);
        wr(gd.data(), 8 * (size_t)gn);
        wr(gs.data(), 8 * (size_t)gn);
      }
      if (op == 9) {
        MergedOut o;
        o.rc = 0;
        o.hits = 0;
        std::vector<int64_t> tids(nt);
        std::vector<int32_t> fcs(nt);
        for (int i = 0; i < nt; i++) {
          // distinct termids: Msg39's facet lists name their term by it and
          // Msg3a finds it with getQueryTermByTermId64 (Msg3a.cpp:1156)
          tids[i] = 1000003LL * (i + 1);
          fcs[i] = t[i].field_code;
          if (s_tab && i < s_tab->m_q->m_numTerms) s_tab->m_q->m_qterms[i].m_termId = tids[i];
        }
        std::vector<ShardReply> sh(1);
        if (rc == 0) {
          ref_msg39_reply(d.data(), s.data(), r.n, &p, o9[0] != 0, o9[2], r.hits - r.filtered, sh[0]);
          o.rc = ref_msg3a_full(mode, sh, p.docs_to_get, p.site_clustering != 0, o9[1] != 0, o9[0] != 0, tids, fcs, o);
        } else {
          o.rc = rc;
        }
        write_merged(o);
      }
      if (op == 4) {
        wr(&s_answered, 4);
        wr(&s_used_nodes, 4);
        for (int i = 0; i < r.n; i++) {
          const int32_t v = i < (int)s_ints.size() ? s_ints[i] : 0;
          wr(&v, 4);
        }
        // i32 words, then the plan (ngroups; per group flags0, nsub, nsub x (term, flags))
        const int32_t np = (int32_t)s_plan.size();
        wr(&np, 4);
        wr(s_plan.data(), 4 * (size_t)np);
      }
      s_adapter = 0;
    } else if (op == 2) {
      int32_t n, rm;
      int64_t mrs;
      rd(&n, 4);
      rd(&rm, 4);
      rd(&mrs, 8);
      if (n < 0 || n > 256) return 4;
      std::vector<std::vector<uint8_t> > bufs(n);
      std::vector<const uint8_t *> ptrs(n);
      std::vector<int64_t> sizes(n);
      int64_t tot = 0;
      for (int i = 0; i < n; i++) {
        rd(&sizes[i], 8);
        bufs[i].resize(sizes[i] + 1);
        rd(bufs[i].data(), sizes[i]);
        ptrs[i] = bufs[i].data();
        tot += sizes[i];
      }
      std::vector<uint8_t> out(tot + 64);
      int64_t sz = ref_posdb_merge(ptrs.data(), sizes.data(), n, rm, mrs, out.data(), tot + 64);
      wr(&sz, 8);
      if (sz > 0) wr(out.data(), sz);
      wr(&s_merge_s, 8);
    } else if (op == 6) {
      // merge_r with start/end keys: i32 mode (0 merge_r, 1 with the
      // adapter), i32 n, i32 remove_neg, i64 min_rec_sizes, 18 B start key,
      // 18 B end key, n x (i64 size, bytes)  ->  i64 size (or -errno), bytes,
      // 18 B m_lastKey, i32 m_lastKeyIsValid, 18 B m_endKey, i32 answered
      int32_t mode, n, rm;
      int64_t mrs;
      char sk[18], ek[18];
      rd(&mode, 4);
      rd(&n, 4);
      rd(&rm, 4);
      rd(&mrs, 8);
      rd(sk, 18);
      rd(ek, 18);
      if (n < 0 || n > 256) return 4;
      std::vector<std::vector<uint8_t> > bufs(n);
      std::vector<const uint8_t *> ptrs(n);
      std::vector<int64_t> sizes(n);
      int64_t tot = 0;
      for (int i = 0; i < n; i++) {
        rd(&sizes[i], 8);
        bufs[i].resize(sizes[i] + 1);
        rd(bufs[i].data(), sizes[i]);
        ptrs[i] = bufs[i].data();
        tot += sizes[i];
      }
      std::vector<uint8_t> out(tot + 64);
      char lk[18], ekey[18];
      int32_t lv = 0, ans = 0;
      memset(lk, 0, 18);
      memset(ekey, 0, 18);
      int64_t sz = ref_posdb_merge_r(mode, ptrs.data(), sizes.data(), n, rm, mrs, sk, ek, out.data(), tot + 64, lk,
                                     &lv, ekey, &ans);
      wr(&sz, 8);
      if (sz > 0) wr(out.data(), sz);
      wr(lk, 18);
      wr(&lv, 4);
      wr(ekey, 18);
      wr(&ans, 4);
    } else if (op == 3) {
      // Msg3a merge: i32 nshards, i32 docs_to_get, per shard i32 n,
      // n x i64 docid, n x f64 score  ->  i32 n (or -errno), n x i64, n x f64
      int32_t ns, dtg;
      rd(&ns, 4);
      rd(&dtg, 4);
      if (ns < 0 || ns > MAX_SHARDS) return 4;
      std::vector<int32_t> cnt(ns);
      std::vector<std::vector<int64_t> > dd(ns);
      std::vector<std::vector<double> > ss(ns);
      std::vector<const int64_t *> dp(ns);
      std::vector<const double *> sp(ns);
      for (int j = 0; j < ns; j++) {
        rd(&cnt[j], 4);
        if (cnt[j] < 0) return 4;
        dd[j].resize(cnt[j] + 1);
        ss[j].resize(cnt[j] + 1);
        rd(dd[j].data(), 8 * (size_t)cnt[j]);
        rd(ss[j].data(), 8 * (size_t)cnt[j]);
        dp[j] = dd[j].data();
        sp[j] = ss[j].data();
      }
      std::vector<int64_t> od;
      std::vector<double> os;
      int rc = ref_msg3a_merge(ns, dtg, cnt.data(), dp.data(), sp.data(), od, os);
      int32_t n = rc ? -rc : (int32_t)od.size();
      wr(&n, 4);
      if (n > 0) {
        wr(od.data(), 8 * (size_t)n);
        wr(os.data(), 8 * (size_t)n);
      }
    } else if (op == 8) {
      // Msg3a over full replies: i32 nshards, i32 docs_to_get, i32
      // doSiteClustering, i32 hideAllClustered, i32 familyFilter, i32 nqt,
      // nqt x i64 m_termId, nqt x i32 m_fieldCode; per shard i32 n, i32 recs
      // (0/1), n x i64 docid, n x f64 score, [n x 12-byte cluster rec], i32
      // m_estimatedHits, i32 facet list bytes + bytes, i32 counts (0/1) +
      // nqt x i64  ->  write_merged
      int32_t h[6];
      rd(h, sizeof h);
      const int32_t ns = h[0], nqt = h[5];
      if (ns < 0 || ns > MAX_SHARDS || nqt < 0 || nqt > MAXT) return 4;
      std::vector<int64_t> tids(nqt);
      std::vector<int32_t> fcs(nqt);
      rd(tids.data(), 8 * (size_t)nqt);
      rd(fcs.data(), 4 * (size_t)nqt);
      std::vector<ShardReply> sh(ns);
      for (int j = 0; j < ns; j++) {
        int32_t n, hr, fb, hc;
        rd(&n, 4);
        rd(&hr, 4);
        if (n < 0) return 4;
        sh[j].docids.resize(n);
        sh[j].scores.resize(n);
        rd(sh[j].docids.data(), 8 * (size_t)n);
        rd(sh[j].scores.data(), 8 * (size_t)n);
        if (hr) {
          sh[j].recs.resize(12 * (size_t)n);
          rd(sh[j].recs.data(), 12 * (size_t)n);
        }
        rd(&sh[j].hits, 4);
        rd(&fb, 4);
        if (fb < 0) return 4;
        sh[j].facets.resize(fb);
        rd(sh[j].facets.data(), fb);
        rd(&hc, 4);
        if (hc) {
          sh[j].fcounts.resize(nqt);
          rd(sh[j].fcounts.data(), 8 * (size_t)nqt);
        }
      }
      MergedOut o;
      o.rc = ref_msg3a_full(0, sh, h[1], h[2] != 0, h[3] != 0, h[4] != 0, tids, fcs, o);
      write_merged(o);
    } else {
      return 5;
    }
    fflush(s_proto);
  }
  return 0;
}
