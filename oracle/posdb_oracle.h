/* TEST INFRASTRUCTURE ONLY -- the CPU restatement ("oracle") of the
 * reference's Posdb query-scoring path.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it; the product never does.
 *
 * Parity status: PINNED.  The posdb key codec is pinned by the reference's
 * own known-answer test (Posdb.cpp:24-86, tests/test_codec.py).  The query
 * path (intersectLists10_r + TopTree) and the list merge (merge_r ->
 * posdbMerge_r) are pinned against the reference's own code, compiled
 * unmodified into oracle/_ref/gbref (oracle/ref.mk): bit-exact on the
 * committed golden vectors (tests/golden/, tests/test_golden.py) and on fresh
 * seeds (tests/test_reference.py).  This file restates the reference
 * algorithm line by line, citing file:line.
 */
#ifndef GB_POSDB_ORACLE_H
#define GB_POSDB_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* one query term as Query::set2 leaves it (Query.h:404-580) */
typedef struct orc_qterm {
  int32_t is_required;              /* QueryTerm::m_isRequired                 */
  int32_t term_sign;                /* m_termSign ('-' -> BF_NEGATIVE)         */
  int32_t field_code;               /* m_fieldCode (0: plain word/phrase)      */
  int32_t piped;                    /* m_piped                                 */
  int32_t synonym_of;               /* index of m_synonymOf, -1 if none        */
  int32_t left_phrase_term;         /* m_leftPhraseTermNum, -1 if none         */
  int32_t right_phrase_term;        /* m_rightPhraseTermNum, -1 if none        */
  int32_t is_wiki_half_stop_bigram; /* m_isWikiHalfStopBigram                  */
  int32_t qpos;                     /* m_qword->m_posNum                       */
  int32_t wiki_phrase_id;           /* m_qword->m_wikiPhraseId                 */
  int32_t quote_start;              /* m_qword->m_quoteStart (-1 none)         */
  float   tf_weight;                /* Msg39Request::ptr_termFreqWeights[i]    */
  float   number_float;             /* m_qword->m_float (range terms; gbref only) */
  int32_t number_int;               /* m_qword->m_int                          */
} orc_qterm;

/* same layout as gbgpu_params (include/gbgpu.h) */
typedef struct orc_params {
  int32_t docs_to_get;      /* Msg39Request::m_docsToGet               */
  int32_t real_max_top;     /* m_realMaxTop (clamped to MAX_TOP=10)    */
  int32_t language;         /* m_language                              */
  int32_t site_clustering;  /* m_doSiteClustering (TopTree domain caps) */
  int32_t num_docid_splits; /* m_numDocIdSplits: Msg39's split loop      */
  float   same_lang_weight; /* m_sameLangWeight                        */
  int32_t do_max_score_algo;/* m_doMaxScoreAlgo                        */
  int32_t get_docid_scoring_info; /* m_getDocIdScoringInfo (gbref only; the oracle
                                     does not restate the second pass)  */
  double  max_serp_score;   /* m_maxSerpScore                          */
  int64_t min_serp_docid;   /* m_minSerpDocId (nonzero: paging filter) */
  /* the "&sites=" whitelist (Msg39Request::size_whiteList > 1 and
   * Msg2::m_whiteLists[0..m_w), Posdb.cpp:793-835, 5294, 5544-5572) */
  int32_t use_whitelist;
  int32_t n_white_lists;
  const struct orc_list *white_lists;
  /* boolean queries (makeDocIdVoteBufForBoolQuery_r, Posdb.cpp:8006-8249):
   * the expression as its truth table over QueryTermInfo bit vectors
   * (bit v = Query::matchesBoolQuery(v)), as gbgpu_params carries it */
  int32_t is_boolean;
  int32_t bool_ngroups;
  const uint8_t *bool_table;
  /* gbfacetint:/gbfacetfloat: ranges (QueryWord::m_numFacetRanges,
   * m_facetRange{Int,Float}{A,B}, Query.h:389-393), as gbgpu_params */
  int32_t n_facet_ranges;
  int32_t pad_f;
  const struct orc_facet_ranges *facet_ranges;
} orc_params;

typedef struct orc_facet_ranges {
  int32_t term;        /* the facet query term */
  int32_t n;           /* ranges (<= 256) */
  const int32_t *a, *b; /* [A, B) bounds: int32, or float bits for gbfacetfloat */
} orc_facet_ranges;

/* The facet tables of the last orc_query (QueryTerm::m_facetHashTable and
 * m_numDocsThatHaveFacet, Posdb.cpp:1000-1067, 5575-5631, 7362-7542,
 * 5002-5038 / 7786-7796), serialized into `w` (cap int32 words): i32 nterms;
 * per facet term: i32 term, u64 docs (2 words), i32 n, n x (i32 key, i32
 * count, i32 outside, i64 docid, i64 sum, i32 max, i32 min) with keys
 * ascending.  Returns the words written, or -1 if cap is too small. */
int orc_last_facets(int32_t *w, int cap);
/* stale-mbuf docids of the last orc_query: scored from earlier docids' bytes
 * (defined) and skipped (bytes no docid of the pass wrote) */
void orc_last_stale(int32_t *defined, int32_t *undefined);

typedef struct orc_list {
  const uint8_t *bytes;
  int64_t size;
} orc_list;

typedef struct orc_result {
  int64_t hits;        /* m_docIdVoteBuf.length()/6                          */
  int32_t filtered;    /* m_filtered                                          */
  int32_t docs_wanted; /* TopTree::m_docsWanted (0: no tree allocated)        */
  int32_t n;           /* entries written (TopTree read high -> low; all of
                          m_numUsedNodes with site clustering)            */
  int32_t corrupt;     /* intersectLists10_r bailed on a corrupt list          */
} orc_result;

/* Runs init/allocTopTree/setQueryTermInfo/intersectLists10_r semantics on
 * copies of the lists (the caller's bytes are not mutated).  docids/scores
 * must hold `cap` entries.  Returns 0, or an errno-style code. */
int orc_query(const orc_qterm *terms, const uint8_t *const *lists, const int64_t *sizes,
              int nterms, const orc_params *p, int64_t *docids, float *scores, int cap,
              orc_result *out);

/* Bare intersection: the docids surviving addDocIdVotes/rmDocIdVotes, in
 * vote-buffer order.  Returns count (or -errno); writes up to cap docids. */
int64_t orc_intersect(const orc_qterm *terms, const uint8_t *const *lists, const int64_t *sizes,
                      int nterms, int64_t *docids, int64_t cap, const orc_params *prm);

/* RdbList::merge_r -> posdbMerge_r (RdbList.cpp:1658-1756, 3065-3568) into an
 * empty list, with prepareForMerge's bound (RdbList.cpp:410-491): min_rec_sizes
 * is the caller's minRecSizes (-1: no limit).  Lists oldest first, each
 * starting with an 18-byte key.  Returns bytes written to out (cap bytes). */
int64_t orc_posdb_merge(const uint8_t *const *lists, const int64_t *sizes, int n,
                        int remove_neg_keys, int64_t min_rec_sizes, uint8_t *out, int64_t cap);

/* weight tables of initWeights (Posdb.cpp:1105-1197), for table tests */
/* Msg3a::mergeLists (Msg3a.cpp:971-1503), no site clustering / facets:
 * returns the merged count, or -errno; out arrays hold docs_to_get entries */
int32_t orc_msg3a_merge(const int64_t *const *docids, const double *const *scores, const int32_t *counts,
                        int nshards, int32_t docs_to_get, int64_t *out_docids, double *out_scores);

/* Msg3a::mergeLists whole (Msg3a.cpp:971-1503) over full Msg39Replies
 * (Msg39.h:169-208; the layout of gbgpu_reply): the <=2-per-site cap over
 * cluster records (1342-1379), the facet-table merge (1089-1240) and the
 * per-term facet doc counts and hits gotAllShardReplies sums (792-802).
 * Merged facet entries go out by term, then key ascending, with the first
 * merged entry's m_docId (the reference picks one at random, 1232-1233).
 * Returns 0 or an errno-style code. */
typedef struct orc_reply {
  int32_t n, hits;
  const int64_t *docids;
  const double *scores;
  const uint8_t *cluster_recs; /* n x 12 bytes, or NULL */
  const uint8_t *facet_list;
  int32_t facet_list_size, nqt;
  const int64_t *facet_docs;   /* nqt, or NULL */
} orc_reply;
typedef struct orc_merge_req {
  int32_t docs_to_get, site_clustering, hide_all_clustered, family_filter, nqt, pad;
  const int64_t *term_ids;
  const int32_t *field_codes;
} orc_merge_req;
typedef struct orc_facet_entry {
  int32_t term, key, count, outside;
  int64_t docid, sum;
  int32_t max, min;
} orc_facet_entry;
int orc_msg3a_full(const orc_merge_req *rq, const orc_reply *rep, int nshards, int64_t *out_docids,
                   double *out_scores, uint8_t *out_recs, int32_t *out_n, int64_t *out_hits, int64_t *out_fdocs,
                   orc_facet_entry *facets, int32_t facets_cap, int32_t *n_facets);

void orc_weights(float *density32, float *wordspam16, float *linker16, float *hashgroup11,
                 float *diversity16);

#ifdef __cplusplus
}
#endif
#endif
