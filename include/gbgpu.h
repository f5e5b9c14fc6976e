/* gbgpu -- MI355X-native Posdb query scoring, C ABI (the drop-in boundary).
 *
 * Replaces the body of PosdbTable::intersectLists10_r (Posdb.cpp:5437-7806)
 * behind the unchanged Msg39::intersectLists sequence (Msg39.cpp:884-1053):
 *
 *   reference call (file:line)                        gbgpu entry point
 *   ------------------------------------------------  ---------------------------
 *   PosdbTable::init            Posdb.cpp:722-786      gbgpu_query(...terms, lists)
 *   PosdbTable::allocTopTree    Posdb.cpp:838-1090     gbgpu_docs_wanted()/internal
 *   PosdbTable::setQueryTermInfo Posdb.cpp:4354-4869   internal (host plan)
 *   PosdbTable::intersectLists10_r Posdb.cpp:5437-7806 gbgpu_query / _resident
 *   TopTree::addNode / getHighNode TopTree.cpp:195-516 gbgpu_result (high -> low)
 *   Msg3a::mergeLists           Msg3a.cpp:971-1503     gbgpu_allgather_topk (RCCL) /
 *                                                      gbgpu_merge_topk (host lists);
 *     (site cap, facet merge)                          gbgpu_allgather_replies (RCCL) /
 *                                                      gbgpu_merge_replies(_device)
 *   RdbList::posdbMerge_r       RdbList.cpp:3065-3568  gbgpu_merge_posdb
 *   Msg3::readList -> RdbScan   Msg3.cpp:553-731,       gbgpu_file_upload /
 *     (a Posdb file read)       RdbScan.cpp:319-361    gbgpu_file_list (in HBM)
 *   Msg5::mergeLists_r          Msg5.cpp:1415-1471,    gbgpu_termlist_merge (the
 *     (files + tree, merge_r)   1621-1795             pieces merged in HBM)
 *
 * Conventions: plain pointers and sizes only; the caller owns
 * every input and output buffer and they are never mutated; the library owns
 * device memory.  Functions return 0 or a positive errno-style code that the
 * Msg39 adapter copies into PosdbTable::m_errno; no exceptions cross the ABI.
 *
 * Concurrency: one context per GPU, shared by every INTERSECT thread of the
 * process.  A context owns 1..64 query slots (gbgpu_set_query_slots), each
 * with its own HIP stream and buffers over the shared resident lists; the
 * blocking entry points (gbgpu_query, gbgpu_query_resident) are re-entrant
 * and take a free slot, waiting for one when all are busy.  The slot-explicit
 * enqueue/collect pair is for a single caller per slot.  A list freed while a
 * query in flight still reads it is released when that query is collected.
 */
#ifndef GBGPU_H
#define GBGPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GBGPU_ABI_VERSION 13

/* error codes beyond errno.h (Errno.h numbering is not reused) */
#define GBGPU_ENODEVICE   1001 /* no HIP device / extension not usable        */
#define GBGPU_EUNSUPPORTED 1002 /* request mode outside the GPU path */
#define GBGPU_ECORRUPT    1003 /* corrupt posdb list (Posdb.cpp:6289-6302)    */
#define GBGPU_EHIP        1004 /* HIP runtime error                           */
#define GBGPU_ECAPACITY   1005 /* a fixed device capacity was exceeded        */

typedef struct gbgpu_ctx gbgpu_ctx;

/* One query term, as Query::set2 leaves Query::m_qterms[i] (Query.h:404-580)
 * and Msg39Request::ptr_termFreqWeights[i] (Msg39.h:152). */
typedef struct gbgpu_qterm {
  int32_t is_required;              /* m_isRequired                                  */
  int32_t term_sign;                /* m_termSign: '-' -> BF_NEGATIVE (Posdb.cpp:4570) */
  int32_t field_code;               /* m_fieldCode: plain fields, gbsortby:/gbrevsortby:
                                       float (54/55), range terms gbmin:/gbmax:/gbequal:
                                       (56-57, 61-62, 66-67; own list only, positive),
                                       gbsortby: int (59/60: gbgpu_result::int_scores);
                                       facets gbfacetstr:/int:/float: (63-65:
                                       gbgpu_result::facets) */
  int32_t piped;                    /* m_piped                                       */
  int32_t synonym_of;               /* index of m_synonymOf, -1 if none              */
  int32_t left_phrase_term;         /* m_leftPhraseTermNum, -1 if none               */
  int32_t right_phrase_term;        /* m_rightPhraseTermNum, -1 if none              */
  int32_t is_wiki_half_stop_bigram; /* m_isWikiHalfStopBigram                        */
  int32_t qpos;                     /* m_qword->m_posNum                             */
  int32_t wiki_phrase_id;           /* m_qword->m_wikiPhraseId                       */
  int32_t quote_start;              /* m_qword->m_quoteStart, -1 if none             */
  float   tf_weight;                /* ptr_termFreqWeights[i]                        */
  float    number_float;            /* m_qword->m_float: gbmin:/gbmax:/gbequal: float bound  */
  int32_t  number_int;              /* m_qword->m_int: the int range terms' bound (56-57, 61-62,
                                       66-67 filter votes by the key's number, Posdb.cpp:4948-4999) */
} gbgpu_qterm;

/* A posdb termlist exactly as Msg2::getList(i) holds it: first key 18 bytes,
 * then 12/6-byte compressed keys (RdbList.cpp:282-327).  Host memory. */
typedef struct gbgpu_list {
  const uint8_t *bytes;
  int64_t size;
} gbgpu_list;

/* Msg39Request scalars read by PosdbTable (Msg39.h:94-147).  Zero-filled
 * trailing fields reproduce a request without paging and without the max-score
 * prefilter; Msg39Request::reset() (Msg39.h:36-82) sets do_max_score_algo=1. */
typedef struct gbgpu_params {
  int32_t docs_to_get;      /* m_docsToGet                                        */
  int32_t real_max_top;     /* m_realMaxTop (clamped to MAX_TOP = 10)              */
  int32_t language;         /* m_language                                         */
  int32_t site_clustering;  /* m_doSiteClustering: TopTree domain caps
                               (TopTree.cpp:64-186, 312-516) and the pruning they
                               make live (minWinningScore, Posdb.cpp:7699-7704;
                               getMaxPossibleScore 7811-7960; ring buffer
                               6365-6504), replayed in docid order on the GPU   */
  int32_t num_docid_splits; /* m_numDocIdSplits: >1 runs Msg39's docid-split loop
                               (Msg39.cpp:345-457) inside gbgpu_query/_resident:
                               one pass per docid piece [d0, d1+2] into one TopTree
                               sized at the first piece (Posdb.cpp:859-877); hits
                               and filtered are the sums over pieces.  The
                               enqueue/collect form returns EUNSUPPORTED for it */
  float   same_lang_weight; /* m_sameLangWeight                                   */
  int32_t do_max_score_algo;/* m_doMaxScoreAlgo: per-term getMaxPossibleScore
                               prefilter (Posdb.cpp:6046-6047, 6327-6346)         */
  int32_t get_docid_scoring_info; /* m_getDocIdScoringInfo: the per-docid score
                               breakdown second pass (Posdb.cpp:6116-6244,
                               7554-7665, 7752-7775) into gbgpu_result's
                               docid/pair/single score arrays, also over docid
                               splits (one second pass per piece; GBGPU_EUNSUPPORTED
                               only where the reference's buffers would fill and
                               kick records out, Posdb.cpp:7588-7665) */
  double  max_serp_score;   /* m_maxSerpScore  } paging of a widget's next page:   */
  int64_t min_serp_docid;   /* m_minSerpDocId  } nonzero enables the filter of
                               Posdb.cpp:4379-4381, 7327-7347 (counted in
                               gbgpu_result::filtered).  With a gbsortby int term
                               the tree's m_intScore is compared with
                               (int32_t)max_serp_score as x86-64 truncates it
                               (INT32_MIN when out of range or NaN), Posdb.cpp:
                               7330-7336                                         */
  /* The "&sites=" whitelist: use_whitelist = (Msg39Request::size_whiteList > 1)
   * (Posdb.cpp:800-801); white_lists = Msg2::m_whiteLists[0..m_w), host
   * memory, not mutated.  A docid is voted only if the 5 bytes at rec+7 of its
   * smallest-group key (docid and siteRank's top bit) are those of some record
   * of a whitelist list (Posdb.cpp:5294, 5544-5572); with no records at all,
   * nothing is.  Zero-filled: no whitelist. */
  int32_t use_whitelist;
  int32_t n_white_lists;
  const struct gbgpu_list *white_lists;
  /* Boolean queries (Query::m_isBoolean): the docid set is the union of every
   * group's sublists, negative groups included, each docid carrying the bit
   * vector of the QueryTermInfos it occurs in (QueryTerm::m_bitNum = the
   * group index, Posdb.cpp:4485-4721), kept where the query's expression
   * holds for that vector (makeDocIdVoteBufForBoolQuery_r, Posdb.cpp:
   * 8006-8249); its score is the number of bits set, times sameLangWeight on
   * a language match (Posdb.cpp:6514-6534, 7247-7256; m_siteRankMultiplier is
   * 0, Posdb.cpp:774).  The expression comes as its truth table: bit v
   * (byte v >> 3, bit v & 7) = Query::matchesBoolQuery over vector v, for
   * every v < 2^bool_ngroups; bool_ngroups must equal the plan's
   * m_numQueryTermInfos (<= 16; more is GBGPU_EUNSUPPORTED).  The whitelist
   * does not apply (the boolean vote never reads it).  Zero: not boolean. */
  int32_t is_boolean;
  int32_t bool_ngroups;
  const uint8_t *bool_table;
  /* Facet terms (gbfacetstr: / gbfacetint: / gbfacetfloat:, field codes
   * 63-65) are required terms whose termlists hold a 32-bit value where the
   * word position is; the result carries each one's QueryTerm::
   * m_facetHashTable (gbgpu_result::facets).  A gbfacetint:/gbfacetfloat:
   * term may bucket its values into [A, B) ranges (QueryWord::
   * m_numFacetRanges, m_facetRange{Int,Float}{A,B}, Query.h:389-393; floats
   * by their 32-bit patterns).  Zero-filled: no ranges. */
  int32_t n_facet_ranges;
  int32_t pad_f;
  const struct gbgpu_facet_ranges *facet_ranges;
} gbgpu_params;

typedef struct gbgpu_facet_ranges {
  int32_t term;          /* the facet query term                       */
  int32_t n;             /* ranges, <= 256                              */
  const int32_t *a, *b;  /* bounds [a[k], b[k]): int32 or float bits    */
} gbgpu_facet_ranges;

/* One entry of a facet term's table: the value's (or its range's A) 32
 * bits and Posdb.h:401-413's FacetEntry -- the search results with that
 * value (m_count, one vote per docid), the last of them (m_docId), the sum
 * (int64, or a double's bits for gbfacetfloat), max and min of their values,
 * and the value's count over the whole termlist buffer
 * (m_outsideSearchResultsCount, countUniqueDocids, Posdb.cpp:5002-5038). */
typedef struct gbgpu_facet_entry {
  int32_t term;     /* the facet query term                            */
  int32_t key;      /* HashTableX key                                  */
  int32_t count;    /* FacetEntry: m_count                             */
  int32_t outside;  /*             m_outsideSearchResultsCount         */
  int64_t docid;    /*             m_docId                             */
  int64_t sum;      /*             m_sum                               */
  int32_t max, min; /*             m_max, m_min                        */
} gbgpu_facet_entry;


/* The second pass's score info (m_getDocIdScoringInfo, Posdb.cpp:6116-6244,
 * 7554-7665): byte-for-byte the layout of the reference's DocIdScore /
 * PairScore / SingleScore (Posdb.h:767-866) on x86-64, so the adapter copies
 * the three arrays into m_scoreInfoBuf / m_pairScoreBuf / m_singleScoreBuf.
 * Fields the reference leaves unset (m_termFreq*, the two pointers, padding)
 * are zero here. */
typedef struct gbgpu_pair_score {
  float   final_score;
  int8_t  is_synonym1, is_synonym2, is_half_stop_wiki_bigram1, is_half_stop_wiki_bigram2;
  int8_t  diversity_rank1, diversity_rank2, density_rank1, density_rank2;
  int8_t  word_spam_rank1, word_spam_rank2, hash_group1, hash_group2;
  int8_t  in_same_wiki_phrase, fixed_distance;
  int32_t word_pos1, word_pos2;
  int64_t term_freq1, term_freq2;
  float   tf_weight1, tf_weight2;
  int32_t qterm_num1, qterm_num2;
  int8_t  bflags1, bflags2;
  int32_t qdist;
} gbgpu_pair_score;
typedef struct gbgpu_single_score {
  float   final_score;
  int8_t  is_synonym, is_half_stop_wiki_bigram, diversity_rank, density_rank, word_spam_rank, hash_group;
  int32_t word_pos;
  int64_t term_freq;
  float   tf_weight;
  int32_t qterm_num;
  int8_t  bflags;
} gbgpu_single_score;
typedef struct gbgpu_docid_score {
  int64_t docid;
  double  final_score;
  int8_t  site_rank;
  int32_t doc_lang;
  int32_t num_required_terms;
  int32_t num_pairs, num_singles;
  int32_t pairs_offset, singles_offset;  /* byte offsets into the pair / single arrays, -1 if none */
  void   *pair_scores, *single_scores;   /* NULL */
} gbgpu_docid_score;

/* The observable PosdbTable state Msg39 reads (Msg39.cpp:402-435, 1346-1420). */
typedef struct gbgpu_result {
  int64_t *docids;     /* caller-owned, `capacity` entries; TopTree high -> low   */
  float   *scores;     /* caller-owned, `capacity` entries (TopNode::m_score)     */
  int32_t  capacity;
  int32_t  n;          /* entries written: every TopTree node (m_numUsedNodes;
                          <= docs_wanted without site clustering), <= capacity */
  int64_t  hits;       /* m_docIdVoteBuf.length()/6: exact intersection size       */
  int32_t  filtered;   /* m_filtered                                               */
  int32_t  docs_wanted;/* TopTree::m_docsWanted (0: no tree was allocated)          */
  /* optional: the intersected docid set itself -- the docids of
   * m_docIdVoteBuf after addDocIdVotes/rmDocIdVotes (Posdb.cpp:5154-5171,
   * 5281-5290, 4871-4946), ascending.  NULL to skip.  With docid splits it is
   * the union over the pieces (boundary docids once). */
  int64_t *hit_docids;   /* caller-owned, hit_capacity entries                     */
  int64_t  hit_capacity;
  int64_t  n_hit_docids; /* entries written (min(set size, hit_capacity))          */
  /* with gbgpu_params::get_docid_scoring_info: the second pass's records for
   * the first min(n, docs_to_get) docids of the tree, high -> low, one
   * DocIdScore each, their PairScores / SingleScores in the reference's append
   * order.  With docid splits every piece's second pass appends its own
   * records (the tree's first docs_to_get nodes inside the piece's docid
   * range, Posdb.cpp:6160-6193), so the arrays need room for up to
   * (pieces x docs_to_get) docids.  Caller-owned arrays of *_cap entries;
   * *_n = entries written (ENOSPC if an array is too small). */
  gbgpu_docid_score  *docid_scores;  int32_t docid_scores_cap;  int32_t n_docid_scores;
  gbgpu_pair_score   *pair_scores;   int32_t pair_scores_cap;   int32_t n_pair_scores;
  gbgpu_single_score *single_scores; int32_t single_scores_cap; int32_t n_single_scores;
  /* optional, `capacity` entries: TopNode::m_intScore when a gbsortby int
   * term makes the tree use integer scores (scores[] are then 0.0, as the
   * reference's m_score); 0 otherwise.  NULL to skip. */
  int32_t *int_scores;
  /* with facet terms: every facet term's table (Posdb.cpp:1000-1067,
   * 5575-5631, 7362-7542), entries by term then key ascending, n_facets of
   * them (ENOSPC when that exceeds facets_cap; NULL: not written), and
   * facet_docs[term] = m_numDocsThatHaveFacet (countUniqueDocids' count,
   * Posdb.cpp:7786-7796) for each of the nterms terms (0 for a term with no
   * table: not a facet term, or a query that ended before allocTopTree; over
   * docid splits a facet term with an empty list still has its table, as the
   * Query's tables go on over the pieces).  Both NULL: no facet pass.  Facets
   * run with site clustering, over docid splits and in boolean queries, at
   * most 4 facet terms, each a group of its own list alone
   * (GBGPU_EUNSUPPORTED otherwise).  ENOSPC: only n_facets is valid (over docid
   * splits the call returns before the tree and the score-info outputs are
   * written): call again with facets_cap >= n_facets. */
  gbgpu_facet_entry *facets;
  int32_t facets_cap;
  int32_t n_facets;
  uint64_t *facet_docs;
} gbgpu_result;

int         gbgpu_open(int device, gbgpu_ctx **out);
void        gbgpu_close(gbgpu_ctx *ctx);
const char *gbgpu_strerror(int code);
int         gbgpu_abi_version(void);

/* allocTopTree sizing (Posdb.cpp:838-930): TopTree::m_docsWanted for a query
 * (with docid splits: list_sizes are the first piece's lists).  With site
 * clustering the tree may hold more nodes than this (TopTree.cpp:64-186):
 * gbgpu_tree_capacity() is the most a result can carry. */
int32_t gbgpu_docs_wanted(const gbgpu_params *p, const int64_t *list_sizes, int nterms);
int32_t gbgpu_tree_capacity(const gbgpu_params *p, const int64_t *list_sizes, int nterms);

/* Full drop-in: lists[] are 1-1 with terms[] (Msg2::getList(i)).  Uploads the
 * lists, intersects, scores and returns the top tree.  Synchronous. */
int gbgpu_query(gbgpu_ctx *ctx, const gbgpu_qterm *terms, int nterms, const gbgpu_list *lists,
                const gbgpu_params *p, gbgpu_result *out);

/* Device-resident index: upload a termlist once (the first-key swap of
 * Posdb.cpp:5671-5703 is applied to the device copy) and query it many times. */
int gbgpu_list_upload(gbgpu_ctx *ctx, const uint8_t *bytes, int64_t size, int32_t *handle);
int gbgpu_list_free(gbgpu_ctx *ctx, int32_t handle);

/* Resident Rdb files (the read path into HBM): a Posdb file
 * image (termlists back to back, as Msg3 reads them from disk, size a
 * multiple of 6) is uploaded once; a termlist or a docid-range piece of one is
 * then cut from it on the device with no host copy.  gbgpu_file_list is
 * RdbScan's read (RdbScan.cpp:319-361) over HBM: `offset`/`size` are the byte
 * range the caller's RdbMap gives (Msg3.cpp:534-584: RdbMap::getPageRange, getKey);
 * when the key at `offset` is compressed (12 or 6 bytes), `key18` is the full
 * key RdbScan writes in its place (m_startKey, the map's page key) -- it must
 * match the stored bytes, else EINVAL; for an 18-byte first key it may be
 * NULL.  The new list handle is a gbgpu_list_upload list (its own copy, the
 * same checks), freed with gbgpu_list_free; the file stays until
 * gbgpu_file_free. */
int gbgpu_file_upload(gbgpu_ctx *ctx, const uint8_t *bytes, int64_t size, int32_t *file);
int gbgpu_file_list(gbgpu_ctx *ctx, int32_t file, int64_t offset, int64_t size, const uint8_t *key18,
                    int32_t *handle);
/* The termlists of one query cut together (Msg2 hands Msg3 all of a query's
 * reads at once): n cuts as gbgpu_file_list's, key18s NULL or n entries each
 * NULL or a map key; one device round trip for the heads and one for the
 * checks whatever n is.  All or nothing: on an error no handle is created and
 * handles[] holds -1. */
int gbgpu_file_lists(gbgpu_ctx *ctx, int32_t file, int n, const int64_t *offsets, const int64_t *sizes,
                     const uint8_t *const *key18s, int32_t *handles);
int gbgpu_file_free(gbgpu_ctx *ctx, int32_t file);

/* Msg5's read of one termlist (Msg5.cpp:1415-1471 prepare, 1621-1795
 * mergeLists_r): the termlist's range from every Posdb file (Msg3's reads,
 * oldest file first) and the in-memory tree's list (newest, last) merged by
 * RdbList::merge_r's posdb rules (gbgpu_merge_posdb: newest equal key wins,
 * remove_neg_keys drops surviving delete keys -- Msg2 reads queries with it
 * on -- and the min_rec_sizes bound) into ONE resident list, the handle a
 * gbgpu_list_upload list would be (the same checks; free with
 * gbgpu_list_free).  A file piece is a byte range of a resident file image
 * with its map key when the range starts at a compressed key, as
 * gbgpu_file_list takes it; a host piece (file < 0) is a list in host memory
 * whose first key is 18 bytes (the tree's list, RdbTree::getList).  Every
 * piece stays in HBM: the file cuts are device copies, the merge runs on the
 * device.  RdbList::constrain's trim to the exact start/end keys stays with
 * the caller (the ranges passed are the ones it keeps).  When merged_out is
 * not NULL the merged list's bytes are also copied there (merged_cap bytes;
 * ENOSPC if they do not fit) with their size in *merged_size.  Synchronous. */
typedef struct gbgpu_piece {
  int32_t file;          /* resident file handle, or -1: `bytes` in host memory */
  int32_t pad;
  int64_t offset, size;  /* the byte range (of the file, or of `bytes`)          */
  const uint8_t *key18;  /* the map key at `offset` when it is compressed, or NULL */
  const uint8_t *bytes;  /* file < 0: the host list                               */
} gbgpu_piece;
int gbgpu_termlist_merge(gbgpu_ctx *ctx, const gbgpu_piece *pieces, int n, int remove_neg_keys,
                         int64_t min_rec_sizes, int32_t *handle, uint8_t *merged_out, int64_t merged_cap,
                         int64_t *merged_size);
/* gbgpu_query and gbgpu_query_resident are re-entrant: Msg39 runs several
 * intersect threads at once (Msg39.cpp:1019-1027, Parms.cpp:12356); each call
 * takes a free query slot (its own HIP stream and buffers over the shared
 * resident lists) and waits for one when all are busy. */
int gbgpu_query_resident(gbgpu_ctx *ctx, const gbgpu_qterm *terms, int nterms,
                         const int32_t *handles, const gbgpu_params *p, gbgpu_result *out);

/* Query slots: a context starts with one; grow the pool to n (<= 64) so that
 * n queries can be in flight at once.  Returns 0 or an errno-style code. */
int gbgpu_set_query_slots(gbgpu_ctx *ctx, int n);
int gbgpu_query_slots(gbgpu_ctx *ctx);

/* Asynchronous form: enqueue a resident query on a slot's stream (no host
 * synchronisation; EBUSY if that slot still holds an uncollected query),
 * then collect its result (waits for that slot's stream only). */
int gbgpu_query_slot_enqueue(gbgpu_ctx *ctx, int slot, const gbgpu_qterm *terms, int nterms,
                             const int32_t *handles, const gbgpu_params *p);
int gbgpu_query_slot_collect(gbgpu_ctx *ctx, int slot, gbgpu_result *out);
/* slot 0 shorthands */
int gbgpu_query_resident_enqueue(gbgpu_ctx *ctx, const gbgpu_qterm *terms, int nterms,
                                 const int32_t *handles, const gbgpu_params *p);
int gbgpu_query_collect(gbgpu_ctx *ctx, gbgpu_result *out);
/* a slot's HIP stream (hipStream_t), for callers that order work on it */
void *gbgpu_slot_stream(gbgpu_ctx *ctx, int slot);
void *gbgpu_stream(gbgpu_ctx *ctx); /* slot 0 */
/* device copy of the last query's top list (the Msg39Reply payload for an RCCL
 * allgather): *n uint32 order-preserving score keys (0 = empty slot), then at
 * the next 256-byte boundary *n int64 docids.  Valid after gbgpu_query_collect. */
int gbgpu_last_topk_device(gbgpu_ctx *ctx, void **dev_ptr, int32_t *n);

/* Msg3a::mergeLists (Msg3a.cpp:1315-1467) without site clustering, on the
 * host: the shards' replies as Msg39 sends them (docids, double scores --
 * m_score, or (double)m_intScore for gbsortby int queries, Msg39.cpp:
 * 1661-1664).  The loop takes the best shard head each step (higher double
 * score; on equal scores the lower docid; on equal docids the earlier
 * shard), passes over a docid already merged, and stops at `k` entries; a
 * reply need not be sorted.  Pinned to the reference's own mergeLists
 * (tests/golden/x_*.npz). */
int gbgpu_merge_topk(const int64_t *const *shard_docids, const double *const *shard_scores,
                     const int32_t *shard_counts, int nshards, int32_t k,
                     int64_t *out_docids, double *out_scores, int32_t *out_n);

/* The device merge gbgpu_allgather_topk runs after its all-gather, on replies
 * given from the host (one per shard: counts[r] entries as Msg39 sends them,
 * double scores, and the shard's hit count); for checking the merge without
 * a multi-GPU node.  Same rules as gbgpu_merge_topk. */
int gbgpu_merge_topk_device(gbgpu_ctx *ctx, int nranks, int32_t k, const int32_t *counts, const int64_t *shard_hits,
                            const int64_t *const *shard_docids, const double *const *shard_scores,
                            int64_t *docids, double *scores, int32_t *n, int64_t *hits);

/* Exchange ordering.  Every rank must issue its collectives in the same
 * order, but a process runs several INTERSECT threads (Msg39.cpp:1019-1027,
 * up to `mct`) whose queries finish in any order.  A sequencer admits
 * exactly one caller at a time, in increasing sequence number: the caller
 * holding query `seq` waits in gbgpu_seq_enter until every smaller number
 * has left.  Sequence numbers are agreed across ranks (the front end that
 * sends one Msg39Request to every shard numbers it) and
 * each must be entered and left on every rank exactly once, starting at
 * `first`.  gbgpu_seq_enter returns 0 when admitted, ETIMEDOUT after
 * timeout_ms (< 0: wait forever), EINVAL for a number already past or
 * already admitted; gbgpu_seq_leave returns EINVAL unless `seq` is the one
 * admitted.  Host code only (no device): the context's own sequencer orders
 * gbgpu_allgather_topk, and a caller with its own transport may use one. */
typedef struct gbgpu_seq gbgpu_seq;
int gbgpu_seq_open(uint64_t first, gbgpu_seq **out);
int gbgpu_seq_enter(gbgpu_seq *s, uint64_t seq, int timeout_ms);
int gbgpu_seq_leave(gbgpu_seq *s, uint64_t seq);
uint64_t gbgpu_seq_next(const gbgpu_seq *s); /* the number admitted next */
void gbgpu_seq_close(gbgpu_seq *s);

/* Msg39 -> Msg3a over RCCL: one context per GPU, each
 * holding one docid range of the index (a shard).  Rank 0 makes the id with
 * gbgpu_comm_unique_id and the caller ships it to every rank; each rank then
 * calls gbgpu_comm_init (collective; the exchange sequence starts at 0).
 * gbgpu_allgather_topk replaces the collect of a slot's enqueued query:
 * that shard's reply -- the first min(nodes, k) of its TopTree as Msg39
 * sends it (double scores: m_score, or (double)m_intScore for gbsortby int)
 * and its hit count -- is all-gathered over xGMI and merged on the device by
 * Msg3a::mergeLists' rules (gbgpu_merge_topk; the clusterdb site cap of
 * Msg3a.cpp:1342-1379 needs cluster records and is not applied).  Every
 * rank receives the same merged list and the summed hit count; `local` (may
 * be NULL) receives the shard's own result.  `seq` is the query's exchange
 * sequence number: the call waits (timeout_ms, as gbgpu_seq_enter) until
 * every smaller number has been exchanged on this rank, so concurrent
 * callers issue the collectives in the same order on every rank.  slot < 0
 * sends an empty reply (a shard whose query failed still takes part). */
#define GBGPU_COMM_ID_BYTES 128
int gbgpu_comm_unique_id(uint8_t *id);
int gbgpu_comm_init(gbgpu_ctx *ctx, int nranks, int rank, const uint8_t *id);
int gbgpu_allgather_topk(gbgpu_ctx *ctx, int slot, uint64_t seq, int timeout_ms, int32_t k, int64_t *docids,
                         double *scores, int32_t *n, int64_t *hits, gbgpu_result *local);
/* Msg3a::mergeLists whole (Msg3a.cpp:971-1503) over full Msg39Replies: the
 * shards' CR_OK nodes with their 12-byte clusterdb records, as Msg39 builds
 * the reply after Msg51 and setClusterLevels (Msg39.cpp:1201-1344,
 * 1346-1684), and their facet lists.  On top of gbgpu_merge_topk's rules:
 * with site clustering a head whose record has n0 and n1 both non-zero is
 * dropped when familyFilter is on and it is adult, or when its 26-bit site
 * hash (non-zero) already has 2 results -- 1 with hideAllClustered -- and is
 * counted against its site otherwise, before the docid test (1342-1385);
 * each term's facet entries from every reply are merged into its table
 * (1089-1240: count, outside count, int64 sums, double sums in reply order,
 * min/max by the reference's count-zero rule; a list naming a termid the
 * query lacks ends the walk, for that reply and every later one; m_docId: the first entry's -- the
 * reference picks one at random, 1232-1233); and the hits and every term's
 * m_numDocsThatHaveFacet are summed as gotAllShardReplies does (792-802).
 * The caller keeps Msg3a::sortFacetEntries (923-962), which orders its
 * hash table for display. */
typedef struct gbgpu_reply {       /* one Msg39Reply (Msg39.h:169-208)          */
  int32_t n;                       /* m_numDocIds                               */
  int32_t hits;                    /* m_estimatedHits (an int32 on the wire)    */
  const int64_t *docids;           /* ptr_docIds, n                             */
  const double  *scores;           /* ptr_scores, n                             */
  const uint8_t *cluster_recs;     /* ptr_clusterRecs, n x 12-byte key_t; NULL
                                      when size_clusterRecs is 0                 */
  const uint8_t *facet_list;       /* ptr_facetHashList: per facet term i64
                                      termid, i32 n, n x (i32 key, FacetEntry)  */
  int32_t facet_list_size;         /* size_facetHashList                        */
  int32_t nqt;                     /* m_nqt (must equal the request's)           */
  const int64_t *facet_docs;       /* ptr_numDocsThatHaveFacetList (nqt), or NULL */
} gbgpu_reply;
typedef struct gbgpu_merge_req {   /* what mergeLists reads of Msg3a / the request */
  int32_t docs_to_get;             /* Msg3a::m_docsToGet (> 0, <= 4096 on the device) */
  int32_t site_clustering;         /* m_r->m_doSiteClustering                   */
  int32_t hide_all_clustered;      /* m_r->m_hideAllClustered                   */
  int32_t family_filter;           /* m_r->m_familyFilter                        */
  int32_t nqt;                     /* m_q->m_numTerms (<= 64)                    */
  int32_t pad;
  const int64_t *term_ids;         /* m_q->m_qterms[i].m_termId                  */
  const int32_t *field_codes;      /* m_q->m_qterms[i].m_fieldCode               */
} gbgpu_merge_req;
typedef struct gbgpu_merged {      /* what mergeLists and gotAllShardReplies leave */
  int64_t *docids;                 /* m_docIds, cap entries                      */
  double  *scores;                 /* m_scores                                   */
  uint8_t *cluster_recs;           /* m_clusterRecs (12 bytes each; with site
                                      clustering), or NULL                       */
  int32_t  cap;
  int32_t  n;                      /* m_numDocIds                                */
  int64_t  hits;                   /* m_numTotalEstimatedHits                    */
  int64_t *facet_docs;             /* nqt: QueryTerm::m_numDocsThatHaveFacet, or NULL */
  gbgpu_facet_entry *facets;       /* every term's m_facetHashTable, by term then
                                      key; ENOSPC past facets_cap (n_facets set) */
  int32_t  facets_cap;
  int32_t  n_facets;
} gbgpu_merged;
/* on the host */
int gbgpu_merge_replies(const gbgpu_merge_req *req, const gbgpu_reply *replies, int nshards, gbgpu_merged *out);
/* the same merge on the device, over replies given from the host */
int gbgpu_merge_replies_device(gbgpu_ctx *ctx, const gbgpu_merge_req *req, const gbgpu_reply *replies,
                               int nshards, gbgpu_merged *out);
/* The exchange of full replies over RCCL: every rank passes its own shard's
 * reply (after Msg51 and the CR_OK filter), the replies are all-gathered
 * over xGMI (a fixed-size head, then the bodies at the largest one's size)
 * and merged on the device; every rank receives the same merged result.
 * Sequenced like gbgpu_allgather_topk (one sequence for both); `mine` may
 * be NULL (an empty reply: a shard whose query failed still takes part). */
int gbgpu_allgather_replies(gbgpu_ctx *ctx, uint64_t seq, int timeout_ms, const gbgpu_merge_req *req,
                            const gbgpu_reply *mine, gbgpu_merged *out);

/* the exchange sequence number this context admits next (a single-threaded
 * caller's default `seq`); calls refused before admission (a bad k, a null
 * output, ETIMEDOUT) leave it unchanged */
uint64_t gbgpu_exchange_next(gbgpu_ctx *ctx);

/* RdbList::posdbMerge_r (RdbList.cpp:3065-3568), as RdbList::merge_r
 * (RdbList.cpp:1658-1756) calls it after prepareForMerge (410-491): merge n
 * (<= 256) sorted posdb lists, oldest first, each starting with an 18-byte
 * key (else EINVAL); on equal keys (bfcmpPosdb, RdbList.h:620-641) only the
 * newest list's survives; remove_neg_keys drops surviving delete keys; the
 * output is re-compressed and stops after the first key that reaches
 * min(sum of sizes, min_rec_sizes + 36, out_cap) bytes (min_rec_sizes < 0:
 * no bound; 0: nothing).  ENOSPC if a key would start within 18 bytes of
 * out_cap (give out_cap >= sum of sizes + 64).  Host buffers. */
int gbgpu_merge_posdb(gbgpu_ctx *ctx, const gbgpu_list *lists, int n, int remove_neg_keys,
                      int64_t min_rec_sizes, uint8_t *out, int64_t out_cap, int64_t *out_size);
/* Same on device-resident runs (each 16-byte aligned, readable up to its size
 * rounded up to 16) into a device buffer (2-byte aligned).  Synchronous. */
int gbgpu_merge_posdb_device(gbgpu_ctx *ctx, const uint8_t *const *dev_lists, const int64_t *sizes, int n,
                             int remove_neg_keys, int64_t min_rec_sizes, uint8_t *dev_out,
                             int64_t out_cap, int64_t *out_size);
/* The last key the last merge wrote, as 18 bytes with the compression bits
 * cleared -- what posdbMerge_r leaves in RdbList::m_lastKey (RdbList.cpp:
 * 3521-3535), from which merge_r's caller shrinks m_endKey (3544-3565).
 * 0, or ENOENT if the merge wrote no key. */
int gbgpu_merge_last_key(gbgpu_ctx *ctx, uint8_t *key18);
/* Whether the last merge stopped at its bound with input keys left unmerged:
 * posdbMerge_r's numLists > 0 after its loop, the second condition (beside
 * m_listSize >= the bound) of its m_endKey shrink (RdbList.cpp:3537-3565). */
int gbgpu_merge_input_left(gbgpu_ctx *ctx, int32_t *left);
/* Device timings of the last merge (HIP events), ms: [0] total, [1] decode,
 * [2] partition, [3] tile count pass, [4] tile offset scan, [5] tile write
 * pass; and the number of keys decoded and of merge tiles. */
int gbgpu_merge_timings(gbgpu_ctx *ctx, float *ms6, int64_t *nkeys, int64_t *ntiles);
/* The pipeline of the last merge: 2 = decoded keys (every key decoded to
 * HBM, then tiles gather them), 0 = none.  (1, a tile pipeline decoding the
 * compressed runs in LDS, was measured slower and retired.) */
int gbgpu_merge_path(gbgpu_ctx *ctx);

/* Per-query device timings of a slot's last query (HIP events on its stream),
 * in milliseconds: [0]=total, [1]=candidate extraction, [2]=list probe scan,
 * [3]=compaction, [4]=scoring, [5]=top-k.  Enable with gbgpu_set_profiling. */
int gbgpu_set_profiling(gbgpu_ctx *ctx, int enable);
int gbgpu_slot_timings(gbgpu_ctx *ctx, int slot, float *ms6, int64_t *scan_bytes);
int gbgpu_last_timings(gbgpu_ctx *ctx, float *ms6, int64_t *scan_bytes); /* slot 0 */
/* Work counts of a slot's last collected query, for per-kernel rooflines:
 * [0] bytes of every list it scanned, [1] of the smallest group's lists
 * (candidate extraction), [2] of the probed lists, [3] candidates,
 * [4] survivors (hits), [5] bytes of the survivors' runs (mini-merge input,
 * one copy per group a list serves), [6] TopTree nodes (site clustering). */
int gbgpu_slot_stats(gbgpu_ctx *ctx, int slot, int64_t *stats8);

/* The achievable-HBM ceiling of SURVEY.md §8(d): 16-B/lane streaming read and
 * copy kernels over `bytes`-sized buffers (give >> 256 MiB), `iters` passes
 * each; GB/s of bytes read (read) and read + written (copy). */
int gbgpu_bandwidth_ceiling(gbgpu_ctx *ctx, int64_t bytes, int iters, double *read_gbps, double *copy_gbps);

#ifdef __cplusplus
}
#endif
#endif
