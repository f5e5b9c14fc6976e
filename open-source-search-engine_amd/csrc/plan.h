// Query plan: the host-side restatement of PosdbTable::setQueryTermInfo
// (Posdb.cpp:4354-4869) and allocTopTree sizing (Posdb.cpp:838-930), plus the
// POD image of it that the kernels read from device memory.
#ifndef GBGPU_PLAN_H
#define GBGPU_PLAN_H

#include <stdint.h>

#include "../../include/gbgpu.h"

namespace gbgpu {

// Posdb.h:102-108
enum : uint8_t {
  BF_HALFSTOPWIKIBIGRAM = 0x01,
  BF_PIPED = 0x02,
  BF_SYNONYM = 0x04,
  BF_NEGATIVE = 0x08,
  BF_BIGRAM = 0x10,
  BF_NUMBER = 0x20,
  BF_FACET = 0x40,
};
constexpr uint8_t BF_EXCLUDE = BF_PIPED | BF_NEGATIVE | BF_NUMBER | BF_FACET;

constexpr int REF_MAX_SUBLISTS = 50;  // Posdb.h:417
// GPU-path capacities (EUNSUPPORTED beyond)
constexpr int MAXG = 16;     // QueryTermInfos (required term groups)
constexpr int MAXSUB = 32;   // sublists per group (MAXL: one group may hold every list)
constexpr int MAXL = 32;     // distinct lists referenced by one query
constexpr int MAXG0 = 8;     // sublists of the smallest group (candidate arrays)
constexpr uint32_t NEG_BIT = 0x80000000u;

// One QueryTermInfo (Posdb.h:421-451), host form.
struct GroupInfo {
  int qterm;                       // m_qtermNum
  int nsub;                        // m_numSubLists
  int sub_term[REF_MAX_SUBLISTS];  // query-term index of each sublist
  uint8_t flags[REF_MAX_SUBLISTS]; // m_bigramFlags (incl. written-but-uncounted slots)
  int64_t total;                   // m_totalSubListsSize (pre-swap sizes)
  float tfw;
  int qpos, wiki, quote;
};

struct HostPlan {
  int nqt = 0;
  int ngroups = 0;
  GroupInfo g[MAXG * 4];
  int min_listi = -1;
  int64_t min_list_size = 0;
  int32_t docs_wanted = 0;
  int real_max_top = 10;
  int sortby_group = -1;  // m_sortByTermInfoNum(Int) (gbsortby:/gbrevsortby:, Posdb.cpp:4413-4425)
  int sortby_int = 0;     // the int form: TopTree integer scores (m_useIntScores)
};

// Query::m_fieldCode values PosdbTable treats specially (Query.h:118-132);
// every other field code is an ordinary term list to it
enum : int32_t {
  FIELD_GBSORTBYFLOAT = 54,
  FIELD_GBREVSORTBYFLOAT = 55,
  FIELD_GBNUMBERMIN = 56,
  FIELD_GBNUMBERMAX = 57,
  FIELD_GBSORTBYINT = 59,
  FIELD_GBREVSORTBYINT = 60,
  FIELD_GBNUMBERMININT = 61,
  FIELD_GBNUMBERMAXINT = 62,
  FIELD_GBFACETSTR = 63,
  FIELD_GBFACETINT = 64,
  FIELD_GBFACETFLOAT = 65,
  FIELD_GBNUMBEREQUALINT = 66,
  FIELD_GBNUMBEREQUALFLOAT = 67,
};
// a field code the GPU path does not implement (range, int sortby, facets)
// range terms: (mode, int?) of a field code, mode 0 if not one
inline int range_mode(int32_t fc, int *is_int) {
  *is_int = fc == FIELD_GBNUMBERMININT || fc == FIELD_GBNUMBERMAXINT || fc == FIELD_GBNUMBEREQUALINT;
  if (fc == FIELD_GBNUMBERMIN || fc == FIELD_GBNUMBERMININT) return 1;
  if (fc == FIELD_GBNUMBERMAX || fc == FIELD_GBNUMBERMAXINT) return 2;
  if (fc == FIELD_GBNUMBEREQUALFLOAT || fc == FIELD_GBNUMBEREQUALINT) return 3;
  return 0;
}

// Device image.  Lists are addressed by a dense id 0..nlists-1.
struct DevList {
  const uint8_t *p;     // swapped list (12-byte first key), 16-B aligned, zero padded
  const uint32_t *pm;   // its page map: run starts before each CHUNK_UNITS-unit page
  uint32_t units;       // (size-6)/6
  uint32_t group_bits;  // positive groups containing this list (+NEG_BIT if in a negative group)
  int32_t g0_array;     // index among the smallest group's candidate arrays, -1 if none
  int32_t probe;        // k_probe direction: 0 not scanned, PROBE_BY_CAND, PROBE_BY_RUN
  // a list several positive groups use is shrunk in place once per use
  // (shrinkSubLists, Posdb.cpp:5334-5428): the first use (owner_group,
  // owner_sub) sees it clean, every later one sees the re-shrunk buffer
  int16_t owner_group, owner_sub;
  int32_t uses;         // positive group sublist positions naming this list
  // range term (gbmin:/gbmax:/gbequal:, Posdb.cpp:4948-4999): a docid is voted
  // by this list only if a key of its run holds a number in range
  int32_t rmode;        // 0 none, 1 min (>=), 2 max (<=), 3 equal
  int32_t rint;         // compare getInt (1) or getFloat (0)
  float rf;             // m_qword->m_float
  int32_t ri;           // m_qword->m_int
};
constexpr int32_t PROBE_BY_CAND = 1;  // dense list: candidates search the chunk's run starts
constexpr int32_t PROBE_BY_RUN = 2;   // sparse list: run starts look up the candidate directory

struct DevPlan {
  int ngroups;
  int nlists;
  uint32_t pos_mask;
  int real_max_top;
  int language;
  float same_lang_weight;
  float site_rank_multiplier;
  int nqt;  // Query::m_numTerms (scoreMatrix stride)
  // paging filter (Posdb.cpp:4379-4381, 7327-7347): m_hasMaxSerpScore
  int has_serp;
  double max_serp_score;
  int64_t min_serp_docid;
  int32_t max_serp_int;  // (int32_t)m_maxSerpScore, the bound for integer scores (Posdb.cpp:7330-7336)
  // the "&sites=" whitelist (Posdb.cpp:793-835, 5294, 5544-5572): sorted
  // 5-byte values (bytes 7..11 of a key: docid + siteRank's top bit); a
  // group-0 candidate whose run head is not among them is rejected
  // (k_write_runs writes wrej[slot], k_compact skips it)
  int use_white;
  int use_rej;          // wrej[] marks slots not voted (whitelist or a range term's first group)
  uint32_t nwhite;
  const uint64_t *white;
  uint8_t *wrej;
  // site clustering: the pruning bounds (Posdb.cpp:6327-6504, 7811-7960)
  uint32_t reshare_mask;   // bit l: list l is shrunk more than once (uses >= 2)
  int clustering;
  int do_max_score;        // m_doMaxScoreAlgo
  int has_facet;           // m_hasFacetTerm: the scoring filter is skipped (Posdb.cpp:6353-6356)
  int min_listi;           // m_minListi (group whose positions seed the ring buffer)
  int all_same_wiki;       // m_allInSameWikiPhrase (Posdb.cpp:5764-5778)
  // groups, in QueryTermInfo order
  uint8_t gflags0[MAXG];            // m_bigramFlags[0]
  uint8_t gnsub[MAXG];
  uint8_t gsub[MAXG][MAXSUB];       // dense list id per original sublist index
  uint8_t gsubflags[MAXG][MAXSUB];  // m_bigramFlags[x]
  float tfw[MAXG];
  int32_t qpos[MAXG], wiki[MAXG], quote[MAXG];
  int32_t qterm[MAXG];  // m_qtermNum (the second pass's score info)
  int32_t sortby_group;  // gbsortby: the group whose first key's number is the score (-1: none)
  int32_t sortby_int;    // ... read as int32: the TopTree orders by m_intScore (TopTree.cpp:216-219, 270-274)
  // candidate arrays (sublists of m_minListi, distinct lists, in order)
  int g0n;
  int g0list[MAXG0];
  uint64_t g0base[MAXG0 + 1];  // slot base of each array (prefix of upper bounds)
  // per candidate array, a docid-bucket directory: entry (epoch << 32 | i)
  // at bucket (docid - g0dmin) >> g0sh names SOME candidate i of that bucket
  // (k_write_runs); entries of older queries carry an older epoch
  uint32_t epoch;
  uint32_t g0sh[MAXG0];
  uint64_t g0dmin[MAXG0], g0dmax[MAXG0];
  uint64_t g0dir[MAXG0];       // first entry of each array's directory
  uint32_t probed_mask;        // bit l: k_probe scans list l (its matches are bitmap bits)
  uint32_t group_lists[MAXG];  // bit l: list l is a sublist of group g
  uint32_t neg_lists;          // bit l: list l is a sublist of a negative group
  uint8_t list_mult[MAXL];     // positive groups list l is a sublist of (its runs' record copies)
  // boolean queries (makeDocIdVoteBufForBoolQuery_r, Posdb.cpp:8006-8249):
  // every distinct list is a candidate array (their union is the docid set),
  // a docid's QueryTermInfo bit vector is the OR of its lists' group masks,
  // and it survives where the truth table has that vector's bit
  int boolean;
  uint16_t bool_gmask[MAXL];   // bit g: list l is a sublist of group g (negative groups too)
  const uint8_t *bool_table;   // 2^ngroups bits (the staging buffer's tail)
  uint64_t dbg_doc;            // diagnostic (GBGPU_PROBE_DEBUG_DOC): k_probe traces this docid's runs
  unsigned long long *dbg_buf; // into this buffer: a count, then 16-word records
  DevList lists[MAXL];
  // run-driven probe work (PROBE_BY_RUN lists) without a per-wave table:
  // wave nwork_cand + i scans run_span units of list rseg_list[s], the
  // segment s with rseg_wbase[s] <= i < rseg_wbase[s + 1], from unit
  // (i - rseg_wbase[s]) * run_span; the candidate-driven waves come first
  // and read the staged ProbeWork array
  uint32_t nwork_cand;
  uint32_t nrseg;
  uint32_t run_span;
  uint32_t rseg_list[MAXL];
  uint32_t rseg_wbase[MAXL + 1];
};

// setQueryTermInfo + minListi; returns 0 or error.
int build_host_plan(const gbgpu_qterm *terms, int nterms, const int64_t *sizes,
                    const gbgpu_params *p, HostPlan *hp);
int32_t docs_wanted(const gbgpu_params *p, const int64_t *sizes, int nterms);
// TopTree::setNumNodes (TopTree.cpp:64-101): node count of a tree of
// docs_wanted entries (docs_wanted+1 without site clustering)
int64_t tree_nodes(int32_t docs_wanted, bool site_clustering);

}  // namespace gbgpu

#endif
