/* Synthetic posdb corpus generator.
 *
 * Not part of the drop-in boundary: this is the bench/test data source.  It
 * produces compressed posdb termlists in exactly the byte format Msg2 hands
 * to PosdbTable (first key 18 bytes, then 12/6-byte keys; RdbList.cpp:282-327)
 * for a stratified-uniform docid universe, so that every docid-range shard of
 * a large corpus can be generated independently on its own rank.
 */
#ifndef GBGPU_SYNTH_H
#define GBGPU_SYNTH_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* corpus: N docs, docid(i) = i*S + h(i)%S with S = 2^38/N (sorted, distinct) */
typedef struct gb_synth_corpus {
  int64_t  num_docs;       /* N for the whole corpus                          */
  uint64_t seed;           /* 0x6B1A57 in the benchmark                       */
  int64_t  doc_begin;      /* generate docs [doc_begin, doc_end) only          */
  int64_t  doc_end;        /*   (a docid-range shard); doc_end<=0 -> N         */
  int32_t  max_positions;  /* P truncation, 64                                */
  int32_t  num_threads;    /* host threads, <=0 -> hardware concurrency        */
} gb_synth_corpus;

enum {
  GB_SYNTH_WORD    = 0,  /* independent term, membership prob p                   */
  GB_SYNTH_SYNONYM = 1,  /* like WORD, F bit (isSynonym) set for half its docs     */
  GB_SYNTH_BIGRAM  = 2   /* docs having terms a and b, then kept with prob p;      */
                         /* positions copied from term a (or align_to + 2)         */
};

typedef struct gb_synth_term {
  uint64_t term_id;      /* 48-bit termid                                          */
  double   p;            /* membership probability (df/N) or bigram keep prob      */
  int32_t  kind;         /* GB_SYNTH_*                                             */
  int32_t  a, b;         /* component term indices for BIGRAM, else -1             */
  int32_t  align_to;     /* BIGRAM: index of a bigram whose positions+2 we reuse   */
                         /*   for 70% of shared docs (quoted phrases), else -1     */
  int32_t  syn_frac_pct; /* % of docs whose keys carry the isSynonym F bit         */
} gb_synth_term;

/* Generate the lists of all `nterms` terms over the corpus shard.  On success
 * out_bufs[t] is a malloc'd buffer of out_sizes[t] bytes (NULL/0 if empty)
 * that the caller frees with gb_synth_free.  Returns 0 or an errno code. */
int  gb_synth_lists(const gb_synth_corpus *corpus, const gb_synth_term *terms, int nterms,
                    uint8_t **out_bufs, int64_t *out_sizes);
void gb_synth_free(void *p);

/* docid of document i of the corpus */
uint64_t gb_synth_docid(const gb_synth_corpus *corpus, int64_t i);

/* Config 5: nruns sorted, compressed posdb runs ("tiered
 * files", oldest first) of relative sizes 1:2:4:...; about total_keys keys
 * over nterms Zipf-weighted termids, ~1+Geometric(0.5) positions per
 * (term, doc); each key is a delete key with probability neg_frac and also
 * copied (delete bit flipped half the time) into another run with
 * probability dup_frac.  Deterministic for a seed, whatever nthreads.
 * out_bufs[r] are malloc'd (gb_synth_free). */
int gb_synth_merge_runs(int64_t total_keys, int nruns, uint64_t seed, double dup_frac, double neg_frac,
                        int nterms, int nthreads, uint8_t **out_bufs, int64_t *out_sizes);

/* RdbList::addRecord posdb compression of a sorted array of 18-byte keys
 * (RdbList.cpp:282-327).  out must hold 18*n bytes; returns bytes written. */
int64_t gb_posdb_compress(const uint8_t *keys18, int64_t n, uint8_t *out);

/* Posdb::makeKey (Posdb.cpp:374-460) */
void gb_posdb_make_key(uint8_t *out18, uint64_t termId, uint64_t docId, uint32_t wordPos,
                       uint32_t densityRank, uint32_t diversityRank, uint32_t wordSpamRank,
                       uint32_t siteRank, uint32_t hashGroup, uint32_t langId,
                       uint32_t multiplier, int isSynonym, int isDelKey, int shardByTermId);

#ifdef __cplusplus
}
#endif
#endif
