/* TEST INFRASTRUCTURE ONLY (see posdb_oracle.h).
 *
 * Restatement of Msg3a::mergeLists (Msg3a.cpp:971-1503) without site
 * clustering or facets: the k-way merge of the shards' Msg39 replies
 * (docids + double scores, each as Msg39 sends it, Msg39.cpp:1633-1684).
 * Pinned against the reference's own Msg3a::mergeLists driven by
 * oracle/_ref/gbref (tests/golden/x_*.npz).
 */
#include "posdb_oracle.h"

#include <errno.h>
#include <stdlib.h>

int32_t orc_msg3a_merge(const int64_t *const *docids, const double *const *scores, const int32_t *counts,
                        int nshards, int32_t docs_to_get, int64_t *out_docids, double *out_scores) {
  if (nshards < 0 || docs_to_get <= 0) return -EINVAL;
  /* nd = min(docsToGet, sum of reply counts), Msg3a.cpp:1261-1270 */
  int64_t nd2 = 0;
  for (int j = 0; j < nshards; j++) nd2 += counts[j];
  const int64_t nd = nd2 < docs_to_get ? nd2 : docs_to_get;
  int32_t *cur = (int32_t *)calloc(nshards ? nshards : 1, sizeof(int32_t));
  /* htable (Msg3a.cpp:1299-1301, 1381-1385, 1459): every docid taken or
   * passed over while the merge runs; a linear list suffices here */
  int64_t *seen = (int64_t *)malloc(sizeof(int64_t) * (size_t)(nd2 ? nd2 : 1));
  int64_t nseen = 0;
  int32_t n = 0;
  if (!cur || !seen) {
    free(cur);
    free(seen);
    return -ENOMEM;
  }
  (void)nd;
  for (;;) {
    /* mergeLoop, Msg3a.cpp:1315-1339: the first shard wins unless a later
     * head has a higher score, or an equal score and a lower docid */
    int maxj = -1;
    for (int j = 0; j < nshards; j++) {
      if (cur[j] >= counts[j]) continue;
      if (maxj == -1) { maxj = j; continue; }
      const double sj = scores[j][cur[j]], sm = scores[maxj][cur[maxj]];
      if (sj < sm) continue;
      if (sj > sm) { maxj = j; continue; }
      if (docids[j][cur[j]] < docids[maxj][cur[maxj]]) { maxj = j; continue; }
    }
    if (maxj == -1) break;
    const int64_t d = docids[maxj][cur[maxj]];
    int dup = 0;
    for (int64_t i = 0; i < nseen; i++)
      if (seen[i] == d) { dup = 1; break; }
    if (!dup) {
      if (n < docs_to_get) {
        out_docids[n] = d;
        out_scores[n] = scores[maxj][cur[maxj]];
        n++;
      }
      seen[nseen++] = d;
    }
    cur[maxj]++;  /* skip: the shard's cursor moves on (Msg3a.cpp:1461-1465) */
    if (n >= docs_to_get) break;
  }
  free(cur);
  free(seen);
  return n;
}

/* ---- Msg3a::mergeLists whole: cluster records and facet lists ---------- */
#include <string.h>

/* Clusterdb.h:113-121 on a 12-byte key_t (n0 at 0, n1 at 8) */
static uint64_t rec_n0(const uint8_t *r) { uint64_t v; memcpy(&v, r, 8); return v; }
static uint32_t rec_n1(const uint8_t *r) { uint32_t v; memcpy(&v, r + 8, 4); return v; }

static int fe_cmp(const void *a, const void *b) {
  const orc_facet_entry *x = (const orc_facet_entry *)a, *y = (const orc_facet_entry *)b;
  if (x->term != y->term) return x->term < y->term ? -1 : 1;
  if (x->key != y->key) return x->key < y->key ? -1 : 1;
  return 0;
}

int orc_msg3a_full(const orc_merge_req *rq, const orc_reply *rep, int nshards, int64_t *out_docids,
                   double *out_scores, uint8_t *out_recs, int32_t *out_n, int64_t *out_hits, int64_t *out_fdocs,
                   orc_facet_entry *facets, int32_t facets_cap, int32_t *n_facets) {
  if (!rq || nshards < 0 || rq->docs_to_get <= 0 || rq->nqt < 0 || !out_n) return EINVAL;
  const int32_t nqt = rq->nqt;
  int64_t tot = 0, hits = 0;
  for (int j = 0; j < nshards; j++) {
    /* gotAllShardReplies: m_nqt must be the query's (Msg3a.cpp:755-761) */
    if (rep[j].n < 0 || rep[j].nqt != nqt) return EINVAL;
    /* with clustering mergeLists reads every head's record (1342-1347) */
    if (rq->site_clustering && rep[j].n > 0 && !rep[j].cluster_recs) return EINVAL;
    tot += rep[j].n;
    hits += rep[j].hits; /* 792 */
  }
  if (out_hits) *out_hits = hits;
  /* 794-802: every term's m_numDocsThatHaveFacet, summed */
  for (int k = 0; k < nqt; k++) {
    int64_t c = 0;
    for (int j = 0; j < nshards; j++)
      if (rep[j].facet_docs) c += rep[j].facet_docs[k];
    if (out_fdocs) out_fdocs[k] = c;
  }
  /* 1129-1240: each reply's facet lists into the terms' tables, reply by
   * reply, entry by entry (the table here: a list searched linearly) */
  int64_t cap = 1;
  for (int j = 0; j < nshards; j++) cap += rep[j].facet_list_size / 36 + 1;
  orc_facet_entry *tab = (orc_facet_entry *)calloc((size_t)cap, sizeof(orc_facet_entry));
  int64_t nt = 0;
  if (!tab) return ENOMEM;
  int stop = 0;
  for (int j = 0; j < nshards && !stop; j++) {
    const uint8_t *p = rep[j].facet_list, *last = p + (p ? rep[j].facet_list_size : 0);
    if (!p) continue;
    while (p < last) {
      int64_t tid;
      int32_t nh;
      if (last - p < 12) { free(tab); return ENODATA; }
      memcpy(&tid, p, 8);
      memcpy(&nh, p + 8, 4);
      p += 12;
      /* getQueryTermByTermId64 (Query.h:883-889): the first term with it */
      int term = -1;
      for (int i = 0; i < nqt; i++)
        if (rq->term_ids[i] == tid) { term = i; break; }
      /* 1157-1162: `break` leaves the loop over the replies: this reply's
       * later lists and every later reply's are not merged */
      if (term < 0) { stop = 1; break; }
      if (nh < 0 || (int64_t)nh * 36 > last - p) { free(tab); return ENODATA; }
      const int isfloat = rq->field_codes[term] == 65, isint = rq->field_codes[term] == 64;
      for (int32_t e = 0; e < nh; e++, p += 36) {
        orc_facet_entry fe;
        fe.term = term;
        memcpy(&fe.key, p, 4);
        memcpy(&fe.count, p + 4, 4);
        memcpy(&fe.outside, p + 8, 4);
        memcpy(&fe.docid, p + 12, 8);
        memcpy(&fe.sum, p + 20, 8);
        memcpy(&fe.max, p + 28, 4);
        memcpy(&fe.min, p + 32, 4);
        orc_facet_entry *f2 = NULL;
        for (int64_t t = 0; t < nt; t++)
          if (tab[t].term == term && tab[t].key == fe.key) { f2 = &tab[t]; break; }
        if (!f2) { tab[nt++] = fe; continue; } /* addKey (1190-1193) */
        if (isfloat) { /* 1197-1213 */
          double s1, s2;
          float mn1, mn2, mx1, mx2;
          memcpy(&s1, &fe.sum, 8);
          memcpy(&s2, &f2->sum, 8);
          s2 += s1;
          memcpy(&f2->sum, &s2, 8);
          memcpy(&mn1, &fe.min, 4);
          memcpy(&mn2, &f2->min, 4);
          if (f2->count == 0 || (fe.count != 0 && mn1 < mn2)) mn2 = mn1;
          memcpy(&f2->min, &mn2, 4);
          memcpy(&mx1, &fe.max, 4);
          memcpy(&mx2, &f2->max, 4);
          if (f2->count == 0 || (fe.count != 0 && mx1 > mx2)) mx2 = mx1;
          memcpy(&f2->max, &mx2, 4);
        }
        if (isint) { /* 1214-1220 */
          f2->sum = (int64_t)((uint64_t)f2->sum + (uint64_t)fe.sum);
          if (f2->count == 0 || (fe.count != 0 && fe.min < f2->min)) f2->min = fe.min;
          if (f2->count == 0 || (fe.count != 0 && fe.max > f2->max)) f2->max = fe.max;
        }
        f2->count = (int32_t)((uint32_t)f2->count + (uint32_t)fe.count);
        f2->outside = (int32_t)((uint32_t)f2->outside + (uint32_t)fe.outside);
        /* 1232-1233: m_docId = either entry's at random; the first kept here */
      }
    }
  }
  qsort(tab, (size_t)nt, sizeof *tab, fe_cmp);
  if (n_facets) *n_facets = (int32_t)nt;
  if (facets && nt > facets_cap) { free(tab); return ENOSPC; }
  if (facets) memcpy(facets, tab, sizeof *tab * (size_t)nt);
  free(tab);
  /* 1315-1467: the merge loop, the site cap before the docid test */
  int32_t *cur = (int32_t *)calloc(nshards ? nshards : 1, sizeof(int32_t));
  int64_t *seen = (int64_t *)malloc(sizeof(int64_t) * (size_t)(tot + 1));
  uint32_t *site = (uint32_t *)malloc(sizeof(uint32_t) * (size_t)(tot + 1));
  int32_t *scnt = (int32_t *)malloc(sizeof(int32_t) * (size_t)(tot + 1));
  int64_t nseen = 0, nsite = 0;
  int32_t n = 0;
  if (!cur || !seen || !site || !scnt) {
    free(cur); free(seen); free(site); free(scnt);
    return ENOMEM;
  }
  while (n < rq->docs_to_get) {
    int maxj = -1;
    for (int j = 0; j < nshards; j++) {
      if (cur[j] >= rep[j].n) continue;
      if (maxj == -1) { maxj = j; continue; }
      const double sj = rep[j].scores[cur[j]], sm = rep[maxj].scores[cur[maxj]];
      if (sj < sm) continue;
      if (sj > sm) { maxj = j; continue; }
      if (rep[j].docids[cur[j]] < rep[maxj].docids[cur[maxj]]) { maxj = j; continue; }
    }
    if (maxj == -1) break;
    const int64_t d = rep[maxj].docids[cur[maxj]];
    const uint8_t *rec = rq->site_clustering ? rep[maxj].cluster_recs + 12 * (size_t)cur[maxj] : NULL;
    cur[maxj]++;
    if (rec && rec_n0(rec) != 0 && rec_n1(rec) != 0) {
      if (rq->family_filter && ((rec_n0(rec) >> 34) & 1)) continue;
      const uint32_t sh = (uint32_t)(rec_n0(rec) >> 2) & 0x03FFFFFF;
      int64_t s = -1;
      for (int64_t t = 0; t < nsite; t++)
        if (site[t] == sh) { s = t; break; }
      if (s >= 0) {
        if (sh && scnt[s] >= 2) continue;
        if (sh && scnt[s] >= 1 && rq->hide_all_clustered) continue;
        scnt[s]++;
      } else {
        site[nsite] = sh;
        scnt[nsite++] = 1;
      }
    }
    int dup = 0;
    for (int64_t t = 0; t < nseen; t++)
      if (seen[t] == d) { dup = 1; break; }
    if (dup) continue;
    out_docids[n] = d;
    out_scores[n] = rep[maxj].scores[cur[maxj] - 1];
    if (rq->site_clustering && out_recs) memcpy(out_recs + 12 * (size_t)n, rec, 12);
    n++;
    seen[nseen++] = d;
  }
  free(cur); free(seen); free(site); free(scnt);
  *out_n = n;
  return 0;
}
