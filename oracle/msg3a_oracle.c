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
