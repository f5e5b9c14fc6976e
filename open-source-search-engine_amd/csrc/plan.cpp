// Host restatement of PosdbTable::setQueryTermInfo (Posdb.cpp:4354-4869) and
// PosdbTable::allocTopTree's TopTree sizing (Posdb.cpp:838-930).  Runs on the
// caller's INTERSECT thread before any device work, like the reference.
#include "plan.h"

#include <cerrno>
#include <cstring>

namespace gbgpu {

int32_t docs_wanted(const gbgpu_params *p, const int64_t *sizes, int nterms) {
  int64_t nn1 = p->docs_to_get, nn2 = 0;
  for (int k = 0; k < nterms; k++) {
    if (sizes[k] <= 0) continue;                    // empty list
    nn2 += (int64_t)(int32_t)sizes[k] / (18 - 6);   // m_listSize / (sizeof(POSDBKEY)-6)
  }
  if (p->num_docid_splits > 1) {      // Posdb.cpp:859-877 (sizes: the first piece's lists)
    if (nn2 < 100) nn2 = 100;
    nn2 *= p->num_docid_splits;
    nn2 *= 2;
    if (nn1 < 100) nn1 = 100;
    nn1 *= p->num_docid_splits;
    nn1 *= 2;
  }
  int64_t nn = nn2;
  if (nn1 < nn2) nn = nn1;
  if (nn == 0) return 0;              // no tree allocated
  if (nn < 30) nn = 30;               // Posdb.cpp:897
  if (p->site_clustering) nn *= 2;    // Posdb.cpp:900
  if (nn > 2000000000) nn = 2000000000;
  if (nn > (int64_t)p->docs_to_get * 2 && nn > 60) nn = (int64_t)p->docs_to_get * 2;
  return (int32_t)nn;                 // TopTree::setNumNodes -> m_docsWanted
}

int64_t tree_nodes(int32_t dw, bool site_clustering) {
  if (!site_clustering) return (int64_t)dw + 1;  // TopTree.cpp:88
  int64_t rmax = (int64_t)dw * 2;                // m_ridiculousMax, TopTree.cpp:76-77
  if (rmax < 50) rmax = 50;
  int64_t n = rmax * 256;
  if (n > 2000000000LL) n = 2000000000LL;        // MAXDOCIDSTOCOMPUTE (Msg40.h:25)
  return n;
}

int build_host_plan(const gbgpu_qterm *qt, int nqt, const int64_t *sizes, const gbgpu_params *p,
                    HostPlan *hp) {
  hp->nqt = nqt;
  hp->ngroups = 0;
  hp->min_listi = -1;
  hp->min_list_size = 0;
  hp->real_max_top = p->real_max_top > 10 ? 10 : p->real_max_top;
  hp->sortby_group = -1;
  hp->sortby_int = 0;
  int nrg = 0;
  for (int i = 0; i < nqt; i++) {
    if (!qt[i].is_required) continue;
    if (nrg >= (int)(sizeof(hp->g) / sizeof(hp->g[0]))) return GBGPU_EUNSUPPORTED;
    GroupInfo &g = hp->g[nrg];
    std::memset(&g, 0, sizeof g);
    g.qterm = i;
    g.qpos = qt[i].qpos;
    g.wiki = qt[i].wiki_phrase_id;
    g.quote = qt[i].quote_start;
    int nn = 0;
    const int left = qt[i].left_phrase_term, right = qt[i].right_phrase_term;
    const uint8_t piped = qt[i].piped ? BF_PIPED : 0;
    bool leftAdded = false, rightAdded = false;
    // m_subLists[nn] / m_bigramFlags[nn] are written even when the list is
    // empty; nn only advances for non-empty lists (Posdb.cpp:4487 etc.)
    auto add = [&](int term, uint8_t fl) -> bool {
      if (nn >= REF_MAX_SUBLISTS) return false;
      g.sub_term[nn] = term;
      g.flags[nn] = fl;
      if (sizes[term] > 0) nn++;
      return true;
    };
    bool ok = true;
    if (left >= 0 && qt[left].is_wiki_half_stop_bigram) {
      leftAdded = true;
      ok &= add(left, BF_HALFSTOPWIKIBIGRAM | piped);
      for (int k = 0; k < nqt; k++)
        if (qt[k].synonym_of == left) ok &= add(k, BF_HALFSTOPWIKIBIGRAM | BF_SYNONYM | piped);
    }
    if (right >= 0 && qt[right].is_wiki_half_stop_bigram) {
      rightAdded = true;
      ok &= add(right, BF_HALFSTOPWIKIBIGRAM | piped);
      for (int k = 0; k < nqt; k++)
        if (qt[k].synonym_of == right) ok &= add(k, BF_HALFSTOPWIKIBIGRAM | BF_SYNONYM | piped);
    }
    // numeric term lists carry a float where the word position is
    // (Posdb.cpp:4572-4577); gbsortby: scores by it (4413-4417, 7265-7269)
    const bool sortbyf = qt[i].field_code == FIELD_GBSORTBYFLOAT || qt[i].field_code == FIELD_GBREVSORTBYFLOAT;
    const bool sortbyi = qt[i].field_code == FIELD_GBSORTBYINT || qt[i].field_code == FIELD_GBREVSORTBYINT;
    const bool sortby = sortbyf || sortbyi;
    int rint;
    const bool number = sortby || range_mode(qt[i].field_code, &rint) != 0;
    // the last sortby term wins; the int form also switches the tree
    // (m_sortByTermNum and m_sortByTermNumInt are separate in the reference:
    // with both, the float sets `score` and the int the tree -- not emulated)
    if (sortby) {
      if (hp->sortby_group >= 0 && hp->sortby_int != (int)sortbyi) return GBGPU_EUNSUPPORTED;
      hp->sortby_group = nrg;
      hp->sortby_int = sortbyi;
    }
    const bool facet = qt[i].field_code >= FIELD_GBFACETSTR && qt[i].field_code <= FIELD_GBFACETFLOAT;
    ok &= add(i, (uint8_t)(piped | (qt[i].term_sign == '-' ? BF_NEGATIVE : 0) | (number ? BF_NUMBER : 0) |
                           (facet ? BF_FACET : 0)));  // Posdb.cpp:4572-4602
    if (left >= 0 && !leftAdded) {
      ok &= add(left, piped | BF_BIGRAM);
      for (int k = 0; k < nqt; k++)
        if (qt[k].synonym_of == left) ok &= add(k, BF_SYNONYM | piped);
    }
    if (right >= 0 && !rightAdded) {
      ok &= add(right, BF_BIGRAM | piped);
      for (int k = 0; k < nqt; k++)
        if (qt[k].synonym_of == right) ok &= add(k, BF_SYNONYM | piped);
    }
    for (int k = 0; k < nqt; k++)
      if (qt[k].synonym_of == i) ok &= add(k, BF_SYNONYM | piped);
    if (!ok || nn >= REF_MAX_SUBLISTS) return E2BIG;  // "too many sublists"
    g.nsub = nn;
    g.tfw = qt[i].tf_weight;
    g.total = 0;
    for (int q = 0; q < nn; q++) g.total += sizes[g.sub_term[q]];
    nrg++;
  }
  hp->ngroups = nrg;
  for (int i = 0; i < nrg; i++) {
    if (hp->g[i].flags[0] & BF_NEGATIVE) continue;
    int64_t total = hp->g[i].total;
    if (total < hp->min_list_size || hp->min_listi == -1) {
      hp->min_list_size = total;
      hp->min_listi = i;
    }
  }
  hp->docs_wanted = docs_wanted(p, sizes, nqt);
  return 0;
}

}  // namespace gbgpu
