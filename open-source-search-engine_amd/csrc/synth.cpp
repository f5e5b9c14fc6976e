// Synthetic Zipfian posdb corpus generator.
//
// Everything about a (doc, term) pair is a pure function of (seed, doc index,
// termId), so any docid-range shard of a corpus can be generated on its own
// rank and concatenated shards equal the whole-corpus lists.  Lists are
// encoded with the posdb append compression of RdbList::addRecord
// (RdbList.cpp:282-327).
#include "../../include/gbgpu_synth.h"
#include "posdb_key.h"

#include <algorithm>
#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

namespace {

inline uint64_t mix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ULL;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}
inline uint64_t H(uint64_t seed, uint64_t a, uint64_t b, uint64_t c = 0) {
  return mix64(seed ^ mix64(a ^ mix64(b ^ mix64(c + 0x632be59bd9b4e019ULL))));
}
inline double U01(uint64_t h) { return (double)(h >> 11) * (1.0 / 9007199254740992.0); }

struct Ctx {
  const gb_synth_corpus *c;
  const gb_synth_term *t;
  int nt;
  uint64_t stride;
};

struct Key {  // decoded posting, one position of one (doc, term)
  uint32_t pos, hg, dens, wsr, syn;
};

// hash-group mix: body .80, title .05, heading .04, inlist .03,
// inlinktext .04, inurl .02, meta .02
inline uint32_t pick_hashgroup(double u) {
  if (u < 0.80) return GB_HG_BODY;
  if (u < 0.85) return GB_HG_TITLE;
  if (u < 0.89) return GB_HG_HEADING;
  if (u < 0.92) return GB_HG_INLIST;
  if (u < 0.96) return GB_HG_INLINKTEXT;
  if (u < 0.98) return GB_HG_INURL;
  return GB_HG_INMETATAG;
}

bool has_term(const Ctx &x, int j, int64_t i) {
  const gb_synth_term &t = x.t[j];
  double u = U01(H(x.c->seed, (uint64_t)i, t.term_id, 1));
  if (t.kind == GB_SYNTH_BIGRAM) {
    if (t.a < 0 || t.b < 0) return false;
    if (!has_term(x, t.a, i) || !has_term(x, t.b, i)) return false;
  }
  return u < t.p;
}

// positions/attributes of term j in doc i (assumes has_term)
void term_keys(const Ctx &x, int j, int64_t i, std::vector<Key> &out) {
  const gb_synth_term &t = x.t[j];
  const uint64_t s = x.c->seed;
  out.clear();
  uint32_t syn = 0;
  if (t.syn_frac_pct > 0 && (H(s, (uint64_t)i, t.term_id, 7) % 100) < (uint64_t)t.syn_frac_pct) syn = 1;
  if (t.kind == GB_SYNTH_BIGRAM) {
    std::vector<Key> base;
    bool aligned = false;
    if (t.align_to >= 0 && has_term(x, t.align_to, i) && U01(H(s, (uint64_t)i, t.term_id, 8)) < 0.7) {
      term_keys(x, t.align_to, i, base);
      for (auto &k : base) k.pos += 2;
      aligned = true;
    } else {
      term_keys(x, t.a, i, base);
    }
    // keep a geometric prefix of the component's positions
    uint32_t n = 1;
    uint64_t g = H(s, (uint64_t)i, t.term_id, 9);
    while ((g & 1) && n < base.size()) { n++; g >>= 1; }
    if (aligned) n = (uint32_t)base.size();
    for (uint32_t k = 0; k < n && k < base.size(); k++) {
      Key kk = base[k];
      if (kk.pos > GB_MAXWORDPOS) continue;
      kk.syn = syn;
      kk.dens = (uint32_t)(H(s, (uint64_t)i, t.term_id, 100 + k) % 32);
      out.push_back(kk);
    }
    return;
  }
  // P = 1 + Geometric(0.5), truncated
  uint32_t P = 1;
  uint64_t g = H(s, (uint64_t)i, t.term_id, 2);
  uint32_t maxp = x.c->max_positions > 0 ? (uint32_t)x.c->max_positions : 64;
  while ((g & 1) && P < maxp) {
    P++;
    g >>= 1;
    if (P % 60 == 0) g = H(s, (uint64_t)i, t.term_id, 3 + P);
  }
  uint32_t pos = (uint32_t)(H(s, (uint64_t)i, t.term_id, 4) % 1024);
  for (uint32_t k = 0; k < P; k++) {
    uint64_t h = H(s, (uint64_t)i, t.term_id, 1000 + k);
    Key kk;
    if (k) pos += 2 + (uint32_t)(h % 39);  // gaps U[2,40]
    if (pos > GB_MAXWORDPOS) break;
    kk.pos = pos;
    kk.hg = pick_hashgroup(U01(mix64(h ^ 0x1111)));
    kk.dens = (uint32_t)((h >> 20) % 32);
    uint64_t h2 = mix64(h ^ 0x2222);
    kk.wsr = (U01(h2) < 0.8) ? 15u : (uint32_t)((h2 >> 40) % 16);
    kk.syn = syn;
    out.push_back(kk);
  }
}

// One thread: docs [i0, i1).  Emits each term's keys as "continuation"
// encoding: every docid run opens with a 12-byte key (termid factored out).
void gen_range(const Ctx &x, int64_t i0, int64_t i1, std::vector<std::vector<uint8_t>> &out) {
  out.assign(x.nt, {});
  std::vector<Key> keys;
  uint8_t k18[18];
  const uint64_t s = x.c->seed;
  for (int64_t i = i0; i < i1; i++) {
    uint64_t docid = (uint64_t)i * x.stride + H(s, (uint64_t)i, 0, 5) % x.stride;
    uint32_t siteRank = (uint32_t)(H(s, (uint64_t)i, 0, 6) % 16);
    uint64_t hl = H(s, (uint64_t)i, 0, 7);
    uint32_t langId = (U01(hl) < 0.9) ? 1u : (uint32_t)((hl >> 40) % 64);
    for (int j = 0; j < x.nt; j++) {
      if (!has_term(x, j, i)) continue;
      term_keys(x, j, i, keys);
      if (keys.empty()) continue;
      // keys sort by (wordPos, hg, ...) within a docid; positions are distinct
      std::sort(keys.begin(), keys.end(), [](const Key &a, const Key &b) {
        if (a.pos != b.pos) return a.pos < b.pos;
        return a.hg < b.hg;
      });
      auto &buf = out[j];
      bool first = true;
      uint32_t lastpos = 0xffffffffu;
      for (auto &k : keys) {
        if (k.pos == lastpos) continue;
        lastpos = k.pos;
        gb_make_key(k18, x.t[j].term_id, docid, k.pos, k.dens, 15, k.wsr, siteRank, k.hg, langId,
                    0, k.syn, 0, 0);
        if (first) {
          k18[0] |= 0x02;
          buf.insert(buf.end(), k18, k18 + 12);
          first = false;
        } else {
          k18[0] |= 0x06;
          buf.insert(buf.end(), k18, k18 + 6);
        }
      }
    }
  }
}

}  // namespace

extern "C" uint64_t gb_synth_docid(const gb_synth_corpus *c, int64_t i) {
  uint64_t stride = (1ULL << 38) / (uint64_t)c->num_docs;
  if (stride == 0) stride = 1;
  return (uint64_t)i * stride + H(c->seed, (uint64_t)i, 0, 5) % stride;
}

extern "C" int gb_synth_lists(const gb_synth_corpus *c, const gb_synth_term *terms, int nterms,
                              uint8_t **out_bufs, int64_t *out_sizes) {
  if (!c || !terms || nterms <= 0 || c->num_docs <= 0 || c->num_docs > (1LL << 38)) return EINVAL;
  Ctx x{c, terms, nterms, (1ULL << 38) / (uint64_t)c->num_docs};
  int64_t i0 = c->doc_begin < 0 ? 0 : c->doc_begin;
  int64_t i1 = (c->doc_end <= 0 || c->doc_end > c->num_docs) ? c->num_docs : c->doc_end;
  if (i1 < i0) i1 = i0;
  int nth = c->num_threads > 0 ? c->num_threads : (int)std::thread::hardware_concurrency();
  if (nth < 1) nth = 1;
  if ((i1 - i0) < 100000) nth = 1;
  std::vector<std::vector<std::vector<uint8_t>>> parts(nth);
  std::vector<std::thread> th;
  for (int t = 0; t < nth; t++) {
    int64_t a = i0 + (i1 - i0) * t / nth, b = i0 + (i1 - i0) * (t + 1) / nth;
    th.emplace_back([&, t, a, b] { gen_range(x, a, b, parts[t]); });
  }
  for (auto &t : th) t.join();
  for (int j = 0; j < nterms; j++) {
    int64_t tot = 0;
    for (int t = 0; t < nth; t++) tot += (int64_t)parts[t][j].size();
    out_bufs[j] = nullptr;
    out_sizes[j] = 0;
    if (tot == 0) continue;
    uint8_t *p = (uint8_t *)std::malloc((size_t)tot + 6);
    if (!p) return ENOMEM;
    int64_t off = 0;
    bool first = true;
    for (int t = 0; t < nth; t++) {
      auto &v = parts[t][j];
      if (v.empty()) continue;
      if (first) {
        // the list's first key carries the termid: 12 -> 18 bytes
        std::memcpy(p, v.data(), 12);
        p[0] &= (uint8_t)~0x06;
        uint64_t tid = terms[j].term_id & GB_TERMID_MASK;
        // n2 bytes 10-11 hold docid hi bits (already in the 12 bytes); 12-17 termid
        for (int b = 0; b < 6; b++) p[12 + b] = (uint8_t)(tid >> (8 * b));
        std::memcpy(p + 18, v.data() + 12, v.size() - 12);
        off = 18 + (int64_t)v.size() - 12;
        first = false;
      } else {
        std::memcpy(p + off, v.data(), v.size());
        off += (int64_t)v.size();
      }
      std::vector<uint8_t>().swap(v);
    }
    out_bufs[j] = p;
    out_sizes[j] = off;
  }
  return 0;
}

extern "C" void gb_synth_free(void *p) { std::free(p); }

// ------------------------------------------------ tiered runs (config 5)
namespace {

struct Rng {  // splitmix64 stream
  uint64_t s;
  uint64_t next() { return mix64(s += 0x9e3779b97f4a7c15ULL); }
  double u() { return U01(next()); }
};

// RdbList::addRecord compression (RdbList.cpp:282-327) into one run
struct RunOut {
  std::vector<uint8_t> b;
  uint8_t hi[6], lo[6];
  bool any = false;
  void add(const uint8_t *k) {
    if (any && std::memcmp(hi, k + 12, 6) == 0) {
      if (std::memcmp(lo, k + 6, 6) == 0) {
        b.insert(b.end(), k, k + 6);
        b[b.size() - 6] = (uint8_t)((k[0] & 0xf9) | 0x06);
        return;
      }
      b.insert(b.end(), k, k + 12);
      b[b.size() - 12] = (uint8_t)((k[0] & 0xf9) | 0x02);
      std::memcpy(lo, k + 6, 6);
      return;
    }
    b.insert(b.end(), k, k + 18);
    b[b.size() - 18] = (uint8_t)(k[0] & 0xf9);
    std::memcpy(lo, k + 6, 6);
    std::memcpy(hi, k + 12, 6);
    any = true;
  }
};

}  // namespace

extern "C" int gb_synth_merge_runs(int64_t total_keys, int nruns, uint64_t seed, double dup_frac, double neg_frac,
                                   int nterms, int nthreads, uint8_t **out_bufs, int64_t *out_sizes) {
  if (total_keys < 0 || nruns < 1 || nruns > 30 || nterms < 1 || !out_bufs || !out_sizes) return EINVAL;
  // termids sorted; Zipf weight by a random rank, so key counts are not
  // correlated with termid order
  std::vector<uint64_t> tid(nterms);
  std::vector<double> w(nterms);
  for (int j = 0; j < nterms; j++) tid[j] = (H(seed, (uint64_t)j, 11) & GB_TERMID_MASK) | 1;
  std::sort(tid.begin(), tid.end());
  std::vector<int> rank(nterms);
  for (int j = 0; j < nterms; j++) rank[j] = j;
  for (int j = nterms - 1; j > 0; j--) std::swap(rank[j], rank[H(seed, (uint64_t)j, 12) % (uint64_t)(j + 1)]);
  double ws = 0;
  for (int j = 0; j < nterms; j++) ws += (w[j] = 1.0 / (1.0 + rank[j]));
  std::vector<int64_t> cnt(nterms);
  for (int j = 0; j < nterms; j++) cnt[j] = (int64_t)((double)total_keys * w[j] / ws);
  // run r gets 2^r / (2^nruns - 1) of the keys
  std::vector<double> cum(nruns);
  double acc = 0, tw = (double)((1ULL << nruns) - 1);
  for (int r = 0; r < nruns; r++) cum[r] = (acc += (double)(1ULL << r) / tw);
  int nth = nthreads > 0 ? nthreads : (int)std::thread::hardware_concurrency();
  nth = std::max(1, std::min(nth, nterms));
  // contiguous term ranges of about equal key counts
  std::vector<int> cut(nth + 1, nterms);
  cut[0] = 0;
  {
    int64_t tot = 0, run = 0;
    for (auto c : cnt) tot += c;
    int t = 1;
    for (int j = 0; j < nterms && t < nth; j++) {
      run += cnt[j];
      while (t < nth && run >= tot * t / nth) cut[t++] = j + 1;
    }
  }
  std::vector<std::vector<RunOut>> parts(nth, std::vector<RunOut>(nruns));
  std::vector<std::thread> th;
  for (int t = 0; t < nth; t++) {
    th.emplace_back([&, t] {
      auto &R = parts[t];
      uint8_t k[18];
      for (int j = cut[t]; j < cut[t + 1]; j++) {
        Rng g{H(seed, (uint64_t)j, 13)};
        const int64_t want = cnt[j];
        if (want <= 0) continue;
        // ~1+Geometric(0.5) positions per doc: docs = want/2, sorted by
        // uniform gaps over the 38-bit docid space
        const uint64_t ndoc = std::max<int64_t>(1, want / 2);
        const uint64_t gap = std::max<uint64_t>(1, ((1ULL << 38) - 1) / ndoc * 2);
        uint64_t docid = 0;
        int64_t made = 0;
        while (made < want) {
          docid += 1 + g.next() % gap;
          if (docid >= (1ULL << 38)) break;
          const uint32_t sr = (uint32_t)(g.next() % 16);
          const uint32_t lang = g.u() < 0.9 ? 1u : (uint32_t)(g.next() % 64);
          int P = 1;
          while (P < 64 && g.u() < 0.5) P++;
          uint32_t pos = (uint32_t)(g.next() % (GB_MAXWORDPOS - 64 * 40));
          for (int q = 0; q < P && made < want; q++, made++) {
            pos += 2 + (uint32_t)(g.next() % 39);
            const double uh = g.u();
            const uint32_t hg = pick_hashgroup(uh);
            const uint32_t dens = (uint32_t)(g.next() % 32);
            const uint32_t spam = g.u() < 0.8 ? 15u : (uint32_t)(g.next() % 16);
            const int syn = g.u() < 0.05;
            gb_make_key(k, tid[j], docid, pos, dens, 15, spam, sr, hg, lang, 0, syn, 0, 0);
            const double ur = g.u();
            int r = 0;
            while (r < nruns - 1 && ur >= cum[r]) r++;
            if (g.u() < neg_frac) k[0] &= 0xfe;  // delete key
            R[r].add(k);
            if (g.u() < dup_frac) {  // a copy in another run; its delete bit may flip
              int r2 = (int)(g.next() % (uint64_t)nruns);
              if (r2 == r) r2 = (r2 + 1) % nruns;
              if (nruns > 1) {
                uint8_t d[18];
                std::memcpy(d, k, 18);
                if (g.u() < 0.5) d[0] ^= 0x01;
                R[r2].add(d);
              }
            }
          }
        }
      }
    });
  }
  for (auto &x : th) x.join();
  for (int r = 0; r < nruns; r++) {
    int64_t tot = 0;
    for (int t = 0; t < nth; t++) tot += (int64_t)parts[t][r].b.size();
    out_bufs[r] = nullptr;
    out_sizes[r] = 0;
    if (!tot) continue;
    uint8_t *p = (uint8_t *)std::malloc((size_t)tot);
    if (!p) {
      for (int q = 0; q < r; q++) std::free(out_bufs[q]);
      return ENOMEM;
    }
    int64_t off = 0;
    for (int t = 0; t < nth; t++) {
      auto &v = parts[t][r].b;
      if (!v.empty()) std::memcpy(p + off, v.data(), v.size());
      off += (int64_t)v.size();
      std::vector<uint8_t>().swap(v);
    }
    out_bufs[r] = p;
    out_sizes[r] = off;
  }
  return 0;
}

extern "C" int64_t gb_posdb_compress(const uint8_t *keys, int64_t n, uint8_t *out) {
  int64_t o = 0;
  const uint8_t *hi = nullptr, *lo = nullptr;  // RdbList m_listPtrHi / m_listPtrLo
  for (int64_t i = 0; i < n; i++) {
    const uint8_t *k = keys + 18 * i;
    if (hi && std::memcmp(hi, k + 12, 6) == 0) {
      if (std::memcmp(lo, k + 6, 6) == 0) {
        std::memcpy(out + o, k, 6);
        out[o] |= 0x06;
        o += 6;
        continue;
      }
      std::memcpy(out + o, k, 12);
      lo = out + o + 6;
      out[o] |= 0x02;
      o += 12;
      continue;
    }
    std::memcpy(out + o, k, 18);
    lo = out + o + 6;
    hi = out + o + 12;
    o += 18;
  }
  return o;
}

extern "C" void gb_posdb_make_key(uint8_t *out, uint64_t termId, uint64_t docId, uint32_t wordPos,
                                  uint32_t densityRank, uint32_t diversityRank, uint32_t wordSpamRank,
                                  uint32_t siteRank, uint32_t hashGroup, uint32_t langId,
                                  uint32_t multiplier, int isSynonym, int isDelKey, int shardByTermId) {
  gb_make_key(out, termId, docId, wordPos, densityRank, diversityRank, wordSpamRank, siteRank,
              hashGroup, langId, multiplier, isSynonym, isDelKey, shardByTermId);
}
