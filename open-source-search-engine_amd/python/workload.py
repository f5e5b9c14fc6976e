"""Query plans and synthetic corpora for the benchmark configs (BASELINE.json).

A query plan is the list of ``QTerm`` records ``Query::set2`` leaves in
``Query::m_qterms`` (Query.cpp:137-1965, shapes verified in SURVEY.md §8(d)):
words are required terms, adjacent-word bigrams are non-required terms linked
through ``m_leftPhraseTermNum``/``m_rightPhraseTermNum``, a quoted phrase of
n>=3 words becomes n-1 required bigram terms sharing ``m_quoteStart``, a
``-word`` is a required term with sign '-', and synonyms point back with
``m_synonymOf``.  Term-frequency weights follow getTermFreqWeight
(Posdb.cpp:1225-1252) on the synthetic document frequencies.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

import numpy as np

from gbgpu import (QTerm, Params, TermSpec, SYNTH_BIGRAM, SYNTH_SYNONYM, SYNTH_WORD, synth_lists)


def tf_weight(term_freq: float, num_docs: int) -> float:
    """getTermFreqWeight (Posdb.cpp:1225-1252), float arithmetic as written."""
    fw = np.float32(term_freq)
    if num_docs:
        fw = np.float32(fw / np.float32(num_docs))
    if fw > 0.50:
        fw = np.float32(0.50)
    return float(np.float32(0.50 + float(fw)))


@dataclass
class Word:
    name: str
    p: float                    # document frequency / N
    sign: int = 0               # ord('-') for a negative term
    piped: int = 0
    wiki: int = 0               # m_wikiPhraseId
    synonyms: Sequence[float] = ()   # membership probabilities of synonym terms


@dataclass
class Query:
    """A built query: plan terms + synthetic specs (1-1) + docs-to-get."""
    name: str
    terms: List[QTerm]
    specs: List[TermSpec]
    spec_of_term: List[int]
    docs_to_get: int = 100

    def params(self, real_max_top=10, language=0, same_lang_weight=20.0, site_clustering=0,
               num_docid_splits=1, max_serp_score=0.0, min_serp_docid=0) -> Params:
        """Msg39Request as reset() (Msg39.h:36-82) leaves it, but clustering off
        unless asked (the parity default, SURVEY.md §7 hard part 1)."""
        return Params(self.docs_to_get, real_max_top, language, site_clustering, num_docid_splits,
                      same_lang_weight, 1, 0, max_serp_score, min_serp_docid)


def _tid(seed: int, k: int) -> int:
    x = (seed * 0x9E3779B97F4A7C15 + k * 0xBF58476D1CE4E5B9 + 0x1234567) & ((1 << 64) - 1)
    x ^= x >> 29
    x = (x * 0x94D049BB133111EB) & ((1 << 64) - 1)
    return (x ^ (x >> 31)) & ((1 << 48) - 1)


def build_query(name: str, words: Sequence[Word], num_docs: int, *, seed: int = 1,
                bigram_keep: float = 0.5, quoted: Optional[Tuple[int, int]] = None,
                half_stop_bigram: Optional[int] = None, docs_to_get: int = 100,
                bigram_syn_pct: int = 50) -> Query:
    """Words in query order.  ``quoted=(a, b)`` quotes words a..b (inclusive,
    b-a >= 2): those words are replaced by required bigram terms sharing one
    quote id, as Query::set2 does for a quoted phrase of 3+ words.
    ``half_stop_bigram=i`` flags the bigram (i, i+1) as a wiki half-stop bigram."""
    terms: List[QTerm] = []
    specs: List[TermSpec] = []
    spec_of_term: List[int] = []
    word_term = {}
    word_spec = {}
    qpos = {i: 2 * i for i in range(len(words))}
    # words (skipping quoted ones)
    for i, w in enumerate(words):
        if quoted and quoted[0] <= i <= quoted[1]:
            continue
        word_term[i] = len(terms)
        word_spec[i] = len(specs)
        spec_of_term.append(len(specs))
        terms.append(QTerm(1, w.sign, 0, w.piped, -1, -1, -1, 0, qpos[i], w.wiki, -1,
                           tf_weight(w.p * num_docs, num_docs)))
        specs.append(TermSpec(_tid(seed, i), w.p, SYNTH_WORD))
    # adjacent-word bigrams between unquoted words (not required)
    for i in range(len(words) - 1):
        if i in word_term and (i + 1) in word_term and not words[i].sign and not words[i + 1].sign:
            a, b = word_term[i], word_term[i + 1]
            bt = len(terms)
            hs = 1 if half_stop_bigram == i else 0
            spec_of_term.append(len(specs))
            terms.append(QTerm(0, 0, 0, 0, -1, -1, -1, hs, qpos[i], words[i].wiki, -1,
                               tf_weight(bigram_keep * words[i].p * words[i + 1].p * num_docs, num_docs)))
            specs.append(TermSpec(_tid(seed, 100 + i), bigram_keep, SYNTH_BIGRAM, word_spec[i],
                                  word_spec[i + 1], -1, bigram_syn_pct))
            terms[a].right_phrase_term = bt
            terms[b].left_phrase_term = bt
    # quoted phrase -> required bigram terms with a shared quote start
    if quoted:
        qa, qb = quoted
        # component words exist only as generator inputs (not query terms)
        comp = {}
        for i in range(qa, qb + 1):
            comp[i] = len(specs)
            specs.append(TermSpec(_tid(seed, 200 + i), words[i].p, SYNTH_WORD))
        prev_bigram_spec = -1
        for i in range(qa, qb):
            spec_of_term.append(len(specs))
            terms.append(QTerm(1, ord('*'), 0, 0, -1, -1, -1, 0, qpos[i], words[i].wiki, qpos[qa],
                               tf_weight(0.6 * words[i].p * words[i + 1].p * num_docs, num_docs)))
            spec_index = len(specs)
            specs.append(TermSpec(_tid(seed, 300 + i), 0.6, SYNTH_BIGRAM, comp[i], comp[i + 1],
                                  prev_bigram_spec, 0))
            prev_bigram_spec = spec_index
    # synonyms (not required)
    for i, w in enumerate(words):
        for s, ps in enumerate(w.synonyms):
            if i not in word_term:
                continue
            spec_of_term.append(len(specs))
            terms.append(QTerm(0, 0, 0, 0, word_term[i], -1, -1, 0, qpos[i], w.wiki, -1,
                               tf_weight(ps * num_docs, num_docs)))
            specs.append(TermSpec(_tid(seed, 400 + 10 * i + s), ps, SYNTH_SYNONYM, -1, -1, -1, 100))
    return Query(name, terms, specs, spec_of_term, docs_to_get)


def generate(q: Query, num_docs: int, seed: int = 0x6B1A57, doc_begin: int = 0, doc_end: int = 0,
             threads: int = 0) -> List[bytes]:
    """Lists 1-1 with q.terms (the generator may need extra component specs,
    e.g. the words of a quoted phrase; those lists are dropped)."""
    lists = synth_lists(num_docs, q.specs, seed=seed, doc_begin=doc_begin, doc_end=doc_end, threads=threads)
    return [lists[k] for k in q.spec_of_term]


# ----------------------------------------------------------- bench configs
def config_two_term(num_docs: int, docs_to_get: int = 100, seed: int = 1) -> Query:
    """Configs 1/2: 2-term AND with its bigram (df ~ 0.1 N, 0.02 N at 100M)."""
    if num_docs <= 100000:
        words = [Word("a", 0.30), Word("b", 0.15)]
        keep = 0.44
    else:
        words = [Word("a", 0.10), Word("b", 0.02)]
        keep = 1.0
    return build_query("two_term", words, num_docs, seed=seed, bigram_keep=keep, docs_to_get=docs_to_get)


def config3_queries(num_docs: int, docs_to_get: int = 100, seed: int = 3) -> List[Query]:
    """Config 3: ten fixed 3-5 term queries, three with a quoted phrase."""
    rng = np.random.default_rng(seed)
    qs = []
    for k in range(10):
        nw = int(rng.integers(3, 6))
        ps = [float(x) for x in np.sort(rng.uniform(0.02, 0.2, nw))[::-1]]
        words = [Word(f"w{k}_{i}", ps[i]) for i in range(nw)]
        quoted = None
        if k in (2, 5, 8):
            quoted = (0, 2)
            for i in range(3):
                words[i].p = max(words[i].p, 0.15)
        qs.append(build_query(f"q3_{k}", words, num_docs, seed=seed * 100 + k, bigram_keep=0.5,
                              quoted=quoted, docs_to_get=docs_to_get))
    return qs


# -------------------------------------------------------------- case files
def write_case(path: str, q: Query, lists: Sequence[bytes], params: Params) -> None:
    """GBQ1 case file (tests/golden): header, then per term its QTerm fields,
    tf weight and list bytes."""
    with open(path, "wb") as f:
        f.write(b"GBQ1")
        f.write(struct.pack("<i", len(q.terms)))
        f.write(struct.pack("<6i", params.docs_to_get, params.real_max_top, params.language,
                            params.site_clustering, params.num_docid_splits, 0))
        f.write(struct.pack("<f", params.same_lang_weight))
        for t, l in zip(q.terms, lists):
            f.write(struct.pack("<11i", t.is_required, t.term_sign, t.field_code, t.piped, t.synonym_of,
                                t.left_phrase_term, t.right_phrase_term, t.is_wiki_half_stop_bigram, t.qpos,
                                t.wiki_phrase_id, t.quote_start))
            f.write(struct.pack("<f", t.tf_weight))
            f.write(struct.pack("<q", len(l)))
            f.write(l)


def read_case(path: str):
    with open(path, "rb") as f:
        data = f.read()
    assert data[:4] == b"GBQ1"
    (nt,) = struct.unpack_from("<i", data, 4)
    hdr = struct.unpack_from("<6i", data, 8)
    (slw,) = struct.unpack_from("<f", data, 32)
    off = 36
    terms, lists = [], []
    for _ in range(nt):
        f = struct.unpack_from("<11i", data, off)
        off += 44
        (tfw,) = struct.unpack_from("<f", data, off)
        off += 4
        (sz,) = struct.unpack_from("<q", data, off)
        off += 8
        terms.append(QTerm(*f, tfw))
        lists.append(data[off:off + sz])
        off += sz
    params = Params(hdr[0], hdr[1], hdr[2], hdr[3], hdr[4], slw)
    return terms, lists, params


def write_result(path: str, docids, scores, hits: int, filtered: int, docs_wanted: int) -> None:
    with open(path, "wb") as f:
        f.write(b"GBR1")
        f.write(struct.pack("<qiii", hits, filtered, len(docids), docs_wanted))
        for d, s in zip(docids, scores):
            f.write(struct.pack("<q", int(d)))
            f.write(np.float32(s).tobytes())


def read_result(path: str):
    with open(path, "rb") as f:
        data = f.read()
    assert data[:4] == b"GBR1"
    hits, filtered, n, dw = struct.unpack_from("<qiii", data, 4)
    docids = np.zeros(n, np.int64)
    scores = np.zeros(n, np.float32)
    for i in range(n):
        docids[i] = struct.unpack_from("<q", data, 24 + 12 * i)[0]
        scores[i] = np.frombuffer(data[32 + 12 * i:36 + 12 * i], dtype=np.float32)[0]
    return dict(hits=hits, filtered=filtered, docids=docids, scores=scores, docs_wanted=dw)
