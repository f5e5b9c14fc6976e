"""ctypes binding of the gbgpu C ABI (include/gbgpu.h, include/gbgpu_synth.h).

The product is the C-ABI library ``lib/libgbgpu.so``; this module is the thin
Python view of it that the tests and ``bench.py`` use (the Gigablast host would
bind the same symbols from C++).  Loading fails loudly if
the library is missing: there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import errno
import os
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.dirname(_HERE)
LIB_PATH = os.path.join(PKG_DIR, "lib", "libgbgpu.so")

GBGPU_ENODEVICE = 1001
GBGPU_EUNSUPPORTED = 1002
GBGPU_ECORRUPT = 1003
GBGPU_EHIP = 1004
GBGPU_ECAPACITY = 1005


class QTerm(ctypes.Structure):
    """gbgpu_qterm == Query::m_qterms[i] (+ its tf weight)."""

    _fields_ = [
        ("is_required", ctypes.c_int32),
        ("term_sign", ctypes.c_int32),
        ("field_code", ctypes.c_int32),
        ("piped", ctypes.c_int32),
        ("synonym_of", ctypes.c_int32),
        ("left_phrase_term", ctypes.c_int32),
        ("right_phrase_term", ctypes.c_int32),
        ("is_wiki_half_stop_bigram", ctypes.c_int32),
        ("qpos", ctypes.c_int32),
        ("wiki_phrase_id", ctypes.c_int32),
        ("quote_start", ctypes.c_int32),
        ("tf_weight", ctypes.c_float),
        ("number_float", ctypes.c_float),  # m_qword->m_float (range terms)
        ("number_int", ctypes.c_int32),    # m_qword->m_int
    ]


class Params(ctypes.Structure):
    _fields_ = [
        ("docs_to_get", ctypes.c_int32),
        ("real_max_top", ctypes.c_int32),
        ("language", ctypes.c_int32),
        ("site_clustering", ctypes.c_int32),
        ("num_docid_splits", ctypes.c_int32),
        ("same_lang_weight", ctypes.c_float),
        ("do_max_score_algo", ctypes.c_int32),
        ("get_docid_scoring_info", ctypes.c_int32),
        ("max_serp_score", ctypes.c_double),
        ("min_serp_docid", ctypes.c_int64),
        ("use_whitelist", ctypes.c_int32),
        ("n_white_lists", ctypes.c_int32),
        ("white_lists", ctypes.c_void_p),
        ("is_boolean", ctypes.c_int32),
        ("bool_ngroups", ctypes.c_int32),
        ("bool_table", ctypes.c_void_p),
        ("n_facet_ranges", ctypes.c_int32),
        ("pad_f", ctypes.c_int32),
        ("facet_ranges", ctypes.c_void_p),
    ]

    def _copy(self):
        q = Params.from_buffer_copy(self)
        for a in ("_keep", "_white", "_btok", "_btable", "_bkeep", "_franges", "_fkeep"):
            if hasattr(self, a):
                setattr(q, a, getattr(self, a))
        return q

    def with_facets(self, ranges):
        """A copy of these params carrying gbfacetint:/gbfacetfloat: ranges:
        [(term, A[], B[]), ...] as int32 bit patterns (floats by their bits)
        -- QueryWord::m_facetRange{Int,Float}{A,B} (Query.h:389-393)."""
        q = self._copy()
        arr = (FacetRanges * max(1, len(ranges)))()
        keep = []
        for i, (term, a, b) in enumerate(ranges):
            aa = (ctypes.c_int32 * max(1, len(a)))(*[int(x) for x in a])
            bb = (ctypes.c_int32 * max(1, len(b)))(*[int(x) for x in b])
            keep += [aa, bb]
            arr[i] = FacetRanges(int(term), len(a), ctypes.cast(aa, ctypes.c_void_p), ctypes.cast(bb, ctypes.c_void_p))
        keep.append(arr)
        q._fkeep = keep
        q.n_facet_ranges = len(ranges)
        q.facet_ranges = ctypes.cast(arr, ctypes.c_void_p) if ranges else None
        q._franges = [(int(t), [int(x) for x in a], [int(x) for x in b]) for t, a, b in ranges]
        return q

    def with_whitelist(self, lists):
        """A copy of these params carrying the "&sites=" whitelist lists
        (Msg2::m_whiteLists; Posdb.cpp:793-835, 5294).  The copy keeps the
        list buffers alive."""
        q = self._copy()
        q._keep = [ctypes.create_string_buffer(bytes(l), max(1, len(l))) for l in lists]
        arr = (ListRef * max(1, len(lists)))(*[ListRef(ctypes.cast(k, ctypes.c_void_p), len(l))
                                               for k, l in zip(q._keep, lists)])
        q._keep.append(arr)
        q.use_whitelist = 1
        q.n_white_lists = len(lists)
        q.white_lists = ctypes.cast(arr, ctypes.c_void_p) if lists else None
        q._white = [bytes(l) for l in lists]
        for a in ("_btok", "_btable", "_bkeep"):
            if hasattr(self, a):
                setattr(q, a, getattr(self, a))
        return q

    def with_boolean(self, table: bytes, ngroups: int, tokens=None):
        """A copy of these params for a boolean query: the expression's truth
        table over the plan's QueryTermInfo bit vectors (bit v = byte v >> 3,
        bit v & 7), and -- for the reference harness only -- the expression
        tokens it is built from (ref_binding: operand term >= 0, OP_OR -1,
        OP_AND -2, OP_NOT -3, '(' -4, ')' -5)."""
        q = self._copy()  # keeps the buffers the pointers name (facet ranges, whitelist)
        table = bytes(table)
        q._bkeep = ctypes.create_string_buffer(table, max(1, len(table)))
        q.is_boolean = 1
        q.bool_ngroups = int(ngroups)
        q.bool_table = ctypes.cast(q._bkeep, ctypes.c_void_p)
        q._btable = table
        q._btok = list(tokens) if tokens is not None else getattr(self, "_btok", None)
        return q


class ListRef(ctypes.Structure):
    _fields_ = [("bytes", ctypes.c_void_p), ("size", ctypes.c_int64)]


class FacetRanges(ctypes.Structure):
    _fields_ = [("term", ctypes.c_int32), ("n", ctypes.c_int32), ("a", ctypes.c_void_p), ("b", ctypes.c_void_p)]


class Piece(ctypes.Structure):
    """gbgpu_piece: a file range (file >= 0) or a host list (file = -1)."""
    _fields_ = [("file", ctypes.c_int32), ("pad", ctypes.c_int32), ("offset", ctypes.c_int64),
                ("size", ctypes.c_int64), ("key18", ctypes.c_void_p), ("bytes", ctypes.c_void_p)]


class PairScore(ctypes.Structure):
    """gbgpu_pair_score == the reference's PairScore (Posdb.h:767-800)."""

    _fields_ = [
        ("final_score", ctypes.c_float),
        ("is_synonym1", ctypes.c_int8), ("is_synonym2", ctypes.c_int8),
        ("is_half_stop_wiki_bigram1", ctypes.c_int8), ("is_half_stop_wiki_bigram2", ctypes.c_int8),
        ("diversity_rank1", ctypes.c_int8), ("diversity_rank2", ctypes.c_int8),
        ("density_rank1", ctypes.c_int8), ("density_rank2", ctypes.c_int8),
        ("word_spam_rank1", ctypes.c_int8), ("word_spam_rank2", ctypes.c_int8),
        ("hash_group1", ctypes.c_int8), ("hash_group2", ctypes.c_int8),
        ("in_same_wiki_phrase", ctypes.c_int8), ("fixed_distance", ctypes.c_int8),
        ("word_pos1", ctypes.c_int32), ("word_pos2", ctypes.c_int32),
        ("term_freq1", ctypes.c_int64), ("term_freq2", ctypes.c_int64),
        ("tf_weight1", ctypes.c_float), ("tf_weight2", ctypes.c_float),
        ("qterm_num1", ctypes.c_int32), ("qterm_num2", ctypes.c_int32),
        ("bflags1", ctypes.c_int8), ("bflags2", ctypes.c_int8),
        ("qdist", ctypes.c_int32),
    ]


class SingleScore(ctypes.Structure):
    """gbgpu_single_score == the reference's SingleScore (Posdb.h:802-816)."""

    _fields_ = [
        ("final_score", ctypes.c_float),
        ("is_synonym", ctypes.c_int8), ("is_half_stop_wiki_bigram", ctypes.c_int8),
        ("diversity_rank", ctypes.c_int8), ("density_rank", ctypes.c_int8),
        ("word_spam_rank", ctypes.c_int8), ("hash_group", ctypes.c_int8),
        ("word_pos", ctypes.c_int32),
        ("term_freq", ctypes.c_int64),
        ("tf_weight", ctypes.c_float),
        ("qterm_num", ctypes.c_int32),
        ("bflags", ctypes.c_int8),
    ]


class DocIdScore(ctypes.Structure):
    """gbgpu_docid_score == the reference's DocIdScore (Posdb.h:818-866)."""

    _fields_ = [
        ("docid", ctypes.c_int64),
        ("final_score", ctypes.c_double),
        ("site_rank", ctypes.c_int8),
        ("doc_lang", ctypes.c_int32),
        ("num_required_terms", ctypes.c_int32),
        ("num_pairs", ctypes.c_int32), ("num_singles", ctypes.c_int32),
        ("pairs_offset", ctypes.c_int32), ("singles_offset", ctypes.c_int32),
        ("pair_scores", ctypes.c_void_p), ("single_scores", ctypes.c_void_p),
    ]


PAIR_DT, SINGLE_DT, DOCID_DT = np.dtype(PairScore), np.dtype(SingleScore), np.dtype(DocIdScore)


class Result(ctypes.Structure):
    _fields_ = [
        ("docids", ctypes.POINTER(ctypes.c_int64)),
        ("scores", ctypes.POINTER(ctypes.c_float)),
        ("capacity", ctypes.c_int32),
        ("n", ctypes.c_int32),
        ("hits", ctypes.c_int64),
        ("filtered", ctypes.c_int32),
        ("docs_wanted", ctypes.c_int32),
        ("hit_docids", ctypes.POINTER(ctypes.c_int64)),
        ("hit_capacity", ctypes.c_int64),
        ("n_hit_docids", ctypes.c_int64),
        ("docid_scores", ctypes.c_void_p), ("docid_scores_cap", ctypes.c_int32), ("n_docid_scores", ctypes.c_int32),
        ("pair_scores", ctypes.c_void_p), ("pair_scores_cap", ctypes.c_int32), ("n_pair_scores", ctypes.c_int32),
        ("single_scores", ctypes.c_void_p), ("single_scores_cap", ctypes.c_int32),
        ("n_single_scores", ctypes.c_int32),
        ("int_scores", ctypes.POINTER(ctypes.c_int32)),
        ("facets", ctypes.c_void_p), ("facets_cap", ctypes.c_int32), ("n_facets", ctypes.c_int32),
        ("facet_docs", ctypes.POINTER(ctypes.c_uint64)),
    ]


# gbgpu_facet_entry: one entry of a facet term's QueryTerm::m_facetHashTable
FACET_DT = np.dtype([("term", "<i4"), ("key", "<i4"), ("count", "<i4"), ("outside", "<i4"), ("docid", "<i8"),
                     ("sum", "<i8"), ("max", "<i4"), ("min", "<i4")])
FACET_FIELDS = (63, 64, 65)  # gbfacetstr: / gbfacetint: / gbfacetfloat:


class Reply(ctypes.Structure):
    """gbgpu_reply: one Msg39Reply (Msg39.h:169-208)"""
    _fields_ = [("n", ctypes.c_int32), ("hits", ctypes.c_int32), ("docids", ctypes.c_void_p),
                ("scores", ctypes.c_void_p), ("cluster_recs", ctypes.c_void_p), ("facet_list", ctypes.c_void_p),
                ("facet_list_size", ctypes.c_int32), ("nqt", ctypes.c_int32), ("facet_docs", ctypes.c_void_p)]


class MergeReq(ctypes.Structure):
    _fields_ = [("docs_to_get", ctypes.c_int32), ("site_clustering", ctypes.c_int32),
                ("hide_all_clustered", ctypes.c_int32), ("family_filter", ctypes.c_int32), ("nqt", ctypes.c_int32),
                ("pad", ctypes.c_int32), ("term_ids", ctypes.c_void_p), ("field_codes", ctypes.c_void_p)]


class Merged(ctypes.Structure):
    _fields_ = [("docids", ctypes.c_void_p), ("scores", ctypes.c_void_p), ("cluster_recs", ctypes.c_void_p),
                ("cap", ctypes.c_int32), ("n", ctypes.c_int32), ("hits", ctypes.c_int64),
                ("facet_docs", ctypes.c_void_p), ("facets", ctypes.c_void_p), ("facets_cap", ctypes.c_int32),
                ("n_facets", ctypes.c_int32)]


# gbgpu_facet_entry (40 bytes)
FACET_ENTRY = np.dtype([("term", "<i4"), ("key", "<i4"), ("count", "<i4"), ("outside", "<i4"), ("docid", "<i8"),
                        ("sum", "<i8"), ("max", "<i4"), ("min", "<i4")])


class FullReplies:
    """ctypes views of a Msg3a request and its shards' full replies (dicts of
    docids, scores, recs (bytes or None), hits, facets (bytes), fcounts
    (int64[nqt] or None); tests/msg3a_cases.py) and the output buffers."""

    def __init__(self, req, shards, cap=None, facets_cap=None):
        self.keep = []
        nqt = len(req["tids"])
        self.tids = np.ascontiguousarray(req["tids"], np.int64)
        self.fcs = np.ascontiguousarray(req["fcs"], np.int32)
        self.req = MergeReq(req["docs_to_get"], req["clus"], req["hide"], req["family"], nqt, 0,
                            self.tids.ctypes.data, self.fcs.ctypes.data)
        self.reps = (Reply * max(1, len(shards)))()
        for j, s in enumerate(shards):
            d = np.ascontiguousarray(s["docids"], np.int64)
            sc = np.ascontiguousarray(s["scores"], np.float64)
            rec = ctypes.create_string_buffer(s["recs"], max(1, len(s["recs"]))) if s["recs"] is not None else None
            fl = ctypes.create_string_buffer(s["facets"], max(1, len(s["facets"])))
            fc = np.ascontiguousarray(s["fcounts"], np.int64) if s.get("fcounts") is not None else None
            self.keep += [d, sc, rec, fl, fc]
            self.reps[j] = Reply(len(d), s["hits"], d.ctypes.data, sc.ctypes.data,
                                 ctypes.cast(rec, ctypes.c_void_p) if rec is not None else None,
                                 ctypes.cast(fl, ctypes.c_void_p) if s["facets"] else None, len(s["facets"]), nqt,
                                 fc.ctypes.data if fc is not None else None)
        self.n = len(shards)
        cap = cap if cap is not None else max(1, req["docs_to_get"])
        fcap = facets_cap if facets_cap is not None else sum(len(s["facets"]) // 36 for s in shards) + 1
        self.od = np.zeros(cap, np.int64)
        self.os = np.zeros(cap, np.float64)
        self.orec = np.zeros(12 * cap, np.uint8)
        self.ofd = np.zeros(max(1, nqt), np.int64)
        self.ofac = np.zeros(max(1, fcap), FACET_ENTRY)
        self.out = Merged(self.od.ctypes.data, self.os.ctypes.data, self.orec.ctypes.data, cap, 0, 0,
                          self.ofd.ctypes.data, self.ofac.ctypes.data, fcap, 0)
        self.nqt = nqt
        self.clus = req["clus"]

    def result(self):
        """-> dict(docids, scores, recs (bytes or None), hits, fdocs, facets (FACET_ENTRY[]))"""
        n = self.out.n
        return dict(docids=self.od[:n].copy(), scores=self.os[:n].copy(),
                    recs=self.orec[:12 * n].tobytes() if self.clus else None, hits=self.out.hits,
                    fdocs=self.ofd[:self.nqt].copy(), facets=self.ofac[:self.out.n_facets].copy(),
                    n_facets=self.out.n_facets)


def merge_replies(req, shards, **kw):
    """gbgpu_merge_replies: Msg3a::mergeLists whole on the host"""
    x = FullReplies(req, shards, **kw)
    _check(load().gbgpu_merge_replies(ctypes.byref(x.req), x.reps, x.n, ctypes.byref(x.out)), "gbgpu_merge_replies")
    return x.result()


class SynthCorpus(ctypes.Structure):
    _fields_ = [
        ("num_docs", ctypes.c_int64),
        ("seed", ctypes.c_uint64),
        ("doc_begin", ctypes.c_int64),
        ("doc_end", ctypes.c_int64),
        ("max_positions", ctypes.c_int32),
        ("num_threads", ctypes.c_int32),
    ]


class SynthTerm(ctypes.Structure):
    _fields_ = [
        ("term_id", ctypes.c_uint64),
        ("p", ctypes.c_double),
        ("kind", ctypes.c_int32),
        ("a", ctypes.c_int32),
        ("b", ctypes.c_int32),
        ("align_to", ctypes.c_int32),
        ("syn_frac_pct", ctypes.c_int32),
    ]


SYNTH_WORD, SYNTH_SYNONYM, SYNTH_BIGRAM = 0, 1, 2

# every symbol include/gbgpu.h and include/gbgpu_synth.h declare
EXPORTS = [
    "gbgpu_open", "gbgpu_close", "gbgpu_strerror", "gbgpu_abi_version", "gbgpu_docs_wanted",
    "gbgpu_tree_capacity",
    "gbgpu_query", "gbgpu_list_upload", "gbgpu_list_free", "gbgpu_query_resident",
    "gbgpu_file_upload", "gbgpu_file_list", "gbgpu_file_lists", "gbgpu_file_free",
    "gbgpu_query_resident_enqueue", "gbgpu_query_collect", "gbgpu_stream",
    "gbgpu_last_topk_device", "gbgpu_merge_topk", "gbgpu_merge_posdb", "gbgpu_set_profiling",
    "gbgpu_last_timings", "gbgpu_set_query_slots", "gbgpu_query_slots", "gbgpu_query_slot_enqueue",
    "gbgpu_query_slot_collect", "gbgpu_slot_stream", "gbgpu_slot_timings", "gbgpu_slot_stats",
    "gbgpu_bandwidth_ceiling", "gbgpu_comm_unique_id", "gbgpu_comm_init", "gbgpu_allgather_topk",
    "gbgpu_merge_topk_device", "gbgpu_seq_open", "gbgpu_seq_enter", "gbgpu_seq_leave", "gbgpu_seq_next",
    "gbgpu_seq_close", "gbgpu_exchange_next", "gbgpu_merge_replies", "gbgpu_merge_replies_device",
    "gbgpu_allgather_replies",
    "gbgpu_merge_posdb_device", "gbgpu_merge_timings", "gbgpu_merge_path", "gbgpu_merge_last_key", "gbgpu_merge_input_left", "gbgpu_termlist_merge", "gb_synth_merge_runs",
    "gb_synth_lists", "gb_synth_free", "gb_synth_docid", "gb_posdb_compress", "gb_posdb_make_key",
]

DIAG_LIB_PATH = os.path.join(PKG_DIR, "lib", "libgbgpu_diag.so")
ALT_LIB_PATH = os.path.join(PKG_DIR, "lib", "libgbgpu_alt.so")  # an A/B build (Makefile `alt`), bench.py only
_libs = {}


def load(path: str = LIB_PATH) -> ctypes.CDLL:
    """The product library (default), or the diagnostic build
    (DIAG_LIB_PATH: the same sources with -DGBGPU_DIAG, which honours the
    GBGPU_*_MODE switches of scripts/ and tests/test_replay.py)."""
    if path in _libs:
        return _libs[path]
    if not os.path.exists(path):
        raise RuntimeError(f"gbgpu native library not built: {path} (run __graft_entry__.build())")
    lib = ctypes.CDLL(path)
    vp, i32, i64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
    lib.gbgpu_open.argtypes = [ctypes.c_int, ctypes.POINTER(vp)]
    lib.gbgpu_close.argtypes = [vp]
    lib.gbgpu_close.restype = None
    lib.gbgpu_strerror.argtypes = [ctypes.c_int]
    lib.gbgpu_strerror.restype = ctypes.c_char_p
    lib.gbgpu_docs_wanted.argtypes = [ctypes.POINTER(Params), ctypes.POINTER(i64), ctypes.c_int]
    lib.gbgpu_docs_wanted.restype = i32
    lib.gbgpu_tree_capacity.argtypes = [ctypes.POINTER(Params), ctypes.POINTER(i64), ctypes.c_int]
    lib.gbgpu_tree_capacity.restype = i32
    lib.gbgpu_query.argtypes = [vp, ctypes.POINTER(QTerm), ctypes.c_int, ctypes.POINTER(ListRef),
                                ctypes.POINTER(Params), ctypes.POINTER(Result)]
    lib.gbgpu_list_upload.argtypes = [vp, vp, i64, ctypes.POINTER(i32)]
    lib.gbgpu_list_free.argtypes = [vp, i32]
    lib.gbgpu_file_upload.argtypes = [vp, vp, i64, ctypes.POINTER(i32)]
    lib.gbgpu_file_list.argtypes = [vp, i32, i64, i64, vp, ctypes.POINTER(i32)]
    lib.gbgpu_file_lists.argtypes = [vp, i32, ctypes.c_int, ctypes.POINTER(i64), ctypes.POINTER(i64), vp,
                                     ctypes.POINTER(i32)]
    lib.gbgpu_file_free.argtypes = [vp, i32]
    lib.gbgpu_termlist_merge.argtypes = [vp, vp, ctypes.c_int, ctypes.c_int, i64, ctypes.POINTER(i32), vp, i64,
                                         ctypes.POINTER(i64)]
    lib.gbgpu_query_resident.argtypes = [vp, ctypes.POINTER(QTerm), ctypes.c_int, ctypes.POINTER(i32),
                                         ctypes.POINTER(Params), ctypes.POINTER(Result)]
    lib.gbgpu_query_resident_enqueue.argtypes = [vp, ctypes.POINTER(QTerm), ctypes.c_int,
                                                 ctypes.POINTER(i32), ctypes.POINTER(Params)]
    lib.gbgpu_query_collect.argtypes = [vp, ctypes.POINTER(Result)]
    lib.gbgpu_stream.argtypes = [vp]
    lib.gbgpu_stream.restype = vp
    lib.gbgpu_last_topk_device.argtypes = [vp, ctypes.POINTER(vp), ctypes.POINTER(i32)]
    lib.gbgpu_merge_topk.argtypes = [ctypes.POINTER(ctypes.POINTER(i64)),
                                     ctypes.POINTER(ctypes.POINTER(ctypes.c_double)),
                                     ctypes.POINTER(i32), ctypes.c_int, i32, ctypes.POINTER(i64),
                                     ctypes.POINTER(ctypes.c_double), ctypes.POINTER(i32)]
    lib.gbgpu_merge_posdb.argtypes = [vp, ctypes.POINTER(ListRef), ctypes.c_int, ctypes.c_int, i64, vp,
                                      i64, ctypes.POINTER(i64)]
    lib.gbgpu_merge_posdb_device.argtypes = [vp, ctypes.POINTER(vp), ctypes.POINTER(i64), ctypes.c_int,
                                             ctypes.c_int, i64, vp, i64, ctypes.POINTER(i64)]
    lib.gbgpu_merge_last_key.argtypes = [vp, vp]
    lib.gbgpu_merge_input_left.argtypes = [vp, ctypes.POINTER(i32)]
    lib.gbgpu_merge_path.argtypes = [vp]
    lib.gbgpu_merge_timings.argtypes = [vp, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(i64),
                                        ctypes.POINTER(i64)]
    lib.gb_synth_merge_runs.argtypes = [i64, ctypes.c_int, ctypes.c_uint64, ctypes.c_double, ctypes.c_double,
                                        ctypes.c_int, ctypes.c_int, ctypes.POINTER(vp), ctypes.POINTER(i64)]
    lib.gbgpu_set_profiling.argtypes = [vp, ctypes.c_int]
    lib.gbgpu_last_timings.argtypes = [vp, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(i64)]
    lib.gbgpu_set_query_slots.argtypes = [vp, ctypes.c_int]
    lib.gbgpu_query_slots.argtypes = [vp]
    lib.gbgpu_query_slot_enqueue.argtypes = [vp, ctypes.c_int, ctypes.POINTER(QTerm), ctypes.c_int,
                                             ctypes.POINTER(i32), ctypes.POINTER(Params)]
    lib.gbgpu_query_slot_collect.argtypes = [vp, ctypes.c_int, ctypes.POINTER(Result)]
    lib.gbgpu_slot_stream.argtypes = [vp, ctypes.c_int]
    lib.gbgpu_slot_stream.restype = vp
    lib.gbgpu_slot_timings.argtypes = [vp, ctypes.c_int, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(i64)]
    lib.gbgpu_slot_stats.argtypes = [vp, ctypes.c_int, ctypes.POINTER(i64)]
    lib.gbgpu_seq_open.argtypes = [ctypes.c_uint64, ctypes.POINTER(vp)]
    lib.gbgpu_seq_enter.argtypes = [vp, ctypes.c_uint64, ctypes.c_int]
    lib.gbgpu_seq_leave.argtypes = [vp, ctypes.c_uint64]
    lib.gbgpu_seq_next.argtypes = [vp]
    lib.gbgpu_seq_next.restype = ctypes.c_uint64
    lib.gbgpu_seq_close.argtypes = [vp]
    lib.gbgpu_seq_close.restype = None
    lib.gbgpu_comm_unique_id.argtypes = [vp]
    lib.gbgpu_comm_init.argtypes = [vp, ctypes.c_int, ctypes.c_int, vp]
    lib.gbgpu_exchange_next.argtypes = [vp]
    lib.gbgpu_exchange_next.restype = ctypes.c_uint64
    lib.gbgpu_allgather_topk.argtypes = [vp, ctypes.c_int, ctypes.c_uint64, ctypes.c_int, i32, ctypes.POINTER(i64),
                                         ctypes.POINTER(ctypes.c_double), ctypes.POINTER(i32), ctypes.POINTER(i64),
                                         ctypes.POINTER(Result)]
    lib.gbgpu_merge_topk_device.argtypes = [vp, ctypes.c_int, i32, ctypes.POINTER(i32), ctypes.POINTER(i64),
                                               ctypes.POINTER(ctypes.POINTER(i64)),
                                               ctypes.POINTER(ctypes.POINTER(ctypes.c_double)),
                                               ctypes.POINTER(i64), ctypes.POINTER(ctypes.c_double),
                                               ctypes.POINTER(i32), ctypes.POINTER(i64)]
    lib.gbgpu_merge_replies.argtypes = [ctypes.POINTER(MergeReq), ctypes.POINTER(Reply), ctypes.c_int,
                                        ctypes.POINTER(Merged)]
    lib.gbgpu_merge_replies_device.argtypes = [vp, ctypes.POINTER(MergeReq), ctypes.POINTER(Reply), ctypes.c_int,
                                               ctypes.POINTER(Merged)]
    lib.gbgpu_allgather_replies.argtypes = [vp, ctypes.c_uint64, ctypes.c_int, ctypes.POINTER(MergeReq),
                                            ctypes.POINTER(Reply), ctypes.POINTER(Merged)]
    lib.gbgpu_bandwidth_ceiling.argtypes = [vp, i64, ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                            ctypes.POINTER(ctypes.c_double)]
    lib.gb_synth_lists.argtypes = [ctypes.POINTER(SynthCorpus), ctypes.POINTER(SynthTerm), ctypes.c_int,
                                   ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(i64)]
    lib.gb_synth_free.argtypes = [vp]
    lib.gb_synth_free.restype = None
    lib.gb_synth_docid.argtypes = [ctypes.POINTER(SynthCorpus), i64]
    lib.gb_synth_docid.restype = ctypes.c_uint64
    lib.gb_posdb_compress.argtypes = [vp, i64, vp]
    lib.gb_posdb_compress.restype = i64
    lib.gb_posdb_make_key.argtypes = [vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                                      ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                      ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int,
                                      ctypes.c_int, ctypes.c_int]
    lib.gb_posdb_make_key.restype = None
    _libs[path] = lib
    return lib


class GbgpuError(RuntimeError):
    def __init__(self, code: int, what: str = ""):
        self.code = code
        msg = load().gbgpu_strerror(code).decode()
        super().__init__(f"gbgpu error {code} ({msg}) {what}")


def _check(rc: int, what: str = "") -> None:
    if rc != 0:
        raise GbgpuError(rc, what)


# ---------------------------------------------------------------- synthesis
@dataclass
class TermSpec:
    term_id: int
    p: float
    kind: int = SYNTH_WORD
    a: int = -1
    b: int = -1
    align_to: int = -1
    syn_frac_pct: int = 0


def synth_lists(num_docs: int, specs: Sequence[TermSpec], seed: int = 0x6B1A57, doc_begin: int = 0,
                doc_end: int = 0, max_positions: int = 64, threads: int = 0) -> List[bytes]:
    lib = load()
    c = SynthCorpus(num_docs, seed, doc_begin, doc_end, max_positions, threads)
    n = len(specs)
    arr = (SynthTerm * n)(*[SynthTerm(s.term_id, s.p, s.kind, s.a, s.b, s.align_to, s.syn_frac_pct)
                            for s in specs])
    bufs = (ctypes.c_void_p * n)()
    sizes = (ctypes.c_int64 * n)()
    _check(lib.gb_synth_lists(ctypes.byref(c), arr, n, bufs, sizes), "gb_synth_lists")
    out = []
    for i in range(n):
        if sizes[i]:
            out.append(ctypes.string_at(bufs[i], sizes[i]))
            lib.gb_synth_free(bufs[i])
        else:
            out.append(b"")
    return out


class MergeRuns:
    """Config-5 tiered runs made by gb_synth_merge_runs (csrc/synth.cpp), kept in
    the generator's own buffers: .arrays are numpy uint8 views; free() releases."""

    def __init__(self, total_keys: int, nruns: int = 8, seed: int = 5, dup_frac: float = 0.05,
                 neg_frac: float = 0.01, nterms: int = 20000, nthreads: int = 0):
        import numpy as np
        lib = load()
        self._lib = lib
        self._bufs = (ctypes.c_void_p * nruns)()
        self.sizes = (ctypes.c_int64 * nruns)()
        _check(lib.gb_synth_merge_runs(int(total_keys), nruns, seed, dup_frac, neg_frac, nterms, nthreads,
                                       self._bufs, self.sizes), "gb_synth_merge_runs")
        self.arrays = []
        for i in range(nruns):
            n = self.sizes[i]
            if n:
                a = np.ctypeslib.as_array((ctypes.c_uint8 * n).from_address(self._bufs[i]))
            else:
                a = np.zeros(0, np.uint8)
            self.arrays.append(a)

    def as_bytes(self):
        return [a.tobytes() for a in self.arrays]

    def free(self):
        for i in range(len(self.arrays)):
            if self._bufs[i]:
                self._lib.gb_synth_free(self._bufs[i])
                self._bufs[i] = None
        self.arrays = []


def synth_merge_runs(total_keys: int, **kw):
    """Config-5 runs as bytes (small sizes; see MergeRuns for large ones)."""
    m = MergeRuns(total_keys, **kw)
    try:
        return m.as_bytes()
    finally:
        m.free()


def make_key(term_id, docid, wordpos, density, diversity, spam, siterank, hashgroup, langid,
             multiplier=0, syn=0, delkey=0, shard_by_termid=0) -> bytes:
    buf = ctypes.create_string_buffer(18)
    load().gb_posdb_make_key(buf, term_id, docid, wordpos, density, diversity, spam, siterank, hashgroup,
                             langid, multiplier, syn, delkey, shard_by_termid)
    return buf.raw


def compress(keys18: bytes) -> bytes:
    n = len(keys18) // 18
    out = ctypes.create_string_buffer(max(1, 18 * n))
    inb = ctypes.create_string_buffer(keys18, max(1, len(keys18)))
    m = load().gb_posdb_compress(inb, n, out)
    return out.raw[:m]


def docs_wanted(params: Params, sizes: Sequence[int]) -> int:
    arr = (ctypes.c_int64 * max(1, len(sizes)))(*sizes)
    return load().gbgpu_docs_wanted(ctypes.byref(params), arr, len(sizes))


def tree_capacity(params: Params, sizes: Sequence[int]) -> int:
    arr = (ctypes.c_int64 * max(1, len(sizes)))(*sizes)
    return load().gbgpu_tree_capacity(ctypes.byref(params), arr, len(sizes))


# ------------------------------------------------------------------- engine
@dataclass
class QueryResult:
    docids: np.ndarray
    scores: np.ndarray
    hits: int
    filtered: int
    docs_wanted: int
    hit_docids: Optional[np.ndarray] = None  # the intersected docid set (when asked for)
    # the second pass's score info (get_docid_scoring_info): structured arrays
    # of DOCID_DT / PAIR_DT / SINGLE_DT
    docid_scores: Optional[np.ndarray] = None
    pair_scores: Optional[np.ndarray] = None
    single_scores: Optional[np.ndarray] = None
    # TopNode::m_intScore under a gbsortby int term (scores are then 0.0)
    int_scores: Optional[np.ndarray] = None
    # facet terms: {term: (m_numDocsThatHaveFacet, {key: (count, outside,
    # docid, sum, max, min)})}, the tables QueryTerm::m_facetHashTable holds
    facets: Optional[dict] = None


class Engine:
    """One gbgpu context on one device: resident lists shared by its query
    slots (one HIP stream each; a context starts with one slot)."""

    def __init__(self, device: int = 0, diag: bool = False, path: Optional[str] = None):
        self.lib = load(path or (DIAG_LIB_PATH if diag else LIB_PATH))
        self.ctx = ctypes.c_void_p()
        _check(self.lib.gbgpu_open(device, ctypes.byref(self.ctx)), "gbgpu_open")
        self._keep = {}
        self._xseq = 0  # next exchange sequence number (allgather_topk)

    def close(self) -> None:
        if self.ctx:
            self.lib.gbgpu_close(self.ctx)
            self.ctx = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def upload(self, data: bytes) -> int:
        h = ctypes.c_int32()
        buf = ctypes.create_string_buffer(data, max(1, len(data)))
        _check(self.lib.gbgpu_list_upload(self.ctx, buf, len(data), ctypes.byref(h)), "upload")
        return h.value

    def free(self, handle: int) -> None:
        _check(self.lib.gbgpu_list_free(self.ctx, handle), "free")

    def file_upload(self, data: bytes) -> int:
        """A Posdb Rdb file image into HBM; returns its file handle."""
        h = ctypes.c_int32()
        buf = ctypes.create_string_buffer(bytes(data), len(data))
        _check(self.lib.gbgpu_file_upload(self.ctx, buf, len(data), ctypes.byref(h)), "file_upload")
        return h.value

    def file_list(self, fh: int, offset: int, size: int, key18: Optional[bytes] = None) -> int:
        """RdbScan's read of [offset, offset+size) of a resident file as a
        resident list handle; key18 = the map's full key for a compressed
        first key."""
        h = ctypes.c_int32()
        k = None
        if key18 is not None:
            assert len(key18) == 18
            k = ctypes.create_string_buffer(bytes(key18), 18)
        _check(self.lib.gbgpu_file_list(self.ctx, fh, offset, size, k, ctypes.byref(h)), "file_list")
        return h.value

    def file_lists(self, fh: int, offsets, sizes, key18s=None):
        """gbgpu_file_lists: a query's cuts together (all or nothing); key18s
        None or one entry a cut, each None or the map's full key."""
        n = len(offsets)
        assert len(sizes) == n and (key18s is None or len(key18s) == n)
        off = (ctypes.c_int64 * max(n, 1))(*offsets)
        sz = (ctypes.c_int64 * max(n, 1))(*sizes)
        hs = (ctypes.c_int32 * max(n, 1))()
        keys, kp = None, None
        if key18s is not None:
            keys = [None if k is None else ctypes.create_string_buffer(bytes(k), 18) for k in key18s]
            for k in key18s:
                assert k is None or len(k) == 18
            kp = (ctypes.c_void_p * max(n, 1))(*[None if k is None else ctypes.addressof(k) for k in keys])
        _check(self.lib.gbgpu_file_lists(self.ctx, fh, n, off, sz, kp, hs), "file_lists")
        return list(hs)[:n]

    def termlist_merge(self, pieces, remove_neg_keys: bool = True, min_rec_sizes: int = -1, want_bytes=False):
        """Msg5's read of one termlist: pieces oldest first, each (file handle,
        offset, size, key18-or-None) or bytes (the tree's list, newest last),
        merged on the device into a resident list.  Returns the handle, or
        (handle, merged bytes) with want_bytes."""
        arr = (Piece * max(1, len(pieces)))()
        keep = []
        total = 0
        for i, pc in enumerate(pieces):
            if isinstance(pc, (bytes, bytearray)):
                b = ctypes.create_string_buffer(bytes(pc), max(1, len(pc)))
                keep.append(b)
                arr[i] = Piece(-1, 0, 0, len(pc), None, ctypes.cast(b, ctypes.c_void_p))
                total += len(pc)
            else:
                fh, off, size, key = pc
                kb = None
                if key is not None:
                    kb = ctypes.create_string_buffer(bytes(key), 18)
                    keep.append(kb)
                arr[i] = Piece(fh, 0, off, size, ctypes.cast(kb, ctypes.c_void_p) if kb else None, None)
                total += size + 18
        h = ctypes.c_int32()
        n = ctypes.c_int64()
        out = ctypes.create_string_buffer(max(1, total + 64)) if want_bytes else None
        _check(self.lib.gbgpu_termlist_merge(self.ctx, arr, len(pieces), 1 if remove_neg_keys else 0, min_rec_sizes,
                                             ctypes.byref(h), out, total + 64 if want_bytes else 0, ctypes.byref(n)),
               "gbgpu_termlist_merge")
        return (h.value, out.raw[:n.value]) if want_bytes else h.value

    def file_free(self, fh: int) -> None:
        _check(self.lib.gbgpu_file_free(self.ctx, fh), "file_free")

    @staticmethod
    def info_arrays(params: Params, nterms: int):
        """Score-info output arrays sized for the request's worst case
        (every group pair and group recording real_max_top entries; with
        docid splits every piece's second pass appends up to docs_to_get
        docids)."""
        if not params.get_docid_scoring_info:
            return None
        pieces = 1 if params.num_docid_splits <= 1 else params.num_docid_splits + 1
        nd = max(1, params.docs_to_get) * pieces
        ng = max(1, min(nterms, 16))
        rmt = max(1, params.real_max_top)
        return (np.zeros(nd, DOCID_DT), np.zeros(max(1, nd * ng * (ng - 1) // 2 * rmt), PAIR_DT),
                np.zeros(nd * ng * rmt, SINGLE_DT))

    facet_cap = 1 << 16  # facet table entries a result holds

    @classmethod
    def _result(cls, cap: int, hit_cap: int = 0, info=None, nfacet_terms: int = 0, fterms=()):
        d = (ctypes.c_int64 * max(cap, 1))()
        s = (ctypes.c_float * max(cap, 1))()
        r = Result(ctypes.cast(d, ctypes.POINTER(ctypes.c_int64)), ctypes.cast(s, ctypes.POINTER(ctypes.c_float)),
                   cap, 0, 0, 0, 0)
        h = None
        if hit_cap > 0:
            h = np.zeros(hit_cap, np.int64)
            r.hit_docids = h.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))
            r.hit_capacity = hit_cap
        r._ints = (ctypes.c_int32 * max(cap, 1))()
        r.int_scores = ctypes.cast(r._ints, ctypes.POINTER(ctypes.c_int32))
        if info is not None:
            r.docid_scores, r.docid_scores_cap = info[0].ctypes.data, len(info[0])
            r.pair_scores, r.pair_scores_cap = info[1].ctypes.data, len(info[1])
            r.single_scores, r.single_scores_cap = info[2].ctypes.data, len(info[2])
        r._fac = None
        if nfacet_terms:
            r._fac = (np.zeros(cls.facet_cap, FACET_DT), np.zeros(nfacet_terms, np.uint64), fterms)
            r.facets, r.facets_cap = r._fac[0].ctypes.data, cls.facet_cap
            r.facet_docs = r._fac[1].ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))
        return r, d, s, h

    @staticmethod
    def _facet_terms(terms):
        """(facet_docs entries, the facet terms) of a request: its terms, when one is a facet term"""
        ft = [i for i, t in enumerate(terms) if t.field_code in FACET_FIELDS]
        return (len(terms) if ft else 0), ft

    @staticmethod
    def _pack(r, d, s, h=None, info=None) -> QueryResult:
        n = r.n
        q = QueryResult(np.frombuffer(d, dtype=np.int64, count=n).copy(),
                        np.frombuffer(s, dtype=np.float32, count=n).copy(), r.hits, r.filtered, r.docs_wanted,
                        None if h is None else h[:r.n_hit_docids].copy())
        q.int_scores = np.frombuffer(r._ints, dtype=np.int32, count=n).copy()
        if info is not None:
            q.docid_scores = info[0][:r.n_docid_scores].copy()
            q.pair_scores = info[1][:r.n_pair_scores].copy()
            q.single_scores = info[2][:r.n_single_scores].copy()
        if r._fac is not None:
            ents, docs, fterms = r._fac
            q.facets = {t: (int(docs[t]), {}) for t in fterms}
            for e in ents[:r.n_facets]:
                q.facets[int(e["term"])][1][int(e["key"])] = tuple(
                    int(e[f]) for f in ("count", "outside", "docid", "sum", "max", "min"))
        return q

    @staticmethod
    def host_lists(lists: Sequence[bytes]):
        """Host copies of the lists and the gbgpu_list array naming them
        (keep the returned tuple alive while the refs are in use)."""
        keep = [ctypes.create_string_buffer(bytes(l), max(1, len(l))) for l in lists]
        refs = (ListRef * max(len(lists), 1))(*[ListRef(ctypes.cast(k, ctypes.c_void_p), len(l))
                                                for k, l in zip(keep, lists)])
        return keep, refs

    def query(self, terms: Sequence[QTerm], lists, params: Params, cap: int = 4096,
              hit_cap: int = 0) -> QueryResult:
        """gbgpu_query over host lists: a sequence of bytes, or host_lists()'s tuple.
        hit_cap > 0 also returns the intersected docid set (up to hit_cap)."""
        n = len(terms)
        qt = (QTerm * max(n, 1))(*terms)
        keep, refs = lists if isinstance(lists, tuple) else self.host_lists(lists)
        info = self.info_arrays(params, n)
        r, d, s, h = self._result(cap, hit_cap, info, *self._facet_terms(terms))
        rc = self.lib.gbgpu_query(self.ctx, qt, n, refs, ctypes.byref(params), ctypes.byref(r))
        self.last_n_facets = r.n_facets  # the table size after ENOSPC (call again with room)
        _check(rc, "query")
        return self._pack(r, d, s, h, info)

    def query_resident(self, terms: Sequence[QTerm], handles: Sequence[int], params: Params,
                       cap: int = 4096, hit_cap: int = 0) -> QueryResult:
        n = len(terms)
        qt = (QTerm * max(n, 1))(*terms)
        hh = (ctypes.c_int32 * max(n, 1))(*handles)
        info = self.info_arrays(params, n)
        r, d, s, h = self._result(cap, hit_cap, info, *self._facet_terms(terms))
        rc = self.lib.gbgpu_query_resident(self.ctx, qt, n, hh, ctypes.byref(params), ctypes.byref(r))
        self.last_n_facets = r.n_facets
        _check(rc, "query")
        return self._pack(r, d, s, h, info)

    def set_slots(self, n: int) -> None:
        _check(self.lib.gbgpu_set_query_slots(self.ctx, n), "set_query_slots")

    def slots(self) -> int:
        return self.lib.gbgpu_query_slots(self.ctx)

    def enqueue(self, terms: Sequence[QTerm], handles: Sequence[int], params: Params, slot: int = 0) -> None:
        n = len(terms)
        qt = (QTerm * max(n, 1))(*terms)
        hh = (ctypes.c_int32 * max(n, 1))(*handles)
        _check(self.lib.gbgpu_query_slot_enqueue(self.ctx, slot, qt, n, hh, ctypes.byref(params)), "enqueue")

    def collect(self, cap: int = 4096, slot: int = 0, hit_cap: int = 0, terms=()) -> QueryResult:
        """terms: the enqueued query's terms, for its facet tables"""
        r, d, s, h = self._result(cap, hit_cap, None, *self._facet_terms(terms))
        _check(self.lib.gbgpu_query_slot_collect(self.ctx, slot, ctypes.byref(r)), "collect")
        return self._pack(r, d, s, h)

    def set_profiling(self, on: bool) -> None:
        _check(self.lib.gbgpu_set_profiling(self.ctx, 1 if on else 0))

    def last_timings(self, slot: int = 0):
        ms = (ctypes.c_float * 6)()
        sb = ctypes.c_int64()
        _check(self.lib.gbgpu_slot_timings(self.ctx, slot, ms, ctypes.byref(sb)))
        return list(ms), sb.value

    def stats(self, slot: int = 0):
        """gbgpu_slot_stats: work counts of the slot's last collected query."""
        st = (ctypes.c_int64 * 8)()
        _check(self.lib.gbgpu_slot_stats(self.ctx, slot, st))
        keys = ["scan_bytes", "g0_bytes", "probe_bytes", "candidates", "survivors", "survivor_run_bytes",
                "tree_nodes"]
        return dict(zip(keys, list(st)))

    def bandwidth_ceiling(self, nbytes: int = 2 << 30, iters: int = 10):
        r, c = ctypes.c_double(), ctypes.c_double()
        _check(self.lib.gbgpu_bandwidth_ceiling(self.ctx, nbytes, iters, ctypes.byref(r), ctypes.byref(c)))
        return r.value, c.value

    # ------------------------------------------------ Msg3a exchange (RCCL)
    @staticmethod
    def comm_unique_id() -> bytes:
        buf = ctypes.create_string_buffer(128)
        _check(load().gbgpu_comm_unique_id(buf), "gbgpu_comm_unique_id")
        return buf.raw

    def comm_init(self, nranks: int, rank: int, uid: bytes) -> None:
        b = ctypes.create_string_buffer(bytes(uid), 128)
        _check(self.lib.gbgpu_comm_init(self.ctx, nranks, rank, b), "gbgpu_comm_init")
        self._xseq = 0

    def allgather_topk(self, k: int, slot: int = 0, seq: Optional[int] = None, timeout_ms: int = -1):
        """Collects the slot's query as this shard's reply and returns the
        Msg3a merge of every rank's reply: (docids, scores float64, total hits).
        seq: the query's exchange sequence number, agreed by every rank (None:
        this engine's next, for single-threaded callers); slot < 0 sends an
        empty reply."""
        if seq is None:
            seq = self._xseq
        d = np.zeros(max(k, 1), np.int64)
        sc = np.zeros(max(k, 1), np.float64)
        n, h = ctypes.c_int32(), ctypes.c_int64()
        rc = self.lib.gbgpu_allgather_topk(self.ctx, slot, seq, timeout_ms,
                                           k, d.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                                           sc.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), ctypes.byref(n),
                                           ctypes.byref(h), None)
        # an admitted call uses its number up whatever its outcome (the rank
        # took part in the collective with an empty reply on failure); a call
        # refused before admission (bad k, ETIMEDOUT) does not: the context's
        # sequencer says which number comes next
        self._xseq = int(self.lib.gbgpu_exchange_next(self.ctx))
        _check(rc, "gbgpu_allgather_topk")
        return d[:n.value], sc[:n.value], h.value

    def merge_topk_device(self, shards, k: int, shard_hits=None):
        ns = len(shards)
        keep = []
        dptrs = (ctypes.POINTER(ctypes.c_int64) * ns)()
        sptrs = (ctypes.POINTER(ctypes.c_double) * ns)()
        cnts = (ctypes.c_int32 * ns)()
        hh = (ctypes.c_int64 * ns)(*(shard_hits or [0] * ns))
        for i, (dd, ss) in enumerate(shards):
            dd = np.ascontiguousarray(dd, dtype=np.int64)
            ss = np.ascontiguousarray(ss, dtype=np.float64)
            keep += [dd, ss]
            dptrs[i] = dd.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))
            sptrs[i] = ss.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
            cnts[i] = len(dd)
        od = np.zeros(k, np.int64)
        osc = np.zeros(k, np.float64)
        n, h = ctypes.c_int32(), ctypes.c_int64()
        _check(self.lib.gbgpu_merge_topk_device(self.ctx, ns, k, cnts, hh, dptrs, sptrs,
                                                   od.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                                                   osc.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                                                   ctypes.byref(n), ctypes.byref(h)), "gbgpu_merge_topk_device")
        return od[:n.value], osc[:n.value], h.value

    def merge_replies_device(self, req, shards, **kw):
        """gbgpu_merge_replies_device: Msg3a::mergeLists whole on the device"""
        x = FullReplies(req, shards, **kw)
        _check(self.lib.gbgpu_merge_replies_device(self.ctx, ctypes.byref(x.req), x.reps, x.n, ctypes.byref(x.out)),
               "gbgpu_merge_replies_device")
        return x.result()

    def allgather_replies(self, req, shard, seq: Optional[int] = None, timeout_ms: int = -1, **kw):
        """gbgpu_allgather_replies: this rank's full reply (None: an empty
        one) exchanged over RCCL and merged on the device"""
        if seq is None:
            seq = self._xseq
        x = FullReplies(req, [shard] if shard is not None else [], **kw)
        rc = self.lib.gbgpu_allgather_replies(self.ctx, seq, timeout_ms, ctypes.byref(x.req),
                                              x.reps if shard is not None else None, ctypes.byref(x.out))
        self._xseq = int(self.lib.gbgpu_exchange_next(self.ctx))
        _check(rc, "gbgpu_allgather_replies")
        return x.result()

    def stream(self) -> int:
        return self.lib.gbgpu_stream(self.ctx) or 0

    def merge_posdb(self, runs: Sequence[bytes], remove_neg_keys: bool, min_rec_sizes: int = -1,
                    cap: Optional[int] = None) -> bytes:
        """RdbList::merge_r -> posdbMerge_r (RdbList.cpp:3065-3568) of host runs, oldest first."""
        n = len(runs)
        refs = (ListRef * max(n, 1))()
        keep = []
        for i, r in enumerate(runs):
            b = ctypes.create_string_buffer(bytes(r), max(len(r), 1))
            keep.append(b)
            refs[i].bytes = ctypes.cast(b, ctypes.c_void_p)
            refs[i].size = len(r)
        if cap is None:
            cap = sum(len(r) for r in runs) + 64
        out = ctypes.create_string_buffer(max(cap, 1))
        osz = ctypes.c_int64()
        _check(self.lib.gbgpu_merge_posdb(self.ctx, refs, n, int(bool(remove_neg_keys)), int(min_rec_sizes), out,
                                          cap, ctypes.byref(osz)), "gbgpu_merge_posdb")
        return out.raw[:osz.value]

    def merge_posdb_device(self, ptrs: Sequence[int], sizes: Sequence[int], remove_neg_keys: bool,
                           min_rec_sizes: int, out_ptr: int, cap: int) -> int:
        """Device-resident form (pointers from torch tensors); returns the output size."""
        n = len(ptrs)
        p = (ctypes.c_void_p * max(n, 1))(*ptrs)
        sz = (ctypes.c_int64 * max(n, 1))(*sizes)
        osz = ctypes.c_int64()
        _check(self.lib.gbgpu_merge_posdb_device(self.ctx, p, sz, n, int(bool(remove_neg_keys)), int(min_rec_sizes),
                                                 out_ptr, cap, ctypes.byref(osz)), "gbgpu_merge_posdb_device")
        return osz.value

    def merge_last_key(self):
        """RdbList::m_lastKey after the last merge (18 bytes), None if it wrote nothing."""
        k = ctypes.create_string_buffer(18)
        rc = self.lib.gbgpu_merge_last_key(self.ctx, k)
        if rc == 2:  # ENOENT
            return None
        _check(rc, "gbgpu_merge_last_key")
        return k.raw

    def merge_input_left(self) -> bool:
        """Whether the last merge stopped at its bound with input keys left
        (posdbMerge_r's numLists > 0 at its end, RdbList.cpp:3541-3542)."""
        v = ctypes.c_int32()
        _check(self.lib.gbgpu_merge_input_left(self.ctx, ctypes.byref(v)), "gbgpu_merge_input_left")
        return bool(v.value)

    def merge_timings(self):
        ms = (ctypes.c_float * 6)()
        nk, nt = ctypes.c_int64(), ctypes.c_int64()
        _check(self.lib.gbgpu_merge_timings(self.ctx, ms, ctypes.byref(nk), ctypes.byref(nt)))
        return list(ms), nk.value, nt.value

    def merge_path(self):
        """2: the last merge ran (the decoded-key pipeline), 0: none yet."""
        return self.lib.gbgpu_merge_path(self.ctx)

    def last_topk_device(self):
        p = ctypes.c_void_p()
        n = ctypes.c_int32()
        _check(self.lib.gbgpu_last_topk_device(self.ctx, ctypes.byref(p), ctypes.byref(n)))
        return p.value, n.value


class Seq:
    """gbgpu_seq: admits one caller at a time in increasing sequence number
    (include/gbgpu.h "Exchange ordering").  Host code only."""

    def __init__(self, first: int = 0):
        self.lib = load()
        h = ctypes.c_void_p()
        _check(self.lib.gbgpu_seq_open(first, ctypes.byref(h)), "gbgpu_seq_open")
        self.h = h

    def enter(self, seq: int, timeout_ms: int = -1) -> None:
        _check(self.lib.gbgpu_seq_enter(self.h, seq, timeout_ms), "gbgpu_seq_enter")

    def leave(self, seq: int) -> None:
        _check(self.lib.gbgpu_seq_leave(self.h, seq), "gbgpu_seq_leave")

    def next(self) -> int:
        return int(self.lib.gbgpu_seq_next(self.h))

    def close(self) -> None:
        if self.h:
            self.lib.gbgpu_seq_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def merge_topk(shards, k: int):
    """Msg3a::mergeLists over [(docids int64[], scores float64[]), ...] (the
    Msg39 reply's double scores; float32 input is widened as Msg39 does)."""
    lib = load()
    ns = len(shards)
    keep = []
    dptrs = (ctypes.POINTER(ctypes.c_int64) * max(ns, 1))()
    sptrs = (ctypes.POINTER(ctypes.c_double) * max(ns, 1))()
    cnts = (ctypes.c_int32 * max(ns, 1))()
    for i, (d, s) in enumerate(shards):
        d = np.ascontiguousarray(d, dtype=np.int64)
        s = np.ascontiguousarray(s, dtype=np.float64)
        keep += [d, s]
        dptrs[i] = d.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))
        sptrs[i] = s.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
        cnts[i] = len(d)
    od = np.zeros(max(k, 1), dtype=np.int64)
    os_ = np.zeros(max(k, 1), dtype=np.float64)
    n = ctypes.c_int32()
    _check(lib.gbgpu_merge_topk(dptrs, sptrs, cnts, ns, k, od.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                                os_.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), ctypes.byref(n)))
    return od[:n.value], os_[:n.value]
