"""ctypes view of oracle/liboracle.so -- the CPU restatement used as the checker.

Test infrastructure only (see oracle/posdb_oracle.h)."""
import ctypes
import os

import numpy as np

import gbgpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_lib = None


class OrcResult(ctypes.Structure):
    _fields_ = [("hits", ctypes.c_int64), ("filtered", ctypes.c_int32), ("docs_wanted", ctypes.c_int32),
                ("n", ctypes.c_int32), ("corrupt", ctypes.c_int32)]


def lib():
    global _lib
    if _lib is None:
        _lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "liboracle.so"))
        _lib.orc_last_facets.argtypes = [ctypes.POINTER(ctypes.c_int32), ctypes.c_int]
        _lib.orc_last_stale.argtypes = [ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32)]
        _lib.orc_last_stale.restype = None
        _lib.orc_query.argtypes = [ctypes.POINTER(gbgpu.QTerm), ctypes.POINTER(ctypes.c_void_p),
                                   ctypes.POINTER(ctypes.c_int64), ctypes.c_int, ctypes.POINTER(gbgpu.Params),
                                   ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_float), ctypes.c_int,
                                   ctypes.POINTER(OrcResult)]
        _lib.orc_intersect.argtypes = [ctypes.POINTER(gbgpu.QTerm), ctypes.POINTER(ctypes.c_void_p),
                                       ctypes.POINTER(ctypes.c_int64), ctypes.c_int,
                                       ctypes.POINTER(ctypes.c_int64), ctypes.c_int64,
                                       ctypes.POINTER(gbgpu.Params)]
        _lib.orc_intersect.restype = ctypes.c_int64
        _lib.orc_weights.argtypes = [ctypes.POINTER(ctypes.c_float)] * 5
        _lib.orc_posdb_merge.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_int64),
                                         ctypes.c_int, ctypes.c_int, ctypes.c_int64, ctypes.c_void_p,
                                         ctypes.c_int64]
        _lib.orc_posdb_merge.restype = ctypes.c_int64
        _lib.orc_msg3a_merge.argtypes = [ctypes.POINTER(ctypes.POINTER(ctypes.c_int64)),
                                         ctypes.POINTER(ctypes.POINTER(ctypes.c_double)),
                                         ctypes.POINTER(ctypes.c_int32), ctypes.c_int, ctypes.c_int32,
                                         ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_double)]
        _lib.orc_msg3a_merge.restype = ctypes.c_int32
    return _lib


def _lists(lists):
    keep = [ctypes.create_string_buffer(l, max(1, len(l))) for l in lists]
    ptrs = (ctypes.c_void_p * max(1, len(lists)))(*[ctypes.cast(k, ctypes.c_void_p) for k in keep])
    sizes = (ctypes.c_int64 * max(1, len(lists)))(*[len(l) for l in lists])
    return keep, ptrs, sizes


def query(terms, lists, params, cap=4096):
    L = lib()
    keep, ptrs, sizes = _lists(lists)
    qt = (gbgpu.QTerm * max(1, len(terms)))(*terms)
    d = np.zeros(cap, np.int64)
    s = np.zeros(cap, np.float32)
    r = OrcResult()
    rc = L.orc_query(qt, ptrs, sizes, len(terms), ctypes.byref(params),
                     d.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                     s.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), cap, ctypes.byref(r))
    if rc:
        raise RuntimeError(f"orc_query rc={rc}")
    sd, su = ctypes.c_int32(), ctypes.c_int32()
    L.orc_last_stale(ctypes.byref(sd), ctypes.byref(su))
    return dict(docids=d[:r.n].copy(), scores=s[:r.n].copy(), hits=r.hits, filtered=r.filtered,
                docs_wanted=r.docs_wanted, corrupt=r.corrupt, facets=last_facets(),
                stale=(sd.value, su.value))


def last_facets():
    """the facet tables of the last orc_query: {term: (docs, {key: (count,
    outside, docid, sum, max, min)})}, as ref_binding reads the reference's"""
    L = lib()
    cap = 1 << 22
    w = np.zeros(cap, np.int32)
    n = L.orc_last_facets(w.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), cap)
    assert n >= 1
    out, k = {}, 1
    for _ in range(int(w[0])):
        term = int(w[k])
        docs = int(w[k + 1:k + 3].view(np.uint64)[0])
        ne = int(w[k + 3])
        k += 4
        ents = {}
        for _ in range(ne):
            r = w[k:k + 9]
            ents[int(r[0])] = (int(r[1]), int(r[2]), int(r[3:5].view(np.int64)[0]), int(r[5:7].view(np.int64)[0]),
                               int(r[7]), int(r[8]))
            k += 9
        out[term] = (docs, ents)
    return out


def intersect(terms, lists, cap=1 << 24, params=None):
    L = lib()
    keep, ptrs, sizes = _lists(lists)
    qt = (gbgpu.QTerm * max(1, len(terms)))(*terms)
    d = np.zeros(cap, np.int64)
    n = L.orc_intersect(qt, ptrs, sizes, len(terms), d.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), cap,
                        ctypes.byref(params) if params is not None else None)
    if n < 0:
        raise RuntimeError(f"orc_intersect rc={n}")
    return d[:n].copy()


def weights():
    arrs = [np.zeros(32, np.float32), np.zeros(16, np.float32), np.zeros(16, np.float32),
            np.zeros(11, np.float32), np.zeros(16, np.float32)]
    lib().orc_weights(*[a.ctypes.data_as(ctypes.POINTER(ctypes.c_float)) for a in arrs])
    return dict(density=arrs[0], wordspam=arrs[1], linker=arrs[2], hashgroup=arrs[3], diversity=arrs[4])


def msg3a_merge(shards, docs_to_get):
    """oracle/msg3a_oracle.c: Msg3a::mergeLists over [(docids, scores float64), ...]."""
    L = lib()
    ns = len(shards)
    keep = []
    dp = (ctypes.POINTER(ctypes.c_int64) * max(ns, 1))()
    sp = (ctypes.POINTER(ctypes.c_double) * max(ns, 1))()
    cnt = (ctypes.c_int32 * max(ns, 1))()
    for i, (d, s) in enumerate(shards):
        d = np.ascontiguousarray(d, np.int64)
        s = np.ascontiguousarray(s, np.float64)
        keep += [d, s]
        dp[i] = d.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))
        sp[i] = s.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
        cnt[i] = len(d)
    od = np.zeros(max(docs_to_get, 1), np.int64)
    os_ = np.zeros(max(docs_to_get, 1), np.float64)
    n = L.orc_msg3a_merge(dp, sp, cnt, ns, docs_to_get, od.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                          os_.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
    if n < 0:
        raise RuntimeError(f"orc_msg3a_merge rc={n}")
    return od[:n].copy(), os_[:n].copy()


def msg3a_full(req, shards):
    """oracle/msg3a_oracle.c orc_msg3a_full: Msg3a::mergeLists whole over full
    replies (msg3a_cases.full_cases); the same dict as gbgpu.merge_replies."""
    L = lib()
    if not getattr(L, "_full", False):
        vp = ctypes.c_void_p
        L.orc_msg3a_full.argtypes = [ctypes.POINTER(gbgpu.MergeReq), ctypes.POINTER(gbgpu.Reply), ctypes.c_int,
                                     vp, vp, vp, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int64),
                                     vp, vp, ctypes.c_int32, ctypes.POINTER(ctypes.c_int32)]
        L._full = True
    x = gbgpu.FullReplies(req, shards)
    n, h, nf = ctypes.c_int32(), ctypes.c_int64(), ctypes.c_int32()
    rc = L.orc_msg3a_full(ctypes.byref(x.req), x.reps, x.n, x.od.ctypes.data, x.os.ctypes.data, x.orec.ctypes.data,
                          ctypes.byref(n), ctypes.byref(h), x.ofd.ctypes.data, x.ofac.ctypes.data, x.out.facets_cap,
                          ctypes.byref(nf))
    if rc:
        raise RuntimeError(f"orc_msg3a_full rc={rc}")
    x.out.n, x.out.hits, x.out.n_facets = n.value, h.value, nf.value
    return x.result()
