"""Driver for oracle/_ref/gbref -- the REFERENCE's own PosdbTable / TopTree /
RdbList::merge_r compiled unmodified from /root/reference (oracle/ref.mk).

Test infrastructure only: it pins the CPU restatement (oracle/posdb_oracle.c)
and generates tests/golden/ fixtures.  It exists only where the reference
sources were present at build time; ``available()`` says whether it does.
One long-lived child process serves every request over stdin/stdout."""
import atexit
import ctypes
import os
import struct
import subprocess

import numpy as np

import gbgpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.environ.get('GBREF_EXE', os.path.join(ROOT, 'oracle', '_ref', 'gbref'))
# the same harness with INTEGRATION.md's adapter and libgbgpu.so linked in
# (oracle/ref.mk): op 4 runs the adapter body in the reference's Msg39 sequence
EXE_GPU = os.path.join(ROOT, 'oracle', '_ref', 'gbref_gpu')
_procs = {}


class OrcResult(ctypes.Structure):
    _fields_ = [("hits", ctypes.c_int64), ("filtered", ctypes.c_int32), ("docs_wanted", ctypes.c_int32),
                ("n", ctypes.c_int32), ("corrupt", ctypes.c_int32)]


def available(exe=None) -> bool:
    return os.access(exe or EXE, os.X_OK)


def _p(exe=None):
    exe = exe or EXE
    pr = _procs.get(exe)
    if pr is None or pr.poll() is not None:
        pr = subprocess.Popen([exe], stdin=subprocess.PIPE, stdout=subprocess.PIPE)
        _procs[exe] = pr
        if len(_procs) == 1:
            atexit.register(close)
    return pr


def close():
    for exe, pr in list(_procs.items()):
        try:
            pr.stdin.close()
            pr.wait(timeout=10)
        except Exception:
            pr.kill()
        del _procs[exe]


def _read(n, exe=None):
    p = _p(exe)
    b = p.stdout.read(n)
    if len(b) != n:
        rc = p.poll()
        raise RuntimeError(f"gbref died (rc={rc}) after {len(b)}/{n} bytes")
    return b


def query(terms, lists, params, cap=4096, votes=False, reps=1, white=None, mode=None, exe=None, op=None,
          op9=(0, 0, 3)):
    """Same result dict as oracle_binding.query (+ 'votes', 'seconds').
    white: the whitelist lists (Msg2::m_whiteLists) when params.use_whitelist.
    mode (op 4, the gbref_gpu build): 0 the CPU body, 1 INTEGRATION.md's
    adapter; adds 'answered' (passes the adapter answered), 'used_nodes'
    (TopTree::m_numUsedNodes) and 'int_scores' (the nodes' m_intScore)."""
    p = _p(exe)
    rd = lambda n: _read(n, exe)  # noqa: E731
    qt = (gbgpu.QTerm * max(1, len(terms)))(*terms)
    if op == 7:
        head = struct.pack("<ii", 7, len(terms))
    elif op == 9:
        head = struct.pack("<iiiiii", 9, mode, *op9, len(terms))
    else:
        head = struct.pack("<ii", 1, len(terms)) if mode is None else struct.pack("<iii", 4, mode, len(terms))
    req = [head, bytes(params), bytes(qt)[:ctypes.sizeof(gbgpu.QTerm) * len(terms)]]
    for l in lists:
        req.append(struct.pack("<q", len(l)))
        req.append(bytes(l))
    req.append(struct.pack("<iii", cap, 1 if votes else 0, reps))
    white = list(white or [])
    req.append(struct.pack("<i", len(white)))
    for l in white:
        req.append(struct.pack("<q", len(l)))
        req.append(bytes(l))
    btok = list(getattr(params, "_btok", None) or [])  # a boolean query's expression
    req.append(struct.pack("<i", len(btok)))
    req.append(np.asarray(btok, np.int32).tobytes())
    fr = list(getattr(params, "_franges", None) or [])  # facet ranges: (term, a[], b[]) as int32 bits
    req.append(struct.pack("<i", len(fr)))
    for term, a, b in fr:
        req.append(struct.pack("<ii", term, len(a)))
        req.append(np.asarray(a, np.int32).tobytes())
        req.append(np.asarray(b, np.int32).tobytes())
    p.stdin.write(b"".join(req))
    p.stdin.flush()
    r = OrcResult.from_buffer_copy(rd(ctypes.sizeof(OrcResult)))
    d = np.frombuffer(rd(8 * r.n), np.int64).copy()
    s = np.frombuffer(rd(4 * r.n), np.float32).copy()
    (nv,) = struct.unpack("<q", rd(8))
    v = np.frombuffer(rd(8 * nv), np.int64).copy()
    (sec,) = struct.unpack("<d", rd(8))
    info = []
    for _ in range(3):  # m_scoreInfoBuf, m_pairScoreBuf, m_singleScoreBuf
        (nb,) = struct.unpack("<q", rd(8))
        info.append(rd(nb) if nb else b"")
    (bng,) = struct.unpack("<i", rd(4))
    btable = rd(((1 << bng) + 7) // 8) if bng >= 0 else None
    (nft,) = struct.unpack("<i", rd(4))
    facets = {}
    for _ in range(nft):  # QueryTerm::m_facetHashTable: term -> (docs, {key: FacetEntry tuple})
        term, docs, ne = struct.unpack("<iQi", rd(16))
        ents = {}
        for _ in range(ne):
            key, cnt, outside, docid, fsum, fmax, fmin = struct.unpack("<iiiqqii", rd(36))
            ents[key] = (cnt, outside, docid, fsum, fmax, fmin)
        facets[term] = (docs, ents)
    out = dict(docids=d, scores=s, hits=r.hits, filtered=r.filtered, docs_wanted=r.docs_wanted,
               corrupt=r.corrupt, votes=v, seconds=sec, score_info=info[0], pair_scores=info[1],
               single_scores=info[2], bool_groups=bng, bool_table=btable, facets=facets)
    if op == 7:
        (no,) = struct.unpack("<i", rd(4))
        if no < 0:
            raise RuntimeError(f"gbref msg3a rc={-no}")
        out["msg3a_docids"] = np.frombuffer(rd(8 * no), np.int64).copy()
        out["msg3a_scores"] = np.frombuffer(rd(8 * no), np.float64).copy()
        grc, gn, gh = struct.unpack("<iiq", rd(16))
        out.update(shard_rc=grc, shard_hits=gh)
        out["shard_docids"] = np.frombuffer(rd(8 * gn), np.int64).copy()
        out["shard_scores"] = np.frombuffer(rd(8 * gn), np.float64).copy()
    if op == 9:
        out["merged"] = _read_merged(rd)
    elif mode is not None:
        answered, used = struct.unpack("<ii", rd(8))
        out.update(answered=answered, used_nodes=used, int_scores=np.frombuffer(rd(4 * r.n), np.int32).copy())
        (npl,) = struct.unpack("<i", rd(4))
        w = list(np.frombuffer(rd(4 * npl), np.int32))
        groups, k = [], 1
        for _ in range(w[0] if w else 0):  # setQueryTermInfo's QueryTermInfos
            flags0, nsub = int(w[k]), int(w[k + 1])
            subs = [(int(w[k + 2 + 2 * x]), int(w[k + 3 + 2 * x])) for x in range(nsub)]
            groups.append(dict(flags0=flags0, subs=subs))
            k += 2 + 2 * nsub
        out["plan"] = groups
    if r.corrupt < 0:
        raise RuntimeError(f"gbref query rc={-r.corrupt}")
    return out


def shard_msg3a(terms, lists, params, mode, family=0, hide=0, nsites=3, white=None, exe=None):
    """op 9 (gbref_gpu): the query through Msg39 (mode 0 the CPU body, 1
    INTEGRATION.md's adapter), its reply built as Msg39 builds it over a
    synthetic clusterdb (CR_OK nodes, cluster records, facet lists), and
    that reply merged by Msg3a (mode 0 the reference's gotAllShardReplies
    sums and mergeLists, 1 INTEGRATION.md 4b's gbgpuMsg3aReplies over the
    one-rank exchange).  Returns the query result with 'merged'."""
    return query(terms, lists, params, cap=1 << 16, white=white, mode=mode, exe=exe or EXE_GPU, op=9,
                 op9=(family, hide, nsites))


def posdb_merge(lists, remove_neg_keys, min_rec_sizes=-1, timed=False):
    p = _p()
    req = [struct.pack("<iiiq", 2, len(lists), 1 if remove_neg_keys else 0, min_rec_sizes)]
    for l in lists:
        req.append(struct.pack("<q", len(l)))
        req.append(bytes(l))
    p.stdin.write(b"".join(req))
    p.stdin.flush()
    (n,) = struct.unpack("<q", _read(8))
    out = _read(n) if n > 0 else b""
    (sec,) = struct.unpack("<d", _read(8))
    if n < 0:
        raise RuntimeError(f"gbref merge rc={n}")
    if timed:
        return out, sec
    return out


def shard_query(terms, lists, params, white=None, exe=None):
    """op 7 (gbref_gpu): the query through the reference's CPU body, its
    TopTree merged by the reference's Msg3a::mergeLists as the one shard's
    reply ('msg3a_docids' / 'msg3a_scores'), and the same query through
    INTEGRATION.md's gbgpuShardQuery as shard 0 of a one-rank RCCL
    exchange ('shard_rc', 'shard_docids', 'shard_scores', 'shard_hits')."""
    return query(terms, lists, params, cap=1 << 16, white=white, exe=exe or EXE_GPU, op=7)


def posdb_merge_r(lists, remove_neg_keys, min_rec_sizes=-1, start_key=None, end_key=None, mode=0, exe=None):
    """op 6: RdbList::merge_r for posdb with a key range (mode 0), or with
    INTEGRATION.md's gbgpuMergePosdb where merge_r calls posdbMerge_r (mode 1,
    gbref_gpu).  Returns dict(list, last_key, last_valid, end_key, answered)."""
    p = _p(exe)
    sk = bytes(start_key) if start_key is not None else bytes(18)
    ek = bytes(end_key) if end_key is not None else b"\xff" * 18
    req = [struct.pack("<iiiiq", 6, mode, len(lists), 1 if remove_neg_keys else 0, min_rec_sizes), sk, ek]
    for l in lists:
        req.append(struct.pack("<q", len(l)))
        req.append(bytes(l))
    p.stdin.write(b"".join(req))
    p.stdin.flush()
    rd = lambda n: _read(n, exe)  # noqa: E731
    (n,) = struct.unpack("<q", rd(8))
    out = rd(n) if n > 0 else b""
    lk = rd(18)
    (lv,) = struct.unpack("<i", rd(4))
    ek2 = rd(18)
    (ans,) = struct.unpack("<i", rd(4))
    if n < 0:
        raise RuntimeError(f"gbref merge_r rc={n}")
    return dict(list=out, last_key=lk, last_valid=lv, end_key=ek2, answered=ans)


def msg3a_merge(shards, docs_to_get):
    """The reference's own Msg3a::mergeLists (Msg3a.cpp:971-1503) over
    [(docids int64[], scores float64[]), ...] replies; no site clustering.
    Returns (docids int64[], scores float64[])."""
    p = _p()
    req = [struct.pack("<iii", 3, len(shards), docs_to_get)]
    for d, s in shards:
        d = np.ascontiguousarray(d, np.int64)
        s = np.ascontiguousarray(s, np.float64)
        assert len(d) == len(s)
        req += [struct.pack("<i", len(d)), d.tobytes(), s.tobytes()]
    p.stdin.write(b"".join(req))
    p.stdin.flush()
    (n,) = struct.unpack("<i", _read(4))
    if n < 0:
        raise RuntimeError(f"gbref msg3a rc={-n}")
    d = np.frombuffer(_read(8 * n), np.int64).copy()
    s = np.frombuffer(_read(8 * n), np.float64).copy()
    return d, s


def _read_merged(rd):
    """write_merged's response -> dict(docids, scores, recs, hits, fdocs, tables)"""
    from msg3a_cases import FE
    (n,) = struct.unpack("<i", rd(4))
    if n < 0:
        return dict(rc=-n)
    d = np.frombuffer(rd(8 * n), np.int64).copy()
    s = np.frombuffer(rd(8 * n), np.float64).copy()
    (hr,) = struct.unpack("<i", rd(4))
    recs = rd(12 * n) if hr else None
    (hits, nqt) = struct.unpack("<qi", rd(12))
    fdocs = np.frombuffer(rd(8 * nqt), np.int64).copy()
    tables = []
    for _ in range(nqt):
        (ne,) = struct.unpack("<i", rd(4))
        tables.append(np.frombuffer(rd(36 * ne), FE).copy())
    return dict(rc=0, docids=d, scores=s, recs=recs, hits=hits, fdocs=fdocs, tables=tables)


def msg3a_full(req, shards, exe=None):
    """op 8: the reference's own Msg3a::mergeLists over full Msg39Replies
    (cluster records, facet lists, facet counts; msg3a_cases.full_cases),
    with the hits and facet counts summed as gotAllShardReplies does."""
    p = _p(exe)
    nqt = len(req["tids"])
    out = [struct.pack("<7i", 8, len(shards), req["docs_to_get"], req["clus"], req["hide"], req["family"], nqt),
           np.asarray(req["tids"], np.int64).tobytes(), np.asarray(req["fcs"], np.int32).tobytes()]
    for s in shards:
        n = len(s["docids"])
        out.append(struct.pack("<ii", n, 1 if s["recs"] is not None else 0))
        out += [np.asarray(s["docids"], np.int64).tobytes(), np.asarray(s["scores"], np.float64).tobytes()]
        if s["recs"] is not None:
            assert len(s["recs"]) == 12 * n
            out.append(s["recs"])
        out.append(struct.pack("<ii", s["hits"], len(s["facets"])))
        out.append(s["facets"])
        fc = s.get("fcounts")
        out.append(struct.pack("<i", 1 if fc is not None else 0))
        if fc is not None:
            out.append(np.asarray(fc, np.int64).tobytes())
    p.stdin.write(b"".join(out))
    p.stdin.flush()
    return _read_merged(lambda n: _read(n, exe))
