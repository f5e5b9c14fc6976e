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
_proc = None


class OrcResult(ctypes.Structure):
    _fields_ = [("hits", ctypes.c_int64), ("filtered", ctypes.c_int32), ("docs_wanted", ctypes.c_int32),
                ("n", ctypes.c_int32), ("corrupt", ctypes.c_int32)]


def available() -> bool:
    return os.access(EXE, os.X_OK)


def _p():
    global _proc
    if _proc is None or _proc.poll() is not None:
        _proc = subprocess.Popen([EXE], stdin=subprocess.PIPE, stdout=subprocess.PIPE)
        atexit.register(close)
    return _proc


def close():
    global _proc
    if _proc is not None:
        try:
            _proc.stdin.close()
            _proc.wait(timeout=10)
        except Exception:
            _proc.kill()
        _proc = None


def _read(n):
    p = _p()
    b = p.stdout.read(n)
    if len(b) != n:
        rc = p.poll()
        raise RuntimeError(f"gbref died (rc={rc}) after {len(b)}/{n} bytes")
    return b


def query(terms, lists, params, cap=4096, votes=False, reps=1, white=None):
    """Same result dict as oracle_binding.query (+ 'votes', 'seconds').
    white: the whitelist lists (Msg2::m_whiteLists) when params.use_whitelist."""
    p = _p()
    qt = (gbgpu.QTerm * max(1, len(terms)))(*terms)
    req = [struct.pack("<ii", 1, len(terms)), bytes(params), bytes(qt)[:ctypes.sizeof(gbgpu.QTerm) * len(terms)]]
    for l in lists:
        req.append(struct.pack("<q", len(l)))
        req.append(bytes(l))
    req.append(struct.pack("<iii", cap, 1 if votes else 0, reps))
    white = list(white or [])
    req.append(struct.pack("<i", len(white)))
    for l in white:
        req.append(struct.pack("<q", len(l)))
        req.append(bytes(l))
    p.stdin.write(b"".join(req))
    p.stdin.flush()
    r = OrcResult.from_buffer_copy(_read(ctypes.sizeof(OrcResult)))
    d = np.frombuffer(_read(8 * r.n), np.int64).copy()
    s = np.frombuffer(_read(4 * r.n), np.float32).copy()
    (nv,) = struct.unpack("<q", _read(8))
    v = np.frombuffer(_read(8 * nv), np.int64).copy()
    (sec,) = struct.unpack("<d", _read(8))
    info = []
    for _ in range(3):  # m_scoreInfoBuf, m_pairScoreBuf, m_singleScoreBuf
        (nb,) = struct.unpack("<q", _read(8))
        info.append(_read(nb) if nb else b"")
    if r.corrupt < 0:
        raise RuntimeError(f"gbref query rc={-r.corrupt}")
    return dict(docids=d, scores=s, hits=r.hits, filtered=r.filtered, docs_wanted=r.docs_wanted,
                corrupt=r.corrupt, votes=v, seconds=sec, score_info=info[0], pair_scores=info[1],
                single_scores=info[2])


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
