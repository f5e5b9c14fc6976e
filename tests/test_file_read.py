"""The read path into HBM: resident Posdb file images and
termlists cut from them on the device (gbgpu_file_upload / gbgpu_file_list,
RdbScan.cpp:319-361 over HBM).

  * whole termlists cut from a file answer the reference's fixtures exactly;
  * a piece starting at a compressed key (12-byte run head or 6-byte position
    key), with the full key RdbScan would write in its place, answers exactly
    what the same bytes uploaded from the host answer;
  * a wrong or missing map key, a cut that is not a key start and an
    out-of-range cut are refused."""
import glob
import os

import numpy as np
import pytest

from test_golden import check, load_query

HERE = os.path.dirname(os.path.abspath(__file__))
FIX = sorted(glob.glob(os.path.join(HERE, "golden", "q_*.npz")))
IDS = [os.path.basename(p)[2:-4] for p in FIX]


def key_starts(lst: bytes):
    """(offset, key size) of every key in a Posdb list (Posdb.h:271-288)."""
    out, off = [], 0
    while off < len(lst):
        b0 = lst[off]
        ks = 6 if b0 & 0x04 else 12 if b0 & 0x02 else 18
        out.append((off, ks))
        off += ks
    assert off == len(lst)
    return out


def full_key(lst: bytes, starts, i):
    """The 18-byte key of the i-th key: its stored bytes, the docid half of the
    last 12/18-byte key and the termid of the last 18-byte key before it."""
    off, ks = starts[i]
    mid = next(o for o, k in reversed(starts[:i + 1]) if k >= 12)
    top = next(o for o, k in reversed(starts[:i + 1]) if k == 18)
    k = bytearray(lst[top:top + 18])
    k[6:12] = lst[mid + 6:mid + 12]
    k[0:ks] = lst[off:off + ks]
    k[0] &= 0xF9
    return bytes(k)


def test_key_walk_and_full_key_roundtrip():
    """Host helpers on a fixture list (CPU): every key restored to 18 bytes
    re-compresses to the list's bytes."""
    import gbgpu
    terms, lists, params, exp = load_query(FIX[0])
    lst = next(x for x in lists if len(x) > 18)
    st = key_starts(lst)
    keys = b"".join(full_key(lst, st, i) for i in range(len(st)))
    assert gbgpu.compress(keys) == lst


def _file(lists):
    offs, o = [], 0
    for x in lists:
        offs.append(o)
        o += len(x)
    return b"".join(lists), offs


@pytest.mark.gpu
@pytest.mark.parametrize("path", FIX, ids=IDS)
def test_gpu_file_termlists_vs_reference(engine, path):
    terms, lists, params, exp = load_query(path)
    blob, offs = _file(lists)
    fh = engine.file_upload(blob)
    hs = []
    try:
        hs = [engine.file_list(fh, o, len(x)) for o, x in zip(offs, lists)]
        r = engine.query_resident(terms, hs, params, cap=1 << 16, hit_cap=max(1, exp["hits"]))
        check(dict(docids=r.docids, scores=r.scores, hits=r.hits, docs_wanted=r.docs_wanted, filtered=r.filtered,
                   hit_docids=r.hit_docids), exp, os.path.basename(path))
    finally:
        for h in hs:
            engine.free(h)
        engine.file_free(fh)


PIECE_FIX = FIX[::3]


@pytest.mark.gpu
@pytest.mark.parametrize("kind", [12, 6])
@pytest.mark.parametrize("path", PIECE_FIX, ids=IDS[::3])
def test_gpu_file_pieces_match_host_upload(engine, path, kind):
    """Every list cut at a key of size `kind` in its second half: the device
    cut and the host-built list (map key + the rest) answer the same."""
    terms, lists, params, exp = load_query(path)
    blob, offs = _file(lists)
    rng = np.random.default_rng(len(blob))
    cuts, host = [], []
    for x in lists:
        st = key_starts(x) if x else []
        cand = [i for i, (o, k) in enumerate(st) if k == kind and i >= len(st) // 2]
        if not cand:
            cuts.append((0, None))  # the whole list
            host.append(x)
            continue
        i = int(rng.choice(cand))
        k18 = full_key(x, st, i)
        cuts.append((st[i][0], k18))
        host.append(k18 + x[st[i][0] + kind:])
    fh = engine.file_upload(blob)
    hd, hh = [], []
    try:
        for (c, k18), o, x in zip(cuts, offs, lists):
            hd.append(engine.file_list(fh, o + c, len(x) - c, k18))
        hh = [engine.upload(x) for x in host]
        a = engine.query_resident(terms, hd, params, cap=1 << 16, hit_cap=1 << 20)
        b = engine.query_resident(terms, hh, params, cap=1 << 16, hit_cap=1 << 20)
        assert a.hits == b.hits and a.docs_wanted == b.docs_wanted and a.filtered == b.filtered
        assert np.array_equal(a.docids, b.docids)
        assert np.array_equal(a.scores.view(np.uint32), b.scores.view(np.uint32))
        assert np.array_equal(a.hit_docids, b.hit_docids)
    finally:
        for h in hd + hh:
            engine.free(h)
        engine.file_free(fh)


@pytest.mark.gpu
def test_gpu_file_list_refusals(engine):
    import gbgpu
    terms, lists, params, exp = load_query(FIX[0])
    x = next(x for x in lists if len(x) > 64)
    st = key_starts(x)
    i12 = next(i for i, (o, k) in enumerate(st) if k == 12)
    i6 = next(i for i, (o, k) in enumerate(st) if k == 6)
    fh = engine.file_upload(x)
    try:
        def code(*a):
            with pytest.raises(gbgpu.GbgpuError) as e:
                engine.file_list(fh, *a)
            return e.value.code

        o12 = st[i12][0]
        good = full_key(x, st, i12)
        bad = bytearray(good)
        bad[9] ^= 0x10  # another docid
        assert code(o12, len(x) - o12, bytes(bad)) == 22  # EINVAL: not this key
        assert code(o12, len(x) - o12, None) == 22  # a compressed key needs the map's key
        if i6 > 0 and st[i6 - 1][1] == 12:
            # the docid half of a run head is not a key start
            assert code(st[i6 - 1][0] + 6, len(x) - st[i6 - 1][0] - 6, good) == gbgpu.GBGPU_ECORRUPT
        assert code(0, len(x) + 6, None) == 22  # past the file
        assert code(3, 18, None) == 22  # not on a 6-byte unit
        h = engine.file_list(fh, o12, len(x) - o12, good)
        engine.free(h)
    finally:
        engine.file_free(fh)
    with pytest.raises(gbgpu.GbgpuError):
        engine.file_free(fh)  # already freed
