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

import gbgpu
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

        def run(hs):
            try:
                return engine.query_resident(terms, hs, params, cap=1 << 16, hit_cap=1 << 20)
            except gbgpu.GbgpuError as e:
                return e.code

        a, b = run(hd), run(hh)
        if isinstance(a, int) or isinstance(b, int):
            # a cut can leave docids whose trailing group merges empty (the
            # stale-mbuf case), which site clustering declines: both alike
            assert a == b == gbgpu.GBGPU_EUNSUPPORTED and params.site_clustering
            return
        assert a.hits == b.hits and a.docs_wanted == b.docs_wanted and a.filtered == b.filtered
        assert np.array_equal(a.docids, b.docids)
        assert np.array_equal(a.scores.view(np.uint32), b.scores.view(np.uint32))
        assert np.array_equal(a.hit_docids, b.hit_docids)
    finally:
        for h in hd + hh:
            engine.free(h)
        engine.file_free(fh)


@pytest.mark.gpu
@pytest.mark.parametrize("slots", [1, 3])
def test_gpu_recut_lists_answer_as_resident(engine, slots):
    """Termlists cut, queried, freed and cut again from one resident file, as
    the read path serves query after query (bench.py's file_read leg): every
    answer equals the same lists' uploaded once.  The big list re-cut into
    the memory its predecessor just left was scanned from stale bytes while
    lists came from the stream-ordered pool (round 6: wrong top docids and
    second-long probes in 1-in-2 queries at config 2's 180 MB list)."""
    from workload import config_two_term, generate
    n = 30_000_000
    q = config_two_term(n, docs_to_get=100, seed=7)
    lists = generate(q, n, doc_begin=0, doc_end=n, threads=8)
    p = q.params()
    hs = [engine.upload(x) for x in lists]
    blob, offs = _file(lists)
    fh = engine.file_upload(blob)
    del blob
    engine.set_slots(max(slots, engine.slots()))
    live = {}
    try:
        ref = engine.query_resident(q.terms, hs, p)
        for i in range(12 + slots):
            sl = i % slots
            if sl in live:
                r = engine.collect(cap=4096, slot=sl)
                for h in live.pop(sl):
                    engine.free(h)
                assert r.hits == ref.hits and np.array_equal(r.docids, ref.docids), i
                assert np.array_equal(r.scores.view(np.uint32), ref.scores.view(np.uint32)), i
            if i < 12:
                if i % 2:  # a query's cuts together (gbgpu_file_lists) and one by one
                    fl = engine.file_lists(fh, offs, [len(x) for x in lists])
                else:
                    fl = [engine.file_list(fh, o, len(x)) for o, x in zip(offs, lists)]
                engine.enqueue(q.terms, fl, p, slot=sl)
                live[sl] = fl
    finally:
        for sl, fl in live.items():
            engine.collect(cap=4096, slot=sl)
            for h in fl:
                engine.free(h)
        for h in hs:
            engine.free(h)
        engine.file_free(fh)


@pytest.mark.gpu
@pytest.mark.parametrize("path", PIECE_FIX[:4], ids=IDS[::3][:4])
def test_gpu_file_lists_batch(engine, path):
    """gbgpu_file_lists: a query's cuts together -- pieces at compressed keys
    with their map keys, whole lists without, an empty one -- answer what the
    same cuts made one by one answer; a batch with one bad cut creates no
    handle (the next cut gets the handle a leak would have taken)."""
    terms, lists, params, exp = load_query(path)
    blob, offs = _file(lists)
    rng = np.random.default_rng(len(blob) + 1)
    cut_o, cut_s, keys = [], [], []
    for o, x in zip(offs, lists):
        st = key_starts(x) if x else []
        cand = [i for i, (_, k) in enumerate(st) if k < 18 and i >= len(st) // 2]
        if cand and rng.random() < 0.7:
            i = int(rng.choice(cand))
            cut_o.append(o + st[i][0])
            cut_s.append(len(x) - st[i][0])
            keys.append(full_key(x, st, i))
        else:
            cut_o.append(o)
            cut_s.append(len(x))
            keys.append(None)
    fh = engine.file_upload(blob)
    hb, hs = [], []
    try:
        hb = engine.file_lists(fh, cut_o, cut_s, keys)
        hs = [engine.file_list(fh, o, n, k) for o, n, k in zip(cut_o, cut_s, keys)]

        def run(h):
            try:
                return engine.query_resident(terms, h, params, cap=1 << 16, hit_cap=1 << 20)
            except gbgpu.GbgpuError as e:
                return e.code

        a, b = run(hb), run(hs)
        if isinstance(a, int) or isinstance(b, int):
            assert a == b
        else:
            assert a.hits == b.hits and np.array_equal(a.docids, b.docids)
            assert np.array_equal(a.scores.view(np.uint32), b.scores.view(np.uint32))
            assert np.array_equal(a.hit_docids, b.hit_docids)
        # all or nothing
        probe = engine.file_list(fh, cut_o[0], cut_s[0], keys[0])
        engine.free(probe)
        bad_o = list(cut_o) + [cut_o[0] + 1]  # off a key boundary: EINVAL
        bad_s = list(cut_s) + [6]
        with pytest.raises(gbgpu.GbgpuError):
            engine.file_lists(fh, bad_o, bad_s, list(keys) + [None])
        again = engine.file_list(fh, cut_o[0], cut_s[0], keys[0])
        engine.free(again)
        assert again == probe
        assert engine.file_lists(fh, [], [], None) == []
    finally:
        for h in hb + hs:
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


# --------------------------------------------------- Msg5: files + tree merged
# tests/golden/r_msg5_*.npz (make_golden.save_msg5): every query term's list
# spread over three Posdb files and the tree, with cross-file duplicates and
# delete keys; the reference merged them with RdbList::merge_r (removeNegRecs,
# as Msg2 reads for a query; Msg5.cpp:1621-1795) and ran its PosdbTable on
# the merged lists.
from test_golden import split_blob  # noqa: E402

M5 = sorted(glob.glob(os.path.join(HERE, "golden", "r_msg5_*.npz")))
M5_IDS = [os.path.basename(p)[2:-4] for p in M5]


def load_msg5(path):
    z = np.load(path, allow_pickle=False)
    files = split_blob(z["file_sizes"], z["file_blob"])
    tree = split_blob(z["tree_sizes"], z["tree_blob"])
    merged = split_blob(z["merged_sizes"], z["merged_blob"])
    return files, z["file_offs"], tree, merged


def test_msg5_fixtures_present():
    assert len(M5) >= 4


@pytest.mark.parametrize("path", M5, ids=M5_IDS)
def test_oracle_msg5_merge_vs_reference(path):
    """the oracle's posdbMerge_r over each term's pieces (file cuts oldest
    first, the tree last) gives the reference's merged bytes, and its
    PosdbTable on them the reference's answer"""
    import oracle_binding as orc
    from test_golden import orc_merge
    files, offs, tree, merged = load_msg5(path)
    terms, lists, params, exp = load_query(path)
    for t in range(len(terms)):
        pieces = [files[f][offs[t, f, 0]:offs[t, f, 0] + offs[t, f, 1]] for f in range(3)] + [tree[t]]
        assert orc_merge(pieces, 1, -1) == merged[t], t
    assert lists == merged
    r = orc.query(terms, lists, params, cap=1 << 16)
    check(r, exp, os.path.basename(path))


@pytest.mark.gpu
@pytest.mark.parametrize("path", M5, ids=M5_IDS)
def test_gpu_msg5_termlist_merge(engine, path):
    """gbgpu_termlist_merge: each term's ranges cut from the three resident
    file images and the tree's host list, merged in HBM into a resident list
    -- byte for byte the reference's merge_r output -- then queried: the
    reference's answer, intersected docid set included."""
    files, offs, tree, merged = load_msg5(path)
    terms, lists, params, exp = load_query(path)
    fh = [engine.file_upload(f) for f in files]
    hs = []
    try:
        for t in range(len(terms)):
            pieces = [(fh[f], int(offs[t, f, 0]), int(offs[t, f, 1]), None) for f in range(3)] + [tree[t]]
            h, mb = engine.termlist_merge(pieces, True, -1, want_bytes=True)
            hs.append(h)
            assert mb == merged[t], (os.path.basename(path), t)
        r = engine.query_resident(terms, hs, params, cap=1 << 16, hit_cap=max(1, exp["hits"]))
        check(dict(docids=r.docids, scores=r.scores, hits=r.hits, docs_wanted=r.docs_wanted, filtered=r.filtered,
                   hit_docids=r.hit_docids), exp, os.path.basename(path))
    finally:
        for h in hs:
            engine.free(h)
        for f in fh:
            engine.file_free(f)


@pytest.mark.gpu
def test_gpu_msg5_bounds_and_refusals(engine):
    """merge_r's minRecSizes bound against the oracle; a file piece cut at a
    compressed key takes the map key; a host piece must start with an
    18-byte key (merge_r's rule); out-of-range cuts are refused."""
    import gbgpu
    from test_golden import orc_merge
    files, offs, tree, merged = load_msg5(M5[0])
    fh = [engine.file_upload(f) for f in files]
    try:
        t = 0
        pieces = [(fh[f], int(offs[t, f, 0]), int(offs[t, f, 1]), None) for f in range(3)] + [tree[t]]
        host = [files[f][offs[t, f, 0]:offs[t, f, 0] + offs[t, f, 1]] for f in range(3)] + [tree[t]]
        for mrs in (1, 100, len(merged[t]) // 2):
            h, mb = engine.termlist_merge(pieces, True, mrs, want_bytes=True)
            engine.free(h)
            assert mb == orc_merge_mrs(host, 1, mrs), mrs
        # cut file 0's range after its first key: the map key restores it
        lst = host[0]
        st = key_starts(lst)
        i = next(k for k in range(1, len(st)) if st[k][1] < 18)
        off, ks = st[i]
        key = full_key(lst, st, i)
        p2 = [(fh[0], int(offs[t, 0, 0]) + off, len(lst) - off, key)] + pieces[1:]
        h, mb = engine.termlist_merge(p2, True, -1, want_bytes=True)
        engine.free(h)
        cut = bytearray(key) + lst[off + ks:]
        assert mb == orc_merge_mrs([bytes(cut)] + host[1:], 1, -1)
        with pytest.raises(gbgpu.GbgpuError):  # a compressed head without its map key
            engine.termlist_merge([(fh[0], int(offs[t, 0, 0]) + off, len(lst) - off, None)])
        with pytest.raises(gbgpu.GbgpuError):  # past the file's end
            engine.termlist_merge([(fh[0], len(files[0]) - 6, 12, None)])
        with pytest.raises(gbgpu.GbgpuError):  # a host list whose first key is compressed
            engine.termlist_merge([lst[off:]])
    finally:
        for f in fh:
            engine.file_free(f)


def orc_merge_mrs(lists, rm, mrs):
    import ctypes
    import oracle_binding as orc
    keep, ptrs, sizes = orc._lists(lists)
    cap = sum(map(len, lists)) + 64
    out = ctypes.create_string_buffer(cap)
    n = orc.lib().orc_posdb_merge(ptrs, sizes, len(lists), rm, mrs, out, cap)
    assert n >= 0
    return out.raw[:n]
