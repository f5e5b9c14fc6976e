"""Field terms (row f4): gbsortby:/gbrevsortby: float terms score a docid
by the float its numeric termlist stores where the word position is
(Posdb.cpp:4413-4417, 4572-4577, 6050-6051, 6350, 7265-7269), and plain
text field terms (title:, site: ...) are ordinary lists to PosdbTable.
Fixtures: tests/golden/f_*.npz, made by `python3 tests/make_golden.py
sortby` / `range` from the reference harness (oracle/_ref/gbref).  Range
terms (gbmin:/gbmax:/gbequal:, float and int; Posdb.cpp:4948-4999,
5056-5121, 5242-5298) vote a docid only if a key of its run holds a number
in range.  The C oracle restates them too and is pinned to the same
fixtures (CPU tests below).  gbsortby int terms make the TopTree order by m_intScore
(gbgpu_result::int_scores).  Facet terms return GBGPU_EUNSUPPORTED."""
import glob
import os
import struct

import numpy as np
import pytest

import gbgpu
import oracle_binding as orc
from test_golden import check, load_query

HERE = os.path.dirname(os.path.abspath(__file__))
FCASES = sorted(glob.glob(os.path.join(HERE, "golden", "f_*.npz")))
IDS = [os.path.basename(p)[2:-4] for p in FCASES]


def test_fixtures_present():
    assert len(FCASES) >= 6


@pytest.mark.parametrize("path", FCASES, ids=IDS)
def test_oracle_fields_vs_reference(path):
    terms, lists, params, exp = load_query(path)
    check(orc.query(terms, lists, params, cap=1 << 16), exp, os.path.basename(path))
    assert np.array_equal(orc.intersect(terms, lists, params=params), exp["votes"])


def first_numbers(lst, fmt):
    """docid -> the number in bytes 2..5 of its run's first key"""
    import posdb_py
    out = {}
    for key in posdb_py.full_keys(lst):
        out.setdefault(int.from_bytes(key[7:12], "little") >> 2, struct.unpack(fmt, bytes(key[2:6]))[0])
    return out


@pytest.mark.parametrize("path", [p for p in FCASES if "sortby" in p and "sortbyint" not in p],
                         ids=[i for i in IDS if "sortby" in i and "sortbyint" not in i])
def test_sortby_scores_are_the_stored_floats(path):
    """The reference's scores are the sortby keys' floats, unrewritten: a
    numeric group found in one sublist is not mini-merged (Posdb.cpp:
    6638-6647)."""
    terms, lists, params, exp = load_query(path)
    import posdb_py
    floats = set()
    for key in posdb_py.full_keys(lists[-1]):
        floats.add(struct.unpack("<f", bytes(key[2:6]))[0])
    assert all(float(s) in floats for s in exp["scores"])


@pytest.mark.gpu
@pytest.mark.parametrize("path", FCASES, ids=IDS)
def test_gpu_fields_vs_reference(engine, path):
    terms, lists, params, exp = load_query(path)
    r = engine.query(terms, lists, params, cap=1 << 16, hit_cap=max(1, exp["hits"]))
    check(dict(docids=r.docids, scores=r.scores, hits=r.hits, docs_wanted=r.docs_wanted, filtered=r.filtered,
               hit_docids=r.hit_docids), exp, os.path.basename(path))
    if "sortbyint" in path:
        # TopNode::m_intScore: the int of the docid's first key (the order is
        # the reference's, checked above; m_score is 0.0 there and here)
        nums = first_numbers(lists[-1], "<i")
        assert [nums[int(d)] for d in r.docids] == list(r.int_scores)
        assert list(r.int_scores) == sorted(r.int_scores, reverse=True)


@pytest.mark.gpu
@pytest.mark.parametrize("fc", [63, 64, 65])
def test_gpu_facet_field_codes_vs_oracle(engine, fc):
    """a fixture's numeric term read as a facet term (gbfacetstr:/int:/float:):
    its group drops out of the scorers as a numeric one does, and the facet
    tables come back as the oracle builds them (test_facets.py has the rest)"""
    import oracle_binding as orc
    terms, lists, params, _ = load_query(FCASES[0])
    terms = list(terms)
    last = gbgpu.QTerm(*[getattr(terms[-1], f) for f, _ in gbgpu.QTerm._fields_])
    last.field_code = fc
    terms[-1] = last
    exp = orc.query(terms, lists, params, cap=1 << 16)
    r = engine.query(terms, lists, params, cap=1 << 16)
    assert r.hits == exp["hits"] and np.array_equal(r.docids, exp["docids"])
    assert np.array_equal(r.scores.view(np.uint32), exp["scores"].view(np.uint32))
    assert r.facets == exp["facets"]


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2, 3])
@pytest.mark.parametrize("fc,vf,vi,ints", [(56, 40.0, 0, False), (57, 60.0, 0, False), (67, 12.5, 0, False),
                                           (61, 0, 90, True), (62, 0, 30, True), (54, 0, 0, False),
                                           (59, 0, 0, True)])
def test_gpu_fields_vs_oracle(engine, seed, fc, vf, vi, ints):
    """Larger seeded corpora (40 k docs) than the fixtures, GPU vs the oracle:
    top tree, hits, the intersected docid set."""
    import qkinds
    from numlists import number_list
    from workload import generate
    N = 40000
    for q in qkinds.kinds(N, seed=seed)[:5]:
        lists = generate(q, N, seed=7000 + seed)
        terms = list(q.terms)
        t = gbgpu.QTerm(1, 0, fc, 0, -1, -1, -1, 0, max(x.qpos for x in terms) + 2, 0, -1, 1.0)
        t.number_float, t.number_int = vf, vi
        terms.append(t)
        lists = list(lists) + [number_list(lists, 0.6, seed=seed, kmax=3, ints=ints)]
        params = q.params()
        o = orc.query(terms, lists, params, cap=1 << 16)
        ov = orc.intersect(terms, lists, params=params)
        r = engine.query(terms, lists, params, cap=1 << 16, hit_cap=max(1, o["hits"]))
        label = f"{q.name} fc={fc} seed={seed}"
        assert r.hits == o["hits"], label
        assert np.array_equal(r.hit_docids, ov), label
        assert np.array_equal(r.docids, o["docids"]), label
        assert np.array_equal(np.asarray(r.scores, np.float32).view(np.uint32),
                              np.asarray(o["scores"], np.float32).view(np.uint32)), label


@pytest.mark.gpu
@pytest.mark.parametrize("fc,vf,vi,ints", [(54, 0, 0, False), (56, 40.0, 0, False), (62, 0, 30, True)])
def test_gpu_fields_clustering_vs_oracle(engine, fc, vf, vi, ints):
    """Field terms under site clustering (the default request): the TopTree
    domain caps with the sortby float score, and the prefilters off for
    gbsortby (Posdb.cpp:6050-6051, 6350)."""
    import qkinds
    from numlists import number_list
    from workload import generate
    N = 40000
    for q in qkinds.kinds(N, seed=4)[:5]:
        lists = generate(q, N, seed=7100)
        terms = list(q.terms)
        t = gbgpu.QTerm(1, 0, fc, 0, -1, -1, -1, 0, max(x.qpos for x in terms) + 2, 0, -1, 1.0)
        t.number_float, t.number_int = vf, vi
        terms.append(t)
        lists = list(lists) + [number_list(lists, 0.6, seed=5, kmax=3, ints=ints)]
        params = q.params(site_clustering=1)
        o = orc.query(terms, lists, params, cap=1 << 16)
        r = engine.query(terms, lists, params, cap=1 << 16)
        label = f"{q.name} fc={fc}"
        assert (r.hits, r.filtered, r.docs_wanted) == (o["hits"], o["filtered"], o["docs_wanted"]), label
        assert np.array_equal(r.docids, o["docids"]), label
        assert np.array_equal(np.asarray(r.scores, np.float32).view(np.uint32),
                              np.asarray(o["scores"], np.float32).view(np.uint32)), label


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2])
@pytest.mark.parametrize("fc", [59, 60])
def test_gpu_int_sortby_paging_vs_oracle(engine, seed, fc):
    """gbsortby int with the widget's paging filter (Posdb.cpp:7330-7336):
    m_intScore against (int32_t)m_maxSerpScore -- fractional bounds of both
    signs truncate toward zero, ties on the bound compare the docid with
    m_minSerpDocId, and an out-of-range or NaN bound is INT32_MIN (x86-64's
    cvttsd2si), which drops every docid above it."""
    import qkinds
    from numlists import number_list
    from workload import generate
    N = 40000
    q = qkinds.kinds(N, seed=seed)[0]
    lists = generate(q, N, seed=7200 + seed)
    terms = list(q.terms)
    t = gbgpu.QTerm(1, 0, fc, 0, -1, -1, -1, 0, max(x.qpos for x in terms) + 2, 0, -1, 1.0)
    terms.append(t)
    lists = list(lists) + [number_list(lists, 0.6, seed=seed, kmax=2, ints=True)]
    base = engine.query(terms, lists, q.params(), cap=1 << 16)
    mid = len(base.docids) // 2
    v = int(base.int_scores[mid])
    d = int(base.docids[mid])
    bounds = [v + 0.75, v - 0.75, -v - 0.5, 0.25 - abs(v), 1e12, -1e12, float("nan")]
    for b in bounds:
        params = q.params(max_serp_score=b, min_serp_docid=d)
        o = orc.query(terms, lists, params, cap=1 << 16)
        r = engine.query(terms, lists, params, cap=1 << 16)
        label = f"fc={fc} seed={seed} bound={b}"
        assert (r.hits, r.filtered, r.docs_wanted) == (o["hits"], o["filtered"], o["docs_wanted"]), label
        assert np.array_equal(r.docids, o["docids"]), label


@pytest.mark.gpu
def test_gpu_int_sortby_int32_min_declined(engine):
    """m_intScore INT32_MIN (Posdb.cpp:7271-7279) has no survivor key of its
    own on the device (key 0 means "not scored"): a query that scores such a
    docid is declined (EUNSUPPORTED, the adapter runs the CPU body) instead
    of reporting INT32_MIN + 1; INT32_MIN + 1 itself, and INT32_MIN on keys
    no scored docid holds, are answered exactly."""
    import struct
    import posdb_py
    import qkinds
    from numlists import number_list
    from workload import generate
    N = 20000
    q = qkinds.kinds(N, seed=3)[0]
    lists = generate(q, N, seed=7300)
    terms = list(q.terms)
    terms.append(gbgpu.QTerm(1, 0, 59, 0, -1, -1, -1, 0, max(x.qpos for x in terms) + 2, 0, -1, 1.0))
    nl = number_list(lists, 0.6, seed=3, kmax=2, ints=True)
    keys = posdb_py.full_keys(nl)

    def with_values(pick):
        ks = []
        for k in keys:
            k = bytearray(k)
            v = pick(int.from_bytes(k[7:12], "little") >> 2, struct.unpack("<i", bytes(k[2:6]))[0])
            k[2:6] = struct.pack("<i", v)
            ks.append(bytes(k))
        return posdb_py.encode_keys(ks)

    p = q.params()
    base = orc.query(terms, list(lists) + [nl], p, cap=1 << 16)
    assert len(base["docids"]) > 10
    top = int(base["docids"][0])
    # INT32_MIN + 1 everywhere: answered, as the oracle
    l1 = list(lists) + [with_values(lambda d, v: -(1 << 31) + 1)]
    r = engine.query(terms, l1, p, cap=1 << 16)
    o = orc.query(terms, l1, p, cap=1 << 16)
    assert np.array_equal(r.docids, o["docids"]) and r.hits == o["hits"]
    # INT32_MIN on a scored docid: declined
    l2 = list(lists) + [with_values(lambda d, v: -(1 << 31) if d == top else v)]
    with pytest.raises(gbgpu.GbgpuError) as ei:
        engine.query(terms, l2, p, cap=1 << 16)
    assert ei.value.code == gbgpu.GBGPU_EUNSUPPORTED
    # INT32_MIN on a docid the query does not score (not voted): answered
    voted = set(int(x) for x in orc.intersect(terms, list(lists) + [nl], params=p))
    other = next(int.from_bytes(k[7:12], "little") >> 2 for k in keys
                 if (int.from_bytes(k[7:12], "little") >> 2) not in voted)
    l3 = list(lists) + [with_values(lambda d, v: -(1 << 31) if d == other else v)]
    r = engine.query(terms, l3, p, cap=1 << 16)
    o = orc.query(terms, l3, p, cap=1 << 16)
    assert np.array_equal(r.docids, o["docids"]) and r.hits == o["hits"]
