"""Facet terms (gbfacetstr: / gbfacetint: / gbfacetfloat:): each facet query
term's QueryTerm::m_facetHashTable and m_numDocsThatHaveFacet.

The reference fills them inside intersectLists10_r: every docid that reaches
the TopTree walks its run in the facet list and votes once per entry -- the
value itself, or with ranges the first range holding it, keyed by its A
value (Posdb.cpp:5575-5631, 7362-7542) -- and countUniqueDocids
(5002-5038, 7786-7796) walks the facet list's whole buffer, the survivors'
runs shrinkSubLists wrote over its start and then the list's own bytes past
them, counting each record's value in an existing entry and each record
longer than 6 bytes.

Parity: the reference's own fixtures (tests/golden/q_facet_*.npz: int, str
and float facets, ranges of both, the paging filter, docsToGet 10) pin the
oracle (test_golden.py runs them on CPU and GPU); here the GPU runs against
the oracle on seeded corpora over several query kinds, facet shapes and
range sets, with and without site clustering, through gbgpu_query, the
resident path and enqueue/collect, and the modes the library does not
restate fail loudly."""
import struct

import numpy as np
import pytest

import gbgpu
import oracle_binding as orc
import qkinds
from numlists import number_list
from workload import generate

FACET_STR, FACET_INT, FACET_FLOAT = 63, 64, 65


def fl(x):
    return struct.unpack("<i", struct.pack("<f", x))[0]


# (field code, ints, keys per docid, share of docids, ranges)
SHAPES = {
    "int": (FACET_INT, True, 3, 0.8, None),
    "int_ranges": (FACET_INT, True, 4, 0.7, ([-20, 0, 50, 100, 50], [0, 50, 100, 300, 60])),
    "float": (FACET_FLOAT, False, 2, 0.9, None),
    "float_ranges": (FACET_FLOAT, False, 3, 0.8, ([fl(0.0), fl(20.0), fl(55.5)], [fl(20.0), fl(55.5), fl(100.0)])),
    "str": (FACET_STR, True, 1, 0.6, None),
    "sparse": (FACET_INT, True, 6, 0.05, None),
}


def facet_query(q, lists, shape, seed, two=False):
    """q's terms and lists with one (or two) facet terms appended"""
    fc, ints, kmax, frac, ranges = SHAPES[shape]
    terms = list(q.terms)
    qp = max(t.qpos for t in terms) + 2
    terms.append(gbgpu.QTerm(1, 0, fc, 0, -1, -1, -1, 0, qp, 0, -1, 1.0))
    lists = list(lists) + [number_list(lists, frac, seed=seed, kmax=kmax, ints=ints)]
    fr = []
    if ranges:
        fr.append((len(terms) - 1, ranges[0], ranges[1]))
    if two:
        terms.append(gbgpu.QTerm(1, 0, FACET_STR, 0, -1, -1, -1, 0, qp + 2, 0, -1, 1.0))
        lists.append(number_list(lists[:len(q.terms)], 0.7, seed=seed + 1, kmax=2, ints=True, termid=0x3C3C3C3C3C4))
    return terms, lists, fr


def params_of(q, fr, docs_to_get=None, **kw):
    p = q.params(**kw)
    if docs_to_get is not None:
        p.docs_to_get = docs_to_get
    return p.with_facets(fr) if fr else p


def same(r, exp, label):
    assert r.hits == exp["hits"], label
    assert r.filtered == exp["filtered"], label
    assert np.array_equal(r.docids, exp["docids"]), label
    assert np.array_equal(r.scores.view(np.uint32), exp["scores"].view(np.uint32)), label
    assert r.facets == exp["facets"], label


def test_oracle_facet_tables_shape():
    """The restatement's tables on a seeded corpus: one per facet term, a
    range set's entries keyed by its A values (each present once), every
    count at most the scored docids, and m_numDocsThatHaveFacet at least the
    intersected docids (each survivor's run head is a 12-byte record)."""
    q = qkinds.kinds(3000, seed=4)[1]
    lists = generate(q, 3000, seed=41)
    for shape in ("int", "int_ranges", "float_ranges"):
        terms, fl_, fr = facet_query(q, lists, shape, seed=7)
        p = params_of(q, fr)
        r = orc.query(terms, fl_, p, cap=1 << 16)
        ft = len(terms) - 1
        assert list(r["facets"]) == [ft], shape
        docs, ents = r["facets"][ft]
        assert docs >= r["hits"], shape
        scored = r["hits"] - 0  # no paging filter: every scored docid reaches the tree
        for key, (cnt, outside, docid, s, mx, mn) in ents.items():
            assert 0 <= cnt <= scored, shape
            if not fr:  # each vote's value is a record of a survivor's run
                assert outside >= cnt, shape
        if fr:
            assert set(ents) == set(fr[0][1]), shape


def test_facet_result_abi_layout():
    """gbgpu_facet_entry / gbgpu_result's facet fields as the binding reads them"""
    assert gbgpu.FACET_DT.itemsize == 40
    names = [f[0] for f in gbgpu.Result._fields_]
    assert names[-4:] == ["facets", "facets_cap", "n_facets", "facet_docs"]


KINDS = [0, 1, 3, 4, 8]  # config-2 two-term, three_word, negative, synonyms, five_word


@pytest.mark.gpu
@pytest.mark.parametrize("shape", list(SHAPES))
@pytest.mark.parametrize("kind", KINDS)
def test_gpu_facets_vs_oracle(engine, kind, shape):
    q = qkinds.kinds(20000, seed=5)[kind]
    lists = generate(q, 20000, seed=500 + kind)
    terms, fl_, fr = facet_query(q, lists, shape, seed=90 + kind)
    for it, kw in enumerate([{}, dict(docs_to_get=7), dict(language=5)]):
        p = params_of(q, fr, **kw)
        exp = orc.query(terms, fl_, p, cap=1 << 16)
        r = engine.query(terms, fl_, p, cap=1 << 16)
        same(r, exp, f"{q.name} {shape} it={it}")


@pytest.mark.gpu
@pytest.mark.parametrize("shape", ["int", "float_ranges", "str"])
@pytest.mark.parametrize("kind", [0, 1, 3])
def test_gpu_facets_with_site_clustering(engine, kind, shape):
    """Site clustering (the Msg39 default): the prefilters skip docids, which
    then cast no facet vote, and a facet term turns the scoring filter off
    (Posdb.cpp:6353-6356); small docsToGet so minWinningScore goes live early"""
    q = qkinds.kinds(20000, seed=11)[kind]
    lists = generate(q, 20000, seed=1100 + kind)
    terms, fl_, fr = facet_query(q, lists, shape, seed=110 + kind)
    for dtg in (10, 50):
        p = params_of(q, fr, docs_to_get=dtg, site_clustering=1)
        exp = orc.query(terms, fl_, p, cap=1 << 16)
        r = engine.query(terms, fl_, p, cap=1 << 16)
        same(r, exp, f"{q.name} {shape} clustered docs {dtg}")


@pytest.mark.gpu
@pytest.mark.parametrize("shape", ["int", "int_ranges", "float", "str"])
@pytest.mark.parametrize("kind", [0, 1, 3])
def test_gpu_facets_over_docid_splits(engine, kind, shape):
    """Docid splits (the default /search request): each piece's votes go on
    from the tables the pieces before left -- an entry's last voter is not
    counted again where the pieces overlap, a float sum keeps accumulating in
    docid order -- and each piece's records count in every entry the table
    holds; with and without site clustering"""
    q = qkinds.kinds(20000, seed=12)[kind]
    lists = generate(q, 20000, seed=1200 + kind)
    terms, fl_, fr = facet_query(q, lists, shape, seed=120 + kind)
    for kw in (dict(num_docid_splits=3), dict(num_docid_splits=5, site_clustering=1, docs_to_get=10)):
        p = params_of(q, fr, **kw)
        exp = orc.query(terms, fl_, p, cap=1 << 16)
        r = engine.query(terms, fl_, p, cap=1 << 16)
        same(r, exp, f"{q.name} {shape} {kw}")


@pytest.mark.gpu
@pytest.mark.parametrize("resident", [False, True])
def test_gpu_facets_over_splits_enospc_then_room(engine, resident):
    """INTEGRATION.md 3b's retry: the adapter sizes the facet buffer from the
    first piece's lists; when the whole range's tables hold more entries the
    call returns ENOSPC with n_facets set (and nothing else valid), and the
    call again with room for n_facets entries answers exactly.  The facet
    list's records sit mostly in the last piece, as the retry meets them."""
    q = qkinds.kinds(20000, seed=13)[1]
    lists = generate(q, 20000, seed=1301)
    terms, fl_, fr = facet_query(q, lists, "int", seed=131)
    for kw in (dict(num_docid_splits=4), dict(num_docid_splits=5, site_clustering=1, docs_to_get=10)):
        p = params_of(q, fr, **kw)
        exp = orc.query(terms, fl_, p, cap=1 << 16)
        n = sum(len(v[1]) for v in exp["facets"].values())
        assert n > 8
        old = gbgpu.Engine.facet_cap
        hs = [engine.upload(x) for x in fl_] if resident else None
        try:
            gbgpu.Engine.facet_cap = 3  # what a first piece's lists might size
            with pytest.raises(gbgpu.GbgpuError) as ei:
                if resident:
                    engine.query_resident(terms, hs, p, cap=1 << 16)
                else:
                    engine.query(terms, fl_, p, cap=1 << 16)
            assert ei.value.code == 28  # ENOSPC
            assert engine.last_n_facets == n, (engine.last_n_facets, n)
            gbgpu.Engine.facet_cap = engine.last_n_facets  # exactly the room asked for
            r = engine.query_resident(terms, hs, p, cap=1 << 16) if resident else engine.query(terms, fl_, p, cap=1 << 16)
            same(r, exp, f"retry {kw}")
        finally:
            gbgpu.Engine.facet_cap = old
            for h in hs or ():
                engine.free(h)


@pytest.mark.gpu
@pytest.mark.parametrize("shape", ["int", "float_ranges", "str"])
def test_gpu_facets_in_boolean_queries(engine, shape):
    """A facet term in a boolean query (the reference's q_bool_facet_*
    fixtures pin the mode): the expression's vote buffer, the facet group's
    run voted from where the docid has one -- a docid the truth table admits
    without it casts no vote -- on random truth tables over the groups"""
    q = qkinds.kinds(20000, seed=14)[1]
    lists = generate(q, 20000, seed=1400)
    terms, fl_, fr = facet_query(q, lists, shape, seed=140)
    ng = sum(1 for t in terms if t.is_required)
    rng = np.random.default_rng(141)
    for it in range(4):
        bits = rng.integers(0, 2, 1 << ng)
        bits[0] = 0  # a docid in no group is never voted
        tb = np.packbits(bits.astype(np.uint8), bitorder="little").tobytes()
        tb = tb + bytes(max(0, (1 << ng) // 8 - len(tb)))
        p = params_of(q, fr).with_boolean(tb, ng)
        exp = orc.query(terms, fl_, p, cap=1 << 16)
        same(engine.query(terms, fl_, p, cap=1 << 16), exp, f"{shape} table {it}")


@pytest.mark.gpu
def test_gpu_facets_paging_and_two_terms(engine):
    """the paging filter (only the docids that reach the tree vote) and two
    facet terms in one query, through the resident path and enqueue/collect"""
    q = qkinds.kinds(20000, seed=6)[1]
    lists = generate(q, 20000, seed=61)
    terms, fl_, fr = facet_query(q, lists, "int_ranges", seed=62, two=True)
    full = orc.query(terms, fl_, params_of(q, fr), cap=1 << 16)
    pos = len(full["docids"]) // 2
    p = params_of(q, fr, max_serp_score=float(full["scores"][pos]), min_serp_docid=int(full["docids"][pos]))
    exp = orc.query(terms, fl_, p, cap=1 << 16)
    assert len(exp["facets"]) == 2
    same(engine.query(terms, fl_, p, cap=1 << 16), exp, "host lists")
    hs = [engine.upload(x) for x in fl_]
    try:
        same(engine.query_resident(terms, hs, p, cap=1 << 16), exp, "resident")
        engine.enqueue(terms, hs, p)
        same(engine.collect(cap=1 << 16, terms=terms), exp, "enqueue/collect")
    finally:
        for h in hs:
            engine.free(h)


@pytest.mark.gpu
def test_gpu_facets_large(engine):
    """200k docids, a dense int facet of up to 6 values per docid: the
    parallel tail walk and the LDS-held outside counts at scale"""
    q = qkinds.kinds(200000, seed=8)[0]
    lists = generate(q, 200000, seed=81)
    terms, fl_, fr = facet_query(q, lists, "int", seed=82)
    fl_[-1] = number_list(lists, 0.9, seed=83, kmax=6, ints=True)
    p = params_of(q, fr)
    same(engine.query(terms, fl_, p, cap=1 << 16), orc.query(terms, fl_, p, cap=1 << 16), "200k")


@pytest.mark.gpu
def test_gpu_facets_capacity_and_refusals(engine):
    q = qkinds.kinds(5000, seed=9)[1]
    lists = generate(q, 5000, seed=91)
    terms, fl_, fr = facet_query(q, lists, "int", seed=92)
    p = params_of(q, fr)
    exp = orc.query(terms, fl_, p, cap=1 << 16)
    n = len(exp["facets"][len(terms) - 1][1])
    assert n > 4
    old = gbgpu.Engine.facet_cap
    try:
        gbgpu.Engine.facet_cap = 4  # fewer entries than the table holds: ENOSPC, not a truncated table
        with pytest.raises(gbgpu.GbgpuError) as ei:
            engine.query(terms, fl_, p, cap=1 << 16)
        assert ei.value.code == 28  # ENOSPC
    finally:
        gbgpu.Engine.facet_cap = old
    big = list(range(300))
    with pytest.raises(gbgpu.GbgpuError) as ei:
        engine.query(terms, fl_, q.params().with_facets([(len(terms) - 1, big, [x + 1 for x in big])]), cap=1 << 16)
    assert ei.value.code == 22  # EINVAL: more ranges than QueryWord holds
