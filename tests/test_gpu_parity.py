"""GPU path vs the oracle, through the C ABI on cuda:0.

Bar (BASELINE.json north_star): intersected docid sets bit-exact; top-k
docids and order identical; scores within 1e-5 relative.  The engine is
written to round exactly like the reference, so scores are also checked
bit for bit."""
import numpy as np
import pytest

import gbgpu
import oracle_binding as orc
import qkinds
from workload import Word, build_query, config_two_term, generate

pytestmark = pytest.mark.gpu
REL_TOL = 1e-5


def check(res, exp, label=""):
    assert res.hits == exp["hits"], label
    assert res.docs_wanted == exp["docs_wanted"], label
    if "filtered" in exp:
        assert res.filtered == exp["filtered"], label
    if res.hit_docids is not None and "votes" in exp:
        # the intersected docid set itself (m_docIdVoteBuf), not only its size
        assert np.array_equal(res.hit_docids, exp["votes"]), label
    assert len(res.docids) == len(exp["docids"]), label
    assert np.array_equal(res.docids, exp["docids"]), label
    rel = np.abs(res.scores.astype(np.float64) - exp["scores"]) / np.maximum(1e-30, np.abs(exp["scores"]))
    assert np.all(rel <= REL_TOL), (label, rel.max())
    assert np.array_equal(res.scores.view(np.uint32), exp["scores"].view(np.uint32)), label


def oracle(terms, lists, p, cap=1 << 16):
    exp = orc.query(terms, lists, p, cap=cap)
    exp["votes"] = orc.intersect(terms, lists, params=p)
    return exp


def gpu(engine, terms, lists, p, cap=1 << 16):
    return engine.query(terms, lists, p, cap=cap, hit_cap=1 << 22)


@pytest.mark.parametrize("seed", [1, 2, 3])
@pytest.mark.parametrize("kind", range(len(qkinds.kinds())))
def test_parity_kinds(engine, kind, seed):
    q = qkinds.kinds(20000, seed=seed)[kind]
    lists = generate(q, 20000, seed=1000 + seed)
    p = q.params()
    check(gpu(engine, q.terms, lists, p), oracle(q.terms, lists, p), f"{q.name} seed={seed}")


@pytest.mark.parametrize("kind", [0, 1, 2, 3, 4])
def test_parity_paging_filter(engine, kind):
    # m_maxSerpScore / m_minSerpDocId (Posdb.cpp:4379-4381, 7327-7347)
    q = qkinds.kinds(20000, seed=8)[kind]
    lists = generate(q, 20000, seed=800 + kind)
    full = orc.query(q.terms, lists, q.params())
    for pos in (0, len(full["docids"]) // 2):
        if not len(full["docids"]):
            break
        p = q.params(max_serp_score=float(full["scores"][pos]), min_serp_docid=int(full["docids"][pos]))
        check(gpu(engine, q.terms, lists, p), oracle(q.terms, lists, p), f"{q.name} pos={pos}")


def test_corrupt_list_fails_loudly(engine):
    # an 18-byte key inside a termlist is what intersectLists10_r bails on
    # (Posdb.cpp:6289-6302); the GPU path refuses the list (GBGPU_ECORRUPT)
    # instead of scanning it, and a truncated 12-byte key likewise
    q = qkinds.kinds(5000, seed=1)[0]
    lists = generate(q, 5000)
    import posdb_py
    runs = posdb_py.decode_runs(lists[0])
    off = runs[len(runs) // 2][1]                 # a 12-byte run head mid-list
    bad = bytearray(lists[0])
    bad[off] &= 0xf9                              # -> reads as an 18-byte key
    trunc = lists[0][:runs[1][1] + 6]              # ends inside a 12-byte key
    for ls in ([bytes(bad), lists[1], lists[2]], [trunc, lists[1], lists[2]]):
        with pytest.raises(gbgpu.GbgpuError) as e:
            engine.query(q.terms, ls, q.params())
        assert e.value.code == gbgpu.GBGPU_ECORRUPT
    with pytest.raises(gbgpu.GbgpuError) as e:
        engine.upload(bytes(bad))
    assert e.value.code == gbgpu.GBGPU_ECORRUPT
    # the context stays usable
    check(gpu(engine, q.terms, lists, q.params()), oracle(q.terms, lists, q.params()), "after corrupt")


@pytest.mark.parametrize("docs_to_get,real_max_top,language", [(10, 10, 0), (300, 3, 1), (1, 1, 7)])
def test_parity_request_params(engine, docs_to_get, real_max_top, language):
    q = qkinds.kinds(30000, seed=4)[2]
    q.docs_to_get = docs_to_get
    lists = generate(q, 30000, seed=77)
    p = q.params(real_max_top=real_max_top, language=language, same_lang_weight=20.0)
    check(engine.query(q.terms, lists, p), orc.query(q.terms, lists, p))


def test_parity_larger_lists(engine):
    # ~2M docs: lists of several MB, many probe blocks per list
    q = config_two_term(2_000_000, docs_to_get=100, seed=9)
    lists = generate(q, 2_000_000, seed=5)
    p = q.params()
    check(gpu(engine, q.terms, lists, p), oracle(q.terms, lists, p))


def test_resident_repeat_is_idempotent(engine):
    q = qkinds.kinds(20000, seed=1)[1]
    lists = generate(q, 20000)
    hs = [engine.upload(l) for l in lists]
    try:
        r1 = engine.query_resident(q.terms, hs, q.params())
        for _ in range(3):
            r2 = engine.query_resident(q.terms, hs, q.params())
            assert np.array_equal(r1.docids, r2.docids)
            assert np.array_equal(r1.scores.view(np.uint32), r2.scores.view(np.uint32))
            assert r1.hits == r2.hits
    finally:
        for h in hs:
            engine.free(h)


def test_empty_lists(engine):
    q = qkinds.kinds(5000, seed=1)[0]
    lists = generate(q, 5000)
    for ls in ([lists[0], b"", b""], [b"", b"", b""], [lists[0], b"", lists[2]]):
        p = q.params()
        check(engine.query(q.terms, ls, p), orc.query(q.terms, ls, p))


def test_unsupported_modes_fail_loudly(engine):
    q = qkinds.kinds(5000, seed=1)[0]
    lists = generate(q, 5000)
    p = q.params()
    terms = list(q.terms)
    terms[0] = gbgpu.QTerm(*[getattr(terms[0], f) for f, _ in gbgpu.QTerm._fields_])
    terms[0].field_code = 63  # a facet term (gbfacetstr:); test_fields.py covers the others
    with pytest.raises(gbgpu.GbgpuError) as e:
        engine.query(terms, lists, p)
    assert e.value.code == gbgpu.GBGPU_EUNSUPPORTED
    # the scoring-info second pass (test_scoreinfo.py pins it against the
    # reference, docid splits and stale-byte docids included): resident lists
    # take the same path, or decline the same way
    hs = [engine.upload(l) for l in lists]
    try:
        for p3 in (q.params(), q.params(num_docid_splits=2)):
            p3.get_docid_scoring_info = 1
            try:
                a = engine.query(q.terms, lists, p3)
            except gbgpu.GbgpuError as e:  # a getWordPosList path not replayed
                assert e.code == gbgpu.GBGPU_EUNSUPPORTED
                with pytest.raises(gbgpu.GbgpuError):
                    engine.query_resident(q.terms, hs, p3)
                continue
            b = engine.query_resident(q.terms, hs, p3)
            if p3.num_docid_splits <= 1:  # over splits each piece's second pass adds its own
                assert len(a.docid_scores) == min(len(a.docids), p3.docs_to_get)
            # field-wise (numpy leaves a structured copy's padding unset)
            assert np.array_equal(a.docid_scores, b.docid_scores)
            assert np.array_equal(a.pair_scores, b.pair_scores)
            assert np.array_equal(a.single_scores, b.single_scores)
    finally:
        for h in hs:
            engine.free(h)


def test_query_slots_in_flight_together(engine):
    # four different queries in flight at once, one per slot, each checked
    engine.set_slots(4)
    assert engine.slots() >= 4
    kinds = qkinds.kinds(20000, seed=6)
    jobs = []
    for slot in range(4):
        q = kinds[slot % len(kinds)]
        lists = generate(q, 20000, seed=300 + slot)
        hs = [engine.upload(l) for l in lists]
        jobs.append((slot, q, lists, hs))
    try:
        for slot, q, _, hs in jobs:
            engine.enqueue(q.terms, hs, q.params(), slot=slot)
        for slot, q, lists, _ in reversed(jobs):
            check(engine.collect(slot=slot), orc.query(q.terms, lists, q.params()), f"slot {slot} {q.name}")
    finally:
        for *_, hs in jobs:
            for h in hs:
                engine.free(h)


def test_query_resident_reentrant_from_threads(engine):
    # Msg39's intersect threads call in concurrently
    from concurrent.futures import ThreadPoolExecutor
    engine.set_slots(4)
    q = qkinds.kinds(20000, seed=7)[2]
    lists = generate(q, 20000, seed=71)
    hs = [engine.upload(l) for l in lists]
    try:
        exp = orc.query(q.terms, lists, q.params())
        with ThreadPoolExecutor(6) as ex:
            results = list(ex.map(lambda _: engine.query_resident(q.terms, hs, q.params()), range(24)))
        for r in results:
            check(r, exp, "threaded")
    finally:
        for h in hs:
            engine.free(h)


@pytest.mark.parametrize("splits", [2, 5, 16])
@pytest.mark.parametrize("kind", [0, 2, 3, 9, 12])
def test_parity_docid_splits(engine, kind, splits):
    # Msg39's docid-split loop: pieces found on the device by binary search
    # over run starts, one TopTree over all pieces
    q = qkinds.kinds(20000, seed=6)[kind]
    lists = generate(q, 20000, seed=600 + splits)
    p = q.params()
    p.num_docid_splits = splits
    check(gpu(engine, q.terms, lists, p), oracle(q.terms, lists, p), f"{q.name} S={splits}")


def test_parity_docid_splits_resident_large(engine):
    q = config_two_term(2_000_000, docs_to_get=100, seed=9)
    lists = generate(q, 2_000_000, seed=5)
    p = q.params()
    p.num_docid_splits = 5
    hs = [engine.upload(l) for l in lists]
    try:
        exp = orc.query(q.terms, lists, p)
        for _ in range(2):
            check(engine.query_resident(q.terms, hs, p), exp, "two_term 2M S=5")
    finally:
        for h in hs:
            engine.free(h)


# ---------------------------------------------------------- site clustering
# m_doSiteClustering (the Msg39Request default): TopTree domain caps and the
# minWinningScore pruning they make live, replayed in docid order on the GPU

@pytest.mark.parametrize("seed", [1, 2])
@pytest.mark.parametrize("kind", range(len(qkinds.kinds())))
def test_parity_site_clustering(engine, kind, seed):
    q = qkinds.kinds(20000, seed=seed)[kind]
    lists = generate(q, 20000, seed=1100 + seed)
    for dtg in (q.docs_to_get, 13):
        q.docs_to_get = dtg
        p = q.params(site_clustering=1)
        check(gpu(engine, q.terms, lists, p), oracle(q.terms, lists, p), f"{q.name} seed={seed} dtg={dtg}")


def _skewed(n, seed, ndom, frac):
    rng = np.random.default_rng(seed)
    doms = rng.choice(256, ndom, replace=False)
    out = set()
    while len(out) < n:
        d = int(rng.integers(0, 1 << 38))
        if rng.random() < frac:
            d = (d & ~0x3fc0) | (int(doms[rng.integers(0, ndom)]) << 6)
        out.add(d)
    return sorted(out)


@pytest.mark.parametrize("ndom,frac,dtg", [(1, 0.9, 10), (2, 0.8, 37), (5, 0.6, 60), (20, 0.5, 100)])
def test_parity_site_clustering_skewed_domains(engine, ndom, frac, dtg):
    # m_ridiculousMax / m_cap / m_partial (TopTree.cpp:64-186, 355-418)
    import posdb_py
    for kind in (0, 1, 3):
        q = qkinds.kinds(8000, seed=9)[kind]
        lists = generate(q, 8000, seed=900 + ndom)
        nd = len({int(d) for l in lists for d in posdb_py.docids(l)})
        lists = posdb_py.remap_docids(lists, _skewed(nd, ndom, ndom, frac))
        q.docs_to_get = dtg
        for mx in (1, 0):
            p = q.params(site_clustering=1)
            p.do_max_score_algo = mx
            check(gpu(engine, q.terms, lists, p), oracle(q.terms, lists, p), f"{q.name} ndom={ndom} mx={mx}")


@pytest.mark.parametrize("splits", [2, 5, 16])
def test_parity_site_clustering_docid_splits(engine, splits):
    for kind in (0, 2, 3, 9):
        q = qkinds.kinds(20000, seed=10)[kind]
        lists = generate(q, 20000, seed=1200 + splits)
        p = q.params(site_clustering=1, num_docid_splits=splits)
        check(gpu(engine, q.terms, lists, p), oracle(q.terms, lists, p), f"{q.name} S={splits}")


def test_parity_site_clustering_pruning_large(engine):
    # 300k docs: the prefilters prune and change the tree vs scoring every docid
    q = build_query("three", [Word("a", 0.3), Word("b", 0.2), Word("c", 0.25)], 300_000, seed=1)
    q.docs_to_get = 50
    lists = generate(q, 300_000, seed=1)
    p = q.params(site_clustering=1)
    check(gpu(engine, q.terms, lists, p), oracle(q.terms, lists, p), "three 300k")
    q2 = config_two_term(2_000_000, docs_to_get=100, seed=9)
    lists2 = generate(q2, 2_000_000, seed=5)
    p2 = q2.params(site_clustering=1)
    check(gpu(engine, q2.terms, lists2, p2), oracle(q2.terms, lists2, p2), "two_term 2M")


# ------------------------------------------- every survivor's score, exactly
# docs_to_get large enough that the TopTree holds every scored survivor, so
# each docid's score is compared, not only the top's.  The seeds include
# queries whose shared bigram lists are shrunk in place twice by the
# reference (shrinkSubLists re-reads the list's original extent, Posdb.cpp:
# 5334-5428): the second group's copy of the list's last survivor run picks
# up the stale 6-byte units that follow the first shrink's output.
RESHRINK_CASES = [(2, "q3_0"), (8, "three_word"), (8, "piped"), (11, "five_word"), (14, "q3_0"),
                  (16, "wiki_halfstop"), (17, "five_word")]


@pytest.mark.parametrize("seed,name", RESHRINK_CASES)
def test_parity_every_survivor_reshrunk_lists(engine, seed, name):
    q = [k for k in qkinds.kinds(20000, seed=seed) if k.name == name][0]
    lists = generate(q, 20000, seed=seed)
    q.docs_to_get = 1500
    p = q.params()
    exp = oracle(q.terms, lists, p)
    assert exp["hits"] <= 1500
    check(gpu(engine, q.terms, lists, p), exp, f"{name} seed={seed}")
    p = q.params(site_clustering=1)
    check(gpu(engine, q.terms, lists, p), oracle(q.terms, lists, p), f"{name} seed={seed} clustering")


@pytest.mark.parametrize("kind", range(len(qkinds.kinds())))
def test_parity_every_survivor(engine, kind):
    q = qkinds.kinds(12000, seed=21)[kind]
    lists = generate(q, 12000, seed=21)
    q.docs_to_get = 1500
    p = q.params()
    exp = oracle(q.terms, lists, p)
    if exp["hits"] > 1500:
        pytest.skip("more survivors than one TopTree can hold here")
    check(gpu(engine, q.terms, lists, p), exp, q.name)


@pytest.mark.parametrize("kind", [0, 1, 2, 4, 6])
@pytest.mark.parametrize("clus,splits", [(0, 1), (1, 1), (0, 4)])
def test_parity_whitelist(engine, kind, clus, splits):
    # the "&sites=" whitelist (Posdb.cpp:793-835, 5294, 5544-5572): site lists
    # over part of the docids, some with siteRank's top bit flipped, 6-byte
    # keys inside; through gbgpu_query and the resident path
    from posdb_py import site_lists
    q = qkinds.kinds(30000, seed=4)[kind]
    lists = generate(q, 30000, seed=6100 + kind)
    wl = site_lists(lists, 2 + kind % 2, 0.35, seed=kind, flip_frac=0.05, multi_frac=0.2)
    p = q.params(site_clustering=clus, num_docid_splits=splits).with_whitelist(wl)
    exp = oracle(q.terms, lists, p)
    check(gpu(engine, q.terms, lists, p), exp, f"{q.name} white")
    hs = [engine.upload(l) for l in lists]
    try:
        check(engine.query_resident(q.terms, hs, p, cap=1 << 16), exp, f"{q.name} white resident")
    finally:
        for h in hs:
            engine.free(h)
    # an empty whitelist votes nothing
    p0 = q.params(site_clustering=clus, num_docid_splits=splits).with_whitelist([])
    r0 = gpu(engine, q.terms, lists, p0)
    assert r0.hits == 0 and len(r0.docids) == 0
