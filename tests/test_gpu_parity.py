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
    assert len(res.docids) == len(exp["docids"]), label
    assert np.array_equal(res.docids, exp["docids"]), label
    rel = np.abs(res.scores.astype(np.float64) - exp["scores"]) / np.maximum(1e-30, np.abs(exp["scores"]))
    assert np.all(rel <= REL_TOL), (label, rel.max())
    assert np.array_equal(res.scores.view(np.uint32), exp["scores"].view(np.uint32)), label


@pytest.mark.parametrize("seed", [1, 2, 3])
@pytest.mark.parametrize("kind", range(len(qkinds.kinds())))
def test_parity_kinds(engine, kind, seed):
    q = qkinds.kinds(20000, seed=seed)[kind]
    lists = generate(q, 20000, seed=1000 + seed)
    p = q.params()
    exp = orc.query(q.terms, lists, p)
    res = engine.query(q.terms, lists, p)
    check(res, exp, f"{q.name} seed={seed}")


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
    check(engine.query(q.terms, lists, p), orc.query(q.terms, lists, p))


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
    p.site_clustering = 1
    with pytest.raises(gbgpu.GbgpuError) as e:
        engine.query(q.terms, lists, p)
    assert e.value.code == gbgpu.GBGPU_EUNSUPPORTED


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
    check(engine.query(q.terms, lists, p), orc.query(q.terms, lists, p), f"{q.name} S={splits}")


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
