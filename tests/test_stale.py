"""The stale-mbuf case: a docid whose trailing merged group comes out empty
(its keys there were all BF_BIGRAM keys with syn bits, skipped by the
mini-merge, Posdb.cpp:6687-6692) has every scorer read the mbuf bytes at
that group's place -- bytes its own merges never wrote.  mbuf is a local of
intersectLists10_r (Posdb.cpp:6007) that each docid's merges overwrite from
the start (6559), so those bytes are what the docids before it in the pass
left there; where no earlier docid wrote them they are the stack's
(undefined: the oracle and the GPU skip that docid).

Parity: the reference's own fixtures (tests/golden/q_stale_*.npz: the second
word's list empty, so half the hits are stale docids, each with defined
bytes) pin the oracle, which keeps a real mbuf over the pass (test_golden.py
runs them on CPU and GPU); here the GPU (k_stale_find / k_stale_fix after the
pass) runs against the oracle on seeded corpora, defined and undefined
bytes alike, with paging and over docid splits, and with site clustering
(the writers among the docids the replay's prefilter did not skip), over
docid splits too."""
import numpy as np
import pytest

import gbgpu
import oracle_binding as orc
import qkinds
from workload import generate


def stale_case(seed, n=6000, kind=0):
    q = qkinds.kinds(n, seed=seed)[kind]
    lists = generate(q, n, seed=2000 + seed)
    return q, [lists[0], b"", lists[2]]


def test_oracle_stale_counts():
    """the shape makes stale docids in every seed; most seeds have some whose
    bytes no earlier docid wrote"""
    undef = 0
    for seed in range(1, 7):
        q, lists = stale_case(seed)
        r = orc.query(q.terms, lists, q.params(), cap=1 << 16)
        d, u = r["stale"]
        assert d > 0
        undef += u
    assert undef > 0


@pytest.mark.gpu
@pytest.mark.parametrize("seed", list(range(1, 13)))
def test_gpu_stale_vs_oracle(engine, seed):
    q, lists = stale_case(seed, n=20000)
    for dtg in (50, 400):
        q.docs_to_get = dtg
        p = q.params()
        exp = orc.query(q.terms, lists, p, cap=1 << 16)
        r = engine.query(q.terms, lists, p, cap=1 << 16)
        label = f"seed {seed} docs {dtg} stale {exp['stale']}"
        assert r.hits == exp["hits"], label
        assert r.filtered == exp["filtered"], label
        assert np.array_equal(r.docids, exp["docids"]), label
        assert np.array_equal(r.scores.view(np.uint32), exp["scores"].view(np.uint32)), label


@pytest.mark.gpu
def test_gpu_stale_paging_and_splits(engine):
    q, lists = stale_case(3, n=20000)
    full = orc.query(q.terms, lists, q.params(), cap=1 << 16)
    pos = len(full["docids"]) // 2
    for p in (q.params(max_serp_score=float(full["scores"][pos]), min_serp_docid=int(full["docids"][pos])),
              q.params(num_docid_splits=3)):
        exp = orc.query(q.terms, lists, p, cap=1 << 16)
        r = engine.query(q.terms, lists, p, cap=1 << 16)
        assert (r.hits, r.filtered) == (exp["hits"], exp["filtered"])
        assert np.array_equal(r.docids, exp["docids"])
        assert np.array_equal(r.scores.view(np.uint32), exp["scores"].view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", list(range(1, 9)))
def test_gpu_stale_with_clustering_vs_oracle(engine, seed):
    """with site clustering the replay's prefilter skips decide which docids
    write mbuf: the stale survivors are scored with the writers among the
    docids the replay did not skip, and replayed until the scores settle
    (stale_fix_clustered); the oracle keeps a real mbuf over the sequential
    pass"""
    q, lists = stale_case(seed, n=20000)
    for dtg in (50, 200):
        q.docs_to_get = dtg
        p = q.params(site_clustering=1)
        exp = orc.query(q.terms, lists, p, cap=1 << 16)
        label = f"seed {seed} docs {dtg} stale {exp['stale']}"
        r = engine.query(q.terms, lists, p, cap=1 << 16)
        assert r.hits == exp["hits"], label
        assert r.filtered == exp["filtered"], label
        assert np.array_equal(r.docids, exp["docids"]), label
        assert np.array_equal(r.scores.view(np.uint32), exp["scores"].view(np.uint32)), label


@pytest.mark.gpu
def test_gpu_stale_with_clustering_paging(engine):
    q, lists = stale_case(3, n=20000)
    full = orc.query(q.terms, lists, q.params(site_clustering=1), cap=1 << 16)
    pos = len(full["docids"]) // 2
    p = q.params(site_clustering=1, max_serp_score=float(full["scores"][pos]), min_serp_docid=int(full["docids"][pos]))
    exp = orc.query(q.terms, lists, p, cap=1 << 16)
    r = engine.query(q.terms, lists, p, cap=1 << 16)
    assert (r.hits, r.filtered) == (exp["hits"], exp["filtered"])
    assert np.array_equal(r.docids, exp["docids"])
    assert np.array_equal(r.scores.view(np.uint32), exp["scores"].view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 3, 6])
def test_gpu_stale_with_clustering_over_splits(engine, seed):
    """Msg39's default request: site clustering over docid splits, the tree
    carried between the pieces; each piece's mbuf is its own call's, and a
    stale fix replays the piece again from the tree it started with"""
    q, lists = stale_case(seed, n=20000)
    for dtg in (50, 200):
        q.docs_to_get = dtg
        p = q.params(site_clustering=1, num_docid_splits=3)
        exp = orc.query(q.terms, lists, p, cap=1 << 16)
        label = f"seed {seed} docs {dtg} stale {exp['stale']}"
        r = engine.query(q.terms, lists, p, cap=1 << 16)
        assert (r.hits, r.filtered) == (exp["hits"], exp["filtered"]), label
        assert np.array_equal(r.docids, exp["docids"]), label
        assert np.array_equal(r.scores.view(np.uint32), exp["scores"].view(np.uint32)), label
