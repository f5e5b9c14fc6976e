"""Live pinning: the oracle restatement vs the REFERENCE's own code
(oracle/_ref/gbref, built from the unmodified /root/reference sources) on
fresh seeds, wider than the committed golden vectors.  Skipped where the
reference was not available at build time (e.g. the GPU box)."""
import ctypes

import numpy as np
import pytest

import oracle_binding as orc
import qkinds
import ref_binding as ref
from mergegen import tiered_runs
from workload import config_two_term, generate

pytestmark = pytest.mark.skipif(not ref.available(), reason="oracle/_ref/gbref not built (no /root/reference)")


def same(a, b, label):
    assert a["hits"] == b["hits"], label
    assert a["docs_wanted"] == b["docs_wanted"], label
    assert np.array_equal(a["docids"], b["docids"]), label
    assert np.array_equal(a["scores"].view(np.uint32), b["scores"].view(np.uint32)), label


@pytest.mark.parametrize("seed", [11, 12, 13])
def test_kinds_vs_reference(seed):
    N = 15000
    for q in qkinds.kinds(N, seed=seed):
        lists = generate(q, N, seed=seed * 7)
        p = q.params()
        r = ref.query(q.terms, lists, p, votes=True)
        same(orc.query(q.terms, lists, p), r, f"{q.name} seed={seed}")
        assert np.array_equal(orc.intersect(q.terms, lists), r["votes"]), q.name


def test_two_term_large_vs_reference():
    q = config_two_term(300_000, docs_to_get=100, seed=21)
    lists = generate(q, 300_000, seed=21)
    same(orc.query(q.terms, lists, q.params()), ref.query(q.terms, lists, q.params()), "two_term 300k")


@pytest.mark.parametrize("seed", range(4))
def test_merge_vs_reference(seed):
    runs = tiered_runs(20000 + 15000 * seed, seed=100 + seed, nterms=[2, 40, 400, 1][seed])
    keep, ptrs, sizes = orc._lists(runs)
    cap = sum(map(len, runs)) + 64
    for rm in (0, 1):
        for mrs in (-1, 0, 1, 4096, 100_000):
            out = ctypes.create_string_buffer(cap)
            n = orc.lib().orc_posdb_merge(ptrs, sizes, len(runs), rm, mrs, out, cap)
            assert out.raw[:n] == ref.posdb_merge(runs, rm, mrs), (seed, rm, mrs)


@pytest.mark.parametrize("splits", [2, 3, 7])
def test_docid_splits_vs_reference(splits):
    # Msg39's docid-split loop (Msg39.cpp:345-457) played by the harness with
    # the reference's own RdbList::constrain per piece
    N = 8000
    for q in qkinds.kinds(N, seed=31):
        lists = generate(q, N, seed=splits)
        for dtg in (q.docs_to_get, 700):
            q.docs_to_get = dtg
            p = q.params()
            p.num_docid_splits = splits
            same(orc.query(q.terms, lists, p), ref.query(q.terms, lists, p), f"{q.name} S={splits} dtg={dtg}")


def skewed_docids(n, seed, ndom=3, frac=0.7):
    """n distinct sorted docids, `frac` of them in `ndom` domains (domHash8 =
    bits 6..13 of the docid, Titledb.h:114-115): drives TopTree's per-domain
    caps (m_cap, m_partial, m_ridiculousMax, TopTree.cpp:64-186, 355-399)."""
    rng = np.random.default_rng(seed)
    doms = rng.choice(256, ndom, replace=False)
    out = set()
    while len(out) < n:
        d = int(rng.integers(0, 1 << 38))
        if rng.random() < frac:
            d = (d & ~0x3fc0) | (int(doms[rng.integers(0, ndom)]) << 6)
        out.add(d)
    return sorted(out)


def compare_full(q, lists, p, label):
    r = ref.query(q.terms, lists, p, cap=1 << 16, votes=True)
    o = orc.query(q.terms, lists, p, cap=1 << 16)
    same(o, r, label)
    assert o["filtered"] == r["filtered"], label
    return r


@pytest.mark.parametrize("seed", [41, 42])
def test_site_clustering_vs_reference(seed):
    # Msg39Request defaults (Msg39.h:36-82): m_doSiteClustering and
    # m_doMaxScoreAlgo on -- the TopTree holds more than docsWanted nodes and
    # the getMaxPossibleScore / ring-buffer prefilters prune
    N = 15000
    for q in qkinds.kinds(N, seed=seed):
        lists = generate(q, N, seed=seed * 3)
        for dtg in (q.docs_to_get, 10, 137):
            q.docs_to_get = dtg
            r = compare_full(q, lists, q.params(site_clustering=1), f"{q.name} dtg={dtg}")
            assert len(r["docids"]) > 0 or r["hits"] == 0


@pytest.mark.parametrize("ndom,frac", [(1, 0.9), (3, 0.7), (12, 0.5)])
def test_site_clustering_skewed_domains_vs_reference(ndom, frac):
    import posdb_py
    N = 6000
    for q in qkinds.kinds(N, seed=51)[:6]:
        lists = generate(q, N, seed=ndom)
        nd = len({int(d) for l in lists for d in posdb_py.docids(l)})
        lists = posdb_py.remap_docids(lists, skewed_docids(nd, seed=ndom, ndom=ndom, frac=frac))
        for dtg in (10, 25, 60):
            q.docs_to_get = dtg
            for mx in (1, 0):
                p = q.params(site_clustering=1)
                p.do_max_score_algo = mx
                compare_full(q, lists, p, f"{q.name} ndom={ndom} dtg={dtg} mx={mx}")


@pytest.mark.parametrize("splits", [2, 5])
def test_site_clustering_docid_splits_vs_reference(splits):
    N = 8000
    for q in qkinds.kinds(N, seed=61)[:8]:
        lists = generate(q, N, seed=splits + 60)
        p = q.params(site_clustering=1, num_docid_splits=splits)
        compare_full(q, lists, p, f"{q.name} S={splits}")


def test_paging_filter_vs_reference():
    # the widget's next page: m_maxSerpScore / m_minSerpDocId (Posdb.cpp:4379-4381,
    # 7327-7347) drop docids scoring above the last shown one (m_filtered)
    N = 15000
    for q in qkinds.kinds(N, seed=71):
        lists = generate(q, N, seed=71)
        full = ref.query(q.terms, lists, q.params())
        if len(full["docids"]) < 3:
            continue
        for pos in (0, len(full["docids"]) // 2, len(full["docids"]) - 1):
            for clus in (0, 1):
                p = q.params(site_clustering=clus, max_serp_score=float(full["scores"][pos]),
                             min_serp_docid=int(full["docids"][pos]))
                r = compare_full(q, lists, p, f"{q.name} pos={pos} clus={clus}")
                assert clus or r["filtered"] >= pos
