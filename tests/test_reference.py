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
