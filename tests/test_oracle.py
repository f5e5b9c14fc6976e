"""The CPU restatement (oracle/) against independent recomputation.

Parity of the oracle with the reference's PosdbTable scores is unpinned
(DESIGN.md §Oracle); these tests pin what can be recomputed independently:
the intersected docid set (bit-exact, from a separate numpy decoder), the
weight tables' closed forms, the TopTree contract, and the committed golden
vectors (regression)."""
import glob
import os

import numpy as np
import pytest

import gbgpu
import oracle_binding as orc
import posdb_py
import qkinds
from workload import generate, read_case, read_result

BF_NEG = ord('-')


def expected_intersection(q, lists):
    """Groups as setQueryTermInfo builds them for these well-formed plans."""
    terms = q.terms
    sets = [set(posdb_py.docids(l)) if l else set() for l in lists]
    pos, neg = [], []
    for i, t in enumerate(terms):
        if not t.is_required:
            continue
        members = {i}
        for x in (t.left_phrase_term, t.right_phrase_term):
            if x >= 0:
                members.add(x)
                members |= {k for k, u in enumerate(terms) if u.synonym_of == x}
        members |= {k for k, u in enumerate(terms) if u.synonym_of == i}
        u = set().union(*[sets[m] for m in members])
        (neg if t.term_sign == BF_NEG else pos).append(u)
    if not pos:
        return set()
    r = set.intersection(*pos)
    for n in neg:
        r -= n
    return r


@pytest.mark.parametrize("kind", range(len(qkinds.kinds())))
def test_oracle_intersection_matches_numpy(kind):
    q = qkinds.kinds()[kind]
    lists = generate(q, 20000)
    got = orc.intersect(q.terms, lists)
    assert list(got) == sorted(got)
    assert set(got.tolist()) == expected_intersection(q, lists)
    res = orc.query(q.terms, lists, q.params())
    assert res["hits"] == len(got)
    assert set(res["docids"].tolist()) <= set(got.tolist())


@pytest.mark.parametrize("kind", range(len(qkinds.kinds())))
def test_oracle_topk_contract(kind):
    q = qkinds.kinds()[kind]
    lists = generate(q, 20000)
    res = orc.query(q.terms, lists, q.params())
    s, d = res["scores"], res["docids"]
    assert np.all(s > 0)
    # TopTree read high->low: score desc, then docid asc
    for i in range(1, len(s)):
        assert (s[i - 1] > s[i]) or (s[i - 1] == s[i] and d[i - 1] < d[i])
    assert len(s) <= res["docs_wanted"]
    # deterministic (no hidden state between calls)
    res2 = orc.query(q.terms, lists, q.params())
    assert np.array_equal(res2["docids"], d) and np.array_equal(res2["scores"].view(np.uint32), s.view(np.uint32))


def test_oracle_does_not_mutate_inputs():
    q = qkinds.kinds()[0]
    lists = generate(q, 5000)
    copies = [bytes(l) for l in lists]
    orc.query(q.terms, lists, q.params())
    assert copies == lists


def test_weight_tables():
    w = orc.weights()
    # density: 0.35 * 1.03445^i in float, capped at 1 (Posdb.cpp:1117-1125)
    s = np.float32(0.35)
    for i in range(32):
        if s > 1.0:
            s = np.float32(1.0)
        assert w["density"][i] == s
        s = np.float32(float(s) * 1.03445)
    assert np.array_equal(w["wordspam"], (np.arange(1, 17, dtype=np.float32) / np.float32(16)))
    assert np.array_equal(w["linker"], np.sqrt(1.0 + np.arange(16)).astype(np.float32))
    assert list(w["hashgroup"]) == [1.0, 8.0, 1.5, np.float32(0.3), np.float32(0.1), 16.0, 1.0, 0.0, 4.0, 1.0,
                                    np.float32(0.2)]
    assert np.all(w["diversity"] == 1.0)


def test_empty_and_missing_lists():
    q = qkinds.kinds()[0]
    lists = generate(q, 5000)
    # a required term whose own list is empty still matches through its
    # bigram sublist (the group is the union, Posdb.cpp:4555-4654)
    res = orc.query(q.terms, [lists[0], b"", lists[2]], q.params())
    assert res["hits"] == len(set(posdb_py.docids(lists[2])) & set(posdb_py.docids(lists[0])))
    # ... and with every sublist of the group empty: minListSize 0 -> no work
    res = orc.query(q.terms, [lists[0], b"", b""], q.params())
    assert res["hits"] == 0 and len(res["docids"]) == 0
    # all lists empty -> no top tree at all
    res = orc.query(q.terms, [b"", b"", b""], q.params())
    assert res["docs_wanted"] == 0 and res["hits"] == 0


def test_docs_wanted_sizing():
    # allocTopTree: min(docsToGet, sum(size/12)), floored at 30, capped 2x
    p = gbgpu.Params(10, 10, 0, 0, 1, 20.0)
    assert gbgpu.docs_wanted(p, [18]) == 30
    assert gbgpu.docs_wanted(p, [0, 0]) == 0
    p.docs_to_get = 100
    assert gbgpu.docs_wanted(p, [12 * 1000]) == 100
    assert gbgpu.docs_wanted(p, [12 * 50]) == 50
    assert gbgpu.docs_wanted(p, [12 * 5]) == 30


GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.mark.parametrize("case", sorted(glob.glob(os.path.join(GOLDEN, "*.case"))))
def test_oracle_golden(case):
    terms, lists, params = read_case(case)
    exp = read_result(case[:-5] + ".res")
    res = orc.query(terms, lists, params)
    assert res["hits"] == exp["hits"]
    assert np.array_equal(res["docids"], exp["docids"])
    assert np.array_equal(res["scores"].view(np.uint32), exp["scores"].view(np.uint32))
