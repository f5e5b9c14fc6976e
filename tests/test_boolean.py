"""Boolean queries (Query::m_isBoolean): makeDocIdVoteBufForBoolQuery_r
(Posdb.cpp:8006-8249) and the boolean branches of intersectLists10_r
(6312-6316, 6514-6534, 6833-6834, 7247-7256).

The docid set is the union of every group's sublists (negative groups too),
each docid carrying the bit vector of the QueryTermInfos it occurs in; it is
kept where the expression holds (the ABI takes the expression as its truth
table over those vectors) and scored as the number of bits set times the
same-language weight.  Parity: the reference's own fixtures
(tests/golden/q_bool_*.npz: six expressions x two seeds, site clustering,
docid splits, paging, a language, a whitelist, a negative term, an empty
smallest group, synonyms) pin the oracle (test_golden.py covers them on CPU
and GPU); here the GPU runs against the oracle on seeded corpora with random
truth tables -- any table is a valid expression input -- and the refused
modes fail loudly."""
import numpy as np
import pytest

import gbgpu
import oracle_binding as orc
import qkinds
from workload import generate


def table(ng, rng, density=0.5):
    nv = 1 << ng
    bits = rng.random(nv) < density
    bits[0] = rng.random() < 0.5  # the empty vector: only docids of no group reach it (none)
    out = np.zeros((nv + 7) // 8, np.uint8)
    for v in np.nonzero(bits)[0]:
        out[v >> 3] |= 1 << (v & 7)
    return out.tobytes()



KINDS = [1, 3, 4, 6, 0]  # three_word, negative, synonyms, piped, config-2 two-term


def test_oracle_boolean_random_tables():
    rng = np.random.default_rng(5)
    for k in KINDS:
        q = qkinds.kinds(4000, seed=7)[k]
        lists = generate(q, 4000, seed=70 + k)
        ng = sum(1 for t in q.terms if t.is_required)
        for _ in range(3):
            p = q.params().with_boolean(table(ng, rng), ng)
            r = orc.query(q.terms, lists, p)
            v = orc.intersect(q.terms, lists, params=p)
            assert r["hits"] == len(v)
            assert np.all(np.diff(v) > 0)  # sorted by docid, each once (dcmp6)
            # every score is a bit count times the same-language weight
            s = np.asarray(r["scores"], np.float64) / p.same_lang_weight
            assert np.all((s >= 1) & (s <= ng) & (s == np.round(s)))


@pytest.mark.gpu
@pytest.mark.parametrize("clus", [0, 1])
@pytest.mark.parametrize("kind", KINDS)
def test_gpu_boolean_vs_oracle(engine, kind, clus):
    rng = np.random.default_rng(100 + kind + 10 * clus)
    q = qkinds.kinds(20000, seed=3)[kind]
    lists = generate(q, 20000, seed=300 + kind)
    ng = sum(1 for t in q.terms if t.is_required)
    for it in range(4):
        p = q.params(site_clustering=clus, language=(it & 1) * 5).with_boolean(table(ng, rng, 0.3 + 0.15 * it), ng)
        exp = orc.query(q.terms, lists, p, cap=1 << 16)
        exp["votes"] = orc.intersect(q.terms, lists, params=p)
        r = engine.query(q.terms, lists, p, cap=1 << 16, hit_cap=1 << 22)
        label = f"{q.name} clus={clus} it={it}"
        assert r.hits == exp["hits"], label
        assert np.array_equal(r.hit_docids, exp["votes"]), label
        assert r.docs_wanted == exp["docs_wanted"], label
        assert r.filtered == exp["filtered"], label
        assert np.array_equal(r.docids, exp["docids"]), label
        assert np.array_equal(r.scores.view(np.uint32), exp["scores"].view(np.uint32)), label


@pytest.mark.gpu
@pytest.mark.parametrize("splits", [2, 5])
def test_gpu_boolean_docid_splits_vs_oracle(engine, splits):
    rng = np.random.default_rng(splits)
    q = qkinds.kinds(20000, seed=4)[1]
    lists = generate(q, 20000, seed=404)
    p = q.params(num_docid_splits=splits).with_boolean(table(3, rng), 3)
    exp = orc.query(q.terms, lists, p, cap=1 << 16)
    r = engine.query(q.terms, lists, p, cap=1 << 16)
    assert (r.hits, r.filtered) == (exp["hits"], exp["filtered"])
    assert np.array_equal(r.docids, exp["docids"])
    assert np.array_equal(r.scores.view(np.uint32), exp["scores"].view(np.uint32))


@pytest.mark.gpu
def test_gpu_boolean_refused_modes(engine):
    q = qkinds.kinds(5000, seed=1)[1]
    lists = generate(q, 5000)
    tab = bytes([0xa8])
    with pytest.raises(gbgpu.GbgpuError) as e:  # the table must be over the plan's groups
        engine.query(q.terms, lists, q.params().with_boolean(tab, 2))
    assert e.value.code == 22  # EINVAL
    terms = list(q.terms)
    terms[0] = gbgpu.QTerm(*[getattr(terms[0], f) for f, _ in gbgpu.QTerm._fields_])
    terms[0].field_code = 54  # gbsortby: reads a mini-merged list that may be stale
    with pytest.raises(gbgpu.GbgpuError) as e:
        engine.query(terms, lists, q.params().with_boolean(tab, 3))
    assert e.value.code == gbgpu.GBGPU_EUNSUPPORTED
