"""Golden vectors produced by the REFERENCE's own PosdbTable / TopTree /
RdbList::merge_r (tests/make_golden.py, oracle/_ref/gbref).

CPU tests pin the oracle (oracle/posdb_oracle.c, posdb_merge_oracle.c) to the
reference; GPU tests check the HIP path against the same vectors through the
C ABI.  Bar: docid sets and top-k order bit-exact, scores bit-exact (the
north_star tolerance 1e-5 relative is asserted too)."""
import ctypes
import glob
import os

import numpy as np
import pytest

import gbgpu
import oracle_binding as orc

HERE = os.path.dirname(os.path.abspath(__file__))
QCASES = sorted(glob.glob(os.path.join(HERE, "golden", "q_*.npz")))
MCASES = sorted(glob.glob(os.path.join(HERE, "golden", "m_*.npz")))
REL_TOL = 1e-5


def split_blob(sizes, blob):
    out, off = [], 0
    for s in sizes:
        out.append(blob[off:off + s].tobytes())
        off += s
    return out


def load_query(path):
    z = np.load(path, allow_pickle=False)
    terms = [gbgpu.QTerm(*[int(x) for x in row], float(w)) for row, w in zip(z["qterms"], z["tfw"])]
    if "qnum_f" in z:  # range terms' bounds (m_qword->m_float / m_int)
        for t, f, i in zip(terms, z["qnum_f"], z["qnum_i"]):
            t.number_float, t.number_int = float(f), int(i)
    pr = z["params"]
    # the harness ran Msg39Request::reset() (m_doMaxScoreAlgo = true) before
    # the fields a fixture names
    do_max = int(pr[5]) if len(pr) > 5 else 1
    params = gbgpu.Params(int(pr[0]), int(pr[1]), int(pr[2]), int(pr[3]), int(pr[4]), float(z["same_lang_weight"]),
                          do_max, 0, float(z["max_serp_score"]) if "max_serp_score" in z else 0.0,
                          int(z["min_serp_docid"]) if "min_serp_docid" in z else 0)
    if "use_whitelist" in z and int(z["use_whitelist"]):
        params = params.with_whitelist(split_blob(z["white_sizes"], z["white_blob"]))
    if "franges_term" in z:  # gbfacetint:/gbfacetfloat: ranges
        fr, off = [], 0
        for t, n in zip(z["franges_term"], z["franges_n"]):
            fr.append((int(t), z["franges_a"][off:off + n].tolist(), z["franges_b"][off:off + n].tolist()))
            off += int(n)
        params = params.with_facets(fr)
    if "bool_tok" in z:  # a boolean query: its expression and the reference's truth table
        params = params.with_boolean(z["bool_table"].tobytes(), int(z["bool_groups"]), [int(x) for x in z["bool_tok"]])
    lists = split_blob(z["list_sizes"], z["list_blob"])
    exp = dict(docids=z["docids"], scores=z["score_bits"].view(np.float32), hits=int(z["hits"]),
               docs_wanted=int(z["docs_wanted"]), votes=z["votes"],
               filtered=int(z["filtered"]) if "filtered" in z else None)
    if "facet_term" in z:
        exp["facets"], off = {}, 0
        for t, d, n in zip(z["facet_term"], z["facet_docs"], z["facet_n"]):
            keys = z["facet_keys"][off:off + n]
            vals = z["facet_vals"][off:off + n]
            exp["facets"][int(t)] = (int(d), {int(k): tuple(int(x) for x in v) for k, v in zip(keys, vals)})
            off += int(n)
    return terms, lists, params, exp


def check(got, exp, label):
    assert got["hits"] == exp["hits"], label
    if exp.get("facets") is not None and got.get("facets") is not None:
        # QueryTerm::m_facetHashTable entry by entry, and m_numDocsThatHaveFacet
        assert got["facets"] == exp["facets"], label
    assert got["docs_wanted"] == exp["docs_wanted"], label
    if exp.get("filtered") is not None:
        assert got["filtered"] == exp["filtered"], label
    if got.get("hit_docids") is not None:
        # the intersected docid set itself (m_docIdVoteBuf), bit-exact
        assert np.array_equal(got["hit_docids"], exp["votes"]), label
    assert np.array_equal(got["docids"], exp["docids"]), label
    g = np.asarray(got["scores"], np.float32)
    rel = np.abs(g.astype(np.float64) - exp["scores"]) / np.maximum(1e-30, np.abs(exp["scores"]))
    assert np.all(rel <= REL_TOL), (label, rel.max() if len(rel) else 0)
    assert np.array_equal(g.view(np.uint32), exp["scores"].view(np.uint32)), label


def orc_merge(lists, rm, mrs):
    keep, ptrs, sizes = orc._lists(lists)
    cap = sum(map(len, lists)) + 64
    out = ctypes.create_string_buffer(cap)
    n = orc.lib().orc_posdb_merge(ptrs, sizes, len(lists), rm, mrs, out, cap)
    assert n >= 0, n
    return out.raw[:n]


def test_fixtures_present():
    assert len(QCASES) >= 30 and len(MCASES) >= 4


@pytest.mark.parametrize("path", QCASES, ids=[os.path.basename(p)[2:-4] for p in QCASES])
def test_oracle_query_vs_reference(path):
    terms, lists, params, exp = load_query(path)
    got = orc.query(terms, lists, params, cap=1 << 16)
    check(got, exp, os.path.basename(path))


@pytest.mark.parametrize("path", QCASES, ids=[os.path.basename(p)[2:-4] for p in QCASES])
def test_oracle_intersection_vs_reference(path):
    terms, lists, params, exp = load_query(path)
    # m_docIdVoteBuf after intersectLists10_r: the exact intersected docid set
    assert np.array_equal(orc.intersect(terms, lists, params=params), exp["votes"])


@pytest.mark.parametrize("path", MCASES, ids=[os.path.basename(p)[2:-4] for p in MCASES])
def test_oracle_merge_vs_reference(path):
    z = np.load(path, allow_pickle=False)
    runs = split_blob(z["run_sizes"], z["run_blob"])
    outs = split_blob(z["out_sizes"], z["out_blob"])
    for rm, mrs, want in zip(z["remove_neg"], z["min_rec_sizes"], outs):
        assert orc_merge(runs, int(rm), int(mrs)) == want, (int(rm), int(mrs))


@pytest.mark.gpu
@pytest.mark.parametrize("path", QCASES, ids=[os.path.basename(p)[2:-4] for p in QCASES])
def test_gpu_query_vs_reference(engine, path):
    terms, lists, params, exp = load_query(path)
    r = engine.query(terms, lists, params, cap=1 << 16, hit_cap=max(1, exp["hits"]))
    check(dict(docids=r.docids, scores=r.scores, hits=r.hits, docs_wanted=r.docs_wanted, filtered=r.filtered,
               hit_docids=r.hit_docids, facets=r.facets), exp, os.path.basename(path))
