"""Full-size parity on the GPU: the exact workloads bench.py times
(BASELINE.json configs 2-5), checked against the oracle at full size.

* config 2: the 100M-doc 2-term query (219 MB of lists) -- every query the
  bench rotates over, intersected docid set, hit count, top-k docids and
  score bits; also with site clustering (the Msg39Request default);
* config 3: the bench's ten 3-5 word queries (config3_queries(1e8, seed=3),
  628 MB of lists each on average);
* config 4: all eight 125M-doc shards of the 1B-doc index (docid-range
  sharding), each checked on its own, then the device Msg3a merge of their
  replies against the oracle's mergeLists and the unsharded query;
* config 5: the 4.4 GB eight-run merge, output bytes vs the oracle.

The oracle runs at ~1 GB/s of lists, so each case costs a few seconds."""
import ctypes

import numpy as np
import pytest

import gbgpu
import oracle_binding as orc
from workload import config3_queries, config_two_term, generate

pytestmark = pytest.mark.gpu

N2 = 100_000_000


def check_full(res, terms, lists, p, label):
    exp = orc.query(terms, lists, p, cap=1 << 16)
    votes = orc.intersect(terms, lists)
    assert res.hits == exp["hits"] == len(votes), label
    assert np.array_equal(res.hit_docids, votes), label
    assert res.docs_wanted == exp["docs_wanted"], label
    assert res.filtered == exp["filtered"], label
    assert np.array_equal(res.docids, exp["docids"]), label
    assert np.array_equal(res.scores.view(np.uint32), exp["scores"].view(np.uint32)), label
    return exp


def resident(engine, lists, terms, p):
    hs = [engine.upload(l) for l in lists]
    try:
        return engine.query_resident(terms, hs, p, cap=1 << 16, hit_cap=1 << 24)
    finally:
        for h in hs:
            engine.free(h)


@pytest.mark.parametrize("seed", [1, 2, 7])
def test_config2_fullsize(engine, seed):
    # bench.py rotates config 2 over queries with these seeds (distinct termIds)
    q = config_two_term(N2, docs_to_get=100, seed=seed)
    lists = generate(q, N2, threads=16)
    check_full(resident(engine, lists, q.terms, q.params()), q.terms, lists, q.params(), f"config2 seed={seed}")


def test_config2_fullsize_site_clustering(engine):
    q = config_two_term(N2, docs_to_get=100, seed=1)
    lists = generate(q, N2, threads=16)
    p = q.params(site_clustering=1)
    check_full(resident(engine, lists, q.terms, p), q.terms, lists, p, "config2 clustering")


@pytest.mark.parametrize("k", range(10))
def test_config3_bench_queries(engine, k):
    q = config3_queries(N2, docs_to_get=100)[k]
    lists = generate(q, N2, threads=16)
    check_full(resident(engine, lists, q.terms, q.params()), q.terms, lists, q.params(), q.name)


def test_config4_shards_and_merge(engine):
    # 1B docs, docid-range shards of 125M docs (one per GPU on the 8-GPU node):
    # all 8 shards in turn on this GPU, each bit-exact against the oracle, then
    # the device Msg3a merge (k_xmerge, the kernel gbgpu_allgather_topk runs
    # after its all-gather) of the 8 replies == the oracle's mergeLists of
    # them == the unsharded 1B-doc query's top 100 and hit count
    total, per = 1_000_000_000, 125_000_000
    q = config_two_term(total, docs_to_get=100, seed=1)
    p = q.params()
    replies, hits = [], []
    for r in range(8):
        lists = generate(q, total, doc_begin=r * per, doc_end=(r + 1) * per, threads=16)
        res = resident(engine, lists, q.terms, p)
        check_full(res, q.terms, lists, p, f"config4 shard {r}")
        n = min(len(res.docids), p.docs_to_get)
        replies.append((res.docids[:n], res.scores[:n].astype(np.float64)))
        hits.append(res.hits)
        del lists
    d, s, h = engine.merge_topk_device(replies, 100, hits)
    ed, es = orc.msg3a_merge(replies, 100)
    assert np.array_equal(d, ed) and np.array_equal(s, es)
    full = generate(q, total, threads=16)
    exp = orc.query(q.terms, full, p, cap=1 << 12)
    assert h == exp["hits"]
    assert np.array_equal(d, exp["docids"][:100])
    assert np.array_equal(s, exp["scores"][:100].astype(np.float64))


def test_config5_fullsize_merge(engine):
    # 400M keys in 8 tiered runs (1:2:..:128), ~4.4 GB: GPU bytes == oracle
    # bytes
    import torch
    m = gbgpu.MergeRuns(400_000_000, nruns=8, seed=5, nterms=20000, nthreads=16)
    try:
        sizes = [len(a) for a in m.arrays]
        cap = sum(sizes) + 64
        dev = [torch.from_numpy(a).to("cuda") for a in m.arrays]
        out = torch.empty(cap, dtype=torch.uint8, device="cuda")
        n = engine.merge_posdb_device([x.data_ptr() for x in dev], sizes, 0, -1, out.data_ptr(), cap)
        del dev
        ptrs = (ctypes.c_void_p * 8)(*[a.ctypes.data for a in m.arrays])
        sz = (ctypes.c_int64 * 8)(*sizes)
        ob = np.empty(cap, np.uint8)
        no = orc.lib().orc_posdb_merge(ptrs, sz, 8, 0, -1, ob.ctypes.data, cap)
        assert n == no
        assert np.array_equal(out[:n].cpu().numpy(), ob[:no])
    finally:
        m.free()
