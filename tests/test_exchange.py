"""Msg39 -> Msg3a exchange through the C ABI on the GPU.

gbgpu_allgather_topk all-gathers every shard's reply over RCCL and merges
them on the device (k_xmerge) by Msg3a::mergeLists' rules (Msg3a.cpp:
971-1503).  One GPU box cannot run several ranks, so the device merge is
checked on its own (gbgpu_merge_topk_device) against the reference's own
mergeLists (tests/golden/x_*.npz) and against the oracle restatement on
seeded reply sets, and the whole collective runs as a one-rank communicator.
The multi-rank ordering (gbgpu_seq) is covered on CPU (test_shards_gloo.py)."""
import errno

import numpy as np
import pytest

import gbgpu
import msg3a_cases
import oracle_binding as orc
import qkinds
from test_msg3a import FIX, load_fixture, same
from workload import generate

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("path", FIX, ids=[p.rsplit("/", 1)[1][:-4] for p in FIX])
def test_device_merge_matches_reference_fixture(engine, path):
    shards, k, ed, es = load_fixture(path)
    hits = list(range(1, len(shards) + 1))
    d, s, h = engine.merge_topk_device(shards, k, hits)
    assert h == sum(hits)
    assert same(d, s, ed, es)


@pytest.mark.parametrize("nranks", [1, 2, 3, 8, 64])
def test_device_merge_matches_oracle(engine, nranks):
    rng = np.random.default_rng(nranks * 7)
    for it, k in enumerate((1, 10, 100, 300, 4096)):
        shards = msg3a_cases.partitioned(rng, nranks, int(rng.integers(0, 200)), int(rng.integers(1, 40)),
                                         int_scores=bool(it % 2))
        if it == 3:  # replicas
            shards = (shards + shards)[:max(nranks, 2)]
        ed, es = orc.msg3a_merge(shards, k)
        d, s, _ = engine.merge_topk_device(shards, k, [0] * len(shards))
        assert same(d, s, ed, es), (nranks, k)


@pytest.mark.parametrize("nranks", [2, 3, 8])
def test_device_merge_nan_scores_shard_order(engine, nranks):
    # NaN scores make Msg3a's comparisons partial: its scan over the shards
    # in order (Msg3a.cpp:1323-1334) falls through to the docid compare on
    # any NaN, so the pick depends on the shard order -- which the device
    # merge walks as the reference does (parity with the reference's own
    # rules as restated by the oracle and the host merge; no reference
    # fixture holds NaN)
    rng = np.random.default_rng(nranks * 13 + 1)
    for k in (5, 50, 400):
        shards = msg3a_cases.partitioned(rng, nranks, int(rng.integers(20, 120)), int(rng.integers(1, 10)))
        shards = [(d, np.where(rng.random(len(sc)) < 0.2, np.nan, sc)) for d, sc in shards]
        ed, es = orc.msg3a_merge(shards, k)
        hd, hs = gbgpu.merge_topk(shards, k)
        d, s, _ = engine.merge_topk_device(shards, k, [0] * len(shards))
        assert same(d, s, ed, es), (nranks, k)
        assert same(hd, hs, ed, es), (nranks, k)


def test_allgather_topk_one_rank():
    # the whole collective (pack, RCCL all-gather, device merge) as one rank
    q = qkinds.kinds(20000, seed=3)[2]
    lists = generate(q, 20000, seed=33)
    p = q.params()
    exp = orc.query(q.terms, lists, p)
    with gbgpu.Engine(0) as eng:
        eng.comm_init(1, 0, gbgpu.Engine.comm_unique_id())
        hs = [eng.upload(l) for l in lists]
        for k in (10, q.docs_to_get, 2 * q.docs_to_get):
            eng.enqueue(q.terms, hs, p, slot=0)
            d, s, h = eng.allgather_topk(k, slot=0)
            m = min(k, len(exp["docids"]))
            ed, es = orc.msg3a_merge([(exp["docids"][:m], exp["scores"][:m].astype(np.float64))], k)
            assert same(d, s, ed, es)
            assert h == exp["hits"]
            assert np.array_equal(d, exp["docids"][:m])
            assert np.array_equal(s, exp["scores"][:m].astype(np.float64))
        # gbsortby int: the tree orders by m_intScore and the wire carries
        # (double)m_intScore (Msg39.cpp:1663-1664)
        from numlists import number_list
        terms = list(q.terms)
        t = gbgpu.QTerm(1, 0, 59, 0, -1, -1, -1, 0, max(x.qpos for x in terms) + 2, 0, -1, 1.0)
        terms.append(t)
        lists3 = list(lists) + [number_list(lists, 0.7, seed=9, ints=True)]
        hs3 = [eng.upload(l) for l in lists3]
        ref = eng.query_resident(terms, hs3, p, cap=1 << 12)
        eng.enqueue(terms, hs3, p, slot=0)
        d, s, h = eng.allgather_topk(q.docs_to_get, slot=0)
        m = min(q.docs_to_get, len(ref.docids))
        assert np.array_equal(d, ref.docids[:m])
        assert np.array_equal(s, ref.int_scores[:m].astype(np.float64))
        # an empty shard (all lists empty) replies with nothing
        hs2 = [eng.upload(b"") for _ in lists]
        eng.enqueue(q.terms, hs2, p, slot=0)
        d, s, h = eng.allgather_topk(10, slot=0)
        assert len(d) == 0 and h == 0
        # a shard with no query of its own (slot < 0) sends an empty reply
        d, s, h = eng.allgather_topk(10, slot=-1)
        assert len(d) == 0 and h == 0
        # sequence numbers: an explicit number already past is refused
        with pytest.raises(gbgpu.GbgpuError):
            eng.allgather_topk(10, slot=-1, seq=0, timeout_ms=0)

        # a failure after admission still takes part in the collective (an
        # empty reply) and uses its sequence number up, so the next exchange
        # pairs with the other ranks' next one: an idle slot, a bad slot
        nxt = eng._xseq
        with pytest.raises(gbgpu.GbgpuError) as ei:
            eng.allgather_topk(10, slot=0)  # slot 0 holds no query
        assert ei.value.code == errno.EINVAL
        with pytest.raises(gbgpu.GbgpuError):
            eng.allgather_topk(10, slot=999)
        assert eng._xseq == nxt + 2
        eng.enqueue(q.terms, hs, p, slot=0)
        d, s, h = eng.allgather_topk(q.docs_to_get, slot=0, seq=nxt + 2, timeout_ms=1000)
        m = min(q.docs_to_get, len(exp["docids"]))
        assert np.array_equal(d, exp["docids"][:m]) and h == exp["hits"]
        # a number whose turn never comes times out and is not used up
        with pytest.raises(gbgpu.GbgpuError) as ei:
            eng.allgather_topk(10, slot=-1, seq=nxt + 5, timeout_ms=10)
        assert ei.value.code == errno.ETIMEDOUT
        assert eng._xseq == nxt + 3


def test_allgather_refused_k_leaves_sequence():
    """A k out of range is refused before admission: the default sequence
    number is not used up, so the next default call is admitted at once
    (it would wait forever on a number never entered otherwise)."""
    with gbgpu.Engine(0) as eng:
        eng.comm_init(1, 0, gbgpu.Engine.comm_unique_id())
        for bad in (0, -1, 4097):
            with pytest.raises(gbgpu.GbgpuError) as ei:
                eng.allgather_topk(bad, slot=-1)
            assert ei.value.code == errno.EINVAL
            assert eng._xseq == 0
        d, s, h = eng.allgather_topk(10, slot=-1, timeout_ms=5000)
        assert len(d) == 0 and h == 0 and eng._xseq == 1


@pytest.mark.parametrize("name", ["q_clus_prune_100k", "q_clus_dense", "q_clus_three_word"])
def test_allgather_clustered_register_overflow(name):
    """A clustered query whose TopTree outgrows k_tree_seq's register
    columns (forced here: one column, GBGPU_REPLAY_MODE=3 in the diagnostic
    build) replays on the device before the exchange packs the result block,
    so the all-gathered reply is the query's final tree, not a stale one."""
    import os
    from test_golden import load_query
    terms, lists, params, exp = load_query(os.path.join(os.path.dirname(__file__), "golden", name + ".npz"))
    k = max(1, min(len(exp["docids"]), 4096))
    old = os.environ.get("GBGPU_REPLAY_MODE")
    os.environ["GBGPU_REPLAY_MODE"] = "3"
    try:
        eng = gbgpu.Engine(0, diag=True)
    finally:
        if old is None:
            del os.environ["GBGPU_REPLAY_MODE"]
        else:
            os.environ["GBGPU_REPLAY_MODE"] = old
    try:
        eng.comm_init(1, 0, gbgpu.Engine.comm_unique_id())
        hs = [eng.upload(l) for l in lists]
        # a previous, different query leaves its result in the slot's buffers
        other = [eng.upload(l) for l in lists[::-1]]
        eng.enqueue(terms, other, params, slot=0)
        eng.collect(slot=0)
        eng.enqueue(terms, hs, params, slot=0)
        d, s, h = eng.allgather_topk(k, slot=0)
        m = min(k, len(exp["docids"]))
        assert np.array_equal(d, exp["docids"][:m]), name
        assert np.array_equal(s, exp["scores"][:m].astype(np.float64)), name
        assert h == exp["hits"]
    finally:
        eng.close()
