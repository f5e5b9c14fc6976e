"""Msg39 -> Msg3a exchange through the C ABI on the GPU.

gbgpu_allgather_topk all-gathers every shard's reply over RCCL and merges
them on the device by Msg3a::mergeLists' rules (Msg3a.cpp:1315-1467).  One
GPU box cannot run several ranks, so the device merge is checked on its own
against the host restatement (gbgpu_merge_topk) for 1-8 shards with ties and
duplicate docids, and the whole collective runs as a one-rank communicator.
The multi-rank exchange semantics are covered on CPU (test_shards_gloo.py)."""
import numpy as np
import pytest

import gbgpu
import oracle_binding as orc
import qkinds
from workload import generate

pytestmark = pytest.mark.gpu


def random_replies(rng, nranks, k, ties, dup):
    shards = []
    pool = rng.choice(1 << 38, size=nranks * k * 2, replace=False)
    for r in range(nranks):
        n = int(rng.integers(0, k + 1))
        sc = np.sort(rng.choice(np.arange(1, 50 if ties else 100000), size=n).astype(np.float32))[::-1]
        dd = pool[r * 2 * k:r * 2 * k + n].copy()
        if dup and r > 0 and n:
            m = int(rng.integers(0, n))
            dd[:m] = shards[0][0][:m] if len(shards[0][0]) >= m else dd[:m]
            sc[:m] = shards[0][1][:m] if len(shards[0][1]) >= m else sc[:m]
        # each reply sorted best first: score desc, docid asc
        o = np.lexsort((dd, -sc.astype(np.float64)))
        shards.append((dd[o], sc[o]))
    return shards


@pytest.mark.parametrize("nranks", [1, 2, 3, 8])
@pytest.mark.parametrize("ties,dup", [(False, False), (True, False), (True, True)])
def test_device_merge_matches_msg3a(engine, nranks, ties, dup):
    rng = np.random.default_rng(nranks * 7 + ties * 3 + dup)
    for k in (1, 10, 100, 300):
        shards = random_replies(rng, nranks, k, ties, dup)
        hits = [int(x) for x in rng.integers(0, 1 << 40, nranks)]
        d, s, h = engine.merge_replies_device(shards, k, hits)
        ed, es = gbgpu.merge_topk(shards, k)
        assert h == sum(hits)
        assert np.array_equal(d, ed), (nranks, k)
        assert np.array_equal(s, es), (nranks, k)


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
