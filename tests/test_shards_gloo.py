"""Multi-GPU decomposition on CPU, world_size 2 over gloo, through the
library's own exchange pieces: the sequencer (gbgpu_seq, the ordering
gbgpu_allgather_topk applies) and the host Msg3a merge (gbgpu_merge_topk,
the rules k_xmerge applies after the RCCL all-gather).

Each rank holds one docid range of every termlist and
serves several queries from concurrent threads -- as Msg39's INTERSECT
threads do, taking requests in arrival order -- that finish in a different
order on each rank.  Every thread
enters the sequencer with the query's agreed sequence number before its
collective, so the all-gathers pair the same query on both ranks; the
merged top list and the summed hit count must equal the unsharded query's
(without site clustering a docid's score depends only on its own keys).
The shard results come from the oracle here (the GPU scorer is parity
checked on its own in the -m gpu tests)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

N = 60000
KINDS = [0, 2, 5]
THREADS = 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _queries():
    import qkinds
    qs = []
    for kind in KINDS:
        q = qkinds.kinds(N, seed=11)[kind]
        q.docs_to_get = 50
        qs.append(q)
    return qs * 2  # each query twice: six exchanges


def _rank(rank, world, port, out):
    import sys
    import threading
    import time
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [here, os.path.join(os.path.dirname(here), "open-source-search-engine_amd", "python")]
    import torch.distributed as dist
    import gbgpu
    import oracle_binding as orc
    from workload import generate
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        qs = _queries()
        per = N // world
        sq = gbgpu.Seq(0)
        results = {}
        errors = []
        # queries are dispatched to the threads in arrival (= sequence) order,
        # as Msg39 hands requests to its INTERSECT threads; each takes its own
        # time (a rank-specific delay), so they finish out of order
        todo = list(range(len(qs)))
        todo_mu = threading.Lock()

        def serve(t):
            try:
                rng = np.random.default_rng(rank * 10 + t)
                while True:
                    with todo_mu:
                        if not todo:
                            return
                        seq = todo.pop(0)
                    q = qs[seq]
                    lists = generate(q, N, seed=21 + seq % len(KINDS), doc_begin=rank * per,
                                     doc_end=(rank + 1) * per if rank < world - 1 else N)
                    r = orc.query(q.terms, lists, q.params())
                    time.sleep(float(rng.random()) * 0.2)
                    n = min(len(r["docids"]), q.docs_to_get)
                    reply = (seq, r["docids"][:n], r["scores"][:n].astype(np.float64), int(r["hits"]))
                    sq.enter(seq, timeout_ms=60000)
                    try:
                        got = [None] * world
                        dist.all_gather_object(got, reply)
                    finally:
                        sq.leave(seq)
                    if any(g[0] != seq for g in got):
                        errors.append(("paired different queries", seq, [g[0] for g in got]))
                        continue
                    d, s = gbgpu.merge_topk([(g[1], g[2]) for g in got], q.docs_to_get)
                    results[seq] = (sum(g[3] for g in got), d.tolist(), s.tolist())
            except Exception as e:  # reported to the parent
                errors.append(repr(e))

        th = [threading.Thread(target=serve, args=(t,)) for t in range(THREADS)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=120)
        out.put((rank, results, errors, sq.next()))
    finally:
        dist.destroy_process_group()


def test_two_shards_concurrent_exchange_equals_unsharded():
    import oracle_binding as orc
    from workload import generate
    qs = _queries()
    ctx = mp.get_context("spawn")
    out = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, out)) for r in range(2)]
    for p in procs:
        p.start()
    got = [out.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, results, errors, nxt in got:
        assert not errors, errors
        assert nxt == len(qs)
        assert sorted(results) == list(range(len(qs)))
        for seq, (hits, d, s) in results.items():
            q = qs[seq]
            exp = orc.query(q.terms, generate(q, N, seed=21 + seq % len(KINDS)), q.params())
            n = len(exp["docids"])
            assert hits == exp["hits"], (rank, seq)
            assert d[:n] == exp["docids"].tolist(), (rank, seq)
            assert np.array_equal(np.array(s[:n], np.float32).view(np.uint32), exp["scores"].view(np.uint32))
