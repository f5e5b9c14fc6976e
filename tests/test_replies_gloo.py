"""Msg3a::mergeLists whole across two ranks on CPU, world_size 2 over gloo:
the full-reply form of the exchange with the library's own
pieces -- the sequencer (gbgpu_seq, the order gbgpu_allgather_replies
admits exchanges in) and the host merge of full replies
(gbgpu_merge_replies, the rules the device merge after the RCCL all-gather
applies: the site cap over cluster records, the facet tables, the summed
hits and facet counts).

Each rank holds a contiguous block of the shards of every reference fixture
(tests/golden/x3_*: the reference's own Msg3a::mergeLists over 3-8 shard
replies, gbref op 8), serves the fixtures from concurrent threads that finish
in a rank-specific order, all-gathers its replies under the fixture's
sequence number, and merges the gathered replies in rank order, which is the
fixture's shard order.  Every rank's result must be the reference's."""
import glob
import os
import socket

import numpy as np
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
FIX = sorted(glob.glob(os.path.join(HERE, "golden", "x3_*.npz")))
THREADS = 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, out):
    import sys
    import threading
    import time
    sys.path[:0] = [HERE, os.path.join(os.path.dirname(HERE), "open-source-search-engine_amd", "python")]
    import torch.distributed as dist
    import gbgpu
    import msg3a_cases
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cases = [msg3a_cases.load_full(p) for p in FIX]
        sq = gbgpu.Seq(0)
        results, errors = {}, []
        todo = list(range(len(cases)))
        mu = threading.Lock()

        def serve(t):
            try:
                rng = np.random.default_rng(rank * 10 + t)
                while True:
                    with mu:
                        if not todo:
                            return
                        seq = todo.pop(0)
                    name, req, shards, _ = cases[seq]
                    ns = len(shards)
                    lo, hi = rank * ns // world, (rank + 1) * ns // world
                    mine = shards[lo:hi]  # this rank's Msg39 replies
                    time.sleep(float(rng.random()) * 0.1)
                    sq.enter(seq, timeout_ms=60000)
                    try:
                        got = [None] * world
                        dist.all_gather_object(got, (seq, mine))
                    finally:
                        sq.leave(seq)
                    if any(g[0] != seq for g in got):
                        errors.append(("paired different exchanges", seq, [g[0] for g in got]))
                        continue
                    gathered = [r for g in got for r in g[1]]
                    results[seq] = gbgpu.merge_replies(req, gathered)
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


def test_two_ranks_full_reply_exchange_equals_reference():
    import msg3a_cases
    from test_msg3a_full import check
    cases = [msg3a_cases.load_full(p) for p in FIX]
    assert len(cases) >= 10
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
        assert nxt == len(cases)
        assert sorted(results) == list(range(len(cases)))
        for seq, res in results.items():
            name, req, shards, exp = cases[seq]
            check(req, shards, exp, res, f"rank {rank} {name}")
