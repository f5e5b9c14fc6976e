"""Multi-GPU decomposition on CPU, world_size 2 over gloo (the same exchange
bench.py runs over RCCL): each rank takes one docid range of every termlist
(SURVEY.md §8(e)), scores it (here with the oracle -- the GPU scorer is parity
checked on its own in test_gpu_parity.py), the top lists are all-gathered and
merged Msg3a-style.  The merged top-k and the summed hit count must equal the
unsharded query's: without site clustering a docid's score depends only on its
own keys."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

N = 60000


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, kind, k, out):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [here, os.path.join(os.path.dirname(here), "open-source-search-engine_amd", "python")]
    import torch.distributed as dist
    import oracle_binding as orc
    import qkinds
    from shard_merge import gather_merge
    from workload import generate
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q = qkinds.kinds(N, seed=11)[kind]
        q.docs_to_get = k
        per = N // world
        lists = generate(q, N, seed=21, doc_begin=rank * per, doc_end=(rank + 1) * per if rank < world - 1 else N)
        r = orc.query(q.terms, lists, q.params())
        hits, d, s = gather_merge(r["docids"], r["scores"], r["hits"], k, device="cpu")
        if rank == 0:
            out.put((hits, d.tolist(), s.astype(np.float32).tolist()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("kind", [0, 2, 5])
def test_two_shards_merge_equals_unsharded(kind):
    import oracle_binding as orc
    import qkinds
    from workload import generate
    q = qkinds.kinds(N, seed=11)[kind]
    q.docs_to_get = 50
    full = generate(q, N, seed=21)
    exp = orc.query(q.terms, full, q.params())
    ctx = mp.get_context("spawn")
    out = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, kind, 50, out)) for r in range(2)]
    for p in procs:
        p.start()
    hits, d, s = out.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert hits == exp["hits"]
    n = len(exp["docids"])
    assert d[:n] == exp["docids"].tolist()
    assert np.array_equal(np.array(s[:n], np.float32).view(np.uint32), exp["scores"].view(np.uint32))
