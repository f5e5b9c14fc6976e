"""Msg3a::mergeLists (Msg3a.cpp:971-1503), the global merge of the shards'
Msg39 replies, on CPU.

* the oracle restatement (oracle/msg3a_oracle.c) and the library's host merge
  (gbgpu_merge_topk) against the reference's own mergeLists (fixtures
  tests/golden/x_*.npz from oracle/_ref/gbref, and live where gbref exists);
* the exchange sequencer (gbgpu_seq) that makes concurrent INTERSECT threads
  issue the collectives in the same order on every rank.
The device merge (k_xmerge) is checked against the same fixtures in
test_exchange.py (GPU)."""
import glob
import os
import threading
import time

import numpy as np
import pytest

import gbgpu
import msg3a_cases
import oracle_binding as orc

GOLD = os.path.join(os.path.dirname(__file__), "golden")
FIX = sorted(glob.glob(os.path.join(GOLD, "x_*.npz")))


def load_fixture(path):
    z = np.load(path)
    shards, o = [], 0
    for c in z["counts"]:
        shards.append((z["docids"][o:o + c], z["scores"][o:o + c]))
        o += int(c)
    return shards, int(z["docs_to_get"]), z["exp_docids"], z["exp_scores"]


def same(d, s, ed, es):
    return np.array_equal(d, ed) and np.array_equal(np.asarray(s, np.float64).view(np.uint64),
                                                    np.asarray(es, np.float64).view(np.uint64))


def test_fixtures_present():
    assert len(FIX) >= 13


@pytest.mark.parametrize("path", FIX, ids=[os.path.basename(p)[:-4] for p in FIX])
def test_oracle_matches_reference_fixture(path):
    shards, k, ed, es = load_fixture(path)
    d, s = orc.msg3a_merge(shards, k)
    assert same(d, s, ed, es)


@pytest.mark.parametrize("path", FIX, ids=[os.path.basename(p)[:-4] for p in FIX])
def test_host_merge_matches_reference_fixture(path):
    shards, k, ed, es = load_fixture(path)
    d, s = gbgpu.merge_topk(shards, k)
    assert same(d, s, ed, es)


def test_oracle_matches_live_reference():
    import ref_binding as ref
    if not ref.available():
        pytest.skip("oracle/_ref/gbref not built here")
    rng = np.random.default_rng(5)
    for it in range(40):
        ns = int(rng.integers(1, 12))
        shards = msg3a_cases.partitioned(rng, ns, int(rng.integers(0, 80)), int(rng.integers(1, 30)),
                                         int_scores=bool(it % 3 == 0))
        if it % 4 == 1:  # replicas: the same docids on several shards
            shards = shards + shards[: max(1, ns // 2)]
        k = int(rng.integers(1, 200))
        ed, es = ref.msg3a_merge(shards, k)
        d, s = orc.msg3a_merge(shards, k)
        assert same(d, s, ed, es), (it, ns, k)
        d, s = gbgpu.merge_topk(shards, k)
        assert same(d, s, ed, es), (it, ns, k)


# ------------------------------------------------------------ the sequencer
def test_seq_admits_in_order():
    sq = gbgpu.Seq(5)
    order = []
    lock = threading.Lock()
    seqs = list(range(5, 25))
    rng = np.random.default_rng(1)
    rng.shuffle(seqs)

    def worker(x):
        time.sleep(float(rng.random()) * 0.01)
        sq.enter(x)
        with lock:
            order.append(x)
        sq.leave(x)

    th = [threading.Thread(target=worker, args=(x,)) for x in seqs]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=30)
    assert order == list(range(5, 25))
    assert sq.next() == 25


def test_seq_errors_and_timeout():
    sq = gbgpu.Seq(0)
    with pytest.raises(gbgpu.GbgpuError):
        sq.enter(1, timeout_ms=20)  # 0 never came: ETIMEDOUT
    sq.enter(0)
    with pytest.raises(gbgpu.GbgpuError):
        sq.enter(0, timeout_ms=0)  # already admitted
    with pytest.raises(gbgpu.GbgpuError):
        sq.leave(1)  # not the admitted one
    sq.leave(0)
    with pytest.raises(gbgpu.GbgpuError):
        sq.enter(0, timeout_ms=0)  # already past
    sq.enter(1, timeout_ms=0)
    sq.leave(1)
    assert sq.next() == 2
