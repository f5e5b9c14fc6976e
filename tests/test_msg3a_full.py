"""Msg3a::mergeLists whole (Msg3a.cpp:971-1503) over full
Msg39Replies: cluster records and the <=2-per-site cap (1342-1379, with the
family filter and hideAllClustered), facet lists merged into the query
terms' tables (1089-1240), the summed hits and facet doc counts that
gotAllShardReplies adds (792-802).

Pinned to the reference's own mergeLists (oracle/_ref/gbref op 8 made
tests/golden/x3_*.npz from the reply sets of msg3a_cases.full_cases).  The
facet merge picks each merged entry's m_docId with rand() (1232-1233): a
fixture's m_docId must be one of the merged entries' docids, and ours is the
first one's; every other field is compared exactly.

CPU: the oracle restatement and the host merge (gbgpu_merge_replies) against
the fixtures.  GPU: the device merge (gbgpu_merge_replies_device) against the
fixtures, and the RCCL exchange (gbgpu_allgather_replies) as a one-rank
communicator against the oracle."""
import errno
import glob
import os

import numpy as np
import pytest

import gbgpu
import msg3a_cases
import oracle_binding as orc

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FIX = sorted(glob.glob(os.path.join(GOLD, "x3_*.npz")))


def _entries(exp):
    """the fixture's tables as FACET_ENTRY rows, by term then key"""
    rows = []
    for t, tab in enumerate(exp["tables"]):
        for e in tab:
            rows.append((t, int(e["key"]), int(e["count"]), int(e["outside"]), int(e["docid"]), int(e["sum"]),
                         int(e["max"]), int(e["min"])))
    return rows


def check(req, shards, exp, got, label=""):
    assert np.array_equal(got["docids"], exp["docids"]), label
    assert np.array_equal(got["scores"].view(np.uint64), exp["scores"].view(np.uint64)), label
    if req["clus"]:
        assert got["recs"] == exp["recs"], label
    assert got["hits"] == exp["hits"], label
    assert np.array_equal(got["fdocs"], exp["fdocs"]), label
    want = _entries(exp)
    have = [tuple(int(x[f]) for f in ("term", "key", "count", "outside", "docid", "sum", "max", "min"))
            for x in got["facets"]]
    assert len(have) == len(want), (label, len(have), len(want))
    contrib = msg3a_cases.facet_contributions(req, shards)
    for w, h in zip(want, have):
        assert w[:4] + w[5:] == h[:4] + h[5:], (label, w, h)
        c = contrib[(w[0], w[1])]
        assert w[4] in c, (label, w)   # the reference's random pick is one of them
        assert h[4] == c[0], (label, h)  # ours: the first merged entry's


def test_fixtures_present():
    assert len(FIX) >= 12


@pytest.mark.parametrize("path", FIX, ids=[os.path.basename(p)[:-4] for p in FIX])
def test_oracle_matches_reference_fixture(path):
    _, req, shards, exp = msg3a_cases.load_full(path)
    check(req, shards, exp, orc.msg3a_full(req, shards), "oracle")


@pytest.mark.parametrize("path", FIX, ids=[os.path.basename(p)[:-4] for p in FIX])
def test_host_merge_matches_reference_fixture(path):
    _, req, shards, exp = msg3a_cases.load_full(path)
    check(req, shards, exp, gbgpu.merge_replies(req, shards), "host")


def test_fixture_cases_exercise_every_rule():
    """the fixtures hold what the rules act on: capped sites, adult records
    under the family filter, zero and half-zero records, a hideAll request,
    merged facet entries with counts of 0, an unknown termid"""
    seen = dict(capped=0, family=0, zero_rec=0, low=0, hide=0, merged_facet=0, unknown=0)
    for path in FIX:
        name, req, shards, exp = msg3a_cases.load_full(path)
        nomerge = orc.msg3a_full(dict(req, clus=0), shards)
        if req["clus"] and len(exp["docids"]) < len(nomerge["docids"]):
            seen["capped"] += 1
        seen["family"] += bool(req["family"])
        seen["hide"] += bool(req["hide"])
        for s in shards:
            r = s["recs"] or b""
            for i in range(0, len(r), 12):
                n0 = int.from_bytes(r[i:i + 8], "little")
                n1 = int.from_bytes(r[i + 8:i + 12], "little")
                seen["zero_rec"] += n0 == 0
                seen["low"] += n0 != 0 and n1 == 0
        seen["merged_facet"] += sum(len(v) > 1 for v in msg3a_cases.facet_contributions(req, shards).values())
        seen["unknown"] += "termid" in name
    assert all(v > 0 for v in seen.values()), seen


def test_host_merge_refusals():
    name, req, shards, exp = msg3a_cases.load_full(FIX[0])
    bad = dict(shards[0], recs=None)
    with pytest.raises(gbgpu.GbgpuError):  # clustering needs every head's record
        gbgpu.merge_replies(req, [bad] + shards[1:])
    with pytest.raises(gbgpu.GbgpuError):  # a truncated facet list
        gbgpu.merge_replies(req, [dict(shards[0], facets=shards[0]["facets"][:-5])])
    with pytest.raises(gbgpu.GbgpuError):
        gbgpu.merge_replies(dict(req, docs_to_get=0), shards)
    # ENOSPC past facets_cap, with n_facets set
    x = gbgpu.FullReplies(req, shards, facets_cap=1)
    rc = gbgpu.load().gbgpu_merge_replies(gbgpu.ctypes.byref(x.req), x.reps, x.n, gbgpu.ctypes.byref(x.out))
    assert rc == errno.ENOSPC
    assert x.out.n_facets == sum(len(t) for t in exp["tables"])


def test_seeded_host_vs_oracle():
    rng = np.random.default_rng(99)
    for it in range(30):
        ns = int(rng.integers(1, 9))
        fcs = [0] + [int(x) for x in rng.choice([63, 64, 65], size=int(rng.integers(0, 4)))]
        req = dict(docs_to_get=int(rng.choice([1, 5, 10, 50, 300])), clus=int(rng.integers(0, 2)),
                   hide=int(rng.integers(0, 2)), family=int(rng.integers(0, 2)),
                   tids=[1000003 * (i + 1) for i in range(len(fcs))], fcs=fcs)
        fterms = [(t, f) for t, f in zip(req["tids"], fcs) if f]
        shards = []
        for j in range(ns):
            lo = int(rng.integers(1, 1 << 37))
            x = msg3a_cases.full_reply(rng, lo, lo + 5000, int(rng.integers(0, 80)), int(rng.integers(1, 8)),
                                       fterms, np.arange(-30, 30, 2))
            x["fcounts"] = rng.integers(0, 1000, len(fcs)).astype(np.int64)
            shards.append(x)
        if it % 5 == 4:
            shards = shards + shards[:1]  # a twin
        a = orc.msg3a_full(req, shards)
        b = gbgpu.merge_replies(req, shards)
        for k in ("docids", "fdocs"):
            assert np.array_equal(a[k], b[k]), (it, k)
        assert np.array_equal(a["scores"].view(np.uint64), b["scores"].view(np.uint64)), it
        assert a["recs"] == b["recs"] and a["hits"] == b["hits"], it
        assert np.array_equal(a["facets"], b["facets"]), it


# ------------------------------------------------------------------ the GPU
@pytest.mark.gpu
@pytest.mark.parametrize("path", FIX, ids=[os.path.basename(p)[:-4] for p in FIX])
def test_device_merge_matches_reference_fixture(engine, path):
    _, req, shards, exp = msg3a_cases.load_full(path)
    check(req, shards, exp, engine.merge_replies_device(req, shards), "device")


@pytest.mark.gpu
def test_device_merge_seeded_vs_oracle(engine):
    rng = np.random.default_rng(7)
    for it in range(40):
        ns = int(rng.integers(1, 17))
        fcs = [0] + [int(x) for x in rng.choice([63, 64, 65], size=int(rng.integers(0, 4)))]
        req = dict(docs_to_get=int(rng.choice([1, 10, 100, 1000, 4096])), clus=int(rng.integers(0, 2)),
                   hide=int(rng.integers(0, 2)), family=int(rng.integers(0, 2)),
                   tids=[1000003 * (i + 1) for i in range(len(fcs))], fcs=fcs)
        fterms = [(t, f) for t, f in zip(req["tids"], fcs) if f]
        shards = []
        for j in range(ns):
            lo = int(rng.integers(1, 1 << 37))
            x = msg3a_cases.full_reply(rng, lo, lo + 40000, int(rng.integers(0, 400)), int(rng.integers(1, 30)),
                                       fterms, np.arange(-3000, 3000, 7))
            x["fcounts"] = rng.integers(0, 1000, len(fcs)).astype(np.int64)
            shards.append(x)
        a = orc.msg3a_full(req, shards)
        b = engine.merge_replies_device(req, shards)
        assert np.array_equal(a["docids"], b["docids"]), it
        assert np.array_equal(a["scores"].view(np.uint64), b["scores"].view(np.uint64)), it
        assert a["recs"] == b["recs"] and a["hits"] == b["hits"], it
        assert np.array_equal(a["fdocs"], b["fdocs"]), it
        assert np.array_equal(a["facets"], b["facets"]), it


@pytest.mark.gpu
def test_device_merge_refusals(engine):
    _, req, shards, _ = msg3a_cases.load_full(FIX[0])
    with pytest.raises(gbgpu.GbgpuError):
        engine.merge_replies_device(dict(req, docs_to_get=5000), shards)  # past XFMAX
    with pytest.raises(gbgpu.GbgpuError):
        engine.merge_replies_device(req, [dict(shards[0], facets=shards[0]["facets"][:-5])])


@pytest.mark.gpu
def test_allgather_replies_one_rank():
    """the RCCL exchange of full replies as a one-rank communicator: every
    fixture shard's reply alone, against the oracle's merge of it"""
    with gbgpu.Engine(0) as eng:
        eng.comm_init(1, 0, gbgpu.Engine.comm_unique_id())
        for path in FIX:
            name, req, shards, _ = msg3a_cases.load_full(path)
            for s in shards:
                a = orc.msg3a_full(req, [s])
                b = eng.allgather_replies(req, s)
                assert np.array_equal(a["docids"], b["docids"]), name
                assert np.array_equal(a["scores"].view(np.uint64), b["scores"].view(np.uint64)), name
                assert a["recs"] == b["recs"] and a["hits"] == b["hits"], name
                assert np.array_equal(a["fdocs"], b["fdocs"]), name
                assert np.array_equal(a["facets"], b["facets"]), name
        # an empty reply (a failed shard) still takes part
        _, req, _, _ = msg3a_cases.load_full(FIX[0])
        e = eng.allgather_replies(req, None)
        assert len(e["docids"]) == 0 and e["hits"] == 0 and len(e["facets"]) == 0
