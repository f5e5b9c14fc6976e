"""INTEGRATION.md's adapter, executed inside the reference's own Msg39 sequence.

oracle/_ref/gbref_gpu is the reference harness (oracle/ref_harness.cpp, the
unmodified PosdbTable / TopTree compiled from /root/reference by
oracle/ref.mk) with INTEGRATION.md's cpp blocks and libgbgpu.so linked in.
Its op 4 runs one query twice through init -> allocTopTree ->
allocWhiteListTable -> setQueryTermInfo (Msg39.cpp:884-1053), once with the
CPU body of intersectLists10_r and once with the adapter body
(gbgpuIntersectLists: gbgpu_query, then the GPU's tree re-inserted into the
reference's TopTree by gbgpuFillTree), and reads back what Msg39 reads:
the TopTree high -> low (m_score, m_intScore, m_docId), m_numUsedNodes
(Msg39::setClusterRecs requires it equal to the node count,
Msg39.cpp:1250), m_docIdVoteBuf.length()/6, m_filtered and the score-info
SafeBufs.  Both must agree, and agree with the fixture the plain reference
harness made (tests/golden/).

On a GPU box the adapter must answer every fixture whose mode the GPU path
supports; without a GPU (this container) it declines (ENODEVICE) and the CPU
body runs, which the non-GPU test checks."""
import glob
import os

import numpy as np
import pytest

import gbgpu
import ref_binding as ref
from test_golden import check, load_query

HERE = os.path.dirname(os.path.abspath(__file__))
QCASES = sorted(glob.glob(os.path.join(HERE, "golden", "q_*.npz")) + glob.glob(os.path.join(HERE, "golden", "f_*.npz")))
SCASES = sorted(glob.glob(os.path.join(HERE, "golden", "s_*.npz")))
IDS = [os.path.basename(p)[:-4] for p in QCASES]
SIDS = [os.path.basename(p)[:-4] for p in SCASES]

needs_gpu_build = pytest.mark.skipif(not ref.available(ref.EXE_GPU), reason="oracle/_ref/gbref_gpu not built")


def run(path, mode, info=False):
    """mode 0: the CPU body; 1: the body adapter; 2: the body adapter and,
    with docid splits, Msg39's split loop replaced by gbgpuDocIdSplits."""
    terms, lists, params, exp = load_query(path)
    if info:
        params.get_docid_scoring_info = 1
    white = getattr(params, "_white", None)
    r = ref.query(terms, lists, params, cap=1 << 16, votes=False, white=white, mode=mode, exe=ref.EXE_GPU)
    # TopNode::m_intScore is set only with a gbsortby int term (Posdb.cpp:
    # 7271-7279, m_useIntScores); elsewhere it is whatever the node held
    r["ints_defined"] = any(t.field_code in (59, 60) for t in terms)
    return r, exp, params


def same_tree(cpu, gpu, label, msg39=False):
    assert gpu["used_nodes"] == cpu["used_nodes"] == len(cpu["docids"]), label
    assert np.array_equal(gpu["docids"], cpu["docids"]), label
    assert np.array_equal(gpu["scores"].view(np.uint32), cpu["scores"].view(np.uint32)), label
    if cpu["ints_defined"]:
        assert np.array_equal(gpu["int_scores"], cpu["int_scores"]), label
    if msg39:
        # gbgpuDocIdSplits leaves Msg39::m_numTotalHits (the pieces' vote
        # counts less m_filtered, Msg39.cpp:409-414), reported as hits
        assert gpu["hits"] == cpu["hits"] - cpu["filtered"], label
        fields = ("docs_wanted", "corrupt")
    else:
        fields = ("hits", "filtered", "docs_wanted", "corrupt")
    for f in fields:
        assert gpu[f] == cpu[f], (label, f, gpu[f], cpu[f])
    # the facet terms' QueryTerm::m_facetHashTable and m_numDocsThatHaveFacet
    assert gpu["facets"] == cpu["facets"], label


def splits(params):
    return params.num_docid_splits > 1


@needs_gpu_build
def test_adapter_build_falls_back_without_gpu():
    """No GPU (this container): the adapter declines and the reference's own
    body runs -- the binary is the reference plus a dormant adapter."""
    if os.path.exists("/dev/kfd"):
        pytest.skip("a GPU is present: test_gpu_adapter_* cover it")
    for path in QCASES[:6]:
        cpu, exp, _ = run(path, 0)
        gpu, _, _ = run(path, 1)
        assert gpu["answered"] == 0
        same_tree(cpu, gpu, path)
        check(cpu, exp, path)


@pytest.mark.gpu
@needs_gpu_build
@pytest.mark.parametrize("path", QCASES, ids=IDS)
def test_gpu_adapter_in_reference_msg39(path):
    """Every q_/f_ fixture through the reference's Msg39 sequence with the
    adapters in: the body adapter for one-piece queries, gbgpuDocIdSplits
     for the docid-split loop."""
    cpu, exp, params = run(path, 0)
    gpu, _, _ = run(path, 2)
    label = os.path.basename(path)
    check(cpu, exp, label)  # the CPU body of this binary is the fixture's reference
    if cpu["docs_wanted"] == 0:
        assert gpu["answered"] == 0, label  # every list empty: Msg39 runs no pass (Msg39.cpp:945-948)
    else:
        assert gpu["answered"] == 1, (label, "the adapter declined a supported query")
    same_tree(cpu, gpu, label, msg39=splits(params) and gpu["answered"] == 1)


@pytest.mark.gpu
@needs_gpu_build
@pytest.mark.parametrize("path", SCASES, ids=SIDS)
def test_gpu_adapter_score_info_in_reference_msg39(path):
    """The second pass's SafeBufs the adapter fills (m_scoreInfoBuf,
    m_pairScoreBuf, m_singleScoreBuf) against the CPU body's, field by field
    (test_scoreinfo.same: m_termFreq* and padding excepted); over docid
    splits through gbgpuDocIdSplits.  The adapter declines exactly the
    fixtures the library declines (test_scoreinfo.EXPECTED_DECLINE: none; the
    stale-bytes fixtures are replayed), and answers every other."""
    from test_scoreinfo import EXPECTED_DECLINE, same
    cpu, exp, params = run(path, 0, info=True)
    gpu, _, _ = run(path, 2, info=True)
    label = os.path.basename(path)
    name = label[2:-4]
    same_tree(cpu, gpu, label, msg39=splits(params) and gpu["answered"] == 1)
    if name in EXPECTED_DECLINE:
        assert gpu["answered"] == 0, (label, "expected a decline")
        return
    assert gpu["answered"] == 1, (label, "the adapter declined")
    for key, dt in (("score_info", gbgpu.DOCID_DT), ("pair_scores", gbgpu.PAIR_DT), ("single_scores", gbgpu.SINGLE_DT)):
        same(np.frombuffer(gpu[key], dt), np.frombuffer(cpu[key], dt), f"{label} {key}")


# ------------------------------------------------ the shard
# one shard's whole-range pass: a docid-split fixture's hit count is the
# pieces' sum with their overlap (Msg39.cpp:409-414), the shard's the exact one
SHARD_CASES = [p for p in QCASES if not os.path.basename(p).startswith(("q_clus", "f_sortbyint_clus", "q_stale_clus"))
               and "splits" not in os.path.basename(p)]


@pytest.mark.gpu
@needs_gpu_build
@pytest.mark.parametrize("path", SHARD_CASES, ids=[os.path.basename(p)[:-4] for p in SHARD_CASES])
def test_gpu_adapter_shard_query(path):
    """gbgpuShardQuery as shard 0 of a one-rank exchange inside gbref_gpu
    (gbgpuJoin, then the resident query on a slot and gbgpu_allgather_topk)
    against the reference's own Msg3a::mergeLists over the CPU body's
    TopTree.  Site clustering is left out: Msg3a's site cap needs clusterdb
    records (VERDICT r04 Missing 6)."""
    terms, lists, params, exp = load_query(path)
    r = ref.shard_query(terms, lists, params, white=getattr(params, "_white", None))
    label = os.path.basename(path)
    assert r["shard_rc"] == 0, (label, r["shard_rc"])
    assert np.array_equal(r["shard_docids"], r["msg3a_docids"]), label
    assert np.array_equal(r["shard_scores"], r["msg3a_scores"]), label
    assert r["shard_hits"] == r["hits"], label


# ------------------------------ Msg3a over full replies
# every query fixture -- site-clustered and facet ones included -- as one
# shard: the reply Msg39 builds (CR_OK nodes, cluster records over gbref's
# synthetic clusterdb, facet lists and counts), merged by Msg3a; the GPU
# side is the adapter body plus gbgpuMsg3aReplies (the one-rank exchange)
REPLY_CASES = [p for p in QCASES if "splits" not in os.path.basename(p)]


@pytest.mark.gpu
@needs_gpu_build
@pytest.mark.parametrize("path", REPLY_CASES, ids=[os.path.basename(p)[:-4] for p in REPLY_CASES])
def test_gpu_adapter_msg3a_replies(path):
    terms, lists, params, exp = load_query(path)
    label = os.path.basename(path)
    white = getattr(params, "_white", None)
    for family, hide, nsites in ((0, 0, 3), (1, 1, 5)):
        cpu = ref.shard_msg3a(terms, lists, params, 0, family, hide, nsites, white=white)["merged"]
        gpu = ref.shard_msg3a(terms, lists, params, 1, family, hide, nsites, white=white)["merged"]
        tag = (label, family, hide, nsites)
        assert cpu["rc"] == 0, tag
        assert gpu["rc"] == 0, (tag, gpu["rc"])
        assert np.array_equal(gpu["docids"], cpu["docids"]), tag
        assert np.array_equal(gpu["scores"].view(np.uint64), cpu["scores"].view(np.uint64)), tag
        assert gpu["recs"] == cpu["recs"], tag
        assert gpu["hits"] == cpu["hits"], tag
        assert np.array_equal(gpu["fdocs"], cpu["fdocs"]), tag
        assert len(gpu["tables"]) == len(cpu["tables"]), tag
        for a, b in zip(gpu["tables"], cpu["tables"]):
            # m_docId of a merged entry is the reference's rand() pick; one
            # reply: the entry itself
            assert np.array_equal(a, b), tag


# -------------------------------------------- the merge
def _merge_cases():
    from test_golden import MCASES, split_blob
    out = []
    for path in MCASES:
        z = np.load(path, allow_pickle=False)
        runs = split_blob(z["run_sizes"], z["run_blob"])
        out.append((os.path.basename(path)[:-4], runs))
    return out


def _keys(runs):
    """a few start/end keys inside the runs' key range (full 18-byte keys
    with the compression bits cleared), the open range included"""
    ks = [r[:18] for r in runs if len(r) >= 18]
    ks.sort(key=lambda k: (k[12:18][::-1], k[6:12][::-1], k[0:6][::-1]))
    mid = ks[len(ks) // 2] if ks else bytes(18)
    neg = bytes([mid[0] & 0xFE]) + mid[1:]  # a delete key: merge_r's dangling-negative fix
    return [(bytes(18), b"\xff" * 18), (bytes(18), mid), (bytes(18), neg)]


def merge_check(runs, label, mode_exe):
    total = sum(map(len, runs))
    for rm in (0, 1):
        for mrs in (-1, 1, 100, total // 3, total - 7, total + 100):
            for sk, ek in _keys(runs):
                cpu = ref.posdb_merge_r(runs, rm, mrs, sk, ek, mode=0, exe=mode_exe)
                gpu = ref.posdb_merge_r(runs, rm, mrs, sk, ek, mode=1, exe=mode_exe)
                tag = (label, rm, mrs, ek.hex())
                assert gpu["list"] == cpu["list"], tag
                assert gpu["last_valid"] == cpu["last_valid"], tag
                if cpu["last_valid"]:
                    assert gpu["last_key"] == cpu["last_key"], tag
                assert gpu["end_key"] == cpu["end_key"], tag
                yield gpu


@needs_gpu_build
def test_adapter_merge_declines_without_gpu():
    if os.path.exists("/dev/kfd"):
        pytest.skip("a GPU is present: test_gpu_adapter_merge covers it")
    name, runs = _merge_cases()[0]
    for g in merge_check(runs, name, ref.EXE_GPU):
        assert g["answered"] == 0


@pytest.mark.gpu
@needs_gpu_build
@pytest.mark.parametrize("case", range(6))
def test_gpu_adapter_merge_in_reference_merge_r(case):
    """RdbList::merge_r with gbgpuMergePosdb where it calls posdbMerge_r,
    against the unchanged merge_r on the reference's own merge fixtures and on
    seeded tiered runs: the list bytes, m_lastKey (and its valid flag) and
    m_endKey after the shrink of RdbList.cpp:3537-3565, for removeNegKeys
    on/off, cuts on both sides of the total and end keys inside the range."""
    from mergegen import tiered_runs
    cases = _merge_cases()
    if case < len(cases):
        name, runs = cases[case]
    else:
        name, runs = "tiered", tiered_runs(3000, nruns=5, seed=case, dup_frac=0.1, neg_frac=0.05, nterms=4)
    n = 0
    for g in merge_check(runs, name, ref.EXE_GPU):
        assert g["answered"] == 1
        n += 1
    assert n > 0
