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
    terms, lists, params, exp = load_query(path)
    if info:
        params.get_docid_scoring_info = 1
    white = getattr(params, "_white", None)
    r = ref.query(terms, lists, params, cap=1 << 16, votes=False, white=white, mode=mode, exe=ref.EXE_GPU)
    # TopNode::m_intScore is set only with a gbsortby int term (Posdb.cpp:
    # 7271-7279, m_useIntScores); elsewhere it is whatever the node held
    r["ints_defined"] = any(t.field_code in (59, 60) for t in terms)
    return r, exp, params


def same_tree(cpu, gpu, label):
    assert gpu["used_nodes"] == cpu["used_nodes"] == len(cpu["docids"]), label
    assert np.array_equal(gpu["docids"], cpu["docids"]), label
    assert np.array_equal(gpu["scores"].view(np.uint32), cpu["scores"].view(np.uint32)), label
    if cpu["ints_defined"]:
        assert np.array_equal(gpu["int_scores"], cpu["int_scores"]), label
    for f in ("hits", "filtered", "docs_wanted", "corrupt"):
        assert gpu[f] == cpu[f], (label, f, gpu[f], cpu[f])


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
    cpu, exp, params = run(path, 0)
    gpu, _, _ = run(path, 1)
    label = os.path.basename(path)
    check(cpu, exp, label)  # the CPU body of this binary is the fixture's reference
    if splits(params):
        # the body sees one docid piece per call and declines splits (they
        # are replaced at the Msg39 level): CPU body
        assert gpu["answered"] == 0, label
    elif cpu["docs_wanted"] == 0:
        assert gpu["answered"] == 0, label  # every list empty: Msg39 runs no pass (Msg39.cpp:945-948)
    else:
        assert gpu["answered"] == 1, (label, "the adapter declined a supported query")
    same_tree(cpu, gpu, label)


@pytest.mark.gpu
@needs_gpu_build
@pytest.mark.parametrize("path", SCASES, ids=SIDS)
def test_gpu_adapter_score_info_in_reference_msg39(path):
    """The second pass's SafeBufs the adapter fills (m_scoreInfoBuf,
    m_pairScoreBuf, m_singleScoreBuf) against the CPU body's, field by field
    (test_scoreinfo.same: m_termFreq* and padding excepted)."""
    from test_scoreinfo import same
    cpu, exp, params = run(path, 0, info=True)
    gpu, _, _ = run(path, 1, info=True)
    label = os.path.basename(path)
    same_tree(cpu, gpu, label)
    if not gpu["answered"]:
        return  # declined (splits, or a second-pass path not replayed): the CPU body ran
    for key, dt in (("score_info", gbgpu.DOCID_DT), ("pair_scores", gbgpu.PAIR_DT), ("single_scores", gbgpu.SINGLE_DT)):
        same(np.frombuffer(gpu[key], dt), np.frombuffer(cpu[key], dt), f"{label} {key}")
