"""The second pass's score info (m_getDocIdScoringInfo; Posdb.cpp:6116-6244,
3247-3298, 4195-4280, 7554-7665) against the REFERENCE's own buffers
(tests/golden/s_*.npz, made by `python3 tests/make_golden.py scoreinfo` from
oracle/_ref/gbref).  The oracle does not restate the second pass: these
fixtures are its only pin.

Bar: every field of every DocIdScore / PairScore / SingleScore bit-exact, in
the reference's order, offsets included.  Not compared: m_termFreq* (the
reference leaves them unset: SafeBuf garbage), the two pointers and padding."""
import glob
import os

import numpy as np
import pytest

import gbgpu
import si_predict
from test_golden import check, load_query

HERE = os.path.dirname(os.path.abspath(__file__))
SCASES = sorted(glob.glob(os.path.join(HERE, "golden", "s_*.npz")))
IDS = [os.path.basename(p)[2:-4] for p in SCASES]
SKIP = {"term_freq1", "term_freq2", "term_freq", "pair_scores", "single_scores"}
DECLINED = set()


def ref_buffers(path):
    z = np.load(path, allow_pickle=False)
    return (np.frombuffer(z["score_info"].tobytes(), gbgpu.DOCID_DT),
            np.frombuffer(z["pair_scores"].tobytes(), gbgpu.PAIR_DT),
            np.frombuffer(z["single_scores"].tobytes(), gbgpu.SINGLE_DT))


IN_BODY = {0, 2, 3, 10}  # HASHGROUP_BODY, _HEADING, _INLIST, _INMENU (Posdb.cpp:1122-1126)
INLINKTEXT = 5


def fixed_undefined(ps):
    """PairScores whose m_fixedDistance the reference never assigns in the
    call (getTermPairScoreForAny, Posdb.cpp:3784-3794, 3982-3992): a
    distance of 50 or more between positions of one modified hash group
    other than inlink text.  It then holds whatever the uninitialised local
    held (known divergences): not compared."""
    mhg1 = np.where(np.isin(ps["hash_group1"], list(IN_BODY)), 0, ps["hash_group1"])
    mhg2 = np.where(np.isin(ps["hash_group2"], list(IN_BODY)), 0, ps["hash_group2"])
    dist = np.abs(ps["word_pos2"].astype(np.int64) - ps["word_pos1"].astype(np.int64))
    return (dist >= 50) & (mhg1 == mhg2) & (mhg1 != INLINKTEXT)


def same(got, exp, label):
    assert len(got) == len(exp), (label, len(got), len(exp))
    for f in exp.dtype.names:
        if f in SKIP:
            continue
        g, e = got[f], exp[f]
        if g.dtype.kind == "f":  # bit patterns (final scores, tf weights)
            g, e = g.view(f"u{g.itemsize}"), e.view(f"u{e.itemsize}")
        diff = g != e
        if f == "fixed_distance" and "hash_group1" in exp.dtype.names:
            diff &= ~fixed_undefined(exp)
        bad = np.nonzero(diff)[0]
        assert not len(bad), (label, f, int(bad[0]), got[f][bad[0]], exp[f][bad[0]])


def test_layout():
    # include/gbgpu.h mirrors the reference's x86-64 layout (Posdb.h:767-866)
    assert (gbgpu.PAIR_DT.itemsize, gbgpu.SINGLE_DT.itemsize, gbgpu.DOCID_DT.itemsize) == (72, 40, 64)
    assert gbgpu.PAIR_DT.fields["qdist"][1] == 68
    assert gbgpu.DOCID_DT.fields["pairs_offset"][1] == 36


def test_fixtures_present():
    assert len(SCASES) >= 12


@pytest.mark.parametrize("path", SCASES, ids=IDS)
def test_reference_buffers_consistent(path):
    """The fixtures themselves: one DocIdScore per top docid, high -> low,
    offsets pointing at each docid's own records."""
    terms, lists, params, exp = load_query(path)
    d, p, s = ref_buffers(path)
    n = min(len(exp["docids"]), params.docs_to_get)
    if params.num_docid_splits > 1:
        # one second pass per docid-split piece, appended in piece order:
        # each piece's docids lie in its own range, and docids a later piece
        # kicked out of the tree keep their records (Posdb.cpp:6160-6193)
        assert len(d) >= n and len(set(d["docid"].tolist())) == len(d)
        assert set(exp["docids"][:n].tolist()) <= set(d["docid"].tolist())
        n = 0
    else:
        assert np.array_equal(d["docid"], exp["docids"][:n])
    # the second pass rescores: equal to the first pass's score except where
    # getWordPosList missed the docid in a sublist (si_predict)
    missed = {doc for _, doc in si_predict.misses(lists, exp["votes"], exp["docids"][:n])}
    if any(t.field_code in (59, 60) for t in terms):
        n = 0  # gbsortby int: m_finalScore is (double)m_intScore, m_score 0.0 (Posdb.cpp:7557-7560)
    keep = np.array([int(x) not in missed for x in d["docid"][:n]], bool)
    assert np.array_equal(d["final_score"][:n].astype(np.float32).view(np.uint32)[keep],
                          exp["scores"][:n].view(np.uint32)[keep])
    assert d["num_pairs"].sum() == len(p) and d["num_singles"].sum() == len(s)
    po = np.concatenate([[0], np.cumsum(d["num_pairs"])[:-1]]) * gbgpu.PAIR_DT.itemsize
    so = np.concatenate([[0], np.cumsum(d["num_singles"])[:-1]]) * gbgpu.SINGLE_DT.itemsize
    assert np.array_equal(np.where(d["num_pairs"] > 0, po, -1), d["pairs_offset"])
    assert np.array_equal(np.where(d["num_singles"] > 0, so, -1), d["singles_offset"])


@pytest.mark.gpu
@pytest.mark.parametrize("path", SCASES, ids=IDS)
def test_gpu_scoreinfo_vs_reference(engine, path):
    """Bit-exact where the GPU path answers; it may decline (EUNSUPPORTED,
    the adapter then runs the CPU body) only where the reference's
    getWordPosList misses a top docid in some sublist -- when the miss
    empties a group's mini-merged list the reference scores stale mbuf
    bytes (known divergences)."""
    terms, lists, params, exp = load_query(path)
    params.get_docid_scoring_info = 1
    label = os.path.basename(path)
    try:
        r = engine.query(terms, lists, params, cap=1 << 16)
    except gbgpu.GbgpuError as e:
        assert e.code == gbgpu.GBGPU_EUNSUPPORTED, label
        assert si_predict.misses(lists, exp["votes"], exp["docids"][:params.docs_to_get]), label
        DECLINED.add(label)
        return
    check(dict(docids=r.docids, scores=r.scores, hits=r.hits, docs_wanted=r.docs_wanted, filtered=r.filtered),
          exp, label)
    d, p, s = ref_buffers(path)
    same(r.docid_scores, d, label + " DocIdScore")
    same(r.pair_scores, p, label + " PairScore")
    same(r.single_scores, s, label + " SingleScore")


@pytest.mark.gpu
def test_gpu_scoreinfo_declines_bounded(engine):
    """Runs after the parametrized cases: most fixtures are answered."""
    if len(DECLINED) == 0 and not SCASES:
        pytest.skip("no fixtures")
    print("declined:", sorted(DECLINED))
    assert len(DECLINED) <= len(SCASES) // 2, sorted(DECLINED)


@pytest.mark.gpu
def test_gpu_scoreinfo_splits_answered(engine):
    """Score info over docid splits (the default HTML request) is answered
    on the GPU for every split fixture, not left to the CPU body."""
    split = [p for p in SCASES if "splits" in os.path.basename(p)]
    assert len(split) >= 5
    answered = 0
    for path in split:
        terms, lists, params, exp = load_query(path)
        params.get_docid_scoring_info = 1
        try:
            r = engine.query(terms, lists, params, cap=1 << 16)
        except gbgpu.GbgpuError as e:
            # only the stale-bytes case (a getWordPosList miss) declines
            assert e.code == gbgpu.GBGPU_EUNSUPPORTED
            assert si_predict.misses(lists, exp["votes"], exp["docids"]), os.path.basename(path)
            continue
        d, p, s = ref_buffers(path)
        same(r.docid_scores, d, os.path.basename(path))
        answered += 1
    assert answered >= len(split) - 2, (answered, len(split))


@pytest.mark.gpu
def test_gpu_scoreinfo_enospc(engine):
    path = os.path.join(HERE, "golden", "s_five_word.npz")  # no getWordPosList misses
    terms, lists, params, exp = load_query(path)
    params.get_docid_scoring_info = 1
    keep, refs = engine.host_lists(lists)
    info = list(engine.info_arrays(params, len(terms)))
    info[1] = info[1][:3]  # too few PairScores
    r, d, s, h = engine._result(64, 0, info)
    import ctypes
    qt = (gbgpu.QTerm * len(terms))(*terms)
    rc = engine.lib.gbgpu_query(engine.ctx, qt, len(terms), refs, ctypes.byref(params), ctypes.byref(r))
    assert rc == 28  # ENOSPC
    d0, p0, _ = ref_buffers(path)
    assert r.n_pair_scores == len(p0) and r.n_docid_scores == len(d0)
