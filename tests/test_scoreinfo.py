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
# The fixtures with a tree docid whose LAST merged group's mini-merged list
# comes out empty in the second pass (getWordPosList misses), so the
# reference's scorers read the mbuf bytes an earlier docid of the call left
# there.  test_decline_set_is_the_stale_bytes_set derives the
# set from the reference's own QueryTermInfo groups (gbref) and si_predict's
# restated lookups.  The GPU replays those bytes (k_si_stale: the latest
# earlier second-pass docid that wrote them, else the first pass's last) and
# is compared with the reference's buffers on them like on every other.
STALE_BYTES = {"clus2_synonyms", "piped", "sortbyint_info1_synonyms", "sortbyint_info2_three_word",
               "splits2_c0_three_word", "three_word", "wiki_halfstop"}
# the fixtures the GPU declines (GBGPU_EUNSUPPORTED: bytes no docid of the
# call wrote, or a first-pass writer under site clustering): none
EXPECTED_DECLINE = set()
BF_HALF, BF_SYN, BF_NEG, BF_BIGRAM, BF_NUM, BF_FACET = 0x01, 0x04, 0x08, 0x10, 0x20, 0x40


def stale_docids(path):
    """Tree docids whose last merged group is empty in the second pass: the
    reference's groups (ref harness op 4, setQueryTermInfo's QueryTermInfos),
    the sublists getWordPosList finds (si_predict), a numeric group found in
    one sublist not merged (Posdb.cpp:6638-6647), BF_BIGRAM keys with syn
    bits dropped by the mini-merge (6687-6692).  Over docid splits the lists
    are the whole ranges, not the pieces' (a superset of the pieces' misses)."""
    import ref_binding as ref
    terms, lists, params, exp = load_query(path)
    if params.is_boolean:  # no mini-merged list is read in a boolean query's passes
        return set(), params.num_docid_splits
    params.get_docid_scoring_info = 1
    r = ref.query(terms, lists, params, cap=1 << 16, mode=0, white=getattr(params, "_white", None))
    docs = [int(x) for x in exp["docids"][:min(len(exp["docids"]), params.docs_to_get)]]
    miss = set(si_predict.misses(lists, exp["votes"], docs))
    runs = {}
    for li, lst in enumerate(lists):
        img = si_predict.image(lst)
        runs[li] = {d: (img, p, q) for d, p, q in si_predict.runs(img)}
    out = []
    for d in docs:
        empty = None
        for g in r["plan"]:
            if g["flags0"] & BF_NEG:
                continue
            live = [(li, fl) for li, fl in g["subs"] if d in runs[li] and (li, d) not in miss]
            if len(live) == 1 and (live[0][1] & (BF_FACET | BF_NUM)) and not (live[0][1] & (BF_SYN | BF_HALF)):
                continue
            recs = False
            for li, fl in live:
                img, p, q = runs[li][d]
                recs |= any(not ((fl & BF_BIGRAM) and (img[k + 2] & 0x03)) for k in [p] + list(range(p + 12, q, 6)))
            empty = not recs
        if empty:
            out.append(d)
    return out, params.num_docid_splits


def ref_buffers(path):
    z = np.load(path, allow_pickle=False)
    return (np.frombuffer(z["score_info"].tobytes(), gbgpu.DOCID_DT),
            np.frombuffer(z["pair_scores"].tobytes(), gbgpu.PAIR_DT),
            np.frombuffer(z["single_scores"].tobytes(), gbgpu.SINGLE_DT))


IN_BODY = {0, 2, 3, 10}  # HASHGROUP_BODY, _HEADING, _INLIST, _INMENU (Posdb.cpp:1122-1126)
INLINKTEXT = 5


def fixed_unassigning(ps):
    """PairScores at which getTermPairScoreForAny leaves m_fixedDistance
    unassigned (Posdb.cpp:3784-3794, 3982-3992): a distance of 50 or more
    between positions of one modified hash group other than inlink text.
    The flag then carries the value of the call's previous assignment -- or,
    when no pair of the call assigned it yet, the uninitialised local
    (Posdb.cpp:3730)."""
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
            # the GPU carries the flag across the call's pairs as the
            # reference does, and marks 2 the pairs scored before any
            # assignment: only those read an undefined value, and only an
            # unassigning pair may be one
            und = got["fixed_distance"] == 2
            assert not np.any(und & ~fixed_unassigning(exp)), (label, "2 at an assigning pair")
            diff &= ~und
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
    if params.is_boolean:
        # a boolean query's second pass takes m_docId from docIdPtr, restarted
        # at the vote buffer (Posdb.cpp:6119, 6514-6534): its first docids,
        # ascending, no pair or single records (the scorers are jumped over)
        assert len(p) == 0 and len(s) == 0
        assert np.all(d["pairs_offset"] == -1) and np.all(d["singles_offset"] == -1)
        assert np.all(d["site_rank"] == 0) and np.all(d["doc_lang"] == 0)
        votes = np.sort(np.asarray(exp["votes"], np.int64))
        if params.num_docid_splits == 1:
            assert set(d["docid"].tolist()) <= set(votes[:n].tolist())
            assert np.all(np.diff(d["docid"]) > 0)
        return
    if params.num_docid_splits > 1:
        # one second pass per docid-split piece, appended in piece order:
        # each piece's docids lie in its own range, and docids a later piece
        # kicked out of the tree keep their records (Posdb.cpp:6160-6193)
        assert len(d) >= n and len(set(d["docid"].tolist())) == len(d)
        assert set(exp["docids"][:n].tolist()) <= set(d["docid"].tolist())
        # the pieces in order (Msg39.cpp:345-457: piece j covers docids
        # [j, j+1] x MAX_DOCID / splits), and inside a piece the tree order
        # high -> low, which the final tree keeps for the docids still in it
        delta = 0x3fffffffff // params.num_docid_splits
        piece = np.minimum(d["docid"] // delta, params.num_docid_splits - 1)
        assert np.all(np.diff(piece) >= 0), "pieces out of order"
        rank = {int(x): i for i, x in enumerate(exp["docids"])}
        for j in np.unique(piece):
            r = [rank[int(x)] for x in d["docid"][piece == j] if int(x) in rank]
            assert r == sorted(r), ("tree order inside piece", int(j))
        n = 0
    else:
        assert np.array_equal(d["docid"], exp["docids"][:n])
    # the second pass rescores: equal to the first pass's score except where
    # getWordPosList missed the docid in a sublist (si_predict)
    missed = {doc for _, doc in si_predict.misses(lists, exp["votes"], exp["docids"][:n])}
    if any(t.field_code in (59, 60) for t in terms):
        # gbsortby int: m_finalScore is (double)m_intScore, m_score 0.0
        # (Posdb.cpp:7557-7560): against the reference tree's m_intScore
        import ref_binding as ref
        if n and ref.available():
            ints = ref.query(terms, lists, params, cap=1 << 16, votes=False, mode=0)["int_scores"][:n]
            keep = np.array([int(x) not in missed for x in d["docid"][:n]], bool)
            assert np.array_equal(d["final_score"][:n][keep], ints.astype(np.float64)[keep])
        n = 0
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
        assert label[2:-4] in EXPECTED_DECLINE, (label, "declined outside the expected set")
        DECLINED.add(label[2:-4])
        return
    assert label[2:-4] not in EXPECTED_DECLINE, (label, "answered an expected decline")
    check(dict(docids=r.docids, scores=r.scores, hits=r.hits, docs_wanted=r.docs_wanted, filtered=r.filtered),
          exp, label)
    d, p, s = ref_buffers(path)
    same(r.docid_scores, d, label + " DocIdScore")
    same(r.pair_scores, p, label + " PairScore")
    same(r.single_scores, s, label + " SingleScore")


@pytest.mark.gpu
def test_gpu_scoreinfo_declines_exactly(engine):
    """Runs after the parametrized cases: the GPU declined exactly the
    expected fixtures (none: the stale-bytes ones are replayed)."""
    if not SCASES:
        pytest.skip("no fixtures")
    assert DECLINED == EXPECTED_DECLINE, sorted(DECLINED ^ EXPECTED_DECLINE)


def test_decline_set_is_the_stale_bytes_set():
    """STALE_BYTES from the reference: without docid splits exactly the
    fixtures with a stale-bytes docid; a split fixture in the set has one in
    its whole-range view (each piece's second pass sees its own lists)."""
    import ref_binding as ref
    if not ref.available():
        pytest.skip("oracle/_ref/gbref not built (GPU box)")
    plain, split, split_names = set(), set(), set()
    for path in SCASES:
        st, ns = stale_docids(path)
        name = os.path.basename(path)[2:-4]
        if ns > 1:
            split_names.add(name)
        if st:
            (split if ns > 1 else plain).add(name)
    exp_plain = STALE_BYTES - split_names
    assert plain == exp_plain, sorted(plain ^ exp_plain)
    assert STALE_BYTES - exp_plain <= split, sorted((STALE_BYTES - exp_plain) - split)


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
