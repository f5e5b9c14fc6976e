"""Site-clustering TopTree replay: k_tree_seq (block filter + register tree)
and its two fall-backs, against the reference's fixtures.

The default engine runs k_tree_seq for whole-range clustered queries
(test_golden covers it).  Here a second engine forces
  GBGPU_REPLAY_MODE=1  the one-wave LDS-tree k_tree_replay for every pass;
  GBGPU_REPLAY_MODE=3  k_tree_seq with one register column (64 nodes), so
                       any query whose tree grows past 64 nodes overflows
                       (tree_err = 2) and collect() replays the same entries
                       through k_tree_replay.
Both must reproduce the reference's TopTree (TopTree.cpp:206-516 driven by
Posdb.cpp:6137-7706) exactly."""
import glob
import os

import numpy as np
import pytest

from test_golden import check, load_query

HERE = os.path.dirname(os.path.abspath(__file__))
CLUS = sorted(p for p in glob.glob(os.path.join(HERE, "golden", "q_*.npz"))
              if load_query(p)[2].site_clustering)
IDS = [os.path.basename(p)[2:-4] for p in CLUS]


def test_clustering_fixtures_present():
    assert len(CLUS) >= 6


@pytest.fixture(scope="module", params=["1", "3"], ids=["lds_replay", "reg_overflow"])
def mode_engine(request):
    import gbgpu
    old = os.environ.get("GBGPU_REPLAY_MODE")
    os.environ["GBGPU_REPLAY_MODE"] = request.param
    try:
        e = gbgpu.Engine(0, diag=True)  # the switch is read by the diagnostic build only
    finally:
        if old is None:
            del os.environ["GBGPU_REPLAY_MODE"]
        else:
            os.environ["GBGPU_REPLAY_MODE"] = old
    yield e
    e.close()


@pytest.mark.gpu
@pytest.mark.parametrize("path", CLUS, ids=IDS)
def test_gpu_replay_modes_vs_reference(mode_engine, path):
    terms, lists, params, exp = load_query(path)
    r = mode_engine.query(terms, lists, params, cap=1 << 16, hit_cap=max(1, exp["hits"]))
    check(dict(docids=r.docids, scores=r.scores, hits=r.hits, docs_wanted=r.docs_wanted, filtered=r.filtered,
               hit_docids=r.hit_docids), exp, os.path.basename(path))


# --------------------------------------------------------------------------
# The block replay's filter, checked on the host (no GPU): k_tree_seq rules
# out, per segment, every entry that cannot be offered under any tree state
# reachable from the segment-start state, and replays only the rest.  Here a
# host model of the replay loop (k_tree_replay's per-docid test and
# TopTree::addNode with the domain caps, TopTree.cpp:206-516, as tree_add
# restates it) runs every entry, and again through the segment filter with
# the same premise and the same raw walk when the m_numNodes delete breaks it;
# both must leave the same tree and the same m_filtered.


def _dom(d):
    return (d & 0x3FC0) >> 6  # Titledb.h:114-115


def _cs(s):
    return int(np.int64(np.float32(s))) & 0xFFFFFFFF  # tree_cs: (uint32)(int64)score


class _Tree:
    def __init__(self, dw, cap, partial, ridiculous, num_nodes):
        self.dw, self.cap, self.partial, self.rid, self.nn = dw, cap, np.float32(partial), ridiculous, num_nodes
        self.nodes = []  # best first: (score, docid)
        self.dom = {}
        self.vc = np.float32(0.0)

    @staticmethod
    def better(a, b):
        return a[0] > b[0] or (a[0] == b[0] and a[1] < b[1])

    def _uncount(self, h):
        c = self.dom.get(h, 0)
        if c < self.cap:
            self.vc = np.float32(np.float64(self.vc) - 1.0)
        elif c == self.cap:
            self.vc = np.float32(self.vc - self.partial)
        self.dom[h] = c - 1

    def add(self, s, d):
        e, h = (s, d), _dom(d)
        if self.vc >= self.dw and self.nodes and not self.better(e, self.nodes[-1]):
            return
        p = sum(1 for x in self.nodes if self.better(x, e))
        if p < len(self.nodes) and self.nodes[p] == e:
            return
        dele = None
        if self.dom.get(h, 0) >= self.rid:
            dn = [x for x in self.nodes if _dom(x[1]) == h]
            m = min(dn, key=lambda x: (_cs(x[0]), x[1]))
            if (_cs(s), d) <= (_cs(m[0]), m[1]):
                return
            dele = m
        self.nodes.insert(p, e)
        self.dom[h] = self.dom.get(h, 0) + 1
        c = self.dom[h]
        if c < self.cap:
            self.vc = np.float32(np.float64(self.vc) + 1.0)
        elif c == self.cap:
            self.vc = np.float32(self.vc + self.partial)
        if dele is not None:
            self._uncount(h)
            self.nodes.remove(dele)
        while self.nodes and (np.float64(self.vc) - 1.0 >= self.dw or len(self.nodes) == self.nn):
            self._uncount(_dom(self.nodes[-1][1]))
            self.nodes.pop()


_STATS = {"resumes": 0, "candidates": 0, "entries": 0}


def _replay(entries, params, seg=None):
    t = _Tree(*params)
    st = {"mws": np.float32(-1.0), "called": False, "filtered": 0}

    def offer(e):  # the per-docid test of the reference loop (Posdb.cpp:6322-6504, 7699-7704)
        s, b, d, serp, scored = e
        live = not (b <= st["mws"])
        full = t.vc >= t.dw
        rej = st["called"] and full and t.nodes and not t.better((s, d), t.nodes[-1])
        if live and scored and not rej:
            t.add(s, d)
            st["called"] = True
            if len(t.nodes) > t.dw:
                st["mws"] = np.float32(t.nodes[-1][0])
            return True
        if live and serp:
            st["filtered"] += 1
        return False

    if seg is None:
        for e in entries:
            offer(e)
        return t.nodes, st["filtered"]
    for s0 in range(0, len(entries), seg):
        part = entries[s0:s0 + seg]
        pref = st["called"] and t.vc >= t.dw and bool(t.nodes)
        L = min(st["mws"], np.float32(t.nodes[-1][0])) if t.nodes else st["mws"]
        bot = t.nodes[-1] if t.nodes else None
        cand = [i for i, e in enumerate(part)
                if (e[4] or e[3]) and (not pref or (not (e[1] <= L) and (e[3] or t.better((e[0], e[2]), bot))))]
        _STATS["candidates"] += len(cand)
        _STATS["entries"] += len(part)
        resume = None
        for i in cand:
            if offer(part[i]) and pref and not (t.vc >= t.dw):
                resume = i + 1  # the premise broke: the rest of the segment raw
                break
        if resume is not None:
            _STATS["resumes"] += 1
            for e in part[resume:]:
                offer(e)
    return t.nodes, st["filtered"]


def _entries(rng, n, ndom, serp_frac):
    docids = np.sort(rng.choice(1 << 20, n, replace=False)).astype(np.int64)
    docids = np.unique((docids & ~0x3FC0) | (rng.integers(0, ndom, n) << 6))
    m = len(docids)
    # some tied scores; prefilter bounds mostly, not always, above the score
    scores = np.round(rng.gamma(2.0, 10.0, m), int(rng.integers(1, 4))).astype(np.float32)
    bounds = (scores * rng.uniform(0.9, 1.5, m)).astype(np.float32)
    serp = rng.random(m) < serp_frac
    scored = rng.random(m) < 0.97
    return [(float(scores[i]), float(bounds[i]), int(docids[i]), bool(serp[i]), bool(scored[i])) for i in range(m)]


# (domains, docsWanted, m_cap, m_ridiculousMax, m_numNodes): diverse domains
# (the tree fills: the filter rules most entries out), few domains (the caps
# keep it from filling), a small ridiculousMax (domain-minimum deletes), and a
# small m_numNodes beside over-cap domains (the premise breaks: raw walks)
CASES = [(256, 20, 2, 50, 10 ** 6), (40, 30, 2, 60, 10 ** 6), (6, 25, 2, 50, 10 ** 6),
         (64, 12, 2, 3, 10 ** 6), (12, 10, 2, 50, 14), (16, 8, 2, 50, 12)]


@pytest.mark.parametrize("case", range(len(CASES)))
@pytest.mark.parametrize("seed", range(3))
def test_block_replay_filter_is_exact(case, seed):
    ndom, dw, cap, rid, nn = CASES[case]
    rng = np.random.default_rng(100 * case + seed)
    entries = _entries(rng, 3000, ndom, 0.05 if seed == 1 else 0.0)
    params = (dw, cap, (dw % 50) / 50.0, rid, nn)
    want = _replay(entries, params)
    for seg in (64, 256, 4096):
        assert _replay(entries, params, seg) == want, (case, seed, seg)


def test_block_replay_filter_paths_taken():
    """The diverse-domain cases rule most entries out; the small-m_numNodes
    cases break the premise (raw walks)."""
    seen = []
    for case in range(len(CASES)):
        for k in _STATS:
            _STATS[k] = 0
        test_block_replay_filter_is_exact(case, 0)
        seen.append(dict(_STATS))
    for case in (0, 1, 3):
        assert seen[case]["candidates"] < seen[case]["entries"] / 2, (case, seen[case])
    assert seen[4]["resumes"] > 0 and seen[5]["resumes"] > 0, seen
