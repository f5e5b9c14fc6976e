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
        e = gbgpu.Engine(0)
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
