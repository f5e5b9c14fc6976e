"""Diagnostic: a score-info fixture's second-pass stale-byte docids through
the diagnostic build (GBGPU_SI_DEBUG prints each one's writers and every
docid's mbuf bytes), and the reference's records of the first mismatching
DocIdScore beside the GPU's."""
import os
import sys

os.environ["GBGPU_SI_DEBUG"] = "1"
here = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(here, "..", "tests"), os.path.join(here, "..", "open-source-search-engine_amd", "python")]
import numpy as np  # noqa: E402

import gbgpu  # noqa: E402
from test_golden import load_query  # noqa: E402
from test_scoreinfo import ref_buffers  # noqa: E402

name = sys.argv[1]
path = os.path.join(here, "..", "tests", "golden", f"s_{name}.npz")
terms, lists, params, exp = load_query(path)
params.get_docid_scoring_info = 1
with gbgpu.Engine(0, diag=True) as eng:
    r = eng.query(terms, lists, params, cap=1 << 16)
d, p, s = ref_buffers(path)
gd, gp, gs = r.docid_scores, r.pair_scores, r.single_scores
for i in range(len(d)):
    if d["final_score"][i] != gd["final_score"][i]:
        print("mismatch at", i, "docid", d["docid"][i], gd["docid"][i], d["final_score"][i], gd["final_score"][i])
        for nm, a, b, ka, kb in (("pairs", p, gp, "pairs_offset", "num_pairs"), ("singles", s, gs, "singles_offset", "num_singles")):
            sz = a.dtype.itemsize
            ea = a[d[ka][i] // sz: d[ka][i] // sz + d[kb][i]] if d[kb][i] else a[:0]
            eb = b[gd[ka][i] // sz: gd[ka][i] // sz + gd[kb][i]] if gd[kb][i] else b[:0]
            print(nm, "ref", len(ea), "gpu", len(eb))
            for x, y in zip(ea, eb):
                print("  ref", x)
                print("  gpu", y)
        break
