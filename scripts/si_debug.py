"""Diagnostic: which DocIdScores differ between the GPU path and a score-info fixture."""
import sys
import os
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "tests"),
                os.path.join(os.path.dirname(__file__), "..", "open-source-search-engine_amd", "python")]
import torch  # noqa: F401  (HIP runtime first)
torch.cuda.init()
import numpy as np
import gbgpu
import si_predict
from test_golden import load_query
from test_scoreinfo import ref_buffers

path = sys.argv[1]
terms, lists, params, exp = load_query(path)
params.get_docid_scoring_info = 1
eng = gbgpu.Engine(0)
r = eng.query(terms, lists, params, cap=1 << 16)
d, p, s = ref_buffers(path)
gd = set(int(x) for x in r.docid_scores["docid"])
rd = [int(x) for x in d["docid"]]
print("missing on GPU:", [x for x in rd if x not in gd])
print("predicted misses:", si_predict.misses(lists, exp["votes"], exp["docids"][:params.docs_to_get]))
for k, x in enumerate(rd):
    if x not in gd:
        print("ref entry", d[k])
        po, ps = d[k]["pairs_offset"] // 72, d[k]["singles_offset"] // 40
        print("ref pairs", p[po:po + d[k]["num_pairs"]])
        print("ref singles", s[ps:ps + d[k]["num_singles"]])
print("gpu n", len(r.docid_scores), "pairs", len(r.pair_scores), "singles", len(r.single_scores),
      "ref pairs", len(p), "singles", len(s))
