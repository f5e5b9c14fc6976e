"""diagnostic: GPU vs reference score-info docids for one split fixture"""
import os
import sys
import numpy as np
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..", "tests"), os.path.join(HERE, "..", "open-source-search-engine_amd", "python")]
import gbgpu
from test_scoreinfo import ref_buffers, load_query
path = os.path.join(HERE, "..", "tests", "golden", sys.argv[1])
terms, lists, params, exp = load_query(path)
params.get_docid_scoring_info = 1
with gbgpu.Engine(0) as eng:
    r = eng.query(terms, lists, params, cap=1 << 16)
d, p, s = ref_buffers(path)
delta = ((1 << 38) - 1) // params.num_docid_splits
print("tree exp", exp["docids"][:params.docs_to_get].tolist())
print("tree got", r.docids[:params.docs_to_get].tolist())
g = r.docid_scores["docid"].tolist()
e = d["docid"].tolist()
print("ref ", [(x, x // delta) for x in e])
print("gpu ", [(x, x // delta) for x in g])
print("missing", set(e) - set(g), "extra", set(g) - set(e))
gp = r.pair_scores
print("pairs", len(gp), len(p))
owner = {}
for x in d:
    if x["num_pairs"] > 0:
        for k in range(x["num_pairs"]):
            owner[x["pairs_offset"] // gbgpu.PAIR_DT.itemsize + k] = int(x["docid"])
for i in range(max(0, 56), min(len(p), 66)):
    print(i, owner.get(i), "ref", p[i]["final_score"], p[i]["word_pos1"], p[i]["word_pos2"], p[i]["qterm_num1"], p[i]["qterm_num2"],
          "gpu", gp[i]["final_score"], gp[i]["word_pos1"], gp[i]["word_pos2"], gp[i]["qterm_num1"], gp[i]["qterm_num2"])
