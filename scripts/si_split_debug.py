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
