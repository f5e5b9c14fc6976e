"""Diagnostic: every survivor's score, GPU vs oracle, on one query (prints the
re-shrink table with GBGPU_DEBUG_EXT=1)."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "open-source-search-engine_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import gbgpu  # noqa: E402
import oracle_binding as orc  # noqa: E402
import qkinds  # noqa: E402
from workload import generate  # noqa: E402

q = qkinds.kinds(20000, seed=1)[8]
lists = generate(q, 20000, seed=1001)
q.docs_to_get = 1500
p = q.params()
exp = orc.query(q.terms, lists, p, cap=4096)
with gbgpu.Engine(0) as eng:
    r = eng.query(q.terms, lists, p, cap=4096, hit_cap=1 << 20)
print("hits", r.hits, exp["hits"], "n", len(r.docids), len(exp["docids"]))
g = dict(zip(r.docids.tolist(), r.scores.tolist()))
e = dict(zip(exp["docids"].tolist(), exp["scores"].tolist()))
bad = [(d, g.get(d), e.get(d)) for d in set(g) | set(e) if g.get(d) != e.get(d)]
print("mismatches", len(bad), sorted(bad)[:20])
