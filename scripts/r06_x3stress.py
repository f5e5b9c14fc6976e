"""diagnostic: the one-rank exchange of full replies called repeatedly on the
x3 fixture shards with the request flags varied, against the oracle"""
import glob
import os
import sys
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
sys.path.insert(0, os.path.join(HERE, "..", "open-source-search-engine_amd", "python"))
import numpy as np  # noqa: E402
import gbgpu  # noqa: E402
import msg3a_cases  # noqa: E402
import oracle_binding as orc  # noqa: E402
bad = tot = 0
with gbgpu.Engine(0) as eng:
    eng.comm_init(1, 0, gbgpu.Engine.comm_unique_id())
    for path in sorted(glob.glob(os.path.join(HERE, "..", "tests", "golden", "x3_*.npz"))):
        name, req, shards, _ = msg3a_cases.load_full(path)
        for it in range(6):
            for s in shards:
                r2 = dict(req, family=it & 1, hide=(it >> 1) & 1)
                a = orc.msg3a_full(r2, [s])
                b = eng.allgather_replies(r2, s)
                tot += 1
                if not np.array_equal(a["docids"], b["docids"]):
                    bad += 1
                    print("MISMATCH", name, it, len(a["docids"]), len(b["docids"]), b["docids"][:3], flush=True)
print("total", tot, "bad", bad)
