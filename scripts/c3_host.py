"""Diagnostic: host cost of the config-3 query loop (12 slots) of the tree
at ROOT (argv[1], default this one): per query, the enqueue call and the
collect call (which waits for the GPU), and the wall time."""
import os
import sys
import time

ROOT = os.path.abspath(sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "open-source-search-engine_amd", "python"))

import gbgpu  # noqa: E402
from workload import config3_queries, generate  # noqa: E402

N = 100_000_000
SLOTS = 12
qs = config3_queries(N, docs_to_get=100)
with gbgpu.Engine(0) as eng:
    hs = [[eng.upload(l) for l in generate(q, N, threads=16)] for q in qs]
    ps = [q.params() for q in qs]
    eng.set_slots(SLOTS)
    for rep in range(3):
        te = [0.0] * len(qs)
        tc = [0.0] * len(qs)
        t0 = time.perf_counter()
        nq = 100
        for i in range(nq):
            slot = i % SLOTS
            if i >= SLOTS:
                t = time.perf_counter()
                eng.collect(cap=4096, slot=slot)
                tc[(i - SLOTS) % len(qs)] += time.perf_counter() - t
            j = i % len(qs)
            t = time.perf_counter()
            eng.enqueue(qs[j].terms, hs[j], ps[j], slot=slot)
            te[j] += time.perf_counter() - t
        for i in range(nq - SLOTS, nq):
            eng.collect(cap=4096, slot=i % SLOTS)
        el = time.perf_counter() - t0
        print(f"rep {rep}: {nq / el:.1f} q/s; enqueue ms/query by query:",
              " ".join(f"{1e3 * x / (nq / len(qs)):.3f}" for x in te),
              "| collect:", " ".join(f"{1e3 * x / (nq / len(qs)):.3f}" for x in tc), flush=True)
