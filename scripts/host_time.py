"""Diagnostic: host cost of the config-2 query loop.

Runs the bench's round-robin loop (2 slots, 4 distinct queries) and splits
the wall time into the host's enqueue calls and the collect calls (which
wait for the GPU), per query."""
import os
import sys
import time

here = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(here, "..", "open-source-search-engine_amd", "python"))

import gbgpu  # noqa: E402
from workload import config_two_term, generate  # noqa: E402

N = int(os.environ.get("HT_DOCS", 100_000_000))
SLOTS = int(os.environ.get("HT_SLOTS", 2))
NQ = 300
qs = [config_two_term(N, docs_to_get=100, seed=s + 1) for s in range(4)]
with gbgpu.Engine(0) as eng:
    hs = [[eng.upload(l) for l in generate(q, N, threads=16)] for q in qs]
    ps = [q.params() for q in qs]
    eng.set_slots(SLOTS)
    for rep in range(2):
        te = tc = 0.0
        t0 = time.perf_counter()
        for i in range(NQ):
            slot = i % SLOTS
            if i >= SLOTS:
                t = time.perf_counter()
                eng.collect(cap=4096, slot=slot)
                tc += time.perf_counter() - t
            j = i % len(qs)
            t = time.perf_counter()
            eng.enqueue(qs[j].terms, hs[j], ps[j], slot=slot)
            te += time.perf_counter() - t
        for i in range(NQ - SLOTS, NQ):
            t = time.perf_counter()
            eng.collect(cap=4096, slot=i % SLOTS)
            tc += time.perf_counter() - t
        wall = time.perf_counter() - t0
        print(f"rep {rep}: slots {SLOTS} {NQ / wall:.0f} q/s; per query: wall {wall / NQ * 1e6:.1f} us, "
              f"enqueue {te / NQ * 1e6:.1f} us, collect {tc / NQ * 1e6:.1f} us")
