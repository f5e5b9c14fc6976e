"""Diagnostic: host-side timing of the clustered rotation with several slots
in flight (enqueue / collect durations, q/s), no profiler attached."""
import os
import sys
import time

ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "open-source-search-engine_amd", "python"))
os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("HWQ", "8")
import numpy as np  # noqa: E402
import torch  # noqa: E402
import gbgpu  # noqa: E402
from workload import config_two_term, generate  # noqa: E402

torch.cuda.set_device(0)
eng = gbgpu.Engine(0)
N = 100_000_000
qs = [config_two_term(N, docs_to_get=100, seed=s + 1) for s in range(int(os.environ.get("NQ", "8")))]
handles = []
for q in qs:
    handles.append([eng.upload(l) for l in generate(q, N, threads=16)])
for clus in [int(x) for x in os.environ.get("CLUS", "0 1").split()]:
    pc = [q.params(site_clustering=clus) for q in qs]
    for slots in [int(x) for x in os.environ.get("SLOTS", "1 2 4").split()]:
        eng.set_slots(slots)
        nq = int(os.environ.get("NQUERY", "64"))
        te, tc = [], []
        for rep in range(2):
            t0 = time.perf_counter()
            for i in range(nq):
                s = i % slots
                if i >= slots:
                    a = time.perf_counter()
                    eng.collect(cap=4096, slot=s)
                    tc.append(time.perf_counter() - a)
                a = time.perf_counter()
                eng.enqueue(qs[i % len(qs)].terms, handles[i % len(qs)], pc[i % len(qs)], slot=s)
                te.append(time.perf_counter() - a)
                if te[-1] > 2e-3:
                    print(f"  slow enqueue rep {rep} i {i} slot {s} query {i % len(qs)}: {1e3 * te[-1]:.2f} ms", flush=True)
            for i in range(max(0, nq - slots), nq):
                eng.collect(cap=4096, slot=i % slots)
            el = time.perf_counter() - t0
        print(f"clus {clus} slots {slots}: q/s {nq / el:.1f}  enqueue us mean {1e6 * np.mean(te):.1f} max {1e6 * np.max(te):.1f}"
              f"  collect-wait us mean {1e6 * np.mean(tc):.1f}", flush=True)
eng.close()
