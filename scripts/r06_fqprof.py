"""Round 6: where the file_read leg's time goes with queries in flight --
host clocks around gbgpu_file_list, enqueue, collect and free in the
bench's loop (config 2's first query, 4 slots)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "open-source-search-engine_amd", "python")]
os.environ["GPU_MAX_HW_QUEUES"] = "16"
import numpy as np  # noqa: E402
import bench  # noqa: E402
import gbgpu  # noqa: E402
from workload import config_two_term, generate  # noqa: E402

eng = gbgpu.Engine(0)
total = bench.CFG2_DOCS
q = config_two_term(total, docs_to_get=100, seed=1)
lists = generate(q, total, doc_begin=0, doc_end=total, threads=16)
p = q.params()
eng.set_slots(4)
fh = eng.file_upload(b"".join(lists))
offs = np.cumsum([0] + [len(x) for x in lists[:-1]]).tolist()
print("lists", [len(x) for x in lists], flush=True)
hs = [eng.upload(x) for x in lists]
ref = eng.query_resident(q.terms, hs, p)
print("ref", ref.hits, ref.docids[:3], flush=True)
bad = 0


def check(r, where):
    global bad
    if r.hits != ref.hits or not np.array_equal(r.docids, ref.docids):
        bad += 1
        if bad < 5:
            print("MISMATCH", where, r.hits, r.docids[:3], flush=True)
for fs in (1, 4):
    tm = dict(cut=0.0, enq=0.0, col=0.0, free=0.0)
    live = {}
    n, w = int(os.environ.get("FQ_N", "60")), 8
    for i in range(n + w + fs):
        if i == w:
            t0 = time.perf_counter()
            tm = dict(cut=0.0, enq=0.0, col=0.0, free=0.0)
        sl = i % fs
        if sl in live:
            a = time.perf_counter()
            check(eng.collect(cap=4096, slot=sl), (fs, i))
            b = time.perf_counter()
            for h in live.pop(sl):
                eng.free(h)
            c = time.perf_counter()
            tm["col"] += b - a
            tm["free"] += c - b
        if i < n + w:
            a = time.perf_counter()
            fl = [eng.file_list(fh, o, len(x)) for o, x in zip(offs, lists)]
            b = time.perf_counter()
            eng.enqueue(q.terms, fl, p, slot=sl)
            c = time.perf_counter()
            live[sl] = fl
            tm["cut"] += b - a
            tm["enq"] += c - b
    el = time.perf_counter() - t0
    print(f"in flight {fs}: {n/el:.1f} q/s; per query us: " +
          " ".join(f"{k} {v/n*1e6:.0f}" for k, v in tm.items()), flush=True)
print("mismatches", bad, flush=True)
# the cut alone, back to back
a = time.perf_counter()
for _ in range(20):
    for h in [eng.file_list(fh, o, len(x)) for o, x in zip(offs, lists)]:
        eng.free(h)
print(f"cut+free alone: {(time.perf_counter()-a)/20*1e6:.0f} us per query", flush=True)
