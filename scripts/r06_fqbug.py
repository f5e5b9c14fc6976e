"""Round 6: file-cut lists through the slot API (one query at a time) gave
other top docids than the resident lists and ~1 s collects
(scripts/r06_fqprof.py).  Which step makes the difference: the same loop
with the resident lists, with query_resident, and with cuts, each with the
slot's device timings and work counts."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "open-source-search-engine_amd", "python")]
os.environ["GPU_MAX_HW_QUEUES"] = "16"
import numpy as np  # noqa: E402
import bench  # noqa: E402
import gbgpu  # noqa: E402
from workload import config_two_term, generate  # noqa: E402

total = int(os.environ.get("FQ_DOCS", bench.CFG2_DOCS))
lib = os.environ.get("GBGPU_LIB", "")
eng = gbgpu.Engine(0, path=os.path.join(gbgpu.PKG_DIR, "lib", lib) if lib else None)
eng.set_profiling(True)
q = config_two_term(total, docs_to_get=100, seed=1)
lists = generate(q, total, doc_begin=0, doc_end=total, threads=16)
p = q.params()
eng.set_slots(4)
hs = [eng.upload(x) for x in lists]
r0 = eng.query(q.terms, eng.host_lists(lists), p)
ref = eng.query_resident(q.terms, hs, p)
print("host==resident", np.array_equal(r0.docids, ref.docids), flush=True)
fh = eng.file_upload(b"".join(lists))
offs = np.cumsum([0] + [len(x) for x in lists[:-1]]).tolist()


def show(tag, r):
    ms, _ = eng.last_timings(0)
    st = eng.stats(0)
    ok = r.hits == ref.hits and np.array_equal(r.docids, ref.docids)
    print(f"{tag}: ok={ok} hits={r.hits} ms={[round(x, 3) for x in ms]} cand={st['candidates']} "
          f"surv={st['survivors']} runb={st['survivor_run_bytes']} top={r.docids[:3]}", flush=True)


for it in range(int(os.environ.get("FQ_A", "4"))):
    eng.enqueue(q.terms, hs, p, slot=0)
    show(f"A resident enqueue {it}", eng.collect(cap=4096, slot=0))
for it in range(4):
    fl = [eng.file_list(fh, o, len(x)) for o, x in zip(offs, lists)]
    show(f"B cut query_resident {it}", eng.query_resident(q.terms, fl, p))
    for h in fl:
        eng.free(h)
for it in range(4):
    fl = [eng.file_list(fh, o, len(x)) for o, x in zip(offs, lists)]
    eng.enqueue(q.terms, fl, p, slot=0)
    show(f"C cut enqueue {it}", eng.collect(cap=4096, slot=0))
    for h in fl:
        eng.free(h)
for it in range(3):
    fl = [eng.file_list(fh, o, len(x)) for o, x in zip(offs, lists)]
    show(f"D cut query_resident kept {it}", eng.query_resident(q.terms, fl, p))
    eng.enqueue(q.terms, fl, p, slot=0)
    show(f"D cut enqueue kept {it}", eng.collect(cap=4096, slot=0))
    for h in fl:
        eng.free(h)
