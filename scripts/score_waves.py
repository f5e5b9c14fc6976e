"""Diagnostic: per-wave timing of k_score on the config-2 query.

Runs with GBGPU_SCORE_MODE=2, which makes k_score record each wave's start
and end clock (s_memrealtime, 100 MHz), its survivors and the largest
record count among its lanes; prints the launch span, the start ramp and
the slowest waves."""
import os
import sys

import numpy as np

here = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(here, "..", "open-source-search-engine_amd", "python"))
dump = os.path.abspath(os.environ.setdefault("GBGPU_SCORE_DUMP", "gpurun_out/sdbg.bin"))
os.environ["GBGPU_SCORE_MODE"] = "2"
if os.path.exists(dump):
    os.remove(dump)

import gbgpu  # noqa: E402
from workload import config_two_term, generate  # noqa: E402

N = int(os.environ.get("SW_DOCS", 100_000_000))
q = config_two_term(N, docs_to_get=100, seed=1)
lists = generate(q, N, threads=16)
with gbgpu.Engine(0, diag=True) as eng:
    hs = [eng.upload(l) for l in lists]
    for _ in range(3):
        eng.query_resident(q.terms, hs, q.params(), cap=128)
d = np.fromfile(dump, dtype=np.uint64).reshape(3, -1, 8)[-1]
t0, t1, dmax = d[:, 0].astype(np.int64), d[:, 1].astype(np.int64), d[:, 2].astype(np.int64)
its, rsum = (d[:, 3] >> 32).astype(np.int64), (d[:, 3] & 0xffffffff).astype(np.int64)
act = its > 0
base = t0.min()
dur = (t1 - t0) * 10 / 1000.0  # us
print(f"blocks {len(d)} active waves {act.sum()} survivors {its.sum()} records {rsum.sum()}")
print(f"span {(t1.max() - base) * 10 / 1000:.1f} us; start ramp: last active start {(t0[act].max() - base) * 10 / 1000:.1f} us,"
      f" idle waves end by {(t1[~act].max() - base) * 10 / 1000 if (~act).any() else 0:.1f} us")
da = dur[act]
print("active wave duration us: p50 %.1f p90 %.1f p99 %.1f max %.1f" % tuple(np.percentile(da, [50, 90, 99, 100])))
print("max records per lane in wave: p50 %d p90 %d p99 %d max %d" % tuple(np.percentile(dmax[act], [50, 90, 99, 100])))
seg = d[:, 4:7].astype(np.float64) / 1000.0  # kcycles (s_memtime)
print("segments (kcycles, max over lanes of per-lane sums; mean over active waves): setup %.1f merge %.1f score %.1f"
      % tuple(seg[act].mean(axis=0)))
mm = d[:, 7]
mseg = np.stack([(mm & 0xfffff), (mm >> 20) & 0xfffff, (mm >> 40) & 0xfffff], axis=1).astype(np.float64) / 1000.0
print("mini-merge (kcycles): run locations %.1f staging %.1f merge loop %.1f" % tuple(mseg[act].mean(axis=0)))
o = np.argsort(-dur)[:12]
for b in o:
    print(f"  block {b}: start {(t0[b] - base) * 10 / 1000:.1f} us dur {dur[b]:.1f} us its {its[b]} maxrec {dmax[b]} sumrec {rsum[b]}"
          f" seg {seg[b, 0]:.1f}/{seg[b, 1]:.1f}/{seg[b, 2]:.1f} kcyc")
for lo, hi in ((0, 8), (8, 16), (16, 32), (32, 64), (64, 1 << 30)):
    m = act & (dmax >= lo) & (dmax < hi)
    if m.any():
        print(f"  maxrec [{lo},{hi}): waves {m.sum()} mean dur {dur[m].mean():.1f} us")
