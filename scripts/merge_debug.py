"""Full-size config-5 check: GPU merge vs oracle, and merge(output) == output."""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "open-source-search-engine_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import gbgpu  # noqa: E402
import oracle_binding as orc  # noqa: E402

keys = int(float(sys.argv[1])) if len(sys.argv) > 1 else 400_000_000
m = gbgpu.MergeRuns(keys, nruns=8, seed=5, nterms=20000, nthreads=16)
sizes = [len(a) for a in m.arrays]
dev = [torch.from_numpy(a).to("cuda") for a in m.arrays]
cap = sum(sizes) + 64
out = torch.empty(cap, dtype=torch.uint8, device="cuda")
eng = gbgpu.Engine(0)
n = eng.merge_posdb_device([d.data_ptr() for d in dev], sizes, 0, -1, out.data_ptr(), cap)
print("gpu n", n, eng.merge_timings(), flush=True)
out2 = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
n2 = eng.merge_posdb_device([out.data_ptr()], [n], 0, -1, out2.data_ptr(), n + 64)
print("gpu n2", n2, eng.merge_timings(), flush=True)
g = out[:n].cpu().numpy()
g2 = out2[:n2].cpu().numpy()
ml = min(n, n2)
d = np.nonzero(g[:ml] != g2[:ml])[0]
print("idempotent diff count", len(d), "first", d[:5], flush=True)
if len(d):
    i = int(d[0])
    print("out ", g[max(0, i - 36):i + 36].tobytes().hex())
    print("out2", g2[max(0, i - 36):i + 36].tobytes().hex())
t = time.time()
ptrs = (ctypes.c_void_p * 8)(*[a.ctypes.data for a in m.arrays])
sz = (ctypes.c_int64 * 8)(*sizes)
ob = np.empty(cap, np.uint8)
no = orc.lib().orc_posdb_merge(ptrs, sz, 8, 0, -1, ob.ctypes.data, cap)
print("oracle n", no, time.time() - t, flush=True)
ml = min(n, no)
d = np.nonzero(g[:ml] != ob[:ml])[0]
print("vs oracle diff count", len(d), "first", d[:5], flush=True)
if len(d):
    i = int(d[0])
    print("gpu   ", g[max(0, i - 36):i + 36].tobytes().hex())
    print("oracle", ob[max(0, i - 36):i + 36].tobytes().hex())
m.free()
