"""Config-5 timing probe: gb_synth_merge_runs -> device tensors -> gbgpu_merge_posdb_device."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "open-source-search-engine_amd", "python"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import gbgpu  # noqa: E402

keys = int(float(sys.argv[1])) if len(sys.argv) > 1 else 400_000_000
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 3
t0 = time.time()
m = gbgpu.MergeRuns(keys, nruns=8, seed=5, nterms=20000, nthreads=16)
sizes = [len(a) for a in m.arrays]
print(f"gen {time.time()-t0:.1f}s total {sum(sizes)/1e9:.3f} GB sizes {sizes}", flush=True)
dev = [torch.from_numpy(a).to("cuda") if len(a) else torch.zeros(16, dtype=torch.uint8, device="cuda")
       for a in m.arrays]
m.free()
cap = sum(sizes) + 64
out = torch.empty(cap, dtype=torch.uint8, device="cuda")
eng = gbgpu.Engine(0)
for rm in ((0, 1) if iters >= 3 else (0,)):
    for it in range(iters):
        torch.cuda.synchronize()
        t = time.perf_counter()
        n = eng.merge_posdb_device([d.data_ptr() for d in dev], sizes, rm, -1, out.data_ptr(), cap)
        el = time.perf_counter() - t
        ms, nk, nt = eng.merge_timings()
        print(f"rm={rm} out {n/1e9:.3f} GB wall {el*1e3:.1f} ms dev {[round(x,2) for x in ms]} keys {nk} tiles {nt} "
              f"alg GB/s {(sum(sizes)+n)/ (ms[0]/1e3) / 1e9:.0f} path {eng.merge_path()}", flush=True)
eng.close()
