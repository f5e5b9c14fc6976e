"""Benchmark: Posdb query scoring on MI355X (BASELINE.json metric).

One step = one query over a synthetic Zipfian posdb index resident in HBM.
At N=1 the workload is config 2 (100M docs, 2-term AND + bigram, top-100),
rotating over 16 distinct 2-term queries (distinct termIds, ~3.5 GB of lists,
far above the 256 MiB Infinity Cache, so the list scan reads HBM).  At N>1 the
index is docid-range sharded, 125M docs per GPU -- at N=8 exactly config 4's
1B-doc index -- every rank scores its shard and the shards' top lists are
all-gathered over RCCL and merged on the device Msg3a-style
(gbgpu_allgather_topk, Msg3a.cpp:1315-1467).

    python bench.py --gpus 1 --steps 400 --warmup 5
    torchrun --nproc-per-node N bench.py --gpus N ...

Prints one JSON line (rank 0).  value = aggregate posdb list bytes scanned
per second (GB/s, all ranks); queries/sec beside it.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "open-source-search-engine_amd", "python"))

# Every query in flight needs a hardware queue of its own: HIP maps streams
# onto GPU_MAX_HW_QUEUES queues (4 by default, one taken by the upload
# stream), and slots sharing a queue run their kernels in turn -- a
# clustered query's one-CU TopTree replay then blocks the other's scan.
# Set before HIP initialises (torch / the library load below).
HW_QUEUES = 16
if int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0) < HW_QUEUES:
    os.environ["GPU_MAX_HW_QUEUES"] = str(HW_QUEUES)

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
CFG2_DOCS = 100_000_000
CFG4_DOCS_PER_GPU = 125_000_000  # 1B docs over 8 GPUs


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_threads():
    """The host threads this process may use (the GPU box gives a share of a
    larger machine: `nproc` overstates it; the box exports OMP_NUM_THREADS)."""
    n = len(os.sched_getaffinity(0))
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return max(1, min(n, share) if share > 0 else n)


# ------------------------------------------------------------ CPU baselines
def _gbref_requests(terms, lists, params, reps):
    """op=1 request bytes of oracle/_ref/gbref (see tests/ref_binding.py)."""
    import ctypes
    import struct
    import gbgpu
    qt = (gbgpu.QTerm * max(1, len(terms)))(*terms)
    req = [struct.pack("<ii", 1, len(terms)), bytes(params), bytes(qt)[:ctypes.sizeof(gbgpu.QTerm) * len(terms)]]
    for l in lists:
        req.append(struct.pack("<q", len(l)))
        req.append(bytes(l))
    req.append(struct.pack("<iiii", 128, 0, reps, 0))  # no whitelist lists
    req.append(struct.pack("<ii", 0, 0))  # no boolean expression, no facet ranges
    return b"".join(req)


def _gbref_run(exe, req, nproc):
    """nproc gbref processes each serving the same request; returns the per
    process median seconds inside intersectLists10_r and the hit counts."""
    import ctypes
    import struct
    procs = [subprocess.Popen([exe], stdin=subprocess.PIPE, stdout=subprocess.PIPE) for _ in range(nproc)]
    outs = [None] * nproc

    def drive(i):
        p = procs[i]
        p.stdin.write(req)
        p.stdin.close()
        outs[i] = p.stdout.read()
        p.wait()

    th = [threading.Thread(target=drive, args=(i,)) for i in range(nproc)]
    t0 = time.perf_counter()
    for t in th:
        t.start()
    for t in th:
        t.join()
    wall = time.perf_counter() - t0
    res = []
    for o in outs:
        # orc_result: hits i64, filtered i32, docs_wanted i32, n i32, corrupt i32
        hits, _, _, n, corrupt = struct.unpack_from("<qiiii", o, 0)
        off = 24 + 12 * n
        (nv,) = struct.unpack_from("<q", o, off)
        (sec,) = struct.unpack_from("<d", o, off + 8 + 8 * nv)
        if corrupt < 0:
            raise RuntimeError(f"gbref rc {-corrupt}")
        res.append((sec, hits))
    return res, wall


def cpu_baseline_query(q, lists, budget_s=20.0, clustering=False):
    """The reference's own PosdbTable::intersectLists10_r (oracle/_ref/gbref,
    compiled from the unmodified sources, -O2 as its Makefile) on the SAME
    full-size lists as the GPU, timed inside the harness (list copies, which
    the reference mutates, excluded): 1 thread, then one process per host
    thread of this box's share running the same query.  Falls back to the C
    restatement (kind "port") where the reference was not built.  clustering:
    the same with m_doSiteClustering (Msg39's default request: the prefilters
    and the TopTree's domain caps, Posdb.cpp:6322-6504, TopTree.cpp:312-516)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    p = q.params(site_clustering=1) if clustering else q.params()
    nbytes = sum(len(l) for l in lists)
    exe = os.path.join(ROOT, "oracle", "_ref", "gbref")
    threads = cpu_threads()
    out = {"unit": "GB/s", "cpu_model": cpu_model(), "host_threads_available": threads,
           "sample": f"the full config-2 query ({nbytes/1e6:.1f} MB of lists, the GPU's first rotation query)"}
    if os.access(exe, os.X_OK):
        one, _ = _gbref_run(exe, _gbref_requests(q.terms, lists, p, 1), 1)
        t1 = max(one[0][0], 1e-6)
        reps1 = int(max(3, min(50, budget_s * 0.3 / t1)))
        r1, _ = _gbref_run(exe, _gbref_requests(q.terms, lists, p, reps1), 1)
        per1 = r1[0][0]
        repsn = int(max(2, min(50, budget_s * 0.6 / t1)))
        rn, wall = _gbref_run(exe, _gbref_requests(q.terms, lists, p, repsn), threads)
        qps_n = sum(1.0 / max(s, 1e-9) for s, _ in rn)
        out.update({
            "kind": "reference",
            "value": round(nbytes / per1 / 1e9, 4),
            "cores": 1,
            "queries_per_sec": round(1.0 / per1, 3),
            "throughput": {"cores": threads, "queries_per_sec": round(qps_n, 3),
                           "value": round(nbytes * qps_n / 1e9, 4), "unit": "GB/s",
                           "note": f"{threads} gbref processes, each the same query {repsn}x "
                                   f"(median per process), {wall:.1f} s wall"},
            "hits": int(r1[0][1]),
            "detail": f"oracle/_ref/gbref: median of {reps1} runs inside intersectLists10_r, 1 thread",
        })
        return out
    import oracle_binding as orc
    t0 = time.perf_counter()
    reps = 0
    while True:
        orc.query(q.terms, lists, p)
        reps += 1
        if time.perf_counter() - t0 > budget_s * 0.5 or reps >= 20:
            break
    per = (time.perf_counter() - t0) / reps
    out.update({"kind": "port", "value": round(nbytes / per / 1e9, 4), "cores": 1,
                "queries_per_sec": round(1.0 / per, 3),
                "detail": f"oracle/posdb_oracle.c (reference not built here), {reps} reps"})
    return out


# ---------------------------------------------------------------- config 3
def bench_config3(eng, num_docs, steps, slots, with_cpu):
    """Config 3 (BASELINE.json): the ten fixed 3-5 word queries, three with a
    quoted phrase (term-pair proximity path), over a 100M-doc index resident in
    HBM; queries run round-robin with `slots` of them in flight."""
    from workload import config3_queries, generate

    qs = config3_queries(num_docs, docs_to_get=100)
    t0 = time.time()
    hs, qbytes, first_lists = [], [], None
    for q in qs:
        lists = generate(q, num_docs, threads=16)
        if first_lists is None:
            first_lists = lists
        hs.append([eng.upload(l) for l in lists])
        qbytes.append(sum(len(l) for l in lists))
    log(f"[config3] generated + uploaded {sum(qbytes)/1e9:.2f} GB of lists in {time.time()-t0:.1f}s")
    ps = [q.params() for q in qs]

    def run(nq):
        for i in range(nq):
            slot = i % slots
            if i >= slots:
                eng.collect(cap=4096, slot=slot)
            j = i % len(qs)
            eng.enqueue(qs[j].terms, hs[j], ps[j], slot=slot)
        for i in range(max(0, nq - slots), nq):
            eng.collect(cap=4096, slot=i % slots)

    # warm-up: every (slot, query) pair the timed rotation meets, so no slot
    # grows its buffers inside the timed region
    run(len(qs) * slots // math.gcd(len(qs), slots))
    eng.set_profiling(True)
    dev = []
    for j, q in enumerate(qs):
        eng.enqueue(q.terms, hs[j], ps[j], slot=0)
        eng.collect(cap=4096, slot=0)
        dev.append(eng.last_timings(slot=0)[0])
    eng.set_profiling(False)
    nq = max(steps, len(qs)) // len(qs) * len(qs)
    t = time.perf_counter()
    run(nq)
    el = time.perf_counter() - t
    scanned = sum(qbytes) * (nq // len(qs))
    for h in hs:
        for x in h:
            eng.free(x)
    r = {
        "workload": "config 3: 10 fixed 3-5 word queries (3 with a quoted phrase), top-100, 100M docs",
        "queries": nq,
        "queries_per_sec": round(nq / el, 2),
        "keys_scanned_GBps": round(scanned / el / 1e9, 2),
        "pct_hbm_peak_keys_scanned": round(100.0 * scanned / el / 1e9 / HBM_PEAK_GBS, 2),
        "avg_list_bytes_per_query": int(np.mean(qbytes)),
        "device_ms_per_query": [round(float(x[0]), 4) for x in dev],
        "phase_ms_mean": dict(zip(["total", "candidates", "probe", "compact", "score", "topk"],
                                  [round(float(v), 4) for v in np.mean(np.array(dev), axis=0)])),
    }
    if with_cpu:
        exe = os.path.join(ROOT, "oracle", "_ref", "gbref")
        if os.access(exe, os.X_OK):
            res, _ = _gbref_run(exe, _gbref_requests(qs[0].terms, first_lists, ps[0], 2), 1)
            sec = res[0][0]
            r["cpu_baseline"] = {"value": round(qbytes[0] / sec / 1e9, 4), "unit": "GB/s", "cores": 1,
                                 "kind": "reference", "queries_per_sec": round(1.0 / sec, 3),
                                 "sample": f"config-3 query {qs[0].name} at full size ({qbytes[0]/1e6:.0f} MB), "
                                           f"oracle/_ref/gbref median of 2 runs inside intersectLists10_r"}
    return r


# ---------------------------------------------------------------- config 5
def bench_merge(eng, steps, total_keys, with_cpu):
    """Config 5 (BASELINE.json): RdbList::posdbMerge_r of 8 tiered posdb runs
    (sizes 1:2:..:128, 5% of keys repeated across runs, 1% delete keys), runs
    and output resident in HBM (gbgpu_merge_posdb_device)."""
    import torch
    import gbgpu

    t0 = time.time()
    m = gbgpu.MergeRuns(total_keys, nruns=8, seed=5, nterms=20000, nthreads=16)
    sizes = [len(a) for a in m.arrays]
    dev = [torch.from_numpy(a).to("cuda") if len(a) else torch.zeros(16, dtype=torch.uint8, device="cuda")
           for a in m.arrays]
    m.free()
    log(f"[merge] generated + uploaded {sum(sizes)/1e9:.2f} GB of runs in {time.time()-t0:.1f}s")
    cap = sum(sizes) + 64
    out = torch.empty(cap, dtype=torch.uint8, device="cuda")
    ptrs = [d.data_ptr() for d in dev]
    res = {}
    for rm in (1, 0):  # removeNegKeys=0 (the disk merge) last: its output stays in `out`
        eng.merge_posdb_device(ptrs, sizes, rm, -1, out.data_ptr(), cap)  # warmup
        wall, dev_ms = [], []
        for _ in range(steps):
            torch.cuda.synchronize()
            t = time.perf_counter()
            n = eng.merge_posdb_device(ptrs, sizes, rm, -1, out.data_ptr(), cap)
            wall.append(time.perf_counter() - t)
            ms, nkeys, ntiles = eng.merge_timings()
            dev_ms.append(ms)
        res[rm] = (n, float(np.median(wall)), np.mean(np.array(dev_ms), axis=0), nkeys, ntiles)
    n, w, ms, nkeys, ntiles = res[0]
    out2 = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    n2 = eng.merge_posdb_device([out.data_ptr()], [n], 0, -1, out2.data_ptr(), n + 64)
    idem = bool(n2 == n and torch.equal(out[:n], out2[:n]))
    in_b = float(sum(sizes))
    r = {
        "workload": "config 5: RdbList::posdbMerge_r of 8 tiered posdb runs (1:2:..:128), 5% cross-run "
                    "duplicates, 1% delete keys, removeNegKeys=0 (disk merge), resident in HBM",
        "input_bytes": int(in_b),
        "output_bytes": int(n),
        "keys": int(nkeys),
        "ms_per_merge": round(w * 1e3, 3),
        "input_GBps": round(in_b / w / 1e9, 2),
        "in_plus_out_GBps": round((in_b + n) / w / 1e9, 2),
        "keys_per_s": round(nkeys / w, 1),
        "phase_ms": dict(zip(["total", "decode", "partition", "tile_merge", "offsets", "copy"],
                             [round(float(x), 3) for x in ms])),
        "tiles": int(ntiles),
        "remove_neg_keys_ms": round(res[1][1] * 1e3, 3),
        "idempotent": idem,
        "roofline": {"bound": "hbm", "achieved": round((in_b + n) / (ms[0] / 1e3) / 1e9, 2), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round((in_b + n) / (ms[0] / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                     "note": "whole merge, algorithmic bytes = input + output"},
    }
    del dev, out, out2
    if with_cpu:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        sample_keys = 20_000_000
        runs = gbgpu.synth_merge_runs(sample_keys, nruns=8, seed=5, nterms=20000, nthreads=16)
        sb = sum(map(len, runs))
        try:
            import ref_binding as ref
            if not ref.available():
                raise RuntimeError("gbref not built")
            secs = [ref.posdb_merge(runs, False, -1, timed=True)[1] for _ in range(3)]
            ref.close()
            sec = float(np.median(secs))
            r["cpu_baseline"] = {"value": round(sb / sec / 1e9, 4), "unit": "GB/s (input)", "cores": 1,
                                 "kind": "reference",
                                 "sample": f"{sample_keys} keys ({sb/1e6:.0f} MB) of the same generator, the "
                                           f"reference's own RdbList::merge_r (oracle/_ref/gbref), median of 3"}
        except Exception as e:  # reference not built: the C restatement
            import ctypes
            import oracle_binding as orc
            keep, p, sz = orc._lists(runs)
            buf = ctypes.create_string_buffer(sb + 64)
            t = time.perf_counter()
            orc.lib().orc_posdb_merge(p, sz, len(runs), 0, -1, buf, sb + 64)
            el = time.perf_counter() - t
            r["cpu_baseline"] = {"value": round(sb / el / 1e9, 4), "unit": "GB/s (input)", "cores": 1,
                                 "kind": "port", "reference_error": repr(e)[:120],
                                 "sample": f"{sample_keys} keys ({sb/1e6:.0f} MB), oracle/posdb_merge_oracle.c"}
    return r


def pmc_traffic(kernel_prefix: str):
    """HBM bytes per launch of a kernel from the newest committed rocprofv3 PMC
    pass (profiles/rNN_*pmc_traffic.json, the highest round), corrected per
    MI355X_MICROARCH.md (scripts/pmc_traffic.py)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]_*pmc_traffic.json")))
    if not files:
        return None, None
    d = json.load(open(files[-1]))
    for k, v in d["kernels"].items():
        if k.startswith(kernel_prefix):
            return v.get("hbm_bytes_per_launch_corrected"), os.path.basename(files[-1])
    return None, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--docs-per-gpu", type=int, default=0, help="0: 100M at N=1 (config 2), 125M at N>1 (config 4)")
    ap.add_argument("--docs-to-get", type=int, default=100)
    ap.add_argument("--queries", type=int, default=16, help="distinct config-2 queries the steps rotate over")
    ap.add_argument("--slots", type=int, default=12, help="queries in flight per GPU (query slots)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-merge", action="store_true", help="skip the config-5 list merge measurement")
    ap.add_argument("--no-config3", action="store_true", help="skip the config-3 query-mix measurement")
    ap.add_argument("--no-file-read", action="store_true", help="skip the resident-file read measurement")
    ap.add_argument("--no-clustering", action="store_true",
                    help="skip the config-2 rotation with site clustering (the Msg39 default)")
    ap.add_argument("--no-ceiling", action="store_true", help="skip the streaming-bandwidth ceiling")
    ap.add_argument("--merge-keys", type=int, default=400_000_000, help="config-5 keys (~4.4 GB of runs)")
    ap.add_argument("--exchange", action="store_true",
                    help="run the RCCL Msg3a exchange even on one GPU (a one-rank communicator)")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: WORLD_SIZE={world} != --gpus {args.gpus}; using WORLD_SIZE")

    import torch
    import torch.distributed as dist
    import gbgpu
    from workload import config_two_term, generate

    torch.cuda.set_device(local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    per = args.docs_per_gpu or (CFG2_DOCS if world == 1 else CFG4_DOCS_PER_GPU)
    total = per * world
    # GBGPU_DIAG=1: the diagnostic build (lib/libgbgpu_diag.so), whose
    # GBGPU_*_MODE switches time kernel phases; never the measured product
    # GBGPU_LIB=alt: the A/B build (lib/libgbgpu_alt.so, Makefile `alt`);
    # GBGPU_LIB=<name>.so: another A/B build under lib/ (scripts/bisect_libs.sh)
    lib = os.environ.get("GBGPU_LIB", "")
    eng = gbgpu.Engine(local_rank, diag=os.environ.get("GBGPU_DIAG") == "1",
                       path=gbgpu.ALT_LIB_PATH if lib == "alt" else
                       os.path.join(gbgpu.PKG_DIR, "lib", lib) if lib.endswith(".so") else None)
    exchange = world > 1 or args.exchange
    if exchange and world == 1:
        eng.comm_init(1, 0, gbgpu.Engine.comm_unique_id())
    if world > 1:
        # the library's own communicator for the Msg3a exchange
        uid = torch.zeros(128, dtype=torch.uint8, device="cuda")
        if rank == 0:
            uid.copy_(torch.frombuffer(bytearray(gbgpu.Engine.comm_unique_id()), dtype=torch.uint8))
        dist.broadcast(uid, 0)
        eng.comm_init(world, rank, bytes(uid.cpu().numpy()))

    # the rotation: distinct 2-term queries (distinct termIds), each with its
    # own lists; every rank holds its docid range of each list
    qs = [config_two_term(total, docs_to_get=args.docs_to_get, seed=s + 1) for s in range(args.queries)]
    t0 = time.time()
    handles, qbytes, first_lists = [], [], None
    for q in qs:
        lists = generate(q, total, doc_begin=rank * per, doc_end=(rank + 1) * per, threads=16)
        if first_lists is None:
            first_lists = lists
        handles.append([eng.upload(l) for l in lists])
        qbytes.append(sum(len(l) for l in lists))
    log(f"[rank {rank}] generated + uploaded {len(qs)} queries, {sum(qbytes)/1e9:.2f} GB of lists "
        f"in {time.time()-t0:.1f}s")
    ps = [q.params() for q in qs]
    k = ps[0].docs_to_get
    slots = max(1, args.slots)
    eng.set_slots(slots)

    def finish(slot):
        if not exchange:
            return eng.collect(cap=4096, slot=slot).hits
        _, _, hits = eng.allgather_topk(k, slot=slot)
        return hits

    def run(nq):
        """nq queries round-robin over the rotation with `slots` in flight (a
        slot's previous query is collected before it is reused)."""
        hits = 0
        for i in range(nq):
            slot = i % slots
            if i >= slots:
                hits = finish(slot)
            j = i % len(qs)
            eng.enqueue(qs[j].terms, handles[j], ps[j], slot=slot)
        for i in range(max(0, nq - slots), nq):
            hits = finish(i % slots)
        return hits

    run(args.warmup * slots)
    # per-phase device times (HIP events on the slot stream) and work counts,
    # one query at a time over the whole rotation (untimed)
    eng.set_profiling(True)
    phase, stats = [], []
    for rep in range(2):
        for j, q in enumerate(qs):
            eng.enqueue(q.terms, handles[j], ps[j], slot=0)
            finish(0)
            if rep:
                phase.append(eng.last_timings(slot=0)[0])
                stats.append(eng.stats(slot=0))
    eng.set_profiling(False)

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    hits = run(args.steps)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    # bytes of the steps actually run on this rank (round-robin rotation)
    my_bytes = float(sum(qbytes[i % len(qs)] for i in range(args.steps)))
    if world > 1:
        t = torch.tensor([el, my_bytes], dtype=torch.float64, device="cuda")
        tt = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(tt, t)
        el = max(float(x[0]) for x in tt)
        agg_bytes = sum(float(x[1]) for x in tt)
    else:
        agg_bytes = my_bytes

    ms_per_step = el * 1000.0 / args.steps
    qps = args.steps / el
    gbs = agg_bytes / el / 1e9

    ph = np.array(phase)
    names = ["total", "candidates", "probe", "compact", "score", "topk"]
    sum_ms = ph.sum(axis=0)
    tot = {key: float(sum(st[key] for st in stats)) for key in stats[0]}
    # algorithmic bytes per kernel, summed over the rotation
    kern_bytes = {
        "candidates": tot["g0_bytes"] + 8.0 * tot["candidates"],
        "probe": tot["probe_bytes"],
        "compact": 8.0 * tot["candidates"] + 16.0 * tot["survivors"],
        "score": tot["survivor_run_bytes"] + 12.0 * tot["survivors"],
    }
    kernels = {}
    for i, nm in enumerate(names[1:], start=1):
        entry = {"ms_per_query": round(float(sum_ms[i]) / len(phase), 4)}
        if nm in kern_bytes and sum_ms[i] > 0:
            a = kern_bytes[nm] / (sum_ms[i] / 1e3) / 1e9
            entry.update({"algorithmic_bytes_per_query": int(kern_bytes[nm] / len(phase)),
                          "achieved_GBps": round(a, 1), "frac_of_peak": round(a / HBM_PEAK_GBS, 4)})
        kernels[nm] = entry
    probe_achieved = kern_bytes["probe"] / (sum_ms[2] / 1e3) / 1e9
    ceiling = None
    if rank == 0 and not args.no_ceiling:
        rd, cp = eng.bandwidth_ceiling(4 << 30, 8)
        ceiling = {"read_GBps": round(rd, 1), "copy_GBps": round(cp, 1),
                   "kernel": "k_stream_read / k_stream_copy (16 B/lane, 4 GiB buffers, 8 passes)"}
    traffic, traffic_src = pmc_traffic("k_probe")
    result = {
        "metric": "queries/sec + posdb keys scanned GB/s (% HBM peak), 1/2/4/8 MI355X",
        "value": round(gbs, 3),
        "unit": "GB/s",
        "queries_per_sec": round(qps, 3),
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "queries_in_flight": slots,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic Zipfian posdb lists (SURVEY.md §8(d) generator), resident in HBM",
        "config": {
            "workload": ("config 2: 2-term AND (+bigram sublist), top-100, 100M docs" if world == 1 else
                         f"config 4: {total/1e9:.3g}B-doc index docid-sharded, {per/1e6:.0f}M docs per GPU, "
                         f"per-GPU top-100 + RCCL allgather + device Msg3a merge"),
            "rotation": f"{len(qs)} distinct 2-term queries (distinct termIds), round-robin",
            "docs_per_gpu": per,
            "docs_total": total,
            "list_bytes_per_gpu_rotation": int(sum(qbytes)),
            "list_bytes_per_query_mean": int(np.mean(qbytes)),
            "hits_last": int(hits),
            "pct_hbm_peak_keys_scanned": round(100.0 * gbs / (HBM_PEAK_GBS * world), 2),
        },
        "device_ms_per_query": round(float(sum_ms[0]) / len(phase), 4),
        "phase_ms": {nm: round(float(sum_ms[i]) / len(phase), 4) for i, nm in enumerate(names)},
        "kernels": kernels,
        "roofline": {
            "bound": "hbm",
            "kernel": "k_probe (the list scan: every sublist but the candidate array's)",
            "achieved": round(probe_achieved, 2),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(probe_achieved / HBM_PEAK_GBS, 4),
            "ceiling": ceiling,
            "frac_of_ceiling": round(probe_achieved / ceiling["read_GBps"], 4) if ceiling else None,
            "traffic": traffic,
            "traffic_source": traffic_src,
            "algorithmic_bytes_per_launch": int(kern_bytes["probe"] / len(phase)),
            "timing": "HIP events around the launch on the slot stream, mean over the rotation",
        },
    }
    if rank == 0 and world == 1 and not args.no_clustering:
        # the same rotation as Msg39 sends it by default: m_doSiteClustering
        # (Msg39.h:41) -- the prefilter bounds (k_bound) and the in-docid-order
        # TopTree replay (k_tree_replay) instead of the radix top-k
        pc = [q.params(site_clustering=1) for q in qs]
        eng.set_profiling(True)
        cdev = []
        for j, q in enumerate(qs):
            eng.enqueue(q.terms, handles[j], pc[j], slot=0)
            eng.collect(cap=4096, slot=0)
            cdev.append(eng.last_timings(slot=0)[0])
        eng.set_profiling(False)
        nc = max(4 * slots * len(qs), args.steps)  # steady state: fill and drain are a few queries
        # every slot's clustering buffers (replay entries, ranks, the TopTree
        # result block) sized before the clock starts
        nw = 4 * slots
        for i in range(nw):
            slot = i % slots
            if i >= slots:
                eng.collect(cap=4096, slot=slot)
            eng.enqueue(qs[i % len(qs)].terms, handles[i % len(qs)], pc[i % len(qs)], slot=slot)
        for i in range(nw - slots, nw):
            eng.collect(cap=4096, slot=i % slots)
        t_c = time.perf_counter()
        for i in range(nc):
            slot = i % slots
            if i >= slots:
                eng.collect(cap=4096, slot=slot)
            eng.enqueue(qs[i % len(qs)].terms, handles[i % len(qs)], pc[i % len(qs)], slot=slot)
        for i in range(max(0, nc - slots), nc):
            eng.collect(cap=4096, slot=i % slots)
        el_c = time.perf_counter() - t_c
        cb = float(sum(qbytes[i % len(qs)] for i in range(nc)))
        cd = np.array(cdev)
        result["clustering"] = {
            "workload": "config 2 with site clustering (Msg39's default request), same rotation",
            "queries": nc,
            "queries_in_flight": slots,
            "queries_per_sec": round(nc / el_c, 3),
            "keys_scanned_GBps": round(cb / el_c / 1e9, 3),
            "device_ms_per_query": round(float(cd[:, 0].mean()), 4),
            "phase_ms": dict(zip(["total", "candidates", "probe", "compact", "score", "bound+replay"],
                                 [round(float(v), 4) for v in cd.mean(axis=0)])),
        }
    if rank == 0 and world == 1:
        # the C-ABI's host-buffer entry (gbgpu_query: lists in pageable host
        # memory, uploaded per call) -- PCIe-inclusive, reported beside `value`
        n_pc = 10
        host = eng.host_lists(first_lists)
        r0 = eng.query(qs[0].terms, host, ps[0])
        t_pc = time.perf_counter()
        for _ in range(n_pc):
            r_pc = eng.query(qs[0].terms, host, ps[0])
        el_pc = time.perf_counter() - t_pc
        if r_pc.hits != r0.hits:
            raise RuntimeError("host-buffer query results differ between calls")
        result["pcie_inclusive"] = {
            "queries_per_sec": round(n_pc / el_pc, 3),
            "keys_scanned_GBps": round(qbytes[0] * n_pc / el_pc / 1e9, 3),
            "note": "gbgpu_query with the lists in pageable host memory, uploaded every call; not `value`",
        }
        del host
    if rank == 0 and world == 1 and not args.no_file_read:
        # the read path into HBM (f3): the lists as one resident Posdb file
        # image, each query cutting its termlists from it on the device
        # (gbgpu_file_list, RdbScan's read) and freeing them after
        blob = b"".join(first_lists)
        fh = eng.file_upload(blob)
        del blob
        offs = np.cumsum([0] + [len(x) for x in first_lists[:-1]]).tolist()
        n_fr = 20
        for it in range(n_fr + 2):
            if it == 2:
                t_fr = time.perf_counter()
            fl = eng.file_lists(fh, offs, [len(x) for x in first_lists])  # the query's reads together
            r_fr = eng.query_resident(qs[0].terms, fl, ps[0])
            for h in fl:
                eng.free(h)
            if r_fr.hits != r0.hits or not np.array_equal(r_fr.docids, r0.docids):
                raise RuntimeError("file-cut query differs from the host-buffer query")
        el_fr = time.perf_counter() - t_fr
        # the same with queries in flight: the next query's termlists are cut
        # (upload stream) while earlier ones run on their slots
        fs = min(int(os.environ.get("GBGPU_FR_INFLIGHT", "4")), slots)
        n_fq, w_fq = 120, 2 * fs  # the first 2*fs queries warm the slots (untimed)
        live = {}
        for i in range(n_fq + w_fq + fs):
            if i == w_fq:
                t_fq = time.perf_counter()
            sl = i % fs
            if sl in live:
                r_fq = eng.collect(cap=4096, slot=sl)
                for h in live.pop(sl):
                    eng.free(h)
                if r_fq.hits != r0.hits or not np.array_equal(r_fq.docids, r0.docids):
                    raise RuntimeError("file-cut query differs from the host-buffer query")
            if i < n_fq + w_fq:
                fl = eng.file_lists(fh, offs, [len(x) for x in first_lists])
                eng.enqueue(qs[0].terms, fl, ps[0], slot=sl)
                live[sl] = fl
        el_fq = time.perf_counter() - t_fq
        eng.file_free(fh)
        result["file_read"] = {
            "queries_per_sec": round(n_fr / el_fr, 3),
            "keys_scanned_GBps": round(qbytes[0] * n_fr / el_fr / 1e9, 3),
            "in_flight": {"queries": fs, "queries_per_sec": round(n_fq / el_fq, 3)},
            "note": "termlists cut per query from a resident Posdb file image (gbgpu_file_lists: the query's "
                    "cuts together, each image built by its structure/page-map/granule pass), queried, freed; one query at a time, and with "
                    "`in_flight.queries` queries in flight; not `value`",
        }
        # Msg5's read of a termlist (f3, gbgpu_termlist_merge): three resident
        # files, each holding a third of config 2's docid range, cut and merged
        # on the device with the tree's list (the first 1 000 docs again: the
        # newest copies of keys the first file holds, replaced in the merge),
        # into resident lists the query then reads.  The merged lists are
        # config 2's own, so the answer must be r0's.
        thirds = [generate(qs[0], total, doc_begin=j * per // 3, doc_end=(j + 1) * per // 3, threads=16)
                  for j in range(3)]
        tree = generate(qs[0], total, doc_begin=0, doc_end=1000, threads=1)
        fhs, offs3 = [], []
        for fl in thirds:
            fhs.append(eng.file_upload(b"".join(fl)))
            offs3.append(np.cumsum([0] + [len(x) for x in fl[:-1]]).tolist())

        def pieces(t):
            return [(fhs[j], int(offs3[j][t]), len(thirds[j][t]), None) for j in range(3) if thirds[j][t]] + \
                   ([tree[t]] if tree[t] else [])

        nt = len(first_lists)
        in_bytes = sum(len(thirds[j][t]) for j in range(3) for t in range(nt)) + sum(len(x) for x in tree)
        n_m = 20
        for it in range(n_m + 2):  # merge + query, checked
            if it == 2:
                t_mq = time.perf_counter()
            hl = [eng.termlist_merge(pieces(t)) for t in range(nt)]
            r_m = eng.query_resident(qs[0].terms, hl, ps[0])
            for h in hl:
                eng.free(h)
            if r_m.hits != r0.hits or not np.array_equal(r_m.docids, r0.docids):
                raise RuntimeError("Msg5-merged query differs from the host-buffer query")
        el_mq = time.perf_counter() - t_mq
        t_m = time.perf_counter()
        for it in range(n_m):  # the merges alone
            for t in range(nt):
                eng.free(eng.termlist_merge(pieces(t)))
        el_m = time.perf_counter() - t_m
        for fh in fhs:
            eng.file_free(fh)
        del thirds, tree
        result["msg5_merge"] = {
            "queries_per_sec": round(n_m / el_mq, 3),
            "merge_only_per_sec": round(n_m / el_m, 3),
            "merge_in_GBps": round(in_bytes * n_m / el_m / 1e9, 3),
            "bytes_in_per_query": in_bytes,
            "note": "each config-2 termlist merged on the device (gbgpu_termlist_merge: three file cuts, "
                    "docid thirds, plus a 1 000-doc tree list) into a resident list, then queried; one query "
                    "at a time; merge_only_per_sec: the merges without the query; not `value`",
        }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline_query(qs[0], first_lists)
        if "clustering" in result:
            result["clustering"]["cpu_baseline"] = cpu_baseline_query(qs[0], first_lists, budget_s=10.0, clustering=True)
    for hs in handles:
        for h in hs:
            eng.free(h)
    del first_lists
    if rank == 0 and world == 1 and not args.no_config3:
        result["config3"] = bench_config3(eng, CFG2_DOCS, max(args.steps // 4, 50), slots, not args.no_cpu_baseline)
    if rank == 0 and world == 1 and not args.no_merge:
        result["config5_merge"] = bench_merge(eng, max(3, min(args.steps, 10)), args.merge_keys,
                                              not args.no_cpu_baseline)
    eng.close()
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
