"""Benchmark: Posdb query scoring on MI355X (BASELINE.json metric).

One step = one query (config 2: 2-term AND + its bigram, top-100) over a
synthetic Zipfian posdb index resident in HBM.  At N GPUs the index is
docid-range sharded (100M docs per GPU, weak scaling, mirroring one Msg39 per
shard); every rank scores its shard, the per-shard top-k lists are
all-gathered over RCCL and merged Msg3a-style (Msg3a.cpp:1315-1467).

    python bench.py --gpus 1 --steps 20 --warmup 3
    torchrun --nproc-per-node N bench.py --gpus N ...

Prints one JSON line (rank 0).  value = aggregate posdb list bytes scanned
per second (GB/s); queries/sec is reported beside it.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "open-source-search-engine_amd", "python"))

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def cpu_baseline(q, num_docs_total: int, budget_s: float = 12.0):
    """Oracle (CPU restatement, 1 thread) on a bounded docid-range slice of the
    same corpus; reports list GB/s and queries/s on the slice."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_binding as orc
    from workload import generate

    sample_docs = min(num_docs_total, 2_000_000)
    lists = generate(q, num_docs_total, doc_begin=0, doc_end=sample_docs, threads=16)
    p = q.params()
    nbytes = sum(len(l) for l in lists)
    t0 = time.perf_counter()
    reps = 0
    while True:
        orc.query(q.terms, lists, p)
        reps += 1
        el = time.perf_counter() - t0
        if el >= budget_s or reps >= 2000:
            break
    per_q = el / reps
    out = {
        "value": round(nbytes / per_q / 1e9, 4),
        "unit": "GB/s",
        "cores": 1,
        "kind": "port",
        "qps_on_sample": round(1.0 / per_q, 3),
        "est_qps_full_index": round((sample_docs / num_docs_total) / per_q, 4),
        "sample": f"docs [0,{sample_docs}) of the same {num_docs_total}-doc corpus and query "
                  f"({nbytes/1e6:.1f} MB of lists), oracle/posdb_oracle.c single thread, {reps} reps, "
                  f"{el:.1f} s",
    }
    # the reference's own PosdbTable::intersectLists10_r (oracle/_ref/gbref,
    # built from the unmodified sources) on the same slice, when it was built
    try:
        import ref_binding as ref
        if ref.available():
            exp = orc.query(q.terms, lists, p)
            r1 = ref.query(q.terms, lists, p, reps=1)
            assert r1["hits"] == exp["hits"] and np.array_equal(r1["docids"], exp["docids"])
            nrep = int(max(3, min(2000, budget_s / max(r1["seconds"], 1e-6))))
            t0 = time.perf_counter()
            rr = ref.query(q.terms, lists, p, reps=nrep)
            el2 = time.perf_counter() - t0
            per_r = rr["seconds"]  # median of nrep runs, timed inside the harness
            out.update({
                "value": round(nbytes / per_r / 1e9, 4),
                "kind": "reference",
                "qps_on_sample": round(1.0 / per_r, 3),
                "est_qps_full_index": round((sample_docs / num_docs_total) / per_r, 4),
                "port_value": round(nbytes / per_q / 1e9, 4),
                "sample": f"docs [0,{sample_docs}) of the same {num_docs_total}-doc corpus and query "
                          f"({nbytes/1e6:.1f} MB of lists), the reference's PosdbTable (oracle/_ref/gbref, "
                          f"-O2 as its Makefile) single thread, median of {nrep} runs incl. the per-run "
                          f"list copy, {el2:.1f} s; port_value = oracle/posdb_oracle.c, {reps} reps",
            })
    except Exception as e:  # the reference build is optional (absent where /root/reference was)
        out["reference_error"] = repr(e)[:200]
    return out


def bench_config3(eng, num_docs: int, steps: int, slots: int):
    """Config 3 (BASELINE.json): the ten fixed 3-5 word queries, three with a
    quoted phrase (term-pair proximity path), over a 100M-doc index resident in
    HBM; queries run round-robin with `slots` of them in flight."""
    from workload import config3_queries, generate

    qs = config3_queries(num_docs, docs_to_get=100)
    t0 = time.time()
    hs, qbytes = [], []
    for q in qs:
        lists = generate(q, num_docs, threads=16)
        hs.append([eng.upload(l) for l in lists])
        qbytes.append(sum(len(l) for l in lists))
    log(f"[config3] generated + uploaded {sum(qbytes)/1e9:.2f} GB of lists in {time.time()-t0:.1f}s")
    ps = [q.params() for q in qs]

    def run(nq):
        hits = []
        for i in range(nq):
            slot = i % slots
            if i >= slots:
                hits.append(eng.collect(cap=4096, slot=slot).hits)
            j = i % len(qs)
            eng.enqueue(qs[j].terms, hs[j], ps[j], slot=slot)
        for i in range(max(0, nq - slots), nq):
            hits.append(eng.collect(cap=4096, slot=i % slots).hits)
        return hits

    run(len(qs))
    eng.set_profiling(True)
    dev = []
    for j, q in enumerate(qs):
        eng.enqueue(q.terms, hs[j], ps[j], slot=0)
        eng.collect(cap=4096, slot=0)
        dev.append(eng.last_timings(slot=0)[0][0])
    eng.set_profiling(False)
    nq = max(steps, len(qs)) // len(qs) * len(qs)
    t = time.perf_counter()
    run(nq)
    el = time.perf_counter() - t
    scanned = sum(qbytes) * (nq // len(qs))
    for h in hs:
        for x in h:
            eng.free(x)
    return {
        "workload": "config 3: 10 fixed 3-5 word queries (3 with a quoted phrase), top-100, 100M docs",
        "queries": nq,
        "queries_per_sec": round(nq / el, 2),
        "keys_scanned_GBps": round(scanned / el / 1e9, 2),
        "pct_hbm_peak_keys_scanned": round(100.0 * scanned / el / 1e9 / HBM_PEAK_GBS, 2),
        "avg_list_bytes_per_query": int(np.mean(qbytes)),
        "device_ms_per_query": [round(float(x), 4) for x in dev],
    }


def bench_merge(eng, steps: int, total_keys: int, with_cpu: bool):
    """Config 5 (BASELINE.json): RdbList::posdbMerge_r of 8 tiered posdb runs
    (sizes 1:2:..:128, 5% of keys repeated across runs, 1% delete keys),
    runs and output resident in HBM (gbgpu_merge_posdb_device).  Reports the
    merge rate (input bytes/s and (input+output) bytes/s), per-phase device
    times, a size-independent check (merging the output alone returns it) and
    the oracle's single-thread rate on a bounded sample of the same generator."""
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
    # size-independent property: the merged list is canonical, so merging it
    # alone reproduces it byte for byte
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
        import ctypes
        import oracle_binding as orc
        sample_keys = 20_000_000
        runs = gbgpu.synth_merge_runs(sample_keys, nruns=8, seed=5, nterms=20000, nthreads=16)
        keep, p, sz = orc._lists(runs)
        scap = sum(map(len, runs)) + 64
        buf = ctypes.create_string_buffer(scap)
        t = time.perf_counter()
        reps = 0
        while True:
            orc.lib().orc_posdb_merge(p, sz, len(runs), 0, -1, buf, scap)
            reps += 1
            el = time.perf_counter() - t
            if el > 8.0 or reps >= 20:
                break
        sb = sum(map(len, runs))
        r["cpu_baseline"] = {"value": round(sb / (el / reps) / 1e9, 4), "unit": "GB/s (input)", "cores": 1,
                             "kind": "port",
                             "sample": f"{sample_keys} keys ({sb/1e6:.0f} MB) of the same generator, "
                                       f"oracle/posdb_merge_oracle.c single thread, {reps} reps, {el:.1f} s"}
    return r


def pmc_traffic(kernel_prefix: str):
    """HBM bytes per launch of a kernel from the committed rocprofv3 PMC passes
    (profiles/*pmc_traffic.json, newest), corrected per MI355X_MICROARCH.md."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc_traffic.json")))
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
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--docs-per-gpu", type=int, default=100_000_000)
    ap.add_argument("--docs-to-get", type=int, default=100)
    ap.add_argument("--slots", type=int, default=2, help="queries in flight per GPU (query slots)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-merge", action="store_true", help="skip the config-5 list merge measurement")
    ap.add_argument("--no-config3", action="store_true", help="skip the config-3 query-mix measurement")
    ap.add_argument("--merge-keys", type=int, default=400_000_000, help="config-5 keys (~4.4 GB of runs)")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: WORLD_SIZE={world} != --gpus {args.gpus}; using WORLD_SIZE")

    import torch
    import torch.distributed as dist
    import gbgpu
    from shard_merge import gather_merge
    from workload import config_two_term, generate

    torch.cuda.set_device(local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    per = args.docs_per_gpu
    total = per * world
    q = config_two_term(total, docs_to_get=args.docs_to_get)
    t0 = time.time()
    lists = generate(q, total, doc_begin=rank * per, doc_end=(rank + 1) * per, threads=16)
    log(f"[rank {rank}] generated {sum(map(len, lists))/1e6:.1f} MB of lists in {time.time()-t0:.1f}s")

    eng = gbgpu.Engine(local_rank)
    handles = [eng.upload(l) for l in lists]
    list_bytes = sum(len(l) for l in lists)
    p = q.params()
    k = p.docs_to_get

    slots = max(1, args.slots)
    eng.set_slots(slots)

    def finish(r):
        """Msg39Reply -> Msg3a: per-shard top lists all-gathered over RCCL and
        merged (shard_merge.py); returns (total hits, merged docids)."""
        if world == 1:
            return r.hits, r.docids[:k]
        hits, d, _ = gather_merge(r.docids, r.scores, r.hits, k, device="cuda")
        return hits, d

    def run(nq):
        """nq queries with `slots` of them in flight (round-robin over the
        slots: a slot's previous query is collected before it is reused)."""
        hits, top = 0, None
        for i in range(nq):
            slot = i % slots
            if i >= slots:
                hits, top = finish(eng.collect(cap=4096, slot=slot))
            eng.enqueue(q.terms, handles, p, slot=slot)
        for i in range(max(0, nq - slots), nq):
            hits, top = finish(eng.collect(cap=4096, slot=i % slots))
        return hits, top

    run(args.warmup * slots)
    # per-phase device times and the probe roofline: queries one at a time
    # (untimed; concurrent queries would overlap each other's events)
    eng.set_profiling(True)
    phase_ms = []
    for _ in range(max(5, args.steps // 2)):
        eng.enqueue(q.terms, handles, p, slot=0)
        finish(eng.collect(cap=4096, slot=0))
        ms, scan_bytes = eng.last_timings(slot=0)
        phase_ms.append(ms)
    eng.set_profiling(False)
    probe_ms = [m[2] for m in phase_ms]
    total_dev_ms = [m[0] for m in phase_ms]

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    hits, top = run(args.steps)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
        lb = torch.tensor([list_bytes], dtype=torch.float64, device="cuda")
        dist.all_reduce(lb)
        agg_list_bytes = float(lb.item())
    else:
        agg_list_bytes = float(list_bytes)

    ms_per_step = el * 1000.0 / args.steps
    qps = args.steps / el
    gbs = agg_list_bytes * qps / 1e9
    # dominant kernel: k_probe, algorithmic bytes = bytes of the lists it scans
    probe_bytes = float(list_bytes - len(lists[1]) if len(lists[1]) else list_bytes)
    _, scan_bytes = eng.last_timings()
    avg_probe_ms = float(np.mean(probe_ms))
    achieved = probe_bytes / (avg_probe_ms / 1000.0) / 1e9 if avg_probe_ms > 0 else 0.0
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
        "device_ms_per_query": round(float(np.mean(total_dev_ms)), 4),
        "phase_ms": dict(zip(["total", "candidates", "probe", "compact", "score", "topk"],
                             [round(float(x), 4) for x in np.mean(np.array(phase_ms), axis=0)])),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic Zipfian posdb lists (SURVEY.md §8(d) generator), resident in HBM",
        "config": {
            "workload": "config 2: 2-term AND (+bigram sublist), top-100, 100M docs per GPU, docid-range shards",
            "docs_per_gpu": per,
            "docs_total": total,
            "list_bytes_per_gpu": list_bytes,
            "hits": int(hits),
            "pct_hbm_peak_keys_scanned": round(100.0 * gbs / (HBM_PEAK_GBS * world), 2),
        },
        "roofline": {
            "bound": "hbm",
            "kernel": "k_probe",
            "achieved": round(achieved, 2),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "traffic_source": traffic_src,
            "algorithmic_bytes_per_launch": int(probe_bytes),
        },
    }
    if rank == 0 and world == 1:
        # the C-ABI's host-buffer entry (gbgpu_query: lists in pageable host
        # memory, uploaded per call) -- PCIe-inclusive, reported beside `value`
        n_pc = 10
        host = eng.host_lists(lists)
        eng.query(q.terms, host, p)
        t_pc = time.perf_counter()
        for _ in range(n_pc):
            r_pc = eng.query(q.terms, host, p)
        el_pc = time.perf_counter() - t_pc
        if r_pc.hits != hits:
            raise RuntimeError(f"host-buffer query hits {r_pc.hits} != resident {hits}")
        result["pcie_inclusive"] = {
            "queries_per_sec": round(n_pc / el_pc, 3),
            "keys_scanned_GBps": round(list_bytes * n_pc / el_pc / 1e9, 3),
            "note": "gbgpu_query with the lists in pageable host memory, uploaded every call; not `value`",
        }
    if rank == 0 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(q, per if world == 1 else total)
    for h in handles:
        eng.free(h)
    if rank == 0 and world == 1 and not args.no_config3:
        result["config3"] = bench_config3(eng, per, max(args.steps, 50), slots)
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
