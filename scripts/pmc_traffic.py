"""Per-kernel HBM bytes per launch from two rocprofv3 --pmc passes (FETCH_SIZE,
WRITE_SIZE, in KiB) of the config-2 bench, written as the JSON bench.py reads
(profiles/rNN_*pmc_traffic.json).  Correction (MI355X_MICROARCH.md, HBM
section): on gfx950 FETCH_SIZE reports half the bytes of wide coalesced
streaming reads (16 B/lane), so it is doubled for the kernels whose list
reads are 16-B lane loads (WIDE) and taken as is for the others (their loads
are 2-8 B); WRITE_SIZE is taken as is.

  python3 scripts/pmc_traffic.py FETCH_CSV WRITE_CSV OUT_JSON [note]"""
import collections
import csv
import json
import sys


# kernels whose HBM reads are 16-B lane loads (v4 chunk / window loads)
WIDE = {"k_probe", "k_write_runs", "k_page_count", "k_validate", "k_list_scan", "k_stream_read", "k_stream_copy"}


def is_wide(k):
    return k.split("<")[0] in WIDE


def per_kernel(path, counter):
    tot = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("gbgpu::", "")
        tot[k] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    return {k: (tot[k] / len(disp[k]), len(disp[k])) for k in tot}


def main():
    fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
    write = per_kernel(sys.argv[2], "WRITE_SIZE")
    out = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes, config-2 bench (16-query rotation)",
           "correction": "FETCH_SIZE x 1024 x 2 for 16-B lane readers (gfx950 wide-read halving: " + ", ".join(sorted(WIDE))
                         + "), x 1024 for the others; + WRITE_SIZE x 1024",
           "note": sys.argv[4] if len(sys.argv) > 4 else "", "kernels": {}}
    for k in sorted(set(fetch) | set(write)):
        f, nf = fetch.get(k, (0.0, 0))
        w, nw = write.get(k, (0.0, 0))
        out["kernels"][k] = {"fetch_kib_per_launch": round(f, 1), "write_kib_per_launch": round(w, 1),
                             "launches": max(nf, nw),
                             "fetch_doubled": is_wide(k),
                             "hbm_bytes_per_launch_corrected": int(f * 1024 * (2 if is_wide(k) else 1) + w * 1024)}
    json.dump(out, open(sys.argv[3], "w"), indent=1)
    for k, v in sorted(out["kernels"].items(), key=lambda kv: -kv[1]["hbm_bytes_per_launch_corrected"])[:12]:
        print(f"{k:40s} {v['hbm_bytes_per_launch_corrected'] / 1e6:10.1f} MB/launch  ({v['launches']} launches)")


if __name__ == "__main__":
    main()
