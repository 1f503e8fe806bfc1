#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes (separate FETCH_SIZE and WRITE_SIZE runs of
the same bench command) into profiles/pmc_traffic.json, one section per timed
workload.  bench.py brackets each timed region with k_mark_begin / k_mark_end
(in run order: the C2 steps, the from-traces steps, the steady-state steps);
the i-th bracket's launches are summarised under the i-th name of `workloads`.

Per MI355X_MICROARCH.md §HBM: FETCH_SIZE/WRITE_SIZE are in KiB; on gfx950
FETCH_SIZE reports half of the bytes of a wide coalesced streaming read, so the
read side is doubled ("fetch_bytes_x2"); the raw value is kept too.

usage: pmc_summary.py FETCH.csv WRITE.csv OUT.json TAG [workloads=c2,from_traces,steady] [merge] [steps=2]
("merge": keep OUT.json's other workload sections; each section records its
own tag and sources)"""
import csv
import json
import sys
from collections import defaultdict

KERNELS = {"p1_hist": ("k_hist_rep<false>", "k_hist_trace", "k_p1_hist"), "p1_scatter": ("k_p1_scatter",),
           "p2_hist": ("k_hist_bytes",), "p2_scatter": ("k_p2_scatter",),
           "bucket_triage": ("k_bucket<false, 0>", "k_bucket<false, 1>", "k_bucket<false, 2>"),
           "bucket_spill": ("k_bucket_direct<false>",),
           "count_missing": ("k_count_missing",), "emit_scatter": ("k_scatter(",),
           "bucket_mark": ("k_bucket_mark",), "prefix_or": ("k_prefix_or",), "prefix_flags": ("k_prefix_flags",),
           "prefix_merge": ("k_prefix_merge",), "set_or": ("k_set_or(",), "set_or_new": ("k_set_or_new(",), "set_or_new_or": ("k_set_or_new_or",),
           "m0_index": ("k_m0_index",), "m0_filter": ("k_m0_filter",), "m0_tail": ("k_m0_tail_insert", "k_m0_tail_flush")}


def load(path, counter, nregions):
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter]
    marks = {n: sorted(int(r["Dispatch_Id"]) for r in rows if n in r["Kernel_Name"])
             for n in ("k_mark_begin", "k_mark_end")}
    regions = list(zip(marks["k_mark_begin"], marks["k_mark_end"]))[:nregions]
    out = [defaultdict(list) for _ in regions]
    for r in rows:
        d = int(r.get("Dispatch_Id", 0))
        for i, (lo, hi) in enumerate(regions):
            if not lo < d < hi:
                continue
            for key, pats in KERNELS.items():
                if any(p in r["Kernel_Name"] for p in pats):
                    out[i][key].append(float(r["Counter_Value"]) * 1024.0)
    return out


def main(fetch_csv, write_csv, out_json, tag, workloads="c2,from_traces,steady", merge="", steps="2"):
    names = workloads.split(",")
    steps = int(steps)  # timed steps per region (the PMC passes run bench.py --steps 2)
    old = {}
    if merge == "merge":
        try:
            old = json.load(open(out_json))
        except (OSError, ValueError):
            old = {}
    f, w = load(fetch_csv, "FETCH_SIZE", len(names)), load(write_csv, "WRITE_SIZE", len(names))
    res = {"tag": tag, "source": [fetch_csv, write_csv],
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes of the same command; "
                     "KiB -> bytes; read side doubled per the gfx950 FETCH_SIZE note (exact for wide streaming reads, "
                     "uncalibrated for the random 4-B probes); each workload from its own timed launches "
                     "(bench.py's k_mark_begin / k_mark_end brackets, in run order)", "workloads": {}}
    for i, name in enumerate(names):
        if i >= len(f) or i >= len(w):
            break
        sec = {}
        for k in sorted(set(f[i]) | set(w[i])):
            fb, wb = f[i].get(k, []), w[i].get(k, [])
            if not fb or not wb:
                continue
            fetch, write = sum(fb) / len(fb), sum(wb) / len(wb)
            sec[k] = {"launches": len(fb), "launches_per_step": len(fb) / steps, "fetch_bytes_raw": fetch,
                      "fetch_bytes_x2": 2 * fetch, "write_bytes": write, "hbm_bytes_per_launch": 2 * fetch + write}
        res["workloads"][name] = {"kernels": sec, "tag": tag, "source": [fetch_csv, write_csv], "steps": steps}
    if old:
        for name, sec in old.get("workloads", {}).items():
            if name not in res["workloads"]:
                sec.setdefault("tag", old.get("tag"))
                res["workloads"][name] = sec
    json.dump(res, open(out_json, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:8])
