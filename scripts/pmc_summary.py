#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes (separate FETCH_SIZE and WRITE_SIZE runs of
the same bench command) into profiles/pmc_traffic.json.  The launches kept are
those between the first k_mark_begin / k_mark_end pair (bench.py's C2 timed
steps).

Per MI355X_MICROARCH.md §HBM: FETCH_SIZE/WRITE_SIZE are in KiB; on gfx950
FETCH_SIZE reports half of the bytes of a wide coalesced streaming read, so the
read side is doubled ("fetch_bytes_x2"); the raw value is kept too.  Only the
last STEPS launches of each kernel are summarised (the timed steps)."""
import csv
import json
import sys
from collections import defaultdict

KERNELS = {"p1_hist": "k_hist_rep<false>", "p1_scatter": "k_p1_scatter", "p2_hist": "k_hist_bytes", "p2_scatter": "k_p2_scatter",
           "bucket_triage": "k_bucket<false, false>", "bucket_spill": "k_bucket_direct<false>",
           "triage_claim": "k_claim<true>", "triage_resolve": "k_resolve<true>", "count_missing": "k_count_missing",
           "emit_scatter": "k_scatter("}


def load(path, counter):
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter]
    marks = {n: sorted(int(r["Dispatch_Id"]) for r in rows if n in r["Kernel_Name"]) for n in ("k_mark_begin",
                                                                                                 "k_mark_end")}
    lo = marks["k_mark_begin"][0] if marks["k_mark_begin"] else -1
    hi = marks["k_mark_end"][0] if marks["k_mark_end"] else 1 << 62
    out = defaultdict(list)
    for r in rows:
        d = int(r.get("Dispatch_Id", 0))
        if not lo < d < hi:
            continue
        for key, pat in KERNELS.items():
            if pat in r["Kernel_Name"]:
                out[key].append((d, float(r["Counter_Value"]) * 1024.0))
    return {k: [(0, v) for _, v in sorted(x)] for k, x in out.items()}


def main(fetch_csv, write_csv, out_json, tag, steps="2"):
    steps = int(steps)
    f, w = load(fetch_csv, "FETCH_SIZE"), load(write_csv, "WRITE_SIZE")
    res = {"tag": tag, "source": [fetch_csv, write_csv],
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes of the same command; "
                     "KiB -> bytes; read side doubled per the gfx950 FETCH_SIZE note (exact for wide streaming reads, "
                     "uncalibrated for the random 4-B probes)", "kernels": {}}
    for k in sorted(set(f) | set(w)):
        fl = f.get(k, [])
        wl = w.get(k, [])
        if not fl or not wl:
            continue
        fb = [x[1] for x in fl]  # the timed steps' launches
        wb = [x[1] for x in wl]
        fetch = sum(fb) / len(fb)
        write = sum(wb) / len(wb)
        res["kernels"][k] = {"launches": len(fb), "fetch_bytes_raw": fetch, "fetch_bytes_x2": 2 * fetch,
                             "write_bytes": write, "hbm_bytes_per_launch": 2 * fetch + write}
    json.dump(res, open(out_json, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:6])
