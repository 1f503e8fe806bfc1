#!/usr/bin/env python3
"""Timed-step launches of the triage kernels from a rocprofv3 --kernel-trace
CSV: the launches between the REGION-th k_mark_begin / k_mark_end pair
(bench.py brackets each timed region with sg_ctx_marker; in run order region
0 = C2, 1 = C2 with the ordered outputs, 2 = C2 from traces, 3 = the steady
state), their durations and launch
resources.
usage: trace_summary.py KERNEL_TRACE_CSV COMMAND OUT_JSON [REGION]"""
import csv
import json
import sys
from collections import defaultdict

KERNELS = ["k_hist_rep<false>", "k_hist_trace", "k_p1_scatter<false", "k_hist_bytes", "k_p2_scatter", "k_bucket<false, 0>",
           "k_bucket_direct<false>", "k_bucket_groups", "k_chunk_desc", "k_cuts", "k_scan32_reduce", "k_scan32_apply",
           "k_set_copy"]


def short(name):
    return name.split("(")[0].replace("void ", "").replace("sg::", "")


def region(rows, which):
    """(first, last) dispatch ids of the which-th marked region"""
    b = sorted(int(r["Dispatch_Id"]) for r in rows if short(r["Kernel_Name"]) == "k_mark_begin")
    e = sorted(int(r["Dispatch_Id"]) for r in rows if short(r["Kernel_Name"]) == "k_mark_end")
    return b[which], e[which]


def main(path, command, out, which="0"):
    rows = list(csv.DictReader(open(path)))
    lo, hi = region(rows, int(which))
    sel = defaultdict(list)
    t0, t1 = None, None
    for r in rows:
        d = int(r["Dispatch_Id"])
        if lo < d < hi:
            sel[short(r["Kernel_Name"])].append(r)
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            t0 = s if t0 is None else min(t0, s)
            t1 = e if t1 is None else max(t1, e)
    res = {"command": command, "region": int(which),
           "note": "launches between the region's k_mark_begin / k_mark_end (bench.py's timed steps); microseconds",
           "region_span_us": (t1 - t0) / 1000.0 if t0 is not None else None, "kernels": {}}
    for k in sorted(sel, key=lambda k: -sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in sel[k])):
        rs = sel[k]
        us = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0 for r in rs]
        r0 = rs[-1]
        res["kernels"][k] = {"launches": len(us), "avg_us": round(sum(us) / len(us), 2),
                             "total_us": round(sum(us), 1),
                             "vgpr": r0.get("Arch_VGPR_Count", r0.get("VGPR_Count")),
                             "lds_bytes": r0.get("LDS_Block_Size", r0.get("Lds_Size")),
                             "grid_threads": r0.get("Grid_Size"), "block": r0.get("Workgroup_Size")}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: (v["launches"], v["avg_us"]) for k, v in res["kernels"].items()}))


if __name__ == "__main__":
    main(*sys.argv[1:5])
