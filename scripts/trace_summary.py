#!/usr/bin/env python3
"""Timed-step launches of the triage kernels from a rocprofv3 --kernel-trace
CSV: the last STEPS launches of each kernel (the bench's timed steps come last
in its launch order), their durations, and the launch resources.
usage: trace_summary.py KERNEL_TRACE_CSV STEPS COMMAND OUT_JSON"""
import csv
import json
import sys
from collections import defaultdict

KERNELS = ["k_hist_rep<false>", "k_p1_scatter<false>", "k_hist_rep<true>", "k_p2_scatter", "k_bucket<false>",
           "k_bucket_direct", "k_bucket_groups", "k_chunk_desc", "k_cuts"]


def short(name):
    return name.split("(")[0].replace("void ", "").replace("sg::", "")


def main(path, steps, command, out):
    steps = int(steps)
    rows = defaultdict(list)
    for r in csv.DictReader(open(path)):
        k = short(r["Kernel_Name"])
        if k in KERNELS:
            rows[k].append(r)
    res = {"command": command,
           "note": f"timed-step launches = the last {steps} launches of each kernel; durations in microseconds",
           "kernels": {}}
    for k in KERNELS:
        rs = sorted(rows.get(k, []), key=lambda r: int(r.get("Dispatch_Id", 0)))[-steps:]
        if not rs:
            continue
        us = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0 for r in rs]
        r0 = rs[-1]
        res["kernels"][k] = {"timed_launch_us": [round(u, 1) for u in us], "avg_us": round(sum(us) / len(us), 1),
                             "vgpr": r0.get("Arch_VGPR_Count", r0.get("VGPR_Count")),
                             "lds_bytes": r0.get("LDS_Block_Size", r0.get("Lds_Size")),
                             "grid_threads": r0.get("Grid_Size"), "block": r0.get("Workgroup_Size")}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: v["avg_us"] for k, v in res["kernels"].items()}))


if __name__ == "__main__":
    main(*sys.argv[1:5])
