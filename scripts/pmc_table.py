#!/usr/bin/env python3
"""Per-kernel PMC table from rocprofv3 --pmc runs: for each kernel name, the
counters of its full-size launches (largest grid), averaged per launch.
usage: pmc_table.py DIR [DIR ...]"""
import csv
import sys
from collections import defaultdict


def load(d):
    import glob
    out = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [(grid, value)]
    for path in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(path)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("sg::", "")
            out[k][r["Counter_Name"]].append((int(r["Grid_Size"]), float(r["Counter_Value"])))
    return out


def main():
    tab = defaultdict(dict)
    for d in sys.argv[1:]:
        for k, cs in load(d).items():
            for c, vals in cs.items():
                g = max(v[0] for v in vals)
                full = [v[1] for v in vals if v[0] == g]
                tab[k][c] = sum(full) / len(full)
    for k in sorted(tab):
        print(k)
        for c, v in sorted(tab[k].items()):
            print(f"   {c:28s} {v:16.4g}")


if __name__ == "__main__":
    main()
