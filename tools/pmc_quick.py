#!/usr/bin/env python
"""Average every counter per (kernel, grid) over the pmc CSVs under a directory tree."""
import collections, csv, glob, sys

acc = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:60]
        grid = int(r["Grid_Size"]) // max(int(r["Workgroup_Size"]), 1)
        acc[(k, grid, r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, g, c), v in sorted(acc.items()):
    if "reduce" in k or "pack" in k:
        print(f"{k:60s} grid={g:6d} {c:28s} {sum(v) / len(v):14.1f}  (n={len(v)})")
