#!/usr/bin/env python
"""Average PMC counters per level-0 marching launch over tools/pmc_passes.sh output.

python tools/pmc_table.py gpurun_out/pmc_r2 [--last 31]

Reads every pass directory's *counter_collection.csv, keeps the ic_reduce_kernel
dispatches in dispatch order, keeps the last --last of them (kbench --mode level
--reps 10: one first iteration + 10 x 3 level-0 launches; before them, kbench
--from-solve's own pyramid solve, whose marching launches depend on the batch size)
and prints one line per counter: the average per launch.
"""
import argparse
import collections
import csv
import glob
import json
import os

ap = argparse.ArgumentParser()
ap.add_argument("root")
ap.add_argument("--last", type=int, default=31)
ap.add_argument("--json")
a = ap.parse_args()
avg = {}
for f in sorted(glob.glob(os.path.join(a.root, "**", "*counter_collection.csv"), recursive=True)):
    per = collections.defaultdict(dict)
    for r in csv.DictReader(open(f)):
        if "ic_reduce_kernel" in r["Kernel_Name"]:
            per[r["Counter_Name"]][int(r["Dispatch_Id"])] = float(r["Counter_Value"])
    for name, d in per.items():
        v = [d[k] for k in sorted(d)][-a.last:]
        avg[name] = {"avg": sum(v) / len(v), "launches": len(v), "pass": os.path.relpath(f, a.root)}
for k in sorted(avg):
    print(f"{k:32s} {avg[k]['avg']:.4g}  ({avg[k]['launches']} launches)")
if a.json:
    json.dump(avg, open(a.json, "w"), indent=1)
