#!/usr/bin/env python
"""Summarise rocprofv3 CSV output per (kernel, grid) and derive per-launch HBM traffic.

usage: python tools/prof_summary.py --trace DIR/x_kernel_trace.csv \
           [--fetch DIR/fetch_counter_collection.csv] [--write ...] [--hit ...] \
           --out profiles/r1_summary  (writes .md and .json)

rocprofv3 --stats averages a kernel over every launch of that symbol, and the solver
launches the same `ic_reduce_kernel<32,true,true>` instantiation at all four pyramid
levels; the per-grid split below separates level 0 (the roofline kernel) from the rest.
FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE counts half the bytes of a
coalesced read (MI355X_MICROARCH.md, HBM section) -- we calibrated the same factor on
minmax_kernel, a plain 4 B/lane streaming read of a known byte count -- so HBM read
bytes = 2 * 1024 * FETCH_SIZE.
"""
import argparse
import collections
import csv
import json


def short(name):
    n = name.replace("(anonymous namespace)::", "")
    return n.split("(")[0] if not n.startswith("void ") else n[5:].split("(")[0]


def trace_groups(path):
    g = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        grid = int(r.get("Grid_Size_X") or r.get("Grid_Size"))
        wg = int(r.get("Workgroup_Size_X") or r.get("Workgroup_Size"))
        g[(short(r["Kernel_Name"]), grid // max(wg, 1))].append(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return g


def counter_groups(path):
    g = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        grid = int(r["Grid_Size"]) // max(int(r["Workgroup_Size"]), 1)
        g[(short(r["Kernel_Name"]), grid, r["Counter_Name"])].append(float(r["Counter_Value"]))
    return g


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace", required=True)
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--hit")
    ap.add_argument("--out", required=True)
    ap.add_argument("--title", default="")
    a = ap.parse_args()
    tg = trace_groups(a.trace)
    cg = collections.defaultdict(list)
    for p in (a.fetch, a.write, a.hit):
        if p:
            for k, v in counter_groups(p).items():
                cg[k] += v
    rows = []
    for (k, blocks), d in sorted(tg.items(), key=lambda kv: -sum(kv[1])):
        row = {"kernel": k, "workgroups": blocks, "calls": len(d), "avg_us": sum(d) / len(d),
               "min_us": min(d), "max_us": max(d), "total_us": sum(d)}
        def mean(c):
            v = cg.get((k, blocks, c))
            return sum(v) / len(v) if v else None
        f, w = mean("FETCH_SIZE"), mean("WRITE_SIZE")
        h, m = mean("TCC_HIT_sum"), mean("TCC_MISS_sum")
        if f is not None:
            row["hbm_read_bytes"] = 2 * 1024 * f
        if w is not None:
            row["hbm_write_bytes"] = 1024 * w
        if h is not None and m is not None and h + m > 0:
            row["l2_hit_rate"] = h / (h + m)
        rows.append(row)
    json.dump(rows, open(a.out + ".json", "w"), indent=1)
    with open(a.out + ".md", "w") as fo:
        fo.write(f"# {a.title}\n\n" if a.title else "")
        fo.write("| kernel | workgroups | calls | avg us | min us | max us | HBM read MB/launch | HBM write MB/launch | L2 hit |\n")
        fo.write("|---|---|---|---|---|---|---|---|---|\n")
        for r in rows:
            rd = f"{r['hbm_read_bytes'] / 1e6:.1f}" if "hbm_read_bytes" in r else ""
            wr = f"{r['hbm_write_bytes'] / 1e6:.3f}" if "hbm_write_bytes" in r else ""
            hr = f"{r['l2_hit_rate']:.3f}" if "l2_hit_rate" in r else ""
            fo.write(f"| {r['kernel']} | {r['workgroups']} | {r['calls']} | {r['avg_us']:.1f} | {r['min_us']:.1f} | "
                     f"{r['max_us']:.1f} | {rd} | {wr} | {hr} |\n")
    print(open(a.out + ".md").read())


if __name__ == "__main__":
    main()
