#!/usr/bin/env python
"""Per-level summary of a bench.py rocprofv3 kernel trace (+ optional PMC passes).

usage: python tools/prof_summary.py --trace DIR/bench_kernel_trace.csv \
           [--traffic profiles/r1_l0_traffic.json] --out profiles/r1_summary [--title T]

Every launch is assigned to a pyramid level by the sigma0 min/max pass that opens the
level (the smallest grid opens level 3, each later pass the next finer level), and to the feature layout
(channel-quad kernels carry `true>` / are the split kernel; the NCHW comparison solve
`false>`).  Writes <out>.md and <out>.json: per (layout, level, kernel) the number of
launches and their average / min / max duration, and one solve's timeline.
"""
import argparse
import collections
import csv
import json
import re


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    m = re.match(r"([A-Za-z_0-9]+(<[^>]*>)?)", n)
    return m.group(1) if m else n[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace", required=True)
    ap.add_argument("--traffic")
    ap.add_argument("--out", required=True)
    ap.add_argument("--title", default="")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    mm_grids = sorted({int(r["Grid_Size_X"]) for r in rows if "minmax" in r["Kernel_Name"]})
    top = 3  # coarsest level of the 4-level bench pyramid
    ITERS = 3
    n_red = None
    groups = collections.defaultdict(list)
    level = None
    timeline, cur, solves = [], [], []
    for r in rows:
        name = short(r["Kernel_Name"])
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        if name.startswith("minmax_levels"):
            # one sigma0 pre-pass for all levels opens a solve; levels then advance every
            # ITERS reduce launches (extra level-0 launches after the solve stay level 0)
            level, n_red = top, 0
            if cur:
                solves.append(cur)
                cur = []
        elif "minmax" in name:
            # per-level sigma0 pass (older traces / solves without the pre-pass): the
            # smallest opens level 3, each later one the next finer level
            if int(r["Grid_Size_X"]) == mm_grids[0]:
                level = top
            else:
                level = max((level if level is not None else top) - 1, 0)
            n_red = None
            if level == top and cur:
                solves.append(cur)
                cur = []
        elif n_red is not None and level is not None and name.startswith(("ic_reduce", "ic_split")):
            level = max(top - n_red // ITERS, 0)
            n_red += 1
        if level is None:
            continue
        layout = "nchw" if name.endswith("false>") else "c4"
        if name.startswith(("ic_reduce", "ic_split", "finalize", "minmax")):
            groups[(layout if not name.startswith(("finalize", "minmax")) else "-", level, name)].append(dur)
        cur.append((int(r["Start_Timestamp"]), dur, level, name, int(r["Grid_Size_X"]) // max(int(r["Workgroup_Size_X"]), 1)))
    # one channel-quad solve: the last complete one whose reduce launches are channel-quad
    c4 = [s for s in solves if any(n.endswith("true>") or n.startswith("ic_split") for _, _, _, n, _ in s)]
    one = c4[-1] if c4 else []
    # cut after the level-0 iterations of the solve (bench.py times extra level-0 launches after it)
    n0, cut = 0, len(one)
    for i, (_, _, lv, name, _) in enumerate(one):
        if lv == 0 and name.startswith(("ic_reduce", "ic_split")):
            n0 += 1
            if n0 == 3:
                cut = i + 1
                break
    one = one[:cut]
    out = {"levels": {}, "timeline": []}
    lines = [f"# {a.title}\n" if a.title else "", "## Launches per level (all solves in the trace)\n",
             "| layout | level | kernel | launches | avg us | min us | max us |", "|---|---|---|---|---|---|---|"]
    for (layout, lv, name), d in sorted(groups.items(), key=lambda kv: (kv[0][0], -kv[0][1], kv[0][2])):
        lines.append(f"| {layout} | {lv} | {name} | {len(d)} | {sum(d) / len(d):.1f} | {min(d):.1f} | {max(d):.1f} |")
        out["levels"][f"{layout}/L{lv}/{name}"] = {"launches": len(d), "avg_us": sum(d) / len(d),
                                                   "min_us": min(d), "max_us": max(d)}
    if one:
        t0 = one[0][0]
        lines += ["", "## One channel-quad solve (B = 8 pairs, graph replay)\n",
                  "| start us | duration us | level | kernel | workgroups |", "|---|---|---|---|---|"]
        for st, d, lv, name, wg in one:
            lines.append(f"| {(st - t0) / 1e3:.1f} | {d:.1f} | {lv} | {name} | {wg} |")
            out["timeline"].append({"start_us": (st - t0) / 1e3, "us": d, "level": lv, "kernel": name, "wg": wg})
        wall = (one[-1][0] - t0) / 1e3 + one[-1][1]
        lines.append(f"\nsolve wall {wall:.1f} us, kernel sum {sum(x[1] for x in one):.1f} us")
        out["solve_wall_us"] = wall
    if a.traffic:
        t = json.load(open(a.traffic))
        out["l0_traffic"] = t
        lines += ["", "## Level-0 reduce launch: HBM traffic (separate FETCH_SIZE / WRITE_SIZE passes)\n",
                  f"read {t['read_bytes'] / 1e6:.1f} MB + write {t['write_bytes'] / 1e6:.2f} MB per launch "
                  f"({t['correction']}); algorithmic 668.5 MB -> {t['hbm_bytes'] / 668467200:.2f}x"]
    open(a.out + ".md", "w").write("\n".join(lines) + "\n")
    json.dump(out, open(a.out + ".json", "w"), indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
