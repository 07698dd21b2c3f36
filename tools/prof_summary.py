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


def is_c4(name):
    """ic_reduce_kernel<CT, CS1, TRU, MODE, C4[, FOLD]>: the channel-quad layout's instances"""
    m = re.match(r"ic_reduce_kernel<([^>]*)>", name)
    return bool(m) and m.group(1).split(", ")[4] == "true"


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
    # combine_ICP: the normal-map launch's grid names its level -- the first solve launches
    # them level 3 .. 0 in order (the grids are distinct per level, but since round 5 they
    # are not ordered by level size: the kernel's rows per wave adapt to the level)
    nrm_grids = []
    for r in sorted(rows, key=lambda r: int(r["Start_Timestamp"])):
        g = int(r["Grid_Size_X"])
        if "icp_normals" in r["Kernel_Name"] and g not in nrm_grids:
            nrm_grids.append(g)
    nrm_grids.reverse()  # index = level
    top = 3  # coarsest level of the 4-level bench pyramid
    ITERS = 3
    # bench.py --inflight S replays S graphs on S side streams in the timed region; the
    # default stream (the lowest Stream_Id) carries the solo launches: eager warm-ups, the
    # latency loop (graph replays, nothing else in flight) and the roofline's level-0 group.
    # Level bookkeeping is per stream.
    streams = sorted({int(r.get("Stream_Id", 0) or 0) for r in rows})
    solo_stream = streams[0]
    # packed: the solve packs NCHW features to channel quads on entry (pack_c4 kernels: bench.py's
    # other_layout leg); its channel-quad launches are listed apart from the headline's
    state = collections.defaultdict(lambda: {"level": None, "n_red": None, "cur": [], "solves": [], "packed": False})
    groups = collections.defaultdict(list)
    for r in rows:
        sid = int(r.get("Stream_Id", 0) or 0)
        st = state[sid]
        name = short(r["Kernel_Name"])
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        if name.startswith("minmax_levels") and not nrm_grids:
            # one sigma0 pre-pass for all levels opens a solve; levels then advance every
            # ITERS reduce launches (extra level-0 launches after the solve stay level 0)
            st["level"], st["n_red"], st["packed"] = top, 0, False
            if st["cur"]:
                st["solves"].append(st["cur"])
                st["cur"] = []
        elif nrm_grids and name.startswith("icp_normals"):
            # combine_ICP: each level opens with frame 1's normal map (its grid gives the
            # level: the largest is level 0); its depth1 extrema pass (a minmax_levels_kernel
            # per level) and the sigma0 pre-pass leave the level alone
            st["level"] = nrm_grids.index(int(r["Grid_Size_X"]))
            st["n_red"] = None
            if st["level"] == top:
                st["packed"] = False
            if st["level"] == top and st["cur"]:
                st["solves"].append(st["cur"])
                st["cur"] = []
        elif nrm_grids and "minmax" in name:
            pass
        elif "minmax" in name:
            # per-level sigma0 pass (older traces / solves without the pre-pass): the
            # smallest opens level 3, each later one the next finer level
            if int(r["Grid_Size_X"]) == mm_grids[0]:
                st["level"] = top
            else:
                st["level"] = max((st["level"] if st["level"] is not None else top) - 1, 0)
            st["n_red"] = None
            if st["level"] == top and st["cur"]:
                st["solves"].append(st["cur"])
                st["cur"] = []
        elif st["n_red"] is not None and st["level"] is not None and name.startswith(("ic_reduce", "ic_split")):
            st["level"] = max(top - st["n_red"] // ITERS, 0)
            st["n_red"] += 1
        if name.startswith(("pack_c4_x4", "pack_c4_pair")):  # (pack_c4_kernel: the bench's own input packing)
            st["packed"] = True
        level = st["level"]
        if level is None:
            continue
        layout = ("nchw packed on entry" if st["packed"] else "c4") if (is_c4(name) or not name.startswith("ic_reduce")) \
            else "nchw"
        mode = "solo" if sid == solo_stream else "side streams"
        if name.startswith(("ic_reduce", "ic_split", "finalize", "minmax", "icp_normals", "icp_records")):
            groups[(mode, layout if not name.startswith(("finalize", "minmax", "icp_normals", "icp_records")) else "-",
                    level, name)].append(dur)
        st["cur"].append((int(r["Start_Timestamp"]), dur, level, name,
                          int(r["Grid_Size_X"]) // max(int(r["Workgroup_Size_X"]), 1)))
    for st in state.values():
        if st["cur"]:
            st["solves"].append(st["cur"])
    # one channel-quad solve with nothing else in flight: the last solo one
    solves = state[solo_stream]["solves"]
    c4 = [s for s in solves if any(is_c4(n) or n.startswith("ic_split") for _, _, _, n, _ in s)
          and not any(n.startswith(("pack_c4_x4", "pack_c4_pair")) for _, _, _, n, _ in s)]
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
             "solo = default stream, nothing else in flight (warm-ups, latency loop, the roofline's level-0 "
             "group); side streams = the timed region's graph replays, in flight together (launches overlap), plus "
             "each slot's one eager pre-capture solve\n",
             "| mode | layout | level | kernel | launches | avg us | min us | max us |",
             "|---|---|---|---|---|---|---|---|"]
    for (mode, layout, lv, name), d in sorted(groups.items(), key=lambda kv: (kv[0][0] != "solo", kv[0][1], -kv[0][2], kv[0][3])):
        lines.append(f"| {mode} | {layout} | {lv} | {name} | {len(d)} | {sum(d) / len(d):.1f} | {min(d):.1f} | {max(d):.1f} |")
        out["levels"][f"{mode}/{layout}/L{lv}/{name}"] = {"launches": len(d), "avg_us": sum(d) / len(d),
                                                          "min_us": min(d), "max_us": max(d)}
    if one:
        t0 = one[0][0]
        lines += ["", "## One channel-quad solve (all pairs of one launch, graph replay, nothing else in flight)\n",
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
        # algorithmic bytes per level-0 launch: 640 x 480 px x 272 B (280 with combine_ICP) per pair
        alg = 640 * 480 * (280 if t.get("combine_icp") else 272) * t.get("pairs_per_launch", 8)
        lines += ["", "## Level-0 reduce launch: HBM traffic (separate FETCH_SIZE / WRITE_SIZE passes)\n",
                  f"read {t['read_bytes'] / 1e6:.1f} MB + write {t['write_bytes'] / 1e6:.2f} MB per launch "
                  f"({t['correction']}); algorithmic {alg / 1e6:.1f} MB "
                  f"({t.get('pairs_per_launch', 8)} pairs) -> {t['hbm_bytes'] / alg:.3f}x"]
    open(a.out + ".md", "w").write("\n".join(lines) + "\n")
    json.dump(out, open(a.out + ".json", "w"), indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
