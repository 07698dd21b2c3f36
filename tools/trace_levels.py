"""Per-solve timeline of a bench.py kernel trace: one row per launch of the last full solve.

python tools/trace_levels.py gpurun_out/prof/bench_kernel_trace.csv ["true>" | "false>"]
"""
import csv
import re
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
names = [r["Kernel_Name"] for r in rows]
# a solve starts with the sigma0 extrema pass of level 3 (the smallest grid) and ends before the next
starts = [i for i, r in enumerate(rows) if "minmax" in r["Kernel_Name"] and int(r["Grid_Size_X"]) // 256 <= 16]
want = sys.argv[2] if len(sys.argv) > 2 else "true>"  # c4 solves: ic_reduce_kernel<..., true>
solves = [(a, b) for a, b in zip(starts, starts[1:])
          if any(("ic_reduce" in rows[j]["Kernel_Name"] or "march" in rows[j]["Kernel_Name"])
                 and re.search(r"kernel<([^>]*)>", rows[j]["Kernel_Name"]).group(0).endswith(want)
                 for j in range(a, b))]
i0, i1 = solves[-2]
t0 = int(rows[i0]["Start_Timestamp"])
tot = 0.0
for r in rows[i0:i1]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot += d
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
    print(f"{(int(r['Start_Timestamp']) - t0) / 1e3:9.1f} us  {d:7.1f} us  wg={int(r['Grid_Size_X']) // 256:5d}  {n[:60]}")
end = int(rows[i1 - 1]["End_Timestamp"])
print(f"solve wall {(end - t0) / 1e3:.1f} us, kernel sum {tot:.1f} us")
