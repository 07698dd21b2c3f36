#!/usr/bin/env python
"""HBM traffic of the level-0 reduce launch from rocprofv3 PMC passes (run on the GPU box).

    python tools/pmc_l0.py --out profiles/r1_l0_traffic.json

Runs tools/kbench.py (level 0, channel-quad, `level --from-solve` = the forward / reverse /
forward launch group bench.py times, from the solved poses)
under two separate `rocprofv3 --pmc` passes (FETCH_SIZE; WRITE_SIZE) and writes the
per-launch bytes, corrected as MI355X_MICROARCH.md's HBM section prescribes:
FETCH_SIZE counts half the bytes of a 128-B-request stream on gfx950 (TCC_EA0_RDREQ
x 64 B) -> read bytes = 2 x 1024 x FETCH_SIZE; WRITE_SIZE (KiB) is exact.  The
JSON carries the SHA-256 of the measured kernel's machine code (and of the source file),
so bench.py uses it only while that kernel's code is unchanged.
"""
import argparse
import csv
import glob
import hashlib
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "deep_prob_feature_track_amd", "csrc", "dpft_ic.hip")


LEVEL0_LAUNCHES = 1 + 3 * 10  # kbench --mode level --reps 10


def src_sha():
    return hashlib.sha256(open(SRC, "rb").read()).hexdigest()


def isa_sha(kernel=None):
    """Hash of the measured kernel's machine code (deep_prob_feature_track_amd/build.py)."""
    sys.path.insert(0, ROOT)
    from deep_prob_feature_track_amd import build as B
    lib = os.environ.get("DPFT_LIB")
    return (B.isa_hashes(os.path.abspath(lib)) if lib else json.load(open(B.ISA_OUT))).get(kernel or B.L0_KERNEL)


MODE = {"mode": "level", "load_poses": None}  # --mode reduce: the records-only launches (tools/mk_loads_variant.py)


def run_pass(counter, outdir, groups, icp=False, level=0):
    start = ["--load-poses", os.path.abspath(MODE["load_poses"])] if MODE["load_poses"] else ["--from-solve"]
    cmd = ["timeout", "-s", "KILL", "90", "rocprofv3", "--pmc", counter, "--output-format", "csv", "-d", outdir,
           "-o", "c", "--", sys.executable, os.path.join(ROOT, "tools", "kbench.py"), "--c4", "--level", str(level),
           "--mode", MODE["mode"], *start, "--reps", "10", "--warm-ms", "0", "--groups", str(groups)] + (["--icp"] if icp else [])
    env = dict(os.environ, TMPDIR="/tmp")
    if env.get("DPFT_LIB"):  # a variant library (tools/build_variants.py); the profiler runs from /tmp
        env["DPFT_LIB"] = os.path.abspath(env["DPFT_LIB"])
    subprocess.run(cmd, check=True, cwd="/tmp", env=env)
    return parse(counter, outdir)


def parse(counter, outdir):
    rows, icp_rows = [], []
    for f in glob.glob(os.path.join(outdir, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            if "ic_reduce_kernel" in r["Kernel_Name"]:
                rows.append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
            elif "icp_records_kernel" in r["Kernel_Name"]:  # combine_ICP's own pass, one per reduce launch
                icp_rows.append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    # the last LEVEL0_LAUNCHES are kbench's level-0 launches (its first iteration + reps x 3);
    # before them, its --from-solve pyramid solve (marching launches per level depend on
    # the batch size: levels 1 and 0 at 8 pairs, every level at 128)
    n_last = 10 if MODE["mode"] == "reduce" else LEVEL0_LAUNCHES  # reduce: the 10 records-only launches
    vals = [v for _, v in sorted(rows)[-n_last:]]
    if not vals:
        raise SystemExit(f"no ic_reduce_kernel rows for {counter}")
    if icp_rows:  # a level-0 iteration is the ICP pass + the reduce launch: their bytes together
        ivals = [v for _, v in sorted(icp_rows)[-LEVEL0_LAUNCHES:]]
        vals = [a + b for a, b in zip(vals, ivals)]
    return sum(vals) / len(vals), len(vals)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--groups", type=int, default=16, help="8-pair batches per launch (bench.py --groups)")
    ap.add_argument("--icp", action="store_true", help="the combine_ICP kernel (bench.py --icp)")
    ap.add_argument("--level", type=int, default=0, help="pyramid level of the measured launches (traffic "
                    "of the coarser levels; only level 0 is matched by bench.py)")
    ap.add_argument("--from-dir", help="parse the fetch/ and write/ CSVs under this directory instead of running")
    ap.add_argument("--mode", choices=["level", "reduce"], default="level",
                    help="kbench mode: level (the solve's launch group, default; bench.py matches only this) or "
                         "reduce (records-only launches, for variants whose solve is not valid)")
    ap.add_argument("--load-poses", default=None, help="start poses saved by kbench --save-poses (with --mode reduce)")
    a = ap.parse_args()
    MODE.update(mode=a.mode, load_poses=a.load_poses)
    tmp = os.path.join(ROOT, "gpurun_out", "pmc_l0")
    if a.from_dir:  # re-read the CSVs of an earlier run (same launch shape)
        fetch, nf = parse("FETCH_SIZE", os.path.join(a.from_dir, "fetch"))
        write, nw = parse("WRITE_SIZE", os.path.join(a.from_dir, "write"))
    else:
        fetch, nf = run_pass("FETCH_SIZE", os.path.join(tmp, "fetch"), a.groups, a.icp, a.level)
        write, nw = run_pass("WRITE_SIZE", os.path.join(tmp, "write"), a.groups, a.icp, a.level)
    sys.path.insert(0, ROOT)
    from deep_prob_feature_track_amd import build as B
    kernel = B.L0_KERNEL
    out = {"kernel": f"ic_reduce_kernel<32,Cs=1,tru,U_IC,c4>{' + icp_records_kernel' if a.icp else ''} level {a.level}, {a.groups} x 8 pairs per launch, 640x480 "
                     "(tools/kbench.py --mode level --from-solve)",
           "level": a.level, "pairs_per_launch": 8 * a.groups, "group": 8, "kbench_mode": a.mode,
           "src_sha256": src_sha(), "isa_sha256": isa_sha(kernel), "combine_icp": a.icp,
           **({"isa_sha256_icp": isa_sha(B.ICP_KERNEL)} if a.icp else {}), "launches": {"fetch": nf, "write": nw},
           "FETCH_SIZE_KiB": fetch, "WRITE_SIZE_KiB": write,
           "read_bytes": 2 * 1024 * fetch, "write_bytes": 1024 * write,
           "hbm_bytes": 2 * 1024 * fetch + 1024 * write,
           "correction": "read = 2 x 1024 x FETCH_SIZE (gfx950 tallies 128-B read requests at 64 B), "
                         "write = 1024 x WRITE_SIZE"}
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
