#!/bin/bash
# FETCH_SIZE per launch of tools/mb_layout's G=4 modes (one rocprofv3 pass per mode)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for m in 0 3 4 6; do
  d=gpurun_out/mb_pmc/m$m
  timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $d -o c -- ./tools/mb_layout $m > /dev/null 2>&1 || exit 1
  python - "$d" "$m" <<'PY'
import csv, glob, sys
v = [float(r["Counter_Value"]) for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)
     for r in csv.DictReader(open(f)) if r["Counter_Name"] == "FETCH_SIZE"]
alg = 2 * 64 * 480 * 640 * 32 * 4 / (2 if sys.argv[2] == "1" else 1)
print(f"mode {sys.argv[2]}: {len(v)} launches, read {2 * 1024 * sum(v[5:]) / len(v[5:]) / 1e9:.3f} GB per launch = {2 * 1024 * sum(v[5:]) / len(v[5:]) / alg:.3f} x algorithmic")
PY
done
