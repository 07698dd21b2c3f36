#!/bin/bash
# A/B of library builds on one GPU box (run from the repo root on the box):
#   tools/ab_libs.sh ROUNDS lib1.so lib2.so ... [-- extra bench.py args]
# Runs bench.py (no CPU baseline, no secondary timings) once per library per round,
# interleaved (A B C A B C ...) so clock drift hits every build alike, and prints one line
# per run: library, IC iterations/s, level-0 launch us (HIP events).  Every run has its own
# time limit; the script stops at the first failure.
set -e
rounds=${1:?rounds}; shift
libs=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do libs+=("$1"); shift; done
[ "$1" = "--" ] && shift
mkdir -p gpurun_out
for r in $(seq "$rounds"); do
  for lib in "${libs[@]}"; do
    out=gpurun_out/ab_$(basename "$lib" .so)_$r.json
    DPFT_LIB="$lib" timeout -k 10 150 python bench.py --no-cpu-baseline --no-compare "$@" > "$out.log" 2>&1
    tail -n 1 "$out.log" > "$out"
    python - "$lib" "$out" <<'EOF'
import json, sys
d = json.load(open(sys.argv[2]))
r = d.get("roofline", {})
print(f"{sys.argv[1]:40s} {d['value']:10.1f}  L0 {r.get('kernel_us', 0):8.1f} us  frac {r.get('frac', 0):.4f}", flush=True)
EOF
  done
done
