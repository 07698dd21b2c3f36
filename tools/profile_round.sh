#!/bin/bash
# Round profile set (run on the GPU box from the repo root): tools/profile_round.sh TAG [--icp]
#   gpurun_out/TAG_prof/      rocprofv3 --kernel-trace --stats of bench.py (default, or --icp)
#   gpurun_out/TAG_l0_traffic.json   FETCH_SIZE / WRITE_SIZE passes (tools/pmc_l0.py)
#   gpurun_out/TAG_pmc/       SQ / TCC / TCP / TA passes (tools/pmc_l0_passes.txt) over
#                             the level-0 launch group (kbench --mode level --from-solve)
# --icp: the same for the combine_ICP kernel (cfg5, bench.py --icp).
# Each GPU step has its own time limit; the script stops at the first failure.
set -e
tag=${1:?tag}
icp=${2:-}
root=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$root"
export TMPDIR=/tmp
mkdir -p gpurun_out
bench_extra="--no-cpu-baseline"  # (the kernel profile; bench.py's own line carries the CPU baseline)
[ -n "$icp" ] && bench_extra="--icp --no-cpu-baseline --no-compare"
( cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$root/gpurun_out/${tag}_prof" \
    -o bench -- python3 "$root/bench.py" --steps 100 --warmup 10 $bench_extra ) > "gpurun_out/${tag}_prof.log" 2>&1
timeout -k 10 240 python tools/pmc_l0.py --groups 16 $icp --out "gpurun_out/${tag}_l0_traffic.json" > "gpurun_out/${tag}_traffic.log" 2>&1
PMC_PASSES="$(cat tools/pmc_l0_passes.txt)" timeout -k 10 600 tools/pmc_passes.sh "gpurun_out/${tag}_pmc" -- \
    python3 "$root/tools/kbench.py" --c4 --from-solve --mode level --reps 10 --warm-ms 0 --groups 16 $icp
echo "profile set $tag done"
