#!/bin/bash
# PMC passes (counters only; kernel trace on) over a command: tools/pmc_passes.sh OUTDIR -- cmd...
# One rocprofv3 run per pass; no --pmc combined with sys/runtime traces.
out=$1; shift; shift
mkdir -p "$out"
export TMPDIR=/tmp
i=0
while read -r pass; do
  [ -z "$pass" ] && continue
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $pass --output-format csv -d "$out/p$i" -o pmc -- "$@" > "$out/p$i.log" 2>&1 || { rc=$?; echo "pass $i ($pass) failed rc=$rc"; [ $rc -ge 124 ] && exit 1; }
done <<PASSES
${PMC_PASSES:-SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA}
PASSES
echo "passes done: $i"
