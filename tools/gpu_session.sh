#!/bin/bash
# Run GPU steps in order; each under its own time limit. Stop at the first step
# that times out, aborts, segfaults or otherwise dies abnormally (rc >= 124);
# ordinary test failures (rc 1/2) do not stop later steps.
# usage: tools/gpu_session.sh "name:seconds:command" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; secs="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== $name (limit ${secs}s): $cmd" | tee -a gpurun_out/session.log
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc ($(( $(date +%s) - start ))s)" | tee -a gpurun_out/session.log
  tail -n 15 "gpurun_out/$name.log"
  if [ $rc -ge 124 ]; then echo "abnormal exit, stopping" | tee -a gpurun_out/session.log; exit $rc; fi
done
exit 0
