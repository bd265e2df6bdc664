#!/bin/bash
# Run GPU steps in order on the box, each under its own time limit:
#   tools/gpu_steps.sh "TIMEOUT_S:command" ["TIMEOUT_S:command" ...]
# A test failure (exit 1) does not stop the sequence; anything else non-zero
# (a crash, an abort, a time limit) ends the call there.  Step i's output is
# gpurun_out/step<i>.log.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out
i=0
for step in "$@"; do
  i=$((i + 1))
  to=${step%%:*}
  cmd=${step#*:}
  echo "== step $i (limit ${to}s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$to" bash -c "$cmd" > "gpurun_out/step$i.log" 2>&1
  rc=$?
  echo "rc=$rc after $(( $(date +%s) - start ))s"
  tail -n "${TAIL:-12}" "gpurun_out/step$i.log"
  if [ $rc -gt 1 ]; then
    echo "stopping after step $i (rc=$rc)"
    exit $rc
  fi
done
