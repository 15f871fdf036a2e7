#!/bin/bash
# Runs GPU steps in order, each under its own time limit, output to gpurun_out/$TAG/<name>.log.  A step that
# fails with an ordinary error (exit 1, e.g. a failed test) lets the next step run; a fault, abort, segfault or time
# limit (any other non-zero status) ends the call there.
#   scripts/gpu_steps.sh TAG "name|seconds|command" ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=$1; shift
mkdir -p gpurun_out/$TAG
worst=0
for step in "$@"; do
  name=${step%%|*}; rest=${step#*|}; secs=${rest%%|*}; cmd=${rest#*|}
  echo "=== $name ($secs s): $cmd"
  timeout -k 10 $secs bash -c "$cmd" > gpurun_out/$TAG/$name.log 2>&1
  rc=$?
  tail -${TAILN:-12} gpurun_out/$TAG/$name.log
  echo "=== $name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: $name ended with status $rc"; exit $rc; fi
  # a GPU fault inside a step that still exits 1 (pytest) also ends the call
  if grep -q "HSA_STATUS_ERROR\|illegal memory access\|hipErrorIllegalAddress\|APERTURE_VIOLATION" gpurun_out/$TAG/$name.log; then
    echo "stopping: GPU fault in $name"; exit 3
  fi
  [ $rc -ne 0 ] && worst=1
done
exit $worst
