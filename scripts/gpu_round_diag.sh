#!/bin/bash
# tests -> stamps diagnostic -> bench+profile; stop at first failure
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-rX}
mkdir -p gpurun_out/$TAG
bash scripts/gpu_tests.sh || exit 1
timeout -k 10 400 python scripts/diag_stamps.py > gpurun_out/$TAG/diag.log 2>&1; rc=$?; cat gpurun_out/$TAG/diag.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_bench.sh $TAG
