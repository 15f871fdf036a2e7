#!/bin/bash
# GPU parity suite (tests/test_gpu_parity.py) + smoke; stops at the first failure.  scripts/gpu_parity.sh TAG [pytest args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-parity}; shift
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread "$@" \
  > gpurun_out/$TAG/parity.log 2>&1 || { tail -40 gpurun_out/$TAG/parity.log; exit 1; }
tail -3 gpurun_out/$TAG/parity.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 || { tail -20 gpurun_out/$TAG/smoke.log; exit 1; }
tail -1 gpurun_out/$TAG/smoke.log
