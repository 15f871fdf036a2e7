#!/bin/bash
# the hot-spot clip on the wide pass: parity suite, then the ion-stage timing with and without the clip at
# 1000x1000 (the verdict's workload) and at config 3: scripts/gpu_clip.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-clip}
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  > gpurun_out/$TAG/pytest_parity.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest_parity.log; exit 1; }
tail -3 gpurun_out/$TAG/pytest_parity.log
timeout -k 10 600 python3 -u scripts/time_paths.py 1000 1000 1000 2000 > gpurun_out/$TAG/paths_1000.txt 2>&1 || exit 1
cat gpurun_out/$TAG/paths_1000.txt
timeout -k 10 600 python3 -u scripts/time_paths.py > gpurun_out/$TAG/paths_c3.txt 2>&1 || exit 1
cat gpurun_out/$TAG/paths_c3.txt
