#!/bin/bash
# the >2^32-point GPU test alone
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_huge.py -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_huge.log 2>&1
rc=$?
tail -30 gpurun_out/pytest_huge.log
exit $rc
