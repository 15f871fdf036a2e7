#!/bin/bash
# the sort: GPU tests, timing (scripts/time_sort.py) and a per-kernel rocprofv3 summary: scripts/gpu_sort2.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-sort}
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sort.py > gpurun_out/$TAG/pytest_sort.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest_sort.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest_sort.log
timeout -k 10 200 python3 -u scripts/time_sort.py > gpurun_out/$TAG/time_sort.txt 2>&1 || exit 1
grep -v amdgpu gpurun_out/$TAG/time_sort.txt
cd /tmp && export TMPDIR=/tmp && rm -rf /tmp/sortprof && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/sortprof -o run -- python3 $GRAFT_REPO_ROOT/scripts/time_sort.py > /dev/null 2>&1 || exit 1
f=$(find /tmp/sortprof -name "*kernel_stats.csv" | head -1)
cp $f $GRAFT_REPO_ROOT/gpurun_out/$TAG/sort_kernel_stats.csv
python3 $GRAFT_REPO_ROOT/scripts/short_stats.py $f 20 | tee $GRAFT_REPO_ROOT/gpurun_out/$TAG/sort_kernel_stats_short.txt
