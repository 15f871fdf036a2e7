#!/bin/bash
# A/B of sort variants (scripts/build_sort_variant.sh) on the config-3 dataset, then the sort tests and a
# rocprofv3 kernel-trace of the default library's sort: scripts/gpu_sort_ab.sh [variant ...]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for v in base "$@"; do
  if [ $v = base ]; then L=sm_distributed_amd/libsmg.so; else L=sm_distributed_amd/variants/sort/$v.so; fi
  echo "### $v"; SMG_LIB=$PWD/$L timeout -k 10 120 python -u scripts/time_sort.py || exit $?
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_sort.py || exit $?
mkdir -p gpurun_out/sortprof
cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/sortprof -o run -- python3 $GRAFT_REPO_ROOT/scripts/time_sort.py > /dev/null 2>&1; rc=$?
find /tmp/sortprof -name "*kernel_stats.csv" -exec cp {} $GRAFT_REPO_ROOT/gpurun_out/sortprof/ \;
exit $rc
