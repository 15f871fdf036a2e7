#!/bin/bash
# Per-kernel times of the config-3 flag + sort + scan stage (scripts/prof_sort_stage.py under rocprofv3 stats)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-psort}
mkdir -p gpurun_out/$TAG
rm -rf /tmp/prof_sort
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_sort -o run -- \
  python3 -u scripts/prof_sort_stage.py > gpurun_out/$TAG/stage.txt 2>&1 || { tail -20 gpurun_out/$TAG/stage.txt; exit 1; }
grep -v amdgpu gpurun_out/$TAG/stage.txt
for f in $(find /tmp/prof_sort -name "*kernel_stats.csv"); do cp $f gpurun_out/$TAG/kernel_stats.csv; done
python3 scripts/short_stats.py gpurun_out/$TAG/kernel_stats.csv | tee gpurun_out/$TAG/kernel_stats_short.txt
