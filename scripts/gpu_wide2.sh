#!/bin/bash
# Kernel stats of the 1000x1000 dense workload (normal, forced wide, forced pixel-indexed) and config-5 bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-wide2}
mkdir -p gpurun_out/$TAG
rm -rf /tmp/prof_tp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_tp -o run -- \
  python3 -u scripts/time_paths.py 1000 1000 2100 1000 > gpurun_out/$TAG/time_paths_dense.txt 2>&1 \
  || { tail -20 gpurun_out/$TAG/time_paths_dense.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/$TAG/time_paths_dense.txt
for f in $(find /tmp/prof_tp -name "*kernel_stats.csv"); do cp $f gpurun_out/$TAG/tp_kernel_stats.csv; done
python3 scripts/short_stats.py gpurun_out/$TAG/tp_kernel_stats.csv | tee gpurun_out/$TAG/tp_kernel_stats_short.txt
[ "${C5:-1}" = "1" ] && bash scripts/gpu_config5.sh $TAG/c5
