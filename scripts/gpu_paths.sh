#!/bin/bash
# normal / forced-dense / clip timings at config 3 and at 1000x1000, then a kernel-trace profile of the latter
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-paths}
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python scripts/time_paths.py > gpurun_out/$TAG/c3.txt 2>&1 || { tail -20 gpurun_out/$TAG/c3.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/$TAG/c3.txt
timeout -k 10 300 python scripts/time_paths.py 1000 1000 1000 2000 > gpurun_out/$TAG/c5.txt 2>&1 || { tail -20 gpurun_out/$TAG/c5.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/$TAG/c5.txt
rm -rf /tmp/prof_$TAG
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$TAG -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --nrows 1000 --ncols 1000 --peaks 1000 --n-sf 2000 > gpurun_out/$TAG/prof.log 2>&1 || { tail -30 gpurun_out/$TAG/prof.log; exit 1; }
for f in $(find /tmp/prof_$TAG -name "*kernel_stats.csv"); do cp $f gpurun_out/$TAG/kernel_stats.csv; done
python3 scripts/short_stats.py gpurun_out/$TAG/kernel_stats.csv | tee gpurun_out/$TAG/kernel_stats_short.txt
