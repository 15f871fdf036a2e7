#!/bin/bash
# kernel + HIP runtime timeline of the API step (bench.py, N = 1, 2 timed steps) and of one rank's shard
# (scripts/time_shards.py ONLY_RANK=3 of an 8-way plan): CSV traces for scripts/timeline_gaps.py
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-tl}
mkdir -p gpurun_out/$TAG
rm -rf /tmp/tl_api /tmp/tl_shard
timeout -k 10 400 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d /tmp/tl_api -o run -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --chain-steps 0 > gpurun_out/$TAG/api.log 2>&1 \
  || { tail -20 gpurun_out/$TAG/api.log; exit 1; }
for f in $(find /tmp/tl_api -name "*.csv"); do cp $f gpurun_out/$TAG/api_$(basename $f); done
ONLY_RANK=3 timeout -k 10 400 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d /tmp/tl_shard -o run -- \
  python3 scripts/time_shards.py 8 > gpurun_out/$TAG/shard.log 2>&1 || { tail -20 gpurun_out/$TAG/shard.log; exit 1; }
for f in $(find /tmp/tl_shard -name "*.csv"); do cp $f gpurun_out/$TAG/shard_$(basename $f); done

python3 scripts/timeline_gaps.py gpurun_out/$TAG/api_run_kernel_trace.csv gpurun_out/$TAG/api_run_hip_api_trace.csv > gpurun_out/$TAG/api_timeline.txt
python3 scripts/timeline_gaps.py gpurun_out/$TAG/shard_run_kernel_trace.csv gpurun_out/$TAG/shard_run_hip_api_trace.csv --start slice_count --which -1 > gpurun_out/$TAG/shard_timeline.txt
rm -f gpurun_out/$TAG/*trace.csv
head -60 gpurun_out/$TAG/api_timeline.txt
