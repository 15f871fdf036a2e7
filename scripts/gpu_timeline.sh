#!/bin/bash
# kernel + HIP runtime timeline of the API step (bench.py, N = 1, 2 timed steps) and (SHARD=1) of one rank's shard
# (scripts/time_shards.py ONLY_RANK=3 of an 8-way plan); summarised by scripts/timeline_gaps.py (traces deleted)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-tl}
mkdir -p gpurun_out/$TAG
rm -rf /tmp/tl_api /tmp/tl_shard
timeout -k 10 400 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d /tmp/tl_api -o run -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --chain-steps 0 > gpurun_out/$TAG/api.log 2>&1 \
  || { tail -20 gpurun_out/$TAG/api.log; exit 1; }
K=$(find /tmp/tl_api -name "*kernel_trace.csv" | head -1); H=$(find /tmp/tl_api -name "*hip_api_trace.csv" | head -1)
python3 scripts/timeline_gaps.py $K $H --start ${START:-sort_mark_starts_kernel} > gpurun_out/$TAG/api_timeline.txt || exit 1
if [ "${SHARD:-1}" = "1" ]; then
  ONLY_RANK=3 timeout -k 10 400 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d /tmp/tl_shard -o run -- \
    python3 scripts/time_shards.py 8 > gpurun_out/$TAG/shard.log 2>&1 || { tail -20 gpurun_out/$TAG/shard.log; exit 1; }
  K=$(find /tmp/tl_shard -name "*kernel_trace.csv" | head -1); H=$(find /tmp/tl_shard -name "*hip_api_trace.csv" | head -1)
  python3 scripts/timeline_gaps.py $K $H --start slice_count --which -1 > gpurun_out/$TAG/shard_timeline.txt || exit 1
fi
rm -rf /tmp/tl_api /tmp/tl_shard
head -70 gpurun_out/$TAG/api_timeline.txt
