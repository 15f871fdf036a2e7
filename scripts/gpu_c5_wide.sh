#!/bin/bash
# Config-5 rank-0 shard (8-way plan) scored on one GPU with each wide-pass implementation (scripts/time_shards.py,
# ONLY_RANK=0): per-pass HIP-event times -> gpurun_out/$TAG/c5_rank0_wide{1,0}.txt
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-c5w}
mkdir -p gpurun_out/$TAG
for impl in ${IMPLS:-1 0}; do
  CONFIG=5 SKIP_T1=1 ONLY_RANK=${RANK0:-0} WIDE_IMPL=$impl timeout -k 10 500 python3 -u scripts/time_shards.py 8 \
    > gpurun_out/$TAG/c5_rank0_wide$impl.txt 2>&1 || { tail -20 gpurun_out/$TAG/c5_rank0_wide$impl.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/$TAG/c5_rank0_wide$impl.txt
done
