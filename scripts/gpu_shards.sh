#!/bin/bash
# per-rank critical path of the sharded step on one GPU (scripts/time_shards.py), W = 8 and 2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-shards}
mkdir -p gpurun_out/$TAG
for w in ${WS:-8 2}; do
  timeout -k 10 400 python3 -u scripts/time_shards.py $w > gpurun_out/$TAG/time_shards_$w.txt 2>&1 \
    || { tail -20 gpurun_out/$TAG/time_shards_$w.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/$TAG/time_shards_$w.txt
done
